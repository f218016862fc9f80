// SSD training-target assignment (MultiBoxTarget) for gfx950.
//
// Parity: src/operator/contrib/multibox_target.cc (MultiBoxTargetForward, CPU
// reference semantics: greedy bipartite matching, threshold matching, hard
// negative mining by background probability with a stable order, location
// target encoding with variances) and multibox_target.cu.
//
// MI355X design: one 1024-thread workgroup (16 waves) per image.  IoUs are
// recomputed on the fly from the ground-truth boxes held in LDS instead of
// materialising an [A, G] overlap matrix; the per-anchor match state lives in
// LDS (flags) and in workgroup-private global scratch (best IoU / gt index /
// mining key).  Hard-negative selection is an exact k-smallest select: a
// 32-step radix-style binary search on the IEEE bits of the background
// probability (non-negative floats order like their bit patterns) followed by
// an index-ordered prefix scan for the ties, which reproduces the reference's
// std::stable_sort order without sorting.
#include <stdexcept>

#include "common.h"

namespace mxamd {

namespace {

constexpr int kMbtThreads = 1024;
constexpr int kMbtWaves = kMbtThreads / kWave;
constexpr int kMbtMaxAnchors = 32768;
constexpr int kMbtMaxLabels = 1024;

__device__ __forceinline__ float box_iou(float ax1, float ay1, float ax2, float ay2, const float* g) {
  const float w = fmaxf(0.f, fminf(ax2, g[2]) - fmaxf(ax1, g[0]));
  const float h = fmaxf(0.f, fminf(ay2, g[3]) - fmaxf(ay1, g[1]));
  const float i = w * h;
  const float u = (ax2 - ax1) * (ay2 - ay1) + (g[2] - g[0]) * (g[3] - g[1]) - i;
  return u <= 0.f ? 0.f : i / u;
}

// (value, j, k) lexicographic "better": larger value, then smaller anchor, then smaller gt —
// the first maximum met by the reference's j-major / k-minor scan with strict '>'.
__device__ __forceinline__ bool better(float v, int j, int k, float ov, int oj, int ok) {
  if (oj < 0) return j >= 0;
  if (j < 0) return false;
  if (v != ov) return v > ov;
  if (j != oj) return j < oj;
  return k < ok;
}

__device__ __forceinline__ uint32_t block_sum_u32(uint32_t v, uint32_t* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  const int wave = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) red[wave] = v;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int w = 0; w < kMbtWaves; ++w) t += red[w];
  __syncthreads();
  return t;
}

template <typename T>
__global__ void __launch_bounds__(kMbtThreads)
    multibox_target_kernel(const float* __restrict__ anchors, const float* __restrict__ labels,
                           const T* __restrict__ cls_pred, float* __restrict__ loc_target,
                           float* __restrict__ loc_mask, float* __restrict__ cls_target,
                           float* __restrict__ match_iou_g, int* __restrict__ match_gt_g, uint32_t* __restrict__ key_g,
                           int A, int L, int W, int C, float thr, float ignore_label, float neg_ratio,
                           float neg_thresh, int min_neg, float v0, float v1, float v2, float v3) {
  __shared__ signed char sflag[kMbtMaxAnchors];
  __shared__ float sgt[kMbtMaxLabels * 4];
  __shared__ unsigned char sgflag[kMbtMaxLabels];
  __shared__ float rv[kMbtWaves];
  __shared__ int rj[kMbtWaves], rk[kMbtWaves];
  __shared__ uint32_t red[kMbtWaves];
  __shared__ int s_ng, s_npos;

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const float* lab = labels + static_cast<int64_t>(b) * L * W;
  float* mi = match_iou_g + static_cast<int64_t>(b) * A;
  int* mg = match_gt_g + static_cast<int64_t>(b) * A;
  uint32_t* key = key_g + static_cast<int64_t>(b) * A;

  if (tid == 0) {
    int ng = 0;
    while (ng < L && lab[ng * W] != -1.f) ++ng;   // valid gts end at the first class == -1 row
    s_ng = ng;
    s_npos = 0;
  }
  __syncthreads();
  const int ng = s_ng;
  for (int k = tid; k < ng; k += kMbtThreads) {
#pragma unroll
    for (int c = 0; c < 4; ++c) sgt[k * 4 + c] = lab[k * W + 1 + c];
    sgflag[k] = 0;
  }
  for (int j = tid; j < A; j += kMbtThreads) {
    sflag[j] = -1;
    mi[j] = -1.f;
    mg[j] = -1;
  }
  __syncthreads();

  if (ng > 0) {
    // ---- greedy bipartite stage: each gt claims its best still-free anchor, best pair first
    for (int it = 0; it < ng; ++it) {
      float bv = 1e-6f;
      int bj = -1, bk = -1;
      for (int j = tid; j < A; j += kMbtThreads) {
        if (sflag[j] == 1) continue;
        const float4 a = reinterpret_cast<const float4*>(anchors)[j];
        for (int k = 0; k < ng; ++k) {
          if (sgflag[k]) continue;
          const float v = box_iou(a.x, a.y, a.z, a.w, &sgt[k * 4]);
          if (v > bv) { bv = v; bj = j; bk = k; }
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, kWave);
        const int oj = __shfl_xor(bj, o, kWave);
        const int ok = __shfl_xor(bk, o, kWave);
        if (better(ov, oj, ok, bv, bj, bk)) { bv = ov; bj = oj; bk = ok; }
      }
      if (tid % kWave == 0) {
        rv[tid / kWave] = bv;
        rj[tid / kWave] = bj;
        rk[tid / kWave] = bk;
      }
      __syncthreads();
      if (tid == 0) {
        for (int w = 1; w < kMbtWaves; ++w)
          if (better(rv[w], rj[w], rk[w], rv[0], rj[0], rk[0])) { rv[0] = rv[w]; rj[0] = rj[w]; rk[0] = rk[w]; }
        if (rj[0] >= 0) {
          sflag[rj[0]] = 1;
          sgflag[rk[0]] = 1;
          mi[rj[0]] = rv[0];
          mg[rj[0]] = rk[0];
          ++s_npos;
        }
      }
      __syncthreads();
      if (rj[0] < 0) break;          // uniform: every thread reads the same LDS word
      __syncthreads();               // rj[0] is rewritten by the next iteration's wave leaders
    }

    // ---- threshold stage: remaining anchors take their best gt, positive above the threshold
    if (thr > 0.f) {
      int local = 0;
      for (int j = tid; j < A; j += kMbtThreads) {
        if (sflag[j] == 1) continue;
        const float4 a = reinterpret_cast<const float4*>(anchors)[j];
        float bv = -1.f;
        int bk = -1;
        for (int k = 0; k < ng; ++k) {
          const float v = box_iou(a.x, a.y, a.z, a.w, &sgt[k * 4]);
          if (v > bv) { bv = v; bk = k; }
        }
        mi[j] = bv;
        mg[j] = bk;
        if (bv > thr) { sflag[j] = 1; ++local; }
      }
      const uint32_t tot = block_sum_u32(static_cast<uint32_t>(local), red);
      if (tid == 0) s_npos += static_cast<int>(tot);
    }
    __syncthreads();
    const int npos = s_npos;

    if (neg_ratio > 0.f) {
      int nneg = static_cast<int>(npos * neg_ratio);
      if (nneg > A - npos) nneg = A - npos;
      const int mn = min_neg < A - npos ? min_neg : A - npos;
      if (nneg < mn) nneg = mn;
      if (nneg > 0) {
        // mining key: background softmax probability of each candidate, UINT_MAX otherwise
        const T* cp = cls_pred + static_cast<int64_t>(b) * C * A;
        uint32_t ncand = 0;
        for (int j = tid; j < A; j += kMbtThreads) {
          uint32_t kk = 0xFFFFFFFFu;
          if (sflag[j] != 1) {
            float m_iou = mi[j];
            if (m_iou < 0.f) {
              const float4 a = reinterpret_cast<const float4*>(anchors)[j];
              float bv = -1.f;
              int bk = -1;
              for (int k = 0; k < ng; ++k) {
                const float v = box_iou(a.x, a.y, a.z, a.w, &sgt[k * 4]);
                if (v > bv) { bv = v; bk = k; }
              }
              mi[j] = m_iou = bv;
              mg[j] = bk;
            }
            if (m_iou < neg_thresh && sflag[j] == -1) {
              float mx = static_cast<float>(cp[j]);
              for (int c = 1; c < C; ++c) mx = fmaxf(mx, static_cast<float>(cp[static_cast<int64_t>(c) * A + j]));
              float s = 0.f;
              for (int c = 0; c < C; ++c) s += __expf(static_cast<float>(cp[static_cast<int64_t>(c) * A + j]) - mx);
              const float p = __expf(static_cast<float>(cp[j]) - mx) / s;
              kk = p == p ? __float_as_uint(fmaxf(p, 0.f)) : 0x7F800000u;  // NaN sorts last among candidates
              ++ncand;
            }
          }
          key[j] = kk;
        }
        const uint32_t nc = block_sum_u32(ncand, red);
        const uint32_t want = static_cast<uint32_t>(nneg) < nc ? static_cast<uint32_t>(nneg) : nc;
        if (want > 0) {
          // smallest T with #(key <= T) >= want
          uint32_t lo = 0, hi = 0x7F800000u;
          while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            uint32_t c = 0;
            for (int j = tid; j < A; j += kMbtThreads) c += key[j] <= mid;
            if (block_sum_u32(c, red) >= want) hi = mid; else lo = mid + 1;
          }
          const uint32_t T_ = lo;
          uint32_t cl = 0;
          for (int j = tid; j < A; j += kMbtThreads) {
            if (key[j] < T_) { sflag[j] = 0; ++cl; }
          }
          const uint32_t less = block_sum_u32(cl, red);
          // ties at T_: take the lowest anchor indices (stable order)
          uint32_t need = want - less;
          for (int base = 0; base < A && need > 0; base += kMbtThreads) {
            const int j = base + tid;
            const bool eq = j < A && key[j] == T_;
            const uint64_t bal = __ballot(eq);
            const uint32_t before = __popcll(bal & ((1ull << (tid % kWave)) - 1ull));
            if (tid % kWave == 0) red[tid / kWave] = static_cast<uint32_t>(__popcll(bal));
            __syncthreads();
            uint32_t off = 0, tot = 0;
            for (int w = 0; w < kMbtWaves; ++w) {
              if (w < tid / kWave) off += red[w];
              tot += red[w];
            }
            if (eq && off + before < need) sflag[j] = 0;
            __syncthreads();
            need = tot >= need ? 0 : need - tot;
          }
        }
      }
    } else {
      for (int j = tid; j < A; j += kMbtThreads)
        if (sflag[j] != 1) sflag[j] = 0;
    }
  }
  __syncthreads();

  // ---- outputs
  float* lt = loc_target + static_cast<int64_t>(b) * A * 4;
  float* lm = loc_mask + static_cast<int64_t>(b) * A * 4;
  float* ct = cls_target + static_cast<int64_t>(b) * A;
  for (int j = tid; j < A; j += kMbtThreads) {
    const int f = ng > 0 ? sflag[j] : -1;
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 m = t;
    float c = ignore_label;
    if (f == 1) {
      const int k = mg[j];
      const float4 a = reinterpret_cast<const float4*>(anchors)[j];
      const float* g = &sgt[k * 4];
      const float aw = a.z - a.x, ah = a.w - a.y;
      const float ax = (a.x + a.z) * 0.5f, ay = (a.y + a.w) * 0.5f;
      const float gw = g[2] - g[0], gh = g[3] - g[1];
      const float gx = (g[0] + g[2]) * 0.5f, gy = (g[1] + g[3]) * 0.5f;
      t = make_float4((gx - ax) / aw / v0, (gy - ay) / ah / v1, logf(gw / aw) / v2, logf(gh / ah) / v3);
      m = make_float4(1.f, 1.f, 1.f, 1.f);
      c = lab[k * W] + 1.f;
    } else if (f == 0) {
      c = 0.f;
    }
    reinterpret_cast<float4*>(lt)[j] = t;
    reinterpret_cast<float4*>(lm)[j] = m;
    ct[j] = c;
  }
}

}  // namespace

void multibox_target(int dtype, const float* anchors, const float* labels, const void* cls_pred, float* loc_target,
                     float* loc_mask, float* cls_target, float* match_iou, int* match_gt, uint32_t* key, int B, int A,
                     int L, int W, int C, float thr, float ignore_label, float neg_ratio, float neg_thresh,
                     int min_neg, float v0, float v1, float v2, float v3, hipStream_t s) {
  MXAMD_HOST_CHECK(A > 0 && A <= kMbtMaxAnchors, "multibox_target: anchors per image must be in [1, 32768]");
  MXAMD_HOST_CHECK(L >= 0 && L <= kMbtMaxLabels, "multibox_target: at most 1024 label rows per image");
  MXAMD_HOST_CHECK(W >= 5 && C >= 1 && B >= 1, "multibox_target: label width >= 5, >= 1 class, >= 1 image");
  MXAMD_HOST_CHECK((reinterpret_cast<uintptr_t>(anchors) & 15) == 0 && (reinterpret_cast<uintptr_t>(loc_target) & 15) == 0 &&
                       (reinterpret_cast<uintptr_t>(loc_mask) & 15) == 0,
                   "multibox_target: anchors / loc outputs must be 16-byte aligned");
#define MBT_LAUNCH(T)                                                                                               \
  multibox_target_kernel<T><<<B, kMbtThreads, 0, s>>>(anchors, labels, static_cast<const T*>(cls_pred), loc_target, \
                                                      loc_mask, cls_target, match_iou, match_gt, key, A, L, W, C, thr, \
                                                      ignore_label, neg_ratio, neg_thresh, min_neg, v0, v1, v2, v3)
  switch (dtype) {
    case kF32: MBT_LAUNCH(float); break;
    case kF16: MBT_LAUNCH(__half); break;
    case kBF16: MBT_LAUNCH(__hip_bfloat16); break;
    default: throw std::runtime_error("multibox_target: unsupported dtype");
  }
#undef MBT_LAUNCH
}

// ------------------------------------------------------------------------------ fused SSD training loss
// Parity: the loss of example/ssd/symbol/symbol_builder.py:90-102 -- SoftmaxOutput over the classes with
// ignore_label -1 normalised by the valid anchors ('valid' normalisation), plus smooth_l1(sigma 1) on the
// masked location offsets normalised by the positive anchors (MakeLoss with grad_scale lambda).  The
// reference builds it from separate GPU operators; here one pass over the [B*A] anchor rows computes both
// terms (fp32 arithmetic on f16 / bf16 / f32 predictions), a one-workgroup pass sums the per-block
// partials in a fixed order (deterministic), and the backward writes both gradients in one pass.
namespace {

template <typename T>
__device__ __forceinline__ float ldf(const T* p) { return static_cast<float>(*p); }
template <>
__device__ __forceinline__ float ldf<__half>(const __half* p) { return __half2float(*p); }
template <>
__device__ __forceinline__ float ldf<__hip_bfloat16>(const __hip_bfloat16* p) {
  return __uint_as_float(static_cast<uint32_t>(*reinterpret_cast<const uint16_t*>(p)) << 16);
}
template <typename T>
__device__ __forceinline__ void stf(T* p, float v) { *p = static_cast<T>(v); }
template <>
__device__ __forceinline__ void stf<__half>(__half* p, float v) { *p = __float2half(v); }
template <>
__device__ __forceinline__ void stf<__hip_bfloat16>(__hip_bfloat16* p, float v) { *p = __float2bfloat16(v); }

constexpr int kSslThreads = 256;
constexpr int kSslMaxClasses = 1024;

__device__ __forceinline__ float ssl_block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  const int wave = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) red[wave] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < kSslThreads / kWave; ++w) t += red[w];
  __syncthreads();
  return t;
}

// per anchor row: (cross-entropy if valid, valid, positive, smooth-L1 of the 4 masked offsets)
template <typename T>
__global__ void __launch_bounds__(kSslThreads) ssd_loss_fwd_kernel(const T* __restrict__ cls, const T* __restrict__ loc,
                                                                   const float* __restrict__ cls_t,
                                                                   const float* __restrict__ loc_t,
                                                                   const float* __restrict__ loc_m, int rows, int C1,
                                                                   float* __restrict__ part) {
  __shared__ float red[kSslThreads / kWave];
  const int row = blockIdx.x * kSslThreads + threadIdx.x;
  float ce = 0.f, nv = 0.f, np = 0.f, ls = 0.f;
  if (row < rows) {
    const float t = cls_t[row];
    if (t >= 0.f) {
      const T* l = cls + (int64_t)row * C1;
      float m = -INFINITY;
      for (int c = 0; c < C1; ++c) m = fmaxf(m, ldf(l + c));
      float se = 0.f;
      for (int c = 0; c < C1; ++c) se += __expf(ldf(l + c) - m);
      const int ti = min(static_cast<int>(t), C1 - 1);
      ce = m + __logf(se) - ldf(l + ti);
      nv = 1.f;
      np = t > 0.f ? 1.f : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t o = (int64_t)row * 4 + k;
      const float d = (ldf(loc + o) - loc_t[o]) * loc_m[o];
      const float ad = fabsf(d);
      ls += ad < 1.f ? 0.5f * d * d : ad - 0.5f;
    }
  }
  const float s0 = ssl_block_sum(ce, red), s1 = ssl_block_sum(nv, red), s2 = ssl_block_sum(np, red),
              s3 = ssl_block_sum(ls, red);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s0;
    part[gridDim.x + blockIdx.x] = s1;
    part[2 * gridDim.x + blockIdx.x] = s2;
    part[3 * gridDim.x + blockIdx.x] = s3;
  }
}

// out = [loss, n_valid, n_positive]
__global__ void __launch_bounds__(kSslThreads) ssd_loss_fin_kernel(const float* __restrict__ part, int nblk, float lambd,
                                                                   float* __restrict__ out) {
  __shared__ float red[kSslThreads / kWave];
  float v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float a = 0.f;
    for (int i = threadIdx.x; i < nblk; i += kSslThreads) a += part[q * nblk + i];
    v[q] = ssl_block_sum(a, red);
  }
  if (threadIdx.x == 0) {
    const float nv = fmaxf(v[1], 1.f), np = fmaxf(v[2], 1.f);
    out[0] = v[0] / nv + lambd * v[3] / np;
    out[1] = v[1];
    out[2] = v[2];
  }
}

template <typename T>
__global__ void __launch_bounds__(kSslThreads) ssd_loss_bwd_kernel(const T* __restrict__ cls, const T* __restrict__ loc,
                                                                   const float* __restrict__ cls_t,
                                                                   const float* __restrict__ loc_t,
                                                                   const float* __restrict__ loc_m,
                                                                   const float* __restrict__ stats,
                                                                   const float* __restrict__ gout, int rows, int C1,
                                                                   float lambd, T* __restrict__ dcls,
                                                                   T* __restrict__ dloc) {
  const int row = blockIdx.x * kSslThreads + threadIdx.x;
  if (row >= rows) return;
  const float g = gout[0];
  const float gv = g / fmaxf(stats[1], 1.f);
  const float gp = g * lambd / fmaxf(stats[2], 1.f);
  const float t = cls_t[row];
  const T* l = cls + (int64_t)row * C1;
  T* dl = dcls + (int64_t)row * C1;
  if (t >= 0.f) {
    float m = -INFINITY;
    for (int c = 0; c < C1; ++c) m = fmaxf(m, ldf(l + c));
    float se = 0.f;
    for (int c = 0; c < C1; ++c) se += __expf(ldf(l + c) - m);
    const float inv = 1.f / se;
    const int ti = min(static_cast<int>(t), C1 - 1);
    for (int c = 0; c < C1; ++c) {
      const float p = __expf(ldf(l + c) - m) * inv;
      stf(dl + c, gv * (p - (c == ti ? 1.f : 0.f)));
    }
  } else {
    for (int c = 0; c < C1; ++c) stf(dl + c, 0.f);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t o = (int64_t)row * 4 + k;
    const float mk = loc_m[o];
    const float d = (ldf(loc + o) - loc_t[o]) * mk;
    stf(dloc + o, gp * fminf(fmaxf(d, -1.f), 1.f) * mk);
  }
}

}  // namespace

int ssd_loss_blocks(int rows) { return (rows + kSslThreads - 1) / kSslThreads; }

void ssd_loss_fwd(int dtype, const void* cls, const void* loc, const float* cls_t, const float* loc_t,
                  const float* loc_m, int rows, int C1, float lambd, float* part, float* out, hipStream_t s) {
  MXAMD_HOST_CHECK(rows > 0 && C1 >= 1 && C1 <= kSslMaxClasses, "ssd_loss: bad row / class count");
  const int nblk = ssd_loss_blocks(rows);
#define SSL_FWD(T)                                                                                                   \
  ssd_loss_fwd_kernel<T><<<nblk, kSslThreads, 0, s>>>(static_cast<const T*>(cls), static_cast<const T*>(loc), cls_t, \
                                                     loc_t, loc_m, rows, C1, part)
  switch (dtype) {
    case kF32: SSL_FWD(float); break;
    case kF16: SSL_FWD(__half); break;
    case kBF16: SSL_FWD(__hip_bfloat16); break;
    default: throw std::runtime_error("ssd_loss: unsupported dtype");
  }
#undef SSL_FWD
  ssd_loss_fin_kernel<<<1, kSslThreads, 0, s>>>(part, nblk, lambd, out);
}

void ssd_loss_bwd(int dtype, const void* cls, const void* loc, const float* cls_t, const float* loc_t,
                  const float* loc_m, const float* stats, const float* gout, int rows, int C1, float lambd, void* dcls,
                  void* dloc, hipStream_t s) {
  const int nblk = ssd_loss_blocks(rows);
#define SSL_BWD(T)                                                                                                    \
  ssd_loss_bwd_kernel<T><<<nblk, kSslThreads, 0, s>>>(static_cast<const T*>(cls), static_cast<const T*>(loc), cls_t,  \
                                                     loc_t, loc_m, stats, gout, rows, C1, lambd, static_cast<T*>(dcls), \
                                                     static_cast<T*>(dloc))
  switch (dtype) {
    case kF32: SSL_BWD(float); break;
    case kF16: SSL_BWD(__half); break;
    case kBF16: SSL_BWD(__hip_bfloat16); break;
    default: throw std::runtime_error("ssd_loss: unsupported dtype");
  }
#undef SSL_BWD
}

}  // namespace mxamd
