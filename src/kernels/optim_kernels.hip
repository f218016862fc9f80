// Fused optimizer kernels over flat parameter arenas (gfx950).
//
// Parity: src/operator/optimizer_op.cc/.cu (adam_update, mp_adam semantics of
// the Python Adam: bias correction folded into lr), src/operator/contrib/adamw.cu
// (adamw_update / mp_adamw_update: decoupled weight decay scaled by eta),
// src/operator/optimizer_op.cc lamb_update_phase1/2 (+ mp_ variants) and
// src/operator/contrib/multi_sum_sq.cu / all_finite.cu.
//
// The Trainer keeps every parameter of one (dtype, lr_mult, wd_mult) group in a
// contiguous arena (64-element aligned segments, zero padding), so each update
// is ONE pass over HBM: 16-byte vectors of weight/grad (f16/bf16/f32) plus the
// fp32 optimizer state (and fp32 master weights under multi-precision).
// LAMB's per-parameter trust ratio needs per-segment norms: a chunk table built
// once on the host maps 16K-element chunks to segments; each block reduces its
// chunk in registers + LDS to one partial per chunk, and a finalize kernel sums
// each segment's (contiguous) chunk partials in a fixed order -- no float
// atomics, so the norms (and the update) are bitwise reproducible.
#include <stdexcept>

#include "common.h"

namespace mxamd {

namespace {

// Plain (cached) loads and stores for the optimizer state: a non-temporal policy was measured slower
// on BERT b32 (465k -> 459k tok/s with nt loads, 430k with nt loads + stores; profiles/r5ac_*).
template <typename T>
__device__ __forceinline__ void ldv(const T* p, float (&v)[8]) {
  Vec8<T> t;
  t.load(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = t.get(i);
}
template <typename T>
__device__ __forceinline__ void stv(T* p, const float (&v)[8]) {
  Vec8<T> t;
#pragma unroll
  for (int i = 0; i < 8; ++i) t.set(i, v[i]);
  t.store(p);
}

constexpr int kAdam = 0;   // g += wd*w ; w -= lr * m / (sqrt(v) + eps)
constexpr int kAdamW = 1;  // w -= eta * (lr * m / (sqrt(v) + eps) + wd * w)

template <typename T, int MODE, bool MP>
__global__ void __launch_bounds__(256) flat_adam_kernel(T* __restrict__ w, const T* __restrict__ grad,
                                                        float* __restrict__ mean, float* __restrict__ var,
                                                        float* __restrict__ w32, int64_t nvec, float lr, float beta1,
                                                        float beta2, float eps, float wd, float eta, float rescale,
                                                        float clip, const float* __restrict__ hp) {
  if (hp != nullptr) lr = hp[0];   // device hyper-parameters (HIP-graph replay): bias-corrected lr
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int64_t off = v * 8;
    float g[8], wt[8], m[8], s[8];
    ldv(grad + off, g);
    if (MP) ldv(w32 + off, wt);
    else ldv(w + off, wt);
    ldv(mean + off, m);
    ldv(var + off, s);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float gi = g[i] * rescale;
      if (MODE == kAdam) gi += wd * wt[i];   // adam_update clips AFTER adding wd*w
      if (clip >= 0.f) gi = fminf(fmaxf(gi, -clip), clip);
      m[i] = beta1 * m[i] + (1.f - beta1) * gi;
      s[i] = beta2 * s[i] + (1.f - beta2) * gi * gi;
      const float upd = lr * m[i] / (sqrtf(s[i]) + eps);
      if (MODE == kAdam) wt[i] -= upd;
      else wt[i] -= eta * (upd + wd * wt[i]);
    }
    stv(mean + off, m);
    stv(var + off, s);
    if (MP) stv(w32 + off, wt);
    stv(w + off, wt);
  }
}

struct Chunk {
  int64_t start;  // element offset (multiple of 8)
  int len;        // elements (multiple of 8)
  int seg;
};

// LAMB phase 1: m, v update and r = mhat / (sqrt(vhat) + eps) + wd * w written to `upd`
// (fp32, arena-sized); per-segment sum(w^2) -> nrm[2*seg], sum(r^2) -> nrm[2*seg+1]
template <typename T, bool MP>
__global__ void __launch_bounds__(256) lamb_phase1_kernel(const T* __restrict__ w, const T* __restrict__ grad,
                                                          float* __restrict__ mean, float* __restrict__ var,
                                                          const float* __restrict__ w32, float* __restrict__ upd,
                                                          const Chunk* __restrict__ chunks, float* __restrict__ cpart,
                                                          float beta1, float beta2, float eps, float bc1, float bc2,
                                                          float wd, float rescale, float clip,
                                                          const float* __restrict__ hp) {
  if (hp != nullptr) {   // hp = {lr, bc1, bc2} written before a HIP-graph replay
    bc1 = hp[1];
    bc2 = hp[2];
  }
  const Chunk ck = chunks[blockIdx.x];
  float sw = 0.f, sr = 0.f;
  for (int i8 = threadIdx.x * 8; i8 < ck.len; i8 += 256 * 8) {
    const int64_t off = ck.start + i8;
    float g[8], wt[8], m[8], s[8], r[8];
    ldv(grad + off, g);
    if (MP) ldv(w32 + off, wt);
    else ldv(w + off, wt);
    ldv(mean + off, m);
    ldv(var + off, s);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float gi = g[i] * rescale;
      if (clip >= 0.f) gi = fminf(fmaxf(gi, -clip), clip);
      m[i] = beta1 * m[i] + (1.f - beta1) * gi;
      s[i] = beta2 * s[i] + (1.f - beta2) * gi * gi;
      r[i] = (m[i] / bc1) / (sqrtf(s[i] / bc2) + eps) + wd * wt[i];
      sw += wt[i] * wt[i];
      sr += r[i] * r[i];
    }
    stv(mean + off, m);
    stv(var + off, s);
    stv(upd + off, r);
  }
  sw = wave_sum(sw);
  sr = wave_sum(sr);
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wid] = sw;
    red[1][wid] = sr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {   // this chunk's partials; seg_finalize_kernel sums them per segment
    cpart[2 * blockIdx.x] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    cpart[2 * blockIdx.x + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

// Per-segment totals of per-chunk partials (W values per chunk, out[W*seg + v]).  The block of a
// segment's first chunk reduces the segment: thread t sums chunks first+t, first+t+256, ... while
// they belong to the segment, then a fixed-order wave / LDS tree -- the result never depends on
// scheduling.  Blocks of other chunks exit at once.
template <int W>
__global__ void __launch_bounds__(256) seg_finalize_kernel(const Chunk* __restrict__ chunks, int nchunks,
                                                           const float* __restrict__ cpart, float* __restrict__ out) {
  const int first = blockIdx.x;
  const int seg = chunks[first].seg;
  if (first > 0 && chunks[first - 1].seg == seg) return;
  float acc[W];
#pragma unroll
  for (int v = 0; v < W; ++v) acc[v] = 0.f;
  for (int j = first + threadIdx.x; j < nchunks && chunks[j].seg == seg; j += 256) {
#pragma unroll
    for (int v = 0; v < W; ++v) acc[v] += cpart[W * j + v];
  }
  __shared__ float red[W][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int v = 0; v < W; ++v) {
    const float t = wave_sum(acc[v]);
    if (lane == 0) red[v][wid] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int v = 0; v < W; ++v) out[W * seg + v] = (red[v][0] + red[v][1]) + (red[v][2] + red[v][3]);
  }
}

// LAMB phase 2: w -= lr * ratio(seg) * r, ratio = ||w|| / ||r|| (clamped to [lb, ub] on ||w||; 1 if a norm is 0)
template <typename T, bool MP>
__global__ void __launch_bounds__(256) lamb_phase2_kernel(T* __restrict__ w, float* __restrict__ w32,
                                                          const float* __restrict__ upd,
                                                          const Chunk* __restrict__ chunks,
                                                          const float* __restrict__ nrm, float lr, float lb,
                                                          float ub, const float* __restrict__ hp) {
  if (hp != nullptr) lr = hp[0];
  const Chunk ck = chunks[blockIdx.x];
  float r1 = sqrtf(nrm[2 * ck.seg]);
  const float r2 = sqrtf(nrm[2 * ck.seg + 1]);
  if (lb >= 0.f) r1 = fmaxf(r1, lb);
  if (ub >= 0.f) r1 = fminf(r1, ub);
  const float ratio = (r1 == 0.f || r2 == 0.f) ? 1.f : r1 / r2;
  const float step = lr * ratio;
  for (int i8 = threadIdx.x * 8; i8 < ck.len; i8 += 256 * 8) {
    const int64_t off = ck.start + i8;
    float wt[8], r[8];
    if (MP) ldv(w32 + off, wt);
    else ldv(w + off, wt);
    ldv(upd + off, r);
#pragma unroll
    for (int i = 0; i < 8; ++i) wt[i] -= step * r[i];
    if (MP) stv(w32 + off, wt);
    stv(w + off, wt);
  }
}

// per-chunk sum of squares (multi_sum_sq over an arena): cpart[chunk] = sum(x^2); totals per segment
// by seg_finalize_kernel<1>
template <typename T>
__global__ void __launch_bounds__(256) seg_sumsq_kernel(const T* __restrict__ x, const Chunk* __restrict__ chunks,
                                                        float* __restrict__ cpart) {
  const Chunk ck = chunks[blockIdx.x];
  float s = 0.f;
  for (int i8 = threadIdx.x * 8; i8 < ck.len; i8 += 256 * 8) {
    float v[8];
    ldv(x + ck.start + i8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i] * v[i];
  }
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) cpart[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// flag[0] = 0 when any element is inf/nan (flag preset to 1 by the caller)
template <typename T>
__global__ void __launch_bounds__(256) all_finite_kernel(const T* __restrict__ x, int64_t nvec, float scale,
                                                         int* __restrict__ flag) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  bool ok = true;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float a[8];
    ldv(x + v * 8, a);
#pragma unroll
    for (int i = 0; i < 8; ++i) ok = ok && isfinite(a[i] * scale);
  }
  if (!ok) *flag = 0;
}

inline int flat_blocks(int64_t nvec) {
  int64_t b = (nvec + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

#define MXAMD_OPT_DTYPE(dtype, ...)                                   \
  if (dtype == kF16) { typedef __half T; __VA_ARGS__; }               \
  else if (dtype == kBF16) { typedef __hip_bfloat16 T; __VA_ARGS__; } \
  else { typedef float T; __VA_ARGS__; }

}  // namespace

void flat_adam(int dtype, int mode, void* w, const void* g, float* mean, float* var, float* w32, int64_t n, float lr,
               float beta1, float beta2, float eps, float wd, float eta, float rescale, float clip, const float* hp,
               hipStream_t s) {
  MXAMD_HOST_CHECK(n % 8 == 0, "flat_adam: arena length must be a multiple of 8");
  const int64_t nvec = n / 8;
  dim3 grid(flat_blocks(nvec));
#define L(MODE, MP) hipLaunchKernelGGL((flat_adam_kernel<T, MODE, MP>), grid, dim3(256), 0, s, static_cast<T*>(w), \
                                       static_cast<const T*>(g), mean, var, w32, nvec, lr, beta1, beta2, eps, wd, eta, \
                                       rescale, clip, hp)
  MXAMD_OPT_DTYPE(dtype, {
    if (mode == kAdam) {
      if (w32) L(kAdam, true); else L(kAdam, false);
    } else {
      if (w32) L(kAdamW, true); else L(kAdamW, false);
    }
  })
#undef L
}

// zero a small fp32 buffer with a kernel (a plain kernel node when the launch is HIP-graph captured)
__global__ void __launch_bounds__(256) zero_f32_kernel(float* __restrict__ p, int n) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) p[i] = 0.f;
}

static void zero_f32(float* p, int n, hipStream_t s) {
  int blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks > 0) hipLaunchKernelGGL(zero_f32_kernel, dim3(blocks), dim3(256), 0, s, p, n);
}

// chunks: device array of (start, len, seg) triples (int64, int32, int32 -> 16 bytes each);
// nrm: 2*nseg per-segment norms followed by 2*nchunks per-chunk partials (workspace)
void lamb_update(int dtype, void* w, const void* g, float* mean, float* var, float* w32, float* upd,
                 const void* chunks, int nchunks, float* nrm, int nseg, float lr, float beta1, float beta2, float eps,
                 float bc1, float bc2, float wd, float rescale, float clip, float lb, float ub, const float* hp,
                 hipStream_t s) {
  const Chunk* ck = static_cast<const Chunk*>(chunks);
  float* cpart = nrm + 2 * nseg;
  zero_f32(nrm, 2 * nseg, s);     // segments without chunks (empty parameters) keep norm 0
  MXAMD_OPT_DTYPE(dtype, {
    if (w32) {
      hipLaunchKernelGGL((lamb_phase1_kernel<T, true>), dim3(nchunks), dim3(256), 0, s, static_cast<const T*>(w),
                         static_cast<const T*>(g), mean, var, w32, upd, ck, cpart, beta1, beta2, eps, bc1, bc2, wd,
                         rescale, clip, hp);
    } else {
      hipLaunchKernelGGL((lamb_phase1_kernel<T, false>), dim3(nchunks), dim3(256), 0, s, static_cast<const T*>(w),
                         static_cast<const T*>(g), mean, var, w32, upd, ck, cpart, beta1, beta2, eps, bc1, bc2, wd,
                         rescale, clip, hp);
    }
    hipLaunchKernelGGL(seg_finalize_kernel<2>, dim3(nchunks), dim3(256), 0, s, ck, nchunks, cpart, nrm);
    if (w32) {
      hipLaunchKernelGGL((lamb_phase2_kernel<T, true>), dim3(nchunks), dim3(256), 0, s, static_cast<T*>(w), w32, upd,
                         ck, nrm, lr, lb, ub, hp);
    } else {
      hipLaunchKernelGGL((lamb_phase2_kernel<T, false>), dim3(nchunks), dim3(256), 0, s, static_cast<T*>(w), w32, upd,
                         ck, nrm, lr, lb, ub, hp);
    }
  })
}

// out: nseg per-segment sums followed by nchunks per-chunk partials (workspace)
void seg_sumsq(int dtype, const void* x, const void* chunks, int nchunks, float* out, int nseg, hipStream_t s) {
  const Chunk* ck = static_cast<const Chunk*>(chunks);
  zero_f32(out, nseg, s);
  MXAMD_OPT_DTYPE(dtype, hipLaunchKernelGGL((seg_sumsq_kernel<T>), dim3(nchunks), dim3(256), 0, s,
                                            static_cast<const T*>(x), ck, out + nseg))
  hipLaunchKernelGGL(seg_finalize_kernel<1>, dim3(nchunks), dim3(256), 0, s, ck, nchunks, out + nseg, out);
}

__global__ void set_flag_kernel(int* __restrict__ flag) {
  if (threadIdx.x == 0) *flag = 1;
}

void all_finite(int dtype, const void* x, int64_t n, float scale, int* flag, int init, hipStream_t s) {
  MXAMD_HOST_CHECK(n % 8 == 0, "all_finite: length must be a multiple of 8");
  if (init) hipLaunchKernelGGL(set_flag_kernel, dim3(1), dim3(64), 0, s, flag);   // no memset node (graphs)
  MXAMD_OPT_DTYPE(dtype, hipLaunchKernelGGL((all_finite_kernel<T>), dim3(flat_blocks(n / 8)), dim3(256), 0, s,
                                            static_cast<const T*>(x), n / 8, scale, flag))
}

}  // namespace mxamd
