// NHWC 2-D max / average pooling for gfx950 (forward + backward).
//
// Parity: src/operator/nn/pooling.cc / cudnn_pooling (pool_type max|avg,
// pooling_convention valid|full, count_include_pad).
//
// Memory-bound: every thread owns 8 consecutive channels (one 16-byte
// vector) of one output (forward) or one input (backward) pixel.
//   max forward : y = max over the window, plus a uint8 window index per
//                 element (the argmax) so the backward never re-reads x.
//   max backward: gather form — each input element sums dy of the (few)
//                 windows that cover it and chose it; no atomics, no memset.
//   avg         : forward averages, backward gathers dy / count.
#include <stdexcept>
#include "common.h"

namespace mxamd {

struct PoolGeom {
  int N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw;
  int count_include_pad;
};

// n / d by multiply-high for n < 2^31 (the uint32_t kernels): the three index divisions per vector are
// otherwise ~30-instruction integer routines each, and the stem pooling backward was instruction-bound
struct PDiv {
  uint32_t m, s;
};

static inline PDiv make_pdiv(uint32_t d) {
  // divisors are positive extents below 2^31 (host-checked by the launchers and pool_ok)
  if (d == 0 || d > (1u << 31)) throw std::runtime_error("pool_nhwc: divisor out of range");
  PDiv f;
  f.s = 0;
  while ((1u << f.s) < d) ++f.s;
  f.m = static_cast<uint32_t>((((uint64_t)1 << 32) * (((uint64_t)1 << f.s) - d)) / d + 1);
  return f;
}

struct PoolDivs {
  PDiv cv, w, h;   // C/8, the pixel row length and the column height of the indexed grid
};

template <typename I>
__device__ __forceinline__ void pool_split(I v, I cv, int W, int H, const PoolDivs& dv, int& c8, int& w, int& h,
                                           int& n) {
  if constexpr (sizeof(I) == 4) {
    const uint32_t p = (__umulhi(v, dv.cv.m) + v) >> dv.cv.s;
    c8 = static_cast<int>(v - p * cv) * 8;
    const uint32_t q = (__umulhi(p, dv.w.m) + p) >> dv.w.s;
    w = static_cast<int>(p - q * static_cast<uint32_t>(W));
    const uint32_t r = (__umulhi(q, dv.h.m) + q) >> dv.h.s;
    h = static_cast<int>(q - r * static_cast<uint32_t>(H));
    n = static_cast<int>(r);
  } else {
    c8 = static_cast<int>(v % cv) * 8;
    I p = v / cv;
    w = static_cast<int>(p % static_cast<I>(W));
    p /= static_cast<I>(W);
    h = static_cast<int>(p % static_cast<I>(H));
    n = static_cast<int>(p / static_cast<I>(H));
  }
}

// I: the index type -- uint32_t whenever every element offset fits (the pixel / channel decomposition
// of each vector index is 3 divisions; 64-bit ones are software routines that made the ResNet-50
// stem pooling backward instruction-bound at ~2 TB/s)
template <typename T, bool MAX, typename I>
__global__ void __launch_bounds__(256) pool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                       uint8_t* __restrict__ arg, PoolGeom g, I nvec, PoolDivs dv) {
  const I cv = static_cast<I>(g.C / 8);
  for (I v = static_cast<I>(blockIdx.x) * blockDim.x + threadIdx.x; v < nvec;
       v += static_cast<I>(gridDim.x) * blockDim.x) {
    int c8, wo, ho, n;
    pool_split<I>(v, cv, g.Wo, g.Ho, dv, c8, wo, ho, n);
    const int h0 = ho * g.sh - g.ph, w0 = wo * g.sw - g.pw;
    float acc[8];
    uint8_t am[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc[i] = MAX ? -INFINITY : 0.f;
      am[i] = 0;
    }
    int cnt = 0;
    for (int a = 0; a < g.kh; ++a) {
      const int h = h0 + a;
      if ((unsigned)h >= (unsigned)g.H) continue;
      for (int b = 0; b < g.kw; ++b) {
        const int w = w0 + b;
        if ((unsigned)w >= (unsigned)g.W) continue;
        Vec8<T> vx;
        vx.load(x + ((static_cast<I>(n) * g.H + h) * g.W + w) * g.C + c8);
        ++cnt;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float f = vx.get(i);
          if (MAX) {
            if (f > acc[i]) {
              acc[i] = f;
              am[i] = static_cast<uint8_t>(a * g.kw + b);
            }
          } else {
            acc[i] += f;
          }
        }
      }
    }
    Vec8<T> out;
    if (MAX) {
#pragma unroll
      for (int i = 0; i < 8; ++i) out.set(i, cnt ? acc[i] : 0.f);   // empty window (full convention edge)
      uint2 packed;
      packed.x = am[0] | (am[1] << 8) | (am[2] << 16) | (static_cast<uint32_t>(am[3]) << 24);
      packed.y = am[4] | (am[5] << 8) | (am[6] << 16) | (static_cast<uint32_t>(am[7]) << 24);
      *reinterpret_cast<uint2*>(arg + static_cast<int64_t>(v) * 8) = packed;
    } else {
      int den = cnt;
      if (g.count_include_pad) {
        const int he = min(h0 + g.kh, g.H + g.ph), we = min(w0 + g.kw, g.W + g.pw);
        den = (he - h0) * (we - w0);
      }
      const float inv = den > 0 ? 1.f / den : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) out.set(i, acc[i] * inv);
    }
    out.store(y + static_cast<int64_t>(v) * 8);
  }
}

template <typename T, bool MAX, typename I>
__global__ void __launch_bounds__(256) pool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                       T* __restrict__ dx, PoolGeom g, I nvec, PoolDivs dv) {
  const I cv = static_cast<I>(g.C / 8);
  for (I v = static_cast<I>(blockIdx.x) * blockDim.x + threadIdx.x; v < nvec;
       v += static_cast<I>(gridDim.x) * blockDim.x) {
    int c8, w, h, n;
    pool_split<I>(v, cv, g.W, g.H, dv, c8, w, h, n);
    // output windows covering (h, w): ho*sh - ph <= h <= ho*sh - ph + kh - 1
    const int hp = h + g.ph, wp = w + g.pw;
    const int ho_lo = hp - g.kh + 1 > 0 ? (hp - g.kh + g.sh) / g.sh : 0;
    const int ho_hi = min(hp / g.sh, g.Ho - 1);
    const int wo_lo = wp - g.kw + 1 > 0 ? (wp - g.kw + g.sw) / g.sw : 0;
    const int wo_hi = min(wp / g.sw, g.Wo - 1);
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const I o = ((static_cast<I>(n) * g.Ho + ho) * g.Wo + wo) * g.C + c8;
        Vec8<T> vd;
        vd.load(dy + o);
        if (MAX) {
          const int idx = (h - (ho * g.sh - g.ph)) * g.kw + (w - (wo * g.sw - g.pw));
          const uint2 packed = *reinterpret_cast<const uint2*>(arg + o);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const uint32_t word = i < 4 ? packed.x : packed.y;
            const int a = (word >> ((i & 3) * 8)) & 0xff;
            if (a == idx) acc[i] += vd.get(i);
          }
        } else {
          const int h0 = ho * g.sh - g.ph, w0 = wo * g.sw - g.pw;
          int den;
          if (g.count_include_pad) {
            const int he = min(h0 + g.kh, g.H + g.ph), we = min(w0 + g.kw, g.W + g.pw);
            den = (he - h0) * (we - w0);
          } else {
            const int hs = max(h0, 0), ws = max(w0, 0);
            const int he = min(h0 + g.kh, g.H), we = min(w0 + g.kw, g.W);
            den = (he - hs) * (we - ws);
          }
          const float inv = den > 0 ? 1.f / den : 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[i] += vd.get(i) * inv;
        }
      }
    }
    Vec8<T> out;
#pragma unroll
    for (int i = 0; i < 8; ++i) out.set(i, acc[i]);
    out.store(dx + static_cast<int64_t>(v) * 8);
  }
}

// max forward over a 3x3 window (the ResNet stem): the nine taps are loaded together, predicated (an
// out-of-image tap reads offset 0 and is ignored), instead of in a loop with early continues.
// AFF: the window's input is relu(x * scale[c] + shift[c]) -- the BatchNorm + ReLU in front of the stem
// pooling applied to each tap on the fly (max and ReLU commute, out-of-image taps stay excluded), so the
// normalised activation is never written or re-read; the argmax indexes the largest affine value.
template <typename T, typename I, bool AFF>
__global__ void __launch_bounds__(256) pool_fwd_max3_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                            uint8_t* __restrict__ arg, PoolGeom g, I nvec,
                                                            PoolDivs dv, const float* __restrict__ scale,
                                                            const float* __restrict__ shift) {
  const I cv = static_cast<I>(g.C / 8);
  for (I v = static_cast<I>(blockIdx.x) * blockDim.x + threadIdx.x; v < nvec;
       v += static_cast<I>(gridDim.x) * blockDim.x) {
    int c8, wo, ho, n;
    pool_split<I>(v, cv, g.Wo, g.Ho, dv, c8, wo, ho, n);
    const int h0 = ho * g.sh - g.ph, w0 = wo * g.sw - g.pw;
    Vec8<T> vx[9];
    bool ok[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int h = h0 + t / 3, w = w0 + t % 3;
      ok[t] = (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
      const I o = ok[t] ? ((static_cast<I>(n) * g.H + h) * g.W + w) * g.C + c8 : static_cast<I>(0);
      vx[t].load(x + o);
    }
    float sc[8], sf[8];
    if (AFF) {
      const float4 a0 = *reinterpret_cast<const float4*>(scale + c8);
      const float4 a1 = *reinterpret_cast<const float4*>(scale + c8 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(shift + c8);
      const float4 b1 = *reinterpret_cast<const float4*>(shift + c8 + 4);
      sc[0] = a0.x; sc[1] = a0.y; sc[2] = a0.z; sc[3] = a0.w; sc[4] = a1.x; sc[5] = a1.y; sc[6] = a1.z; sc[7] = a1.w;
      sf[0] = b0.x; sf[1] = b0.y; sf[2] = b0.z; sf[3] = b0.w; sf[4] = b1.x; sf[5] = b1.y; sf[6] = b1.z; sf[7] = b1.w;
    }
    float acc[8];
    uint32_t am[8];
    bool any = false;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc[i] = -INFINITY;
      am[i] = 0;
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (!ok[t]) continue;
      any = true;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float f = AFF ? fmaf(vx[t].get(i), sc[i], sf[i]) : vx[t].get(i);
        if (f > acc[i]) {
          acc[i] = f;
          am[i] = t;
        }
      }
    }
    Vec8<T> out;
#pragma unroll
    for (int i = 0; i < 8; ++i) out.set(i, any ? (AFF ? fmaxf(acc[i], 0.f) : acc[i]) : 0.f);
    uint2 packed;
    packed.x = am[0] | (am[1] << 8) | (am[2] << 16) | (am[3] << 24);
    packed.y = am[4] | (am[5] << 8) | (am[6] << 16) | (am[7] << 24);
    *reinterpret_cast<uint2*>(arg + static_cast<int64_t>(v) * 8) = packed;
    out.store(y + static_cast<int64_t>(v) * 8);
  }
}

// max backward when at most 2 x 2 windows cover an input pixel (kernel <= 2 * stride per axis: the
// ResNet stem's 3x3 / stride 2): the four candidate windows' dy and argmax words are loaded together,
// predicated, instead of in a variable-trip loop of dependent loads
template <typename T, typename I>
__global__ void __launch_bounds__(256) pool_bwd_max2_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                            T* __restrict__ dx, PoolGeom g, I nvec, PoolDivs dv) {
  const I cv = static_cast<I>(g.C / 8);
  for (I v = static_cast<I>(blockIdx.x) * blockDim.x + threadIdx.x; v < nvec;
       v += static_cast<I>(gridDim.x) * blockDim.x) {
    int c8, w, h, n;
    pool_split<I>(v, cv, g.W, g.H, dv, c8, w, h, n);
    const int ho_hi = min((h + g.ph) / g.sh, g.Ho - 1);
    const int wo_hi = min((w + g.pw) / g.sw, g.Wo - 1);
    Vec8<T> vd[4];
    uint2 pk[4];
    int idx[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ho = ho_hi - (t >> 1), wo = wo_hi - (t & 1);
      const int dh = h - (ho * g.sh - g.ph), dw = w - (wo * g.sw - g.pw);
      const bool ok = ho >= 0 && wo >= 0 && dh >= 0 && dh < g.kh && dw >= 0 && dw < g.kw;
      idx[t] = ok ? dh * g.kw + dw : -1;
      const I o = ok ? ((static_cast<I>(n) * g.Ho + ho) * g.Wo + wo) * g.C + c8 : static_cast<I>(0);
      vd[t].load(dy + o);
      pk[t] = *reinterpret_cast<const uint2*>(arg + o);
    }
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t word = i < 4 ? pk[t].x : pk[t].y;
        const int a = (word >> ((i & 3) * 8)) & 0xff;
        if (a == idx[t]) acc[i] += vd[t].get(i);
      }
    }
    Vec8<T> out;
#pragma unroll
    for (int i = 0; i < 8; ++i) out.set(i, acc[i]);
    out.store(dx + static_cast<int64_t>(v) * 8);
  }
}

// ---- BatchNorm + ReLU + max pooling backward (the stem; forward: pool_fwd_max3_kernel<AFF>)
// Gather form per input vector (8 channels of one pixel, as pool_bwd_max2_kernel): the pooled gradient
// routed to it through the <= 2 x 2 covering windows whose argmax chose it, masked by the ReLU recomputed
// from x (dz = routed * [x * scale + shift > 0]).
//   STATS: per-channel sum(dz), sum(dz * (x - mean)) -> channel-major partials [2][C][gridDim.x]; every
//          thread keeps one channel group (blockDim 256 and the grid stride are multiples of C / 8)
//   else : dx = A * dz + B * x + Cc (the BatchNorm backward, coefficients from bn_finalize_backward)
// The dense routed gradient is never written: one gather pass for the statistics and one for dx replace
// the pooling backward's dense write plus the BatchNorm backward's reduction and apply passes.
template <typename T, bool STATS>
__global__ void __launch_bounds__(256) bnpool_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                         const uint8_t* __restrict__ arg, const float* __restrict__ k0,
                                                         const float* __restrict__ k1, const float* __restrict__ k2,
                                                         const float* __restrict__ k3, const float* __restrict__ k4,
                                                         T* __restrict__ dx, float* __restrict__ part, PoolGeom g,
                                                         uint32_t nvec, PoolDivs dv) {
  // STATS: k0 = mean, k1 = fscale, k2 = fshift;  apply: k0 = A, k1 = B, k2 = Cc, k3 = fscale, k4 = fshift
  const uint32_t cv = static_cast<uint32_t>(g.C / 8);
  // C / 8 divides 256 (host-checked), so the grid stride is a multiple of it: a thread's channel group is
  // fixed and its per-channel constants are loaded once
  const int c8f = static_cast<int>((blockIdx.x * 256u + threadIdx.x) % cv) * 8;
  auto ld8c = [&](const float* p, float* o) {
    const float4 u = *reinterpret_cast<const float4*>(p + c8f);
    const float4 w = *reinterpret_cast<const float4*>(p + c8f + 4);
    o[0] = u.x; o[1] = u.y; o[2] = u.z; o[3] = u.w; o[4] = w.x; o[5] = w.y; o[6] = w.z; o[7] = w.w;
  };
  float a[8], b[8], c[8], fs[8], fh[8];
  ld8c(k0, a);
  ld8c(STATS ? k1 : k3, fs);
  ld8c(STATS ? k2 : k4, fh);
  if (!STATS) {
    ld8c(k1, b);
    ld8c(k2, c);
  }
  float s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s1[i] = 0.f;
    s2[i] = 0.f;
  }
  for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < nvec; v += gridDim.x * 256u) {
    int c8, w, h, n;
    pool_split<uint32_t>(v, cv, g.W, g.H, dv, c8, w, h, n);
    const int ho_hi = min((h + g.ph) / g.sh, g.Ho - 1);
    const int wo_hi = min((w + g.pw) / g.sw, g.Wo - 1);
    Vec8<T> vd[4];
    uint2 pk[4];
    int idx[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ho = ho_hi - (t >> 1), wo = wo_hi - (t & 1);
      const int dh = h - (ho * g.sh - g.ph), dw = w - (wo * g.sw - g.pw);
      const bool ok = ho >= 0 && wo >= 0 && dh >= 0 && dh < g.kh && dw >= 0 && dw < g.kw;
      idx[t] = ok ? dh * g.kw + dw : -1;
      const uint32_t o = ok ? ((static_cast<uint32_t>(n) * g.Ho + ho) * g.Wo + wo) * g.C + c8 : 0u;
      vd[t].load(dy + o);
      pk[t] = *reinterpret_cast<const uint2*>(arg + o);
    }
    Vec8<T> vx;
    vx.load(x + static_cast<uint32_t>(v) * 8);
    Vec8<T> out;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t word = i < 4 ? pk[t].x : pk[t].y;
        if (static_cast<int>((word >> ((i & 3) * 8)) & 0xff) == idx[t]) acc += vd[t].get(i);
      }
      const float xi = vx.get(i);
      const float dz = fmaf(xi, fs[i], fh[i]) > 0.f ? acc : 0.f;
      if (STATS) {
        s1[i] += dz;
        s2[i] += dz * (xi - a[i]);
      } else {
        out.set(i, a[i] * dz + b[i] * xi + c[i]);
      }
    }
    if (!STATS) out.store(dx + static_cast<uint32_t>(v) * 8);
  }
  if (STATS) {
    // threads tid, tid + cv, ... share a channel group: combine them through LDS, one partial per block
    __shared__ float red[2][256 * 8];
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[0][tid * 8 + i] = s1[i];
      red[1][tid * 8 + i] = s2[i];
    }
    __syncthreads();
    const int rows = 256 / static_cast<int>(cv);
    for (int q = tid; q < 2 * g.C; q += 256) {
      const int which = q / g.C, ch = q - which * g.C;
      const int grp = ch / 8, e = ch % 8;
      float sum = 0.f;
      for (int r = 0; r < rows; ++r) sum += red[which][(r * cv + grp) * 8 + e];
      part[(static_cast<int64_t>(which) * g.C + ch) * gridDim.x + blockIdx.x] = sum;
    }
  }
}

// The same for the stem's exact geometry (3x3 windows, stride 2, pad 1): a thread takes the 2 x 2 input
// pixels (2a + {0,1}, 2b + {0,1}) of one channel group, which are covered by exactly the four windows
// (a + {0,1}, b + {0,1}) -- pixel (2a, 2b) by (a, b) only, (2a + 1, 2b + 1) by all four -- so the pooled
// gradient and argmax words are gathered once per 4 pixels instead of 4 candidates per pixel.
template <typename T, bool STATS>
__global__ void __launch_bounds__(256) bnpool_bwd_s2_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                            const uint8_t* __restrict__ arg,
                                                            const float* __restrict__ k0, const float* __restrict__ k1,
                                                            const float* __restrict__ k2, const float* __restrict__ k3,
                                                            const float* __restrict__ k4, T* __restrict__ dx,
                                                            float* __restrict__ part, PoolGeom g, int Hb, int Wb,
                                                            uint32_t nvec, PoolDivs dv) {
  const uint32_t cv = static_cast<uint32_t>(g.C / 8);
  const int c8f = static_cast<int>((blockIdx.x * 256u + threadIdx.x) % cv) * 8;
  auto ld8c = [&](const float* p, float* o) {
    const float4 u = *reinterpret_cast<const float4*>(p + c8f);
    const float4 w = *reinterpret_cast<const float4*>(p + c8f + 4);
    o[0] = u.x; o[1] = u.y; o[2] = u.z; o[3] = u.w; o[4] = w.x; o[5] = w.y; o[6] = w.z; o[7] = w.w;
  };
  float ka[8], kb[8], kc[8], fs[8], fh[8];
  ld8c(k0, ka);
  ld8c(STATS ? k1 : k3, fs);
  ld8c(STATS ? k2 : k4, fh);
  if (!STATS) {
    ld8c(k1, kb);
    ld8c(k2, kc);
  }
  float s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s1[i] = 0.f;
    s2[i] = 0.f;
  }
  for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < nvec; v += gridDim.x * 256u) {
    int c8, bb, aa, n;
    pool_split<uint32_t>(v, cv, Wb, Hb, dv, c8, bb, aa, n);
    // the four covering windows (a + ta, b + tb)
    Vec8<T> vd[4];
    uint2 pk[4];
    bool wok[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ho = aa + (t >> 1), wo = bb + (t & 1);
      wok[t] = ho < g.Ho && wo < g.Wo;
      const uint32_t o = wok[t] ? ((static_cast<uint32_t>(n) * g.Ho + ho) * g.Wo + wo) * g.C + c8 : 0u;
      vd[t].load(dy + o);
      pk[t] = *reinterpret_cast<const uint2*>(arg + o);
    }
    // the four input pixels
    Vec8<T> vx[4];
    bool pok[4];
    uint32_t po[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int h = 2 * aa + (q >> 1), w = 2 * bb + (q & 1);
      pok[q] = h < g.H && w < g.W;
      po[q] = pok[q] ? ((static_cast<uint32_t>(n) * g.H + h) * g.W + w) * g.C + c8 : 0u;
      vx[q].load(x + po[q]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int dh = q >> 1, dw = q & 1;
      Vec8<T> out;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int ta = t >> 1, tb = t & 1;
          // tap of pixel q inside window t: row dh - 2 ta + 1, column dw - 2 tb + 1 (pixel (2a, .) is not in
          // window row a + 1: dh = 0, ta = 1 gives row -1)
          if (dh - 2 * ta + 1 < 0 || dw - 2 * tb + 1 < 0) continue;
          const int tap = (dh - 2 * ta + 1) * 3 + (dw - 2 * tb + 1);
          const uint32_t word = i < 4 ? pk[t].x : pk[t].y;
          if (wok[t] && static_cast<int>((word >> ((i & 3) * 8)) & 0xff) == tap) acc += vd[t].get(i);
        }
        const float xi = vx[q].get(i);
        const float dz = (pok[q] && fmaf(xi, fs[i], fh[i]) > 0.f) ? acc : 0.f;
        if (STATS) {
          s1[i] += dz;
          s2[i] += dz * (xi - ka[i]);
        } else {
          out.set(i, ka[i] * dz + kb[i] * xi + kc[i]);
        }
      }
      if (!STATS && pok[q]) out.store(dx + po[q]);
    }
  }
  if (STATS) {
    __shared__ float red[2][256 * 8];
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[0][tid * 8 + i] = s1[i];
      red[1][tid * 8 + i] = s2[i];
    }
    __syncthreads();
    const int rows = 256 / static_cast<int>(cv);
    for (int q = tid; q < 2 * g.C; q += 256) {
      const int which = q / g.C, ch = q - which * g.C;
      const int grp = ch / 8, e = ch % 8;
      float sum = 0.f;
      for (int r = 0; r < rows; ++r) sum += red[which][(r * cv + grp) * 8 + e];
      part[(static_cast<int64_t>(which) * g.C + ch) * gridDim.x + blockIdx.x] = sum;
    }
  }
}

// every element offset of x and y (and the loop index plus one grid stride) fits in 32 bits
static inline bool fits32(const PoolGeom& g) {
  const int64_t big = static_cast<int64_t>(g.N) * g.C * (g.H * static_cast<int64_t>(g.W) > g.Ho * static_cast<int64_t>(g.Wo)
                                                            ? g.H * static_cast<int64_t>(g.W)
                                                            : g.Ho * static_cast<int64_t>(g.Wo));
  // (and every vector index plus one grid stride stays below 2^31 for the multiply-high division)
  return big + 256LL * 32 * 256 * 8 < (1LL << 31);
}

static inline int grid_for(int64_t nvec) {
  int64_t b = (nvec + 255) / 256;
  return static_cast<int>(b < 256 * 32 ? b : 256 * 32);
}

template <typename T>
static void pool_fwd_t(int is_max, const void* x, void* y, uint8_t* arg, const PoolGeom& g, hipStream_t s,
                       const float* scale, const float* shift) {
  const int64_t nvec = static_cast<int64_t>(g.N) * g.Ho * g.Wo * (g.C / 8);
  const bool small = fits32(g);
  if (scale) {
    MXAMD_HOST_CHECK(is_max && small && g.kh == 3 && g.kw == 3 && shift != nullptr &&
                         reinterpret_cast<uintptr_t>(scale) % 16 == 0 && reinterpret_cast<uintptr_t>(shift) % 16 == 0,
                     "pool_nhwc: the BatchNorm+ReLU prologue is built for 3x3 max pooling (32-bit offsets, "
                     "16-byte aligned fp32 scale / shift)");
    hipLaunchKernelGGL((pool_fwd_max3_kernel<T, uint32_t, true>), dim3(grid_for(nvec)), dim3(256), 0, s,
                       static_cast<const T*>(x), static_cast<T*>(y), arg, g, static_cast<uint32_t>(nvec),
                       PoolDivs{make_pdiv(g.C / 8), make_pdiv(g.Wo), make_pdiv(g.Ho)}, scale, shift);
    return;
  }
#define MXAMD_POOL_FWD(MX, I)                                                                               \
  hipLaunchKernelGGL((pool_fwd_kernel<T, MX, I>), dim3(grid_for(nvec)), dim3(256), 0, s,                     \
                     static_cast<const T*>(x), static_cast<T*>(y), arg, g, static_cast<I>(nvec),                   \
                     PoolDivs{make_pdiv(g.C / 8), make_pdiv(g.Wo), make_pdiv(g.Ho)})
  if (is_max && small && g.kh == 3 && g.kw == 3) {
    hipLaunchKernelGGL((pool_fwd_max3_kernel<T, uint32_t, false>), dim3(grid_for(nvec)), dim3(256), 0, s,
                       static_cast<const T*>(x), static_cast<T*>(y), arg, g, static_cast<uint32_t>(nvec),
                       PoolDivs{make_pdiv(g.C / 8), make_pdiv(g.Wo), make_pdiv(g.Ho)}, nullptr, nullptr);
  } else if (is_max) {
    if (small) MXAMD_POOL_FWD(true, uint32_t); else MXAMD_POOL_FWD(true, int64_t);
  } else {
    if (small) MXAMD_POOL_FWD(false, uint32_t); else MXAMD_POOL_FWD(false, int64_t);
  }
#undef MXAMD_POOL_FWD
}

template <typename T>
static void pool_bwd_t(int is_max, const void* dy, const uint8_t* arg, void* dx, const PoolGeom& g, hipStream_t s) {
  const int64_t nvec = static_cast<int64_t>(g.N) * g.H * g.W * (g.C / 8);
  const bool small = fits32(g);
#define MXAMD_POOL_BWD(MX, I)                                                                               \
  hipLaunchKernelGGL((pool_bwd_kernel<T, MX, I>), dim3(grid_for(nvec)), dim3(256), 0, s,                     \
                     static_cast<const T*>(dy), arg, static_cast<T*>(dx), g, static_cast<I>(nvec),                 \
                     PoolDivs{make_pdiv(g.C / 8), make_pdiv(g.W), make_pdiv(g.H)})
  const bool two = (g.kh + g.sh - 1) / g.sh <= 2 && (g.kw + g.sw - 1) / g.sw <= 2;
  if (is_max && two && small) {
    hipLaunchKernelGGL((pool_bwd_max2_kernel<T, uint32_t>), dim3(grid_for(nvec)), dim3(256), 0, s,
                       static_cast<const T*>(dy), arg, static_cast<T*>(dx), g, static_cast<uint32_t>(nvec),
                       PoolDivs{make_pdiv(g.C / 8), make_pdiv(g.W), make_pdiv(g.H)});
  } else if (is_max) {
    if (small) MXAMD_POOL_BWD(true, uint32_t); else MXAMD_POOL_BWD(true, int64_t);
  } else {
    if (small) MXAMD_POOL_BWD(false, uint32_t); else MXAMD_POOL_BWD(false, int64_t);
  }
#undef MXAMD_POOL_BWD
}

static PoolGeom make_geom(int N, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw,
                          int cip) {
  MXAMD_HOST_CHECK(C % 8 == 0, "pool_nhwc: channels must be a multiple of 8");
  MXAMD_HOST_CHECK(kh * kw <= 256, "pool_nhwc: window larger than 256 elements");
  PoolGeom g{N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, cip};
  return g;
}

// scale / shift (optional, fp32 [C]): pool relu(x * scale + shift) instead of x (3x3 max pooling only)
void pool_nhwc_forward(int dtype, int is_max, const void* x, void* y, uint8_t* arg, int N, int H, int W, int C,
                       int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int cip, hipStream_t s,
                       const float* scale, const float* shift) {
  PoolGeom g = make_geom(N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, cip);
  if (dtype == kF16) pool_fwd_t<__half>(is_max, x, y, arg, g, s, scale, shift);
  else if (dtype == kBF16) pool_fwd_t<__hip_bfloat16>(is_max, x, y, arg, g, s, scale, shift);
  else pool_fwd_t<float>(is_max, x, y, arg, g, s, scale, shift);
}

void bn_finalize_backward(const float* part, int nblk, int C, int64_t R, const float* mean, const float* gamma,
                          const float* invstd, float* dgamma, float* dbeta, float* coef, int fix_gamma, int training,
                          int accum, hipStream_t s);

// Partial rows (= blocks) of the statistics pass of bn_pool_backward: 8 blocks per CU to keep enough gathers
// in flight, still few partials per channel for the finalize.
int bn_pool_bwd_blocks() { return 2048; }

// Backward of max_pool(relu(BatchNorm(x))) (3x3 windows, stride >= 2): statistics gather pass -> finalize
// (dgamma / dbeta into dgamma / dbeta, accumulated when accum; coefficients into coef[3][C]) -> dx gather pass.
// part: 2 * bn_pool_bwd_blocks() * C floats of scratch.
void bn_pool_backward(int dtype, const void* x, const void* dy, const uint8_t* arg, void* dx, const float* gamma,
                      const float* mean, const float* invstd, const float* fscale, const float* fshift, float* part,
                      float* dgamma, float* dbeta, float* coef, int N, int H, int W, int C, int Ho, int Wo, int kh,
                      int kw, int sh, int sw, int ph, int pw, int fix_gamma, int training, int accum,
                      hipStream_t s) {
  PoolGeom g = make_geom(N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, 1);
  const int cv = C / 8;
  MXAMD_HOST_CHECK(256 % cv == 0 && fits32(g) && (kh + sh - 1) / sh <= 2 && (kw + sw - 1) / sw <= 2,
                   "bn_pool_backward: C / 8 must divide 256, 32-bit offsets, windows covering <= 2 x 2");
  MXAMD_HOST_CHECK(dtype == kF16 || dtype == kBF16, "bn_pool_backward: f16 / bf16");
  const uint32_t nvec = static_cast<uint32_t>(static_cast<int64_t>(N) * H * W * cv);
  const PoolDivs dv{make_pdiv(cv), make_pdiv(W), make_pdiv(H)};
  const int nb = bn_pool_bwd_blocks();
  const int64_t R = static_cast<int64_t>(N) * H * W;
  if (kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1) {
    // 2 x 2 input pixels per thread, the four covering windows gathered once
    const int Hb = (H + 1) / 2, Wb = (W + 1) / 2;
    MXAMD_HOST_CHECK(Ho == (H - 1) / 2 + 1 && Wo == (W - 1) / 2 + 1, "bn_pool_backward: stride-2 output extent");
    const uint32_t nv4 = static_cast<uint32_t>(static_cast<int64_t>(N) * Hb * Wb * cv);
    const PoolDivs dv4{make_pdiv(cv), make_pdiv(Wb), make_pdiv(Hb)};
#define MXAMD_BNPOOL4(TT)                                                                                          \
    hipLaunchKernelGGL((bnpool_bwd_s2_kernel<TT, true>), dim3(nb), dim3(256), 0, s, static_cast<const TT*>(x),    \
                       static_cast<const TT*>(dy), arg, mean, fscale, fshift, nullptr, nullptr, nullptr, part, g, Hb, \
                       Wb, nv4, dv4);                                                                              \
    bn_finalize_backward(part, nb, C, R, mean, gamma, invstd, dgamma, dbeta, coef, fix_gamma, training, accum, s); \
    hipLaunchKernelGGL((bnpool_bwd_s2_kernel<TT, false>), dim3(grid_for(nv4)), dim3(256), 0, s,                  \
                       static_cast<const TT*>(x), static_cast<const TT*>(dy), arg, coef, coef + C, coef + 2 * C,    \
                       fscale, fshift, static_cast<TT*>(dx), nullptr, g, Hb, Wb, nv4, dv4)
    if (dtype == kF16) {
      MXAMD_BNPOOL4(__half);
    } else {
      MXAMD_BNPOOL4(__hip_bfloat16);
    }
#undef MXAMD_BNPOOL4
    return;
  }
#define MXAMD_BNPOOL(TT)                                                                                           \
  hipLaunchKernelGGL((bnpool_bwd_kernel<TT, true>), dim3(nb), dim3(256), 0, s, static_cast<const TT*>(x),         \
                     static_cast<const TT*>(dy), arg, mean, fscale, fshift, nullptr, nullptr, nullptr, part, g, nvec, \
                     dv);                                                                                          \
  bn_finalize_backward(part, nb, C, R, mean, gamma, invstd, dgamma, dbeta, coef, fix_gamma, training, accum, s);   \
  hipLaunchKernelGGL((bnpool_bwd_kernel<TT, false>), dim3(grid_for(nvec)), dim3(256), 0, s,                       \
                     static_cast<const TT*>(x), static_cast<const TT*>(dy), arg, coef, coef + C, coef + 2 * C,      \
                     fscale, fshift, static_cast<TT*>(dx), nullptr, g, nvec, dv)
  if (dtype == kF16) {
    MXAMD_BNPOOL(__half);
  } else {
    MXAMD_BNPOOL(__hip_bfloat16);
  }
#undef MXAMD_BNPOOL
}

void pool_nhwc_backward(int dtype, int is_max, const void* dy, const uint8_t* arg, void* dx, int N, int H, int W,
                        int C, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int cip,
                        hipStream_t s) {
  PoolGeom g = make_geom(N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, cip);
  if (dtype == kF16) pool_bwd_t<__half>(is_max, dy, arg, dx, g, s);
  else if (dtype == kBF16) pool_bwd_t<__hip_bfloat16>(is_max, dy, arg, dx, g, s);
  else pool_bwd_t<float>(is_max, dy, arg, dx, g, s);
}

}  // namespace mxamd
