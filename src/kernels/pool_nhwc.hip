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
// out-of-image tap reads offset 0 and is ignored), instead of in a loop with early continues
template <typename T, typename I>
__global__ void __launch_bounds__(256) pool_fwd_max3_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                            uint8_t* __restrict__ arg, PoolGeom g, I nvec,
                                                            PoolDivs dv) {
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
        const float f = vx[t].get(i);
        if (f > acc[i]) {
          acc[i] = f;
          am[i] = t;
        }
      }
    }
    Vec8<T> out;
#pragma unroll
    for (int i = 0; i < 8; ++i) out.set(i, any ? acc[i] : 0.f);
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
static void pool_fwd_t(int is_max, const void* x, void* y, uint8_t* arg, const PoolGeom& g, hipStream_t s) {
  const int64_t nvec = static_cast<int64_t>(g.N) * g.Ho * g.Wo * (g.C / 8);
  const bool small = fits32(g);
#define MXAMD_POOL_FWD(MX, I)                                                                               \
  hipLaunchKernelGGL((pool_fwd_kernel<T, MX, I>), dim3(grid_for(nvec)), dim3(256), 0, s,                     \
                     static_cast<const T*>(x), static_cast<T*>(y), arg, g, static_cast<I>(nvec),                   \
                     PoolDivs{make_pdiv(g.C / 8), make_pdiv(g.Wo), make_pdiv(g.Ho)})
  if (is_max && small && g.kh == 3 && g.kw == 3) {
    hipLaunchKernelGGL((pool_fwd_max3_kernel<T, uint32_t>), dim3(grid_for(nvec)), dim3(256), 0, s,
                       static_cast<const T*>(x), static_cast<T*>(y), arg, g, static_cast<uint32_t>(nvec),
                       PoolDivs{make_pdiv(g.C / 8), make_pdiv(g.Wo), make_pdiv(g.Ho)});
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

void pool_nhwc_forward(int dtype, int is_max, const void* x, void* y, uint8_t* arg, int N, int H, int W, int C,
                       int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int cip, hipStream_t s) {
  PoolGeom g = make_geom(N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, cip);
  if (dtype == kF16) pool_fwd_t<__half>(is_max, x, y, arg, g, s);
  else if (dtype == kBF16) pool_fwd_t<__hip_bfloat16>(is_max, x, y, arg, g, s);
  else pool_fwd_t<float>(is_max, x, y, arg, g, s);
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
