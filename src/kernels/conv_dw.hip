// Depthwise convolution (groups == channels, multiplier 1) for gfx950, channels-last (NHWC).
//
// Parity: the depthwise path of src/operator/nn/convolution.cu / depthwise_convolution-inl.h
// (MobileNet v1/v2 blocks), with dilation.  Depthwise conv does R*S MACs per output element, far
// below the MFMA roofline: it is bound by HBM, so the kernels are vector-memory kernels.
//   fwd  : one thread per (n, ho, wo, 8-channel vector); 16-byte loads/stores, consecutive threads
//          take consecutive channel vectors of one pixel (coalesced), the R*S tap weights come
//          from a host-transposed [R*S][C] copy (one 16-byte load per tap), fp32 accumulation;
//          overlapping taps of neighbouring pixels hit L1 / L2.
//   dgrad: the transposed gather (input pixel <- output pixels that read it), same layout.
//   wgrad: each thread owns one channel vector and a strided slice of the output positions,
//          keeps R*S*8 fp32 partial sums in registers, writes them to an fp32 slab row per
//          slice; a finalize kernel sums the slab rows in a fixed order (deterministic, no
//          atomics) and writes (or accumulates into) the weight gradient.
#include "common.h"

namespace mxamd {
namespace {

struct DwGeom {
  int N, H, W, C, Ho, Wo, R, S, sh, sw, ph, pw, dh, dw;
};

constexpr int kDwMaxTaps = 25;  // up to 5x5 kernels keep their partial sums in registers

template <typename T>
__global__ void __launch_bounds__(256) dw_fwd_kernel(const T* __restrict__ x, const T* __restrict__ wt,
                                                     const float* __restrict__ bias, T* __restrict__ y, DwGeom g) {
  const int CV = g.C / 8;
  const int64_t total = (int64_t)g.N * g.Ho * g.Wo * CV;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(t % CV);
    const int64_t pix = t / CV;
    const int wo = (int)(pix % g.Wo);
    const int64_t nh = pix / g.Wo;
    const int ho = (int)(nh % g.Ho), n = (int)(nh / g.Ho);
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = bias ? bias[cv * 8 + i] : 0.f;
    for (int r = 0; r < g.R; ++r) {
      const int hi = ho * g.sh - g.ph + r * g.dh;
      if (hi < 0 || hi >= g.H) continue;
      for (int s = 0; s < g.S; ++s) {
        const int wi = wo * g.sw - g.pw + s * g.dw;
        if (wi < 0 || wi >= g.W) continue;
        Vec8<T> xv, wv;
        xv.load(x + (((int64_t)n * g.H + hi) * g.W + wi) * g.C + cv * 8);
        wv.load(wt + (int64_t)(r * g.S + s) * g.C + cv * 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += xv.get(i) * wv.get(i);
      }
    }
    Vec8<T> out;
#pragma unroll
    for (int i = 0; i < 8; ++i) out.set(i, acc[i]);
    out.store(y + pix * g.C + cv * 8);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) dw_dgrad_kernel(const T* __restrict__ dy, const T* __restrict__ wt,
                                                       T* __restrict__ dx, DwGeom g) {
  const int CV = g.C / 8;
  const int64_t total = (int64_t)g.N * g.H * g.W * CV;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(t % CV);
    const int64_t pix = t / CV;
    const int wi = (int)(pix % g.W);
    const int64_t nh = pix / g.W;
    const int hi = (int)(nh % g.H), n = (int)(nh / g.H);
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    for (int r = 0; r < g.R; ++r) {
      const int hnum = hi + g.ph - r * g.dh;
      if (hnum < 0 || hnum % g.sh) continue;
      const int ho = hnum / g.sh;
      if (ho >= g.Ho) continue;
      for (int s = 0; s < g.S; ++s) {
        const int wnum = wi + g.pw - s * g.dw;
        if (wnum < 0 || wnum % g.sw) continue;
        const int wo = wnum / g.sw;
        if (wo >= g.Wo) continue;
        Vec8<T> gv, wv;
        gv.load(dy + (((int64_t)n * g.Ho + ho) * g.Wo + wo) * g.C + cv * 8);
        wv.load(wt + (int64_t)(r * g.S + s) * g.C + cv * 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += gv.get(i) * wv.get(i);
      }
    }
    Vec8<T> out;
#pragma unroll
    for (int i = 0; i < 8; ++i) out.set(i, acc[i]);
    out.store(dx + pix * g.C + cv * 8);
  }
}

// slab[slice][tap][C]: fp32 partial weight gradients of one slice of the output positions
template <typename T, int TAPS>
__global__ void __launch_bounds__(256) dw_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                       float* __restrict__ slab, int nslice, DwGeom g) {
  const int CV = g.C / 8;
  const int taps = g.R * g.S;
  const int64_t npos = (int64_t)g.N * g.Ho * g.Wo;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)nslice * CV) return;
  const int cv = (int)(t % CV);
  const int slice = (int)(t / CV);
  float acc[TAPS][8];
#pragma unroll
  for (int k = 0; k < TAPS; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[k][i] = 0.f;
  for (int64_t p = slice; p < npos; p += nslice) {
    const int wo = (int)(p % g.Wo);
    const int64_t nh = p / g.Wo;
    const int ho = (int)(nh % g.Ho), n = (int)(nh / g.Ho);
    Vec8<T> gv;
    gv.load(dy + p * g.C + cv * 8);
#pragma unroll
    for (int k = 0; k < TAPS; ++k) {
      if (k >= taps) break;
      const int r = k / g.S, s = k % g.S;
      const int hi = ho * g.sh - g.ph + r * g.dh, wi = wo * g.sw - g.pw + s * g.dw;
      if (hi < 0 || hi >= g.H || wi < 0 || wi >= g.W) continue;
      Vec8<T> xv;
      xv.load(x + (((int64_t)n * g.H + hi) * g.W + wi) * g.C + cv * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[k][i] += gv.get(i) * xv.get(i);
    }
  }
  float* row = slab + (int64_t)slice * taps * g.C + cv * 8;
#pragma unroll
  for (int k = 0; k < TAPS; ++k) {
    if (k >= taps) break;
    float4* dst = reinterpret_cast<float4*>(row + (int64_t)k * g.C);
    dst[0] = make_float4(acc[k][0], acc[k][1], acc[k][2], acc[k][3]);
    dst[1] = make_float4(acc[k][4], acc[k][5], acc[k][6], acc[k][7]);
  }
}

// out[c][tap] (the (C, R, S, 1) weight layout) = sum over slices of slab[slice][tap][c], fixed order
template <typename TO>
__global__ void __launch_bounds__(256) dw_wgrad_finalize_kernel(const float* __restrict__ slab, int nslice, int taps,
                                                                int C, TO* __restrict__ out, int accum) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= taps * C) return;
  const int k = idx / C, c = idx % C;
  float sum = 0.f;
  for (int sl = 0; sl < nslice; ++sl) sum += slab[(int64_t)sl * taps * C + idx];
  TO* dst = out + (int64_t)c * taps + k;
  if (accum) sum += static_cast<float>(*dst);
  *dst = static_cast<TO>(sum);
}

inline int blocks_for(int64_t total) {
  const int64_t b = (total + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

DwGeom make_geom(int N, int H, int W, int C, int Ho, int Wo, int R, int S, int sh, int sw, int ph, int pw, int dh,
                 int dw) {
  MXAMD_HOST_CHECK(C % 8 == 0, "depthwise conv: C must be a multiple of 8");
  MXAMD_HOST_CHECK(R * S <= kDwMaxTaps, "depthwise conv: at most 25 kernel taps");
  return DwGeom{N, H, W, C, Ho, Wo, R, S, sh, sw, ph, pw, dh, dw};
}

template <typename T>
void fwd_t(const void* x, const void* wt, const float* bias, void* y, const DwGeom& g, hipStream_t s) {
  const int64_t total = (int64_t)g.N * g.Ho * g.Wo * (g.C / 8);
  dw_fwd_kernel<T><<<blocks_for(total), 256, 0, s>>>((const T*)x, (const T*)wt, bias, (T*)y, g);
}

template <typename T>
void dgrad_t(const void* dy, const void* wt, void* dx, const DwGeom& g, hipStream_t s) {
  const int64_t total = (int64_t)g.N * g.H * g.W * (g.C / 8);
  dw_dgrad_kernel<T><<<blocks_for(total), 256, 0, s>>>((const T*)dy, (const T*)wt, (T*)dx, g);
}

template <typename T>
void wgrad_t(const void* x, const void* dy, float* slab, int nslice, int out_dtype, void* out, int accum,
             const DwGeom& g, hipStream_t s) {
  const int64_t threads = (int64_t)nslice * (g.C / 8);
  const int taps = g.R * g.S;
  if (taps <= 9)
    dw_wgrad_kernel<T, 9><<<(int)((threads + 255) / 256), 256, 0, s>>>((const T*)x, (const T*)dy, slab, nslice, g);
  else
    dw_wgrad_kernel<T, kDwMaxTaps><<<(int)((threads + 255) / 256), 256, 0, s>>>((const T*)x, (const T*)dy, slab,
                                                                                 nslice, g);
  const int fb = (taps * g.C + 255) / 256;
  switch (out_dtype) {
    case kF32: dw_wgrad_finalize_kernel<float><<<fb, 256, 0, s>>>(slab, nslice, taps, g.C, (float*)out, accum); break;
    case kF16: dw_wgrad_finalize_kernel<__half><<<fb, 256, 0, s>>>(slab, nslice, taps, g.C, (__half*)out, accum); break;
    default:
      dw_wgrad_finalize_kernel<__hip_bfloat16><<<fb, 256, 0, s>>>(slab, nslice, taps, g.C, (__hip_bfloat16*)out,
                                                                   accum);
  }
}

}  // namespace

#define MXAMD_DW_DISPATCH(dtype, FN, ...)                                        \
  switch (dtype) {                                                               \
    case kF32: FN<float>(__VA_ARGS__); break;                                    \
    case kF16: FN<__half>(__VA_ARGS__); break;                                   \
    case kBF16: FN<__hip_bfloat16>(__VA_ARGS__); break;                          \
    default: throw std::runtime_error("depthwise conv: unsupported dtype");      \
  }

// geometry: N, H, W, C, Ho, Wo, R, S, sh, sw, ph, pw, dh, dw
void conv_dw_fwd(int dtype, const void* x, const void* wt, const float* bias, void* y, const int* gm, hipStream_t s) {
  const DwGeom g = make_geom(gm[0], gm[1], gm[2], gm[3], gm[4], gm[5], gm[6], gm[7], gm[8], gm[9], gm[10], gm[11],
                             gm[12], gm[13]);
  MXAMD_DW_DISPATCH(dtype, fwd_t, x, wt, bias, y, g, s);
}

void conv_dw_dgrad(int dtype, const void* dy, const void* wt, void* dx, const int* gm, hipStream_t s) {
  const DwGeom g = make_geom(gm[0], gm[1], gm[2], gm[3], gm[4], gm[5], gm[6], gm[7], gm[8], gm[9], gm[10], gm[11],
                             gm[12], gm[13]);
  MXAMD_DW_DISPATCH(dtype, dgrad_t, dy, wt, dx, g, s);
}

void conv_dw_wgrad(int dtype, const void* x, const void* dy, float* slab, int nslice, int out_dtype, void* out,
                   int accum, const int* gm, hipStream_t s) {
  const DwGeom g = make_geom(gm[0], gm[1], gm[2], gm[3], gm[4], gm[5], gm[6], gm[7], gm[8], gm[9], gm[10], gm[11],
                             gm[12], gm[13]);
  MXAMD_DW_DISPATCH(dtype, wgrad_t, x, dy, slab, nslice, out_dtype, out, accum, g, s);
}

#undef MXAMD_DW_DISPATCH

}  // namespace mxamd
