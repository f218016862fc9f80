// Deformable convolution (v1) and modulated deformable convolution (v2) for gfx950.
//
// Parity: src/operator/contrib/deformable_convolution-inl.h and nn/deformable_im2col.cuh (forward:
// deformable im2col + GEMM; backward: col2im for the data gradient, col2im_coord for the offset /
// mask gradients), modulated_deformable_convolution-inl.h for the mask (v2) variant.  Layout NCHW,
// offsets [N, dg*K*2, Ho, Wo] ((k, 0) = dh, (k, 1) = dw), mask [N, dg*K, Ho, Wo].
//
// Design: the sampling is the memory-bound part, the contraction over (C/g * K) is a plain batched
// GEMM on the columns (hipBLASLt through torch.matmul), so these kernels only gather / scatter:
//   im2col      : one thread per (n, c, l) output position, all K taps in a register loop; for a
//                 fixed tap the threads of a wave write 64 consecutive l -> coalesced column rows,
//                 offsets / mask read coalesced along l, the bilinear corners are the only gathers.
//   col2im      : one thread per (n, c, k, l); the 4 bilinear corners are scattered into an fp32
//                 data-gradient buffer with global (vector-memory) float atomics.  The column
//                 gradients come in fp32 (the coordinate gradient is a difference of products)
//   col2im_coord: one thread per (n, group, k, l) reduces over the group's channels in registers
//                 and writes d(offset_h), d(offset_w) (and d(mask)) once -- no atomics.
// All arithmetic in fp32; storage fp32 / fp16 / bf16.
#include "common.h"

namespace mxamd {
namespace {

template <typename T>
__device__ __forceinline__ float ld(const T* p) {
  return static_cast<float>(*p);
}
template <>
__device__ __forceinline__ float ld<__half>(const __half* p) {
  return __half2float(*p);
}
template <>
__device__ __forceinline__ float ld<__hip_bfloat16>(const __hip_bfloat16* p) {
  return __uint_as_float(static_cast<uint32_t>(*reinterpret_cast<const uint16_t*>(p)) << 16);
}

template <typename T>
__device__ __forceinline__ void st(T* p, float v) {
  *p = static_cast<T>(v);
}
template <>
__device__ __forceinline__ void st<__half>(__half* p, float v) {
  *p = __float2half(v);
}
template <>
__device__ __forceinline__ void st<__hip_bfloat16>(__hip_bfloat16* p, float v) {
  *p = __float2bfloat16(v);
}

struct DeformGeom {
  int N, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw, dg;
};

// The four bilinear corner values of plane `im` around (h, w) (0 outside the image).
template <typename T>
__device__ __forceinline__ void corners(const T* im, int H, int W, int hl, int wl, float v[4]) {
  const int hh = hl + 1, wh = wl + 1;
  v[0] = (hl >= 0 && wl >= 0) ? ld(im + (int64_t)hl * W + wl) : 0.f;
  v[1] = (hl >= 0 && wh <= W - 1) ? ld(im + (int64_t)hl * W + wh) : 0.f;
  v[2] = (hh <= H - 1 && wl >= 0) ? ld(im + (int64_t)hh * W + wl) : 0.f;
  v[3] = (hh <= H - 1 && wh <= W - 1) ? ld(im + (int64_t)hh * W + wh) : 0.f;
}

template <typename T, bool MASK>
__global__ void __launch_bounds__(256) deform_im2col_kernel(const T* __restrict__ x, const T* __restrict__ off,
                                                            const T* __restrict__ msk, T* __restrict__ cols,
                                                            DeformGeom g) {
  const int L = g.Ho * g.Wo, K = g.kh * g.kw;
  const int64_t total = (int64_t)g.N * g.C * L;
  const int cpg = g.C / g.dg;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(t % L);
    const int64_t nc = t / L;
    const int c = (int)(nc % g.C), n = (int)(nc / g.C);
    const int grp = c / cpg;
    const int ho = l / g.Wo, wo = l % g.Wo;
    const T* plane = x + ((int64_t)n * g.C + c) * g.H * g.W;
    const T* o = off + ((int64_t)n * g.dg + grp) * 2 * K * L + l;
    const T* m = MASK ? msk + ((int64_t)n * g.dg + grp) * K * L + l : nullptr;
    T* out = cols + nc * K * L + l;
    for (int k = 0; k < K; ++k) {
      const int i = k / g.kw, j = k % g.kw;
      const float h = ho * g.sh - g.ph + i * g.dh + ld(o + (int64_t)(2 * k) * L);
      const float w = wo * g.sw - g.pw + j * g.dw + ld(o + (int64_t)(2 * k + 1) * L);
      float val = 0.f;
      if (h > -1.f && w > -1.f && h < g.H && w < g.W) {
        const int hl = (int)floorf(h), wl = (int)floorf(w);
        const float lh = h - hl, lw = w - wl;
        float v[4];
        corners(plane, g.H, g.W, hl, wl, v);
        val = (1.f - lh) * (1.f - lw) * v[0] + (1.f - lh) * lw * v[1] + lh * (1.f - lw) * v[2] + lh * lw * v[3];
      }
      if (MASK) val *= ld(m + (int64_t)k * L);
      st(out + (int64_t)k * L, val);
    }
  }
}

template <typename T, bool MASK>
__global__ void __launch_bounds__(256) deform_col2im_kernel(const T* __restrict__ off, const T* __restrict__ msk,
                                                            const float* __restrict__ gcols, float* __restrict__ gx,
                                                            DeformGeom g) {
  const int L = g.Ho * g.Wo, K = g.kh * g.kw;
  const int64_t total = (int64_t)g.N * g.C * K * L;
  const int cpg = g.C / g.dg;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(t % L);
    const int64_t r = t / L;
    const int k = (int)(r % K);
    const int64_t nc = r / K;
    const int c = (int)(nc % g.C), n = (int)(nc / g.C);
    const int grp = c / cpg;
    const int ho = l / g.Wo, wo = l % g.Wo;
    const int i = k / g.kw, j = k % g.kw;
    const int64_t ob = ((int64_t)n * g.dg + grp) * 2 * K * L + l;
    const float h = ho * g.sh - g.ph + i * g.dh + ld(off + ob + (int64_t)(2 * k) * L);
    const float w = wo * g.sw - g.pw + j * g.dw + ld(off + ob + (int64_t)(2 * k + 1) * L);
    if (!(h > -1.f && w > -1.f && h < g.H && w < g.W)) continue;
    float gv = gcols[t];
    if (MASK) gv *= ld(msk + ((int64_t)n * g.dg + grp) * K * L + (int64_t)k * L + l);
    const int hl = (int)floorf(h), wl = (int)floorf(w);
    const float lh = h - hl, lw = w - wl;
    float* plane = gx + nc * g.H * g.W;
    if (hl >= 0 && wl >= 0) atomicAdd(plane + (int64_t)hl * g.W + wl, gv * (1.f - lh) * (1.f - lw));
    if (hl >= 0 && wl + 1 <= g.W - 1) atomicAdd(plane + (int64_t)hl * g.W + wl + 1, gv * (1.f - lh) * lw);
    if (hl + 1 <= g.H - 1 && wl >= 0) atomicAdd(plane + (int64_t)(hl + 1) * g.W + wl, gv * lh * (1.f - lw));
    if (hl + 1 <= g.H - 1 && wl + 1 <= g.W - 1) atomicAdd(plane + (int64_t)(hl + 1) * g.W + wl + 1, gv * lh * lw);
  }
}

template <typename T, bool MASK>
__global__ void __launch_bounds__(256) deform_col2im_coord_kernel(const T* __restrict__ x, const T* __restrict__ off,
                                                                  const T* __restrict__ msk,
                                                                  const float* __restrict__ gcols, T* __restrict__ goff,
                                                                  T* __restrict__ gmsk, DeformGeom g) {
  const int L = g.Ho * g.Wo, K = g.kh * g.kw;
  const int64_t total = (int64_t)g.N * g.dg * K * L;
  const int cpg = g.C / g.dg;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(t % L);
    const int64_t r = t / L;
    const int k = (int)(r % K);
    const int64_t ng = r / K;
    const int grp = (int)(ng % g.dg), n = (int)(ng / g.dg);
    const int ho = l / g.Wo, wo = l % g.Wo;
    const int i = k / g.kw, j = k % g.kw;
    const int64_t ob = ng * 2 * K * L + l;
    const float h = ho * g.sh - g.ph + i * g.dh + ld(off + ob + (int64_t)(2 * k) * L);
    const float w = wo * g.sw - g.pw + j * g.dw + ld(off + ob + (int64_t)(2 * k + 1) * L);
    const float mv = MASK ? ld(msk + ng * K * L + (int64_t)k * L + l) : 1.f;
    float acc_h = 0.f, acc_w = 0.f, acc_m = 0.f;
    if (h > -1.f && w > -1.f && h < g.H && w < g.W) {
      const int hl = (int)floorf(h), wl = (int)floorf(w);
      const float lh = h - hl, lw = w - wl;
      for (int cc = 0; cc < cpg; ++cc) {
        const int c = grp * cpg + cc;
        const T* plane = x + ((int64_t)n * g.C + c) * g.H * g.W;
        const float gv = gcols[(((int64_t)n * g.C + c) * K + k) * L + l];
        float v[4];
        corners(plane, g.H, g.W, hl, wl, v);
        // d(bilinear)/dh and d(bilinear)/dw
        acc_h += gv * (-(1.f - lw) * v[0] - lw * v[1] + (1.f - lw) * v[2] + lw * v[3]);
        acc_w += gv * (-(1.f - lh) * v[0] + (1.f - lh) * v[1] - lh * v[2] + lh * v[3]);
        if (MASK)
          acc_m += gv * ((1.f - lh) * (1.f - lw) * v[0] + (1.f - lh) * lw * v[1] + lh * (1.f - lw) * v[2] +
                         lh * lw * v[3]);
      }
    }
    st(goff + ob + (int64_t)(2 * k) * L, acc_h * mv);
    st(goff + ob + (int64_t)(2 * k + 1) * L, acc_w * mv);
    if (MASK) st(gmsk + ng * K * L + (int64_t)k * L + l, acc_m);
  }
}

inline int grid_for(int64_t total) {
  int64_t b = (total + 255) / 256;
  return (int)(b < 65536 ? (b < 1 ? 1 : b) : 65536);
}

template <typename T>
void im2col_t(const void* x, const void* off, const void* msk, void* cols, const DeformGeom& g, hipStream_t s) {
  const int64_t total = (int64_t)g.N * g.C * g.Ho * g.Wo;
  if (msk)
    deform_im2col_kernel<T, true><<<grid_for(total), 256, 0, s>>>((const T*)x, (const T*)off, (const T*)msk, (T*)cols, g);
  else
    deform_im2col_kernel<T, false><<<grid_for(total), 256, 0, s>>>((const T*)x, (const T*)off, nullptr, (T*)cols, g);
}

template <typename T>
void col2im_t(const void* off, const void* msk, const void* gcols, float* gx, const DeformGeom& g, hipStream_t s) {
  const int64_t total = (int64_t)g.N * g.C * g.kh * g.kw * g.Ho * g.Wo;
  if (msk)
    deform_col2im_kernel<T, true><<<grid_for(total), 256, 0, s>>>((const T*)off, (const T*)msk, (const float*)gcols, gx,
                                                                  g);
  else
    deform_col2im_kernel<T, false><<<grid_for(total), 256, 0, s>>>((const T*)off, nullptr, (const float*)gcols, gx, g);
}

template <typename T>
void coord_t(const void* x, const void* off, const void* msk, const void* gcols, void* goff, void* gmsk,
             const DeformGeom& g, hipStream_t s) {
  const int64_t total = (int64_t)g.N * g.dg * g.kh * g.kw * g.Ho * g.Wo;
  if (msk)
    deform_col2im_coord_kernel<T, true><<<grid_for(total), 256, 0, s>>>(
        (const T*)x, (const T*)off, (const T*)msk, (const float*)gcols, (T*)goff, (T*)gmsk, g);
  else
    deform_col2im_coord_kernel<T, false><<<grid_for(total), 256, 0, s>>>(
        (const T*)x, (const T*)off, nullptr, (const float*)gcols, (T*)goff, nullptr, g);
}

DeformGeom geom(int N, int C, int H, int W, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int dh,
                int dw, int dg) {
  MXAMD_HOST_CHECK(dg > 0 && C % dg == 0, "deformable conv: channels must divide into deformable groups");
  MXAMD_HOST_CHECK(Ho > 0 && Wo > 0 && kh > 0 && kw > 0, "deformable conv: empty output");
  return DeformGeom{N, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw, dg};
}

}  // namespace

#define MXAMD_DISPATCH(dtype, FN, ...)                                          \
  switch (dtype) {                                                              \
    case kF32: FN<float>(__VA_ARGS__); break;                                   \
    case kF16: FN<__half>(__VA_ARGS__); break;                                  \
    case kBF16: FN<__hip_bfloat16>(__VA_ARGS__); break;                         \
    default: throw std::runtime_error("deformable conv: unsupported dtype");    \
  }

void deform_im2col(int dtype, const void* x, const void* off, const void* msk, void* cols, int N, int C, int H, int W,
                   int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int dg,
                   hipStream_t s) {
  const DeformGeom g = geom(N, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw, dg);
  MXAMD_DISPATCH(dtype, im2col_t, x, off, msk, cols, g, s);
}

void deform_col2im(int dtype, const void* off, const void* msk, const void* gcols, float* gx, int N, int C, int H,
                   int W, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int dg,
                   hipStream_t s) {
  const DeformGeom g = geom(N, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw, dg);
  MXAMD_DISPATCH(dtype, col2im_t, off, msk, gcols, gx, g, s);
}

void deform_col2im_coord(int dtype, const void* x, const void* off, const void* msk, const void* gcols, void* goff,
                         void* gmsk, int N, int C, int H, int W, int Ho, int Wo, int kh, int kw, int sh, int sw,
                         int ph, int pw, int dh, int dw, int dg, hipStream_t s) {
  const DeformGeom g = geom(N, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw, dg);
  MXAMD_DISPATCH(dtype, coord_t, x, off, msk, gcols, goff, gmsk, g, s);
}

#undef MXAMD_DISPATCH

}  // namespace mxamd
