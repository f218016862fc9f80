// Deformable convolution (v1) and modulated deformable convolution (v2) for gfx950.
//
// Parity: src/operator/contrib/deformable_convolution-inl.h and nn/deformable_im2col.cuh (forward:
// deformable im2col + GEMM; backward: col2im for the data gradient, col2im_coord for the offset /
// mask gradients), modulated_deformable_convolution-inl.h for the mask (v2) variant.  Layout NCHW,
// offsets [N, dg*K*2, Ho, Wo] ((k, 0) = dh, (k, 1) = dw), mask [N, dg*K, Ho, Wo].
//
// Design: the sampling is the memory-bound part, the contraction over (C/g * K) is a plain GEMM on
// the columns, so these kernels only gather / scatter.  Two column layouts:
//   rows (f16/bf16, the GPU path): cols[n*L + l][c*K + k] -- one K-contiguous row per output pixel,
//         the operand layout of the in-tree MFMA GEMMs (gemm.hip NT for the forward and the column
//         gradient, conv_wgrad.hip TN for the weight gradient); the im2col stages a 64-pixel x CB-channel
//         tile in LDS so both the image gathers (lanes along l) and the row stores (lanes along c*K+k)
//         stay coalesced;
//   planes (fp32 operands): cols[n][c*K + k][l], contracted by torch.matmul.
// Per layout:
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

// bilinear sample of plane `im` at (h, w) (0 outside), the reference's deformable_im2col_bilinear
template <typename T>
__device__ __forceinline__ float bilinear(const T* im, int H, int W, float h, float w) {
  if (!(h > -1.f && w > -1.f && h < H && w < W)) return 0.f;
  const int hl = (int)floorf(h), wl = (int)floorf(w);
  const float lh = h - hl, lw = w - wl;
  const int hh = hl + 1, wh = wl + 1;
  const float v0 = (hl >= 0 && wl >= 0) ? ld(im + (int64_t)hl * W + wl) : 0.f;
  const float v1 = (hl >= 0 && wh <= W - 1) ? ld(im + (int64_t)hl * W + wh) : 0.f;
  const float v2 = (hh <= H - 1 && wl >= 0) ? ld(im + (int64_t)hh * W + wl) : 0.f;
  const float v3 = (hh <= H - 1 && wh <= W - 1) ? ld(im + (int64_t)hh * W + wh) : 0.f;
  return (1.f - lh) * (1.f - lw) * v0 + (1.f - lh) * lw * v1 + lh * (1.f - lw) * v2 + lh * lw * v3;
}

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


// rows layout: workgroup = (n, 64 output pixels, CB channels); wave w samples channels c0+w, c0+w+4, ...
// for its 64 lanes' pixels into an LDS tile [64][CB*K], then the tile leaves as 64 row segments of
// CB*K contiguous elements.
template <typename T, bool MASK>
__global__ void __launch_bounds__(256) deform_im2col_rows_kernel(const T* __restrict__ x, const T* __restrict__ off,
                                                                 const T* __restrict__ msk, T* __restrict__ cols,
                                                                 DeformGeom g, int CB) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* tile = reinterpret_cast<T*>(smem_raw);
  const int L = g.Ho * g.Wo, K = g.kh * g.kw;
  const int CK = g.C * K, CBK = CB * K;
  const int cpg = g.C / g.dg;
  const int ltiles = (L + 63) / 64;
  const int n = blockIdx.x / ltiles;
  const int l0 = (blockIdx.x - n * ltiles) * 64;
  const int c0 = blockIdx.y * CB;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int l = l0 + lane;
  if (l < L) {
    const int ho = l / g.Wo, wo = l - (l / g.Wo) * g.Wo;
    for (int cc = wid; cc < CB; cc += 4) {
      const int c = c0 + cc;
      if (c >= g.C) break;
      const int grp = c / cpg;
      const T* plane = x + ((int64_t)n * g.C + c) * g.H * g.W;
      const T* o = off + ((int64_t)n * g.dg + grp) * 2 * K * L + l;
      const T* m = MASK ? msk + ((int64_t)n * g.dg + grp) * K * L + l : nullptr;
      for (int k = 0; k < K; ++k) {
        const int i = k / g.kw, j = k - (k / g.kw) * g.kw;
        const float h = ho * g.sh - g.ph + i * g.dh + ld(o + (int64_t)(2 * k) * L);
        const float w = wo * g.sw - g.pw + j * g.dw + ld(o + (int64_t)(2 * k + 1) * L);
        float val = bilinear(plane, g.H, g.W, h, w);
        if (MASK) val *= ld(m + (int64_t)k * L);
        st(tile + lane * CBK + cc * K + k, val);
      }
    }
  }
  __syncthreads();
  const int cw = (g.C - c0 < CB ? g.C - c0 : CB) * K;   // valid columns of this tile
  const int nl = (L - l0 < 64 ? L - l0 : 64);
  for (int e = threadIdx.x; e < nl * CBK; e += 256) {
    const int r = e / CBK, j = e - (e / CBK) * CBK;
    if (j < cw) cols[((int64_t)n * L + l0 + r) * CK + (int64_t)c0 * K + j] = tile[r * CBK + j];
  }
}

template <typename T, bool MASK, bool ROWS>
__global__ void __launch_bounds__(256) deform_col2im_kernel(const T* __restrict__ off, const T* __restrict__ msk,
                                                            const float* __restrict__ gcols, float* __restrict__ gx,
                                                            DeformGeom g) {
  const int L = g.Ho * g.Wo, K = g.kh * g.kw;
  const int64_t total = (int64_t)g.N * g.C * K * L;
  const int cpg = g.C / g.dg;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    // planes: t = ((n*C + c)*K + k)*L + l (l fastest);  rows: t = ((n*L + l)*C + c)*K + k (k fastest),
    // in both cases t is also the column-gradient index, so gcols is read coalesced
    int l, k, c, n;
    if (ROWS) {
      k = (int)(t % K);
      const int64_t r = t / K;
      c = (int)(r % g.C);
      const int64_t nl = r / g.C;
      l = (int)(nl % L);
      n = (int)(nl / L);
    } else {
      l = (int)(t % L);
      const int64_t r = t / L;
      k = (int)(r % K);
      const int64_t nc = r / K;
      c = (int)(nc % g.C);
      n = (int)(nc / g.C);
    }
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
    float* plane = gx + ((int64_t)n * g.C + c) * g.H * g.W;
    if (hl >= 0 && wl >= 0) atomicAdd(plane + (int64_t)hl * g.W + wl, gv * (1.f - lh) * (1.f - lw));
    if (hl >= 0 && wl + 1 <= g.W - 1) atomicAdd(plane + (int64_t)hl * g.W + wl + 1, gv * (1.f - lh) * lw);
    if (hl + 1 <= g.H - 1 && wl >= 0) atomicAdd(plane + (int64_t)(hl + 1) * g.W + wl, gv * lh * (1.f - lw));
    if (hl + 1 <= g.H - 1 && wl + 1 <= g.W - 1) atomicAdd(plane + (int64_t)(hl + 1) * g.W + wl + 1, gv * lh * lw);
  }
}

template <typename T, bool MASK, bool ROWS>
__global__ void __launch_bounds__(256) deform_col2im_coord_kernel(const T* __restrict__ x, const T* __restrict__ off,
                                                                  const T* __restrict__ msk,
                                                                  const float* __restrict__ gcols, T* __restrict__ goff,
                                                                  T* __restrict__ gmsk, DeformGeom g) {
  const int L = g.Ho * g.Wo, K = g.kh * g.kw;
  const int64_t total = (int64_t)g.N * g.dg * K * L;
  const int cpg = g.C / g.dg;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    // planes: t = ((n*dg + grp)*K + k)*L + l;  rows: t = ((n*dg + grp)*L + l)*K + k (k fastest: the
    // column-gradient reads of one channel are contiguous across the wave)
    int l, k;
    int64_t ng;
    if (ROWS) {
      k = (int)(t % K);
      const int64_t r = t / K;
      l = (int)(r % L);
      ng = r / L;
    } else {
      l = (int)(t % L);
      const int64_t r = t / L;
      k = (int)(r % K);
      ng = r / K;
    }
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
        const float gv = ROWS ? gcols[((int64_t)n * L + l) * ((int64_t)g.C * K) + (int64_t)c * K + k]
                              : gcols[(((int64_t)n * g.C + c) * K + k) * L + l];
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
void im2col_t(const void* x, const void* off, const void* msk, void* cols, const DeformGeom& g, int rows,
              hipStream_t s) {
  const int64_t total = (int64_t)g.N * g.C * g.Ho * g.Wo;
  if (rows) {
    const int K = g.kh * g.kw;
    int CB = 512 / K;
    CB = CB < 1 ? 1 : (CB > 16 ? 16 : CB);
    const int L = g.Ho * g.Wo;
    const int64_t bx = (int64_t)g.N * ((L + 63) / 64);
    MXAMD_HOST_CHECK(bx < (1ll << 31), "deform_im2col: too many pixels");
    const dim3 grid((unsigned)bx, (unsigned)((g.C + CB - 1) / CB));
    const size_t smem = (size_t)64 * CB * K * sizeof(T);
    MXAMD_HOST_CHECK(smem <= 64 * 1024, "deform_im2col: kernel window too large for the LDS tile");
    if (msk)
      deform_im2col_rows_kernel<T, true><<<grid, 256, smem, s>>>((const T*)x, (const T*)off, (const T*)msk, (T*)cols,
                                                                 g, CB);
    else
      deform_im2col_rows_kernel<T, false><<<grid, 256, smem, s>>>((const T*)x, (const T*)off, nullptr, (T*)cols, g,
                                                                  CB);
    return;
  }
  if (msk)
    deform_im2col_kernel<T, true><<<grid_for(total), 256, 0, s>>>((const T*)x, (const T*)off, (const T*)msk, (T*)cols, g);
  else
    deform_im2col_kernel<T, false><<<grid_for(total), 256, 0, s>>>((const T*)x, (const T*)off, nullptr, (T*)cols, g);
}

template <typename T, bool ROWS>
void col2im_l(const void* off, const void* msk, const void* gcols, float* gx, const DeformGeom& g, hipStream_t s) {
  const int64_t total = (int64_t)g.N * g.C * g.kh * g.kw * g.Ho * g.Wo;
  if (msk)
    deform_col2im_kernel<T, true, ROWS><<<grid_for(total), 256, 0, s>>>((const T*)off, (const T*)msk,
                                                                        (const float*)gcols, gx, g);
  else
    deform_col2im_kernel<T, false, ROWS><<<grid_for(total), 256, 0, s>>>((const T*)off, nullptr, (const float*)gcols,
                                                                         gx, g);
}

template <typename T>
void col2im_t(const void* off, const void* msk, const void* gcols, float* gx, const DeformGeom& g, int rows,
              hipStream_t s) {
  if (rows) col2im_l<T, true>(off, msk, gcols, gx, g, s);
  else col2im_l<T, false>(off, msk, gcols, gx, g, s);
}

template <typename T, bool ROWS>
void coord_l(const void* x, const void* off, const void* msk, const void* gcols, void* goff, void* gmsk,
             const DeformGeom& g, hipStream_t s) {
  const int64_t total = (int64_t)g.N * g.dg * g.kh * g.kw * g.Ho * g.Wo;
  if (msk)
    deform_col2im_coord_kernel<T, true, ROWS><<<grid_for(total), 256, 0, s>>>(
        (const T*)x, (const T*)off, (const T*)msk, (const float*)gcols, (T*)goff, (T*)gmsk, g);
  else
    deform_col2im_coord_kernel<T, false, ROWS><<<grid_for(total), 256, 0, s>>>(
        (const T*)x, (const T*)off, nullptr, (const float*)gcols, (T*)goff, nullptr, g);
}

template <typename T>
void coord_t(const void* x, const void* off, const void* msk, const void* gcols, void* goff, void* gmsk,
             const DeformGeom& g, int rows, hipStream_t s) {
  if (rows) coord_l<T, true>(x, off, msk, gcols, goff, gmsk, g, s);
  else coord_l<T, false>(x, off, msk, gcols, goff, gmsk, g, s);
}


// ---------------------------------------------------------------------------------------------------
// Channels-last path (f16/bf16 training, the SSD extra layers): x [N][H][W][C], offsets [N][L][ld_off]
// (dg*2K used), mask [N][L][ld_msk] (dg*K used), columns [N*L][C*K], data gradient fp32 [N][H][W][C],
// offset / mask gradients [N][L][dg*2K] / [N][L][dg*K].  One wave per output pixel; lanes run along
// channels, so the four bilinear corners of a tap are 128-byte coalesced loads and the data-gradient
// atomics of a corner land on consecutive addresses.  Needs C / dg % 64 == 0 (a 64-channel chunk lies in
// one deformable group: the tap positions are wave-uniform) and K <= 16.
constexpr int kDfMaxK = 16;

struct DeformNhwc {
  DeformGeom g;
  int ld_off, ld_msk;
};

// tap k of pixel (ho, wo): sampling position
__device__ __forceinline__ void tap_pos(const DeformGeom& g, int ho, int wo, int k, float dh_off, float dw_off,
                                        float& h, float& w) {
  const int i = k / g.kw, j = k - (k / g.kw) * g.kw;
  h = ho * g.sh - g.ph + i * g.dh + dh_off;
  w = wo * g.sw - g.pw + j * g.dw + dw_off;
}

template <typename T, bool MASK>
__global__ void __launch_bounds__(256) deform_im2col_nhwc_kernel(const T* __restrict__ x, const T* __restrict__ off,
                                                                 const T* __restrict__ msk, T* __restrict__ cols,
                                                                 DeformNhwc a) {
  __shared__ T tile[4][64 * kDfMaxK];
  const DeformGeom& g = a.g;
  const int L = g.Ho * g.Wo, K = g.kh * g.kw;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t npix = (int64_t)g.N * L;
  const bool valid = (int64_t)blockIdx.x * 4 + wid < npix;     // wave-uniform; idle waves still meet the barriers
  const int64_t pix = valid ? (int64_t)blockIdx.x * 4 + wid : npix - 1;   // n*L + l
  const int n = (int)(pix / L), l = (int)(pix - (int64_t)(pix / L) * L);
  const int ho = l / g.Wo, wo = l - (l / g.Wo) * g.Wo;
  const int cpg = g.C / g.dg;
  const int64_t CK = (int64_t)g.C * K;
  const T* xn = x + (int64_t)n * g.H * g.W * g.C;
  const T* o = off + pix * a.ld_off;
  const T* m = MASK ? msk + pix * a.ld_msk : nullptr;
  T* t = tile[wid];
  for (int c0 = 0; c0 < g.C; c0 += 64) {
    const int c = c0 + lane;
    const int grp = c0 / cpg;
    for (int k = 0; k < K; ++k) {
      float h, w;
      tap_pos(g, ho, wo, k, ld(o + grp * 2 * K + 2 * k), ld(o + grp * 2 * K + 2 * k + 1), h, w);
      float val = 0.f;
      if (h > -1.f && w > -1.f && h < g.H && w < g.W) {
        const int hl = (int)floorf(h), wl = (int)floorf(w);
        const float lh = h - hl, lw = w - wl;
        const int hh = hl + 1, wh = wl + 1;
        const float v0 = (hl >= 0 && wl >= 0) ? ld(xn + ((int64_t)hl * g.W + wl) * g.C + c) : 0.f;
        const float v1 = (hl >= 0 && wh <= g.W - 1) ? ld(xn + ((int64_t)hl * g.W + wh) * g.C + c) : 0.f;
        const float v2 = (hh <= g.H - 1 && wl >= 0) ? ld(xn + ((int64_t)hh * g.W + wl) * g.C + c) : 0.f;
        const float v3 = (hh <= g.H - 1 && wh <= g.W - 1) ? ld(xn + ((int64_t)hh * g.W + wh) * g.C + c) : 0.f;
        val = (1.f - lh) * (1.f - lw) * v0 + (1.f - lh) * lw * v1 + lh * (1.f - lw) * v2 + lh * lw * v3;
      }
      if (MASK) val *= ld(m + grp * K + k);
      st(t + lane * K + k, val);
    }
    __syncthreads();
    T* row = cols + pix * CK + (int64_t)c0 * K;
    if (valid)
      for (int e = lane; e < 64 * K; e += 64) row[e] = t[e];
    __syncthreads();
  }
}

// Backward, one pass over the fp32 column gradient: the data gradient (4 coalesced corner atomics per
// tap) and the offset / mask gradients (per-lane partials over the group's channels, one wave reduction
// per tap at the end of each group).
template <typename T, bool MASK>
__global__ void __launch_bounds__(256) deform_bwd_nhwc_kernel(const T* __restrict__ x, const T* __restrict__ off,
                                                              const T* __restrict__ msk,
                                                              const float* __restrict__ gcols, float* __restrict__ gx,
                                                              T* __restrict__ goff, T* __restrict__ gmsk, DeformNhwc a) {
  __shared__ float tile[4][64 * kDfMaxK];
  const DeformGeom& g = a.g;
  const int L = g.Ho * g.Wo, K = g.kh * g.kw;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t npix = (int64_t)g.N * L;
  const bool valid = (int64_t)blockIdx.x * 4 + wid < npix;
  const int64_t pix = valid ? (int64_t)blockIdx.x * 4 + wid : npix - 1;
  const int n = (int)(pix / L), l = (int)(pix - (int64_t)(pix / L) * L);
  const int ho = l / g.Wo, wo = l - (l / g.Wo) * g.Wo;
  const int cpg = g.C / g.dg;
  const int64_t CK = (int64_t)g.C * K;
  const T* xn = x + (int64_t)n * g.H * g.W * g.C;
  float* gxn = gx + (int64_t)n * g.H * g.W * g.C;
  const T* o = off + pix * a.ld_off;
  const T* m = MASK ? msk + pix * a.ld_msk : nullptr;
  float* t = tile[wid];
  float acc_h[kDfMaxK], acc_w[kDfMaxK], acc_m[kDfMaxK];
#pragma unroll
  for (int k = 0; k < kDfMaxK; ++k) acc_h[k] = acc_w[k] = acc_m[k] = 0.f;
  for (int c0 = 0; c0 < g.C; c0 += 64) {
    const int c = c0 + lane;
    const int grp = c0 / cpg;
    const float* src = gcols + pix * CK + (int64_t)c0 * K;
    for (int e = lane; e < 64 * K; e += 64) t[e] = src[e];     // coalesced chunk -> LDS
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kDfMaxK; ++k) {
      // predicated, not early-exited: the loop stays fully unrolled and acc_*[k] stay in registers
      float h = -2.f, w = -2.f;
      if (k < K) tap_pos(g, ho, wo, k, ld(o + grp * 2 * K + 2 * k), ld(o + grp * 2 * K + 2 * k + 1), h, w);
      if (valid && k < K && h > -1.f && w > -1.f && h < g.H && w < g.W) {
        const float gv = t[lane * K + k];
        const float mv = MASK ? ld(m + grp * K + k) : 1.f;
        const int hl = (int)floorf(h), wl = (int)floorf(w);
        const float lh = h - hl, lw = w - wl;
        const int hh = hl + 1, wh = wl + 1;
        const bool b0 = hl >= 0 && wl >= 0, b1 = hl >= 0 && wh <= g.W - 1;
        const bool b2 = hh <= g.H - 1 && wl >= 0, b3 = hh <= g.H - 1 && wh <= g.W - 1;
        const int64_t p0 = ((int64_t)hl * g.W + wl) * g.C + c, p1 = ((int64_t)hl * g.W + wh) * g.C + c;
        const int64_t p2 = ((int64_t)hh * g.W + wl) * g.C + c, p3 = ((int64_t)hh * g.W + wh) * g.C + c;
        const float v0 = b0 ? ld(xn + p0) : 0.f, v1 = b1 ? ld(xn + p1) : 0.f;
        const float v2 = b2 ? ld(xn + p2) : 0.f, v3 = b3 ? ld(xn + p3) : 0.f;
        const float gm = gv * mv;
        if (b0) atomicAdd(gxn + p0, gm * (1.f - lh) * (1.f - lw));
        if (b1) atomicAdd(gxn + p1, gm * (1.f - lh) * lw);
        if (b2) atomicAdd(gxn + p2, gm * lh * (1.f - lw));
        if (b3) atomicAdd(gxn + p3, gm * lh * lw);
        acc_h[k] += gv * (-(1.f - lw) * v0 - lw * v1 + (1.f - lw) * v2 + lw * v3);
        acc_w[k] += gv * (-(1.f - lh) * v0 + (1.f - lh) * v1 - lh * v2 + lh * v3);
        if (MASK)
          acc_m[k] += gv * ((1.f - lh) * (1.f - lw) * v0 + (1.f - lh) * lw * v1 + lh * (1.f - lw) * v2 + lh * lw * v3);
      }
    }
    __syncthreads();
    if ((c0 + 64) % cpg == 0) {
      // end of deformable group `grp`: reduce the partials over the wave, lane 0 writes the tap gradients
#pragma unroll
      for (int k = 0; k < kDfMaxK; ++k) {
        float vh = acc_h[k], vw = acc_w[k], vm = acc_m[k];
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {
          vh += __shfl_xor(vh, s, 64);
          vw += __shfl_xor(vw, s, 64);
          if (MASK) vm += __shfl_xor(vm, s, 64);
        }
        if (valid && lane == 0 && k < K) {
          const float mv = MASK ? ld(m + grp * K + k) : 1.f;
          st(goff + pix * (2 * K * g.dg) + grp * 2 * K + 2 * k, vh * mv);
          st(goff + pix * (2 * K * g.dg) + grp * 2 * K + 2 * k + 1, vw * mv);
          if (MASK) st(gmsk + pix * (K * g.dg) + grp * K + k, vm);
        }
        acc_h[k] = acc_w[k] = acc_m[k] = 0.f;
      }
    }
  }
}

template <typename T>
void im2col_nhwc_t(const void* x, const void* off, const void* msk, void* cols, const DeformNhwc& a, hipStream_t s) {
  const int64_t pix = (int64_t)a.g.N * a.g.Ho * a.g.Wo;
  const unsigned blocks = (unsigned)((pix + 3) / 4);
  if (msk)
    deform_im2col_nhwc_kernel<T, true><<<blocks, 256, 0, s>>>((const T*)x, (const T*)off, (const T*)msk, (T*)cols, a);
  else
    deform_im2col_nhwc_kernel<T, false><<<blocks, 256, 0, s>>>((const T*)x, (const T*)off, nullptr, (T*)cols, a);
}

template <typename T>
void bwd_nhwc_t(const void* x, const void* off, const void* msk, const void* gcols, float* gx, void* goff, void* gmsk,
                const DeformNhwc& a, hipStream_t s) {
  const int64_t pix = (int64_t)a.g.N * a.g.Ho * a.g.Wo;
  const unsigned blocks = (unsigned)((pix + 3) / 4);
  if (msk)
    deform_bwd_nhwc_kernel<T, true><<<blocks, 256, 0, s>>>((const T*)x, (const T*)off, (const T*)msk,
                                                           (const float*)gcols, gx, (T*)goff, (T*)gmsk, a);
  else
    deform_bwd_nhwc_kernel<T, false><<<blocks, 256, 0, s>>>((const T*)x, (const T*)off, nullptr, (const float*)gcols,
                                                            gx, (T*)goff, nullptr, a);
}

DeformNhwc nhwc_args(const DeformGeom& g, int ld_off, int ld_msk, bool has_msk) {
  const int K = g.kh * g.kw;
  MXAMD_HOST_CHECK((g.C / g.dg) % 64 == 0, "deform (NHWC): channels per deformable group must be a multiple of 64");
  MXAMD_HOST_CHECK(K <= kDfMaxK, "deform (NHWC): at most 16 kernel taps");
  MXAMD_HOST_CHECK(ld_off >= 2 * K * g.dg && (!has_msk || ld_msk >= K * g.dg), "deform (NHWC): offset / mask row stride");
  MXAMD_HOST_CHECK((int64_t)g.N * g.Ho * g.Wo * g.C * K < (1ll << 40), "deform (NHWC): too large");
  return DeformNhwc{g, ld_off, ld_msk};
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
                   int rows, hipStream_t s) {
  const DeformGeom g = geom(N, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw, dg);
  MXAMD_DISPATCH(dtype, im2col_t, x, off, msk, cols, g, rows, s);
}

void deform_col2im(int dtype, const void* off, const void* msk, const void* gcols, float* gx, int N, int C, int H,
                   int W, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int dg,
                   int rows, hipStream_t s) {
  const DeformGeom g = geom(N, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw, dg);
  MXAMD_DISPATCH(dtype, col2im_t, off, msk, gcols, gx, g, rows, s);
}

void deform_col2im_coord(int dtype, const void* x, const void* off, const void* msk, const void* gcols, void* goff,
                         void* gmsk, int N, int C, int H, int W, int Ho, int Wo, int kh, int kw, int sh, int sw,
                         int ph, int pw, int dh, int dw, int dg, int rows, hipStream_t s) {
  const DeformGeom g = geom(N, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw, dg);
  MXAMD_DISPATCH(dtype, coord_t, x, off, msk, gcols, goff, gmsk, g, rows, s);
}

void deform_im2col_nhwc(int dtype, const void* x, const void* off, const void* msk, void* cols, const int* gv,
                        int ld_off, int ld_msk, hipStream_t s) {
  const DeformGeom g = geom(gv[0], gv[1], gv[2], gv[3], gv[4], gv[5], gv[6], gv[7], gv[8], gv[9], gv[10], gv[11],
                            gv[12], gv[13], gv[14]);
  const DeformNhwc a = nhwc_args(g, ld_off, ld_msk, msk != nullptr);
  if (dtype == kF16) im2col_nhwc_t<__half>(x, off, msk, cols, a, s);
  else if (dtype == kBF16) im2col_nhwc_t<__hip_bfloat16>(x, off, msk, cols, a, s);
  else throw std::runtime_error("deform (NHWC): dtype must be f16 or bf16");
}

void deform_bwd_nhwc(int dtype, const void* x, const void* off, const void* msk, const void* gcols, float* gx,
                     void* goff, void* gmsk, const int* gv, int ld_off, int ld_msk, hipStream_t s) {
  const DeformGeom g = geom(gv[0], gv[1], gv[2], gv[3], gv[4], gv[5], gv[6], gv[7], gv[8], gv[9], gv[10], gv[11],
                            gv[12], gv[13], gv[14]);
  const DeformNhwc a = nhwc_args(g, ld_off, ld_msk, msk != nullptr);
  if (dtype == kF16) bwd_nhwc_t<__half>(x, off, msk, gcols, gx, goff, gmsk, a, s);
  else if (dtype == kBF16) bwd_nhwc_t<__hip_bfloat16>(x, off, msk, gcols, gx, goff, gmsk, a, s);
  else throw std::runtime_error("deform (NHWC): dtype must be f16 or bf16");
}

#undef MXAMD_DISPATCH

}  // namespace mxamd
