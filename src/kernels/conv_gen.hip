// General implicit-GEMM convolution on the matrix cores (gfx950): every case the specialised
// NHWC kernels (conv_big / conv_ring / conv_glds / conv_dw / conv_stem) do not take --
// grouped (ResNeXt-style, any channels per group), dilated, 1-D / 2-D / 3-D, odd channel counts,
// fp32 -- plus transposed convolution (Deconvolution) as the data gradient of a convolution.
//
// Reference semantics: src/operator/nn/convolution-inl.h, deconvolution-inl.h:207 and the cuDNN
// wrappers cudnn_convolution-inl.h / cudnn_deconvolution-inl.h:43 (NCHW there; channels-last here).
//
// Layouts (channels last): x [N][D][H][W][C], y [N][Do][Ho][Wo][K], w [K][T][R][S][C/G].
// Three GEMM views share one kernel body (MODE):
//   0 forward : rows = output pixels,     cols = Kg output channels, k = (t, r, s, c)
//   1 dgrad   : rows = input pixels,      cols = Cg input channels,  k = (t, r, s, co); a tap
//               contributes only where (i + pad - tap*dil) divides by the stride
//   2 wgrad   : rows = Kg output channels, cols = (t, r, s, c),        k = output pixels, split
//               over blockIdx.z into fp32 slabs summed afterwards (deterministic)
// Operand fragments are gathered straight into registers: one 16-byte load when 8 consecutive k
// are 8 consecutive channels (channels per group a multiple of 8), else per-element loads with
// zero fill -- the generic path trades peak speed for coverage.  16-bit data runs
// v_mfma_f32_16x16x32_{f16,bf16}; fp32 data the exact-f32 v_mfma_f32_16x16x4_f32.
// Tiles: 256-thread workgroups, 64 x 64 outputs, each wave 32 x 32 (2 x 2 fragments).
#include <stdexcept>

#include "common.h"
#include "mfma.h"

namespace mxamd {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct GeomG {
  int N, D, H, W, C;   // input (C: all channels)
  int K;               // output channels (all groups)
  int G;               // groups
  int T, R, S;         // kernel extent
  int Do, Ho, Wo;      // output extent
  int sd, sh, sw, pd, ph, pw, dd, dh, dw;
};

template <typename T>
struct GFrag;

template <typename T>
struct GFrag16 {
  typedef u32x4 frag;
  static constexpr int KSTEP = 32;
  static constexpr int PER = 8;  // consecutive k per lane
  static __device__ __forceinline__ uint16_t bits(T v) { return __builtin_bit_cast(uint16_t, v); }
  static __device__ __forceinline__ frag pack(const uint16_t (&e)[8]) {
    return frag{e[0] | (uint32_t(e[1]) << 16), e[2] | (uint32_t(e[3]) << 16), e[4] | (uint32_t(e[5]) << 16),
                e[6] | (uint32_t(e[7]) << 16)};
  }
};

template <>
struct GFrag<__half> : GFrag16<__half> {
  static __device__ __forceinline__ f4_t mma(const frag& a, const frag& b, f4_t c) {
    return mfma::Op<__half>::run(a, b, c);
  }
  static __device__ __forceinline__ __half out(float v) { return __float2half(v); }
};
template <>
struct GFrag<__hip_bfloat16> : GFrag16<__hip_bfloat16> {
  static __device__ __forceinline__ f4_t mma(const frag& a, const frag& b, f4_t c) {
    return mfma::Op<__hip_bfloat16>::run(a, b, c);
  }
  static __device__ __forceinline__ __hip_bfloat16 out(float v) { return __float2bfloat16(v); }
};
template <>
struct GFrag<float> {
  typedef float frag;
  static constexpr int KSTEP = 4;
  static constexpr int PER = 1;
  static __device__ __forceinline__ f4_t mma(const frag& a, const frag& b, f4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ float out(float v) { return v; }
};

// ---- per-lane gather context: what a fragment row (A) or column (B) index resolves to once
struct RowCtx {
  int n, z0, y0, x0;  // batch and base input / output coordinate of the pixel (mode-dependent)
  bool ok;
};

// element loader: value at reduction index kk for the lane's row / column context
template <typename T, int MODE, bool ISA>
struct Elem {
  // MODE 0, A: x at (pixel m, tap(kk), c(kk))
  // MODE 0, B: w[g*Kg + col][kk]                (contiguous in kk)
  // MODE 1, A: dy at (pixel m, tap(kk), co(kk))  with the stride predicate
  // MODE 1, B: wT[g*Cg + col][kk]               (host-transposed weight, contiguous in kk)
  // MODE 2, A: dy[p = kk][g*Kg + row]
  // MODE 2, B: x at (pixel p = kk, tap(col), c(col))
};

__device__ __forceinline__ void split_tap(int q, const GeomG& g, int* t, int* r, int* s) {
  *s = q % g.S;
  q /= g.S;
  *r = q % g.R;
  *t = q / g.R;
}

// x value (or 0) at output pixel base (z0, y0, x0) = o*stride - pad, tap (t, r, s), channel c
template <typename T>
__device__ __forceinline__ T x_at(const T* x, const GeomG& g, int n, int z0, int y0, int x0, int t, int r, int s,
                                  int ch) {
  const int zi = z0 + t * g.dd, yi = y0 + r * g.dh, xi = x0 + s * g.dw;
  if ((unsigned)zi >= (unsigned)g.D || (unsigned)yi >= (unsigned)g.H || (unsigned)xi >= (unsigned)g.W) return T(0);
  return x[(((static_cast<int64_t>(n) * g.D + zi) * g.H + yi) * g.W + xi) * g.C + ch];
}

// dy value (or 0) reaching input pixel (zi, yi, xi) through tap (t, r, s), channel co (dgrad)
template <typename T>
__device__ __forceinline__ bool dy_src(const GeomG& g, int zi, int yi, int xi, int t, int r, int s, int64_t* pix,
                                       int n) {
  const int az = zi + g.pd - t * g.dd, ay = yi + g.ph - r * g.dh, ax = xi + g.pw - s * g.dw;
  if (az < 0 || ay < 0 || ax < 0) return false;
  if (az % g.sd || ay % g.sh || ax % g.sw) return false;
  const int oz = az / g.sd, oy = ay / g.sh, ox = ax / g.sw;
  if (oz >= g.Do || oy >= g.Ho || ox >= g.Wo) return false;
  *pix = ((static_cast<int64_t>(n) * g.Do + oz) * g.Ho + oy) * g.Wo + ox;
  return true;
}

template <typename T, int MODE>
__global__ void __launch_bounds__(256) conv_gen_kernel(const T* __restrict__ src, const T* __restrict__ wsrc,
                                                       const float* __restrict__ bias, void* __restrict__ dst,
                                                       GeomG g, int rows, int cols, int kred, int kchunk,
                                                       int vec_a, int vec_b) {
  using F = GFrag<T>;
  constexpr int KS = F::KSTEP;
  constexpr int PER = F::PER;
  const int Cg = g.C / g.G, Kg = g.K / g.G;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int split = (MODE == 2) ? blockIdx.z % (gridDim.z / g.G) : 0;
  const int grp = (MODE == 2) ? blockIdx.z / (gridDim.z / g.G) : blockIdx.z;
  const int row0 = blockIdx.x * 64 + (wv >> 1) * 32;
  const int col0 = blockIdx.y * 64 + (wv & 1) * 32;
  const int l16 = lane & 15;
  const int kq = (PER == 8) ? (lane >> 4) * 8 : (lane >> 4);
  const int k_begin = (MODE == 2) ? split * kchunk : 0;
  const int k_end = (MODE == 2) ? min(kred, k_begin + kchunk) : kred;

  // fragment-row (A) and fragment-column (B) contexts: 2 each per lane
  RowCtx ra[2], rb[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int m = row0 + f * 16 + l16;
    const int c = col0 + f * 16 + l16;
    ra[f].ok = m < rows;
    rb[f].ok = c < cols;
    ra[f].n = ra[f].z0 = ra[f].y0 = ra[f].x0 = 0;
    rb[f].n = rb[f].z0 = rb[f].y0 = rb[f].x0 = 0;
    if (MODE == 0 && ra[f].ok) {  // output pixel -> input base
      int q = m;
      const int ox = q % g.Wo; q /= g.Wo;
      const int oy = q % g.Ho; q /= g.Ho;
      const int oz = q % g.Do;
      ra[f].n = q / g.Do;
      ra[f].z0 = oz * g.sd - g.pd;
      ra[f].y0 = oy * g.sh - g.ph;
      ra[f].x0 = ox * g.sw - g.pw;
    }
    if (MODE == 1 && ra[f].ok) {  // input pixel coordinates
      int q = m;
      ra[f].x0 = q % g.W; q /= g.W;
      ra[f].y0 = q % g.H; q /= g.H;
      ra[f].z0 = q % g.D;
      ra[f].n = q / g.D;
    }
  }

  auto load_a = [&](int f, int k) -> typename F::frag {
    if constexpr (PER == 8) {
      uint16_t e[8];
      const RowCtx& rc = ra[f];
      if (MODE == 0) {
        if (vec_a && rc.ok && k < k_end) {
          const int c = k % Cg;
          int t, r, s;
          split_tap(k / Cg, g, &t, &r, &s);
          const int zi = rc.z0 + t * g.dd, yi = rc.y0 + r * g.dh, xi = rc.x0 + s * g.dw;
          if ((unsigned)zi < (unsigned)g.D && (unsigned)yi < (unsigned)g.H && (unsigned)xi < (unsigned)g.W)
            return *reinterpret_cast<const u32x4*>(
                src + (((static_cast<int64_t>(rc.n) * g.D + zi) * g.H + yi) * g.W + xi) * g.C + grp * Cg + c);
          return u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int kk = k + i;
          T v = T(0);
          if (rc.ok && kk < k_end) {
            int t, r, s;
            split_tap(kk / Cg, g, &t, &r, &s);
            v = x_at(src, g, rc.n, rc.z0, rc.y0, rc.x0, t, r, s, grp * Cg + kk % Cg);
          }
          e[i] = F::bits(v);
        }
        return F::pack(e);
      } else if (MODE == 1) {
        if (vec_a && rc.ok && k < k_end) {
          const int co = k % Kg;
          int t, r, s;
          split_tap(k / Kg, g, &t, &r, &s);
          int64_t pix;
          if (dy_src<T>(g, rc.z0, rc.y0, rc.x0, t, r, s, &pix, rc.n))
            return *reinterpret_cast<const u32x4*>(src + pix * g.K + grp * Kg + co);
          return u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int kk = k + i;
          T v = T(0);
          if (rc.ok && kk < k_end) {
            int t, r, s;
            split_tap(kk / Kg, g, &t, &r, &s);
            int64_t pix;
            if (dy_src<T>(g, rc.z0, rc.y0, rc.x0, t, r, s, &pix, rc.n)) v = src[pix * g.K + grp * Kg + kk % Kg];
          }
          e[i] = F::bits(v);
        }
        return F::pack(e);
      } else {  // wgrad A: dy[p][g*Kg + row]
        const int row = row0 + f * 16 + l16;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int kk = k + i;
          e[i] = F::bits((rc.ok && kk < k_end) ? src[static_cast<int64_t>(kk) * g.K + grp * Kg + row] : T(0));
        }
        return F::pack(e);
      }
    } else {
      const RowCtx& rc = ra[f];
      const int kk = k;
      if (!rc.ok || kk >= k_end) return 0.f;
      if (MODE == 0) {
        int t, r, s;
        split_tap(kk / Cg, g, &t, &r, &s);
        return x_at(src, g, rc.n, rc.z0, rc.y0, rc.x0, t, r, s, grp * Cg + kk % Cg);
      } else if (MODE == 1) {
        int t, r, s;
        split_tap(kk / Kg, g, &t, &r, &s);
        int64_t pix;
        return dy_src<T>(g, rc.z0, rc.y0, rc.x0, t, r, s, &pix, rc.n) ? src[pix * g.K + grp * Kg + kk % Kg] : 0.f;
      } else {
        const int row = row0 + f * 16 + l16;
        return src[static_cast<int64_t>(kk) * g.K + grp * Kg + row];
      }
    }
  };

  auto load_b = [&](int f, int k) -> typename F::frag {
    const int col = col0 + f * 16 + l16;
    const bool ok = rb[f].ok;
    if (MODE == 0 || MODE == 1) {
      // weight rows contiguous in k: [G*colsPerGroup][kred]
      const T* wr = wsrc + (static_cast<int64_t>(grp) * cols + (ok ? col : 0)) * kred;
      if constexpr (PER == 8) {
        if (vec_b && ok && k < k_end) return *reinterpret_cast<const u32x4*>(wr + k);
        uint16_t e[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = F::bits((ok && k + i < k_end) ? wr[k + i] : T(0));
        return F::pack(e);
      } else {
        return (ok && k < k_end) ? wr[k] : 0.f;
      }
    } else {  // wgrad B: x at (output pixel kk, tap(col), channel(col))
      const int c = col % Cg;
      int t, r, s;
      split_tap(col / Cg, g, &t, &r, &s);
      auto at = [&](int kk) -> T {
        if (!ok || kk >= k_end) return T(0);
        int q = kk;
        const int ox = q % g.Wo; q /= g.Wo;
        const int oy = q % g.Ho; q /= g.Ho;
        const int oz = q % g.Do;
        const int n = q / g.Do;
        return x_at(wsrc, g, n, oz * g.sd - g.pd, oy * g.sh - g.ph, ox * g.sw - g.pw, t, r, s, grp * Cg + c);
      };
      if constexpr (PER == 8) {
        uint16_t e[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = F::bits(at(k + i));
        return F::pack(e);
      } else {
        return at(k);
      }
    }
  };

  f4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};

  for (int k0 = k_begin; k0 < k_end; k0 += KS) {
    const int k = k0 + kq;
    const typename F::frag a0 = load_a(0, k), a1 = load_a(1, k);
    const typename F::frag b0 = load_b(0, k), b1 = load_b(1, k);
    acc[0][0] = F::mma(a0, b0, acc[0][0]);
    acc[0][1] = F::mma(a0, b1, acc[0][1]);
    acc[1][0] = F::mma(a1, b0, acc[1][0]);
    acc[1][1] = F::mma(a1, b1, acc[1][1]);
  }

  // epilogue: lane holds rows (lane>>4)*4 + q of each A fragment, column lane & 15 of each B fragment
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = col0 + j * 16 + l16;
      if (col >= cols) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = row0 + i * 16 + (lane >> 4) * 4 + q;
        if (row >= rows) continue;
        const float v = acc[i][j][q];
        if (MODE == 2) {
          // fp32 slab [split][G][Kg][cols]
          float* part = static_cast<float*>(dst);
          part[((static_cast<int64_t>(split) * g.G + grp) * Kg + row) * cols + col] = v;
        } else {
          const int ld = MODE == 0 ? g.K : g.C;
          const int cb = grp * cols + col;
          T* y = static_cast<T*>(dst);
          y[static_cast<int64_t>(row) * ld + cb] = F::out(v + (bias ? bias[cb] : 0.f));
        }
      }
    }
}

template <typename T>
void launch_gen(int mode, const void* src, const void* wsrc, const float* bias, void* dst, const GeomG& g, int splits,
                hipStream_t s) {
  const int Cg = g.C / g.G, Kg = g.K / g.G;
  const int tap = g.T * g.R * g.S;
  int rows, cols, kred;
  if (mode == 0) {
    rows = g.N * g.Do * g.Ho * g.Wo; cols = Kg; kred = tap * Cg;
  } else if (mode == 1) {
    rows = g.N * g.D * g.H * g.W; cols = Cg; kred = tap * Kg;
  } else {
    rows = Kg; cols = tap * Cg; kred = g.N * g.Do * g.Ho * g.Wo;
  }
  const bool half = sizeof(T) == 2;
  const uintptr_t sp = reinterpret_cast<uintptr_t>(src), wp = reinterpret_cast<uintptr_t>(wsrc);
  // 16-byte fragment loads: 8 consecutive k inside one (tap, channel group) run, aligned rows
  int vec_a = 0, vec_b = 0;
  if (half && mode == 0) vec_a = (Cg % 8 == 0 && g.C % 8 == 0 && sp % 16 == 0) ? 1 : 0;
  if (half && mode == 1) vec_a = (Kg % 8 == 0 && g.K % 8 == 0 && sp % 16 == 0) ? 1 : 0;
  if (half && mode != 2) vec_b = (kred % 8 == 0 && wp % 16 == 0) ? 1 : 0;
  constexpr int KS = GFrag<T>::KSTEP;
  int kchunk = kred;
  if (mode == 2) kchunk = ((kred + splits - 1) / splits + KS - 1) / KS * KS;
  dim3 grid((rows + 63) / 64, (cols + 63) / 64, g.G * (mode == 2 ? splits : 1));
  MXAMD_HOST_CHECK(grid.y <= 65535 && grid.z <= 65535, "conv_gen: grid too large");
  switch (mode) {
    case 0:
      hipLaunchKernelGGL((conv_gen_kernel<T, 0>), grid, dim3(256), 0, s, static_cast<const T*>(src),
                         static_cast<const T*>(wsrc), bias, dst, g, rows, cols, kred, kchunk, vec_a, vec_b);
      break;
    case 1:
      hipLaunchKernelGGL((conv_gen_kernel<T, 1>), grid, dim3(256), 0, s, static_cast<const T*>(src),
                         static_cast<const T*>(wsrc), bias, dst, g, rows, cols, kred, kchunk, vec_a, vec_b);
      break;
    default:
      hipLaunchKernelGGL((conv_gen_kernel<T, 2>), grid, dim3(256), 0, s, static_cast<const T*>(src),
                         static_cast<const T*>(wsrc), bias, dst, g, rows, cols, kred, kchunk, vec_a, vec_b);
  }
}

}  // namespace

// mode 0: y = conv(x, w) (+bias)     src = x,  wsrc = w  [K][T][R][S][Cg],  dst = y
// mode 1: dx = conv^T(dy, w)          src = dy, wsrc = wT [G*Cg][T][R][S][Kg] (host-transposed), dst = dx
// mode 2: dW partial slabs            src = dy, wsrc = x, dst = fp32 [splits][G][Kg][T*R*S*Cg]
// geom = [N, D, H, W, C, K, G, T, R, S, Do, Ho, Wo, sd, sh, sw, pd, ph, pw, dd, dh, dw]
void conv_gen(int dtype, int mode, const void* src, const void* wsrc, const float* bias, void* dst, const int* geom,
              int splits, hipStream_t s) {
  GeomG g;
  g.N = geom[0]; g.D = geom[1]; g.H = geom[2]; g.W = geom[3]; g.C = geom[4]; g.K = geom[5]; g.G = geom[6];
  g.T = geom[7]; g.R = geom[8]; g.S = geom[9]; g.Do = geom[10]; g.Ho = geom[11]; g.Wo = geom[12];
  g.sd = geom[13]; g.sh = geom[14]; g.sw = geom[15]; g.pd = geom[16]; g.ph = geom[17]; g.pw = geom[18];
  g.dd = geom[19]; g.dh = geom[20]; g.dw = geom[21];
  MXAMD_HOST_CHECK(g.G >= 1 && g.C % g.G == 0 && g.K % g.G == 0, "conv_gen: channels must divide by groups");
  MXAMD_HOST_CHECK(g.sd >= 1 && g.sh >= 1 && g.sw >= 1 && g.dd >= 1 && g.dh >= 1 && g.dw >= 1,
                   "conv_gen: stride / dilation must be positive");
  MXAMD_HOST_CHECK(mode >= 0 && mode <= 2 && splits >= 1, "conv_gen: bad mode / splits");
  MXAMD_HOST_CHECK((int64_t)g.N * g.D * g.H * g.W * g.C < (1ll << 31) &&
                       (int64_t)g.N * g.Do * g.Ho * g.Wo * g.K < (1ll << 31),
                   "conv_gen: tensor too large for 32-bit pixel indexing");
  if (dtype == kF32) launch_gen<float>(mode, src, wsrc, bias, dst, g, splits, s);
  else if (dtype == kF16) launch_gen<__half>(mode, src, wsrc, bias, dst, g, splits, s);
  else if (dtype == kBF16) launch_gen<__hip_bfloat16>(mode, src, wsrc, bias, dst, g, splits, s);
  else throw std::runtime_error("conv_gen: dtype must be f32, f16 or bf16");
}

}  // namespace mxamd
