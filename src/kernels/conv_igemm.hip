// NHWC implicit-GEMM convolution on CDNA4 matrix cores (gfx950).
//
// Parity: the forward / backward-data convolution of src/operator/nn/convolution.cu
// (cuDNN / MIOpen in the reference).  Designed for MI355X rather than translated:
//
//   GEMM view (forward):  Y[pix][co] = sum_k  Xpatch[pix][k] * W[co][k],
//     pix = (n, ho, wo)  (M = N*Ho*Wo, the row index of the NHWC output),
//     k   = (r, s, c)    (K = R*S*Cin, exactly the OHWI weight row), so both
//     operands are K-contiguous in memory and one 16-byte load is 8 k-values.
//   The kernel computes the transposed tile  C'[co][pix] = W · Xpatchᵀ  with
//   v_mfma_f32_16x16x32_{f16,bf16}; the accumulator layout (col = lane&15,
//   row = 4*(lane>>4)+reg) then gives every lane 4 CONSECUTIVE output channels
//   of one pixel -> 8-byte vector stores into the NHWC output.
//
//   Block: 256 threads = 4 wave64s, each wave owns a 64(co) x 64(pix) sub-tile
//   (4x4 MFMA fragments, 64 fp32 accumulators/lane).  Tile = BCO x BPIX with
//   BCO in {64,128} and BPIX = 256*64/BCO/... (4 waves), BK = 32 or 64.
//   Operands are staged global -> registers -> LDS (double buffered, one
//   barrier per K-step; rows padded by 16 B against bank conflicts), the next
//   K-tile's global loads are issued before the current tile's MFMAs.
//   Grid is remapped so consecutive logical tiles land on the same XCD
//   (bijective remap): the co-tiles of one pixel-tile then share that XCD's L2
//   and the activation tile is fetched from HBM once.
//
//   Backward-data of a stride-1 convolution is the same kernel on dY with the
//   flipped, transposed weight (prepared by the caller).
//
// Requirements (checked by the launcher and ops/kernel_fns.py): Cin % BK == 0,
// Cout % BCO == 0, dilation 1, contiguous NHWC x / OHWI w, 16-byte aligned.
#include "common.h"
#include "mfma.h"

namespace mxamd {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // native vector: stays in VGPRs (HIP uint4 struct copies lower to memcpy -> scratch)

template <typename T>
struct MfmaOp : mfma::Op<T> {};   // 16x16x32 MFMA + epilogue packs (mfma.h)

struct ConvGeom {
  int N, H, W, C;        // input (NHWC)
  int K, R, S;           // output channels, filter size
  int Ho, Wo;
  int sh, sw, ph, pw;
  int M;                 // N*Ho*Wo
  int Ktot;              // R*S*C
};

template <int N, typename T>
__device__ __forceinline__ void load_rows(u32x4 (&r)[N], const T* __restrict__ base, const int (&off)[N], int k0) {
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = *reinterpret_cast<const u32x4*>(base + off[i] + k0);
}

template <int N, typename T>
__device__ __forceinline__ void load_patch(u32x4 (&r)[N], const T* __restrict__ x, const int (&off)[N],
                                           const int (&hi0)[N], const int (&wi0)[N], int dr, int ds, int doff, int H,
                                           int W) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int hi = hi0[i] + dr, wi = wi0[i] + ds;
    if ((unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W)
      r[i] = *reinterpret_cast<const u32x4*>(x + off[i] + doff);
    else
      r[i] = u32x4{0u, 0u, 0u, 0u};
  }
}

template <int N, typename T>
__device__ __forceinline__ void store_rows(T* s, const int (&off)[N], const u32x4 (&r)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) *reinterpret_cast<u32x4*>(s + off[i]) = r[i];
}

template <typename T, int BCO, int BK>
__global__ void __launch_bounds__(256) conv_fwd_igemm_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                             const float* __restrict__ bias, T* __restrict__ y,
                                                             ConvGeom g, int tiles_co) {
  constexpr int WAVES_CO = BCO / 64;
  constexpr int WAVES_PIX = 4 / WAVES_CO;
  constexpr int BPIX = WAVES_PIX * 64;
  constexpr int LDK = BK + 8;                      // padded LDS row (elements)
  constexpr int CH = BK / 8;                       // 16-byte chunks per row
  constexpr int A_LD = BCO * CH / 256;             // weight chunks per thread
  constexpr int B_LD = BPIX * CH / 256;            // activation chunks per thread
  static_assert(A_LD >= 1 && B_LD >= 1, "tile too small");

  __shared__ __attribute__((aligned(16))) T smem[2 * (BCO + BPIX) * LDK];
  T* sA = smem;                                    // [2][BCO][LDK]
  T* sB = smem + 2 * BCO * LDK;                    // [2][BPIX][LDK]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;

  // XCD-aware bijective remap of the linear block id
  const int nblk = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q = nblk >> 3, rr = nblk & 7;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
  const int tco = wgid % tiles_co;
  const int tpix = wgid / tiles_co;
  const int co0 = tco * BCO;
  const int pix0 = tpix * BPIX;

  // ---- per-thread load descriptors (32-bit element offsets; host checks sizes)
  int a_off[A_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    int q2 = tid + i * 256;
    a_off[i] = (co0 + q2 / CH) * g.Ktot + (q2 % CH) * 8;
  }
  int b_off[B_LD], b_hi[B_LD], b_wi[B_LD];
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    int q2 = tid + i * 256;
    int p = pix0 + q2 / CH;
    if (p < g.M) {
      int n = p / (g.Ho * g.Wo);
      int rem = p - n * g.Ho * g.Wo;
      int ho = rem / g.Wo;
      int wo = rem - ho * g.Wo;
      b_hi[i] = ho * g.sh - g.ph;
      b_wi[i] = wo * g.sw - g.pw;
      b_off[i] = ((n * g.H + b_hi[i]) * g.W + b_wi[i]) * g.C + (q2 % CH) * 8;
    } else {
      b_hi[i] = -(1 << 20);  // never in range
      b_wi[i] = 0;
      b_off[i] = 0;
    }
  }
  // LDS write offsets
  int sa_off[A_LD], sb_off[B_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    int q2 = tid + i * 256;
    sa_off[i] = (q2 / CH) * LDK + (q2 % CH) * 8;
  }
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    int q2 = tid + i * 256;
    sb_off[i] = (q2 / CH) * LDK + (q2 % CH) * 8;
  }

  u32x4 ra[A_LD], rb[B_LD];
  const int KT = g.Ktot / BK;
  // k-tile -> (r, s, c0) walked incrementally; C % BK == 0 so a tile never straddles (r, s)
  int t_r = 0, t_s = 0, t_c0 = 0;

#define MXAMD_CONV_GLOAD(kt)                                                         \
  {                                                                                  \
    load_rows<A_LD>(ra, w, a_off, (kt) * BK);                                        \
    load_patch<B_LD>(rb, x, b_off, b_hi, b_wi, t_r, t_s, (t_r * g.W + t_s) * g.C + t_c0, g.H, g.W); \
    t_c0 += BK;                                                                      \
    if (t_c0 == g.C) {                                                               \
      t_c0 = 0;                                                                      \
      if (++t_s == g.S) { t_s = 0; ++t_r; }                                          \
    }                                                                                \
  }
#define MXAMD_CONV_SSTORE(buf)                                                       \
  {                                                                                  \
    store_rows<A_LD>(sA + (buf) * BCO * LDK, sa_off, ra);                            \
    store_rows<B_LD>(sB + (buf) * BPIX * LDK, sb_off, rb);                           \
  }

  float4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int wco = wid % WAVES_CO;
  const int wpix = wid / WAVES_CO;
  const int frag_r = lane & 15;
  const int frag_k = (lane >> 4) * 8;

  MXAMD_CONV_GLOAD(0);
  MXAMD_CONV_SSTORE(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) MXAMD_CONV_GLOAD(kt + 1);
    const T* As = sA + (buf * BCO + wco * 64 + frag_r) * LDK + frag_k;
    const T* Bs = sB + (buf * BPIX + wpix * 64 + frag_r) * LDK + frag_k;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      u32x4 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const u32x4*>(As + i * 16 * LDK + kk);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const u32x4*>(Bs + j * 16 * LDK + kk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = MfmaOp<T>::run(af[i], bf[j], acc[i][j]);
    }
    if (kt + 1 < KT) MXAMD_CONV_SSTORE(buf ^ 1);
    __syncthreads();
  }

#undef MXAMD_CONV_GLOAD
#undef MXAMD_CONV_SSTORE
  // ---- epilogue: lane holds co = base + 4*(lane>>4) + {0..3} for pixel base + (lane&15)
  const int co_l = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = co0 + wco * 64 + i * 16 + co_l;
    float b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
    if (bias) {
      b0 = bias[co];
      b1 = bias[co + 1];
      b2 = bias[co + 2];
      b3 = bias[co + 3];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = pix0 + wpix * 64 + j * 16 + frag_r;
      if (p < g.M) {
        uint2 v = MfmaOp<T>::pack4(acc[i][j][0] + b0, acc[i][j][1] + b1, acc[i][j][2] + b2, acc[i][j][3] + b3);
        *reinterpret_cast<uint2*>(y + (int64_t)p * g.K + co) = v;
      }
    }
  }
}

template <typename T, int BCO, int BK>
static void launch_fwd(const void* x, const void* w, const float* bias, void* y, const ConvGeom& g, hipStream_t s) {
  constexpr int BPIX = (4 / (BCO / 64)) * 64;
  int tiles_co = g.K / BCO;
  int tiles_pix = (g.M + BPIX - 1) / BPIX;
  dim3 grid(tiles_co * tiles_pix);
  hipLaunchKernelGGL((conv_fwd_igemm_kernel<T, BCO, BK>), grid, dim3(256), 0, s, static_cast<const T*>(x),
                     static_cast<const T*>(w), bias, static_cast<T*>(y), g, tiles_co);
}

// Tile choice (variant 0): BCO=128 when Cout allows it (128x128 tile), else 64 x 256.
// BK=64 when Cin is a multiple of 64 (all ResNet layers but the stem).
// variant 1..4 force (BCO, BK) = (128,64) (128,32) (64,64) (64,32): the autotuner
// (ops/kernel_fns.py) times them per shape -- LDS footprint sets blocks/CU
// (73.7 / 41 / 92 / 51 KB -> 2 / 3 / 1 / 3 blocks), which decides latency hiding.
template <typename T>
static void dispatch_fwd(const void* x, const void* w, const float* bias, void* y, const ConvGeom& g, int variant,
                         hipStream_t s) {
  const bool co128 = (g.K % 128) == 0;
  // BK=64 halves the barriers per FLOP but its LDS/VGPR footprint allows only
  // 1-2 blocks per CU; short reductions (1x1 over <=128 channels) are
  // bandwidth-bound and want the occupancy of BK=32 instead.
  const bool bk64 = (g.C % 64) == 0 && g.Ktot >= 256;
  switch (variant) {
    case 1:
      MXAMD_HOST_CHECK(co128 && g.C % 64 == 0, "conv variant 1 needs Cout%128, Cin%64");
      launch_fwd<T, 128, 64>(x, w, bias, y, g, s);
      return;
    case 2:
      MXAMD_HOST_CHECK(co128, "conv variant 2 needs Cout%128");
      launch_fwd<T, 128, 32>(x, w, bias, y, g, s);
      return;
    case 3:
      MXAMD_HOST_CHECK(g.C % 64 == 0, "conv variant 3 needs Cin%64");
      launch_fwd<T, 64, 64>(x, w, bias, y, g, s);
      return;
    case 4:
      launch_fwd<T, 64, 32>(x, w, bias, y, g, s);
      return;
    default:
      break;
  }
  if (co128 && bk64) launch_fwd<T, 128, 64>(x, w, bias, y, g, s);
  else if (co128) launch_fwd<T, 128, 32>(x, w, bias, y, g, s);
  else if (bk64) launch_fwd<T, 64, 64>(x, w, bias, y, g, s);
  else launch_fwd<T, 64, 32>(x, w, bias, y, g, s);
}

void conv_nhwc_fwd(int dtype, const void* x, const void* w, const float* bias, void* y, int N, int H, int W, int C,
                   int K, int R, int S, int sh, int sw, int ph, int pw, int variant, hipStream_t s) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw;
  g.Ho = (H + 2 * ph - R) / sh + 1;
  g.Wo = (W + 2 * pw - S) / sw + 1;
  g.M = N * g.Ho * g.Wo;
  g.Ktot = R * S * C;
  MXAMD_HOST_CHECK(C % 32 == 0 && K % 64 == 0, "conv_nhwc_fwd: need Cin % 32 == 0 and Cout % 64 == 0");
  MXAMD_HOST_CHECK((int64_t)N * H * W * C < (1ll << 31) && (int64_t)g.M * K < (1ll << 31),
                   "conv_nhwc_fwd: tensor too large for 32-bit pixel indexing");
  if (dtype == kF16) dispatch_fwd<__half>(x, w, bias, y, g, variant, s);
  else if (dtype == kBF16) dispatch_fwd<__hip_bfloat16>(x, w, bias, y, g, variant, s);
  else throw std::runtime_error("conv_nhwc_fwd: dtype must be f16 or bf16");
}

}  // namespace mxamd
