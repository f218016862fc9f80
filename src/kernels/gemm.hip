// Dense GEMM on the gfx950 matrix cores:  C[M,N] = act(A[M,K] . B[N,K]^T + bias[N]) (+ addend[M,N])
//
// The layout every FullyConnected pass reduces to once its operands are K-contiguous ("NT"):
//   forward  y  = x . W^T        A = x [tokens, in],  B = W [out, in]
//   dgrad    dx = dy . W         A = dy,              B = W^T (one cached transposed copy per step)
// (the weight gradient, a reduction over tokens, is the TN kernel of conv_wgrad.hip).
//
// Design (CDNA4-first, not a warp-tiled CUDA GEMM):
//   * v_mfma_f32_16x16x32_{f16,bf16}; each 64-lane wave owns a 64(n) x FJ*16(m) block of
//     accumulators, so a lane's four accumulator values are four CONSECUTIVE output columns:
//     the epilogue stores 8 (bf16/f16) or 16 (fp32) contiguous bytes per lane with bias / GELU /
//     ReLU / residual applied in registers -- no separate bias or activation pass over C;
//   * operands stream global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
//     instruction = 8 rows of a BK = 64 tile), 16-byte chunks XOR-swizzled by (row & 7) so the
//     ds_read_b128 fragment reads are conflict-free; a 2-4 stage LDS ring where the wait before a
//     K-step is a counted `s_waitcnt vmcnt` + raw barrier, so the DMAs of the next steps stay in
//     flight across it (a K = 768 GEMM has only 12 steps: latency, not bandwidth, bounds it);
//   * tiles from 64x128 (256 threads, 48 KiB LDS: three workgroups per CU) to 256x256 (512 threads),
//     and 192 / 384-column tiles whose grids fill the 256 CUs in whole waves on transformer shapes;
//     small GEMMs (BERT: 4096 tokens x 768) also split K across workgroups: fp32 partial slabs,
//     summed with the same epilogue by gemm_splitk_reduce -- deterministic, no atomics;
//   * XCD-aware bijective block remap: consecutive tiles of one A row-panel land on one XCD's L2.
//
// Requirements (host-checked): K % 64 == 0, N % BN == 0, 16-byte aligned rows; any M.
#include <cmath>
#include <stdexcept>

#include "common.h"
#include "mfma.h"

namespace mxamd {

namespace {

typedef _Float16 g_half8 __attribute__((ext_vector_type(8)));
typedef __bf16 g_bf16x8 __attribute__((ext_vector_type(8)));
typedef float g_f4 __attribute__((ext_vector_type(4)));
typedef uint32_t g_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void g_lds_void;
typedef __attribute__((address_space(1))) void g_gbl_void;

template <typename T>
struct GMfma : mfma::Op<T> {};   // 16x16x32 MFMA + epilogue packs (mfma.h)

enum GemmAct : int { kActNone = 0, kActRelu = 1, kActGelu = 2 };

__device__ __forceinline__ float gemm_act(float v, int act) {
  if (act == kActRelu) return fmaxf(v, 0.f);
  if (act == kActGelu) return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
  return v;
}

__device__ __forceinline__ void g_glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((g_gbl_void*)src, (g_lds_void*)lds_base, 16, 0, 0);
}

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt at their maxima); gfx9 encoding
template <int N>
__device__ __forceinline__ void g_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// wait until at most n of this wave's VM ops are outstanding (n rounded DOWN to a level: safe)
__device__ __forceinline__ void g_vm_wait_le(int n) {
  if (n >= 48) g_vm_wait<48>();
  else if (n >= 32) g_vm_wait<32>();
  else if (n >= 24) g_vm_wait<24>();
  else if (n >= 16) g_vm_wait<16>();
  else if (n >= 12) g_vm_wait<12>();
  else if (n >= 8) g_vm_wait<8>();
  else if (n >= 6) g_vm_wait<6>();
  else if (n >= 4) g_vm_wait<4>();
  else if (n >= 2) g_vm_wait<2>();
  else g_vm_wait<0>();
}

// this wave's LDS reads retired, then the workgroup barrier -- no vmcnt, so younger LDS-DMAs stay in
// flight across it (__syncthreads() would drain them)
__device__ __forceinline__ void g_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct GemmArgs {
  const void* a;       // [M][lda] (K-contiguous rows)
  const void* b;       // [N][ldb]
  const void* bias;    // [N] (fp32, or the operand dtype when bias_lowp) or null
  const void* addend;  // [M][ldc] (output dtype) or null
  void* c;             // [M][ldc]
  float* ws;           // split-K partial slabs [splits][M][N] (fp32) or null
  int M, N, K, lda, ldb, ldc;
  int act, out_f32, splits, tiles_n, tiles_m, bias_lowp;
};

// bias[n .. n+3] as fp32 (the bias may be kept in the operand dtype: no per-call fp32 copy)
template <typename T>
__device__ __forceinline__ float4 gemm_bias4(const GemmArgs& g, int n) {
  if (g.bias_lowp) return GMfma<T>::unpack4(*reinterpret_cast<const uint2*>(static_cast<const T*>(g.bias) + n));
  return *reinterpret_cast<const float4*>(static_cast<const float*>(g.bias) + n);
}

// WN waves along n (FI*16 columns each), WM waves along m (FJ*16 rows each), NST LDS stages
template <typename T, int WN, int WM, int FJ, int NST, int FI = 4>
__global__ void __launch_bounds__(64 * WN * WM) gemm_nt_kernel(GemmArgs g) {
  constexpr int WAVES = WN * WM;
  constexpr int NT = 64 * WAVES;
  constexpr int BN = WN * FI * 16;
  constexpr int BM = WM * FJ * 16;
  constexpr int B_BYTES = BN * 128;
  constexpr int STAGE = (BN + BM) * 128;
  constexpr int B_INS = BN / (8 * WAVES);
  constexpr int A_INS = BM / (8 * WAVES);
  static_assert(B_INS * 8 * WAVES == BN && A_INS * 8 * WAVES == BM, "tile rows per wave");
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;

  // XCD-aware bijective remap (blocks are dealt round-robin to the 8 XCDs)
  const int nblk = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q = nblk >> 3, rr = nblk & 7;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
  const int per_split = g.tiles_n * g.tiles_m;
  const int split = wg / per_split;
  const int t2 = wg - split * per_split;
  const int tm = t2 / g.tiles_n;
  const int tn = t2 - tm * g.tiles_n;
  const int n0 = tn * BN;
  const int m0 = tm * BM;

  const int KT = g.K / 64;
  const int kt0 = static_cast<int>((static_cast<int64_t>(KT) * split) / g.splits);
  const int kt1 = static_cast<int>((static_cast<int64_t>(KT) * (split + 1)) / g.splits);

  const int lrow = lane >> 3;
  const int gch = (lane & 7) ^ lrow;
  const T* A = static_cast<const T*>(g.a);
  const T* B = static_cast<const T*>(g.b);
  const T* a_src[A_INS];
  const T* b_src[B_INS];
#pragma unroll
  for (int i = 0; i < B_INS; ++i) b_src[i] = B + static_cast<int64_t>(n0 + (i * WAVES + wid) * 8 + lrow) * g.ldb + gch * 8;
#pragma unroll
  for (int i = 0; i < A_INS; ++i) {
    int m = m0 + (i * WAVES + wid) * 8 + lrow;
    m = m < g.M ? m : g.M - 1;  // clamped rows feed output rows that are never stored
    a_src[i] = A + static_cast<int64_t>(m) * g.lda + gch * 8;
  }

  auto issue = [&](int kt, int stage) {
    const int k0 = kt * 64;
    char* sb = smem + stage * STAGE;
#pragma unroll
    for (int i = 0; i < B_INS; ++i) g_glds16(b_src[i] + k0, sb + (i * WAVES + wid) * 1024);
#pragma unroll
    for (int i = 0; i < A_INS; ++i) g_glds16(a_src[i] + k0, sb + B_BYTES + (i * WAVES + wid) * 1024);
  };

  g_f4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = g_f4{0.f, 0.f, 0.f, 0.f};

  const int wn = wid % WN;
  const int wm = wid / WN;
  const int frag_r = lane & 15;
  const int fchunk = lane >> 4;
  const int b_row0 = (wn * FI * 16 + frag_r) * 128;
  const int a_row0 = B_BYTES + (wm * FJ * 16 + frag_r) * 128;
  const int sw = frag_r & 7;

  // NST-stage LDS ring: K-step kt+D (D = NST-1) is issued while step kt computes; before step kt a
  // counted vmcnt wait leaves the DMAs of the steps issued after it in flight
  constexpr int D = NST - 1;
  constexpr int LPT = A_INS + B_INS;  // LDS-DMA wave-instructions per K-step
  const int nk = kt1 - kt0;
  for (int p = 0; p < D && p < nk; ++p) issue(kt0 + p, p);
  int stage = 0;
  for (int it = 0; it < nk; ++it) {
    const int ahead = (nk - 1 - it) < (D - 1) ? (nk - 1 - it) : (D - 1);
    g_vm_wait_le(ahead * LPT);
    g_lds_barrier();
    if (it + D < nk) issue(kt0 + it + D, stage == 0 ? NST - 1 : stage - 1);
    const char* sb = smem + stage * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = ((kk * 4 + fchunk) ^ sw) * 16;
      g_u32x4 bf[FI], af[FJ];
#pragma unroll
      for (int i = 0; i < FI; ++i) bf[i] = *reinterpret_cast<const g_u32x4*>(sb + b_row0 + i * 16 * 128 + ch);
#pragma unroll
      for (int j = 0; j < FJ; ++j) af[j] = *reinterpret_cast<const g_u32x4*>(sb + a_row0 + j * 16 * 128 + ch);
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = GMfma<T>::run(bf[i], af[j], acc[i][j]);
    }
    stage = stage + 1 == NST ? 0 : stage + 1;
  }

  // ---- epilogue: lane holds columns n0 + wn*FI*16 + i*16 + 4*(lane>>4) + {0..3} of row m0 + wm*FJ*16 + j*16 + (lane&15)
  const int cq = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < FI; ++i) {
    const int n = n0 + wn * FI * 16 + i * 16 + cq;
    if (g.splits > 1) {
      float* ws = g.ws + static_cast<int64_t>(split) * g.M * g.N;
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int m = m0 + wm * FJ * 16 + j * 16 + frag_r;
        if (m < g.M)
          *reinterpret_cast<float4*>(ws + static_cast<int64_t>(m) * g.N + n) =
              make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
      continue;
    }
    float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
    if (g.bias) bb = gemm_bias4<T>(g, n);
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int m = m0 + wm * FJ * 16 + j * 16 + frag_r;
      if (m >= g.M) continue;
      float v0 = gemm_act(acc[i][j][0] + bb.x, g.act), v1 = gemm_act(acc[i][j][1] + bb.y, g.act);
      float v2 = gemm_act(acc[i][j][2] + bb.z, g.act), v3 = gemm_act(acc[i][j][3] + bb.w, g.act);
      const int64_t off = static_cast<int64_t>(m) * g.ldc + n;
      if (g.out_f32) {
        float* c = static_cast<float*>(g.c) + off;
        if (g.addend) {
          const float4 ad = *reinterpret_cast<const float4*>(static_cast<const float*>(g.addend) + off);
          v0 += ad.x; v1 += ad.y; v2 += ad.z; v3 += ad.w;
        }
        *reinterpret_cast<float4*>(c) = make_float4(v0, v1, v2, v3);
      } else {
        if (g.addend) {
          const float4 ad = GMfma<T>::unpack4(*reinterpret_cast<const uint2*>(static_cast<const T*>(g.addend) + off));
          v0 += ad.x; v1 += ad.y; v2 += ad.z; v3 += ad.w;
        }
        *reinterpret_cast<uint2*>(static_cast<T*>(g.c) + off) = GMfma<T>::pack4(v0, v1, v2, v3);
      }
    }
  }
}

// Sum of the split-K slabs + the same epilogue; one thread per 4 consecutive outputs.
template <typename T>
__global__ void __launch_bounds__(256) gemm_splitk_reduce_kernel(GemmArgs g) {
  const int64_t n4 = static_cast<int64_t>(g.M) * g.N / 4;
  const int64_t slab = static_cast<int64_t>(g.M) * g.N;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < n4; e += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t flat = e * 4;
    const int m = static_cast<int>(flat / g.N);
    const int n = static_cast<int>(flat - static_cast<int64_t>(m) * g.N);
    float4 s = *reinterpret_cast<const float4*>(g.ws + flat);
    for (int k = 1; k < g.splits; ++k) {
      const float4 p = *reinterpret_cast<const float4*>(g.ws + k * slab + flat);
      s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
    }
    if (g.bias) {
      const float4 bb = gemm_bias4<T>(g, n);
      s.x += bb.x; s.y += bb.y; s.z += bb.z; s.w += bb.w;
    }
    s.x = gemm_act(s.x, g.act); s.y = gemm_act(s.y, g.act); s.z = gemm_act(s.z, g.act); s.w = gemm_act(s.w, g.act);
    const int64_t off = static_cast<int64_t>(m) * g.ldc + n;
    if (g.out_f32) {
      if (g.addend) {
        const float4 ad = *reinterpret_cast<const float4*>(static_cast<const float*>(g.addend) + off);
        s.x += ad.x; s.y += ad.y; s.z += ad.z; s.w += ad.w;
      }
      *reinterpret_cast<float4*>(static_cast<float*>(g.c) + off) = s;
    } else {
      if (g.addend) {
        const float4 ad = GMfma<T>::unpack4(*reinterpret_cast<const uint2*>(static_cast<const T*>(g.addend) + off));
        s.x += ad.x; s.y += ad.y; s.z += ad.z; s.w += ad.w;
      }
      *reinterpret_cast<uint2*>(static_cast<T*>(g.c) + off) = GMfma<T>::pack4(s.x, s.y, s.z, s.w);
    }
  }
}

template <typename T, int WN, int WM, int FJ, int NST, int FI = 4>
void launch_gemm(GemmArgs g, hipStream_t s) {
  constexpr int BN = WN * FI * 16;
  constexpr int BM = WM * FJ * 16;
  constexpr int SMEM = NST * (BN + BM) * 128;
  static_assert(SMEM <= 160 * 1024, "gemm: LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<T, WN, WM, FJ, NST, FI>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  g.tiles_n = g.N / BN;
  g.tiles_m = (g.M + BM - 1) / BM;
  const int blocks = g.tiles_n * g.tiles_m * g.splits;
  hipLaunchKernelGGL((gemm_nt_kernel<T, WN, WM, FJ, NST, FI>), dim3(blocks), dim3(64 * WN * WM), SMEM, s, g);
  if (g.splits > 1) {
    const int64_t n4 = static_cast<int64_t>(g.M) * g.N / 4;
    int rb = static_cast<int>((n4 + 255) / 256);
    rb = rb < 2048 ? rb : 2048;
    hipLaunchKernelGGL((gemm_splitk_reduce_kernel<T>), dim3(rb), dim3(256), 0, s, g);
  }
}

// config -> (BN x BM) tile, LDS stages:
//   0: 128x128 4w 2st   1: 128x64 4w 2st   2: 64x128 4w 2st   3: 256x128 8w 2st   4: 128x256 8w 2st
//   5: 256x256 8w 2st   6: 64x64 2w 2st    7: 128x128 4w 3st  8: 256x128 8w 3st   9: 128x64 4w 4st
//  10: 64x64 2w 4st    11: 128x256 8w 3st  12: 128x64 4w 3st  13: 64x128 4w 3st
// (12 / 13: three 24 KB stages = 72 KB, so two workgroups still share a CU -- the 2-stage tiles wait on
// their single look-ahead stage for ~55 % of their wave cycles, the 4-stage ones keep one workgroup per CU)
//  14: 192x64 4w 3st (48 columns per wave)   15: 192x128 4w 2st (96 columns per wave, 2 WG/CU)
//  16: 192x256 8w 2st   17: 384x128 8w 2st
// (14-17: 192 / 384-column tiles whose grids are whole multiples of the 256 CUs on the transformer
// shapes -- M = 4096 tokens: N = 768 -> 64 x 4 tiles of 192x64, N = 3072 -> 16 x 16 of 192x256 or
// 32 x 8 of 384x128, 512 of 192x128 at two per CU -- where the power-of-two tiles leave a quarter of
// the chip idle in the last wave)
constexpr int kGemmCfgs = 18;
template <typename T>
void dispatch_gemm(int cfg, const GemmArgs& g, hipStream_t s) {
  switch (cfg) {
    case 0: launch_gemm<T, 2, 2, 4, 2>(g, s); break;
    case 1: launch_gemm<T, 2, 2, 2, 2>(g, s); break;
    case 2: launch_gemm<T, 1, 4, 2, 2>(g, s); break;
    case 3: launch_gemm<T, 4, 2, 4, 2>(g, s); break;
    case 4: launch_gemm<T, 2, 4, 4, 2>(g, s); break;
    case 5: launch_gemm<T, 4, 2, 8, 2>(g, s); break;
    case 6: launch_gemm<T, 1, 2, 2, 2>(g, s); break;
    case 7: launch_gemm<T, 2, 2, 4, 3>(g, s); break;
    case 8: launch_gemm<T, 4, 2, 4, 3>(g, s); break;
    case 9: launch_gemm<T, 2, 2, 2, 4>(g, s); break;
    case 10: launch_gemm<T, 1, 2, 2, 4>(g, s); break;
    case 11: launch_gemm<T, 2, 4, 4, 3>(g, s); break;
    case 12: launch_gemm<T, 2, 2, 2, 3>(g, s); break;
    case 13: launch_gemm<T, 1, 4, 2, 3>(g, s); break;
    case 14: launch_gemm<T, 4, 1, 4, 3, 3>(g, s); break;
    case 15: launch_gemm<T, 2, 2, 4, 2, 6>(g, s); break;
    case 16: launch_gemm<T, 2, 4, 4, 2, 6>(g, s); break;
    case 17: launch_gemm<T, 4, 2, 4, 2, 6>(g, s); break;
    default: throw std::runtime_error("gemm_nt: unknown tile config");
  }
}

}  // namespace

int gemm_nt_tile_n(int cfg) {
  static const int bn[kGemmCfgs] = {128, 128, 64, 256, 128, 256, 64, 128, 256, 128, 64, 128, 128, 64,
                                     192, 192, 192, 384};
  MXAMD_HOST_CHECK(cfg >= 0 && cfg < kGemmCfgs, "gemm_nt: unknown tile config");
  return bn[cfg];
}

int gemm_nt_tile_m(int cfg) {
  static const int bm[kGemmCfgs] = {128, 64, 128, 128, 256, 256, 64, 128, 128, 64, 64, 256, 64, 128,
                                     64, 128, 256, 128};
  MXAMD_HOST_CHECK(cfg >= 0 && cfg < kGemmCfgs, "gemm_nt: unknown tile config");
  return bm[cfg];
}

void gemm_nt(int dtype, const void* a, const void* b, const void* bias, const void* addend, void* c, int out_f32,
             int M, int N, int K, int lda, int ldb, int ldc, int act, int cfg, int splits, float* ws, hipStream_t s,
             int bias_lowp) {
  const int bn = gemm_nt_tile_n(cfg);
  MXAMD_HOST_CHECK(M > 0 && K % 64 == 0 && N % bn == 0, "gemm_nt: need K % 64 == 0 and N % tile_n == 0");
  MXAMD_HOST_CHECK(lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0 && lda >= K && ldb >= K && ldc >= N,
                   "gemm_nt: leading dimensions must be 16-byte multiples covering the rows");
  MXAMD_HOST_CHECK(splits >= 1 && splits <= K / 64, "gemm_nt: 1 <= splits <= K / 64");
  MXAMD_HOST_CHECK(splits == 1 || (ws != nullptr && ldc == N), "gemm_nt: split-K needs a workspace and ldc == N");
  MXAMD_HOST_CHECK(act >= 0 && act <= 2, "gemm_nt: act must be 0 (none), 1 (relu) or 2 (gelu)");
  MXAMD_HOST_CHECK(static_cast<int64_t>(M) * lda < (1ll << 40) && static_cast<int64_t>(N) * ldb < (1ll << 40),
                   "gemm_nt: operand too large");
  MXAMD_HOST_CHECK(bias == nullptr || reinterpret_cast<uintptr_t>(bias) % (bias_lowp ? 8 : 16) == 0,
                   "gemm_nt: bias must be 8-byte (16-bit dtype) / 16-byte (fp32) aligned");
  GemmArgs g{a, b, bias, addend, c, ws, M, N, K, lda, ldb, ldc, act, out_f32, splits, 0, 0, bias_lowp ? 1 : 0};
  if (dtype == kF16) dispatch_gemm<__half>(cfg, g, s);
  else if (dtype == kBF16) dispatch_gemm<__hip_bfloat16>(cfg, g, s);
  else throw std::runtime_error("gemm_nt: dtype must be f16 or bf16");
}

}  // namespace mxamd
