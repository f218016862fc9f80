// NHWC implicit-GEMM convolution: persistent workgroups streaming K-steps
// through an N-stage LDS-DMA ring (gfx950).
//
// Why: conv_big.hip's loop (issue tile k+1 -> MFMAs on tile k -> vmcnt(0) +
// barrier) gives each LDS-DMA one K-tile of MFMA time (~0.9 us) to land and
// drains the queue at every barrier, and each workgroup handles ONE output tile,
// so a shape with a short K loop (1x1 convs with Cin = 64..256: 1-4 K-tiles) runs
// load -> compute -> store with nothing overlapping inside the CU.  Here
//
//   * each 512-thread workgroup is persistent: it walks the output tiles
//     wgid, wgid + grid, ... (XCD-aware remap, consecutive tiles on one XCD) and
//     treats (tile, k-tile) as ONE continuous stream of K-steps, so the DMA for
//     the next tile's first K-tiles is in flight while the current tile's last
//     MFMAs and its epilogue run;
//   * NST LDS stages, D = NST-1 K-steps issued ahead; the wait before a step is a
//     counted `s_waitcnt vmcnt(N)` (never 0 in steady state) + raw s_barrier, so
//     younger DMAs stay in flight across the barrier (an LDS-DMA is a VM-counter
//     op: __syncthreads()' fence would drain it);
//   * the epilogue stores straight from the MFMA accumulators with buffer stores
//     (out-of-range pixels get an out-of-bounds offset and are dropped by the
//     hardware), so every wave issues a fixed, known number of VM ops per tile and
//     the vmcnt count N stays exact: N = LPT * (steps issued after this one) +
//     S * (epilogues since this step's DMA was issued);
//   * optional BatchNorm statistics: per-(tile, wave) channel sums of y and y^2
//     (same [2][K][nparts] partials layout as conv_big.hip, consumed by the BN
//     finalize kernel, so the BN statistics pass over y disappears).
//
// Requirements (host-checked): Cin % 64 == 0, Cout % BCO == 0, dilation 1, no bias.
#include <stdexcept>

#include "common.h"
#include "mfma.h"

namespace mxamd {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

// 16x16x32 MFMA (mfma.h); the epilogue keeps its packed pairs in a native 2-vector
template <typename T>
struct MfmaR : mfma::Op<T> {
  static __device__ __forceinline__ u32x2 pack4(float a, float b, float c, float d) {
    return u32x2{mfma::Op<T>::two(a, b), mfma::Op<T>::two(c, d)};
  }
};

struct GeomR {
  int N, H, W, C, K, R, S;
  int Ho, Wo;
  int sh, sw, ph, pw;
  int M;     // N*Ho*Wo
  int Ktot;  // R*S*C
};

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_base, 16, 0, 0);
}

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt left at their maxima); gfx9 encoding
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// Wait until at most `n` VM ops are outstanding, rounding n DOWN to a level (waiting for more
// than necessary is always safe; waiting for fewer is not).
__device__ __forceinline__ void vm_wait_le(int n) {
  if (n >= 48) vm_wait<48>();
  else if (n >= 32) vm_wait<32>();
  else if (n >= 24) vm_wait<24>();
  else if (n >= 16) vm_wait<16>();
  else if (n >= 12) vm_wait<12>();
  else if (n >= 8) vm_wait<8>();
  else if (n >= 6) vm_wait<6>();
  else if (n >= 4) vm_wait<4>();
  else if (n >= 3) vm_wait<3>();
  else if (n >= 2) vm_wait<2>();
  else if (n >= 1) vm_wait<1>();
  else vm_wait<0>();
}

__device__ __forceinline__ void lds_barrier() {
  // all of this wave's LDS reads retired, then the workgroup barrier; the memory clobber keeps the
  // compiler from moving LDS accesses or DMA issues across it.  No vmcnt: younger DMAs stay in flight.
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ float row16_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

constexpr uint32_t kOOB = 0xFFFFFFF0u;   // buffer offset past num_records: the store is dropped

// BCO = WCO*64 output channels x BPIX = (8/WCO)*FJ*16 pixels per tile; NST LDS stages
template <typename T, int WCO, int FJ, int NST, bool STATS>
__global__ void __launch_bounds__(512) conv_ring_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                        T* __restrict__ y, const T* __restrict__ zero, GeomR g,
                                                        int tiles_co, int ntiles, float* __restrict__ part,
                                                        int nparts) {
  constexpr int WPIX = 8 / WCO;
  constexpr int BCO = WCO * 64;
  constexpr int BPIX = WPIX * FJ * 16;
  constexpr int BK = 64;
  constexpr int A_BYTES = BCO * 128;
  constexpr int STAGE = (BCO + BPIX) * 128;
  constexpr int A_INS = BCO / 64;  // LDS-DMA wave-instructions (8 rows x 128 B each) per wave for A
  constexpr int B_INS = BPIX / 64;
  constexpr int LPT = A_INS + B_INS;             // VM ops per wave per K-step
  constexpr int SPT = 4 * FJ + (STATS ? 4 : 0);  // VM ops per wave per tile epilogue
  constexpr int D = NST - 1;                     // K-steps in flight ahead of the one computed
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;

  // XCD-aware bijective remap: workgroups with consecutive wgid share an XCD, and at every
  // round they hold consecutive tiles (neighbouring co tiles of one pixel tile -> shared B panel)
  const int grid = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q = grid >> 3, rr = grid & 7;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
  if (wgid >= ntiles) return;
  const int my_tiles = (ntiles - wgid + grid - 1) / grid;
  const int KT = g.Ktot / BK;
  const int G = my_tiles * KT;

  const int lrow = lane >> 3;
  const int gch = (lane & 7) ^ lrow;
  const T* zsrc = zero + gch * 8;

  // ---------------- issue side: per-row sources of the tile currently being fetched
  int a_off[A_INS];
  int b_base[B_INS], b_hi[B_INS], b_wi[B_INS];
  int i_tile = wgid, i_kt = 0, i_stage = 0;
  auto set_issue_tile = [&](int t) {
    const int tpix = t / tiles_co;
    const int co0 = (t - tpix * tiles_co) * BCO;
    const int pix0 = tpix * BPIX;
#pragma unroll
    for (int i = 0; i < A_INS; ++i) a_off[i] = (co0 + (i * 8 + wid) * 8 + lrow) * g.Ktot + gch * 8;
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const int p = pix0 + (i * 8 + wid) * 8 + lrow;
      if (p < g.M) {
        const int n = p / (g.Ho * g.Wo);
        const int rem = p - n * g.Ho * g.Wo;
        const int ho = rem / g.Wo;
        const int wo = rem - ho * g.Wo;
        b_hi[i] = ho * g.sh - g.ph;
        b_wi[i] = wo * g.sw - g.pw;
        b_base[i] = ((n * g.H + b_hi[i]) * g.W + b_wi[i]) * g.C + gch * 8;
      } else {
        b_hi[i] = -(1 << 20);  // never in range -> zero page
        b_wi[i] = 0;
        b_base[i] = 0;
      }
    }
  };
  auto issue = [&]() {
    const int k0 = i_kt * BK;
    const int rs = k0 / g.C;
    const int c0 = k0 - rs * g.C;
    const int r = rs / g.S;
    const int s = rs - r * g.S;
    char* sbase = smem + i_stage * STAGE;
#pragma unroll
    for (int i = 0; i < A_INS; ++i) glds16(w + a_off[i] + k0, sbase + (i * 8 + wid) * 1024);
    const int doff = (r * g.W + s) * g.C + c0;
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const int hi = b_hi[i] + r, wi = b_wi[i] + s;
      const bool ok = (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
      const T* src = ok ? x + b_base[i] + doff : zsrc;
      glds16(src, sbase + A_BYTES + (i * 8 + wid) * 1024);
    }
    // advance the issue cursor
    i_stage = (i_stage + 1 == NST) ? 0 : i_stage + 1;
    if (++i_kt == KT) {
      i_kt = 0;
      i_tile += grid;
      if (i_tile < ntiles) set_issue_tile(i_tile);
    }
  };

  // ---------------- compute side
  f4_t acc[4][FJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};

  const int wco = wid % WCO;
  const int wpix = wid / WCO;
  const int frag_r = lane & 15;
  const int fchunk = lane >> 4;
  const int a_row0 = (wco * 64 + frag_r) * 128;
  const int b_row0 = A_BYTES + (wpix * FJ * 16 + frag_r) * 128;
  const int swz = frag_r & 7;

  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
      y, 0, static_cast<int>(static_cast<uint32_t>(g.M) * static_cast<uint32_t>(g.K) * sizeof(T)), 0x00020000);
  __amdgpu_buffer_rsrc_t prs;
  if (STATS)
    prs = __builtin_amdgcn_make_buffer_rsrc(part, 0, static_cast<int>(2u * g.K * nparts * 4u), 0x00020000);

  set_issue_tile(i_tile);
  const int npro = G < D ? G : D;
  for (int p = 0; p < npro; ++p) issue();

  int c_tile = wgid, c_kt = 0, c_stage = 0;
  uint32_t epi_hist = 0;  // bit j set: an epilogue ran j+1 steps ago (in the last D steps)
  for (int gi = 0; gi < G; ++gi) {
    // DMA(gi) was issued D steps ago; younger VM ops: the DMAs of the following steps already
    // issued, plus the stores of every epilogue run since then
    const int ahead = (G - 1 - gi) < (D - 1) ? (G - 1 - gi) : (D - 1);
    vm_wait_le(ahead * LPT + __builtin_popcount(epi_hist) * SPT);
    lds_barrier();
    if (gi + D < G) issue();

    const char* sb = smem + c_stage * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = ((kk * 4 + fchunk) ^ swz) * 16;
      u32x4 af[4], bf[FJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const u32x4*>(sb + a_row0 + i * 16 * 128 + ch);
#pragma unroll
      for (int j = 0; j < FJ; ++j) bf[j] = *reinterpret_cast<const u32x4*>(sb + b_row0 + j * 16 * 128 + ch);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = MfmaR<T>::run(af[i], bf[j], acc[i][j]);
    }
    c_stage = (c_stage + 1 == NST) ? 0 : c_stage + 1;

    bool epi = false;
    if (++c_kt == KT) {
      // ---- epilogue of tile c_tile straight from the accumulators.  Lane holds channels
      // co0 + wco*64 + i*16 + 4*(lane>>4) + {0..3} of pixel pix0 + wpix*FJ*16 + j*16 + (lane&15)
      c_kt = 0;
      const int tpix = c_tile / tiles_co;
      const int co0 = (c_tile - tpix * tiles_co) * BCO;
      const int pix0 = tpix * BPIX;
      const int pw0 = pix0 + wpix * FJ * 16 + frag_r;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = co0 + wco * 64 + i * 16 + fchunk * 4;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, q0 = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f;
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
          const int p = pw0 + j * 16;
          const bool ok = p < g.M;
          const f4_t v = acc[i][j];
          const uint32_t off = ok ? (static_cast<uint32_t>(p) * g.K + co) * sizeof(T) : kOOB;
          __builtin_amdgcn_raw_buffer_store_b64(MfmaR<T>::pack4(v[0], v[1], v[2], v[3]), yrs, off, 0, 0);
          if (STATS && ok) {
            s0 += v[0]; s1 += v[1]; s2 += v[2]; s3 += v[3];
            q0 += v[0] * v[0]; q1 += v[1] * v[1]; q2 += v[2] * v[2]; q3 += v[3] * v[3];
          }
        }
        if (STATS) {
          // every lane of a 16-lane row group ends with the group's totals; lane r < 8 of the
          // group stores value r (sums of 4 channels, then sums of squares)
          s0 = row16_sum(s0); s1 = row16_sum(s1); s2 = row16_sum(s2); s3 = row16_sum(s3);
          q0 = row16_sum(q0); q1 = row16_sum(q1); q2 = row16_sum(q2); q3 = row16_sum(q3);
          const int r = frag_r;
          const float v = r == 0 ? s0 : r == 1 ? s1 : r == 2 ? s2 : r == 3 ? s3
                        : r == 4 ? q0 : r == 5 ? q1 : r == 6 ? q2 : q3;
          const int pid = tpix * WPIX + wpix;
          const uint32_t c = static_cast<uint32_t>(co + (r & 3));
          const uint32_t idx = (r >= 4 ? static_cast<uint32_t>(g.K) * nparts : 0u) + c * nparts + pid;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), prs, r < 8 ? idx * 4u : kOOB, 0,
                                                0);
        }
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};
      }
      c_tile += grid;
      epi = true;
    }
    epi_hist = ((epi_hist << 1) | (epi ? 1u : 0u)) & ((1u << D) - 1u);
  }
}

template <int WCO, int FJ, int NST>
struct RingCfg {
  static constexpr int BCO = WCO * 64;
  static constexpr int BPIX = (8 / WCO) * FJ * 16;
  static constexpr int SMEM = NST * (BCO + BPIX) * 128;
};

template <typename T, int WCO, int FJ, int NST, bool STATS>
void launch_ring(const void* x, const void* w, void* y, const void* zero, const GeomR& g, float* part, int nparts,
                 int ncu, hipStream_t s) {
  using Cfg = RingCfg<WCO, FJ, NST>;
  static_assert(Cfg::SMEM <= 160 * 1024, "conv_ring: LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_ring_kernel<T, WCO, FJ, NST, STATS>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::SMEM);
    attr_set = true;
  }
  const int tiles_co = g.K / Cfg::BCO;
  const int tiles_pix = (g.M + Cfg::BPIX - 1) / Cfg::BPIX;
  const int ntiles = tiles_co * tiles_pix;
  const int per_cu = (160 * 1024) / Cfg::SMEM;   // workgroups that fit one CU's LDS
  int grid = ncu * (per_cu < 4 ? per_cu : 4);
  if (grid > ntiles) grid = ntiles;
  hipLaunchKernelGGL((conv_ring_kernel<T, WCO, FJ, NST, STATS>), dim3(grid), dim3(512), Cfg::SMEM, s,
                     static_cast<const T*>(x), static_cast<const T*>(w), static_cast<T*>(y),
                     static_cast<const T*>(zero), g, tiles_co, ntiles, part, nparts);
}

// variant -> tile / stages
//   0: 128x128 x4 stages   1: 256x128 x3   2: 128x256 x3   3: 64x256 x4   4: 256x256 x2   5: 64x128 x4
struct RingTile {
  int bco, bpix;
};
static RingTile ring_tile(int variant) {
  switch (variant) {
    case 0: return {128, 128};
    case 1: return {256, 128};
    case 2: return {128, 256};
    case 3: return {64, 256};
    case 4: return {256, 256};
    case 5: return {64, 128};
    default: throw std::runtime_error("conv_nhwc_fwd_ring: unknown variant");
  }
}

template <typename T, bool STATS>
void dispatch_ring(int variant, const void* x, const void* w, void* y, const void* zero, const GeomR& g, float* part,
                   int nparts, int ncu, hipStream_t s) {
  switch (variant) {
    case 0: launch_ring<T, 2, 2, 4, STATS>(x, w, y, zero, g, part, nparts, ncu, s); break;
    case 1: launch_ring<T, 4, 4, 3, STATS>(x, w, y, zero, g, part, nparts, ncu, s); break;
    case 2: launch_ring<T, 2, 4, 3, STATS>(x, w, y, zero, g, part, nparts, ncu, s); break;
    case 3: launch_ring<T, 1, 2, 4, STATS>(x, w, y, zero, g, part, nparts, ncu, s); break;
    case 4: launch_ring<T, 4, 8, 2, STATS>(x, w, y, zero, g, part, nparts, ncu, s); break;
    case 5: launch_ring<T, 1, 1, 4, STATS>(x, w, y, zero, g, part, nparts, ncu, s); break;
  }
}

int device_cu_count() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  return ncu;
}

}  // namespace

int conv_nhwc_fwd_ring_nparts(int N, int H, int W, int R, int S, int sh, int sw, int ph, int pw, int variant) {
  const RingTile t = ring_tile(variant);
  const int Ho = (H + 2 * ph - R) / sh + 1;
  const int Wo = (W + 2 * pw - S) / sw + 1;
  const int M = N * Ho * Wo;
  return ((M + t.bpix - 1) / t.bpix) * (8 / (t.bco / 64));
}

void conv_nhwc_fwd_ring(int dtype, const void* x, const void* w, void* y, const void* zero, int N, int H, int W, int C,
                        int K, int R, int S, int sh, int sw, int ph, int pw, int variant, float* part, int nparts,
                        hipStream_t s) {
  GeomR g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw;
  g.Ho = (H + 2 * ph - R) / sh + 1;
  g.Wo = (W + 2 * pw - S) / sw + 1;
  g.M = N * g.Ho * g.Wo;
  g.Ktot = R * S * C;
  const RingTile t = ring_tile(variant);
  MXAMD_HOST_CHECK(C % 64 == 0 && K % t.bco == 0, "conv_nhwc_fwd_ring: need Cin % 64 == 0 and Cout % BCO == 0");
  MXAMD_HOST_CHECK((int64_t)N * H * W * C < (1ll << 31) && (int64_t)g.M * K * 2 < (1ll << 32) - 64 &&
                       (int64_t)K * g.Ktot < (1ll << 31),
                   "conv_nhwc_fwd_ring: tensor too large for 32-bit indexing");
  MXAMD_HOST_CHECK(part == nullptr || nparts == conv_nhwc_fwd_ring_nparts(N, H, W, R, S, sh, sw, ph, pw, variant),
                   "conv_nhwc_fwd_ring: wrong BN partials count");
  MXAMD_HOST_CHECK(part == nullptr || (int64_t)2 * K * nparts * 4 < (1ll << 31),
                   "conv_nhwc_fwd_ring: BN partials too large");
  const int ncu = device_cu_count();
  if (dtype == kF16) {
    if (part) dispatch_ring<__half, true>(variant, x, w, y, zero, g, part, nparts, ncu, s);
    else dispatch_ring<__half, false>(variant, x, w, y, zero, g, part, nparts, ncu, s);
  } else if (dtype == kBF16) {
    if (part) dispatch_ring<__hip_bfloat16, true>(variant, x, w, y, zero, g, part, nparts, ncu, s);
    else dispatch_ring<__hip_bfloat16, false>(variant, x, w, y, zero, g, part, nparts, ncu, s);
  } else {
    throw std::runtime_error("conv_nhwc_fwd_ring: dtype must be f16 or bf16");
  }
}

}  // namespace mxamd
