// Streaming pointwise (1x1, stride 1) convolution for small reductions (gfx950).
//
// The 1x1 convolutions of a bottleneck with Cin = 64..512 do ~50-200 FLOP per byte they move, far
// below the MFMA/HBM balance point (~400): they are memory-bound, and the general tiled kernels
// (conv_big / conv_ring) run them at 1.5-3 TB/s because every workgroup walks load -> MFMA ->
// epilogue with little overlap and re-reads the weight panel per tile.  This kernel is built for
// the stream instead:
//
//   * persistent: 2 workgroups per CU walk the pixel tiles (XCD-aware order), so one workgroup's
//     epilogue stores overlap the other's loads and MFMAs;
//   * the whole weight matrix lives in REGISTERS for the kernel's lifetime -- wave (wc, wp) keeps the
//     A fragments of its NOUT/WC output channels over the full reduction (<= 64 VGPRs);
//   * input pixel tiles [BM][KIN] stream through an NST-stage LDS ring by LDS-DMA
//     (global_load_lds_dwordx4, XOR-swizzled 16-byte chunks, out-of-range pixels from a zero page),
//     D = NST-1 tiles in flight; the wait is a counted `s_waitcnt vmcnt(N)` with N known at compile
//     time (every iteration issues the same number of VM ops), never a drain, plus a raw s_barrier;
//   * epilogue: accumulators -> fp16/bf16 [BM][NOUT] LDS image (row pitch +16 B, conflict-free 8-byte
//     writes) -> whole 16-byte row chunks -> coalesced global stores of complete pixel rows;
//   * optional BatchNorm statistics: each thread keeps per-channel sum / sum-of-squares of the
//     rows it stores over ALL its tiles; at the end one partial per workgroup per channel
//     ([2][NOUT][grid] channel-major, the layout bn_nhwc.hip's finalize consumes);
//   * optional addend (y = conv + addend: the identity-shortcut gradient of a tee dgrad), streamed
//     through its own part of each ring stage by the same LDS-DMA rounds;
//   * optional BatchNorm-backward statistics (y is the gradient of a BN(+ReLU) output): the BN's input
//     z (and, for a residual tail, its 1-bit ReLU mask) ride in the stage as well, and each thread
//     accumulates sum(dz) and sum(dz * (z - mean)), dz = y masked by the ReLU, over the rows it stores
//     -- the BN's own backward reduction pass over (y, z) is not run.
//
// Requirements (host-checked): NHWC, KIN in {64,128,256,512}, NOUT in {64..1024} with
// NOUT/WC * KIN <= 8192 (the register budget for the resident weights).
#include <stdexcept>

#include "common.h"
#include "mfma.h"

namespace mxamd {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

template <typename T>
struct PwM : mfma::Op<T> {   // 16x16x32 MFMA + epilogue packs (mfma.h)
  template <typename V>
  static __device__ __forceinline__ f4_t mma(const V& a, const V& b, f4_t c) {
    return mfma::Op<T>::run(a, b, c);
  }
};

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One mask byte from LDS through its aligned dword: the 64 lanes of a store round read 64 consecutive
// bytes, i.e. 16 dwords with 4 lanes each (a broadcast), where byte-wide reads counted as bank conflicts
__device__ __forceinline__ uint32_t lds_byte(const char* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  return (*reinterpret_cast<const uint32_t*>(a & ~static_cast<uintptr_t>(3)) >> ((a & 3u) * 8)) & 0xffu;
}

// pixels per tile: the input stage at most 16 KB and the epilogue image at most 32 KB; with an
// addend, at most 32 pixels (its LDS stage is as large as the image) but whole 8 KB LDS-DMA rounds
// for both the input and the addend stage
// (nout = the output channels one workgroup computes: a slice of the layer's when it is sliced)
constexpr int pw_bm(int kin, int nout, bool add) {   // add: any extra stream (addend / BN-backward)
  const int in_rows = (8192 / kin) > 16 ? (8192 / kin) : 16;    // Cin >= 1024: 16 rows of up to 32 KB
  const int bm0 = (16384 / nout) < in_rows ? (16384 / nout) : in_rows;
  if (!add) return bm0;
  // with an addend: at most 32 pixels and a 16 KB addend stage (deep rings), at least one 16-row
  // fragment per pixel wave (the LDS-DMA rounds of a tile may then be partial: see issue())
  const int wp = 8 / ((nout / 16) < 8 ? (nout / 16) : 8);
  int bm = bm0 < 32 ? bm0 : 32;
  if (bm > 8192 / nout) bm = 8192 / nout;
  if (bm < 16 * wp) bm = 16 * wp;
  return bm;
}

// BN-backward statistics modes of the epilogue (bn_nhwc.hip's ReLU mask sources)
constexpr int kPwBnbNone = 0;
constexpr int kPwBnbPlain = 1;    // no ReLU
constexpr int kPwBnbFromZ = 2;    // mask = z * scale + shift > 0
constexpr int kPwBnbMask = 3;     // 1 bit per element written by the forward

struct PwBnb {
  const void* z;          // the BN's input, [M][NT]
  const uint8_t* mask;    // kPwBnbMask: [M * NT / 8]
  const float* mean;
  const float* scale;     // kPwBnbFromZ
  const float* shift;
  const uint8_t* amask;   // AMK: the addend is masked by these bits ([M * NT / 8]): addend = dy * mask of a
                          // residual tail's ReLU, its d_addend never materialised (kernel_fns._tee_dgrad)
};

template <int KIN, int NOUT, int WPC = 2, bool ADD = false, int BNB = kPwBnbNone, bool AMK = false>
struct PwCfg {
  static constexpr bool EXT = ADD || BNB != kPwBnbNone;    // extra streams besides the input
  static constexpr int BM = pw_bm(KIN, NOUT, EXT);
  static constexpr int WC = NOUT / 16 < 8 ? NOUT / 16 : 8;  // waves along output channels
  static constexpr int WP = 8 / WC;                        // waves along pixels
  static constexpr int FC = NOUT / WC / 16;                // channel fragments per wave
  static constexpr int FP = BM / WP / 16;                  // pixel fragments per wave
  static constexpr int KS = KIN / 32;                      // MFMA k-steps
  static constexpr int ROWB = KIN * 2;                     // input row bytes
  static constexpr int STAGE_IN = BM * ROWB;               // one input tile
  static constexpr int STAGE_ADD = ADD ? BM * NOUT * 2 : 0;  // its addend rows (linear)
  static constexpr int STAGE_Z = BNB ? BM * NOUT * 2 : 0;    // the BN input rows (linear)
  static constexpr int STAGE_M = BNB == kPwBnbMask ? (BM * NOUT / 8 + 1023) / 1024 * 1024 : 0;  // mask bytes
  static constexpr int STAGE_AM = AMK ? (BM * NOUT / 8 + 1023) / 1024 * 1024 : 0;   // addend mask bytes
  static constexpr int STAGE = STAGE_IN + STAGE_ADD + STAGE_Z + STAGE_M + STAGE_AM;
  static constexpr int LPT = STAGE_IN / (512 * 16);        // LDS-DMA instructions per thread per tile
  static constexpr int APT = STAGE_ADD / (512 * 16);       // ... for the addend
  // with an addend, a tile's 1 KB LDS-DMA instructions go round-robin over the 8 waves (rounds may be
  // partial): TI input and TA addend instructions
  static constexpr int TI = STAGE_IN / 1024;
  static constexpr int TA = STAGE_ADD / 1024;
  static constexpr int TZ = STAGE_Z / 1024;
  static constexpr int TM = STAGE_M / 1024;
  static constexpr int TAM = STAGE_AM / 1024;
  static constexpr int PITCH = NOUT * 2 + 16;              // epilogue image row pitch
  static constexpr int EPI = BM * PITCH;
  static constexpr int OCH = NOUT / 8;                     // 16-byte chunks per output row
  static constexpr int SPT = (BM * OCH + 511) / 512;       // 16-byte stores per thread per tile (uniform)
  // deepest ring (<= 4 stages) that keeps WPC workgroups per CU in the 160 KB of LDS
  static constexpr int LDS = WPC == 1 ? 156 * 1024 : 80 * 1024;
  static constexpr int NMAX = EXT ? 6 : 4;
  static constexpr int NST = (NMAX * STAGE + EPI <= LDS) ? NMAX
                           : ((NMAX - 1) * STAGE + EPI <= LDS) ? NMAX - 1
                           : ((NMAX - 2) * STAGE + EPI <= LDS) ? NMAX - 2 : 2;
  static constexpr int D = NST - 1;
  static constexpr int SMEM = NST * STAGE + EPI;
  static_assert(FC >= 1 && FP >= 1, "at least one fragment pair per wave");
  static_assert(EXT || (LPT >= 1 && STAGE_IN % (512 * 16) == 0), "whole LDS-DMA instructions per tile");
  static_assert(!EXT || (STAGE_IN % 1024 == 0 && STAGE_ADD % 1024 == 0 && STAGE_Z % 1024 == 0),
                "whole 1 KB LDS-DMA instructions");
  static_assert(!EXT || WPC == 1, "the extra stages need the LDS of a whole CU");
  static_assert(BNB != kPwBnbMask || (NOUT / 8) % 16 == 0, "mask rows of whole 16-byte chunks");
  static_assert((BM * OCH) % 512 == 0 || BM * OCH < 512, "whole store rounds, or a single partial one");
  static_assert(512 % OCH == 0, "a thread keeps one output chunk");
  static_assert(D * ((TI + 7) / 8 + (TA + 7) / 8 + (TZ + 7) / 8 + (TM + 7) / 8 + (TAM + 7) / 8 + SPT) <
                    (EXT ? 40 : 64),
                "vmcnt range (vm_wait_n covers < 40)");
  static_assert(!AMK || (ADD && (NOUT / 8) % 16 == 0), "the addend mask rides with an addend, whole 16-byte rows");
  // resident weights: a quarter of the VGPR budget (128 at 2 workgroups per CU, 256 at 1)
  static_assert(FC * KS * 4 <= (WPC == 1 ? 128 : 64), "resident weights exceed the register budget");
  static_assert(ROWB % 128 == 0, "rows of whole 128-byte swizzle groups");
};

// Wait until at most `n` VM ops are outstanding, exactly (0 <= n < 40; larger n round down).
__device__ __forceinline__ void vm_wait_n(int n) {
  switch (n) {
#define MXAMD_VMW(K) \
  case K:            \
    vm_wait<K>();    \
    break;
    MXAMD_VMW(0) MXAMD_VMW(1) MXAMD_VMW(2) MXAMD_VMW(3) MXAMD_VMW(4) MXAMD_VMW(5) MXAMD_VMW(6) MXAMD_VMW(7)
    MXAMD_VMW(8) MXAMD_VMW(9) MXAMD_VMW(10) MXAMD_VMW(11) MXAMD_VMW(12) MXAMD_VMW(13) MXAMD_VMW(14) MXAMD_VMW(15)
    MXAMD_VMW(16) MXAMD_VMW(17) MXAMD_VMW(18) MXAMD_VMW(19) MXAMD_VMW(20) MXAMD_VMW(21) MXAMD_VMW(22)
    MXAMD_VMW(23) MXAMD_VMW(24) MXAMD_VMW(25) MXAMD_VMW(26) MXAMD_VMW(27) MXAMD_VMW(28) MXAMD_VMW(29)
    MXAMD_VMW(30) MXAMD_VMW(31) MXAMD_VMW(32) MXAMD_VMW(33) MXAMD_VMW(34) MXAMD_VMW(35) MXAMD_VMW(36)
    MXAMD_VMW(37) MXAMD_VMW(38) MXAMD_VMW(39)
#undef MXAMD_VMW
    default:
      vm_wait<39>();
  }
}

// Wait until at most `n` VM ops are outstanding (n rounded DOWN to an available level: waiting for
// more than necessary is always safe).
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

// NOUT: output channels per workgroup; S: slices of the layer's NOUT * S output channels (the
// workgroups of one tile's slices are adjacent in the XCD-aware order, so they share its input in L2)
template <typename T, int KIN, int NOUT, bool STATS, bool ADD, int WPC, int S, int BNB, bool AMK = false>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2 * WPC))) conv_pw_stream_kernel(
    const T* __restrict__ x, const T* __restrict__ w, T* __restrict__ y, const T* __restrict__ zero, int M, int ntiles,
    float* __restrict__ part, const T* __restrict__ addend, int wt, PwBnb bnb) {
  using C = PwCfg<KIN, NOUT, WPC, ADD, BNB, AMK>;
  constexpr bool EXT = C::EXT;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wc = wid % C::WC, wp = wid / C::WC;
  const int grid = gridDim.x;
  // XCD-aware: workgroups sharing an XCD take consecutive tiles
  const int xcd = blockIdx.x & 7;
  const int q8 = grid >> 3, r8 = grid & 7;
  const int wg0 = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
  constexpr int NT = NOUT * S;             // the layer's output channels (row stride of y / addend)
  const int slice = S > 1 ? wg0 % S : 0;
  const int wg = S > 1 ? wg0 / S : wg0;    // tile walker within the slice
  const int gs = grid / S;                 // tile walkers per slice (the grid is a multiple of S)

  // ---- resident weights: A fragments of this wave's channels, all k-steps
  u32x4 wa[C::FC][C::KS];
  if (!wt) {
#pragma unroll
    for (int f = 0; f < C::FC; ++f)
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        const int co = slice * NOUT + wc * C::FC * 16 + f * 16 + (lane & 15);
        wa[f][s] = *reinterpret_cast<const u32x4*>(w + static_cast<int64_t>(co) * KIN + s * 32 + (lane >> 4) * 8);
      }
  } else {
    // w is [KIN][NT] (a dgrad's untransposed weight): lane loads 8 consecutive channels of one input
    // row of the fragment's 32 x 16 block (row lane/2, channels (lane&1)*8..+8) ...
#pragma unroll
    for (int f = 0; f < C::FC; ++f)
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        const int k = s * 32 + (lane >> 1);
        const int co = slice * NOUT + wc * C::FC * 16 + f * 16 + (lane & 1) * 8;
        wa[f][s] = *reinterpret_cast<const u32x4*>(w + static_cast<int64_t>(k) * NT + co);
      }
  }

  // the weight loads retire here, before the ring starts: inside the loop the only VM ops are the
  // ring's LDS-DMAs and the epilogue stores, so the counted waits below stay exact
  vm_wait<0>();
  if (wt) {
    // ... and the block is transposed through this wave's 1280-byte LDS scratch ([16 ch][40 halves],
    // 16-byte aligned rows): written column-wise, read back as the lane's 8 consecutive k of its channel
    // (the ring's stages are still free; a wave's LDS ops complete in order)
    uint16_t* scr = reinterpret_cast<uint16_t*>(smem + wid * 1280);
#pragma unroll
    for (int f = 0; f < C::FC; ++f)
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        const uint4 v = __builtin_bit_cast(uint4, wa[f][s]);
        const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 8; ++q)
          scr[((lane & 1) * 8 + q) * 40 + (lane >> 1)] = static_cast<uint16_t>(wv[q >> 1] >> ((q & 1) * 16));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        wa[f][s] = *reinterpret_cast<const u32x4*>(scr + (lane & 15) * 40 + (lane >> 4) * 8);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    __syncthreads();
  }
#pragma unroll
  for (int f = 0; f < C::FC; ++f)
#pragma unroll
    for (int s = 0; s < C::KS; ++s) asm volatile("" ::"v"(wa[f][s]));

  // ---- LDS-DMA issue of input tile `t` into ring stage `st`: instruction i of this thread covers
  // bytes [(i*8+wid)*1024, +1024) of the stage (linear destination, swizzled source chunk)
  auto issue = [&](int t, int st) {
    char* sb = smem + st * C::STAGE;
    // input instruction i covers bytes [i*1024, +1024) of the stage (linear destination, swizzled
    // source chunk); without an addend every wave issues LPT, with one instruction i goes to wave i % 8
    constexpr int NI = EXT ? (C::TI + 7) / 8 : C::LPT;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int i = j * 8 + wid;
      if (EXT && i >= C::TI) break;
      const int byte = (i * 64 + lane) * 16;               // destination byte within the stage (linear)
      const int row = byte / C::ROWB;
      const int slot = (byte % C::ROWB) / 16;
      const int chunk = slot ^ (row & 7);               // source chunk for this slot (XOR swizzle)
      const int p = t * C::BM + row;
      const T* src = p < M ? x + static_cast<int64_t>(p) * KIN + chunk * 8 : zero + (chunk & 7) * 8;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(sb + i * 1024), 16, 0, 0);
    }
    // the tile's addend rows, linear after the input (rows past M read the zero page)
#pragma unroll
    for (int j = 0; j < (C::TA + 7) / 8; ++j) {
      const int i = j * 8 + wid;
      if (i >= C::TA) break;
      const int byte = (i * 64 + lane) * 16;
      const int row = byte / (NOUT * 2);
      const int p = t * C::BM + row;
      const T* src = p < M ? addend + static_cast<int64_t>(p) * NT + slice * NOUT + (byte % (NOUT * 2)) / 2 : zero;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(sb + C::STAGE_IN + i * 1024), 16, 0, 0);
    }
    // the BN input rows (same layout as the addend)
#pragma unroll
    for (int j = 0; j < (C::TZ + 7) / 8; ++j) {
      const int i = j * 8 + wid;
      if (i >= C::TZ) break;
      const int byte = (i * 64 + lane) * 16;
      const int row = byte / (NOUT * 2);
      const int p = t * C::BM + row;
      const T* src = p < M ? static_cast<const T*>(bnb.z) + static_cast<int64_t>(p) * NT + slice * NOUT +
                                 (byte % (NOUT * 2)) / 2
                           : zero;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(sb + C::STAGE_IN + C::STAGE_ADD + i * 1024), 16, 0,
                                       0);
    }
    // the mask bytes of the tile's rows ([BM][NOUT / 8]; the stage's tail past them reads the zero page)
#pragma unroll
    for (int j = 0; j < (C::TM + 7) / 8; ++j) {
      const int i = j * 8 + wid;
      if (i >= C::TM) break;
      const int byte = (i * 64 + lane) * 16;
      const int row = byte / (NOUT / 8);
      const int p = t * C::BM + row;
      const void* src = (row < C::BM && p < M)
                            ? static_cast<const void*>(bnb.mask + (static_cast<int64_t>(p) * NT + slice * NOUT) / 8 +
                                                       byte % (NOUT / 8))
                            : static_cast<const void*>(zero);
      __builtin_amdgcn_global_load_lds((gbl_void*)src,
                                       (lds_void*)(sb + C::STAGE_IN + C::STAGE_ADD + C::STAGE_Z + i * 1024), 16, 0, 0);
    }
    // the addend's mask bytes (same layout as the BN mask)
#pragma unroll
    for (int j = 0; j < (C::TAM + 7) / 8; ++j) {
      const int i = j * 8 + wid;
      if (i >= C::TAM) break;
      const int byte = (i * 64 + lane) * 16;
      const int row = byte / (NOUT / 8);
      const int p = t * C::BM + row;
      const void* src = (row < C::BM && p < M)
                            ? static_cast<const void*>(bnb.amask + (static_cast<int64_t>(p) * NT + slice * NOUT) / 8 +
                                                       byte % (NOUT / 8))
                            : static_cast<const void*>(zero);
      __builtin_amdgcn_global_load_lds(
          (gbl_void*)src, (lds_void*)(sb + C::STAGE_IN + C::STAGE_ADD + C::STAGE_Z + C::STAGE_M + i * 1024), 16, 0, 0);
    }
  };
  // LDS-DMA instructions this wave issues per tile (uniform over the wave)
  const int ops_per_tile = EXT ? (C::TI - wid + 7) / 8 + (C::TA - wid + 7) / 8 + (C::TZ - wid + 7) / 8 +
                                      (C::TM - wid + 7) / 8 + (C::TAM - wid + 7) / 8
                                : C::LPT;

  const int my_tiles = wg < ntiles ? (ntiles - wg + gs - 1) / gs : 0;
  for (int j = 0; j < C::D && j < my_tiles; ++j) issue(wg + j * gs, j);

  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s1[e] = 0.f;
    s2[e] = 0.f;
  }
  const int my_c8 = tid % C::OCH;  // this thread's fixed output chunk (8 channels) in the epilogue
  char* epi = smem + C::NST * C::STAGE;
  // BN-backward constants of this thread's 8 channels
  float bmean[8], bsc[8], bsh[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int ch = slice * NOUT + my_c8 * 8 + q;
    bmean[q] = BNB ? bnb.mean[ch] : 0.f;
    bsc[q] = BNB == kPwBnbFromZ ? bnb.scale[ch] : 0.f;
    bsh[q] = BNB == kPwBnbFromZ ? bnb.shift[ch] : 0.f;
  }

  for (int it = 0; it < my_tiles; ++it) {
    const int t = wg + it * gs;
    const int st = it % C::NST;
    if (!EXT) {
      // issue tile it+D (into the stage freed by tile it-1, whose reads ended before the last barrier)
      if (it + C::D < my_tiles) issue(wg + (it + C::D) * gs, (it + C::D) % C::NST);
      // VM ops younger than tile it's DMA: the tiles issued after it, and the epilogue stores of the
      // iterations run since it was issued (tile j < D came from the prologue, tile j >= D from
      // iteration j - D)
      const int later = (my_tiles - 1 - it) < C::D ? (my_tiles - 1 - it) : C::D;
      const int epis = it < C::D ? it : C::D;
      if (later == C::D && epis == C::D) vm_wait<C::D*(C::LPT + C::SPT)>();
      else vm_wait_le(later * C::LPT + epis * C::SPT);
      lds_barrier();
    } else {
      // the store loop reads the addend part of a stage, so tile it+D (into tile it-1's stage) is
      // issued only after the barrier every thread reaches once its stores of tile it-1 are out:
      // younger than tile it's DMA are tiles it+1 .. it+D-1 and the stores of the iterations since
      const int later = (my_tiles - 1 - it) < C::D - 1 ? (my_tiles - 1 - it) : C::D - 1;
      const int epis = it < C::D ? it : C::D;
      vm_wait_n(later * ops_per_tile + epis * C::SPT);
      lds_barrier();
      if (it + C::D < my_tiles) issue(wg + (it + C::D) * gs, (it + C::D) % C::NST);
    }

    // ---- MFMA: C[co][pix] over the tile
    const char* sb = smem + st * C::STAGE;
    f4_t acc[C::FC][C::FP];
#pragma unroll
    for (int f = 0; f < C::FC; ++f)
#pragma unroll
      for (int p = 0; p < C::FP; ++p) acc[f][p] = f4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < C::KS; ++s) {
      u32x4 bf[C::FP];
#pragma unroll
      for (int p = 0; p < C::FP; ++p) {
        const int row = wp * C::FP * 16 + p * 16 + (lane & 15);
        const int chunk = s * 4 + (lane >> 4);
        bf[p] = *reinterpret_cast<const u32x4*>(sb + row * C::ROWB + ((chunk ^ (row & 7)) * 16));
      }
#pragma unroll
      for (int f = 0; f < C::FC; ++f)
#pragma unroll
        for (int p = 0; p < C::FP; ++p) acc[f][p] = PwM<T>::mma(wa[f][s], bf[p], acc[f][p]);
    }
    // ---- epilogue image: lane holds co = base + 4*(lane>>4) + {0..3} of pixel base + (lane & 15)
#pragma unroll
    for (int f = 0; f < C::FC; ++f)
#pragma unroll
      for (int p = 0; p < C::FP; ++p) {
        const int pix = wp * C::FP * 16 + p * 16 + (lane & 15);
        const int co = wc * C::FC * 16 + f * 16 + (lane >> 4) * 4;
        const f4_t v = acc[f][p];
        *reinterpret_cast<uint2*>(epi + pix * C::PITCH + co * 2) = PwM<T>::pack4(v[0], v[1], v[2], v[3]);
      }
    lds_barrier();
    // ---- coalesced row stores (exactly SPT per thread: rows past M go out of range by buffer bounds)
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        y, 0, static_cast<int>(static_cast<uint32_t>(M) * NT * sizeof(T)), 0x00020000);
#pragma unroll
    for (int k = 0; k < C::SPT; ++k) {
      // every lane issues the store (uniform VM-op count per wave for the counted waits): chunks past
      // the tile or rows past M get an out-of-range offset and are dropped by the buffer bounds
      const int e = tid + k * 512;
      const bool in_tile = e < C::BM * C::OCH;
      const int pix = in_tile ? e / C::OCH : 0;
      const int c8 = e % C::OCH;
      const int p = t * C::BM + pix;
      Vec8<T> v;
      v.raw = *reinterpret_cast<const uint4*>(epi + pix * C::PITCH + c8 * 16);
      if (ADD) {
        Vec8<T> a;
        a.raw = *reinterpret_cast<const uint4*>(sb + C::STAGE_IN + pix * (NOUT * 2) + c8 * 16);
        if (AMK) {
          // mask the addend's 16-bit elements with a bitwise AND (a cleared element is +0): bit 2j / 2j+1 of
          // the byte selects the low / high half of dword j
          const uint32_t amb = lds_byte(sb + C::STAGE_IN + C::STAGE_ADD + C::STAGE_Z + C::STAGE_M + pix * (NOUT / 8) + c8);
          auto m2 = [&](int j) -> uint32_t {
            const uint32_t b = (amb >> (2 * j)) & 3u;
            return (b & 1u) * 0xFFFFu | (b >> 1) * 0xFFFF0000u;
          };
          a.raw.x &= m2(0);
          a.raw.y &= m2(1);
          a.raw.z &= m2(2);
          a.raw.w &= m2(3);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) v.set(q, v.get(q) + a.get(q));
      }
      const bool live = in_tile && p < M;
      if (BNB && live) {
        Vec8<T> zv;
        zv.raw = *reinterpret_cast<const uint4*>(sb + C::STAGE_IN + C::STAGE_ADD + pix * (NOUT * 2) + c8 * 16);
        const uint32_t mb =
            BNB == kPwBnbMask ? lds_byte(sb + C::STAGE_IN + C::STAGE_ADD + C::STAGE_Z + pix * (NOUT / 8) + c8)
                              : 0xffu;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float zq = zv.get(q);
          bool keep = true;
          if (BNB == kPwBnbFromZ) keep = fmaf(zq, bsc[q], bsh[q]) > 0.f;
          if (BNB == kPwBnbMask) keep = (mb >> q) & 1u;
          const float dz = keep ? v.get(q) : 0.f;
          s1[q] += dz;
          s2[q] += dz * (zq - bmean[q]);
        }
      }
      const uint32_t off = live ? (static_cast<uint32_t>(p) * NT + slice * NOUT + c8 * 8) * sizeof(T) : 0xFFFFFFF0u;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v.raw), yrs, off, 0, 0);
      if (STATS && live) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float z = v.get(q);
          s1[q] += z;
          s2[q] += z * z;
        }
      }
    }
    (void)my_c8;
  }
  if (STATS || BNB) {
    // every thread's chunk is fixed (tid % OCH): combine the 512/OCH threads of each chunk through
    // LDS, one partial per workgroup per channel
    vm_wait<0>();
    lds_barrier();
    float* red = reinterpret_cast<float*>(smem);
    constexpr int ROWS = 512 / C::OCH;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      red[(tid / C::OCH) * NOUT + my_c8 * 8 + q] = s1[q];
      red[ROWS * NOUT + (tid / C::OCH) * NOUT + my_c8 * 8 + q] = s2[q];
    }
    lds_barrier();
    for (int qq = tid; qq < 2 * NOUT; qq += 512) {
      const int which = qq / NOUT, ch = qq - which * NOUT;
      const float* col = red + which * ROWS * NOUT + ch;
      float a = 0.f;
      for (int r = 0; r < ROWS; ++r) a += col[r * NOUT];
      part[static_cast<int64_t>(which) * NT * gs + static_cast<int64_t>(slice * NOUT + ch) * gs + wg] = a;
    }
  }
}

template <typename T, int KIN, int NOUT, int WPC, int S, bool STATS, bool ADD, int BNB = kPwBnbNone, bool AMK = false>
void launch_pw_v(const void* x, const void* w, void* y, const void* zero, int M, float* part, const void* addend,
                 int grid, hipStream_t s, int wt, const PwBnb& bnb = PwBnb{}) {
  using C = PwCfg<KIN, NOUT, WPC, ADD, BNB, AMK>;
  static_assert(C::SMEM <= C::LDS && C::NST >= 2, "LDS budget / ring depth");
  static bool set = false;
  if (!set) {
    hipFuncSetAttribute(
        reinterpret_cast<const void*>(&conv_pw_stream_kernel<T, KIN, NOUT, STATS, ADD, WPC, S, BNB, AMK>),
        hipFuncAttributeMaxDynamicSharedMemorySize, C::SMEM);
    set = true;
  }
  const int ntiles = (M + C::BM - 1) / C::BM;
  hipLaunchKernelGGL((conv_pw_stream_kernel<T, KIN, NOUT, STATS, ADD, WPC, S, BNB, AMK>), dim3(grid), dim3(512), C::SMEM,
                     s, static_cast<const T*>(x), static_cast<const T*>(w), static_cast<T*>(y),
                     static_cast<const T*>(zero), M, ntiles, part, static_cast<const T*>(addend), wt, bnb);
}

// BN-backward variants built: relu-from-z without an addend (a dgrad feeding BN+ReLU) and the
// residual tail's mask with an addend (a tee dgrad feeding the previous block's tail)
template <int KIN, int NOUT>
constexpr bool pw_bnb_built(bool add, int mode) {
  return add ? (mode == kPwBnbMask && (NOUT / 8) % 16 == 0) : mode == kPwBnbFromZ;
}

template <typename T, int KIN, int NOUT, int S>
bool launch_pw_bnb(const void* x, const void* w, void* y, const void* zero, int M, float* part, const void* addend,
                   int grid, hipStream_t s, int wt, const PwBnb& bnb, int mode) {
  if constexpr ((NOUT / 8) % 16 == 0) {
    if (addend && mode == kPwBnbMask) {
      if (bnb.amask)
        launch_pw_v<T, KIN, NOUT, 1, S, false, true, kPwBnbMask, true>(x, w, y, zero, M, part, addend, grid, s, wt,
                                                                        bnb);
      else
        launch_pw_v<T, KIN, NOUT, 1, S, false, true, kPwBnbMask>(x, w, y, zero, M, part, addend, grid, s, wt, bnb);
      return true;
    }
  }
  if (!addend && mode == kPwBnbFromZ) {
    launch_pw_v<T, KIN, NOUT, 1, S, false, false, kPwBnbFromZ>(x, w, y, zero, M, part, addend, grid, s, wt, bnb);
    return true;
  }
  return false;
}

template <typename T, int KIN, int NOUT, int WPC, int S>
void launch_pw(const void* x, const void* w, void* y, const void* zero, int M, float* part, const void* addend,
               int grid, hipStream_t s, int wt, const PwBnb* bnb, int mode) {
  if (bnb) {
    MXAMD_HOST_CHECK((launch_pw_bnb<T, KIN, NOUT, S>(x, w, y, zero, M, part, addend, grid, s, wt, *bnb, mode)),
                     "conv_pw_stream: BN-backward variant not built");
    return;
  }
  using C = PwCfg<KIN, NOUT, WPC>;
  using CA = PwCfg<KIN, NOUT, 1, true>;
  static_assert(C::SMEM <= C::LDS && CA::SMEM <= CA::LDS, "workgroups per CU");
  static_assert(C::NST >= 2 && CA::NST >= 2, "ring depth");
  if (part) {
    if (addend) launch_pw_v<T, KIN, NOUT, 1, S, true, true>(x, w, y, zero, M, part, addend, grid, s, wt);
    else launch_pw_v<T, KIN, NOUT, WPC, S, true, false>(x, w, y, zero, M, part, addend, grid, s, wt);
  } else {
    if (addend) launch_pw_v<T, KIN, NOUT, 1, S, false, true>(x, w, y, zero, M, part, addend, grid, s, wt);
    else launch_pw_v<T, KIN, NOUT, WPC, S, false, false>(x, w, y, zero, M, part, addend, grid, s, wt);
  }
}

// (Cin, Cout per workgroup, workgroups per CU, slices) built: weight matrices up to 32K elements stay
// resident at two workgroups per CU (128 VGPRs), up to 128K elements at one workgroup per CU; larger
// layers are sliced along Cout (Cout = Cout per workgroup x slices)
#define MXAMD_PW_SHAPES(X)                                                                                  \
  X(64, 64, 2, 1) X(64, 128, 2, 1) X(64, 256, 2, 1) X(128, 128, 2, 1) X(128, 256, 2, 1) X(256, 64, 2, 1)     \
  X(256, 128, 2, 1) X(512, 128, 2, 1) X(128, 512, 1, 1) X(256, 512, 1, 1) X(512, 256, 1, 1) X(256, 512, 1, 2) \
  X(1024, 128, 1, 2) X(512, 256, 1, 8)

template <typename T>
bool dispatch_pw(int kin, int nout, const void* x, const void* w, void* y, const void* zero, int M, float* part,
                 const void* addend, int grid, hipStream_t s, int wt, const PwBnb* bnb, int mode) {
#define MXAMD_PW_CASE(K, N, W, SL)                                        \
  if (kin == K && nout == N * SL) {                                       \
    launch_pw<T, K, N, W, SL>(x, w, y, zero, M, part, addend, grid, s, wt, bnb, mode); \
    return true;                                                          \
  }
  MXAMD_PW_SHAPES(MXAMD_PW_CASE)
#undef MXAMD_PW_CASE
  return false;
}

}  // namespace

// Workgroups per CU (> 0) when conv_pw_stream handles a 1x1 stride-1 NHWC conv with Cin = kin,
// Cout = nout; 0 otherwise.
int conv_pw_stream_ok(int kin, int nout) {
#define MXAMD_PW_OK(K, N, W, SL) \
  if (kin == K && nout == N * SL) return W;
  MXAMD_PW_SHAPES(MXAMD_PW_OK)
#undef MXAMD_PW_OK
  return 0;
}

// Workgroups the kernel launches (= BatchNorm partials per channel when statistics are requested).
// Cout slices of a (Cin, Cout) layer (1 when not sliced, 0 when not built).
int conv_pw_stream_slices(int kin, int nout) {
#define MXAMD_PW_SL(K, N, W, SL) \
  if (kin == K && nout == N * SL) return SL;
  MXAMD_PW_SHAPES(MXAMD_PW_SL)
#undef MXAMD_PW_SL
  return 0;
}

// Whether a BN-backward statistics epilogue is built for (Cin, Cout, addend, mode).
int conv_pw_stream_bnb_ok(int kin, int nout, int add, int mode) {
#define MXAMD_PW_BOK(K, N, W, SL) \
  if (kin == K && nout == N * SL) return pw_bnb_built<K, N>(add != 0, mode) ? 1 : 0;
  MXAMD_PW_SHAPES(MXAMD_PW_BOK)
#undef MXAMD_PW_BOK
  return 0;
}

// add: the launch streams an extra tensor (addend and / or BN-backward input): 1 workgroup per CU
int conv_pw_stream_grid(int M, int kin, int nout, int ncu, int add) {
  const int sl = conv_pw_stream_slices(kin, nout);
  if (sl == 0) return 0;
  const int bm = pw_bm(kin, nout / sl, add != 0);
  const int ntiles = (M + bm - 1) / bm;
  const int wpc = add ? 1 : conv_pw_stream_ok(kin, nout);
  int per = (wpc * ncu + sl - 1) / sl;                 // tile walkers per slice
  if (per > ntiles) per = ntiles;
  return per * sl;
}

// addend_mask (optional, BN-mask mode with an addend only): the addend is dy * these ReLU bits
void conv_pw_stream(int dtype, const void* x, const void* w, void* y, const void* zero, int M, int kin, int nout,
                    float* part, int grid, hipStream_t s, const void* addend, int wt, const void* bn_z,
                    const uint8_t* bn_mask, const float* bn_mean, const float* bn_scale, const float* bn_shift,
                    int bn_mode, const uint8_t* addend_mask) {
  MXAMD_HOST_CHECK(conv_pw_stream_ok(kin, nout), "conv_pw_stream: unsupported (Cin, Cout)");
  MXAMD_HOST_CHECK(grid >= 1 && grid % conv_pw_stream_slices(kin, nout) == 0 &&
                   (int64_t)M * nout * 2 < (1ll << 31) - 64 && (int64_t)M * kin < (1ll << 31),
                   "conv_pw_stream: tensor too large for 32-bit offsets");
  PwBnb bnb{bn_z, bn_mask, bn_mean, bn_scale, bn_shift, addend_mask};
  MXAMD_HOST_CHECK(addend_mask == nullptr || (addend && bn_z && bn_mode == kPwBnbMask),
                   "conv_pw_stream: the addend mask is built for the tee data gradient with the tail's BN statistics");
  const PwBnb* pb = nullptr;
  if (bn_z) {
    MXAMD_HOST_CHECK(part && bn_mean && conv_pw_stream_bnb_ok(kin, nout, addend != nullptr, bn_mode) &&
                         (bn_mode != kPwBnbFromZ || (bn_scale && bn_shift)) && (bn_mode != kPwBnbMask || bn_mask),
                     "conv_pw_stream: BN-backward statistics need partials, mean, a built mode and its mask source");
    pb = &bnb;
  }
  bool ok = false;
  if (dtype == kF16) ok = dispatch_pw<__half>(kin, nout, x, w, y, zero, M, part, addend, grid, s, wt, pb, bn_mode);
  else if (dtype == kBF16)
    ok = dispatch_pw<__hip_bfloat16>(kin, nout, x, w, y, zero, M, part, addend, grid, s, wt, pb, bn_mode);
  MXAMD_HOST_CHECK(ok, "conv_pw_stream: dtype must be f16 or bf16");
}

}  // namespace mxamd
