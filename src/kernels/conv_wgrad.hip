// NHWC convolution weight gradient on CDNA4 matrix cores (gfx950).
//
// Parity: the backward-filter pass of src/operator/nn/convolution.cu (cuDNN
// BackwardFilter / MIOpen wrw in the reference stack).  MI355X-first design:
//
//   dW[k][r][s][c] = sum_pix dY[pix][k] * X[n, ho*sh-ph+r, wo*sw-pw+s, c]
//
//   GEMM view: rows = (r,s,c) ("rsc", the OHWI weight row), cols = k, reduction
//   over output pixels.  Both NHWC operands are CHANNEL-contiguous, so the
//   reduction dimension (pixels) is strided in memory.  Tiles are staged
//   global -> registers -> LDS in their natural [pixel][channel] layout and the
//   MFMA fragments (8 consecutive pixels of one channel per lane) are read with
//   the gfx950 hardware-transposing LDS read ds_read_b64_tr_b16 -- no shuffle,
//   no transposing store.
//
//   Every operand tile is a [64 pixel][64 channel] f16/bf16 "sub-tile" (8 KB,
//   128-byte rows).  The 16-byte chunk index of row r is XORed with
//   swz(r) = 2*((r>>1)&1) | 4*((r>>3)&1): the 8 rows a 32-lane half reads
//   together (rows q, q+8 of a 16-row group) then cover all 64 banks once, so
//   the transposed reads are conflict-free.
//
//   Block = WM x WN waves; wave (wm, wn) owns a (16*FM)(rsc) x 64(k) output
//   tile (FM x 4 v_mfma_f32_16x16x32 fragments, FM = 4 or 8: the 128-row wave
//   tile halves the LDS read traffic per MFMA of the big layers).  A = X^T
//   sub-tiles [wm*FM/4, +FM/4), B = dY sub-tile wn; the accumulator layout (row = 4*(lane>>4)+reg, col = lane&15) gives each
//   lane 4 consecutive rsc of one k -> 16-byte fp32 stores.
//
//   The pixel reduction (12k-800k terms) is split over blocks ("splits");
//   each block writes an fp32 slab [split][K][RSC] and a second kernel sums the
//   slabs and writes / accumulates the f16/bf16/f32 gradient (deterministic,
//   no atomics).  Blocks are remapped XCD-aware so the tiles of one pixel range
//   (which re-read the same dY / X rows) share an L2.
#include <algorithm>
#include <stdexcept>

#include "common.h"
#include "mfma.h"

namespace mxamd {

namespace {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

struct FastDiv {
  uint32_t d, m, s;
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  f.s = 0;
  while ((1u << f.s) < d) ++f.s;
  f.m = static_cast<uint32_t>((((uint64_t)1 << 32) * (((uint64_t)1 << f.s) - d)) / d + 1);
  return f;
}

// n / d for n < 2^31
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) { return (__umulhi(n, f.m) + n) >> f.s; }

template <typename T>
struct Mfma16 : mfma::Op<T> {};   // 16x16x32 MFMA (mfma.h)

struct WgradGeom {
  int N, H, W, C, K, R, S, Ho, Wo, sh, sw, ph, pw;
  int dh, dw;   // dilation: tap (r, s) reads input row ho*sh - ph + r*dh, column wo*sw - pw + s*dw
  int P;        // N*Ho*Wo output pixels (reduction length)
  int RSC;      // R*S*C (GEMM rows)
  int tiles_m;  // RSC / (16*FM*WM)
  int tiles;    // tiles_m * K / (64*WN)
  int plen;     // pixels per split (multiple of 64)
  FastDiv fWo, fHoWo;
};

__device__ __forceinline__ int swz(int row) { return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2); }

// 8 consecutive pixels (rows) of one channel (column) for this lane's MFMA fragment:
// two ds_read_b64_tr_b16 over rows [8g+q] and [8g+4+q] (byte offset `off` already
// includes the row/chunk of this lane; +512 B = 4 rows further).
__device__ __forceinline__ v8s tr_frag(const void* tile, int off) {
  typedef __attribute__((address_space(3))) char lds_char;
  lds_char* base = (lds_char*)(tile);
  v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(base + off));
  v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(base + off + 512));
  return v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <typename T, int WM, int WN, int FM, bool IDENT>
__global__ void __launch_bounds__(64 * WM * WN) conv_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                                  float* __restrict__ slab, WgradGeom g) {
  constexpr int NT = 64 * WM * WN;
  constexpr int MS = FM / 4;               // X sub-tiles per wave
  constexpr int XSUB = WM * MS;            // X sub-tiles per block
  constexpr int NSUB = XSUB + WN;
  constexpr int SUB = 64 * 64;             // elements per sub-tile
  constexpr int CHUNKS = NSUB * 512;       // 16-byte chunks per stage
  constexpr int LPT = (CHUNKS + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) T smem[2 * NSUB * SUB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid % WM;
  const int wn = wid / WM;

  // XCD-aware bijective remap: consecutive logical blocks (the tiles of one split) share an XCD
  const int nblk = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q8 = nblk >> 3, r8 = nblk & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tile = wgid % g.tiles;
  const int split = wgid / g.tiles;
  const int tm = tile % g.tiles_m;
  const int tn = tile / g.tiles_m;
  const int m0 = tm * 64 * XSUB;
  const int n0 = tn * 64 * WN;
  const int pbeg = split * g.plen;
  const int pend = min(g.P, pbeg + g.plen);
  const int KT = (pend - pbeg + 63) >> 6;

  // ---- per-slot load descriptors (fixed across k-steps)
  int s_row[LPT], s_lds[LPT], s_col[LPT], s_r[LPT], s_s[LPT];
  bool s_on[LPT], s_isx[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    const int idx = tid + i * NT;
    s_on[i] = idx < CHUNKS;
    const int sub = s_on[i] ? idx >> 9 : 0;
    const int within = idx & 511;
    const int row = within >> 3, ch = within & 7;
    s_row[i] = row;
    s_lds[i] = sub * SUB + row * 64 + ((ch ^ swz(row)) << 3);
    s_isx[i] = sub < XSUB;
    if (s_isx[i]) {
      const int n = m0 + sub * 64 + ch * 8;  // rsc column
      const int rs = n / g.C;
      s_col[i] = n - rs * g.C;
      s_r[i] = (rs / g.S) * g.dh;
      s_s[i] = (rs - (rs / g.S) * g.S) * g.dw;
    } else {
      s_col[i] = n0 + (sub - XSUB) * 64 + ch * 8;
      s_r[i] = s_s[i] = 0;
    }
  }

  u32x4 reg[LPT];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int p = pbeg + kt * 64 + s_row[i];
      bool ok = s_on[i] && p < pend;
      int off;
      if (!s_isx[i]) {
        off = p * g.K + s_col[i];
      } else if (IDENT) {
        off = p * g.C + s_col[i];
      } else {
        const int nimg = (int)fdiv((uint32_t)p, g.fHoWo);
        const int rem = p - nimg * (g.Ho * g.Wo);
        const int ho = (int)fdiv((uint32_t)rem, g.fWo);
        const int wo = rem - ho * g.Wo;
        const int hi = ho * g.sh - g.ph + s_r[i];
        const int wi = wo * g.sw - g.pw + s_s[i];
        ok = ok && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
        off = ((nimg * g.H + hi) * g.W + wi) * g.C + s_col[i];
      }
      const T* base = s_isx[i] ? x : dy;
      reg[i] = ok ? *reinterpret_cast<const u32x4*>(base + off) : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LPT; ++i)
      if (s_on[i]) *reinterpret_cast<u32x4*>(smem + buf * NSUB * SUB + s_lds[i]) = reg[i];
  };

  // per-lane fragment byte offsets within a sub-tile for the 4 fragments (16 channels each)
  const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
  const int frow = 8 * fg + fq;
  int foff[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) foff[f] = frow * 128 + ((((2 * f) + (fp >> 1)) ^ swz(frow)) << 4) + ((fp & 1) << 3);

  f4_t acc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};

  if (KT > 0) {
    gload(0);
    sstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) gload(kt + 1);
    const T* sx = smem + buf * NSUB * SUB + wm * MS * SUB;
    const T* sd = smem + buf * NSUB * SUB + (XSUB + wn) * SUB;
#pragma unroll
    for (int kk = 0; kk < 64; kk += 32) {
      v8s a[FM], b[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) b[f] = tr_frag(sd, kk * 128 + foff[f]);
#pragma unroll
      for (int f = 0; f < FM; ++f) a[f] = tr_frag(sx + (f >> 2) * SUB, kk * 128 + foff[f & 3]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = Mfma16<T>::run(a[i], b[j], acc[i][j]);
    }
    if (kt + 1 < KT) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: lane holds rsc = base + 4*(lane>>4) + {0..3} for k = base + (lane&15)
  float* out = slab + (size_t)split * g.K * g.RSC;
  const int rsc_l = (lane >> 4) * 4;
  const int k_l = lane & 15;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int rsc = m0 + wm * MS * 64 + i * 16 + rsc_l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = n0 + wn * 64 + j * 16 + k_l;
      *reinterpret_cast<f4_t*>(out + (size_t)k * g.RSC + rsc) = acc[i][j];
    }
  }
}

// the LDS-DMA operand loads use the default cache policy (a non-temporal policy on x / dY measured as
// noise on the ResNet-50 step, profiles/r5x_*)

// LDS-DMA variant: the same sub-tile images filled with global_load_lds_dwordx4
// (one wave-instruction = 8 rows x 128 B of a sub-tile, lane L -> row L>>3,
// position L&7, fetching global chunk (L&7) ^ swz(row)); out-of-range pixels
// come from a zero page.  No staging registers, no ds_write in the loop; the
// next 64-pixel stage is in flight during the current stage's MFMAs.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

template <typename T, int WM, int WN, bool IDENT>
__global__ void __launch_bounds__(64 * WM * WN) conv_wgrad_glds_kernel(const T* __restrict__ x,
                                                                       const T* __restrict__ dy,
                                                                       float* __restrict__ slab,
                                                                       const T* __restrict__ zero, WgradGeom g) {
  constexpr int NW = WM * WN;
  constexpr int NSUB = WM + WN;
  constexpr int SUB = 64 * 64;
  constexpr int NINS = NSUB * 8;                 // wave-instructions per stage
  constexpr int IPW = (NINS + NW - 1) / NW;      // per wave
  __shared__ __attribute__((aligned(1024))) T smem[2 * NSUB * SUB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid % WM;
  const int wn = wid / WM;

  const int nblk = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q8 = nblk >> 3, r8 = nblk & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tile = wgid % g.tiles;
  const int split = wgid / g.tiles;
  const int tm = tile % g.tiles_m;
  const int tn = tile / g.tiles_m;
  const int m0 = tm * 64 * WM;
  const int n0 = tn * 64 * WN;
  const int pbeg = split * g.plen;
  const int pend = min(g.P, pbeg + g.plen);
  const int KT = (pend - pbeg + 63) >> 6;

  // per-instruction descriptors (instruction ins = wid + i*NW: sub-tile ins>>3, row group ins&7)
  const int t = lane >> 3;
  int d_row[IPW], d_col[IPW], d_r[IPW], d_s[IPW], d_lds[IPW];
  bool d_on[IPW], d_isx[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int ins = wid + i * NW;
    d_on[i] = ins < NINS;
    const int sub = d_on[i] ? ins >> 3 : 0;
    const int row = (ins & 7) * 8 + t;
    const int gch = (lane & 7) ^ swz(row);
    d_row[i] = row;
    d_lds[i] = sub * SUB * (int)sizeof(T) + (ins & 7) * 1024;
    d_isx[i] = sub < WM;
    if (d_isx[i]) {
      const int n = m0 + sub * 64;           // first rsc column of the sub-tile (one (r, s): C % 64 == 0)
      const int rs = n / g.C;
      d_col[i] = n - rs * g.C + gch * 8;
      d_r[i] = (rs / g.S) * g.dh;
      d_s[i] = (rs - (rs / g.S) * g.S) * g.dw;
    } else {
      d_col[i] = n0 + (sub - WM) * 64 + gch * 8;
      d_r[i] = d_s[i] = 0;
    }
  }
  const T* zsrc = zero + ((lane & 7) << 3);

  auto issue = [&](int kt, int buf) {
    char* sbase = reinterpret_cast<char*>(smem + buf * NSUB * SUB);
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      if (!d_on[i]) continue;                 // wave-uniform
      const int p = pbeg + kt * 64 + d_row[i];
      bool ok = p < pend;
      const T* src;
      if (!d_isx[i]) {
        src = dy + (int64_t)p * g.K + d_col[i];
      } else if (IDENT) {
        src = x + (int64_t)p * g.C + d_col[i];
      } else {
        const int nimg = (int)fdiv((uint32_t)p, g.fHoWo);
        const int rem = p - nimg * (g.Ho * g.Wo);
        const int ho = (int)fdiv((uint32_t)rem, g.fWo);
        const int wo = rem - ho * g.Wo;
        const int hi = ho * g.sh - g.ph + d_r[i];
        const int wi = wo * g.sw - g.pw + d_s[i];
        ok = ok && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
        src = x + ((int64_t)(nimg * g.H + hi) * g.W + wi) * g.C + d_col[i];
      }
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(ok ? src : zsrc), (lds_void_t*)(sbase + d_lds[i]), 16, 0,
                                       0);
    }
  };

  const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
  const int frow = 8 * fg + fq;
  int foff[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) foff[f] = frow * 128 + ((((2 * f) + (fp >> 1)) ^ swz(frow)) << 4) + ((fp & 1) << 3);

  f4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};

  if (KT > 0) issue(0, 0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) issue(kt + 1, buf ^ 1);
    const T* sx = smem + buf * NSUB * SUB + wm * SUB;
    const T* sd = smem + buf * NSUB * SUB + (WM + wn) * SUB;
#pragma unroll
    for (int kk = 0; kk < 64; kk += 32) {
      v8s a[4], b[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) b[f] = tr_frag(sd, kk * 128 + foff[f]);
#pragma unroll
      for (int f = 0; f < 4; ++f) a[f] = tr_frag(sx, kk * 128 + foff[f]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = Mfma16<T>::run(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }

  float* out = slab + (size_t)split * g.K * g.RSC;
  const int rsc_l = (lane >> 4) * 4;
  const int k_l = lane & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rsc = m0 + wm * 64 + i * 16 + rsc_l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = n0 + wn * 64 + j * 16 + k_l;
      *reinterpret_cast<f4_t*>(out + (size_t)k * g.RSC + rsc) = acc[i][j];
    }
  }
}

// s_waitcnt vmcnt(N) only (gfx9 encoding; expcnt / lgkmcnt at their maxima)
template <int N>
__device__ __forceinline__ void wg_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
// wait until at most n VM ops are outstanding, n rounded DOWN to a level (always safe)
__device__ __forceinline__ void wg_vm_wait_le(int n) {
  if (n >= 32) wg_vm_wait<32>();
  else if (n >= 24) wg_vm_wait<24>();
  else if (n >= 20) wg_vm_wait<20>();
  else if (n >= 16) wg_vm_wait<16>();
  else if (n >= 12) wg_vm_wait<12>();
  else if (n >= 10) wg_vm_wait<10>();
  else if (n >= 8) wg_vm_wait<8>();
  else if (n >= 6) wg_vm_wait<6>();
  else if (n >= 5) wg_vm_wait<5>();
  else if (n >= 4) wg_vm_wait<4>();
  else if (n >= 3) wg_vm_wait<3>();
  else if (n >= 2) wg_vm_wait<2>();
  else if (n >= 1) wg_vm_wait<1>();
  else wg_vm_wait<0>();
}

// Weight gradient with an NST-stage LDS-DMA ring over the pixel (reduction) stream.
// Same sub-tile images / transposed fragment reads as conv_wgrad_glds_kernel, but D = NST-1 pixel
// steps stay in flight across each barrier (counted vmcnt + raw s_barrier instead of
// __syncthreads(), which would drain the DMA queue), and the host plans few, long splits (about one
// workgroup per CU) so the fp32 slab traffic stays small next to the operand stream.
template <typename T, int WM, int WN, int NST, int FM, bool IDENT>
__global__ void __launch_bounds__(64 * WM * WN) conv_wgrad_ring_kernel(const T* __restrict__ x,
                                                                       const T* __restrict__ dy,
                                                                       float* __restrict__ slab,
                                                                       const T* __restrict__ zero, WgradGeom g) {
  constexpr int NW = WM * WN;
  constexpr int MS = FM / 4;               // X sub-tiles (64 rsc) per wave
  constexpr int XSUB = WM * MS;            // X sub-tiles per block
  constexpr int NSUB = XSUB + WN;
  constexpr int SUB = 64 * 64;
  constexpr int STAGE_B = NSUB * SUB * (int)sizeof(T);
  constexpr int NINS = NSUB * 8;                 // wave-instructions per stage
  constexpr int IPW = (NINS + NW - 1) / NW;      // per wave (upper bound)
  constexpr int D = NST - 1;
  extern __shared__ __attribute__((aligned(1024))) char wsm[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid % WM;
  const int wn = wid / WM;

  const int nblk = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q8 = nblk >> 3, r8 = nblk & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tile = wgid % g.tiles;
  const int split = wgid / g.tiles;
  const int tm = tile % g.tiles_m;
  const int tn = tile / g.tiles_m;
  const int m0 = tm * 64 * XSUB;
  const int n0 = tn * 64 * WN;
  const int pbeg = split * g.plen;
  const int pend = min(g.P, pbeg + g.plen);
  const int KT = pend > pbeg ? (pend - pbeg + 63) >> 6 : 0;

  const int t = lane >> 3;
  int d_row[IPW], d_col[IPW], d_r[IPW], d_s[IPW], d_lds[IPW];
  bool d_on[IPW], d_isx[IPW];
  int lpt = 0;   // LDS-DMA instructions this wave issues per pixel step
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int ins = wid + i * NW;
    d_on[i] = ins < NINS;
    lpt += d_on[i] ? 1 : 0;
    const int sub = d_on[i] ? ins >> 3 : 0;
    const int row = (ins & 7) * 8 + t;
    const int gch = (lane & 7) ^ swz(row);
    d_row[i] = row;
    d_lds[i] = sub * SUB * (int)sizeof(T) + (ins & 7) * 1024;
    d_isx[i] = sub < XSUB;
    if (d_isx[i]) {
      const int n = m0 + sub * 64;
      const int rs = n / g.C;
      d_col[i] = n - rs * g.C + gch * 8;
      d_r[i] = (rs / g.S) * g.dh;
      d_s[i] = (rs - (rs / g.S) * g.S) * g.dw;
    } else {
      d_col[i] = n0 + (sub - XSUB) * 64 + gch * 8;
      d_r[i] = d_s[i] = 0;
    }
  }
  const T* zsrc = zero + ((lane & 7) << 3);

  int i_kt = 0, i_stage = 0;
  auto issue = [&]() {
    char* sbase = wsm + i_stage * STAGE_B;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      if (!d_on[i]) continue;                 // wave-uniform
      const int p = pbeg + i_kt * 64 + d_row[i];
      bool ok = p < pend;
      const T* src;
      if (!d_isx[i]) {
        src = dy + (int64_t)p * g.K + d_col[i];
      } else if (IDENT) {
        src = x + (int64_t)p * g.C + d_col[i];
      } else {
        const int nimg = (int)fdiv((uint32_t)p, g.fHoWo);
        const int rem = p - nimg * (g.Ho * g.Wo);
        const int ho = (int)fdiv((uint32_t)rem, g.fWo);
        const int wo = rem - ho * g.Wo;
        const int hi = ho * g.sh - g.ph + d_r[i];
        const int wi = wo * g.sw - g.pw + d_s[i];
        ok = ok && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
        src = x + ((int64_t)(nimg * g.H + hi) * g.W + wi) * g.C + d_col[i];
      }
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(ok ? src : zsrc), (lds_void_t*)(sbase + d_lds[i]), 16, 0,
                                       0);
    }
    ++i_kt;
    i_stage = (i_stage + 1 == NST) ? 0 : i_stage + 1;
  };

  const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
  const int frow = 8 * fg + fq;
  int foff[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) foff[f] = frow * 128 + ((((2 * f) + (fp >> 1)) ^ swz(frow)) << 4) + ((fp & 1) << 3);

  f4_t acc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};

  const int npro = KT < D ? KT : D;
  for (int p = 0; p < npro; ++p) issue();
  int c_stage = 0;
  for (int kt = 0; kt < KT; ++kt) {
    const int ahead = (KT - 1 - kt) < (D - 1) ? (KT - 1 - kt) : (D - 1);
    wg_vm_wait_le(ahead * lpt);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + D < KT) issue();
    const T* sx = reinterpret_cast<const T*>(wsm + c_stage * STAGE_B) + wm * MS * SUB;
    const T* sd = reinterpret_cast<const T*>(wsm + c_stage * STAGE_B) + (XSUB + wn) * SUB;
#pragma unroll
    for (int kk = 0; kk < 64; kk += 32) {
      v8s a[FM], b[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) b[f] = tr_frag(sd, kk * 128 + foff[f]);
#pragma unroll
      for (int f = 0; f < FM; ++f) a[f] = tr_frag(sx + (f >> 2) * SUB, kk * 128 + foff[f & 3]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = Mfma16<T>::run(a[i], b[j], acc[i][j]);
    }
    c_stage = (c_stage + 1 == NST) ? 0 : c_stage + 1;
  }

  float* out = slab + (size_t)split * g.K * g.RSC;
  const int rsc_l = (lane >> 4) * 4;
  const int k_l = lane & 15;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int rsc = m0 + wm * MS * 64 + i * 16 + rsc_l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = n0 + wn * 64 + j * 16 + k_l;
      *reinterpret_cast<f4_t*>(out + (size_t)k * g.RSC + rsc) = acc[i][j];
    }
  }
}

template <typename OutT>
__device__ __forceinline__ void store4(OutT* p, f4_t v);
template <>
__device__ __forceinline__ void store4<float>(float* p, f4_t v) {
  *reinterpret_cast<f4_t*>(p) = v;
}
template <>
__device__ __forceinline__ void store4<__half>(__half* p, f4_t v) {
  __half2 a = __floats2half2_rn(v[0], v[1]), b = __floats2half2_rn(v[2], v[3]);
  uint2 r;
  r.x = *reinterpret_cast<uint32_t*>(&a);
  r.y = *reinterpret_cast<uint32_t*>(&b);
  *reinterpret_cast<uint2*>(p) = r;
}
template <>
__device__ __forceinline__ void store4<__hip_bfloat16>(__hip_bfloat16* p, f4_t v) {
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t b = __float_as_uint(v[i]);
    u[i] = (b + 0x7fffu + ((b >> 16) & 1u)) >> 16;
  }
  uint2 r;
  r.x = u[0] | (u[1] << 16);
  r.y = u[2] | (u[3] << 16);
  *reinterpret_cast<uint2*>(p) = r;
}

template <typename OutT>
__device__ __forceinline__ f4_t load4(const OutT* p);
template <>
__device__ __forceinline__ f4_t load4<float>(const float* p) {
  return *reinterpret_cast<const f4_t*>(p);
}
template <>
__device__ __forceinline__ f4_t load4<__half>(const __half* p) {
  uint2 r = *reinterpret_cast<const uint2*>(p);
  __half2 a = *reinterpret_cast<__half2*>(&r.x), b = *reinterpret_cast<__half2*>(&r.y);
  float2 fa = __half22float2(a), fb = __half22float2(b);
  return f4_t{fa.x, fa.y, fb.x, fb.y};
}
template <>
__device__ __forceinline__ f4_t load4<__hip_bfloat16>(const __hip_bfloat16* p) {
  uint2 r = *reinterpret_cast<const uint2*>(p);
  return f4_t{__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u), __uint_as_float(r.y << 16),
              __uint_as_float(r.y & 0xffff0000u)};
}

// Sum `nrows` slab rows (row r at slab + r*row_stride) column-wise, 4 columns per thread.
// FINAL: out = (accum ? out : 0) + sum (converted to OutT); else the partial sum
// overwrites row 0 of the group (only this thread ever reads those columns).
template <typename OutT, bool FINAL>
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(float* __restrict__ slab, int nrows, int64_t row_stride,
                                                           int rows_per_group, int64_t n, OutT* __restrict__ out,
                                                           int accum) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= n) return;
  const int r0 = blockIdx.y * rows_per_group;
  const int r1 = min(nrows, r0 + rows_per_group);
  float* base = slab + i4;
  f4_t s0 = f4_t{0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, s3 = s0;
  int r = r0;
  for (; r + 3 < r1; r += 4) {
    s0 += *reinterpret_cast<const f4_t*>(base + (int64_t)r * row_stride);
    s1 += *reinterpret_cast<const f4_t*>(base + (int64_t)(r + 1) * row_stride);
    s2 += *reinterpret_cast<const f4_t*>(base + (int64_t)(r + 2) * row_stride);
    s3 += *reinterpret_cast<const f4_t*>(base + (int64_t)(r + 3) * row_stride);
  }
  for (; r < r1; ++r) s0 += *reinterpret_cast<const f4_t*>(base + (int64_t)r * row_stride);
  s0 += s1 + s2 + s3;
  if (FINAL) {
    if (accum) s0 += load4<OutT>(out + i4);
    store4<OutT>(out + i4, s0);
  } else {
    *reinterpret_cast<f4_t*>(base + (int64_t)r0 * row_stride) = s0;
  }
}

template <typename OutT>
void launch_reduce(float* slab, int splits, int64_t n, OutT* out, int accum, hipStream_t s) {
  // enough threads to stream the slab: split the rows into groups when the output is small
  const int64_t cols4 = n / 4;
  const unsigned gx = (unsigned)((cols4 + 255) / 256);
  int groups = (int)std::min<int64_t>(splits, std::max<int64_t>(1, (256 * 256 * 2) / std::max<int64_t>(cols4, 1)));
  const int rpg = (splits + groups - 1) / groups;
  groups = (splits + rpg - 1) / rpg;
  if (groups > 1) {
    hipLaunchKernelGGL((wgrad_reduce_kernel<OutT, false>), dim3(gx, groups), dim3(256), 0, s, slab, splits, n, rpg, n,
                       out, accum);
    hipLaunchKernelGGL((wgrad_reduce_kernel<OutT, true>), dim3(gx, 1), dim3(256), 0, s, slab, groups,
                       (int64_t)rpg * n, groups, n, out, accum);
  } else {
    hipLaunchKernelGGL((wgrad_reduce_kernel<OutT, true>), dim3(gx, 1), dim3(256), 0, s, slab, splits, n, splits, n,
                       out, accum);
  }
}

struct WgradPlan {
  int wm, wn, fm, splits, plen;
};

WgradPlan plan_wgrad(int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, int dh = 1,
                     int dw = 1) {
  WgradPlan pl;
  const int Ho = (H + 2 * ph - dh * (R - 1) - 1) / sh + 1, Wo = (W + 2 * pw - dw * (S - 1) - 1) / sw + 1;
  const int RSC = R * S * C;
  const int64_t P = (int64_t)N * Ho * Wo;
  pl.fm = 4;
  // (FM = 8, a 256x128 block tile, needs 96 KB of LDS -> one block per CU; measured slower than
  // two 128x128 blocks per CU on every ResNet-50 shape, so it is not selected)
  if (RSC % 128 == 0 && K % 128 == 0) { pl.wm = 2; pl.wn = 2; }
  else if (RSC % 192 == 0) { pl.wm = 3; pl.wn = 1; }
  else if (RSC % 128 == 0) { pl.wm = 2; pl.wn = 1; }
  else if (K % 128 == 0) { pl.wm = 1; pl.wn = 2; }
  else { pl.wm = 1; pl.wn = 1; }
  const int64_t tiles = (int64_t)(RSC / (16 * pl.fm * pl.wm)) * (K / (64 * pl.wn));
  const int waves = pl.wm * pl.wn;
  int64_t splits = 4096 / (tiles * waves);
  const int64_t max_by_len = P / 512;                                   // >= 512 pixels per split
  const int64_t max_by_mem = (int64_t)(24 << 20) / ((int64_t)K * RSC);  // slab <= 96 MB
  splits = std::min(splits, std::min(max_by_len, max_by_mem));
  if (splits < 1) splits = 1;
  int64_t plen = (P + splits - 1) / splits;
  plen = (plen + 63) / 64 * 64;
  pl.plen = (int)plen;
  pl.splits = (int)((P + plen - 1) / plen);
  return pl;
}

template <typename T, int WM, int WN, int FM>
void launch_wgrad(const void* x, const void* dy, float* slab, const WgradGeom& g, int splits, bool ident,
                  const void* zero, hipStream_t s) {
  dim3 grid(g.tiles * splits);
  if (zero && FM == 4) {
    if (ident)
      hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, WM, WN, true>), grid, dim3(64 * WM * WN), 0, s,
                         static_cast<const T*>(x), static_cast<const T*>(dy), slab, static_cast<const T*>(zero), g);
    else
      hipLaunchKernelGGL((conv_wgrad_glds_kernel<T, WM, WN, false>), grid, dim3(64 * WM * WN), 0, s,
                         static_cast<const T*>(x), static_cast<const T*>(dy), slab, static_cast<const T*>(zero), g);
    return;
  }
  if (ident)
    hipLaunchKernelGGL((conv_wgrad_kernel<T, WM, WN, FM, true>), grid, dim3(64 * WM * WN), 0, s,
                       static_cast<const T*>(x), static_cast<const T*>(dy), slab, g);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<T, WM, WN, FM, false>), grid, dim3(64 * WM * WN), 0, s,
                       static_cast<const T*>(x), static_cast<const T*>(dy), slab, g);
}

template <typename T>
void dispatch_wgrad(const void* x, const void* dy, float* slab, const WgradGeom& g, const WgradPlan& pl, bool ident,
                    const void* zero, hipStream_t s) {
  if (pl.wm == 2 && pl.wn == 2 && pl.fm == 8) launch_wgrad<T, 2, 2, 8>(x, dy, slab, g, pl.splits, ident, zero, s);
  else if (pl.wm == 2 && pl.wn == 2) launch_wgrad<T, 2, 2, 4>(x, dy, slab, g, pl.splits, ident, zero, s);
  else if (pl.wm == 3) launch_wgrad<T, 3, 1, 4>(x, dy, slab, g, pl.splits, ident, zero, s);
  else if (pl.wm == 2) launch_wgrad<T, 2, 1, 4>(x, dy, slab, g, pl.splits, ident, zero, s);
  else if (pl.wn == 2) launch_wgrad<T, 1, 2, 4>(x, dy, slab, g, pl.splits, ident, zero, s);
  else launch_wgrad<T, 1, 1, 4>(x, dy, slab, g, pl.splits, ident, zero, s);
}

// ring variants: 1: 256x128 (4x2 waves, 3 stages)  2: 128x256 (2x4, 3)  3: 192x64 (3x1, 4)
//                4: 256x64 (4x1, 4)  5: 128x128 (2x2, 4)  6: 256x256 (2x4 waves of 128x64, 2)
//                7: 512x128 (4x2 waves of 128x64, 2)  8: 576x64 (9x1, 2: a whole 3x3x64 weight)
//                9: 64x256 (1x4, 4)      (rsc x k)
struct RingW {
  int wm, wn, nst, fm;
};
static bool ring_wgrad_cfg(int variant, RingW* c) {
  switch (variant) {
    case 1: *c = {4, 2, 3, 4}; return true;
    case 2: *c = {2, 4, 3, 4}; return true;
    case 3: *c = {3, 1, 4, 4}; return true;
    case 4: *c = {4, 1, 4, 4}; return true;
    case 5: *c = {2, 2, 4, 4}; return true;
    case 6: *c = {2, 4, 2, 8}; return true;
    case 7: *c = {4, 2, 2, 8}; return true;
    case 8: *c = {9, 1, 2, 4}; return true;
    case 9: *c = {1, 4, 4, 4}; return true;
    default: return false;
  }
}

static WgradPlan plan_wgrad_ring(const RingW& c, int N, int H, int W, int C, int K, int R, int S, int sh, int sw,
                                 int ph, int pw, int dh = 1, int dw = 1) {
  WgradPlan pl;
  const int Ho = (H + 2 * ph - dh * (R - 1) - 1) / sh + 1, Wo = (W + 2 * pw - dw * (S - 1) - 1) / sw + 1;
  const int RSC = R * S * C;
  const int64_t P = (int64_t)N * Ho * Wo;
  pl.fm = 4;
  pl.wm = c.wm;
  pl.wn = c.wn;
  const int64_t tiles = (int64_t)(RSC / (16 * c.fm * c.wm)) * (K / (64 * c.wn));
  // about one workgroup per CU (the LDS ring fills the CU): whole waves of workgroups, no tail
  int64_t splits = std::max<int64_t>(1, 256 / tiles);
  splits = std::min<int64_t>(splits, std::max<int64_t>(1, P / 256));
  int64_t plen = (P + splits - 1) / splits;
  plen = (plen + 63) / 64 * 64;
  pl.plen = (int)plen;
  pl.splits = (int)((P + plen - 1) / plen);
  return pl;
}

template <typename T, int WM, int WN, int NST, int FM = 4>
static void launch_wgrad_ring(const void* x, const void* dy, float* slab, const WgradGeom& g, int splits, bool ident,
                              const void* zero, hipStream_t s) {
  constexpr int SMEM = NST * (WM * FM / 4 + WN) * 64 * 64 * (int)sizeof(T);
  static_assert(SMEM <= 160 * 1024, "wgrad ring LDS budget");
  static bool attr[2] = {false, false};
  const void* fn = ident ? reinterpret_cast<const void*>(&conv_wgrad_ring_kernel<T, WM, WN, NST, FM, true>)
                         : reinterpret_cast<const void*>(&conv_wgrad_ring_kernel<T, WM, WN, NST, FM, false>);
  if (!attr[ident]) {
    hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr[ident] = true;
  }
  dim3 grid(g.tiles * splits);
  if (ident)
    hipLaunchKernelGGL((conv_wgrad_ring_kernel<T, WM, WN, NST, FM, true>), grid, dim3(64 * WM * WN), SMEM, s,
                       static_cast<const T*>(x), static_cast<const T*>(dy), slab, static_cast<const T*>(zero), g);
  else
    hipLaunchKernelGGL((conv_wgrad_ring_kernel<T, WM, WN, NST, FM, false>), grid, dim3(64 * WM * WN), SMEM, s,
                       static_cast<const T*>(x), static_cast<const T*>(dy), slab, static_cast<const T*>(zero), g);
}

template <typename T>
static void dispatch_wgrad_ring(int variant, const void* x, const void* dy, float* slab, const WgradGeom& g,
                                int splits, bool ident, const void* zero, hipStream_t s) {
  switch (variant) {
    case 1: launch_wgrad_ring<T, 4, 2, 3>(x, dy, slab, g, splits, ident, zero, s); break;
    case 2: launch_wgrad_ring<T, 2, 4, 3>(x, dy, slab, g, splits, ident, zero, s); break;
    case 3: launch_wgrad_ring<T, 3, 1, 4>(x, dy, slab, g, splits, ident, zero, s); break;
    case 4: launch_wgrad_ring<T, 4, 1, 4>(x, dy, slab, g, splits, ident, zero, s); break;
    case 5: launch_wgrad_ring<T, 2, 2, 4>(x, dy, slab, g, splits, ident, zero, s); break;
    case 6: launch_wgrad_ring<T, 2, 4, 2, 8>(x, dy, slab, g, splits, ident, zero, s); break;
    case 7: launch_wgrad_ring<T, 4, 2, 2, 8>(x, dy, slab, g, splits, ident, zero, s); break;
    case 8: launch_wgrad_ring<T, 9, 1, 2, 4>(x, dy, slab, g, splits, ident, zero, s); break;
    case 9: launch_wgrad_ring<T, 1, 4, 4, 4>(x, dy, slab, g, splits, ident, zero, s); break;
  }
}

}  // namespace

// True when ring variant `variant` (1..5) tiles this weight (R*S*C x K) exactly.
int conv_nhwc_wgrad_ring_ok(int C, int K, int R, int S, int variant) {
  RingW c;
  if (!ring_wgrad_cfg(variant, &c)) return 0;
  return (C % 64 == 0 && K % (64 * c.wn) == 0 && (R * S * C) % (16 * c.fm * c.wm) == 0) ? 1 : 0;
}

int64_t conv_nhwc_wgrad_ring_workspace(int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw,
                                       int variant, int dh, int dw) {
  RingW c;
  MXAMD_HOST_CHECK(ring_wgrad_cfg(variant, &c), "conv_nhwc_wgrad_ring: unknown variant");
  WgradPlan pl = plan_wgrad_ring(c, N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw);
  return (int64_t)pl.splits * K * R * S * C;
}

void conv_nhwc_wgrad_ring(int dtype, const void* x, const void* dy, float* slab, int out_dtype, void* out, int accum,
                          int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw,
                          const void* zero, int variant, hipStream_t s, int dh, int dw) {
  RingW c;
  MXAMD_HOST_CHECK(ring_wgrad_cfg(variant, &c) && conv_nhwc_wgrad_ring_ok(C, K, R, S, variant) && zero != nullptr,
                   "conv_nhwc_wgrad_ring: variant does not tile this weight");
  MXAMD_HOST_CHECK(dh >= 1 && dw >= 1, "conv_nhwc_wgrad_ring: dilation must be >= 1");
  WgradGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw;
  g.dh = dh; g.dw = dw;
  g.Ho = (H + 2 * ph - dh * (R - 1) - 1) / sh + 1;
  g.Wo = (W + 2 * pw - dw * (S - 1) - 1) / sw + 1;
  const int64_t P = (int64_t)N * g.Ho * g.Wo;
  MXAMD_HOST_CHECK(P < (1ll << 31) && (int64_t)N * H * W * C < (1ll << 31) && P * K < (1ll << 31),
                   "conv_nhwc_wgrad_ring: tensor too large for 32-bit indexing");
  g.P = (int)P;
  g.RSC = R * S * C;
  WgradPlan pl = plan_wgrad_ring(c, N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw);
  g.tiles_m = g.RSC / (16 * c.fm * c.wm);
  g.tiles = g.tiles_m * (K / (64 * c.wn));
  g.plen = pl.plen;
  g.fWo = make_fastdiv(g.Wo);
  g.fHoWo = make_fastdiv(g.Ho * g.Wo);
  const bool ident = R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0 && dh == 1 && dw == 1;
  if (dtype == kF16) dispatch_wgrad_ring<__half>(variant, x, dy, slab, g, pl.splits, ident, zero, s);
  else if (dtype == kBF16) dispatch_wgrad_ring<__hip_bfloat16>(variant, x, dy, slab, g, pl.splits, ident, zero, s);
  else throw std::runtime_error("conv_nhwc_wgrad_ring: dtype must be f16 or bf16");
  const int64_t n = (int64_t)K * g.RSC;
  if (out_dtype == kF32) launch_reduce<float>(slab, pl.splits, n, static_cast<float*>(out), accum, s);
  else if (out_dtype == kF16) launch_reduce<__half>(slab, pl.splits, n, static_cast<__half*>(out), accum, s);
  else launch_reduce<__hip_bfloat16>(slab, pl.splits, n, static_cast<__hip_bfloat16*>(out), accum, s);
}

// Number of fp32 slab elements conv_nhwc_wgrad needs (splits * K * R*S*C).
int64_t conv_nhwc_wgrad_workspace(int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw,
                                  int dh, int dw) {
  WgradPlan pl = plan_wgrad(N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw);
  return (int64_t)pl.splits * K * R * S * C;
}

// dW (OHWI, dtype out_dtype) = / += wgrad(x, dy).  slab: fp32 workspace of
// conv_nhwc_wgrad_workspace() elements.
// zero: optional >= 128-byte zero page; when given, the LDS-DMA kernel variant runs.
void conv_nhwc_wgrad(int dtype, const void* x, const void* dy, float* slab, int out_dtype, void* out, int accum, int N,
                     int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, const void* zero,
                     hipStream_t s, int dh, int dw) {
  MXAMD_HOST_CHECK(C % 64 == 0 && K % 64 == 0, "conv_nhwc_wgrad: need Cin % 64 == 0 and Cout % 64 == 0");
  MXAMD_HOST_CHECK(dh >= 1 && dw >= 1, "conv_nhwc_wgrad: dilation must be >= 1");
  WgradGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw;
  g.dh = dh; g.dw = dw;
  g.Ho = (H + 2 * ph - dh * (R - 1) - 1) / sh + 1;
  g.Wo = (W + 2 * pw - dw * (S - 1) - 1) / sw + 1;
  const int64_t P = (int64_t)N * g.Ho * g.Wo;
  MXAMD_HOST_CHECK(P < (1ll << 31) && (int64_t)N * H * W * C < (1ll << 31) && P * K < (1ll << 31),
                   "conv_nhwc_wgrad: tensor too large for 32-bit indexing");
  g.P = (int)P;
  g.RSC = R * S * C;
  WgradPlan pl = plan_wgrad(N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw);
  g.tiles_m = g.RSC / (16 * pl.fm * pl.wm);
  g.tiles = g.tiles_m * (K / (64 * pl.wn));
  g.plen = pl.plen;
  g.fWo = make_fastdiv(g.Wo);
  g.fHoWo = make_fastdiv(g.Ho * g.Wo);
  const bool ident = R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0 && dh == 1 && dw == 1;
  if (dtype == kF16) dispatch_wgrad<__half>(x, dy, slab, g, pl, ident, zero, s);
  else if (dtype == kBF16) dispatch_wgrad<__hip_bfloat16>(x, dy, slab, g, pl, ident, zero, s);
  else throw std::runtime_error("conv_nhwc_wgrad: dtype must be f16 or bf16");
  const int64_t n = (int64_t)K * g.RSC;
  if (out_dtype == kF32) launch_reduce<float>(slab, pl.splits, n, static_cast<float*>(out), accum, s);
  else if (out_dtype == kF16) launch_reduce<__half>(slab, pl.splits, n, static_cast<__half*>(out), accum, s);
  else launch_reduce<__hip_bfloat16>(slab, pl.splits, n, static_cast<__hip_bfloat16*>(out), accum, s);
}

// Column-sum of `splits` fp32 rows of length n (a split-K GEMM's partial products) into `out`
// (+= when accum): the split-K 1x1 wgrad candidate reduces straight into the .grad buffer.
void slab_reduce(int out_dtype, float* slab, int splits, int64_t n, void* out, int accum, hipStream_t s) {
  MXAMD_HOST_CHECK(n % 4 == 0 && (reinterpret_cast<uintptr_t>(slab) & 15) == 0 &&
                       (reinterpret_cast<uintptr_t>(out) & (out_dtype == kF32 ? 15 : 7)) == 0 && splits >= 1,
                   "slab_reduce: n % 4 == 0 and aligned slab/out required");
  if (out_dtype == kF32) launch_reduce<float>(slab, splits, n, static_cast<float*>(out), accum, s);
  else if (out_dtype == kF16) launch_reduce<__half>(slab, splits, n, static_cast<__half*>(out), accum, s);
  else launch_reduce<__hip_bfloat16>(slab, splits, n, static_cast<__hip_bfloat16*>(out), accum, s);
}

}  // namespace mxamd
