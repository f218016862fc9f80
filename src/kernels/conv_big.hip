// NHWC implicit-GEMM convolution with 512-thread, up to 256x256 output tiles
// and an LDS-staged epilogue (gfx950).
//
// Why another forward kernel: the 128x128 LDS-DMA kernel (conv_glds.hip)
// moves (128+128) x 128 B of operands through L2 per 2 MFLOP of K-tile, i.e.
// it needs ~34 TB/s of L2 bandwidth to keep the matrix cores busy -- the
// whole per-XCD L2 budget -- so it tops out near 700 TF/s.  A 256x256 tile
// halves operand traffic per FLOP.  Eight waves (2 per SIMD) each own a
// 64(co) x FJ*16(pix) sub-tile of v_mfma_f32_16x16x32 accumulators.
//
//   * operands: global -> LDS by global_load_lds_dwordx4 (LDS-DMA), 128-byte
//     rows (BK = 64 halves), XOR-swizzled 16-byte chunks (chunk ^ (row & 7)),
//     halo / out-of-range pixels fetched from a zero page, 2 stages;
//   * epilogue: the fp32 accumulators (+bias) are rounded and written to LDS as
//     a [pix][co] image (row pitch BCO*2+16 B: conflict-free ds_write_b64), then
//     re-read as 16-byte chunks and stored as whole contiguous pixel rows
//     (BCO*2 bytes per pixel), instead of 16 scattered 32-byte pieces per
//     store instruction;
//   * optional BatchNorm statistics: when `part` is given, each wave writes
//     per-channel partial sum(y) and sum(y^2) over its pixels (channel-major
//     [K][nparts]), which the BN finalize kernel consumes directly -- the
//     separate BN statistics pass over y (a full HBM read) disappears;
//   * optional addend (beta = 1): y = conv(x) + addend, read in the row-store
//     loop (used to fold a residual gradient into a 1x1 dgrad).
//
// Requirements (host-checked): Cin % 64 == 0, Cout % BCO == 0, dilation 1.
#include <stdexcept>
#include <type_traits>

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
struct MfmaB : mfma::Op<T> {};   // 16x16x32 MFMA + epilogue packs (mfma.h)

// Optional BatchNorm-backward statistics fused into the epilogue of a dgrad: y here is the gradient
// dy arriving at a BatchNorm(+ReLU) whose input was z; per (channel, pixel tile) the kernel emits
// sum(dz) and sum(dz * (z - mean)) with dz = dy * relu_mask (mode 2: mask = z*scale+shift > 0,
// mode 3: the forward's 1-bit mask, mode 0: no ReLU), channel-major [2][K][nparts] like the forward
// statistics -- the BatchNorm backward then skips its reduction pass over (dy, z).
struct BnBwdFuse {
  const void* z;
  const float* mean;
  const float* scale;
  const float* shift;
  const uint8_t* mask;
  int mode;
  float* part;
  int nparts;
};

struct GeomB {
  int N, H, W, C, K, R, S;
  int Ho, Wo;
  int sh, sw, ph, pw;
  int M;     // N*Ho*Wo
  int Ktot;  // R*S*C
  // up = 2: y is the 2x-upsampled, zero-filled image [N][2Ho][2Wo][K]: output pixel (n, ho, wo) lands at
  // (n, 2ho, 2wo) and the epilogue writes zeros to its three other 2x2 siblings -- the data gradient of a
  // 1x1 stride-2 convolution in one pass over dX (no memset, no scatter)
  int up;
  int dh, dw;  // dilation: tap (r, s) reads input row ho*sh - ph + r*dh, column wo*sw - pw + s*dw
};

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_base, 16, 0, 0);
}

// sum over the 16 lanes of a row group (lanes sharing lane >> 4)
__device__ __forceinline__ float row16_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

template <int BCO, int BPIX>
struct BigCfg {
  static constexpr int STAGE = (BCO + BPIX) * 128;
  static constexpr int PITCH = BCO * 2 + 16;
  static constexpr int EPI = BPIX * PITCH;
  static constexpr int SMEM = (2 * STAGE > EPI ? 2 * STAGE : EPI);
};

// BCO = WCO * 64 output channels, BPIX = (8 / WCO) * FJ * 16 pixels per block.
// MINB = workgroups per CU the register budget is sized for: MINB 2 caps a wave at 128 VGPRs
// (4 waves per SIMD) and halves the epilogue's register ring -- the variant for single-K-tile
// (reduction 64) convs, whose time is the epilogue's HBM traffic, not MFMA.
// MF = MFMA shape: 16 -> v_mfma_f32_16x16x32 (4 x FJ accumulators of 16x16 per wave), 32 ->
// v_mfma_f32_32x32x16 (2 x FJ/2 accumulators of 32x32; the LDS image then uses the (row >> 1) & 7
// chunk swizzle, which keeps both the 32-row and the 16-row fragment reads conflict-free).
template <typename T, int WCO, int FJ, int MINB, int MF>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2 * MINB))) conv_fwd_big_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                           const float* __restrict__ bias, T* __restrict__ y,
                                                           const T* __restrict__ zero, GeomB g, int tiles_co,
                                                           float* __restrict__ part, int nparts,
                                                           const T* __restrict__ addend, BnBwdFuse bf) {
  constexpr int WPIX = 8 / WCO;
  constexpr int BCO = WCO * 64;
  constexpr int BPIX = WPIX * FJ * 16;
  constexpr int BK = 64;
  constexpr int A_BYTES = BCO * 128;
  constexpr int STAGE = BigCfg<BCO, BPIX>::STAGE;
  constexpr int PITCH = BigCfg<BCO, BPIX>::PITCH;
  constexpr int A_INS = BCO / 64;  // wave-instructions (8 rows each) per wave for A
  // 8 waves x 8 rows per LDS-DMA round; a 224-pixel tile (FJ = 7) takes a half round at the end
  constexpr int B_INS = (BPIX + 63) / 64;
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;

  // XCD-aware bijective remap: consecutive tiles (same pixel tile, neighbouring co tiles) share an XCD's L2
  const int nblk = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q = nblk >> 3, rr = nblk & 7;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
  const int tco = wgid % tiles_co;
  const int tpix = wgid / tiles_co;
  const int co0 = tco * BCO;
  const int pix0 = tpix * BPIX;

  static_assert(MF == 16 || (MF == 32 && FJ % 2 == 0), "conv_big: MFMA shape");
  const int lrow = lane >> 3;
  // this lane's LDS slot (row (i*8 + wid)*8 + lrow, chunk position lane & 7) holds source chunk
  // (lane & 7) ^ swizzle(row); the swizzle is the same for every i (rows 64 apart)
  const int gch = (lane & 7) ^ (MF == 32 ? (((wid & 1) << 2) | (lrow >> 1)) : lrow);

  int a_off[A_INS];
#pragma unroll
  for (int i = 0; i < A_INS; ++i) a_off[i] = (co0 + (i * 8 + wid) * 8 + lrow) * g.Ktot + gch * 8;
  int b_base[B_INS], b_hi[B_INS], b_wi[B_INS];
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
  const T* zsrc = zero + gch * 8;

  const int KT = g.Ktot / BK;
  auto issue = [&](int kt, int stage) {
    const int k0 = kt * BK;
    const int rs = k0 / g.C;
    const int c0 = k0 - rs * g.C;
    const int r = rs / g.S;
    const int s = rs - r * g.S;
    char* sbase = smem + stage * STAGE;
#pragma unroll
    for (int i = 0; i < A_INS; ++i) glds16(w + a_off[i] + k0, sbase + (i * 8 + wid) * 1024);
    const int doff = (r * g.dh * g.W + s * g.dw) * g.C + c0;
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      if (BPIX % 64 != 0 && (i * 8 + wid) * 8 >= BPIX) continue;   // wave-uniform: past the tile
      const int hi = b_hi[i] + r * g.dh, wi = b_wi[i] + s * g.dw;
      const bool ok = (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
      const T* src = ok ? x + b_base[i] + doff : zsrc;
      glds16(src, sbase + A_BYTES + (i * 8 + wid) * 1024);
    }
  };

  constexpr int NI = MF == 32 ? 2 : 4;        // co fragments per wave (64 channels)
  constexpr int NJ = MF == 32 ? FJ / 2 : FJ;   // pixel fragments per wave
  typedef typename std::conditional<MF == 32, mfma::f16x, f4_t>::type acc_t;
  acc_t acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = acc_t{};

  const int wco = wid % WCO;
  const int wpix = wid / WCO;
  const int frag_r = lane & 15;
  const int fchunk = lane >> 4;
  const int a_row0 = (wco * 64 + (MF == 32 ? (lane & 31) : frag_r)) * 128;
  const int b_row0 = A_BYTES + (wpix * FJ * 16 + (MF == 32 ? (lane & 31) : frag_r)) * 128;
  // fragment rows differ from a_row0 / b_row0 by multiples of 16, so the swizzle is per lane
  const int sw = MF == 32 ? ((lane & 31) >> 1) & 7 : frag_r & 7;

  issue(0, 0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int stage = kt & 1;
    if (kt + 1 < KT) issue(kt + 1, stage ^ 1);
    const char* sb = smem + stage * STAGE;
    if constexpr (MF == 32) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int ch = ((kk * 2 + (lane >> 5)) ^ sw) * 16;
        u32x4 af[NI], bf[NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i) af[i] = *reinterpret_cast<const u32x4*>(sb + a_row0 + i * 32 * 128 + ch);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bf[j] = *reinterpret_cast<const u32x4*>(sb + b_row0 + j * 32 * 128 + ch);
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = MfmaB<T>::run32(af[i], bf[j], acc[i][j]);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = ((kk * 4 + fchunk) ^ sw) * 16;
        u32x4 af[NI], bf[NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i) af[i] = *reinterpret_cast<const u32x4*>(sb + a_row0 + i * 16 * 128 + ch);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bf[j] = *reinterpret_cast<const u32x4*>(sb + b_row0 + j * 16 * 128 + ch);
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = MfmaB<T>::run(af[i], bf[j], acc[i][j]);
      }
    }
    __syncthreads();
  }

  // ---- epilogue, stage 1: accumulators (+bias) -> LDS [pix][co] image (+ per-wave BN partials).
  // Every lane owns groups of 4 consecutive channels of one pixel; emit(cl, pl, v) takes one group.
  const int pw0 = wpix * FJ * 16;
  auto bias4 = [&](int cl, float* b) {
#pragma unroll
    for (int t = 0; t < 4; ++t) b[t] = bias ? bias[co0 + cl + t] : 0.f;
  };
  auto write_part = [&](int cl, const float* s, const float* q) {
    const int pid = tpix * WPIX + wpix;
    const int64_t c = co0 + cl;
    float* p1 = part;
    float* p2 = part + static_cast<int64_t>(g.K) * nparts;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      p1[(c + t) * nparts + pid] = s[t];
      p2[(c + t) * nparts + pid] = q[t];
    }
  };
  if constexpr (MF == 32) {
    // lane holds channels wco*64 + i*32 + 8*gq + 4*(lane>>5) + {0..3} (regs 4gq..4gq+3) of pixel
    // pw0 + j*32 + (lane & 31)
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int cl = wco * 64 + i * 32 + gq * 8 + (lane >> 5) * 4;
        float b[4], s4[4] = {0.f, 0.f, 0.f, 0.f}, q4[4] = {0.f, 0.f, 0.f, 0.f};
        bias4(cl, b);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int pl = pw0 + j * 32 + (lane & 31);
          float v[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] = acc[i][j][gq * 4 + t] + b[t];
          *reinterpret_cast<uint2*>(smem + pl * PITCH + cl * 2) = MfmaB<T>::pack4(v[0], v[1], v[2], v[3]);
          if (part != nullptr && pix0 + pl < g.M) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              s4[t] += v[t];
              q4[t] += v[t] * v[t];
            }
          }
        }
        if (part != nullptr) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            s4[t] = row16_sum(s4[t]);
            s4[t] += __shfl_xor(s4[t], 16, 64);
            q4[t] = row16_sum(q4[t]);
            q4[t] += __shfl_xor(q4[t], 16, 64);
          }
          if ((lane & 31) == 0) write_part(cl, s4, q4);
        }
      }
    }
  } else {
    // lane holds co = wco*64 + i*16 + 4*(lane>>4) + {0..3} for pixel pw0 + j*16 + (lane&15)
    const int co_l = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int cl = wco * 64 + i * 16 + co_l;  // channel within the block tile
      float b[4], s4[4] = {0.f, 0.f, 0.f, 0.f}, q4[4] = {0.f, 0.f, 0.f, 0.f};
      bias4(cl, b);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int pl = pw0 + j * 16 + frag_r;
        float v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = acc[i][j][t] + b[t];
        *reinterpret_cast<uint2*>(smem + pl * PITCH + cl * 2) = MfmaB<T>::pack4(v[0], v[1], v[2], v[3]);
        if (part != nullptr && pix0 + pl < g.M) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            s4[t] += v[t];
            q4[t] += v[t] * v[t];
          }
        }
      }
      if (part != nullptr) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          s4[t] = row16_sum(s4[t]);
          q4[t] = row16_sum(q4[t]);
        }
        if (frag_r == 0) write_part(cl, s4, q4);
      }
    }
  }
  __syncthreads();
  // whole pixel rows: BCO*2 bytes = BCO/8 16-byte chunks per pixel
  constexpr int CPR = BCO / 8;
  constexpr int TOTAL = BPIX * CPR;
  constexpr int ITERS = TOTAL / 512;
  static_assert(512 % CPR == 0 && TOTAL % 512 == 0, "each thread keeps one 8-channel group");
  const bool bnb = bf.part != nullptr;
  // BN-backward statistics: this thread's channel group is fixed (tid % CPR)
  float s1[8], s2[8], bm[8], bsc[8], bsh[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    s1[t] = 0.f;
    s2[t] = 0.f;
  }
  if (bnb) {
    const int cb = co0 + (tid % CPR) * 8;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      bm[t] = bf.mean[cb + t];
      bsc[t] = bf.mode == 2 ? bf.scale[cb + t] : 0.f;
      bsh[t] = bf.mode == 2 ? bf.shift[cb + t] : 0.f;
    }
  }
  // The addend / BN input z rows this thread reads are streamed through a register ring D
  // iterations deep: all loads of the first D rows are in flight before the first store, and row
  // e + D is requested as row e retires -- instead of one latency-bound load per row.
  constexpr int DMAX = MINB > 1 ? 4 : 8;
  constexpr int D = ITERS < DMAX ? ITERS : DMAX;
  const T* zsrc_b = static_cast<const T*>(bf.z);
  uint4 ad_ring[D], z_ring[D];
  auto out_pix = [&](int p) -> int64_t {
    if (g.up != 2) return p;
    const int n = p / (g.Ho * g.Wo);
    const int rem = p - n * g.Ho * g.Wo;
    const int ho = rem / g.Wo;
    const int wo = rem - ho * g.Wo;
    return ((int64_t)n * 2 * g.Ho + 2 * ho) * (2 * g.Wo) + 2 * wo;
  };
  auto row_off = [&](int it, int64_t* off) -> bool {
    const int e = tid + it * 512;
    const int pl = e / CPR;
    const int c8 = e - pl * CPR;
    const int p = pix0 + pl;
    *off = out_pix(p < g.M ? p : 0) * g.K + co0 + c8 * 8;
    return p < g.M;
  };
#pragma unroll
  for (int it = 0; it < D; ++it) {
    int64_t off;
    const bool ok = row_off(it, &off);
    if (addend != nullptr && ok) ad_ring[it] = *reinterpret_cast<const uint4*>(addend + off);
    if (bnb && ok) z_ring[it] = *reinterpret_cast<const uint4*>(zsrc_b + off);
  }
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int e = tid + it * 512;
    const int pl = e / CPR;
    const int c8 = e - pl * CPR;
    const int p = pix0 + pl;
    int64_t off;
    const bool ok = row_off(it, &off);
    uint4 ad_cur = ad_ring[it % D], z_cur = z_ring[it % D];
    if (it + D < ITERS) {
      int64_t off2;
      const bool ok2 = row_off(it + D, &off2);
      if (addend != nullptr && ok2) ad_ring[it % D] = *reinterpret_cast<const uint4*>(addend + off2);
      if (bnb && ok2) z_ring[it % D] = *reinterpret_cast<const uint4*>(zsrc_b + off2);
    }
    if (ok) {
      Vec8<T> v;
      v.raw = *reinterpret_cast<const uint4*>(smem + pl * PITCH + c8 * 16);
      if (addend != nullptr) {
        // y = conv + addend (beta = 1): e.g. the identity shortcut's gradient folded into a 1x1 dgrad
        Vec8<T> a;
        a.raw = ad_cur;
#pragma unroll
        for (int t = 0; t < 8; ++t) v.set(t, v.get(t) + a.get(t));
      }
      v.store(y + off);
      if (g.up == 2) {
        // the three zero siblings of this pixel in its 2x2 block of the upsampled image
        const uint4 z4 = {0u, 0u, 0u, 0u};
        const int64_t rowp = (int64_t)2 * g.Wo * g.K;
        *reinterpret_cast<uint4*>(y + off + g.K) = z4;
        *reinterpret_cast<uint4*>(y + off + rowp) = z4;
        *reinterpret_cast<uint4*>(y + off + rowp + g.K) = z4;
      }
      if (bnb) {
        Vec8<T> zv;
        zv.raw = z_cur;
        const uint32_t mb = bf.mode == 3 ? bf.mask[off >> 3] : 0xffu;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const float zt = zv.get(t);
          bool keep = true;
          if (bf.mode == 2) keep = fmaf(zt, bsc[t], bsh[t]) > 0.f;
          if (bf.mode == 3) keep = (mb >> t) & 1u;
          const float dz = keep ? v.get(t) : 0.f;
          s1[t] += dz;
          s2[t] += dz * (zt - bm[t]);
        }
      }
    }
    (void)p;
  }
  if (bnb) {
    // combine the 512/CPR threads of each channel group through LDS, one partial per pixel tile
    constexpr int ROWS = 512 / CPR;
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      red[(tid / CPR) * BCO + (tid % CPR) * 8 + t] = s1[t];
      red[ROWS * BCO + (tid / CPR) * BCO + (tid % CPR) * 8 + t] = s2[t];
    }
    __syncthreads();
    for (int q = tid; q < 2 * BCO; q += 512) {
      const int which = q / BCO, ch = q - which * BCO;
      const float* col = red + which * ROWS * BCO + ch;
      float acc_s = 0.f;
#pragma unroll 8
      for (int r = 0; r < ROWS; ++r) acc_s += col[r * BCO];
      bf.part[(int64_t)which * g.K * bf.nparts + (int64_t)(co0 + ch) * bf.nparts + tpix] = acc_s;
    }
  }
}

template <typename T, int WCO, int FJ, int MINB, int MF = 16>
void launch_big(const void* x, const void* w, const float* bias, void* y, const void* zero, const GeomB& g,
                float* part, int nparts, const void* addend, const BnBwdFuse& bf, hipStream_t s) {
  constexpr int BCO = WCO * 64;
  constexpr int BPIX = (8 / WCO) * FJ * 16;
  constexpr int SMEM = BigCfg<BCO, BPIX>::SMEM;
  static_assert(SMEM <= 160 * 1024, "conv_big: LDS budget");
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_fwd_big_kernel<T, WCO, FJ, MINB, MF>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  const int tiles_co = g.K / BCO;
  const int tiles_pix = (g.M + BPIX - 1) / BPIX;
  // a single K-tile (reduction 64: skinny 1x1 convs, the tee dgrads of the bottleneck's first conv)
  // never touches the second operand stage: launching with only stage 0 + the epilogue image lets
  // two workgroups share a CU for the 128x256 / 256x128 / 64x512 tiles (with the MINB = 2 register
  // budget), so one block's epilogue streams overlap another block's operand loads
  constexpr int ONE_STAGE = BigCfg<BCO, BPIX>::STAGE > BigCfg<BCO, BPIX>::EPI ? BigCfg<BCO, BPIX>::STAGE
                                                                               : BigCfg<BCO, BPIX>::EPI;
  const int smem = g.Ktot / 64 > 1 ? SMEM : ONE_STAGE;
  hipLaunchKernelGGL((conv_fwd_big_kernel<T, WCO, FJ, MINB, MF>), dim3(tiles_co * tiles_pix), dim3(512), smem, s,
                     static_cast<const T*>(x), static_cast<const T*>(w), bias, static_cast<T*>(y),
                     static_cast<const T*>(zero), g, tiles_co, part, nparts, static_cast<const T*>(addend), bf);
}

// variant -> (WCO, FJ): tile BCO x BPIX
//   0: 256 x 256   1: 128 x 256   2: 64 x 512   3: 256 x 128
//   4: 128 x 256   5: 256 x 128 at two workgroups per CU (122 VGPRs; for reduction-64 convs --
//      the 64 x 512 tile does not fit 128 VGPRs without spilling)
//   6..9: the 0..3 tiles on v_mfma_f32_32x32x16
//   16: 256 x 224   17: 128 x 448 (FJ = 7): M = N*H*W of ResNet's 14x14 / 28x28 layers is 196 * 2^k, so
//       256-pixel tiles leave a quarter of the CUs idle in the last round; 224-pixel tiles fill 7/8
static void big_tile(int variant, int* bco, int* bpix) {
  if (variant == 16) { *bco = 256; *bpix = 224; return; }
  if (variant == 17) { *bco = 128; *bpix = 448; return; }
  if (variant == 4) variant = 1;
  if (variant == 5) variant = 3;
  if (variant >= 6 && variant <= 9) variant -= 6;
  switch (variant) {
    case 0: *bco = 256; *bpix = 256; break;
    case 1: *bco = 128; *bpix = 256; break;
    case 2: *bco = 64; *bpix = 512; break;
    case 3: *bco = 256; *bpix = 128; break;
    default: throw std::runtime_error("conv_nhwc_fwd_big: unknown variant");
  }
}

template <typename T>
void dispatch_big(int variant, const void* x, const void* w, const float* bias, void* y, const void* zero,
                  const GeomB& g, float* part, int nparts, const void* addend, const BnBwdFuse& bf, hipStream_t s) {
  switch (variant) {
    case 0: launch_big<T, 4, 8, 1>(x, w, bias, y, zero, g, part, nparts, addend, bf, s); break;
    case 1: launch_big<T, 2, 4, 1>(x, w, bias, y, zero, g, part, nparts, addend, bf, s); break;
    case 2: launch_big<T, 1, 4, 1>(x, w, bias, y, zero, g, part, nparts, addend, bf, s); break;
    case 3: launch_big<T, 4, 4, 1>(x, w, bias, y, zero, g, part, nparts, addend, bf, s); break;
    case 4: launch_big<T, 2, 4, 2>(x, w, bias, y, zero, g, part, nparts, addend, bf, s); break;
    case 5: launch_big<T, 4, 4, 2>(x, w, bias, y, zero, g, part, nparts, addend, bf, s); break;
    case 6: launch_big<T, 4, 8, 1, 32>(x, w, bias, y, zero, g, part, nparts, addend, bf, s); break;
    case 7: launch_big<T, 2, 4, 1, 32>(x, w, bias, y, zero, g, part, nparts, addend, bf, s); break;
    case 8: launch_big<T, 1, 4, 1, 32>(x, w, bias, y, zero, g, part, nparts, addend, bf, s); break;
    case 9: launch_big<T, 4, 4, 1, 32>(x, w, bias, y, zero, g, part, nparts, addend, bf, s); break;
    case 16: launch_big<T, 4, 7, 1>(x, w, bias, y, zero, g, part, nparts, addend, bf, s); break;
    case 17: launch_big<T, 2, 7, 1>(x, w, bias, y, zero, g, part, nparts, addend, bf, s); break;
    default: throw std::runtime_error("conv_nhwc_fwd_big: unknown variant");
  }
}

}  // namespace

// Number of BN-statistics partials per channel the big kernel writes for this conv/variant.
int conv_nhwc_fwd_big_nparts(int N, int H, int W, int R, int S, int sh, int sw, int ph, int pw, int variant) {
  int bco, bpix;
  big_tile(variant, &bco, &bpix);
  const int Ho = (H + 2 * ph - R) / sh + 1;
  const int Wo = (W + 2 * pw - S) / sw + 1;
  const int M = N * Ho * Wo;
  return ((M + bpix - 1) / bpix) * (8 / (bco / 64));
}

// BN-backward partials per channel the big kernel's fused epilogue writes (one per pixel tile).
int conv_nhwc_fwd_big_bwd_nparts(int N, int H, int W, int R, int S, int sh, int sw, int ph, int pw, int variant) {
  int bco, bpix;
  big_tile(variant, &bco, &bpix);
  const int Ho = (H + 2 * ph - R) / sh + 1;
  const int Wo = (W + 2 * pw - S) / sw + 1;
  return (N * Ho * Wo + bpix - 1) / bpix;
}

void conv_nhwc_fwd_big(int dtype, const void* x, const void* w, const float* bias, void* y, const void* zero, int N,
                       int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, int variant,
                       float* part, int nparts, const void* addend, hipStream_t s, const void* bn_z,
                       const float* bn_mean, const float* bn_scale, const float* bn_shift, const uint8_t* bn_mask,
                       int bn_mode, float* bn_part, int bn_nparts, int up, int dh, int dw) {
  GeomB g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw;
  g.dh = dh; g.dw = dw;
  MXAMD_HOST_CHECK(dh >= 1 && dw >= 1, "conv_nhwc_fwd_big: dilation must be >= 1");
  MXAMD_HOST_CHECK((dh == 1 && dw == 1) || (part == nullptr && bn_part == nullptr && up == 0),
                   "conv_nhwc_fwd_big: dilated convolutions take no fused BN epilogue / upsampled output");
  g.Ho = (H + 2 * ph - dh * (R - 1) - 1) / sh + 1;
  g.Wo = (W + 2 * pw - dw * (S - 1) - 1) / sw + 1;
  MXAMD_HOST_CHECK(g.Ho > 0 && g.Wo > 0, "conv_nhwc_fwd_big: empty output");
  g.M = N * g.Ho * g.Wo;
  g.Ktot = R * S * C;
  g.up = up;
  int bco, bpix;
  big_tile(variant, &bco, &bpix);
  MXAMD_HOST_CHECK(C % 64 == 0 && K % bco == 0, "conv_nhwc_fwd_big: need Cin % 64 == 0 and Cout % BCO == 0");
  MXAMD_HOST_CHECK(up == 0 || (up == 2 && addend == nullptr && (int64_t)g.M * 4 * K < (1ll << 31)),
                   "conv_nhwc_fwd_big: the 2x upsampled output takes no addend and must fit 32-bit indexing");
  MXAMD_HOST_CHECK((int64_t)N * H * W * C < (1ll << 31) && (int64_t)g.M * K < (1ll << 31) &&
                       (int64_t)K * g.Ktot < (1ll << 31),
                   "conv_nhwc_fwd_big: tensor too large for 32-bit indexing");
  MXAMD_HOST_CHECK(part == nullptr || nparts == conv_nhwc_fwd_big_nparts(N, H, W, R, S, sh, sw, ph, pw, variant),
                   "conv_nhwc_fwd_big: wrong BN partials count");
  BnBwdFuse bf{bn_z, bn_mean, bn_scale, bn_shift, bn_mask, bn_mode, bn_part, bn_nparts};
  MXAMD_HOST_CHECK(bn_part == nullptr ||
                       (bn_z && bn_mean && bn_nparts == conv_nhwc_fwd_big_bwd_nparts(N, H, W, R, S, sh, sw, ph, pw,
                                                                                     variant) &&
                        (bn_mode != 2 || (bn_scale && bn_shift)) && (bn_mode != 3 || bn_mask)),
                   "conv_nhwc_fwd_big: bad BN-backward epilogue arguments");
  if (dtype == kF16) dispatch_big<__half>(variant, x, w, bias, y, zero, g, part, nparts, addend, bf, s);
  else if (dtype == kBF16) dispatch_big<__hip_bfloat16>(variant, x, w, bias, y, zero, g, part, nparts, addend, bf, s);
  else throw std::runtime_error("conv_nhwc_fwd_big: dtype must be f16 or bf16");
}

}  // namespace mxamd
