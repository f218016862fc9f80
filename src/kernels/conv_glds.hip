// NHWC implicit-GEMM convolution, LDS-DMA pipelined (gfx950).
//
// Same GEMM view as conv_igemm.hip (C'[co][pix] = W . Xpatch^T on
// v_mfma_f32_16x16x32, K = (r, s, c) so both operands are K-contiguous), but
// the operand tiles go global -> LDS directly with global_load_lds_dwordx4
// (the LDS-DMA path) instead of global -> VGPR -> ds_write_b128:
//
//   * no staging registers and no LDS-write instructions in the main loop; the
//     next K-tile's DMA is in flight while the current tile's MFMAs run;
//   * LDS rows are 128 B (BK = 64 halves) with NO padding: one wave-instruction
//     fills 8 rows (lane-linear 1 KB).  Bank conflicts of the ds_read_b128
//     fragment reads are removed by an XOR swizzle of the 16-byte chunk index
//     (chunk ^ (row & 7)), applied on the GLOBAL source address of each lane
//     (lane L of a wave-instruction fetches chunk (L & 7) ^ (L >> 3) of its row)
//     and on the LDS read address -- conflict-free for the 16-lane read groups;
//   * 3x3 halo / out-of-range pixels are DMA'd from a 128-byte zero page, so the
//     LDS image is always fully written (no branches, no EXEC-masked DMA);
//   * 2 LDS stages x 32 KB -> 2 blocks (8 waves) per CU; grid remapped XCD-aware.
//
// Requirements (host-checked): Cin % 64 == 0, Cout % BCO == 0, dilation 1.
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
struct Mfma : mfma::Op<T> {};   // 16x16x32 MFMA + epilogue packs (mfma.h)

struct GeomG {
  int N, H, W, C, K, R, S;
  int Ho, Wo;
  int sh, sw, ph, pw;
  int M;     // N*Ho*Wo
  int Ktot;  // R*S*C
  // output element offset of pixel p = q*Wo + wo (q = n*Ho + ho): q*og + wo*oc + ob (dense: Wo*K, K, 0);
  // a strided map lets a sub-pixel piece of a strided dgrad write its phase of dX in place
  int64_t og, oc, ob;
  // phases of a strided dgrad no tap reaches: this phase also writes zeros at off - ob + zob[i]
  int nz;
  int64_t zob[3];
};

// optional BatchNorm-backward statistics of the output (y is the gradient of a BN(+ReLU) output whose
// input is z; ReLU mask recomputed as z*scale + shift > 0, none when scale/shift are null): per-channel (sum dz, sum dz*(z - mean))
// partials, channel-major [2][K][nparts], one per (pixel tile, pixel wave) -- the BN's own reduction
// pass over (y, z) is then skipped
struct BnbG {
  const void* z;
  const float* mean;
  const float* scale;
  const float* shift;
  float* part;
  int nparts;
};

__device__ __forceinline__ float sum16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_base, 16, 0, 0);
}

template <typename T, int BCO>
__device__ __forceinline__ void glds_body(const T* __restrict__ x, const T* __restrict__ w,
                                          const float* __restrict__ bias, T* __restrict__ y,
                                          const T* __restrict__ zero, const GeomG& g, int tiles_co,
                                          const BnbG& bn, int part_base);

template <typename T, int BCO>
__global__ void __launch_bounds__(256) conv_fwd_glds_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                            const float* __restrict__ bias, T* __restrict__ y,
                                                            const T* __restrict__ zero, GeomG g, int tiles_co,
                                                            BnbG bn) {
  glds_body<T, BCO>(x, w, bias, y, zero, g, tiles_co, bn, 0);
}

// All sub-pixel phases of a strided data gradient in one launch: blockIdx.y picks the phase (its
// taps, padding, output offset and weight slice); phases share dY and the output dX.
constexpr int kMaxPhases = 4;
struct PhaseSet {
  GeomG g[kMaxPhases];
  int64_t w_off[kMaxPhases];   // element offset of the phase's weight slice
};

template <typename T, int BCO>
__global__ void __launch_bounds__(256) conv_phase_glds_kernel(const T* __restrict__ dy, const T* __restrict__ w,
                                                              T* __restrict__ dx, const T* __restrict__ zero,
                                                              PhaseSet ps, int tiles_co, BnbG bn) {
  const int ph = blockIdx.y;
  // each phase's (pixel tile, wave) partials get their own slots
  glds_body<T, BCO>(dy, w + ps.w_off[ph], nullptr, dx, zero, ps.g[ph], tiles_co, bn, ph * bn.nparts / gridDim.y);
}

template <typename T, int BCO>
__device__ __forceinline__ void glds_body(const T* __restrict__ x, const T* __restrict__ w,
                                          const float* __restrict__ bias, T* __restrict__ y,
                                          const T* __restrict__ zero, const GeomG& g, int tiles_co,
                                          const BnbG& bn, int part_base) {
  constexpr int WAVES_CO = BCO / 64;
  constexpr int WAVES_PIX = 4 / WAVES_CO;
  constexpr int BPIX = WAVES_PIX * 64;
  constexpr int BK = 64;
  constexpr int A_BYTES = BCO * 128;
  constexpr int STAGE = (BCO + BPIX) * 128;  // 32 KB
  constexpr int A_INS = BCO / 32;            // wave-instructions (8 rows each) per wave for A
  constexpr int B_INS = BPIX / 32;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

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

  // lane L of a wave-instruction writes LDS row (L >> 3), chunk (L & 7) and fetches global chunk
  // (L & 7) ^ (row & 7) of that row: the swizzled image read back below
  const int lrow = lane >> 3;
  const int gch = (lane & 7) ^ lrow;

  int a_off[A_INS];
#pragma unroll
  for (int i = 0; i < A_INS; ++i) a_off[i] = (co0 + (i * 4 + wid) * 8 + lrow) * g.Ktot + gch * 8;
  int b_base[B_INS], b_hi[B_INS], b_wi[B_INS];
#pragma unroll
  for (int i = 0; i < B_INS; ++i) {
    const int p = pix0 + (i * 4 + wid) * 8 + lrow;
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
    // k-tile kt -> (r, s, c0); C % 64 == 0 so a tile never straddles (r, s)
    const int k0 = kt * BK;
    const int rs = k0 / g.C;
    const int c0 = k0 - rs * g.C;
    const int r = rs / g.S;
    const int s = rs - r * g.S;
    char* sbase = smem + stage * STAGE;
#pragma unroll
    for (int i = 0; i < A_INS; ++i) glds16(w + a_off[i] + k0, sbase + (i * 4 + wid) * 1024);
    const int doff = (r * g.W + s) * g.C + c0;
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const int hi = b_hi[i] + r, wi = b_wi[i] + s;
      const bool ok = (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
      const T* src = ok ? x + b_base[i] + doff : zsrc;
      glds16(src, sbase + A_BYTES + (i * 4 + wid) * 1024);
    }
  };

  f4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4_t{0.f, 0.f, 0.f, 0.f};

  const int wco = wid % WAVES_CO;
  const int wpix = wid / WAVES_CO;
  const int frag_r = lane & 15;
  const int fchunk = lane >> 4;  // 0..3: k = 8*fchunk within a 32-wide k-step
  // byte offsets of this lane's fragment rows inside the A / B images (row & 7 == frag_r & 7 for all 16-row frags)
  const int a_row0 = (wco * 64 + frag_r) * 128;
  const int b_row0 = A_BYTES + (wpix * 64 + frag_r) * 128;
  const int sw = frag_r & 7;

  issue(0, 0);
  __syncthreads();  // s_waitcnt vmcnt(0) + barrier: tile 0 visible
  for (int kt = 0; kt < KT; ++kt) {
    const int stage = kt & 1;
    if (kt + 1 < KT) issue(kt + 1, stage ^ 1);
    const char* sb = smem + stage * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = ((kk * 4 + fchunk) ^ sw) * 16;
      u32x4 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const u32x4*>(sb + a_row0 + i * 16 * 128 + ch);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const u32x4*>(sb + b_row0 + j * 16 * 128 + ch);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = Mfma<T>::run(af[i], bf[j], acc[i][j]);
    }
    __syncthreads();  // next tile's DMA complete (vmcnt(0)) and this tile's reads done
  }

  // ---- epilogue: lane holds co = base + 4*(lane>>4) + {0..3} for pixel base + (lane&15)
  const int co_l = (lane >> 4) * 4;
  const bool bnb = bn.part != nullptr;
  const T* zb = static_cast<const T*>(bn.z);
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
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
    float bm[4], bsc[4], bsh[4];
    if (bnb) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        bm[t] = bn.mean[co + t];
        // no scale/shift: a BN without ReLU -- 0*z + 1 > 0 keeps every element
        bsc[t] = bn.scale ? bn.scale[co + t] : 0.f;
        bsh[t] = bn.shift ? bn.shift[co + t] : 1.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = pix0 + wpix * 64 + j * 16 + frag_r;
      if (p < g.M) {
        uint2 v = Mfma<T>::pack4(acc[i][j][0] + b0, acc[i][j][1] + b1, acc[i][j][2] + b2, acc[i][j][3] + b3);
        const int q = p / g.Wo;
        const int64_t off = q * g.og + (p - q * g.Wo) * g.oc + g.ob;
        *reinterpret_cast<uint2*>(y + off + co) = v;
        for (int z = 0; z < g.nz; ++z) *reinterpret_cast<uint2*>(y + off - g.ob + g.zob[z] + co) = uint2{0u, 0u};
        if (bnb) {
          // statistics of the stored (rounded) gradient, as the BN's own pass would read it
          const float4 dv = Mfma<T>::unpack4(v);
          const float4 zv = Mfma<T>::unpack4(*reinterpret_cast<const uint2*>(zb + off + co));
          const float d4[4] = {dv.x, dv.y, dv.z, dv.w}, z4[4] = {zv.x, zv.y, zv.z, zv.w};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const float dz = fmaf(z4[t], bsc[t], bsh[t]) > 0.f ? d4[t] : 0.f;
            s1[t] += dz;
            s2[t] += dz * (z4[t] - bm[t]);
          }
        }
      }
    }
    if (bnb) {
      // the 16 lanes of a channel group hold different pixels: sum them, one partial per wave
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s1[t] = sum16(s1[t]);
        s2[t] = sum16(s2[t]);
      }
      if (frag_r == 0) {
        const int pid = part_base + tpix * WAVES_PIX + wpix;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          bn.part[static_cast<int64_t>(co + t) * bn.nparts + pid] = s1[t];
          bn.part[(static_cast<int64_t>(g.K) + co + t) * bn.nparts + pid] = s2[t];
        }
      }
    }
  }
}

template <typename T, int BCO>
void launch_glds(const void* x, const void* w, const float* bias, void* y, const void* zero, const GeomG& g,
                 hipStream_t s, const BnbG& bn) {
  constexpr int BPIX = (4 / (BCO / 64)) * 64;
  const int tiles_co = g.K / BCO;
  const int tiles_pix = (g.M + BPIX - 1) / BPIX;
  hipLaunchKernelGGL((conv_fwd_glds_kernel<T, BCO>), dim3(tiles_co * tiles_pix), dim3(256), 0, s,
                     static_cast<const T*>(x), static_cast<const T*>(w), bias, static_cast<T*>(y),
                     static_cast<const T*>(zero), g, tiles_co, bn);
}

}  // namespace

// bco: 128 (128x128 tile) or 64 (64 co x 256 pix).  zero: >= 128 bytes of zeros (device).
// BN-backward partials per channel of a glds launch over M output pixels (pixel tiles x pixel waves).
int conv_glds_bwd_nparts(int M, int bco) {
  const int bpix = bco == 128 ? 128 : 256;
  const int waves_pix = bco == 128 ? 2 : 4;
  return ((M + bpix - 1) / bpix) * waves_pix;
}

void conv_nhwc_fwd_glds(int dtype, const void* x, const void* w, const float* bias, void* y, const void* zero, int N,
                        int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, int bco,
                        hipStream_t s, const void* bn_z, const float* bn_mean, const float* bn_scale,
                        const float* bn_shift, float* bn_part, int bn_nparts) {
  GeomG g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw;
  g.Ho = (H + 2 * ph - R) / sh + 1;
  g.Wo = (W + 2 * pw - S) / sw + 1;
  g.M = N * g.Ho * g.Wo;
  g.Ktot = R * S * C;
  g.og = (int64_t)g.Wo * K;
  g.oc = K;
  g.ob = 0;
  g.nz = 0;
  MXAMD_HOST_CHECK(C % 64 == 0 && K % bco == 0 && (bco == 64 || bco == 128),
                   "conv_nhwc_fwd_glds: need Cin % 64 == 0 and Cout % BCO == 0");
  MXAMD_HOST_CHECK((int64_t)N * H * W * C < (1ll << 31) && (int64_t)g.M * K < (1ll << 31) &&
                       (int64_t)K * g.Ktot < (1ll << 31),
                   "conv_nhwc_fwd_glds: tensor too large for 32-bit indexing");
  const BnbG bn{bn_z, bn_mean, bn_scale, bn_shift, bn_part, bn_nparts};
  MXAMD_HOST_CHECK(!bn_part || (bn_z && bn_mean && !bn_scale == !bn_shift && bn_nparts == conv_glds_bwd_nparts(g.M, bco)),
                   "conv_nhwc_fwd_glds: BN-backward statistics need z, mean, scale, shift and nparts");
  if (dtype == kF16) {
    if (bco == 128) launch_glds<__half, 128>(x, w, bias, y, zero, g, s, bn);
    else launch_glds<__half, 64>(x, w, bias, y, zero, g, s, bn);
  } else if (dtype == kBF16) {
    if (bco == 128) launch_glds<__hip_bfloat16, 128>(x, w, bias, y, zero, g, s, bn);
    else launch_glds<__hip_bfloat16, 64>(x, w, bias, y, zero, g, s, bn);
  } else {
    throw std::runtime_error("conv_nhwc_fwd_glds: dtype must be f16 or bf16");
  }
}

// The sub-pixel phases of a stride-s data gradient in one launch.  Phase i writes dX[n, s*a + ph_i,
// s*b + pw_i, :] for all (a, b) (an Ho x Wo grid, Hx = s*Ho, Wx = s*Wo) as a stride-1 conv of dY
// (N x Hi x Wi x Cin, Cin = the conv's output channels) with its taps: weight slice w + w_off[i]
// laid out [Cout][R_i][S_i][Cin], tap offsets -pad_h[i] / -pad_w[i] (possibly negative).
void conv_nhwc_dgrad_phases_glds(int dtype, const void* dy, const void* w, void* dx, const void* zero, int N, int Hi,
                                 int Wi, int Cin, int Cout, int Ho, int Wo, int stride, int nph, const int* ph,
                                 const int* pw, const int* R, const int* S, const int* pad_h, const int* pad_w,
                                 const int64_t* w_off, int nzero, const int* zph, const int* zpw, int bco,
                                 hipStream_t s, const void* bn_z, const float* bn_mean, const float* bn_scale,
                                 const float* bn_shift, float* bn_part, int bn_nparts) {
  MXAMD_HOST_CHECK(nph >= 1 && nph <= kMaxPhases, "conv_nhwc_dgrad_phases_glds: 1..4 phases");
  MXAMD_HOST_CHECK(nzero >= 0 && nzero <= 3, "conv_nhwc_dgrad_phases_glds: at most 3 zero phases");
  MXAMD_HOST_CHECK(Cin % 64 == 0 && Cout % bco == 0 && (bco == 64 || bco == 128) && stride >= 1 && Ho > 0 &&
                       Wo > 0,
                   "conv_nhwc_dgrad_phases_glds: need Cin % 64 == 0 and Cout % BCO == 0");
  MXAMD_HOST_CHECK((int64_t)N * Hi * Wi * Cin < (1ll << 31), "conv_nhwc_dgrad_phases_glds: dY too large");
  PhaseSet ps;
  const int64_t Wx = (int64_t)stride * Wo;
  for (int i = 0; i < nph; ++i) {
    MXAMD_HOST_CHECK(ph[i] >= 0 && ph[i] < stride && pw[i] >= 0 && pw[i] < stride && R[i] > 0 && S[i] > 0,
                     "conv_nhwc_dgrad_phases_glds: bad phase");
    GeomG& g = ps.g[i];
    g.N = N; g.H = Hi; g.W = Wi; g.C = Cin; g.K = Cout; g.R = R[i]; g.S = S[i];
    g.sh = 1; g.sw = 1; g.ph = pad_h[i]; g.pw = pad_w[i];
    g.Ho = Ho;
    g.Wo = Wo;
    g.M = N * Ho * Wo;
    g.Ktot = R[i] * S[i] * Cin;
    g.og = stride * Wx * Cout;
    g.oc = (int64_t)stride * Cout;
    g.ob = ((int64_t)ph[i] * Wx + pw[i]) * Cout;
    ps.w_off[i] = w_off[i];
    g.nz = i == 0 ? nzero : 0;    // the first phase's blocks also clear the phases no tap reaches
    for (int z = 0; z < nzero && i == 0; ++z) {
      MXAMD_HOST_CHECK(zph[z] >= 0 && zph[z] < stride && zpw[z] >= 0 && zpw[z] < stride,
                       "conv_nhwc_dgrad_phases_glds: bad zero phase");
      g.zob[z] = ((int64_t)zph[z] * Wx + zpw[z]) * Cout;
    }
    MXAMD_HOST_CHECK((int64_t)Cout * g.Ktot < (1ll << 31), "conv_nhwc_dgrad_phases_glds: weight too large");
  }
  const int bpix = bco == 128 ? 128 : 256;
  const int tiles_co = Cout / bco;
  const int tiles_pix = (N * Ho * Wo + bpix - 1) / bpix;
  dim3 grid(tiles_co * tiles_pix, nph);
  // partials: every phase gets conv_glds_bwd_nparts(N*Ho*Wo) slots (nparts = nph * that)
  const BnbG bn{bn_z, bn_mean, bn_scale, bn_shift, bn_part, bn_nparts};
  // (phases no tap reaches hold zero gradient: they add nothing to the statistics)
  MXAMD_HOST_CHECK(!bn_part || (bn_z && bn_mean && !bn_scale == !bn_shift &&
                                bn_nparts == nph * conv_glds_bwd_nparts(N * Ho * Wo, bco)),
                   "conv_nhwc_dgrad_phases_glds: BN-backward statistics need z, mean, scale, shift and nparts");
#define MXAMD_PHASES(T, B)                                                                                  \
  hipLaunchKernelGGL((conv_phase_glds_kernel<T, B>), grid, dim3(256), 0, s, static_cast<const T*>(dy),     \
                     static_cast<const T*>(w), static_cast<T*>(dx), static_cast<const T*>(zero), ps, tiles_co, bn)
  if (dtype == kF16) {
    if (bco == 128) MXAMD_PHASES(__half, 128);
    else MXAMD_PHASES(__half, 64);
  } else if (dtype == kBF16) {
    if (bco == 128) MXAMD_PHASES(__hip_bfloat16, 128);
    else MXAMD_PHASES(__hip_bfloat16, 64);
  } else {
    throw std::runtime_error("conv_nhwc_dgrad_phases_glds: dtype must be f16 or bf16");
  }
#undef MXAMD_PHASES
}

}  // namespace mxamd
