// Fused recurrent layers (RNN tanh/relu, LSTM, GRU) on gfx950.
//
// Reference semantics: src/operator/rnn-inl.h (cuDNN path :418 forward, :743 backward) and the
// CPU kernels of src/operator/rnn_impl.h: gate order LSTM i,f,g,o; GRU r,z,n with the recurrent
// bias of the n gate inside r * (h W_hn + b_hn).
//
// MI355X design (not a cuDNN translation):
//   * the input projection of every time step is ONE large GEMM done by the caller (in-tree
//     MFMA GEMM / hipBLASLt), giving gx[t][n][G*H] in fp32 with the biases folded in;
//   * per time step ONE launch computes, for a 16(batch) x 16(hidden) tile per workgroup (its 4
//     waves split the reduction and combine through LDS), the
//     recurrent GEMM h_{t-1} . W_hh^T of EVERY gate of those hidden units on the matrix cores
//     (v_mfma_f32_16x16x32_{f16,bf16}, or the exact-f32 v_mfma_f32_16x16x4_f32 for fp32
//     layers) and then the cell's pointwise update in registers -- the gate pre-activations
//     never touch memory;
//   * backward is the mirror image: one launch per step computes dh_{t} = dG_{t+1} . W_hh
//     (+ dy_t) for a tile and applies the cell's derivative, writing dG_t for the weight
//     gradients, which the caller then forms as two large GEMMs over all steps;
//   * the time loop runs on the host side of this file (no Python per step), so a whole
//     sequence is a run of back-to-back launches on one stream (and capturable in a HIP graph).
#include <stdexcept>

#include "common.h"
#include "mfma.h"

namespace mxamd {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

enum RnnMode : int { kRnnTanh = 0, kRnnRelu = 1, kLstm = 2, kGru = 3 };

template <int MODE>
struct RnnG {
  static constexpr int G = MODE == kLstm ? 4 : (MODE == kGru ? 3 : 1);      // gates
  static constexpr int SAVE = MODE == kLstm ? 4 : (MODE == kGru ? 4 : 1);   // saved activations per unit
};

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// ---- MFMA fragments.  A is [rows][K] row-major (rows = batch), B^T is [cols][K] row-major
// (cols = hidden units): lane l holds row/col (l & 15) and the K elements of its quarter.
template <typename T>
struct RFrag;

template <typename T>
__device__ __forceinline__ u32x4 load8(const T* row, int k, int K, bool ok, bool aligned) {
  u32x4 v = {0u, 0u, 0u, 0u};
  if (!ok) return v;
  if (aligned) {
    if (k + 8 <= K) v = *reinterpret_cast<const u32x4*>(row + k);
    return v;
  }
  uint16_t e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) e[i] = (k + i < K) ? __builtin_bit_cast(uint16_t, row[k + i]) : uint16_t(0);
  v[0] = e[0] | (uint32_t(e[1]) << 16);
  v[1] = e[2] | (uint32_t(e[3]) << 16);
  v[2] = e[4] | (uint32_t(e[5]) << 16);
  v[3] = e[6] | (uint32_t(e[7]) << 16);
  return v;
}

template <>
struct RFrag<__half> {
  typedef u32x4 frag;
  static constexpr int KSTEP = 32;
  static __device__ __forceinline__ frag load(const __half* row, int k0, int lane, int K, bool ok, bool al) {
    return load8(row, k0 + (lane >> 4) * 8, K, ok, al);
  }
  static __device__ __forceinline__ f4_t mma(const frag& a, const frag& b, f4_t c) {
    return mfma::Op<__half>::run(a, b, c);
  }
  static __device__ __forceinline__ __half from(float v) { return __float2half(v); }
  static __device__ __forceinline__ float to(__half v) { return __half2float(v); }
};

template <>
struct RFrag<__hip_bfloat16> {
  typedef u32x4 frag;
  static constexpr int KSTEP = 32;
  static __device__ __forceinline__ frag load(const __hip_bfloat16* row, int k0, int lane, int K, bool ok, bool al) {
    return load8(row, k0 + (lane >> 4) * 8, K, ok, al);
  }
  static __device__ __forceinline__ f4_t mma(const frag& a, const frag& b, f4_t c) {
    return mfma::Op<__hip_bfloat16>::run(a, b, c);
  }
  static __device__ __forceinline__ __hip_bfloat16 from(float v) { return __float2bfloat16(v); }
  static __device__ __forceinline__ float to(__hip_bfloat16 v) { return __bfloat162float(v); }
};

template <>
struct RFrag<float> {
  static __device__ __forceinline__ f4_t mma1(float a, float b, f4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ float from(float v) { return v; }
  static __device__ __forceinline__ float to(float v) { return v; }
};

__device__ __forceinline__ float4 load4f(const float* row, int k, int K, bool ok, bool aligned) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!ok) return v;
  if (aligned && k + 4 <= K) return *reinterpret_cast<const float4*>(row + k);
  if (k < K) v.x = row[k];
  if (k + 1 < K) v.y = row[k + 1];
  if (k + 2 < K) v.z = row[k + 2];
  if (k + 3 < K) v.w = row[k + 3];
  return v;
}

// acc[g] += A[n0.., kslice] . Bt[g*gstride + j0.., kslice]^T for the 16 x 16 tile, over the k-chunks
// of this wave (the 4 waves of a workgroup interleave chunks; their partial sums are combined after).
template <typename T, int G>
__device__ __forceinline__ void tile_gemm(f4_t (&acc)[G], const T* A, int lda, int nrows, const T* Bt, int ldb,
                                          int gstride, int ncols, int K, int n0, int j0, int lane, int wave,
                                          bool aligned) {
  const int r = lane & 15;
  const bool aok = n0 + r < nrows;
  const bool bok = j0 + r < ncols;
  const T* arow = A + static_cast<int64_t>(aok ? n0 + r : 0) * lda;
  const T* brow[G];
#pragma unroll
  for (int g = 0; g < G; ++g) brow[g] = Bt + static_cast<int64_t>(g * gstride + (bok ? j0 + r : 0)) * ldb;
  if constexpr (sizeof(T) == 4) {
    // exact-f32 MFMA, 4 k per instruction; each lane loads 4 consecutive k (16 bytes) and the 4
    // MFMAs of the chunk take element s of every lane: the k order is permuted identically for A
    // and B, so the sum is unchanged
    const int kq = (lane >> 4) * 4;
#pragma unroll 2
    for (int k0 = wave * 16; k0 < K; k0 += 64) {
      const float4 a = load4f(reinterpret_cast<const float*>(arow), k0 + kq, K, aok, aligned);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float4 b = load4f(reinterpret_cast<const float*>(brow[g]), k0 + kq, K, bok, aligned);
        acc[g] = RFrag<float>::mma1(a.x, b.x, acc[g]);
        acc[g] = RFrag<float>::mma1(a.y, b.y, acc[g]);
        acc[g] = RFrag<float>::mma1(a.z, b.z, acc[g]);
        acc[g] = RFrag<float>::mma1(a.w, b.w, acc[g]);
      }
    }
  } else {
    using F = RFrag<T>;
#pragma unroll 2
    for (int k0 = wave * 32; k0 < K; k0 += 128) {
      const typename F::frag a = F::load(arow, k0, lane, K, aok, aligned);
#pragma unroll
      for (int g = 0; g < G; ++g) acc[g] = F::mma(a, F::load(brow[g], k0, lane, K, bok, aligned), acc[g]);
    }
  }
}

// Combine the 4 waves' partial tiles through LDS: on return, `v[g]` holds element q = wave of the
// summed accumulators (row (lane>>4)*4 + wave, column lane & 15) -- each wave then finishes one
// of the four rows a lane holds.
template <int G>
__device__ __forceinline__ void reduce4(const f4_t (&acc)[G], float (&v)[G], float* red, int lane, int wave) {
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[((wave * G + g) * 4 + q) * 64 + lane] = acc[g][q];
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) t += red[((w * G + g) * 4 + wave) * 64 + lane];
    v[g] = t;
  }
}

// ---------------------------------------------------------------------------------------------
// forward step
template <typename T, int MODE>
__global__ void __launch_bounds__(256) rnn_step_fwd_kernel(const T* __restrict__ hprev, int ldh,
                                                           const float* __restrict__ cprev,
                                                           const T* __restrict__ whh, const float* __restrict__ gx,
                                                           const float* __restrict__ bhh, T* __restrict__ hout,
                                                           int ldo, float* __restrict__ cout,
                                                           float* __restrict__ save, int N, int H, int ntj,
                                                           int aligned) {
  constexpr int G = RnnG<MODE>::G;
  constexpr int SV = RnnG<MODE>::SAVE;
  using F = RFrag<T>;
  __shared__ float red[4 * G * 4 * 64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  // one workgroup per 16 x 16 tile; its 4 waves split the reduction
  const int tn = blockIdx.x / ntj, tj = blockIdx.x - tn * ntj;
  const int n0 = tn * 16, j0 = tj * 16;
  f4_t acc[G];
#pragma unroll
  for (int g = 0; g < G; ++g) acc[g] = f4_t{0.f, 0.f, 0.f, 0.f};
  tile_gemm<T, G>(acc, hprev, ldh, N, whh, H, H, H, H, n0, j0, lane, wave, aligned != 0);
  float pre[G];
  reduce4<G>(acc, pre, red, lane, wave);

  const int j = j0 + (lane & 15);
  const int n = n0 + (lane >> 4) * 4 + wave;   // this wave finishes row q = wave of the lane's four
  if (j >= H || n >= N) return;
  const float* gxr = gx + static_cast<int64_t>(n) * G * H;
  float* sv = save + static_cast<int64_t>(n) * SV * H;
  const int64_t nh = static_cast<int64_t>(n) * H + j;
  float h;
  if (MODE == kLstm) {
    const float i = sigm(pre[0] + gxr[j]);
    const float f = sigm(pre[1 % G] + gxr[H + j]);
    const float g = tanhf(pre[2 % G] + gxr[2 * H + j]);
    const float o = sigm(pre[3 % G] + gxr[3 * H + j]);
    const float c = f * cprev[nh] + i * g;
    h = o * tanhf(c);
    cout[nh] = c;
    sv[j] = i;
    sv[H + j] = f;
    sv[2 * H + j] = g;
    sv[3 * H + j] = o;
  } else if (MODE == kGru) {
    const float r = sigm(pre[0] + gxr[j] + bhh[j]);
    const float z = sigm(pre[1 % G] + gxr[H + j] + bhh[H + j]);
    const float hn = pre[2 % G] + bhh[2 * H + j];
    const float nn = tanhf(gxr[2 * H + j] + r * hn);
    const float hp = F::to(hprev[static_cast<int64_t>(n) * ldh + j]);
    h = (1.f - z) * nn + z * hp;
    sv[j] = r;
    sv[H + j] = z;
    sv[2 * H + j] = nn;
    sv[3 * H + j] = hn;
  } else {
    const float p = pre[0] + gxr[j];
    h = MODE == kRnnTanh ? tanhf(p) : fmaxf(p, 0.f);
    sv[j] = h;
  }
  hout[static_cast<int64_t>(n) * ldo + j] = F::from(h);
}

// ---------------------------------------------------------------------------------------------
// backward step: dh = dG_{t+1} . W_hh (+ dy_t + carried direct terms), then the cell derivative
template <typename T, int MODE>
__global__ void __launch_bounds__(256) rnn_step_bwd_kernel(
    const T* __restrict__ dgh_next, const T* __restrict__ whhT, const T* __restrict__ dy, int ldy,
    const float* __restrict__ dh_last, const float* __restrict__ save, const float* __restrict__ cprev,
    const float* __restrict__ cur_c, float* __restrict__ dc, float* __restrict__ dhd, const T* __restrict__ hprev,
    int ldh, T* __restrict__ dgh, T* __restrict__ dgx, float* __restrict__ dh_out, int N, int H, int ntj,
    int aligned) {
  constexpr int G = RnnG<MODE>::G;
  constexpr int SV = RnnG<MODE>::SAVE;
  using F = RFrag<T>;
  __shared__ float red[4 * 4 * 64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tn = blockIdx.x / ntj, tj = blockIdx.x - tn * ntj;
  const int n0 = tn * 16, j0 = tj * 16;
  f4_t acc[1] = {f4_t{0.f, 0.f, 0.f, 0.f}};
  if (dgh_next != nullptr)
    tile_gemm<T, 1>(acc, dgh_next, G * H, N, whhT, G * H, 0, H, G * H, n0, j0, lane, wave, aligned != 0);
  float dsum[1];
  reduce4<1>(acc, dsum, red, lane, wave);

  const int j = j0 + (lane & 15);
  const int n = n0 + (lane >> 4) * 4 + wave;
  if (j >= H || n >= N) return;
  const int64_t nh = static_cast<int64_t>(n) * H + j;
  float d = dsum[0];
  if (dh_last != nullptr) d += dh_last[nh];
  if (dhd != nullptr) d += dhd[nh];
  if (dh_out != nullptr) {  // final pass: the gradient of the initial state, no cell derivative
    dh_out[nh] = d;
    return;
  }
  if (dy != nullptr) d += F::to(dy[static_cast<int64_t>(n) * ldy + j]);
  const float* sv = save + static_cast<int64_t>(n) * SV * H;
  T* gh = dgh + static_cast<int64_t>(n) * G * H;
  if (MODE == kLstm) {
    const float i = sv[j], f = sv[H + j], g = sv[2 * H + j], o = sv[3 * H + j];
    const float tc = tanhf(cur_c[nh]);
    const float dct = dc[nh] + d * o * (1.f - tc * tc);
    gh[j] = F::from(dct * g * i * (1.f - i));
    gh[H + j] = F::from(dct * cprev[nh] * f * (1.f - f));
    gh[2 * H + j] = F::from(dct * i * (1.f - g * g));
    gh[3 * H + j] = F::from(d * tc * o * (1.f - o));
    dc[nh] = dct * f;
  } else if (MODE == kGru) {
    const float r = sv[j], z = sv[H + j], nn = sv[2 * H + j], hn = sv[3 * H + j];
    const float hp = F::to(hprev[static_cast<int64_t>(n) * ldh + j]);
    const float dn = d * (1.f - z) * (1.f - nn * nn);
    const float dz = d * (hp - nn) * z * (1.f - z);
    const float dr = dn * hn * r * (1.f - r);
    T* gxo = dgx + static_cast<int64_t>(n) * G * H;
    gh[j] = F::from(dr);
    gh[H + j] = F::from(dz);
    gh[2 * H + j] = F::from(dn * r);
    gxo[j] = F::from(dr);
    gxo[H + j] = F::from(dz);
    gxo[2 * H + j] = F::from(dn);
    dhd[nh] = d * z;  // the direct h_{t-1} -> h_t path, added by the previous step's launch
  } else {
    const float h = sv[j];
    gh[j] = F::from(MODE == kRnnTanh ? d * (1.f - h * h) : (h > 0.f ? d : 0.f));
  }
}

template <typename T, int MODE>
void fwd_seq(const float* gx, const void* h0, const float* c0, const void* whh, const float* bhh, void* out,
             int ldo, float* cseq, float* save, int Tn, int N, int H, int reverse, hipStream_t s) {
  constexpr int G = RnnG<MODE>::G;
  constexpr int SV = RnnG<MODE>::SAVE;
  const int ntj = (H + 15) / 16;
  const int blocks = ((N + 15) / 16) * ntj;  // one workgroup (4 waves, split-K) per 16 x 16 tile
  const int vec = sizeof(T) == 4 ? 4 : 8;
  const int aligned = (H % vec == 0 && ldo % vec == 0 && (reinterpret_cast<uintptr_t>(out) % 16) == 0 &&
                       (reinterpret_cast<uintptr_t>(h0) % 16) == 0 && (reinterpret_cast<uintptr_t>(whh) % 16) == 0)
                          ? 1
                          : 0;
  const T* o = static_cast<const T*>(out);
  for (int i = 0; i < Tn; ++i) {
    const int t = reverse ? Tn - 1 - i : i;
    const int tp = reverse ? t + 1 : t - 1;
    const T* hp = i == 0 ? static_cast<const T*>(h0) : o + static_cast<int64_t>(tp) * N * ldo;
    const int ldh = i == 0 ? H : ldo;
    const float* cp = MODE == kLstm ? (i == 0 ? c0 : cseq + static_cast<int64_t>(tp) * N * H) : nullptr;
    hipLaunchKernelGGL((rnn_step_fwd_kernel<T, MODE>), dim3(blocks), dim3(256), 0, s, hp, ldh, cp,
                       static_cast<const T*>(whh), gx + static_cast<int64_t>(t) * N * G * H, bhh,
                       static_cast<T*>(out) + static_cast<int64_t>(t) * N * ldo, ldo,
                       MODE == kLstm ? cseq + static_cast<int64_t>(t) * N * H : nullptr,
                       save + static_cast<int64_t>(t) * N * SV * H, N, H, ntj, aligned);
  }
}

template <typename T, int MODE>
void bwd_seq(const void* whhT, const void* dy, int ldy, const float* dhT, const float* save, const float* cseq,
             const float* c0, const void* h0, const void* out, int ldo, void* dgh, void* dgx, float* dc,
             float* dhd, float* dh0, int Tn, int N, int H, int reverse, hipStream_t s) {
  constexpr int G = RnnG<MODE>::G;
  constexpr int SV = RnnG<MODE>::SAVE;
  const int ntj = (H + 15) / 16;
  const int blocks = ((N + 15) / 16) * ntj;
  const int vec = sizeof(T) == 4 ? 4 : 8;
  const int aligned = ((G * H) % vec == 0 && (reinterpret_cast<uintptr_t>(whhT) % 16) == 0 &&
                       (reinterpret_cast<uintptr_t>(dgh) % 16) == 0)
                          ? 1
                          : 0;
  const T* o = static_cast<const T*>(out);
  const T* dyp = static_cast<const T*>(dy);
  T* gh = static_cast<T*>(dgh);
  T* gxp = static_cast<T*>(dgx);
  const int64_t step = static_cast<int64_t>(N) * G * H;
  // processing order is the reverse of the forward order: i = Tn-1 .. 0 in forward-step index
  for (int i = Tn - 1; i >= 0; --i) {
    const int t = reverse ? Tn - 1 - i : i;
    const int tn = reverse ? t - 1 : t + 1;  // the step processed just before (forward step i+1)
    const int tp = reverse ? t + 1 : t - 1;  // forward step i-1
    const T* next = i == Tn - 1 ? nullptr : gh + tn * step;
    const float* cp = MODE == kLstm ? (i == 0 ? c0 : cseq + static_cast<int64_t>(tp) * N * H) : nullptr;
    const T* hp = i == 0 ? static_cast<const T*>(h0) : o + static_cast<int64_t>(tp) * N * ldo;
    const int ldh = i == 0 ? H : ldo;
    hipLaunchKernelGGL((rnn_step_bwd_kernel<T, MODE>), dim3(blocks), dim3(256), 0, s, next,
                       static_cast<const T*>(whhT), dyp ? dyp + static_cast<int64_t>(t) * N * ldy : nullptr, ldy,
                       i == Tn - 1 ? dhT : nullptr, save + static_cast<int64_t>(t) * N * SV * H, cp,
                       MODE == kLstm ? cseq + static_cast<int64_t>(t) * N * H : nullptr, dc,
                       MODE == kGru ? dhd : nullptr, hp, ldh, gh + t * step, gxp ? gxp + t * step : nullptr,
                       nullptr, N, H, ntj, aligned);
  }
  // dh0 = dG_first . W_hh (+ GRU direct term)
  const int t0 = reverse ? Tn - 1 : 0;
  hipLaunchKernelGGL((rnn_step_bwd_kernel<T, MODE>), dim3(blocks), dim3(256), 0, s, gh + t0 * step,
                     static_cast<const T*>(whhT), static_cast<const T*>(nullptr), 0, static_cast<const float*>(nullptr),
                     save, static_cast<const float*>(nullptr), static_cast<const float*>(nullptr), dc,
                     MODE == kGru ? dhd : nullptr, static_cast<const T*>(nullptr), 0, gh, gxp, dh0, N, H, ntj,
                     aligned);
}

template <typename T>
void fwd_mode(int mode, const float* gx, const void* h0, const float* c0, const void* whh, const float* bhh,
              void* out, int ldo, float* cseq, float* save, int Tn, int N, int H, int reverse, hipStream_t s) {
  switch (mode) {
    case kRnnTanh: fwd_seq<T, kRnnTanh>(gx, h0, c0, whh, bhh, out, ldo, cseq, save, Tn, N, H, reverse, s); break;
    case kRnnRelu: fwd_seq<T, kRnnRelu>(gx, h0, c0, whh, bhh, out, ldo, cseq, save, Tn, N, H, reverse, s); break;
    case kLstm: fwd_seq<T, kLstm>(gx, h0, c0, whh, bhh, out, ldo, cseq, save, Tn, N, H, reverse, s); break;
    case kGru: fwd_seq<T, kGru>(gx, h0, c0, whh, bhh, out, ldo, cseq, save, Tn, N, H, reverse, s); break;
    default: throw std::runtime_error("rnn_fwd_seq: unknown mode");
  }
}

template <typename T>
void bwd_mode(int mode, const void* whhT, const void* dy, int ldy, const float* dhT, const float* save,
              const float* cseq, const float* c0, const void* h0, const void* out, int ldo, void* dgh, void* dgx,
              float* dc, float* dhd, float* dh0, int Tn, int N, int H, int reverse, hipStream_t s) {
#define MXAMD_RNN_BWD(M) \
  bwd_seq<T, M>(whhT, dy, ldy, dhT, save, cseq, c0, h0, out, ldo, dgh, dgx, dc, dhd, dh0, Tn, N, H, reverse, s)
  switch (mode) {
    case kRnnTanh: MXAMD_RNN_BWD(kRnnTanh); break;
    case kRnnRelu: MXAMD_RNN_BWD(kRnnRelu); break;
    case kLstm: MXAMD_RNN_BWD(kLstm); break;
    case kGru: MXAMD_RNN_BWD(kGru); break;
    default: throw std::runtime_error("rnn_bwd_seq: unknown mode");
  }
#undef MXAMD_RNN_BWD
}

}  // namespace

// Forward over a whole sequence for one (layer, direction).  gx: [T][N][G*H] fp32 input projection
// with the biases folded in (GRU: b_ih only; b_hh passed as bhh), h0: [N][H] (dtype), c0: [N][H]
// fp32 (LSTM), whh: [G*H][H] (dtype), out: [T][N][ldo] (this direction's columns), cseq: [T][N][H]
// fp32 (LSTM), save: [T][N][SAVE*H] fp32 activations for the backward.
void rnn_fwd_seq(int dtype, int mode, const float* gx, const void* h0, const float* c0, const void* whh,
                 const float* bhh, void* out, int ldo, float* cseq, float* save, int Tn, int N, int H, int reverse,
                 hipStream_t s) {
  MXAMD_HOST_CHECK(Tn > 0 && N > 0 && H > 0 && ldo >= H, "rnn_fwd_seq: bad sizes");
  MXAMD_HOST_CHECK((int64_t)Tn * N * ldo < (1ll << 31) && (int64_t)Tn * N * 4 * H < (1ll << 31),
                   "rnn_fwd_seq: sequence too large for 32-bit indexing");
  if (dtype == kF32) fwd_mode<float>(mode, gx, h0, c0, whh, bhh, out, ldo, cseq, save, Tn, N, H, reverse, s);
  else if (dtype == kF16) fwd_mode<__half>(mode, gx, h0, c0, whh, bhh, out, ldo, cseq, save, Tn, N, H, reverse, s);
  else if (dtype == kBF16)
    fwd_mode<__hip_bfloat16>(mode, gx, h0, c0, whh, bhh, out, ldo, cseq, save, Tn, N, H, reverse, s);
  else throw std::runtime_error("rnn_fwd_seq: dtype");
}

// Backward over the sequence.  whhT: [H][G*H] (W_hh transposed), dy: [T][N][ldy] output gradient
// (or null), dhT: [N][H] fp32 gradient of the final hidden state (or null), dc: [N][H] fp32 holding
// the gradient of the final cell state on entry and that of c0 on exit (LSTM), dhd: [N][H] fp32
// zeroed scratch (GRU), dh0: [N][H] fp32 output.  dgh / dgx: [T][N][G*H] gate gradients (dgx only
// for GRU, where the n gate's input-side gradient differs).
void rnn_bwd_seq(int dtype, int mode, const void* whhT, const void* dy, int ldy, const float* dhT,
                 const float* save, const float* cseq, const float* c0, const void* h0, const void* out, int ldo,
                 void* dgh, void* dgx, float* dc, float* dhd, float* dh0, int Tn, int N, int H, int reverse,
                 hipStream_t s) {
  MXAMD_HOST_CHECK(Tn > 0 && N > 0 && H > 0, "rnn_bwd_seq: bad sizes");
  MXAMD_HOST_CHECK(mode != kGru || (dgx != nullptr && dhd != nullptr), "rnn_bwd_seq: GRU needs dgx and dhd");
  MXAMD_HOST_CHECK(mode != kLstm || (dc != nullptr && cseq != nullptr && c0 != nullptr),
                   "rnn_bwd_seq: LSTM needs dc, cseq and c0");
  if (dtype == kF32)
    bwd_mode<float>(mode, whhT, dy, ldy, dhT, save, cseq, c0, h0, out, ldo, dgh, dgx, dc, dhd, dh0, Tn, N, H, reverse,
                    s);
  else if (dtype == kF16)
    bwd_mode<__half>(mode, whhT, dy, ldy, dhT, save, cseq, c0, h0, out, ldo, dgh, dgx, dc, dhd, dh0, Tn, N, H,
                     reverse, s);
  else if (dtype == kBF16)
    bwd_mode<__hip_bfloat16>(mode, whhT, dy, ldy, dhT, save, cseq, c0, h0, out, ldo, dgh, dgx, dc, dhd, dh0, Tn, N,
                             H, reverse, s);
  else throw std::runtime_error("rnn_bwd_seq: dtype");
}

}  // namespace mxamd
