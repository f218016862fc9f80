// Fused multi-head self-attention (forward + backward) on gfx950 matrix cores.
//
// Parity: the self-attention block MXNet users build from
// src/operator/contrib/transformer.cu (interleaved_matmul_selfatt_qk ->
// softmax (+ valid-length mask) -> Dropout -> interleaved_matmul_selfatt_valatt,
// transformer.cu:657 onwards), computed here in ONE pass per (batch, head)
// without materialising the (B*H, S, S) score tensor.
//
// Layouts are the reference's: the fused projection qkv is (S, B, H*3*D) with
// [q k v] interleaved per head (D = 64); the output is (S, B, H*D); the
// gradient dqkv has the layout of qkv, so no permute/copy kernels surround the
// op in either direction.
//
// MI355X design (v_mfma_f32_16x16x32_{bf16,f16}, wave64):
//  * forward: block = 4 waves over 64 queries of one (b, h); K (row image) and
//    Vᵀ (transposed image) of the head are staged in LDS once, each wave keeps
//    its 16 queries' Q in registers and walks the keys in 32-key chunks with an
//    online (base-2) softmax.  Scores are computed TRANSPOSED, Sᵀ = K·Qᵀ, so the
//    accumulator (col = query on the lane, rows = keys in registers) is directly
//    the B operand of Oᵀ = Vᵀ·Pᵀ (k order permuted identically on the Vᵀ side),
//    the row statistics are lane-local plus a 4-group shuffle, and no LDS round
//    trip is needed for P.  Writes O and the per-row log-sum-exp (log2 units).
//  * backward = two kernels, neither needs atomics:
//    - dq: same orientation as the forward (per wave 16 queries, all keys):
//      Pᵀ, dPᵀ = V·dOᵀ, dSᵀ = Pᵀ∘(dPᵀ∘Z/(1-p) − Δ), dQᵀ += Kᵀ·dSᵀ; also writes
//      Δ = rowsum(dO∘O) for the second kernel.
//    - dkdv: per wave 16 keys, all queries, the NON-transposed orientation
//      (col = key on the lane), so P and dS feed dVᵀ = dOᵀ·P∘Z/(1-p) and
//      dKᵀ = Qᵀ·dS as B operands; Qᵀ/dOᵀ images in LDS supply the A operands.
//  * dropout: keep(q, k) = hash(seed, (bh*S + q)*S + k) >= p*2^32, a stateless
//    per-element hash, so the backward regenerates the forward's mask in its
//    own orientation; seed_base (device, optional) re-keys HIP-graph replays.
//  * key padding mask: (B, S) with 1 = attend, 0 = padded key (valid_length).
//  * LDS rows are padded (K/Q/dO row images 72 elements, transposed images S+4)
//    so the 16-byte row reads and the 8-byte transposed reads are bank-conflict
//    free across each 16-lane group.
// Requirements (checked by the launchers + ops/attention_fns.py): D == 64,
// S % 32 == 0, S <= 256, 16-byte aligned contiguous tensors.
#include <stdexcept>

#include "common.h"
#include "mfma.h"

namespace mxamd {

namespace {

constexpr int kD = 64;      // head dim
constexpr int kRow = 72;    // padded row image stride (elements)

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

template <typename T>
struct AOp;

template <>
struct AOp<__hip_bfloat16> {
  static __device__ __forceinline__ f4 mma(const u4& a, const u4& b, f4 c) {
    return mfma::Op<__hip_bfloat16>::run(a, b, c);
  }
  static __device__ __forceinline__ uint32_t pack2(float a, float b) {
    uint32_t ua = __float_as_uint(a), ub = __float_as_uint(b);
    ua += 0x7fff + ((ua >> 16) & 1);
    ub += 0x7fff + ((ub >> 16) & 1);
    return (ua >> 16) | (ub & 0xffff0000u);
  }
  static __device__ __forceinline__ float lo(uint32_t v) { return __uint_as_float(v << 16); }
  static __device__ __forceinline__ float hi(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }
};

template <>
struct AOp<__half> {
  static __device__ __forceinline__ f4 mma(const u4& a, const u4& b, f4 c) {
    return mfma::Op<__half>::run(a, b, c);
  }
  static __device__ __forceinline__ uint32_t pack2(float a, float b) {
    __half2 h = __floats2half2_rn(a, b);
    return *reinterpret_cast<uint32_t*>(&h);
  }
  static __device__ __forceinline__ float lo(uint32_t v) {
    return __half2float(__ushort_as_half(static_cast<unsigned short>(v & 0xffffu)));
  }
  static __device__ __forceinline__ float hi(uint32_t v) {
    return __half2float(__ushort_as_half(static_cast<unsigned short>(v >> 16)));
  }
};

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

struct DropKey {
  uint32_t k0, k1, thresh;
  float inv_keep;
  bool on;
  __device__ __forceinline__ DropKey(float p, uint64_t seed, const uint64_t* seed_base) {
    if (seed_base != nullptr) seed += seed_base[0] * 0x9E3779B97F4A7C15ull;
    k0 = (uint32_t)seed;
    k1 = (uint32_t)(seed >> 32);
    thresh = (uint32_t)fminf(p * 4294967296.f, 4294967295.f);
    inv_keep = p < 1.f ? 1.f / (1.f - p) : 0.f;
    on = p > 0.f;
  }
  __device__ __forceinline__ bool keep(uint32_t idx) const { return mix32(mix32(idx ^ k0) + k1) >= thresh; }
};

// stage rows [0, S) of one head component (offset `comp` in a row of stride `ld`) into an LDS
// row image (stride kRow) and/or a transposed image (stride S+4)
template <typename T>
__device__ __forceinline__ void stage(const T* base, size_t row_stride, int S, uint16_t* rows, uint16_t* tr) {
  for (int v = threadIdx.x; v < S * 8; v += blockDim.x) {
    const int r = v >> 3, d0 = (v & 7) * 8;
    const u4 x = *reinterpret_cast<const u4*>(base + (size_t)r * row_stride + d0);
    if (rows != nullptr) *reinterpret_cast<u4*>(rows + r * kRow + d0) = x;
    if (tr != nullptr) {
      const uint16_t* e = reinterpret_cast<const uint16_t*>(&x);
#pragma unroll
      for (int j = 0; j < 8; ++j) tr[(d0 + j) * (S + 4) + r] = e[j];
    }
  }
}

__device__ __forceinline__ u4 lds16(const uint16_t* p) { return *reinterpret_cast<const u4*>(p); }

// A fragment from a transposed image: row `row`, k-chunk at column c0 with the accumulator
// permutation (elements 0..3 = cols c0+4g..+3, 4..7 = cols c0+16+4g..+3)
__device__ __forceinline__ u4 tr_frag(const uint16_t* tr, int ld, int row, int c0, int g) {
  const uint16_t* p = tr + row * ld + c0 + 4 * g;
  const u2 a = *reinterpret_cast<const u2*>(p);
  const u2 b = *reinterpret_cast<const u2*>(p + 16);
  u4 r;
  r[0] = a[0];
  r[1] = a[1];
  r[2] = b[0];
  r[3] = b[1];
  return r;
}

template <typename T>
__device__ __forceinline__ u4 pack8(const float (&v)[8]) {
  u4 r;
  r[0] = AOp<T>::pack2(v[0], v[1]);
  r[1] = AOp<T>::pack2(v[2], v[3]);
  r[2] = AOp<T>::pack2(v[4], v[5]);
  r[3] = AOp<T>::pack2(v[6], v[7]);
  return r;
}

// ------------------------------------------------------------------ forward
template <typename T>
__global__ void __launch_bounds__(256) attn_fwd_kernel(const T* __restrict__ qkv, const float* __restrict__ kmask,
                                                       T* __restrict__ out, float* __restrict__ lse, int S, int B,
                                                       int H, float c, float p, uint64_t seed,
                                                       const uint64_t* __restrict__ seed_base) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* Ks = reinterpret_cast<uint16_t*>(smem);
  uint16_t* Vt = Ks + S * kRow;
  float* mb = reinterpret_cast<float*>(Vt + kD * (S + 4));
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const size_t ld = (size_t)B * H * 3 * kD;  // stride between sequence positions
  const T* head = qkv + (size_t)b * H * 3 * kD + h * 3 * kD;
  stage<T>(head + kD, ld, S, Ks, nullptr);
  stage<T>(head + 2 * kD, ld, S, nullptr, Vt);
  for (int k = threadIdx.x; k < S; k += blockDim.x)
    mb[k] = (kmask == nullptr || kmask[(size_t)b * S + k] != 0.f) ? 0.f : -INFINITY;
  __syncthreads();
  const int q = blockIdx.y * 64 + w * 16 + r;
  if (blockIdx.y * 64 + w * 16 >= S) return;  // no barrier below
  const DropKey dk(p, seed, seed_base);
  const T* qp = head + (size_t)q * ld;
  const u4 qf0 = *reinterpret_cast<const u4*>(qp + 8 * g);
  const u4 qf1 = *reinterpret_cast<const u4*>(qp + 32 + 8 * g);
  f4 o[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) o[m] = f4{0.f, 0.f, 0.f, 0.f};
  float mrun = -INFINITY, l = 0.f;
  const uint32_t rowid = ((uint32_t)bh * S + q) * (uint32_t)S;
  for (int c0 = 0; c0 < S; c0 += 32) {
    f4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
    s0 = AOp<T>::mma(lds16(Ks + (c0 + r) * kRow + 8 * g), qf0, s0);
    s1 = AOp<T>::mma(lds16(Ks + (c0 + 16 + r) * kRow + 8 * g), qf0, s1);
    s0 = AOp<T>::mma(lds16(Ks + (c0 + r) * kRow + 32 + 8 * g), qf1, s0);
    s1 = AOp<T>::mma(lds16(Ks + (c0 + 16 + r) * kRow + 32 + 8 * g), qf1, s1);
    float x[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[i] = s0[i] * c + mb[c0 + 4 * g + i];
      x[4 + i] = s1[i] * c + mb[c0 + 16 + 4 * g + i];
    }
    float mx = x[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) mx = fmaxf(mx, x[i]);
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(mrun, mx);
    const float ms = mn == -INFINITY ? 0.f : mn;
    const float alpha = exp2f(mrun - ms);
    float ps = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      x[i] = exp2f(x[i] - ms);
      ps += x[i];
    }
    l = l * alpha + ps;
    mrun = mn;
    if (dk.on) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (!dk.keep(rowid + c0 + 16 * (i >> 2) + 4 * g + (i & 3))) x[i] = 0.f;
    }
    const u4 pf = pack8<T>(x);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      o[m] *= alpha;
      o[m] = AOp<T>::mma(tr_frag(Vt, S + 4, 16 * m + r, c0, g), pf, o[m]);
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float inv = l > 0.f ? (dk.on ? dk.inv_keep : 1.f) / l : 0.f;
  T* op = out + (size_t)q * B * H * kD + (size_t)b * H * kD + h * kD;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    u2 v;
    v[0] = AOp<T>::pack2(o[m][0] * inv, o[m][1] * inv);
    v[1] = AOp<T>::pack2(o[m][2] * inv, o[m][3] * inv);
    *reinterpret_cast<u2*>(op + 16 * m + 4 * g) = v;
  }
  if (g == 0) lse[(size_t)bh * S + q] = l > 0.f ? mrun + log2f(l) : INFINITY;
}

// ------------------------------------------------------------------ backward: dQ (+ Δ)
template <typename T>
__global__ void __launch_bounds__(256) attn_bwd_dq_kernel(const T* __restrict__ qkv, const float* __restrict__ kmask,
                                                          const T* __restrict__ out, const T* __restrict__ dout,
                                                          const float* __restrict__ lse, float* __restrict__ delta,
                                                          T* __restrict__ dqkv, int S, int B, int H, float c,
                                                          float scale, float p, uint64_t seed,
                                                          const uint64_t* __restrict__ seed_base) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* Ks = reinterpret_cast<uint16_t*>(smem);
  uint16_t* Vs = Ks + S * kRow;
  uint16_t* Kt = Vs + S * kRow;
  float* mb = reinterpret_cast<float*>(Kt + kD * (S + 4));
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const size_t ld = (size_t)B * H * 3 * kD, ldo = (size_t)B * H * kD;
  const T* head = qkv + (size_t)b * H * 3 * kD + h * 3 * kD;
  stage<T>(head + kD, ld, S, Ks, Kt);
  stage<T>(head + 2 * kD, ld, S, Vs, nullptr);
  for (int k = threadIdx.x; k < S; k += blockDim.x)
    mb[k] = (kmask == nullptr || kmask[(size_t)b * S + k] != 0.f) ? 0.f : -INFINITY;
  __syncthreads();
  const int q = blockIdx.y * 64 + w * 16 + r;
  if (blockIdx.y * 64 + w * 16 >= S) return;
  const DropKey dk(p, seed, seed_base);
  const T* qp = head + (size_t)q * ld;
  const u4 qf0 = *reinterpret_cast<const u4*>(qp + 8 * g);
  const u4 qf1 = *reinterpret_cast<const u4*>(qp + 32 + 8 * g);
  const size_t orow = (size_t)q * ldo + (size_t)b * H * kD + h * kD;
  const u4 df0 = *reinterpret_cast<const u4*>(dout + orow + 8 * g);
  const u4 df1 = *reinterpret_cast<const u4*>(dout + orow + 32 + 8 * g);
  float dlt;
  {
    const u4 of0 = *reinterpret_cast<const u4*>(out + orow + 8 * g);
    const u4 of1 = *reinterpret_cast<const u4*>(out + orow + 32 + 8 * g);
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a += AOp<T>::lo(df0[j]) * AOp<T>::lo(of0[j]) + AOp<T>::hi(df0[j]) * AOp<T>::hi(of0[j]);
      a += AOp<T>::lo(df1[j]) * AOp<T>::lo(of1[j]) + AOp<T>::hi(df1[j]) * AOp<T>::hi(of1[j]);
    }
    a += __shfl_xor(a, 16, 64);
    a += __shfl_xor(a, 32, 64);
    dlt = a;
  }
  if (g == 0) delta[(size_t)bh * S + q] = dlt;
  const float lq = lse[(size_t)bh * S + q];
  f4 dq[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) dq[m] = f4{0.f, 0.f, 0.f, 0.f};
  const uint32_t rowid = ((uint32_t)bh * S + q) * (uint32_t)S;
  for (int c0 = 0; c0 < S; c0 += 32) {
    f4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, d0 = s0, d1 = s0;
    s0 = AOp<T>::mma(lds16(Ks + (c0 + r) * kRow + 8 * g), qf0, s0);
    s1 = AOp<T>::mma(lds16(Ks + (c0 + 16 + r) * kRow + 8 * g), qf0, s1);
    s0 = AOp<T>::mma(lds16(Ks + (c0 + r) * kRow + 32 + 8 * g), qf1, s0);
    s1 = AOp<T>::mma(lds16(Ks + (c0 + 16 + r) * kRow + 32 + 8 * g), qf1, s1);
    d0 = AOp<T>::mma(lds16(Vs + (c0 + r) * kRow + 8 * g), df0, d0);
    d1 = AOp<T>::mma(lds16(Vs + (c0 + 16 + r) * kRow + 8 * g), df0, d1);
    d0 = AOp<T>::mma(lds16(Vs + (c0 + r) * kRow + 32 + 8 * g), df1, d0);
    d1 = AOp<T>::mma(lds16(Vs + (c0 + 16 + r) * kRow + 32 + 8 * g), df1, d1);
    float ds[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int kk = c0 + 16 * (i >> 2) + 4 * g + (i & 3);
      const float sv = (i < 4 ? s0[i & 3] : s1[i & 3]) * c + mb[kk];
      const float pv = exp2f(sv - lq);
      float dp = i < 4 ? d0[i & 3] : d1[i & 3];
      if (dk.on) dp = dk.keep(rowid + kk) ? dp * dk.inv_keep : 0.f;
      ds[i] = pv * (dp - dlt);
    }
    const u4 sf = pack8<T>(ds);
#pragma unroll
    for (int m = 0; m < 4; ++m) dq[m] = AOp<T>::mma(tr_frag(Kt, S + 4, 16 * m + r, c0, g), sf, dq[m]);
  }
  T* dp = dqkv + (size_t)q * ld + (size_t)b * H * 3 * kD + h * 3 * kD;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    u2 v;
    v[0] = AOp<T>::pack2(dq[m][0] * scale, dq[m][1] * scale);
    v[1] = AOp<T>::pack2(dq[m][2] * scale, dq[m][3] * scale);
    *reinterpret_cast<u2*>(dp + 16 * m + 4 * g) = v;
  }
}

// ------------------------------------------------------------------ backward: dK, dV
template <typename T>
__global__ void __launch_bounds__(256) attn_bwd_dkdv_kernel(const T* __restrict__ qkv,
                                                            const float* __restrict__ kmask,
                                                            const T* __restrict__ dout, const float* __restrict__ lse,
                                                            const float* __restrict__ delta, T* __restrict__ dqkv,
                                                            int S, int B, int H, float c, float scale, float p,
                                                            uint64_t seed, const uint64_t* __restrict__ seed_base) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* Qs = reinterpret_cast<uint16_t*>(smem);
  uint16_t* Os = Qs + S * kRow;
  uint16_t* Qt = Os + S * kRow;
  uint16_t* Ot = Qt + kD * (S + 4);
  float* ls = reinterpret_cast<float*>(Ot + kD * (S + 4));
  float* dl = ls + S;
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const size_t ld = (size_t)B * H * 3 * kD, ldo = (size_t)B * H * kD;
  const T* head = qkv + (size_t)b * H * 3 * kD + h * 3 * kD;
  stage<T>(head, ld, S, Qs, Qt);
  stage<T>(dout + (size_t)b * H * kD + h * kD, ldo, S, Os, Ot);
  for (int k = threadIdx.x; k < S; k += blockDim.x) {
    ls[k] = lse[(size_t)bh * S + k];
    dl[k] = delta[(size_t)bh * S + k];
  }
  __syncthreads();
  const int key = blockIdx.y * 64 + w * 16 + r;
  if (blockIdx.y * 64 + w * 16 >= S) return;
  const DropKey dk(p, seed, seed_base);
  const T* kp = head + (size_t)key * ld + kD;
  const u4 kf0 = *reinterpret_cast<const u4*>(kp + 8 * g);
  const u4 kf1 = *reinterpret_cast<const u4*>(kp + 32 + 8 * g);
  const u4 vf0 = *reinterpret_cast<const u4*>(kp + kD + 8 * g);
  const u4 vf1 = *reinterpret_cast<const u4*>(kp + kD + 32 + 8 * g);
  const float mbk = (kmask == nullptr || kmask[(size_t)b * S + key] != 0.f) ? 0.f : -INFINITY;
  f4 dk_acc[4], dv_acc[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) dk_acc[m] = dv_acc[m] = f4{0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < S; c0 += 32) {
    f4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, d0 = s0, d1 = s0;
    s0 = AOp<T>::mma(lds16(Qs + (c0 + r) * kRow + 8 * g), kf0, s0);
    s1 = AOp<T>::mma(lds16(Qs + (c0 + 16 + r) * kRow + 8 * g), kf0, s1);
    s0 = AOp<T>::mma(lds16(Qs + (c0 + r) * kRow + 32 + 8 * g), kf1, s0);
    s1 = AOp<T>::mma(lds16(Qs + (c0 + 16 + r) * kRow + 32 + 8 * g), kf1, s1);
    d0 = AOp<T>::mma(lds16(Os + (c0 + r) * kRow + 8 * g), vf0, d0);
    d1 = AOp<T>::mma(lds16(Os + (c0 + 16 + r) * kRow + 8 * g), vf0, d1);
    d0 = AOp<T>::mma(lds16(Os + (c0 + r) * kRow + 32 + 8 * g), vf1, d0);
    d1 = AOp<T>::mma(lds16(Os + (c0 + 16 + r) * kRow + 32 + 8 * g), vf1, d1);
    float pd[8], ds[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int qq = c0 + 16 * (i >> 2) + 4 * g + (i & 3);
      const float sv = (i < 4 ? s0[i & 3] : s1[i & 3]) * c + mbk;
      const float pv = exp2f(sv - ls[qq]);
      float dp = i < 4 ? d0[i & 3] : d1[i & 3];
      float pz = pv;
      if (dk.on) {
        const bool kp2 = dk.keep(((uint32_t)bh * S + qq) * (uint32_t)S + key);
        dp = kp2 ? dp * dk.inv_keep : 0.f;
        pz = kp2 ? pv * dk.inv_keep : 0.f;
      }
      pd[i] = pz;
      ds[i] = pv * (dp - dl[qq]);
    }
    const u4 pf = pack8<T>(pd), sf = pack8<T>(ds);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      dv_acc[m] = AOp<T>::mma(tr_frag(Ot, S + 4, 16 * m + r, c0, g), pf, dv_acc[m]);
      dk_acc[m] = AOp<T>::mma(tr_frag(Qt, S + 4, 16 * m + r, c0, g), sf, dk_acc[m]);
    }
  }
  T* dp = dqkv + (size_t)key * ld + (size_t)b * H * 3 * kD + h * 3 * kD;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    u2 v;
    v[0] = AOp<T>::pack2(dk_acc[m][0] * scale, dk_acc[m][1] * scale);
    v[1] = AOp<T>::pack2(dk_acc[m][2] * scale, dk_acc[m][3] * scale);
    *reinterpret_cast<u2*>(dp + kD + 16 * m + 4 * g) = v;
    v[0] = AOp<T>::pack2(dv_acc[m][0], dv_acc[m][1]);
    v[1] = AOp<T>::pack2(dv_acc[m][2], dv_acc[m][3]);
    *reinterpret_cast<u2*>(dp + 2 * kD + 16 * m + 4 * g) = v;
  }
}

size_t fwd_smem(int S) { return (size_t)S * kRow * 2 + (size_t)kD * (S + 4) * 2 + (size_t)S * 4; }
size_t dq_smem(int S) { return (size_t)2 * S * kRow * 2 + (size_t)kD * (S + 4) * 2 + (size_t)S * 4; }
size_t dkdv_smem(int S) { return (size_t)2 * S * kRow * 2 + (size_t)2 * kD * (S + 4) * 2 + (size_t)2 * S * 4; }

template <typename K>
void allow_smem(K kernel, size_t bytes) {
  if (bytes > 64 * 1024)
    hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)bytes);
}

void check(int S, int D) {
  MXAMD_HOST_CHECK(D == kD, "attention: head dim must be 64");
  MXAMD_HOST_CHECK(S % 32 == 0 && S >= 32 && S <= 256, "attention: seq len must be a multiple of 32 in [32, 256]");
}

}  // namespace

int attention_max_seq() { return 256; }

void attention_forward(int dtype, const void* qkv, const float* kmask, void* out, float* lse, int S, int B, int H,
                       int D, float scale, float p, uint64_t seed, const uint64_t* seed_base, hipStream_t s) {
  check(S, D);
  const dim3 grid(B * H, (S + 63) / 64);
  const size_t sm = fwd_smem(S);
  const float c = scale * 1.4426950408889634f;
  if (dtype == kBF16) {
    allow_smem(attn_fwd_kernel<__hip_bfloat16>, sm);
    hipLaunchKernelGGL(attn_fwd_kernel<__hip_bfloat16>, grid, dim3(256), sm, s,
                       static_cast<const __hip_bfloat16*>(qkv), kmask, static_cast<__hip_bfloat16*>(out), lse, S, B,
                       H, c, p, seed, seed_base);
  } else if (dtype == kF16) {
    allow_smem(attn_fwd_kernel<__half>, sm);
    hipLaunchKernelGGL(attn_fwd_kernel<__half>, grid, dim3(256), sm, s, static_cast<const __half*>(qkv), kmask,
                       static_cast<__half*>(out), lse, S, B, H, c, p, seed, seed_base);
  } else {
    throw std::runtime_error("attention: dtype must be fp16 or bf16");
  }
}

void attention_backward(int dtype, const void* qkv, const float* kmask, const void* out, const void* dout,
                        const float* lse, float* delta, void* dqkv, int S, int B, int H, int D, float scale, float p,
                        uint64_t seed, const uint64_t* seed_base, hipStream_t s) {
  check(S, D);
  const dim3 grid(B * H, (S + 63) / 64);
  const float c = scale * 1.4426950408889634f;
  const size_t s1 = dq_smem(S), s2 = dkdv_smem(S);
  if (dtype == kBF16) {
    typedef __hip_bfloat16 T;
    allow_smem(attn_bwd_dq_kernel<T>, s1);
    allow_smem(attn_bwd_dkdv_kernel<T>, s2);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<T>, grid, dim3(256), s1, s, static_cast<const T*>(qkv), kmask,
                       static_cast<const T*>(out), static_cast<const T*>(dout), lse, delta, static_cast<T*>(dqkv), S,
                       B, H, c, scale, p, seed, seed_base);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<T>, grid, dim3(256), s2, s, static_cast<const T*>(qkv), kmask,
                       static_cast<const T*>(dout), lse, delta, static_cast<T*>(dqkv), S, B, H, c, scale, p, seed,
                       seed_base);
  } else if (dtype == kF16) {
    typedef __half T;
    allow_smem(attn_bwd_dq_kernel<T>, s1);
    allow_smem(attn_bwd_dkdv_kernel<T>, s2);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<T>, grid, dim3(256), s1, s, static_cast<const T*>(qkv), kmask,
                       static_cast<const T*>(out), static_cast<const T*>(dout), lse, delta, static_cast<T*>(dqkv), S,
                       B, H, c, scale, p, seed, seed_base);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<T>, grid, dim3(256), s2, s, static_cast<const T*>(qkv), kmask,
                       static_cast<const T*>(dout), lse, delta, static_cast<T*>(dqkv), S, B, H, c, scale, p, seed,
                       seed_base);
  } else {
    throw std::runtime_error("attention: dtype must be fp16 or bf16");
  }
}

}  // namespace mxamd
