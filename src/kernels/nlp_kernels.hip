// Transformer-path kernels for gfx950: LayerNorm, GELU, softmax, dropout.
//
// Parity: src/operator/nn/layer_norm.cu (LayerNorm fwd/bwd with mean/std
// outputs), src/operator/leaky_relu-inl.h (act_type='gelu', erf form),
// src/operator/nn/softmax-inl.h (softmax / log_softmax along the last axis,
// with temperature) and src/operator/nn/dropout-inl.h (Bernoulli mask,
// scaled by 1/(1-p)).  Design for MI355X:
//
// * rows (hidden <= 8192 or seq <= 8192) are held in registers by ONE wave64
//   (VPL 16-byte vectors per lane); mean/var/max/sum are wave reductions
//   (DPP/permute shuffles), so every row is read from HBM exactly once per pass;
// * a 256-thread block runs 4 rows; grids are sized to fill 256 CUs;
// * LayerNorm dgamma/dbeta: per-block column partials (fp32, LDS combine of the
//   4 waves) + one column-reduce kernel that writes or accumulates the fp32
//   parameter gradient -- no atomics, deterministic;
// * dropout draws Philox-4x32-10 counters keyed by (seed, element index), so the
//   mask is reproducible from the seed and is stored as 1 bit per element.
#include <stdexcept>

#include <cstdlib>

#include "common.h"

namespace mxamd {

namespace {

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&v)[8]) {
  Vec8<T> t;
  t.load(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = t.get(i);
}

template <typename T>
__device__ __forceinline__ void st8(T* p, const float (&v)[8]) {
  Vec8<T> t;
#pragma unroll
  for (int i = 0; i < 8; ++i) t.set(i, v[i]);
  t.store(p);
}

__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// a per-column parameter vector: fp32, or (pt != 0) in the activation dtype T -- bf16/fp16 gamma/beta
// are read as they are instead of through a conversion kernel per call
template <typename T>
__device__ __forceinline__ void ld8p(const void* p, int i8, int pt, float (&v)[8]) {
  if (pt) {
    Vec8<T> t;
    t.load(static_cast<const T*>(p) + i8);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = t.get(i);
  } else {
    ld8f(static_cast<const float*>(p) + i8, v);
  }
}

// ------------------------------------------------------------------ LayerNorm
// x, y: [M, D] (D % 8 == 0, D <= 512*VPL); gamma/beta fp32 [D]; mean/rstd fp32 [M]
template <typename T, int VPL>
__global__ void __launch_bounds__(256) layernorm_fwd_kernel(const T* __restrict__ x, const void* __restrict__ gamma,
                                                            const void* __restrict__ beta, int pt, T* __restrict__ y,
                                                            float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                            int M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nv = D >> 3;
  const T* xr = x + (int64_t)row * D;
  float v[VPL][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + j * 64;
    if (c < nv) {
      ld8(xr + c * 8, v[j]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[j][i];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[j][i] = 0.f;
    }
  }
  const float mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    if (lane + j * 64 < nv) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[j][i] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / D + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
  T* yr = y + (int64_t)row * D;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + j * 64;
    if (c < nv) {
      float g[8], b[8], o[8];
      ld8p<T>(gamma, c * 8, pt, g);
      ld8p<T>(beta, c * 8, pt, b);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[j][i] - mean) * rstd * g[i] + b[i];
      st8(yr + c * 8, o);
    }
  }
}

// dx = rstd * (dy*g - mean(dy*g) - xhat * mean(dy*g*xhat)); per-block partial dgamma/dbeta
template <typename T, int VPL>
__global__ void __launch_bounds__(256) layernorm_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                            const void* __restrict__ gamma, int pt,
                                                            const float* __restrict__ mean_in,
                                                            const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                            float* __restrict__ part, int M, int D) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int nv = D >> 3;
  float pg[VPL][8], pb[VPL][8];
#pragma unroll
  for (int j = 0; j < VPL; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) pg[j][i] = pb[j][i] = 0.f;
  for (int row = blockIdx.x * 4 + w; row < M; row += gridDim.x * 4) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    const T* xr = x + (int64_t)row * D;
    const T* dyr = dy + (int64_t)row * D;
    float xh[VPL][8], gd[VPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + j * 64;
      if (c < nv) {
        float xv[8], dv[8], g[8];
        ld8(xr + c * 8, xv);
        ld8(dyr + c * 8, dv);
        ld8p<T>(gamma, c * 8, pt, g);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xh[j][i] = (xv[i] - mean) * rstd;
          gd[j][i] = dv[i] * g[i];
          s1 += gd[j][i];
          s2 += gd[j][i] * xh[j][i];
          pg[j][i] += dv[i] * xh[j][i];
          pb[j][i] += dv[i];
        }
      }
    }
    const float m1 = wave_sum(s1) / D, m2 = wave_sum(s2) / D;
    T* dxr = dx + (int64_t)row * D;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + j * 64;
      if (c < nv) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = rstd * (gd[j][i] - m1 - xh[j][i] * m2);
        st8(dxr + c * 8, o);
      }
    }
  }
  // combine the 4 waves' column partials through LDS, one row of partials per block
  __shared__ float sh[2][4][512];  // [g|b][wave][column chunk of 512]
  float* pgo = part + (int64_t)blockIdx.x * 2 * D;
  for (int base = 0; base < D; base += 512) {
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + j * 64;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int col = c * 8 + i - base;
        if (c < nv && col >= 0 && col < 512) {
          sh[0][w][col] = pg[j][i];
          sh[1][w][col] = pb[j][i];
        }
      }
    }
    __syncthreads();
    for (int col = threadIdx.x; col < 512 && base + col < D; col += 256) {
      pgo[base + col] = sh[0][0][col] + sh[0][1][col] + sh[0][2][col] + sh[0][3][col];
      pgo[D + base + col] = sh[1][0][col] + sh[1][1][col] + sh[1][2][col] + sh[1][3][col];
    }
    __syncthreads();
  }
}

// out[c] (+)= sum_b part[b][c] for the 2*D columns (dgamma then dbeta):
// 8 columns x 32 row-groups per block (2*768 columns -> 192 blocks: the reduce of the 512 row partials
// covers the chip instead of 48 blocks), LDS combine of the 32 partial sums
template <typename TO>
__global__ void __launch_bounds__(256) column_sum_kernel(const float* __restrict__ part, int nb, int ncol,
                                                         TO* __restrict__ out0, TO* __restrict__ out1, int D,
                                                         int accum) {
  const int cl = threadIdx.x & 7, grp = threadIdx.x >> 3;
  const int col = blockIdx.x * 8 + cl;
  float s0 = 0.f, s1 = 0.f;
  if (col < ncol) {
    int b = grp;
    for (; b + 32 < nb; b += 64) {
      s0 += part[(int64_t)b * ncol + col];
      s1 += part[(int64_t)(b + 32) * ncol + col];
    }
    if (b < nb) s0 += part[(int64_t)b * ncol + col];
  }
  __shared__ float red[32][8];
  red[grp][cl] = s0 + s1;
  __syncthreads();
  if (grp == 0 && col < ncol) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 32; ++g) s += red[g][cl];
    TO* o = col < D ? out0 + col : out1 + (col - D);
    if (accum) s += static_cast<float>(*o);
    *o = static_cast<TO>(s);
  }
}

// ------------------------------------------------------------------ GELU (erf form)
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad_f(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

template <typename T, bool BWD>
__global__ void __launch_bounds__(256) gelu_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                   T* __restrict__ out, int64_t nvec) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float xv[8], o[8];
    ld8(x + v * 8, xv);
    if (BWD) {
      float d[8];
      ld8(dy + v * 8, d);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = d[i] * gelu_grad_f(xv[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = gelu_f(xv[i]);
    }
    st8(out + v * 8, o);
  }
}

// GELU backward over [M][N] rows that also leaves the column sums of dx -- the bias gradient of the Dense
// layer that produced x (BERT's FFN-1) -- as per-block partials part[blockIdx.x][N] (column_sum_partials
// finishes them): the bias-gradient pass re-reading dx is not run. Thread (ct, rl) owns the 8-column groups
// ct, ct + nt, ... and every RL-th row of the block (rows rl, rl + RL, ...), two rows of loads in flight;
// the RL row-lanes combine through LDS ([RL][N] fp32) before the block's partial row is written.
template <typename T>
__global__ void __launch_bounds__(1024) gelu_bwd_colpart_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                                T* __restrict__ dx, float* __restrict__ part, int M,
                                                                int N, int rpb, int nt, int RL) {
  extern __shared__ float gsh[];
  const int G = N / 8;
  const int ct = threadIdx.x % nt, rl = threadIdx.x / nt;
  const int r0 = blockIdx.x * rpb;
  const int r1 = r0 + rpb < M ? r0 + rpb : M;
  for (int g = ct; g < G; g += nt) {
    float s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = 0.f;
    int r = r0 + rl;
    for (; r + RL < r1; r += 2 * RL) {
      float xv[2][8], d[2][8];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t off = (int64_t)(r + u * RL) * N + g * 8;
        ld8(x + off, xv[u]);
        ld8(dy + off, d[u]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          o[i] = d[u][i] * gelu_grad_f(xv[u][i]);
          s[i] += o[i];
        }
        st8(dx + (int64_t)(r + u * RL) * N + g * 8, o);
      }
    }
    if (r < r1) {
      const int64_t off = (int64_t)r * N + g * 8;
      float xv[8], d[8], o[8];
      ld8(x + off, xv);
      ld8(dy + off, d);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        o[i] = d[i] * gelu_grad_f(xv[i]);
        s[i] += o[i];
      }
      st8(dx + off, o);
    }
    float* po = RL > 1 ? gsh + rl * N + g * 8 : part + (int64_t)blockIdx.x * N + g * 8;
    *reinterpret_cast<float4*>(po) = make_float4(s[0], s[1], s[2], s[3]);
    *reinterpret_cast<float4*>(po + 4) = make_float4(s[4], s[5], s[6], s[7]);
  }
  if (RL > 1) {
    __syncthreads();
    for (int c = threadIdx.x; c < N; c += blockDim.x) {
      float a = 0.f;
      for (int q = 0; q < RL; ++q) a += gsh[q * N + c];
      part[(int64_t)blockIdx.x * N + c] = a;
    }
  }
}

// ------------------------------------------------------------------ softmax (last axis)
// y = softmax(x * scale) (LOG: log_softmax); one wave per row, row in registers
template <typename T, int VPL, bool LOG>
__global__ void __launch_bounds__(256) softmax_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int M, int L,
                                                          float scale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nv = L >> 3;
  const T* xr = x + (int64_t)row * L;
  float v[VPL][8];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + j * 64;
    if (c < nv) {
      ld8(xr + c * 8, v[j]);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v[j][i] *= scale;
        mx = fmaxf(mx, v[j][i]);
      }
    }
  }
  mx = wave_max(mx);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    if (lane + j * 64 < nv) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v[j][i] -= mx;
        s += __expf(v[j][i]);
      }
    }
  }
  s = wave_sum(s);
  const float ls = __logf(s), inv = 1.f / s;
  T* yr = y + (int64_t)row * L;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + j * 64;
    if (c < nv) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = LOG ? v[j][i] - ls : __expf(v[j][i]) * inv;
      st8(yr + c * 8, o);
    }
  }
}

// softmax:     dx = scale * y * (dy - sum(dy*y))
// log_softmax: dx = scale * (dy - exp(y) * sum(dy))
template <typename T, int VPL, bool LOG>
__global__ void __launch_bounds__(256) softmax_bwd_kernel(const T* __restrict__ y, const T* __restrict__ dy,
                                                          T* __restrict__ dx, int M, int L, float scale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nv = L >> 3;
  const T* yr = y + (int64_t)row * L;
  const T* dr = dy + (int64_t)row * L;
  float yv[VPL][8], dv[VPL][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + j * 64;
    if (c < nv) {
      ld8(yr + c * 8, yv[j]);
      ld8(dr + c * 8, dv[j]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += LOG ? dv[j][i] : dv[j][i] * yv[j][i];
    }
  }
  s = wave_sum(s);
  T* xr = dx + (int64_t)row * L;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + j * 64;
    if (c < nv) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        o[i] = scale * (LOG ? dv[j][i] - __expf(yv[j][i]) * s : yv[j][i] * (dv[j][i] - s));
      st8(xr + c * 8, o);
    }
  }
}

// ------------------------------------------------------------------ dropout
struct Philox {
  // Philox-4x32-10 (Salmon et al., SC'11)
  static __device__ __forceinline__ uint4 run(uint4 ctr, uint2 key) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      const uint32_t lo0 = ctr.x * 0xD2511F53u, hi0 = __umulhi(ctr.x, 0xD2511F53u);
      const uint32_t lo1 = ctr.z * 0xCD9E8D57u, hi1 = __umulhi(ctr.z, 0xCD9E8D57u);
      ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
      key.x += 0x9E3779B9u;
      key.y += 0xBB67AE85u;
    }
    return ctr;
  }
};

// keep element with probability (1-p): y = x * keep / (1-p); mask byte per 8 elements
template <typename T>
__global__ void __launch_bounds__(256) dropout_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ mask, int64_t nvec, float p,
                                                          uint64_t seed, const uint64_t* __restrict__ seed_base) {
  // seed_base (optional, device): a per-replay counter so a HIP-graph-captured dropout draws fresh masks
  if (seed_base != nullptr) seed += seed_base[0] * 0x9E3779B97F4A7C15ull;
  const uint32_t thresh = (uint32_t)fminf(p * 4294967296.f, 4294967295.f);
  const float sc = p < 1.f ? 1.f / (1.f - p) : 0.f;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const uint4 r0 = Philox::run(make_uint4((uint32_t)v, (uint32_t)(v >> 32), 0u, 0u), key);
    const uint4 r1 = Philox::run(make_uint4((uint32_t)v, (uint32_t)(v >> 32), 1u, 0u), key);
    const uint32_t u[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    float xv[8], o[8];
    ld8(x + v * 8, xv);
    uint32_t bits = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool keep = u[i] >= thresh;
      bits |= (keep ? 1u : 0u) << i;
      o[i] = keep ? xv[i] * sc : 0.f;
    }
    st8(y + v * 8, o);
    mask[v] = (uint8_t)bits;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) dropout_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                          T* __restrict__ dx, int64_t nvec, float p) {
  const float sc = p < 1.f ? 1.f / (1.f - p) : 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float d[8], o[8];
    ld8(dy + v * 8, d);
    const uint32_t bits = mask[v];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = ((bits >> i) & 1u) ? d[i] * sc : 0.f;
    st8(dx + v * 8, o);
  }
}


// ------------------------------------------------------------------ residual + dropout + LayerNorm
// The post-LN transformer sub-layer tail  y = LayerNorm(x + dropout(h)):  one wave per row draws the
// dropout keep bits (the same Philox counters as dropout_fwd_kernel: one draw per 8-element vector),
// forms s = x + keep*h/(1-p) (kept, rounded to T, for the backward), normalises it and writes y -- the
// separate dropout, add and LayerNorm passes (and their launches) collapse into one read of x and h.
template <typename T, int VPL, bool DROP>
__global__ void __launch_bounds__(256) add_dropout_ln_fwd_kernel(
    const T* __restrict__ x, const T* __restrict__ h, const void* __restrict__ gamma, const void* __restrict__ beta,
    int pt, T* __restrict__ y, T* __restrict__ s_out, uint8_t* __restrict__ mask, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, int M, int D, float eps, float p, uint64_t seed,
    const uint64_t* __restrict__ seed_base) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nv = D >> 3;
  if (DROP && seed_base != nullptr) seed += seed_base[0] * 0x9E3779B97F4A7C15ull;
  const uint32_t thresh = (uint32_t)fminf(p * 4294967296.f, 4294967295.f);
  const float sc = p < 1.f ? 1.f / (1.f - p) : 0.f;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  const T* xr = x + (int64_t)row * D;
  const T* hr = h + (int64_t)row * D;
  T* sr = s_out + (int64_t)row * D;
  float v[VPL][8];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + j * 64;
    if (c < nv) {
      float xv[8], hv[8];
      ld8(xr + c * 8, xv);
      ld8(hr + c * 8, hv);
      if (DROP) {
        const int64_t vec = (int64_t)row * nv + c;
        const uint4 r0 = Philox::run(make_uint4((uint32_t)vec, (uint32_t)(vec >> 32), 0u, 0u), key);
        const uint4 r1 = Philox::run(make_uint4((uint32_t)vec, (uint32_t)(vec >> 32), 1u, 0u), key);
        const uint32_t u[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
        uint32_t bits = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const bool keep = u[i] >= thresh;
          bits |= (keep ? 1u : 0u) << i;
          hv[i] = keep ? hv[i] * sc : 0.f;
        }
        mask[vec] = (uint8_t)bits;
      }
      Vec8<T> t;
#pragma unroll
      for (int i = 0; i < 8; ++i) t.set(i, xv[i] + hv[i]);
      t.store(sr + c * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        v[j][i] = t.get(i);          // the rounded sum: what the backward re-reads
        sum += v[j][i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[j][i] = 0.f;
    }
  }
  const float mean = wave_sum(sum) / D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    if (lane + j * 64 < nv) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[j][i] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / D + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
  T* yr = y + (int64_t)row * D;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + j * 64;
    if (c < nv) {
      float g[8], b[8], o[8];
      ld8p<T>(gamma, c * 8, pt, g);
      ld8p<T>(beta, c * 8, pt, b);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[j][i] - mean) * rstd * g[i] + b[i];
      st8(yr + c * 8, o);
    }
  }
}

// its backward: ds = LayerNorm'(s) dy (the residual branch's gradient) and dh = keep * ds / (1-p) in one
// pass, with the dgamma / dbeta column partials of layernorm_bwd_kernel
template <typename T, int VPL, bool DROP>
__global__ void __launch_bounds__(256) add_dropout_ln_bwd_kernel(
    const T* __restrict__ x, const T* __restrict__ dy, const void* __restrict__ gamma, int pt,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, const uint8_t* __restrict__ mask, float p,
    T* __restrict__ dx, T* __restrict__ dh, float* __restrict__ part, float* __restrict__ hpart, int M, int D) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int nv = D >> 3;
  const float sc = p < 1.f ? 1.f / (1.f - p) : 0.f;
  // pg / pb: dgamma / dbeta column partials; ph (hpart != null): column sums of dh -- the bias gradient
  // of the layer that produced h, so that layer's backward needs no reduction pass of its own
  float pg[VPL][8], pb[VPL][8], ph[VPL][8];
#pragma unroll
  for (int j = 0; j < VPL; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) pg[j][i] = pb[j][i] = ph[j][i] = 0.f;
  for (int row = blockIdx.x * 4 + w; row < M; row += gridDim.x * 4) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    const T* xr = x + (int64_t)row * D;
    const T* dyr = dy + (int64_t)row * D;
    float xh[VPL][8], gd[VPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + j * 64;
      if (c < nv) {
        float xv[8], dv[8], g[8];
        ld8(xr + c * 8, xv);
        ld8(dyr + c * 8, dv);
        ld8p<T>(gamma, c * 8, pt, g);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xh[j][i] = (xv[i] - mean) * rstd;
          gd[j][i] = dv[i] * g[i];
          s1 += gd[j][i];
          s2 += gd[j][i] * xh[j][i];
          pg[j][i] += dv[i] * xh[j][i];
          pb[j][i] += dv[i];
        }
      }
    }
    const float m1 = wave_sum(s1) / D, m2 = wave_sum(s2) / D;
    T* dxr = dx + (int64_t)row * D;
    T* dhr = dh + (int64_t)row * D;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + j * 64;
      if (c < nv) {
        float o[8], oh[8];
        const uint32_t bits = DROP ? mask[(int64_t)row * nv + c] : 0xffu;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          o[i] = rstd * (gd[j][i] - m1 - xh[j][i] * m2);
          oh[i] = DROP ? (((bits >> i) & 1u) ? o[i] * sc : 0.f) : o[i];
        }
        st8(dxr + c * 8, o);
        // the sums use the stored (rounded) dh, as a separate reduction over dh would
        Vec8<T> th;
#pragma unroll
        for (int i = 0; i < 8; ++i) th.set(i, oh[i]);
        th.store(dhr + c * 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) ph[j][i] += th.get(i);
      }
    }
  }
  __shared__ float sh[3][4][512];
  float* pgo = part + (int64_t)blockIdx.x * 2 * D;
  float* pho = hpart != nullptr ? hpart + (int64_t)blockIdx.x * D : nullptr;
  for (int base = 0; base < D; base += 512) {
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + j * 64;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int col = c * 8 + i - base;
        if (c < nv && col >= 0 && col < 512) {
          sh[0][w][col] = pg[j][i];
          sh[1][w][col] = pb[j][i];
          sh[2][w][col] = ph[j][i];
        }
      }
    }
    __syncthreads();
    for (int col = threadIdx.x; col < 512 && base + col < D; col += 256) {
      pgo[base + col] = sh[0][0][col] + sh[0][1][col] + sh[0][2][col] + sh[0][3][col];
      pgo[D + base + col] = sh[1][0][col] + sh[1][1][col] + sh[1][2][col] + sh[1][3][col];
      if (pho != nullptr) pho[base + col] = sh[2][0][col] + sh[2][1][col] + sh[2][2][col] + sh[2][3][col];
    }
    __syncthreads();
  }
}

inline int ew_blocks(int64_t nvec) {
  int64_t b = (nvec + 255) / 256;
  return (int)(b > 256 * 16 ? 256 * 16 : (b < 1 ? 1 : b));
}

// rows of up to 512*VPL elements; VPL chosen from {1,2,4,8,16}
inline int pick_vpl(int D) {
  const int nv = D / 8;
  if (nv <= 64) return 1;
  if (nv <= 128) return 2;
  if (nv <= 256) return 4;
  if (nv <= 512) return 8;
  if (nv <= 1024) return 16;
  return 0;
}

#define MXAMD_VPL_SWITCH(vpl, ...)                                   \
  switch (vpl) {                                                     \
    case 1: { constexpr int VPL = 1; __VA_ARGS__; } break;           \
    case 2: { constexpr int VPL = 2; __VA_ARGS__; } break;           \
    case 4: { constexpr int VPL = 4; __VA_ARGS__; } break;           \
    case 8: { constexpr int VPL = 8; __VA_ARGS__; } break;           \
    case 16: { constexpr int VPL = 16; __VA_ARGS__; } break;         \
    default: throw std::runtime_error("row length must be a multiple of 8 and <= 8192"); \
  }

#define MXAMD_DTYPE_SWITCH(dtype, ...)                                \
  if (dtype == kF16) { typedef __half T; __VA_ARGS__; }               \
  else if (dtype == kBF16) { typedef __hip_bfloat16 T; __VA_ARGS__; } \
  else { typedef float T; __VA_ARGS__; }

}  // namespace

// blocks of the backward kernel (each loops over rows): enough to fill the chip, few partial rows
int layernorm_bwd_partials(int M) {
  int nb = (M + 3) / 4;
  return nb > 512 ? 512 : nb;
}

// pt: gamma / beta are in the activation dtype (else fp32)
void layernorm_forward(int dtype, const void* x, const void* gamma, const void* beta, int pt, void* y, float* mean,
                       float* rstd, int M, int D, float eps, hipStream_t s) {
  MXAMD_HOST_CHECK(D % 8 == 0, "layernorm: D must be a multiple of 8");
  const int vpl = pick_vpl(D);
  dim3 grid((M + 3) / 4);
  MXAMD_DTYPE_SWITCH(dtype, MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((layernorm_fwd_kernel<T, VPL>), grid, dim3(256),
                                                                     0, s, static_cast<const T*>(x), gamma, beta, pt,
                                                                     static_cast<T*>(y), mean, rstd, M, D, eps)))
}

// part: fp32 workspace of layernorm_bwd_partials(M) * 2 * D; dgamma/dbeta fp32 [D] (written or accumulated)
void layernorm_backward(int dtype, const void* x, const void* dy, const void* gamma, int pt, const float* mean,
                        const float* rstd, void* dx, float* part, void* dgamma, void* dbeta, int gdtype, int accum,
                        int M, int D, hipStream_t s) {
  MXAMD_HOST_CHECK(D % 8 == 0, "layernorm: D must be a multiple of 8");
  const int vpl = pick_vpl(D);
  const int nb = layernorm_bwd_partials(M);
  MXAMD_DTYPE_SWITCH(dtype, MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((layernorm_bwd_kernel<T, VPL>), dim3(nb),
                                                                     dim3(256), 0, s, static_cast<const T*>(x),
                                                                     static_cast<const T*>(dy), gamma, pt, mean, rstd,
                                                                     static_cast<T*>(dx), part, M, D)))
  // dgamma / dbeta straight into the parameters' gradient buffers in their own dtype (fp32 / bf16 / fp16)
  MXAMD_DTYPE_SWITCH(gdtype, hipLaunchKernelGGL((column_sum_kernel<T>), dim3((2 * D + 7) / 8), dim3(256), 0, s,
                                                part, nb, 2 * D, static_cast<T*>(dgamma), static_cast<T*>(dbeta), D,
                                                accum))
}


// y = LayerNorm(x + dropout_p(h)); s = x + dropout_p(h) (T), mask (1 bit per element, p > 0 only)
void add_dropout_ln_forward(int dtype, const void* x, const void* h, const void* gamma, const void* beta, int pt,
                            void* y, void* s_out, uint8_t* mask, float* mean, float* rstd, int M, int D, float eps,
                            float p, uint64_t seed, const uint64_t* seed_base, hipStream_t s) {
  MXAMD_HOST_CHECK(D % 8 == 0 && (dtype == kF16 || dtype == kBF16), "add_dropout_ln: D % 8 == 0, f16/bf16");
  MXAMD_HOST_CHECK(p == 0.f || mask != nullptr, "add_dropout_ln: dropout needs a mask buffer");
  const int vpl = pick_vpl(D);
  dim3 grid((M + 3) / 4);
  if (dtype == kF16) {
    typedef __half T;
    if (p > 0.f)
      MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((add_dropout_ln_fwd_kernel<T, VPL, true>), grid, dim3(256), 0, s,
                                               (const T*)x, (const T*)h, gamma, beta, pt, (T*)y, (T*)s_out, mask, mean,
                                               rstd, M, D, eps, p, seed, seed_base))
    else
      MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((add_dropout_ln_fwd_kernel<T, VPL, false>), grid, dim3(256), 0, s,
                                               (const T*)x, (const T*)h, gamma, beta, pt, (T*)y, (T*)s_out, mask, mean,
                                               rstd, M, D, eps, p, seed, seed_base))
  } else {
    typedef __hip_bfloat16 T;
    if (p > 0.f)
      MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((add_dropout_ln_fwd_kernel<T, VPL, true>), grid, dim3(256), 0, s,
                                               (const T*)x, (const T*)h, gamma, beta, pt, (T*)y, (T*)s_out, mask, mean,
                                               rstd, M, D, eps, p, seed, seed_base))
    else
      MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((add_dropout_ln_fwd_kernel<T, VPL, false>), grid, dim3(256), 0, s,
                                               (const T*)x, (const T*)h, gamma, beta, pt, (T*)y, (T*)s_out, mask, mean,
                                               rstd, M, D, eps, p, seed, seed_base))
  }
}

// ds (residual gradient) and dh (= dropout'(ds)) of add_dropout_ln_forward; dgamma / dbeta as layernorm_backward
void add_dropout_ln_backward(int dtype, const void* s_in, const void* dy, const void* gamma, int pt, const float* mean,
                             const float* rstd, const uint8_t* mask, float p, void* ds, void* dh, float* part,
                             float* hpart, void* dgamma, void* dbeta, int gdtype, int accum, int M, int D,
                             hipStream_t s) {
  MXAMD_HOST_CHECK(D % 8 == 0 && (dtype == kF16 || dtype == kBF16), "add_dropout_ln: D % 8 == 0, f16/bf16");
  const int vpl = pick_vpl(D);
  const int nb = layernorm_bwd_partials(M);
  if (dtype == kF16) {
    typedef __half T;
    if (p > 0.f)
      MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((add_dropout_ln_bwd_kernel<T, VPL, true>), dim3(nb), dim3(256), 0, s,
                                               (const T*)s_in, (const T*)dy, gamma, pt, mean, rstd, mask, p, (T*)ds,
                                               (T*)dh, part, hpart, M, D))
    else
      MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((add_dropout_ln_bwd_kernel<T, VPL, false>), dim3(nb), dim3(256), 0, s,
                                               (const T*)s_in, (const T*)dy, gamma, pt, mean, rstd, mask, p, (T*)ds,
                                               (T*)dh, part, hpart, M, D))
  } else {
    typedef __hip_bfloat16 T;
    if (p > 0.f)
      MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((add_dropout_ln_bwd_kernel<T, VPL, true>), dim3(nb), dim3(256), 0, s,
                                               (const T*)s_in, (const T*)dy, gamma, pt, mean, rstd, mask, p, (T*)ds,
                                               (T*)dh, part, hpart, M, D))
    else
      MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((add_dropout_ln_bwd_kernel<T, VPL, false>), dim3(nb), dim3(256), 0, s,
                                               (const T*)s_in, (const T*)dy, gamma, pt, mean, rstd, mask, p, (T*)ds,
                                               (T*)dh, part, hpart, M, D))
  }
  MXAMD_DTYPE_SWITCH(gdtype, hipLaunchKernelGGL((column_sum_kernel<T>), dim3((2 * D + 7) / 8), dim3(256), 0, s,
                                                part, nb, 2 * D, static_cast<T*>(dgamma), static_cast<T*>(dbeta), D,
                                                accum))
}

// out[c] (+)= sum_b part[b][c], c < ncol: the column partials an earlier kernel left (add_dropout_ln's dh sums)
void column_sum_partials(int gdtype, const float* part, int nb, int ncol, void* out, int accum, hipStream_t s) {
  MXAMD_DTYPE_SWITCH(gdtype, hipLaunchKernelGGL((column_sum_kernel<T>), dim3((ncol + 7) / 8), dim3(256), 0, s, part,
                                                nb, ncol, static_cast<T*>(out), static_cast<T*>(out), ncol, accum))
}

void gelu_forward(int dtype, const void* x, void* y, int64_t n, hipStream_t s) {
  MXAMD_HOST_CHECK(n % 8 == 0, "gelu: numel must be a multiple of 8");
  MXAMD_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((gelu_kernel<T, false>), dim3(ew_blocks(n / 8)), dim3(256), 0, s,
                                               static_cast<const T*>(x), nullptr, static_cast<T*>(y), n / 8))
}

// row blocks of gelu_backward_colpart for an [M][N] problem (= the partial rows it writes)
int gelu_colpart_blocks(int M, int N) {
  const int nb = M < 256 ? M : 256;
  return nb > 0 ? nb : 1;
}

void gelu_backward_colpart(int dtype, const void* x, const void* dy, void* dx, float* part, int M, int N,
                           hipStream_t s) {
  MXAMD_HOST_CHECK(M > 0 && N % 8 == 0 && (dtype == kF16 || dtype == kBF16), "gelu_backward_colpart: N % 8, f16/bf16");
  const int nb = gelu_colpart_blocks(M, N);
  const int rpb = (M + nb - 1) / nb;
  const int G = N / 8;
  // column threads: every 8-column group once, or a divisor of the group count near 256 (N = 3072: 384
  // groups -> 192 threads x 2) so no thread walks one group more than the others; row-lanes up to 768
  // threads per block (~12 waves per CU over the 256 blocks) while their [RL][N] LDS image fits 48 KB
  int nt = G;
  if (G > 256) {
    nt = 256;
    for (int c : {256, 192, 128}) {
      if (G % c == 0) {
        nt = c;
        break;
      }
    }
  }
  int RL = 768 / nt;
  if (RL > 8) RL = 8;
  if (RL > rpb) RL = rpb;
  if (RL > 12288 / N) RL = 12288 / N;
  if (RL < 1) RL = 1;
  const size_t lds = RL > 1 ? static_cast<size_t>(RL) * N * sizeof(float) : 0;
  MXAMD_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((gelu_bwd_colpart_kernel<T>), dim3(nb), dim3(nt * RL), lds, s,
                                               static_cast<const T*>(x), static_cast<const T*>(dy),
                                               static_cast<T*>(dx), part, M, N, rpb, nt, RL))
}

void gelu_backward(int dtype, const void* x, const void* dy, void* dx, int64_t n, hipStream_t s) {
  MXAMD_HOST_CHECK(n % 8 == 0, "gelu: numel must be a multiple of 8");
  MXAMD_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((gelu_kernel<T, true>), dim3(ew_blocks(n / 8)), dim3(256), 0, s,
                                               static_cast<const T*>(x), static_cast<const T*>(dy),
                                               static_cast<T*>(dx), n / 8))
}

void softmax_forward(int dtype, int log, const void* x, void* y, int M, int L, float scale, hipStream_t s) {
  MXAMD_HOST_CHECK(L % 8 == 0, "softmax: row length must be a multiple of 8");
  const int vpl = pick_vpl(L);
  dim3 grid((M + 3) / 4);
  if (log) {
    MXAMD_DTYPE_SWITCH(dtype, MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((softmax_fwd_kernel<T, VPL, true>), grid,
                                                                       dim3(256), 0, s, static_cast<const T*>(x),
                                                                       static_cast<T*>(y), M, L, scale)))
  } else {
    MXAMD_DTYPE_SWITCH(dtype, MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((softmax_fwd_kernel<T, VPL, false>), grid,
                                                                       dim3(256), 0, s, static_cast<const T*>(x),
                                                                       static_cast<T*>(y), M, L, scale)))
  }
}

void softmax_backward(int dtype, int log, const void* y, const void* dy, void* dx, int M, int L, float scale,
                      hipStream_t s) {
  MXAMD_HOST_CHECK(L % 8 == 0, "softmax: row length must be a multiple of 8");
  const int vpl = pick_vpl(L);
  dim3 grid((M + 3) / 4);
  if (log) {
    MXAMD_DTYPE_SWITCH(dtype, MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((softmax_bwd_kernel<T, VPL, true>), grid,
                                                                       dim3(256), 0, s, static_cast<const T*>(y),
                                                                       static_cast<const T*>(dy),
                                                                       static_cast<T*>(dx), M, L, scale)))
  } else {
    MXAMD_DTYPE_SWITCH(dtype, MXAMD_VPL_SWITCH(vpl, hipLaunchKernelGGL((softmax_bwd_kernel<T, VPL, false>), grid,
                                                                       dim3(256), 0, s, static_cast<const T*>(y),
                                                                       static_cast<const T*>(dy),
                                                                       static_cast<T*>(dx), M, L, scale)))
  }
}

void dropout_forward(int dtype, const void* x, void* y, uint8_t* mask, int64_t n, float p, uint64_t seed,
                     const uint64_t* seed_base, hipStream_t s) {
  MXAMD_HOST_CHECK(n % 8 == 0, "dropout: numel must be a multiple of 8");
  MXAMD_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((dropout_fwd_kernel<T>), dim3(ew_blocks(n / 8)), dim3(256), 0, s,
                                               static_cast<const T*>(x), static_cast<T*>(y), mask, n / 8, p, seed,
                                               seed_base))
}

void dropout_backward(int dtype, const void* dy, const uint8_t* mask, void* dx, int64_t n, float p, hipStream_t s) {
  MXAMD_HOST_CHECK(n % 8 == 0, "dropout: numel must be a multiple of 8");
  MXAMD_DTYPE_SWITCH(dtype, hipLaunchKernelGGL((dropout_bwd_kernel<T>), dim3(ew_blocks(n / 8)), dim3(256), 0, s,
                                               static_cast<const T*>(dy), mask, static_cast<T*>(dx), n / 8, p))
}

// ---------------------------------------------------------------- Embedding (gather / scatter-add)
// Index dtypes: 0 float32 (MXNet's default index arrays), 1 int64, 2 int32; indices are clamped to [0, V).
namespace {

template <typename I>
__device__ __forceinline__ int64_t emb_row(const void* idx, int64_t i, int V) {
  int64_t k = static_cast<int64_t>(static_cast<const I*>(idx)[i]);
  return k < 0 ? 0 : (k >= V ? V - 1 : k);
}

template <typename T, typename I>
__global__ void __launch_bounds__(256) embedding_fwd_kernel(const void* __restrict__ idx, const T* __restrict__ w,
                                                            T* __restrict__ y, int64_t n, int V, int C) {
  const int c8 = C / 8;
  const int64_t total = n * c8;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t row = t / c8;
    const int v = static_cast<int>(t - row * c8);
    Vec8<T> val;
    val.load(w + emb_row<I>(idx, row, V) * C + v * 8);
    val.store(y + row * C + v * 8);
  }
}

// acc[k] += dy[i] for every looked-up row k = idx[i] (fp32 hardware atomics), touched[k] = 1
template <typename T, typename I>
__global__ void __launch_bounds__(256) embedding_scatter_kernel(const void* __restrict__ idx,
                                                                const T* __restrict__ dy, float* __restrict__ acc,
                                                                uint8_t* __restrict__ touched, int64_t n, int V,
                                                                int C) {
  const int c8 = C / 8;
  const int64_t total = n * c8;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t row = t / c8;
    const int v = static_cast<int>(t - row * c8);
    const int64_t k = emb_row<I>(idx, row, V);
    Vec8<T> g;
    g.load(dy + row * C + v * 8);
    float* a = acc + k * C + v * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) unsafeAtomicAdd(a + j, g.get(j));
    if (v == 0) touched[k] = 1;
  }
}

// Small tables (V*C fp32 fits in LDS, e.g. BERT's 2-row token-type embedding): every block
// pre-reduces a chunk of rows in LDS and flushes one global atomic per non-zero entry, so thousands
// of lookups of the same few rows do not serialise on the same global addresses.
constexpr int kEmbSmallFloats = 16384;
template <typename T, typename I>
__global__ void __launch_bounds__(256) embedding_scatter_small_kernel(const void* __restrict__ idx,
                                                                      const T* __restrict__ dy,
                                                                      float* __restrict__ acc,
                                                                      uint8_t* __restrict__ touched, int64_t n,
                                                                      int V, int C, int64_t rows_per_block) {
  __shared__ float lds[kEmbSmallFloats];
  const int vc = V * C;
  for (int i = threadIdx.x; i < vc; i += 256) lds[i] = 0.f;
  __syncthreads();
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  int64_t r1 = r0 + rows_per_block;
  if (r1 > n) r1 = n;
  const int c8 = C / 8;
  const int64_t work = (r1 - r0) * c8;
  for (int64_t t = threadIdx.x; t < work; t += 256) {
    const int64_t row = r0 + t / c8;
    const int v = static_cast<int>(t % c8);
    const int64_t k = emb_row<I>(idx, row, V);
    Vec8<T> g;
    g.load(dy + row * C + v * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicAdd(&lds[k * C + v * 8 + j], g.get(j));
    if (v == 0) touched[k] = 1;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < vc; i += 256) {
    const float a = lds[i];
    if (a != 0.f) unsafeAtomicAdd(acc + i, a);
  }
}

// grad[k] (+)= acc[k] for touched rows (then acc[k] = 0, touched[k] = 0: the scratch is left all-zero
// for the next call); untouched rows are zero-filled unless accumulating.  One wave per row.
template <typename TO>
__global__ void __launch_bounds__(256) embedding_finalize_kernel(float* __restrict__ acc,
                                                                 uint8_t* __restrict__ touched,
                                                                 TO* __restrict__ grad, int V, int C, int accum) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (k >= V) return;
  const bool hit = touched[k] != 0;
  if (!hit && accum) return;
  const int c8 = C / 8;
  for (int v = lane; v < c8; v += 64) {
    Vec8<TO> out;
    float* a = acc + k * C + v * 8;
    if (accum) out.load(grad + k * C + v * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float add = hit ? a[j] : 0.f;
      out.set(j, (accum ? out.get(j) : 0.f) + add);
    }
    out.store(grad + k * C + v * 8);
    if (hit) {
      float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(a) = z;
      *reinterpret_cast<float4*>(a + 4) = z;
    }
  }
  if (hit && lane == 0) touched[k] = 0;
}

#define MXAMD_INDEX_SWITCH(itype, ...)                  \
  if (itype == 0) { typedef float I; __VA_ARGS__; }     \
  else if (itype == 1) { typedef int64_t I; __VA_ARGS__; } \
  else { typedef int32_t I; __VA_ARGS__; }

}  // namespace

void embedding_forward(int dtype, int itype, const void* idx, const void* w, void* y, int64_t n, int V, int C,
                       hipStream_t s) {
  MXAMD_HOST_CHECK(C % 8 == 0, "embedding: output_dim must be a multiple of 8");
  const int blocks = ew_blocks(n * (C / 8));
  MXAMD_DTYPE_SWITCH(dtype, MXAMD_INDEX_SWITCH(itype, hipLaunchKernelGGL((embedding_fwd_kernel<T, I>), dim3(blocks),
                                                                         dim3(256), 0, s, idx,
                                                                         static_cast<const T*>(w),
                                                                         static_cast<T*>(y), n, V, C)))
}

// acc: V*C fp32 and touched: V bytes, both all-zero on entry (and on exit)
void embedding_backward(int dtype, int itype, const void* idx, const void* dy, float* acc, uint8_t* touched,
                        int out_dtype, void* grad, int accum, int64_t n, int V, int C, hipStream_t s) {
  MXAMD_HOST_CHECK(C % 8 == 0, "embedding: output_dim must be a multiple of 8");
  static const bool small_ok = [] {
    const char* e = getenv("MXAMD_EMB_SMALL");
    return e == nullptr || e[0] != '0';
  }();
  if (small_ok && static_cast<int64_t>(V) * C <= kEmbSmallFloats) {
    int64_t rpb = 64;
    while ((n + rpb - 1) / rpb > 512) rpb *= 2;
    const int blocks = static_cast<int>((n + rpb - 1) / rpb);
    MXAMD_DTYPE_SWITCH(dtype, MXAMD_INDEX_SWITCH(itype, hipLaunchKernelGGL((embedding_scatter_small_kernel<T, I>),
                                                                           dim3(blocks), dim3(256), 0, s, idx,
                                                                           static_cast<const T*>(dy), acc, touched,
                                                                           n, V, C, rpb)))
  } else {
    const int blocks = ew_blocks(n * (C / 8));
    MXAMD_DTYPE_SWITCH(dtype, MXAMD_INDEX_SWITCH(itype, hipLaunchKernelGGL((embedding_scatter_kernel<T, I>),
                                                                           dim3(blocks), dim3(256), 0, s, idx,
                                                                           static_cast<const T*>(dy), acc, touched,
                                                                           n, V, C)))
  }
  const dim3 grid((V + 3) / 4);
  MXAMD_DTYPE_SWITCH(out_dtype, hipLaunchKernelGGL((embedding_finalize_kernel<T>), grid, dim3(256), 0, s, acc,
                                                   touched, static_cast<T*>(grad), V, C, accum))
}

}  // namespace mxamd
