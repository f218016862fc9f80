// Softmax cross-entropy, global average pooling (NHWC) and the fused flat
// multi-precision SGD update for gfx950.
//
// Parity: src/operator/nn/softmax.cu + loss (SoftmaxCrossEntropyLoss /
// softmax_cross_entropy), src/operator/nn/pooling.cu (global avg pool),
// src/operator/optimizer_op.cu (mp_sgd_mom_update / multi_mp_sgd_mom_update).
#include <stdexcept>

#include "common.h"

namespace mxamd {

// --------------------------------------------------------------------------
// softmax cross entropy: one wave per row, fp32 math, loss and logsumexp out
// --------------------------------------------------------------------------
template <typename T, typename L>
__global__ void __launch_bounds__(256) softmax_ce_fwd_kernel(const T* __restrict__ logits,
                                                             const L* __restrict__ label, float* __restrict__ loss,
                                                             float* __restrict__ lse, int N, int K) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int lane = threadIdx.x % kWave;
  if (wave >= N) return;
  const T* row = logits + static_cast<int64_t>(wave) * K;
  float m = -INFINITY;
  for (int k = lane; k < K; k += kWave) m = fmaxf(m, static_cast<float>(row[k]));
  m = wave_max(m);
  float s = 0.f;
  for (int k = lane; k < K; k += kWave) s += __expf(static_cast<float>(row[k]) - m);
  s = wave_sum(s);
  if (lane == 0) {
    int lab = static_cast<int>(label[wave]);
    lab = lab < 0 ? 0 : (lab >= K ? K - 1 : lab);
    const float l = logf(s) + m;
    lse[wave] = l;
    loss[wave] = l - static_cast<float>(row[lab]);
  }
}

template <typename T, typename L>
__global__ void __launch_bounds__(256) softmax_ce_bwd_kernel(const T* __restrict__ logits,
                                                             const L* __restrict__ label,
                                                             const float* __restrict__ lse,
                                                             const float* __restrict__ gout, T* __restrict__ dlogits,
                                                             int N, int K) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int lane = threadIdx.x % kWave;
  if (wave >= N) return;
  const int64_t base = static_cast<int64_t>(wave) * K;
  const float l = lse[wave];
  const float g = gout[wave];
  int lab = static_cast<int>(label[wave]);
  lab = lab < 0 ? 0 : (lab >= K ? K - 1 : lab);
  for (int k = lane; k < K; k += kWave) {
    float p = __expf(static_cast<float>(logits[base + k]) - l);
    if (k == lab) p -= 1.f;
    dlogits[base + k] = static_cast<T>(p * g);
  }
}

// --------------------------------------------------------------------------
// global average pooling, NHWC: out[n, c] = mean_hw x[n, hw, c]
// --------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) gap_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int HW, int C) {
  // block: one image n, 256 threads cover 256*8 channels; loop rows of HW
  const int n = blockIdx.y;
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c0 >= C) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const T* base = x + static_cast<int64_t>(n) * HW * C + c0;
  for (int r = 0; r < HW; ++r) {
    Vec8<T> v;
    v.load(base + static_cast<int64_t>(r) * C);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += v.get(i);
  }
  Vec8<T> o;
  const float inv = 1.f / HW;
#pragma unroll
  for (int i = 0; i < 8; ++i) o.set(i, acc[i] * inv);
  o.store(y + static_cast<int64_t>(n) * C + c0);
}

template <typename T>
__global__ void __launch_bounds__(256) gap_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int HW, int C,
                                                      int64_t nvec) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const float inv = 1.f / HW;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int64_t off = v * 8;
    const int64_t c = off % C;
    const int64_t n = off / (static_cast<int64_t>(HW) * C);
    Vec8<T> g, o;
    g.load(dy + n * C + c);
#pragma unroll
    for (int i = 0; i < 8; ++i) o.set(i, g.get(i) * inv);
    o.store(dx + off);
  }
}

// --------------------------------------------------------------------------
// flat multi-precision SGD with momentum (one pass over the arena)
//   g = clip(rescale * grad) + wd * w32 ; mom = momentum * mom - lr * g ; w32 += mom ; w = w32
// --------------------------------------------------------------------------
template <typename T, bool MP, bool MOM>
__global__ void __launch_bounds__(256) flat_sgd_kernel(T* __restrict__ w, const T* __restrict__ grad,
                                                       float* __restrict__ mom, float* __restrict__ w32,
                                                       int64_t nvec, float lr, float wd, float momentum,
                                                       float rescale, float clip, const float* __restrict__ hp) {
  // hp (optional, device): per-step hyper-parameters written before a HIP-graph replay; hp[0] = lr
  if (hp != nullptr) lr = hp[0];
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const int64_t off = v * 8;
    Vec8<T> vw, vg;
    vg.load(grad + off);
    float master[8];
    if (MP) {
      const float4 a = *reinterpret_cast<const float4*>(w32 + off);
      const float4 b = *reinterpret_cast<const float4*>(w32 + off + 4);
      master[0] = a.x; master[1] = a.y; master[2] = a.z; master[3] = a.w;
      master[4] = b.x; master[5] = b.y; master[6] = b.z; master[7] = b.w;
    } else {
      vw.load(w + off);
#pragma unroll
      for (int i = 0; i < 8; ++i) master[i] = vw.get(i);
    }
    float m[8];
    if (MOM) {
      const float4 a = *reinterpret_cast<const float4*>(mom + off);
      const float4 b = *reinterpret_cast<const float4*>(mom + off + 4);
      m[0] = a.x; m[1] = a.y; m[2] = a.z; m[3] = a.w;
      m[4] = b.x; m[5] = b.y; m[6] = b.z; m[7] = b.w;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float g = vg.get(i) * rescale;
      if (clip >= 0.f) g = fminf(fmaxf(g, -clip), clip);
      g += wd * master[i];
      if (MOM) {
        m[i] = momentum * m[i] - lr * g;
        master[i] += m[i];
      } else {
        master[i] -= lr * g;
      }
      vw.set(i, master[i]);
    }
    if (MOM) {
      *reinterpret_cast<float4*>(mom + off) = make_float4(m[0], m[1], m[2], m[3]);
      *reinterpret_cast<float4*>(mom + off + 4) = make_float4(m[4], m[5], m[6], m[7]);
    }
    if (MP) {
      *reinterpret_cast<float4*>(w32 + off) = make_float4(master[0], master[1], master[2], master[3]);
      *reinterpret_cast<float4*>(w32 + off + 4) = make_float4(master[4], master[5], master[6], master[7]);
    }
    vw.store(w + off);
  }
}

// ------------------------------------------------------------------ launchers

void softmax_ce_forward(int dtype, int label_is_int, const void* logits, const void* label, float* loss, float* lse,
                        int N, int K, hipStream_t s) {
  dim3 grid((N + 3) / 4), block(256);
#define L(T, LT) hipLaunchKernelGGL((softmax_ce_fwd_kernel<T, LT>), grid, block, 0, s, static_cast<const T*>(logits), \
                                    static_cast<const LT*>(label), loss, lse, N, K)
  if (dtype == kF16) {
    if (label_is_int) L(__half, int64_t); else L(__half, float);
  } else if (dtype == kBF16) {
    if (label_is_int) L(__hip_bfloat16, int64_t); else L(__hip_bfloat16, float);
  } else {
    if (label_is_int) L(float, int64_t); else L(float, float);
  }
#undef L
}

void softmax_ce_backward(int dtype, int label_is_int, const void* logits, const void* label, const float* lse,
                         const float* gout, void* dlogits, int N, int K, hipStream_t s) {
  dim3 grid((N + 3) / 4), block(256);
#define L(T, LT) hipLaunchKernelGGL((softmax_ce_bwd_kernel<T, LT>), grid, block, 0, s, static_cast<const T*>(logits), \
                                    static_cast<const LT*>(label), lse, gout, static_cast<T*>(dlogits), N, K)
  if (dtype == kF16) {
    if (label_is_int) L(__half, int64_t); else L(__half, float);
  } else if (dtype == kBF16) {
    if (label_is_int) L(__hip_bfloat16, int64_t); else L(__hip_bfloat16, float);
  } else {
    if (label_is_int) L(float, int64_t); else L(float, float);
  }
#undef L
}

void gap_nhwc_forward(int dtype, const void* x, void* y, int N, int HW, int C, hipStream_t s) {
  MXAMD_HOST_CHECK(C % 8 == 0, "gap_nhwc: C must be a multiple of 8");
  dim3 grid((C / 8 + 255) / 256, N), block(256);
  if (dtype == kF16)
    hipLaunchKernelGGL((gap_fwd_kernel<__half>), grid, block, 0, s, static_cast<const __half*>(x),
                       static_cast<__half*>(y), HW, C);
  else if (dtype == kBF16)
    hipLaunchKernelGGL((gap_fwd_kernel<__hip_bfloat16>), grid, block, 0, s,
                       static_cast<const __hip_bfloat16*>(x), static_cast<__hip_bfloat16*>(y), HW, C);
  else
    hipLaunchKernelGGL((gap_fwd_kernel<float>), grid, block, 0, s, static_cast<const float*>(x),
                       static_cast<float*>(y), HW, C);
}

void gap_nhwc_backward(int dtype, const void* dy, void* dx, int N, int HW, int C, hipStream_t s) {
  const int64_t nvec = static_cast<int64_t>(N) * HW * C / 8;
  int blocks = static_cast<int>((nvec + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  if (dtype == kF16)
    hipLaunchKernelGGL((gap_bwd_kernel<__half>), dim3(blocks), dim3(256), 0, s, static_cast<const __half*>(dy),
                       static_cast<__half*>(dx), HW, C, nvec);
  else if (dtype == kBF16)
    hipLaunchKernelGGL((gap_bwd_kernel<__hip_bfloat16>), dim3(blocks), dim3(256), 0, s,
                       static_cast<const __hip_bfloat16*>(dy), static_cast<__hip_bfloat16*>(dx), HW, C, nvec);
  else
    hipLaunchKernelGGL((gap_bwd_kernel<float>), dim3(blocks), dim3(256), 0, s, static_cast<const float*>(dy),
                       static_cast<float*>(dx), HW, C, nvec);
}

void flat_sgd(int dtype, void* w, const void* g, float* mom, float* w32, int64_t n, float lr, float wd,
              float momentum, float rescale, float clip, const float* hp, hipStream_t s) {
  MXAMD_HOST_CHECK(n % 8 == 0, "flat_sgd: arena length must be a multiple of 8");
  const int64_t nvec = n / 8;
  int blocks = static_cast<int>((nvec + 255) / 256);
  if (blocks > 8192) blocks = 8192;
#define L(T, MP, MOM) hipLaunchKernelGGL((flat_sgd_kernel<T, MP, MOM>), dim3(blocks), dim3(256), 0, s, \
                                         static_cast<T*>(w), static_cast<const T*>(g), mom, w32, nvec, lr, wd, \
                                         momentum, rescale, clip, hp)
#define DISPATCH(T)                           \
  if (w32) {                                  \
    if (mom) L(T, true, true); else L(T, true, false);   \
  } else {                                    \
    if (mom) L(T, false, true); else L(T, false, false); \
  }
  if (dtype == kF16) {
    DISPATCH(__half)
  } else if (dtype == kBF16) {
    DISPATCH(__hip_bfloat16)
  } else {
    DISPATCH(float)
  }
#undef DISPATCH
#undef L
}

// --------------------------------------------------------------------------
// 2-bit gradient compression with error feedback (parity: src/kvstore/
// gradient_compression-inl.h quantize_2bit / dequantize_2bit).  Code per
// element: 3 = +threshold, 2 = -threshold, 0 = zero; 4 codes per byte, element
// 4j+k at bits 2k of byte j.  One thread quantises 16 elements into one 32-bit
// word; the decode kernel sums the codes of all ranks (the all-gathered
// buffer) in one pass.
// --------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) twobit_quantize_kernel(const T* __restrict__ g, float* __restrict__ res,
                                                              uint32_t* __restrict__ packed, int64_t n, float thr) {
  const int64_t w = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t base = w * 16;
  if (base >= n) return;
  uint32_t word = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int64_t i = base + k;
    if (i < n) {
      float r = res[i] + static_cast<float>(g[i]);
      uint32_t code = 0;
      if (r >= thr) { code = 3; r -= thr; }
      else if (r <= -thr) { code = 2; r += thr; }
      res[i] = r;
      word |= code << (2 * k);
    }
  }
  packed[w] = word;
}

__global__ void __launch_bounds__(256) twobit_dequantize_sum_kernel(const uint8_t* __restrict__ packed,
                                                                    int64_t row_bytes, int nrows, int64_t n,
                                                                    float thr, float* __restrict__ out) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;   // byte index
  if (j * 4 >= n) return;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < nrows; ++r) {
    const uint32_t b = packed[r * row_bytes + j];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t c = (b >> (2 * k)) & 3u;
      acc[k] += c == 3u ? thr : (c == 2u ? -thr : 0.f);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (j * 4 + k < n) out[j * 4 + k] = acc[k];
}

void twobit_quantize(int dtype, const void* g, float* res, void* packed, int64_t n, float thr, hipStream_t s) {
  MXAMD_HOST_CHECK((reinterpret_cast<uintptr_t>(packed) & 3) == 0, "twobit_quantize: packed must be 4-byte aligned");
  const unsigned blocks = static_cast<unsigned>(((n + 15) / 16 + 255) / 256);
  uint32_t* p = static_cast<uint32_t*>(packed);
  if (dtype == kF32) twobit_quantize_kernel<float><<<blocks, 256, 0, s>>>(static_cast<const float*>(g), res, p, n, thr);
  else if (dtype == kF16)
    twobit_quantize_kernel<__half><<<blocks, 256, 0, s>>>(static_cast<const __half*>(g), res, p, n, thr);
  else twobit_quantize_kernel<__hip_bfloat16><<<blocks, 256, 0, s>>>(static_cast<const __hip_bfloat16*>(g), res, p, n,
                                                                      thr);
}

void twobit_dequantize_sum(const void* packed, int64_t row_bytes, int nrows, int64_t n, float thr, float* out,
                           hipStream_t s) {
  MXAMD_HOST_CHECK(row_bytes * 4 >= n && nrows >= 1, "twobit_dequantize_sum: row too short");
  const unsigned blocks = static_cast<unsigned>(((n + 3) / 4 + 255) / 256);
  twobit_dequantize_sum_kernel<<<blocks, 256, 0, s>>>(static_cast<const uint8_t*>(packed), row_bytes, nrows, n, thr,
                                                      out);
}

}  // namespace mxamd
