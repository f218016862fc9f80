// Shared helpers for the gfx950 (CDNA4, MI355X) kernels.
#pragma once
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MXAMD_HOST_CHECK(cond, msg)                 \
  do {                                              \
    if (!(cond)) throw std::runtime_error(msg);     \
  } while (0)

namespace mxamd {

constexpr int kWave = 64;  // CDNA wavefront width

enum DType : int { kF32 = 0, kF16 = 1, kBF16 = 2 };

// 8 elements of T packed in 16 bytes (or 32 bytes for fp32, loaded as 2x uint4)
template <typename T>
struct Vec8;

template <>
struct Vec8<__half> {
  uint4 raw;
  __device__ __forceinline__ void load(const __half* p) { raw = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void store(__half* p) const { *reinterpret_cast<uint4*>(p) = raw; }
  __device__ __forceinline__ float get(int i) const {
    const __half* h = reinterpret_cast<const __half*>(&raw);
    return __half2float(h[i]);
  }
  __device__ __forceinline__ void set(int i, float v) {
    __half* h = reinterpret_cast<__half*>(&raw);
    h[i] = __float2half(v);
  }
};

template <>
struct Vec8<__hip_bfloat16> {
  uint4 raw;
  __device__ __forceinline__ void load(const __hip_bfloat16* p) { raw = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void store(__hip_bfloat16* p) const { *reinterpret_cast<uint4*>(p) = raw; }
  __device__ __forceinline__ float get(int i) const {
    const uint16_t* h = reinterpret_cast<const uint16_t*>(&raw);
    return __uint_as_float(static_cast<uint32_t>(h[i]) << 16);
  }
  __device__ __forceinline__ void set(int i, float v) {
    __hip_bfloat16 b = __float2bfloat16(v);
    reinterpret_cast<__hip_bfloat16*>(&raw)[i] = b;
  }
};

template <>
struct Vec8<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const float4*>(p);
    b = *reinterpret_cast<const float4*>(p + 4);
  }
  __device__ __forceinline__ void store(float* p) const {
    *reinterpret_cast<float4*>(p) = a;
    *reinterpret_cast<float4*>(p + 4) = b;
  }
  __device__ __forceinline__ float get(int i) const {
    const float* f = reinterpret_cast<const float*>(this);
    return f[i];
  }
  __device__ __forceinline__ void set(int i, float v) { reinterpret_cast<float*>(this)[i] = v; }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

}  // namespace mxamd
