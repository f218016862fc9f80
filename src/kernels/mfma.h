// The CDNA4 matrix-core primitives every MFMA kernel in this directory builds on, in one place:
// v_mfma_f32_16x16x32_{f16,bf16} (run) and v_mfma_f32_32x32x16_{f16,bf16} (run32) on 16-byte A/B
// fragments (8 x 16-bit values per lane, any 16-byte vector type) and the fp32 -> fp16/bf16 packs of
// the epilogues (round-to-nearest-even; bf16 through the hardware convert, so NaN stays NaN).
//
// Fragment maps (lane l):
//   16x16x32: A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15]; C/D col l&15, row 4(l>>4)+reg (reg 0..3)
//   32x32x16: A[row l&31][k 8(l>>5)+j], B[k 8(l>>5)+j][col l&31]; C/D col l&31,
//             row (reg&3) + 8(reg>>2) + 4(l>>5) (reg 0..15)
// Same MACs per cycle; the 32x32 shape needs half the fragment registers per MAC of a square wave tile
// and one 32-row fragment covers what two 16-row ones do.
#pragma once

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mxamd {
namespace mfma {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16x __attribute__((ext_vector_type(16)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));

template <typename T>
struct Op;

template <>
struct Op<__half> {
  template <typename V>
  static __device__ __forceinline__ f4 run(const V& a, const V& b, f4 c) {
    static_assert(sizeof(V) == 16, "MFMA A/B fragments are 16 bytes per lane");
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
  }
  template <typename V>
  static __device__ __forceinline__ f16x run32(const V& a, const V& b, f16x c) {
    static_assert(sizeof(V) == 16, "MFMA A/B fragments are 16 bytes per lane");
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
  }
  static __device__ __forceinline__ uint32_t two(float a, float b) {
    return __builtin_bit_cast(uint32_t, __floats2half2_rn(a, b));
  }
  static __device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
    return uint2{two(a, b), two(c, d)};
  }
  static __device__ __forceinline__ float4 unpack4(uint2 v) {
    const float2 a = __half22float2(__builtin_bit_cast(__half2, v.x));
    const float2 b = __half22float2(__builtin_bit_cast(__half2, v.y));
    return make_float4(a.x, a.y, b.x, b.y);
  }
};

template <>
struct Op<__hip_bfloat16> {
  template <typename V>
  static __device__ __forceinline__ f4 run(const V& a, const V& b, f4 c) {
    static_assert(sizeof(V) == 16, "MFMA A/B fragments are 16 bytes per lane");
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), c, 0, 0, 0);
  }
  template <typename V>
  static __device__ __forceinline__ f16x run32(const V& a, const V& b, f16x c) {
    static_assert(sizeof(V) == 16, "MFMA A/B fragments are 16 bytes per lane");
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), c, 0, 0, 0);
  }
  static __device__ __forceinline__ uint32_t two(float a, float b) {
    return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, __float2bfloat16(a))) |
           (static_cast<uint32_t>(__builtin_bit_cast(uint16_t, __float2bfloat16(b))) << 16);
  }
  static __device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
    return uint2{two(a, b), two(c, d)};
  }
  static __device__ __forceinline__ float4 unpack4(uint2 v) {
    return make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
                       __uint_as_float(v.y & 0xffff0000u));
  }
};

}  // namespace mfma
}  // namespace mxamd
