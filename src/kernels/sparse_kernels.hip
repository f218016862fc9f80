// Compressed-sparse kernels for gfx950 (CSR x dense products).
//
// Parity: src/operator/tensor/dot-inl.h (DotCsrDnsDnsImpl: out = csr . dns,
// DotCsrDnsRspImpl: out = csr^T . dns as a row_sparse array) and
// src/operator/tensor/dot-inl.cuh.
//
// Design (memory-bound, irregular): one 64-lane wave per CSR row.  The row's
// (column, value) pairs are wave-uniform, so every lane walks the same list
// while the lanes stride over the dense operand's columns -- each dense row is
// read with fully coalesced 64-wide accesses and accumulated in fp32
// registers (4 column slots per lane: N <= 256 in one pass, more in chunks).
//   dot(csr, dns)   : lanes own output columns -> plain vector stores.
//   dot(csr^T, dns) : output row = compact slot of the column id (a [K] ->
//                     slot table built on the host side from the unique
//                     column ids); contributions from different CSR rows meet
//                     in fp32 hardware atomics (global_atomic_add_f32).
#include <stdexcept>

#include "common.h"

namespace mxamd {
namespace {

template <typename T>
__device__ __forceinline__ float ld(const T* p) {
  return static_cast<float>(*p);
}
template <>
__device__ __forceinline__ float ld<__hip_bfloat16>(const __hip_bfloat16* p) {
  return __bfloat162float(*p);
}

constexpr int kSlots = 4;   // column slots per lane and pass

template <typename T>
__global__ void __launch_bounds__(256) csr_dns_kernel(const int64_t* __restrict__ indptr,
                                                      const int64_t* __restrict__ indices,
                                                      const T* __restrict__ vals, const T* __restrict__ rhs,
                                                      T* __restrict__ out, int64_t M, int64_t K, int N) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const int64_t j0 = indptr[row], j1 = indptr[row + 1];
  for (int c0 = 0; c0 < N; c0 += 64 * kSlots) {
    float acc[kSlots];
#pragma unroll
    for (int s = 0; s < kSlots; ++s) acc[s] = 0.f;
    for (int64_t j = j0; j < j1; ++j) {
      int64_t k = indices[j];
      if (k < 0 || k >= K) continue;   // malformed ids contribute nothing
      const float v = ld(vals + j);
      const T* r = rhs + k * N;
#pragma unroll
      for (int s = 0; s < kSlots; ++s) {
        const int c = c0 + s * 64 + lane;
        if (c < N) acc[s] = fmaf(v, ld(r + c), acc[s]);
      }
    }
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      const int c = c0 + s * 64 + lane;
      if (c < N) out[row * N + c] = static_cast<T>(acc[s]);
    }
  }
}

// out32[slot[k]] += v * rhs[row]  for every stored (row, k, v)
template <typename T>
__global__ void __launch_bounds__(256) csrT_dns_kernel(const int64_t* __restrict__ indptr,
                                                       const int64_t* __restrict__ indices,
                                                       const T* __restrict__ vals, const T* __restrict__ rhs,
                                                       const int64_t* __restrict__ slot, float* __restrict__ out32,
                                                       int64_t M, int64_t K, int N) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const int64_t j0 = indptr[row], j1 = indptr[row + 1];
  const T* r = rhs + row * N;
  for (int c0 = 0; c0 < N; c0 += 64 * kSlots) {
    float x[kSlots];
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      const int c = c0 + s * 64 + lane;
      x[s] = c < N ? ld(r + c) : 0.f;
    }
    for (int64_t j = j0; j < j1; ++j) {
      const int64_t k = indices[j];
      if (k < 0 || k >= K) continue;
      const int64_t o = slot[k];
      if (o < 0) continue;
      const float v = ld(vals + j);
      float* dst = out32 + o * N;
#pragma unroll
      for (int s = 0; s < kSlots; ++s) {
        const int c = c0 + s * 64 + lane;
        if (c < N) unsafeAtomicAdd(dst + c, v * x[s]);
      }
    }
  }
}

#define MXAMD_SPARSE_SWITCH(dtype, ...)                               \
  if (dtype == kF16) { typedef __half T; __VA_ARGS__; }               \
  else if (dtype == kBF16) { typedef __hip_bfloat16 T; __VA_ARGS__; } \
  else { typedef float T; __VA_ARGS__; }

}  // namespace

void csr_dot_dense(int dtype, const int64_t* indptr, const int64_t* indices, const void* vals, const void* rhs,
                   void* out, int64_t M, int64_t K, int N, hipStream_t s) {
  if (M == 0 || N == 0) return;
  const dim3 grid(static_cast<unsigned>((M + 3) / 4));
  MXAMD_SPARSE_SWITCH(dtype, hipLaunchKernelGGL((csr_dns_kernel<T>), grid, dim3(256), 0, s, indptr, indices,
                                                static_cast<const T*>(vals), static_cast<const T*>(rhs),
                                                static_cast<T*>(out), M, K, N))
}

void csrT_dot_dense(int dtype, const int64_t* indptr, const int64_t* indices, const void* vals, const void* rhs,
                    const int64_t* slot, float* out32, int64_t M, int64_t K, int N, hipStream_t s) {
  if (M == 0 || N == 0) return;
  const dim3 grid(static_cast<unsigned>((M + 3) / 4));
  MXAMD_SPARSE_SWITCH(dtype, hipLaunchKernelGGL((csrT_dns_kernel<T>), grid, dim3(256), 0, s, indptr, indices,
                                                static_cast<const T*>(vals), static_cast<const T*>(rhs), slot,
                                                out32, M, K, N))
}

}  // namespace mxamd
