// Element-wise kernels for gfx950: ReLU forward/backward and broadcasting binary arithmetic.
//
// Parity: src/operator/tensor/elemwise_unary_op_basic.cc (relu, _backward_relu) and
// src/operator/tensor/elemwise_binary_broadcast_op_basic.cc (broadcast_add/sub/mul/div/maximum/minimum,
// elemwise_* as the equal-shape case).
//
// Memory-bound: every lane moves 16 bytes per access (8 x fp16/bf16 or 4 x fp32) and the grid is
// sized to keep 8 workgroups per CU resident.  The broadcast kernel recognises the two layouts that
// carry nearly all of the traffic -- equal shapes and a "row" operand repeated along the leading
// axes (bias over NHWC / [tokens, hidden]) -- and vectorises them; every other broadcast runs the
// general strided kernel (up to 6 dimensions, one element per lane).
#include <stdexcept>

#include "common.h"

namespace mxamd {

namespace {

constexpr int kPwThreads = 256;
constexpr int kPwMaxDims = 6;

enum PwOp { kAdd = 0, kSub = 1, kMul = 2, kDiv = 3, kMax = 4, kMin = 5 };

template <int OP>
__device__ __forceinline__ float pw_apply(float a, float b) {
  if (OP == kAdd) return a + b;
  if (OP == kSub) return a - b;
  if (OP == kMul) return a * b;
  if (OP == kDiv) return a / b;
  if (OP == kMax) return a >= b ? a : b;
  return a <= b ? a : b;
}

// elements per 16-byte vector
template <typename T>
struct PwVec {
  static constexpr int N = 16 / sizeof(T);
};

template <typename T>
__device__ __forceinline__ float to_f(T v) {
  return static_cast<float>(v);
}
template <>
__device__ __forceinline__ float to_f<__half>(__half v) {
  return __half2float(v);
}
template <>
__device__ __forceinline__ float to_f<__hip_bfloat16>(__hip_bfloat16 v) {
  return __bfloat162float(v);
}

template <typename T>
__device__ __forceinline__ T from_f(float v) {
  return static_cast<T>(v);
}
template <>
__device__ __forceinline__ __half from_f<__half>(float v) {
  return __float2half(v);
}
template <>
__device__ __forceinline__ __hip_bfloat16 from_f<__hip_bfloat16>(float v) {
  return __float2bfloat16(v);
}

template <typename T>
union PwPack {
  uint4 raw;
  T e[PwVec<T>::N];
};

inline unsigned pw_blocks(int64_t work) {
  int64_t b = (work + kPwThreads - 1) / kPwThreads;
  if (b > 256 * 8 * 4) b = 256 * 8 * 4;   // grid-stride beyond 4 rounds of full residency
  return static_cast<unsigned>(b < 1 ? 1 : b);
}

// ------------------------------------------------------------------------------------- relu
template <typename T>
__global__ void __launch_bounds__(kPwThreads) relu_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n) {
  constexpr int V = PwVec<T>::N;
  const int64_t nv = n / V;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kPwThreads;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kPwThreads + threadIdx.x; i < nv; i += stride) {
    PwPack<T> p;
    p.raw = reinterpret_cast<const uint4*>(x)[i];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float v = to_f(p.e[k]);
      p.e[k] = from_f<T>(v > 0.f ? v : 0.f);
    }
    reinterpret_cast<uint4*>(y)[i] = p.raw;
  }
  // scalar tail (n % V elements), handled by the first block
  if (blockIdx.x == 0) {
    for (int64_t i = nv * V + threadIdx.x; i < n; i += kPwThreads) {
      const float v = to_f(x[i]);
      y[i] = from_f<T>(v > 0.f ? v : 0.f);
    }
  }
}

// dx = y > 0 ? dy : 0 (y = relu output, or the input: same sign pattern)
template <typename T>
__global__ void __launch_bounds__(kPwThreads) relu_bwd_kernel(const T* __restrict__ y, const T* __restrict__ dy,
                                                              T* __restrict__ dx, int64_t n) {
  constexpr int V = PwVec<T>::N;
  const int64_t nv = n / V;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kPwThreads;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kPwThreads + threadIdx.x; i < nv; i += stride) {
    PwPack<T> py, pd;
    py.raw = reinterpret_cast<const uint4*>(y)[i];
    pd.raw = reinterpret_cast<const uint4*>(dy)[i];
#pragma unroll
    for (int k = 0; k < V; ++k) pd.e[k] = to_f(py.e[k]) > 0.f ? pd.e[k] : from_f<T>(0.f);
    reinterpret_cast<uint4*>(dx)[i] = pd.raw;
  }
  if (blockIdx.x == 0) {
    for (int64_t i = nv * V + threadIdx.x; i < n; i += kPwThreads) dx[i] = to_f(y[i]) > 0.f ? dy[i] : from_f<T>(0.f);
  }
}

// --------------------------------------------------------------------------- binary kernels
// equal shapes (ROW == 0) or b repeated every `row` elements of a (ROW == 1: out[i] = a[i] op b[i % row]),
// `row` a multiple of the vector width; SWAP evaluates b op a (the row operand on the left)
template <typename T, int OP, int ROW, bool SWAP>
__global__ void __launch_bounds__(kPwThreads) binary_vec_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                                T* __restrict__ out, int64_t n, int64_t row) {
  constexpr int V = PwVec<T>::N;
  const int64_t nv = n / V;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kPwThreads;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kPwThreads + threadIdx.x; i < nv; i += stride) {
    PwPack<T> pa, pb;
    pa.raw = reinterpret_cast<const uint4*>(a)[i];
    const int64_t bi = ROW ? (i * V) % row / V : i;
    pb.raw = reinterpret_cast<const uint4*>(b)[bi];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float x = to_f(pa.e[k]), yv = to_f(pb.e[k]);
      pa.e[k] = from_f<T>(SWAP ? pw_apply<OP>(yv, x) : pw_apply<OP>(x, yv));
    }
    reinterpret_cast<uint4*>(out)[i] = pa.raw;
  }
  if (blockIdx.x == 0) {
    for (int64_t i = nv * V + threadIdx.x; i < n; i += kPwThreads) {
      const float x = to_f(a[i]), yv = to_f(b[ROW ? i % row : i]);
      out[i] = from_f<T>(SWAP ? pw_apply<OP>(yv, x) : pw_apply<OP>(x, yv));
    }
  }
}

struct PwGeom {
  int ndim;
  int64_t shape[kPwMaxDims];
  int64_t sa[kPwMaxDims];   // element strides of a (0 on broadcast axes)
  int64_t sb[kPwMaxDims];
};

template <typename T, int OP>
__global__ void __launch_bounds__(kPwThreads) binary_strided_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                                    T* __restrict__ out, int64_t n, PwGeom g) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kPwThreads;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kPwThreads + threadIdx.x; i < n; i += stride) {
    int64_t rem = i, oa = 0, ob = 0;
    for (int d = g.ndim - 1; d >= 0; --d) {
      const int64_t q = rem / g.shape[d];
      const int64_t idx = rem - q * g.shape[d];
      rem = q;
      oa += idx * g.sa[d];
      ob += idx * g.sb[d];
    }
    out[i] = from_f<T>(pw_apply<OP>(to_f(a[oa]), to_f(b[ob])));
  }
}

template <typename T, int OP>
void binary_launch(const T* a, const T* b, T* out, int64_t n, int mode, int64_t row, const PwGeom& g,
                   hipStream_t s) {
  constexpr int V = PwVec<T>::N;
  const unsigned vb = pw_blocks(n / V + 1);
  if (mode == 0) {
    hipLaunchKernelGGL((binary_vec_kernel<T, OP, 0, false>), dim3(vb), dim3(kPwThreads), 0, s, a, b, out, n, row);
  } else if (mode == 1) {
    hipLaunchKernelGGL((binary_vec_kernel<T, OP, 1, false>), dim3(vb), dim3(kPwThreads), 0, s, a, b, out, n, row);
  } else if (mode == 2) {   // a is the row operand: out = a[i % row] op b[i], computed as b op' a
    hipLaunchKernelGGL((binary_vec_kernel<T, OP, 1, true>), dim3(vb), dim3(kPwThreads), 0, s, b, a, out, n, row);
  } else {
    hipLaunchKernelGGL((binary_strided_kernel<T, OP>), dim3(pw_blocks(n)), dim3(kPwThreads), 0, s, a, b, out, n, g);
  }
}

template <typename T>
void binary_dispatch(int op, const T* a, const T* b, T* out, int64_t n, int mode, int64_t row, const PwGeom& g,
                     hipStream_t s) {
  switch (op) {
    case kAdd: binary_launch<T, kAdd>(a, b, out, n, mode, row, g, s); break;
    case kSub: binary_launch<T, kSub>(a, b, out, n, mode, row, g, s); break;
    case kMul: binary_launch<T, kMul>(a, b, out, n, mode, row, g, s); break;
    case kDiv: binary_launch<T, kDiv>(a, b, out, n, mode, row, g, s); break;
    case kMax: binary_launch<T, kMax>(a, b, out, n, mode, row, g, s); break;
    case kMin: binary_launch<T, kMin>(a, b, out, n, mode, row, g, s); break;
    default: throw std::runtime_error("pointwise_binary: unknown op");
  }
}


// ------------------------------------------------------------------------ weight tap transposes
// out[base[z] + c * rstride[z] + k] = w[k][src[z]][c] for every slot z: the flipped / transposed
// [Cin][taps][Cout] weight of a data-gradient conv (and the per-phase tap subsets of a strided one) in
// ONE launch per weight, instead of a flip kernel plus a permute copy (or an int64 index gather).
constexpr int kTapMax = 32;
struct TapTable {
  int src[kTapMax];
  int64_t base[kTapMax];
  int64_t rstride[kTapMax];
};

template <typename E>
__global__ void __launch_bounds__(256) weight_taps_t_kernel(const E* __restrict__ w, E* __restrict__ out, int K, int RS,
                                                            int C, TapTable tt) {
  __shared__ E tile[64][65];
  const int z = blockIdx.z;
  const int k0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int src = tt.src[z];
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int kk = i >> 6, cc = i & 63;
    const int k = k0 + kk, c = c0 + cc;
    if (k < K && c < C) tile[kk][cc] = w[(static_cast<int64_t>(k) * RS + src) * C + c];
  }
  __syncthreads();
  const int64_t base = tt.base[z], rs = tt.rstride[z];
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int cc = i >> 6, kk = i & 63;
    const int k = k0 + kk, c = c0 + cc;
    if (k < K && c < C) out[base + static_cast<int64_t>(c) * rs + k] = tile[kk][cc];
  }
}

// 16-byte version (K, C, every base and row stride multiples of 8 halves): two vector loads per lane
// issued together, an LDS transpose, two vector stores -- the scalar loop above is load-latency bound
__global__ void __launch_bounds__(256) weight_taps_t_vec_kernel(const uint16_t* __restrict__ w,
                                                                uint16_t* __restrict__ out, int K, int RS, int C,
                                                                TapTable tt) {
  __shared__ __attribute__((aligned(16))) uint16_t tile[64][72];
  const int z = blockIdx.z;
  const int k0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int src = tt.src[z];
  const int tid = threadIdx.x;
  uint4 r[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + i * 256;
    const int k = k0 + (v >> 3), c = c0 + (v & 7) * 8;
    r[i] = (k < K && c < C) ? *reinterpret_cast<const uint4*>(w + (static_cast<int64_t>(k) * RS + src) * C + c)
                            : uint4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + i * 256;
    *reinterpret_cast<uint4*>(&tile[v >> 3][(v & 7) * 8]) = r[i];
  }
  __syncthreads();
  const int64_t base = tt.base[z], rs = tt.rstride[z];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + i * 256;
    const int cc = v >> 3, kv = (v & 7) * 8;
    const int c = c0 + cc, k = k0 + kv;
    if (c < C && k < K) {
      uint32_t q[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        q[j] = static_cast<uint32_t>(tile[kv + 2 * j][cc]) | (static_cast<uint32_t>(tile[kv + 2 * j + 1][cc]) << 16);
      *reinterpret_cast<uint4*>(out + base + static_cast<int64_t>(c) * rs + k) = uint4{q[0], q[1], q[2], q[3]};
    }
  }
}

}  // namespace

void weight_taps_t(int elem_bytes, const void* w, void* out, int K, int RS, int C, int n, const int* src,
                   const int64_t* base, const int64_t* rstride, hipStream_t s) {
  MXAMD_HOST_CHECK(n >= 1 && n <= kTapMax, "weight_taps_t: 1..32 tap slots");
  TapTable tt{};
  for (int z = 0; z < n; ++z) {
    MXAMD_HOST_CHECK(src[z] >= 0 && src[z] < RS, "weight_taps_t: tap index out of range");
    tt.src[z] = src[z];
    tt.base[z] = base[z];
    tt.rstride[z] = rstride[z];
  }
  const dim3 grid((C + 63) / 64, (K + 63) / 64, n);
  bool vec = elem_bytes == 2 && K % 8 == 0 && C % 8 == 0 && reinterpret_cast<uintptr_t>(w) % 16 == 0 &&
             reinterpret_cast<uintptr_t>(out) % 16 == 0;
  for (int z = 0; z < n && vec; ++z) vec = base[z] % 8 == 0 && rstride[z] % 8 == 0;
  if (vec)
    hipLaunchKernelGGL(weight_taps_t_vec_kernel, grid, dim3(256), 0, s, static_cast<const uint16_t*>(w),
                       static_cast<uint16_t*>(out), K, RS, C, tt);
  else if (elem_bytes == 2)
    hipLaunchKernelGGL(weight_taps_t_kernel<uint16_t>, grid, dim3(256), 0, s, static_cast<const uint16_t*>(w),
                       static_cast<uint16_t*>(out), K, RS, C, tt);
  else if (elem_bytes == 4)
    hipLaunchKernelGGL(weight_taps_t_kernel<uint32_t>, grid, dim3(256), 0, s, static_cast<const uint32_t*>(w),
                       static_cast<uint32_t*>(out), K, RS, C, tt);
  else
    throw std::runtime_error("weight_taps_t: 2- or 4-byte elements");
}

void relu_forward(int dtype, const void* x, void* y, int64_t n, hipStream_t s) {
  const unsigned blocks = pw_blocks(n / 8 + 1);
  if (dtype == kF16)
    hipLaunchKernelGGL(relu_fwd_kernel<__half>, dim3(blocks), dim3(kPwThreads), 0, s, static_cast<const __half*>(x),
                       static_cast<__half*>(y), n);
  else if (dtype == kBF16)
    hipLaunchKernelGGL(relu_fwd_kernel<__hip_bfloat16>, dim3(blocks), dim3(kPwThreads), 0, s,
                       static_cast<const __hip_bfloat16*>(x), static_cast<__hip_bfloat16*>(y), n);
  else
    hipLaunchKernelGGL(relu_fwd_kernel<float>, dim3(blocks), dim3(kPwThreads), 0, s, static_cast<const float*>(x),
                       static_cast<float*>(y), n);
}

void relu_backward(int dtype, const void* y, const void* dy, void* dx, int64_t n, hipStream_t s) {
  const unsigned blocks = pw_blocks(n / 8 + 1);
  if (dtype == kF16)
    hipLaunchKernelGGL(relu_bwd_kernel<__half>, dim3(blocks), dim3(kPwThreads), 0, s, static_cast<const __half*>(y),
                       static_cast<const __half*>(dy), static_cast<__half*>(dx), n);
  else if (dtype == kBF16)
    hipLaunchKernelGGL(relu_bwd_kernel<__hip_bfloat16>, dim3(blocks), dim3(kPwThreads), 0, s,
                       static_cast<const __hip_bfloat16*>(y), static_cast<const __hip_bfloat16*>(dy),
                       static_cast<__hip_bfloat16*>(dx), n);
  else
    hipLaunchKernelGGL(relu_bwd_kernel<float>, dim3(blocks), dim3(kPwThreads), 0, s, static_cast<const float*>(y),
                       static_cast<const float*>(dy), static_cast<float*>(dx), n);
}

// mode 0: equal shapes; 1: b repeats every `row` elements; 2: a repeats every `row` elements;
// 3: general broadcast described by (ndim, shape, astride, bstride) in elements
void pointwise_binary(int dtype, int op, const void* a, const void* b, void* out, int64_t n, int mode, int64_t row,
                      int ndim, const int64_t* shape, const int64_t* astride, const int64_t* bstride, hipStream_t s) {
  MXAMD_HOST_CHECK(ndim <= kPwMaxDims, "pointwise_binary: at most 6 dimensions");
  MXAMD_HOST_CHECK(mode == 0 || mode == 3 || (row > 0 && row % (dtype == kF32 ? 4 : 8) == 0),
                   "pointwise_binary: row broadcast needs a row length that is a multiple of the vector width");
  PwGeom g{};
  g.ndim = ndim;
  for (int d = 0; d < ndim; ++d) {
    g.shape[d] = shape[d];
    g.sa[d] = astride[d];
    g.sb[d] = bstride[d];
  }
  if (n == 0) return;
  if (dtype == kF16)
    binary_dispatch<__half>(op, static_cast<const __half*>(a), static_cast<const __half*>(b), static_cast<__half*>(out),
                            n, mode, row, g, s);
  else if (dtype == kBF16)
    binary_dispatch<__hip_bfloat16>(op, static_cast<const __hip_bfloat16*>(a), static_cast<const __hip_bfloat16*>(b),
                                    static_cast<__hip_bfloat16*>(out), n, mode, row, g, s);
  else
    binary_dispatch<float>(op, static_cast<const float*>(a), static_cast<const float*>(b), static_cast<float*>(out), n,
                           mode, row, g, s);
}

}  // namespace mxamd
