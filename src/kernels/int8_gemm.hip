// int8 x int8 -> int32 GEMM on the gfx950 i8 matrix cores (v_mfma_i32_16x16x64_i8).
//
// Parity: src/operator/quantization/quantized_fully_connected.cu and
// quantized_conv.cu (cuBLAS/cuDNN int8 GEMMs with int32 accumulation).  The
// framework lowers quantized FullyConnected directly and quantized Convolution
// through an im2col view (ops/quantization_ops.py) onto
//     C[M][N] = sum_k A[M][k] * B[N][k]        (A: activations, B: weights)
//
// Tiling: a 256-thread block (4 waves, 2x2) owns a 64x64 output tile; every
// wave a 32x32 sub-tile = 2x2 MFMA 16x16x64 accumulators (int32).  K advances
// 64 bytes per step: each thread moves one 16-byte row segment of A and of B
// into LDS (64 rows x 64 bytes per operand), then each lane reads its 16-byte
// fragment (row lane&15, k-block lane>>4) for A and B -- the same k mapping for
// both operands, so the products pair matching k regardless of the
// instruction's internal k order.  Out-of-range rows read as zeros; K must be a
// multiple of 64 (the host pads).
#include <stdexcept>

#include "common.h"

namespace mxamd {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) int8_gemm_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
                                                        int32_t* __restrict__ C, int M, int N, int K) {
  __shared__ int4 As[64][4];
  __shared__ int4 Bs[64][4];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int bm = blockIdx.y * 64, bn = blockIdx.x * 64;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int lr = tid >> 2, lc = tid & 3;        // load coordinates: row, 16-byte column
  v4i acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  const int4 zero = make_int4(0, 0, 0, 0);
  for (int k0 = 0; k0 < K; k0 += 64) {
    const int4 a = (bm + lr < M) ? *reinterpret_cast<const int4*>(A + static_cast<int64_t>(bm + lr) * K + k0 + lc * 16)
                                 : zero;
    const int4 b = (bn + lr < N) ? *reinterpret_cast<const int4*>(B + static_cast<int64_t>(bn + lr) * K + k0 + lc * 16)
                                 : zero;
    As[lr][lc] = a;
    Bs[lr][lc] = b;
    __syncthreads();
    v4i af[2], bf[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int4 t = As[wm + i * 16 + (lane & 15)][lane >> 4];
      af[i] = v4i{t.x, t.y, t.z, t.w};
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int4 t = Bs[wn + j * 16 + (lane & 15)][lane >> 4];
      bf[j] = v4i{t.x, t.y, t.z, t.w};
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
  // C/D map of the 16x16 MFMA family: column = lane & 15, row = 4 * (lane >> 4) + register
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = bm + wm + i * 16 + (lane >> 4) * 4 + r;
        const int col = bn + wn + j * 16 + (lane & 15);
        if (row < M && col < N) C[static_cast<int64_t>(row) * N + col] = acc[i][j][r];
      }
}

}  // namespace

void int8_gemm(const int8_t* A, const int8_t* B, int32_t* C, int M, int N, int K, hipStream_t s) {
  MXAMD_HOST_CHECK(K % 64 == 0, "int8_gemm: K must be a multiple of 64 (pad on the host)");
  MXAMD_HOST_CHECK(M > 0 && N > 0, "int8_gemm: empty problem");
  const dim3 grid((N + 63) / 64, (M + 63) / 64);
  hipLaunchKernelGGL(int8_gemm_kernel, grid, dim3(256), 0, s, A, B, C, M, N, K);
}

}  // namespace mxamd
