// 3x3 / stride 1 / pad 1 NHWC convolution with 64 input and 64 output channels, the halo-tile way
// (gfx950): the ResNet-50 56x56 bottleneck conv2 forward and its stride-1 data gradient.
//
// Why a separate kernel: the implicit-GEMM kernels (conv_big / conv_glds) stage, per 64-deep K-step,
// the 64 input channels of ONE tap for every output pixel of the tile -- each input pixel row is
// fetched nine times (once per tap), and with only 64 output channels a 64 x 512 tile does ~29 MACs
// per staged byte: the L2 -> LDS stream, not the matrix cores, sets the time (~500 TF/s).  Here
//   * each persistent workgroup (one per CU) keeps the WHOLE weight tensor (64 co x 9 taps x 64 c,
//     72 KiB) resident in LDS for the launch;
//   * an output tile is 4 image rows (x up to 57 columns) of one image; its input is the 6-row halo
//     patch (6 x W x 128 B), staged ONCE by LDS-DMA and read by all nine taps from LDS, so the
//     staged bytes per MAC drop ~9x (~230 MACs per byte);
//   * the patches are double-buffered: the DMA of the next tile's patch runs under the current
//     tile's 144 MFMAs per wave and its epilogue; the wait before reuse is a counted vmcnt + raw
//     barrier (the epilogue's stores are buffer stores with out-of-range lanes given an
//     out-of-bounds offset, so every wave issues a fixed number of VM ops);
//   * pixels are indexed on a 64-column grid (row r, column c): columns >= W and the left / right
//     halo of each tap read one zero row of LDS instead of being masked in registers, so the nine
//     taps of a fragment are one base address plus a constant;
//   * epilogue straight from the accumulators: bf16/fp16 stores (a lane owns 4 consecutive channels
//     of a pixel), and optionally the BatchNorm statistics of y (per-channel sum / sum of squares
//     accumulated over all the workgroup's tiles: one partial per workgroup) or, for a data
//     gradient feeding BatchNorm(+ReLU) backward, sum(dz) and sum(dz * (z - mean)) with the ReLU
//     mask recomputed from z (modes 0 / 2 of conv_big's BnBwdFuse).
//
// Requirements (host-checked): C == K == 64, R = S = 3, stride 1, pad 1, dilation 1, W <= 57.
#include <stdexcept>

#include "common.h"
#include "mfma.h"

namespace mxamd {

namespace {

typedef float hf4 __attribute__((ext_vector_type(4)));
typedef uint32_t hu32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t hu32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void h_lds_void;
typedef __attribute__((address_space(1))) void h_gbl_void;

constexpr int kTH = 4;                       // output rows per tile
constexpr int kWBytes = 64 * 9 * 128;        // resident weights: [co][tap] rows of 64 channels
constexpr uint32_t kOOB = 0xFFFFFFF0u;       // buffer offset past num_records: access dropped / reads 0

struct HaloGeom {
  int N, H, W, K;
  int tiles_per_img;   // ceil(H / kTH)
  int ntiles;          // N * tiles_per_img
};

struct HaloBnb {       // BatchNorm-backward statistics of the output (a gradient): modes 0 / 2
  const void* z;
  const float* mean;
  const float* scale;
  const float* shift;
  int mode;
  float* part;         // [2][64][nparts]
};

__device__ __forceinline__ void h_glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((h_gbl_void*)src, (h_lds_void*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void h_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void h_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ float h_row16_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

// STATS: 0 none, 1 forward BN statistics of y, 2 BN-backward statistics (HaloBnb)
template <typename T, int STATS>
__global__ void __launch_bounds__(512) conv3x3_halo_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                           T* __restrict__ y, const T* __restrict__ zero, HaloGeom g,
                                                           float* __restrict__ part, HaloBnb bb) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int W = g.W;
  const int patch_rows = (kTH + 2) * W;            // 6 x W rows of 128 B
  const int patch_bytes = (patch_rows + 7) / 8 * 1024;   // whole 8-row DMA groups
  char* const wbuf = smem;
  char* const pbuf0 = smem + kWBytes;
  char* const zrow = pbuf0 + 2 * patch_bytes;      // 128 B of zeros: halo columns, columns >= W
  float* const bnc = reinterpret_cast<float*>(zrow + 128);   // BN-backward: mean / scale / shift [3][64]

  const int grid = gridDim.x;
  const int g0 = blockIdx.x;
  const int my_tiles = g.ntiles > g0 ? (g.ntiles - g0 + grid - 1) / grid : 0;

  const int lrow = lane >> 3;          // DMA: lane -> row lrow of an 8-row group, slot lane & 7
  const int lpos = lane & 7;

  // ---- patch DMA of tile t into buffer b: rows pr = hr * W + wc (hr 0..5 = image rows h0-1..h0+4)
  auto issue_patch = [&](int t, int b) {
    const int n = t / g.tiles_per_img;
    const int h0 = (t - n * g.tiles_per_img) * kTH;
    char* dst = pbuf0 + b * patch_bytes;
    const int ngroups = (patch_rows + 7) / 8;
    for (int gi = wid; gi < ngroups; gi += 8) {    // wave-uniform
      const int pr = gi * 8 + lrow;
      const int hr = pr / W;
      const int wc = pr - hr * W;
      const int h = h0 - 1 + hr;
      const int ch = lpos ^ (pr & 7);
      const bool ok = pr < patch_rows && (unsigned)h < (unsigned)g.H;
      const T* src = ok ? x + ((int64_t)(n * g.H + h) * W + wc) * 64 + ch * 8 : zero + ch * 8;
      h_glds16(src, dst + gi * 1024);
    }
  };
  if (my_tiles == 0) return;
  // ---- prologue: zero row, resident weights (576 rows: 72 DMA groups, 9 per wave), first patch
  if (tid < 8) *reinterpret_cast<hu32x4*>(zrow + tid * 16) = hu32x4{0u, 0u, 0u, 0u};
  if (STATS == 2 && tid < 64) {
    bnc[tid] = bb.mean[tid];
    bnc[64 + tid] = bb.mode == 2 ? bb.scale[tid] : 0.f;
    bnc[128 + tid] = bb.mode == 2 ? bb.shift[tid] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int gi = i * 8 + wid;
    const int row = gi * 8 + lrow;                 // row = co * 9 + tap
    h_glds16(w + (int64_t)row * 64 + (lpos ^ (row & 7)) * 8, wbuf + gi * 1024);
  }
  issue_patch(g0, 0);
  h_vm_wait<0>();
  __syncthreads();

  // ---- per-lane fragment geometry.  Wave wid owns grid pixels q = wid*32 + j*16 + (lane & 15),
  // j = 0, 1 (row q >> 6, column q & 63) and all 64 output channels (4 fragments of 16).
  const int fr = lane & 15;
  const int fc = lane >> 4;            // 16-byte chunk within a 32-channel K-step
  int pr0[2];                          // patch row of tap (r=0, s=0), may be -1
  uint32_t okm[2];                     // bit s: tap column s is inside the image (and the pixel valid)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int q = wid * 32 + j * 16 + fr;
    const int hr = q >> 6, wc = q & 63;
    pr0[j] = hr * W + wc - 1;
    const bool valid = wc < W;
    okm[j] = valid ? ((wc >= 1 ? 1u : 0u) | 2u | (wc + 1 < W ? 4u : 0u)) : 0u;
  }

  // epilogue geometry: lane holds channels 16i + 4*fc + {0..3} of pixel q_j
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
      y, 0, static_cast<int>(static_cast<uint32_t>(g.N) * g.H * W * 64u * sizeof(T)), 0x00020000);
  __amdgpu_buffer_rsrc_t zrs;
  if (STATS == 2)
    zrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(bb.z), 0,
                                            static_cast<int>(static_cast<uint32_t>(g.N) * g.H * W * 64u * sizeof(T)),
                                            0x00020000);
  float s1[4][4], s2[4][4];            // [i][t] per-channel partial sums over this lane's pixels
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) s1[i][t] = s2[i][t] = 0.f;
  // VM ops per wave issued after the next patch's DMA: the 8 epilogue stores (the BN-backward z
  // rows of a tile are loaded BEFORE that DMA, under the tile's MFMAs)
  constexpr int EPI_OPS = 8;

  for (int it = 0; it < my_tiles; ++it) {
    const int t = g0 + it * grid;
    const int b = it & 1;
    const bool more = it + 1 < my_tiles;
    const int n = t / g.tiles_per_img;
    const int h0 = (t - n * g.tiles_per_img) * kTH;
    hu32x2 zv[2][4];
    if (STATS == 2) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q = wid * 32 + j * 16 + fr;
        const int hr = q >> 6, wc = q & 63;
        const int h = h0 + hr;
        const bool ok = wc < W && h < g.H;
        const uint32_t pix = static_cast<uint32_t>((n * g.H + h) * W + wc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t off = ok ? (pix * 64u + static_cast<uint32_t>(i * 16 + fc * 4)) * sizeof(T) : kOOB;
          zv[j][i] = __builtin_amdgcn_raw_buffer_load_b64(zrs, off, 0, 0);
        }
      }
    }
    if (more) issue_patch(t + grid, b ^ 1);
    const char* pb = pbuf0 + b * patch_bytes;

    hf4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = hf4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int r = tap / 3, s = tap - r * 3;
      const char* brow[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int pr = pr0[j] + r * W + s;
        brow[j] = ((okm[j] >> s) & 1u) ? pb + pr * 128 : nullptr;
      }
      int brsw[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) brsw[j] = (pr0[j] + r * W + s) & 7;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = kk * 4 + fc;
        hu32x4 af[4], bf[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = (i * 16 + fr) * 9 + tap;
          af[i] = *reinterpret_cast<const hu32x4*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const char* a = brow[j] ? brow[j] + ((ch ^ brsw[j]) << 4) : zrow + (ch << 4);
          bf[j] = *reinterpret_cast<const hu32x4*>(a);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma::Op<T>::run(af[i], bf[j], acc[i][j]);
      }
    }

    // ---- epilogue: 8 buffer stores per lane (out-of-range pixels dropped), statistics in registers
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = wid * 32 + j * 16 + fr;
      const int hr = q >> 6, wc = q & 63;
      const int h = h0 + hr;
      const bool ok = wc < W && h < g.H;
      const uint32_t pix = static_cast<uint32_t>((n * g.H + h) * W + wc);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t off = ok ? (pix * 64u + static_cast<uint32_t>(i * 16 + fc * 4)) * sizeof(T) : kOOB;
        const hf4 v = acc[i][j];
        const uint2 pk = mfma::Op<T>::pack4(v[0], v[1], v[2], v[3]);
        __builtin_amdgcn_raw_buffer_store_b64(hu32x2{pk.x, pk.y}, yrs, off, 0, 0);
        if (STATS == 1 && ok) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            s1[i][e] += v[e];
            s2[i][e] += v[e] * v[e];
          }
        }
        if (STATS == 2 && ok) {
          // the statistics use the rounded gradient, as the BatchNorm backward reads it
          const float4 dv = mfma::Op<T>::unpack4(pk);
          const float4 zf = mfma::Op<T>::unpack4(uint2{zv[j][i][0], zv[j][i][1]});
          const float dvs[4] = {dv.x, dv.y, dv.z, dv.w};
          const float zfs[4] = {zf.x, zf.y, zf.z, zf.w};
          const int c0 = i * 16 + fc * 4;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool keep = bb.mode == 2 ? fmaf(zfs[e], bnc[64 + c0 + e], bnc[128 + c0 + e]) > 0.f : true;
            const float dz = keep ? dvs[e] : 0.f;
            s1[i][e] += dz;
            s2[i][e] += dz * (zfs[e] - bnc[c0 + e]);
          }
        }
      }
    }
    if (more) {
      // the next patch landed (its DMA is older than this epilogue's EPI_OPS VM ops), then every
      // wave is past its reads of buffer b^1's previous contents and may read the new ones
      h_vm_wait<EPI_OPS>();
      h_barrier();
    }
  }

  if (STATS != 0) {
    // per-channel totals of the workgroup: 16-lane row sums, then the 8 waves through LDS
    h_vm_wait<0>();
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);   // [2][8 waves][64 channels]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = h_row16_sum(s1[i][e]);
        const float c = h_row16_sum(s2[i][e]);
        if (fr == 0) {
          const int ch = i * 16 + fc * 4 + e;
          red[wid * 64 + ch] = a;
          red[512 + wid * 64 + ch] = c;
        }
      }
    __syncthreads();
    if (tid < 128) {
      const int which = tid >> 6, ch = tid & 63;
      float sum = 0.f;
#pragma unroll
      for (int v = 0; v < 8; ++v) sum += red[which * 512 + v * 64 + ch];
      float* out = STATS == 1 ? part : bb.part;
      out[(int64_t)which * 64 * grid + (int64_t)ch * grid + g0] = sum;
    }
  }
}

int halo_smem_bytes(int W) { return kWBytes + 2 * (((kTH + 2) * W + 7) / 8 * 1024) + 128 + 3 * 64 * 4; }

template <typename T, int STATS>
void launch_halo(const void* x, const void* w, void* y, const void* zero, const HaloGeom& g, int grid, float* part,
                 const HaloBnb& bb, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_halo_kernel<T, STATS>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL((conv3x3_halo_kernel<T, STATS>), dim3(grid), dim3(512), halo_smem_bytes(g.W), s,
                     static_cast<const T*>(x), static_cast<const T*>(w), static_cast<T*>(y),
                     static_cast<const T*>(zero), g, part, bb);
}

}  // namespace

static int halo_cu_count() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  return ncu;
}

bool conv3x3_halo_ok(int C, int K, int R, int S, int sh, int sw, int ph, int pw, int W) {
  return C == 64 && K == 64 && R == 3 && S == 3 && sh == 1 && sw == 1 && ph == 1 && pw == 1 && W >= 1 &&
         halo_smem_bytes(W) <= 160 * 1024;
}

// BN partials per channel the kernel writes (one per workgroup) for this geometry
int conv3x3_halo_nparts(int N, int H) {
  const int ntiles = N * ((H + kTH - 1) / kTH);
  const int ncu = halo_cu_count();
  return ntiles < ncu ? ntiles : ncu;
}

void conv3x3_halo(int dtype, const void* x, const void* w, void* y, const void* zero, int N, int H, int W, int C, int K,
                  float* part, int nparts, const void* bn_z, const float* bn_mean, const float* bn_scale,
                  const float* bn_shift, int bn_mode, float* bn_part, hipStream_t s) {
  MXAMD_HOST_CHECK(conv3x3_halo_ok(C, K, 3, 3, 1, 1, 1, 1, W), "conv3x3_halo: needs C = K = 64 and W <= 57");
  MXAMD_HOST_CHECK((int64_t)N * H * W * 64 * 2 < (1ll << 31) - 64, "conv3x3_halo: tensor too large");
  HaloGeom g;
  g.N = N; g.H = H; g.W = W; g.K = K;
  g.tiles_per_img = (H + kTH - 1) / kTH;
  g.ntiles = N * g.tiles_per_img;
  const int grid = conv3x3_halo_nparts(N, H);
  MXAMD_HOST_CHECK(part == nullptr || nparts == grid, "conv3x3_halo: wrong BN partials count");
  MXAMD_HOST_CHECK(bn_part == nullptr || (bn_z && bn_mean && (bn_mode == 0 || (bn_mode == 2 && bn_scale && bn_shift))),
                   "conv3x3_halo: bad BN-backward arguments");
  MXAMD_HOST_CHECK(part == nullptr || bn_part == nullptr, "conv3x3_halo: forward and backward statistics are exclusive");
  HaloBnb bb{bn_z, bn_mean, bn_scale, bn_shift, bn_mode, bn_part};
  if (dtype == kF16) {
    if (bn_part) launch_halo<__half, 2>(x, w, y, zero, g, grid, part, bb, s);
    else if (part) launch_halo<__half, 1>(x, w, y, zero, g, grid, part, bb, s);
    else launch_halo<__half, 0>(x, w, y, zero, g, grid, part, bb, s);
  } else if (dtype == kBF16) {
    if (bn_part) launch_halo<__hip_bfloat16, 2>(x, w, y, zero, g, grid, part, bb, s);
    else if (part) launch_halo<__hip_bfloat16, 1>(x, w, y, zero, g, grid, part, bb, s);
    else launch_halo<__hip_bfloat16, 0>(x, w, y, zero, g, grid, part, bb, s);
  } else {
    throw std::runtime_error("conv3x3_halo: dtype must be f16 or bf16");
  }
}

}  // namespace mxamd
