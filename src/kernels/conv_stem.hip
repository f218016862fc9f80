// Few-channel "stem" convolutions on MFMA (gfx950): NHWC, Cin <= 4, kernel R x S with
// R <= 8, S <= 8, stride 2, Cout = 64 (ResNet's 7x7/2 on RGB, Inception/MobileNet 3x3/2 stems).
//
// Why a dedicated kernel: the implicit-GEMM conv kernels stage 64-channel K-slices, so a 3-channel
// input would waste >95 % of every MFMA; MIOpen's stem kernels cost ~0.35 ms fwd + ~0.35 ms wgrad
// per ResNet-50 step at batch 256 and the wgrad accumulates with atomics (not reproducible).
//
// Tap layout: the reduction runs over taps t = (r * 8 + s) * 4 + c (S padded to 8, C padded to 4
// with zeros), so one 32-deep MFMA K-step is one kernel row r and the 8 taps a lane holds (s = 2g,
// 2g + 1; c = 0..3) are two horizontally adjacent input pixels of 4 channels = 16 contiguous bytes of
// an LDS input patch stored as [row][col][4 x half].  With stride 2 and the patch column of output
// column j at 2j (+ s), the 16-byte read is aligned: one ds_read_b128 per B fragment.
//
// Forward (conv_stem_fwd_kernel): 256 threads, output tiles of 8 rows x 16 columns (128 pixels) x
// 64 channels; wave w owns rows 2w, 2w+1.  A = the weights (row = output channel), kept in VGPRs
// for the whole persistent loop (4 channel fragments x R K-steps); B = patch fragments.  The next
// tile's patch is fetched into registers while the current one computes; the epilogue rounds the
// accumulators into an LDS [pixel][channel] image and stores whole 128-byte pixel rows, and (in
// training) accumulates per-channel sum / sum-of-squares partials per wave -- written once at the
// end, [2][64][nparts] like conv_big.hip, consumed by the BatchNorm finalize.
//
// Weight gradient (conv_stem_wgrad_kernel): dW[k][tap] = sum over pixels dy[p][k] * X[p][tap], the
// pixels being the MFMA reduction dimension: A = dy^T (8 pixels of one channel per lane), B = the
// patch taps of 8 pixels, both gathered from LDS with 16-bit reads.  Each persistent workgroup
// accumulates its pixel tiles in registers and writes one fp32 slab; stem_wgrad_reduce_kernel sums
// the slabs in a fixed order (deterministic) into the real [K][R][S][C] gradient (optionally added
// into an existing .grad buffer).
#include <stdexcept>

#include "common.h"
#include "mfma.h"

namespace mxamd {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
struct StemMfma : mfma::Op<T> {};   // 16x16x32 MFMA + epilogue packs (mfma.h)

struct StemGeom {
  int N, H, W, C, K, R, S;
  int Ho, Wo, ph, pw;
  int tiles_w, tiles_per_img, ntiles;
};

constexpr int kTH = 8;                   // output rows per tile
constexpr int kTW = 16;                  // output columns per tile
constexpr int kPix = kTH * kTW;          // 128 pixels
constexpr int kPH = 2 * (kTH - 1) + 8;   // patch rows (R <= 8)
constexpr int kPW = 2 * (kTW - 1) + 8;   // patch columns (S padded to 8)
constexpr int kPatchBytes = kPH * kPW * 8;
constexpr int kPatchPix = kPH * kPW;
constexpr int kPatchPerThread = (kPatchPix + 255) / 256;
constexpr int kOutPitch = 64 * 2 + 16;   // LDS [pixel][64 ch] image row pitch (bytes)

__device__ __forceinline__ void tile_origin(const StemGeom& g, int tile, int* n, int* oh0, int* ow0) {
  *n = tile / g.tiles_per_img;
  const int rem = tile - *n * g.tiles_per_img;
  const int th = rem / g.tiles_w;
  *oh0 = th * kTH;
  *ow0 = (rem - th * g.tiles_w) * kTW;
}

// fetch the input patch of a tile into registers: patch pixel q = tid + 256 * i holds 4 halves
template <typename T>
__device__ __forceinline__ void fetch_patch(const T* __restrict__ x, const StemGeom& g, int tile, int tid,
                                            uint2 (&reg)[kPatchPerThread]) {
  int n, oh0, ow0;
  tile_origin(g, tile, &n, &oh0, &ow0);
  const int h0 = 2 * oh0 - g.ph, w0 = 2 * ow0 - g.pw;
  const uint16_t* xs = reinterpret_cast<const uint16_t*>(x);
#pragma unroll
  for (int i = 0; i < kPatchPerThread; ++i) {
    const int q = tid + 256 * i;
    uint16_t v[4] = {0, 0, 0, 0};
    if (q < kPatchPix) {
      const int pr = q / kPW, pc = q - (q / kPW) * kPW;
      const int hi = h0 + pr, wi = w0 + pc;
      if ((unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W) {
        const int64_t base = ((static_cast<int64_t>(n) * g.H + hi) * g.W + wi) * g.C;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (c < g.C) v[c] = xs[base + c];
      }
    }
    reg[i].x = static_cast<uint32_t>(v[0]) | (static_cast<uint32_t>(v[1]) << 16);
    reg[i].y = static_cast<uint32_t>(v[2]) | (static_cast<uint32_t>(v[3]) << 16);
  }
}

__device__ __forceinline__ void store_patch(char* patch, int tid, const uint2 (&reg)[kPatchPerThread]) {
#pragma unroll
  for (int i = 0; i < kPatchPerThread; ++i) {
    const int q = tid + 256 * i;
    if (q < kPatchPix) *reinterpret_cast<uint2*>(patch + q * 8) = reg[i];
  }
}

// sum over the 16 lanes that share lane >> 4
__device__ __forceinline__ float sum16(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

constexpr int kWPitch = 8 * 32 * 2 + 32;   // LDS weight image [64 ch][8 rows][32 taps] row pitch (bytes):
                                           // 136 dwords, so the 16 lanes of a ds_read_b128 group start on
                                           // distinct 4-bank slots (132 collided: 4(fr + fg))

template <typename T>
__global__ void __launch_bounds__(256, 3) conv_stem_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                            T* __restrict__ y, StemGeom g,
                                                            float* __restrict__ part, int nparts) {
  // the output image reuses the patch's LDS (a barrier separates the last patch read from the first
  // image write): 53 KB per workgroup, three workgroups per CU -- the kernel waits on its input gathers
  // for most of its cycles, and a third workgroup hides more of that latency
  constexpr int kStage = kPatchBytes > kPix * kOutPitch ? kPatchBytes : kPix * kOutPitch;
  __shared__ __attribute__((aligned(16))) char smem[kStage + 64 * kWPitch];
  char* patch = smem;
  char* outimg = smem;
  char* wimg = smem + kStage;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int fr = lane & 15;     // fragment row / column index
  const int fg = lane >> 4;     // k group: taps s = 2fg, 2fg+1

  // weight image, zero for padded taps: [channel][r][tap (s * 4 + c)], 16-byte padded rows (the 16
  // channels a fragment read touches land on distinct banks)
  const uint16_t* ws = reinterpret_cast<const uint16_t*>(w);
  for (int e = tid; e < 64 * 256; e += 256) {
    const int k = e >> 8, r = (e >> 5) & 7, sc = e & 31, sx = sc >> 2, c = sc & 3;
    const uint16_t v = (r < g.R && sx < g.S && c < g.C) ? ws[((k * g.R + r) * g.S + sx) * g.C + c] : uint16_t(0);
    *reinterpret_cast<uint16_t*>(wimg + k * kWPitch + (r * 32 + sc) * 2) = v;
  }

  float bsum[4][4], bsq[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) bsum[i][q] = bsq[i][q] = 0.f;

  uint2 preg[kPatchPerThread];
  int tile = blockIdx.x;
  if (tile < g.ntiles) fetch_patch(x, g, tile, tid, preg);
  for (; tile < g.ntiles; tile += gridDim.x) {
    __syncthreads();                     // previous tile's patch / output image fully consumed
    store_patch(patch, tid, preg);
    __syncthreads();
    const int next = tile + gridDim.x;
    if (next < g.ntiles) fetch_patch(x, g, next, tid, preg);   // in flight during the MFMAs

    f4_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jf = 0; jf < 2; ++jf) acc[i][jf] = f4_t{0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < g.R; ++r) {
      u32x4 bf[2], af[4];
#pragma unroll
      for (int jf = 0; jf < 2; ++jf) {
        const int prow = 2 * (2 * wv + jf) + r;
        const int pcol = 2 * fr + 2 * fg;
        bf[jf] = *reinterpret_cast<const u32x4*>(patch + (prow * kPW + pcol) * 8);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const u32x4*>(wimg + (16 * i + fr) * kWPitch + (r * 32 + 8 * fg) * 2);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jf = 0; jf < 2; ++jf) acc[i][jf] = StemMfma<T>::run(af[i], bf[jf], acc[i][jf]);
    }

    // epilogue: lane holds channels 16i + 4fg + q of pixel (row 2wv + jf, column fr)
    __syncthreads();                     // every wave's patch reads done: the image overwrites the patch
    int n, oh0, ow0;
    tile_origin(g, tile, &n, &oh0, &ow0);
#pragma unroll
    for (int jf = 0; jf < 2; ++jf) {
      const int ohl = 2 * wv + jf;
      const bool valid = (oh0 + ohl < g.Ho) && (ow0 + fr < g.Wo);
      const int pl = ohl * kTW + fr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f4_t v = acc[i][jf];
        uint2 pk;
        pk.x = StemMfma<T>::two(v[0], v[1]);
        pk.y = StemMfma<T>::two(v[2], v[3]);
        *reinterpret_cast<uint2*>(outimg + pl * kOutPitch + (16 * i + 4 * fg) * 2) = pk;
        if (part != nullptr && valid) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            bsum[i][q] += v[q];
            bsq[i][q] += v[q] * v[q];
          }
        }
      }
    }
    __syncthreads();
    // whole 128-byte pixel rows: 128 pixels x 8 chunks of 16 B = 1024 chunks, 4 per thread
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = tid + 256 * it;
      const int pl = e >> 3, ch = e & 7;
      const int oh = oh0 + pl / kTW, ow = ow0 + (pl % kTW);
      if (oh < g.Ho && ow < g.Wo) {
        const uint4 v = *reinterpret_cast<const uint4*>(outimg + pl * kOutPitch + ch * 16);
        T* dst = y + ((static_cast<int64_t>(n) * g.Ho + oh) * g.Wo + ow) * 64 + ch * 8;
        *reinterpret_cast<uint4*>(dst) = v;
      }
    }
  }
  if (part != nullptr) {
    const int pid = blockIdx.x * 4 + wv;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float s1 = sum16(bsum[i][q]);
        const float s2 = sum16(bsq[i][q]);
        if (fr == 0) {
          const int c = 16 * i + 4 * fg + q;
          part[static_cast<int64_t>(c) * nparts + pid] = s1;
          part[static_cast<int64_t>(64 + c) * nparts + pid] = s2;
        }
      }
  }
}

// taps per K-step = 32 (one kernel row); 8 rows -> 256 tap columns = 16 tap fragments, 4 per wave
constexpr int kTapFrags = 16;
constexpr int kDyPitch = 64 * 2 + 16;

template <typename T>
__global__ void __launch_bounds__(256, 3) conv_stem_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                              float* __restrict__ slab, StemGeom g) {
  __shared__ __attribute__((aligned(16))) char smem[kPatchBytes + kPix * kDyPitch];
  char* patch = smem;
  char* dyimg = smem + kPatchBytes;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int fr = lane & 15;
  const int fg = lane >> 4;
  const int nfr = 2 * g.R;        // live tap fragments (R kernel rows x 32 taps / 16)

  f4_t acc[4][4];                 // [channel fragment][tap fragment wv + 4 t]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = f4_t{0.f, 0.f, 0.f, 0.f};

  uint2 preg[kPatchPerThread];
  int tile = blockIdx.x;
  if (tile < g.ntiles) fetch_patch(x, g, tile, tid, preg);
  for (; tile < g.ntiles; tile += gridDim.x) {
    int n, oh0, ow0;
    tile_origin(g, tile, &n, &oh0, &ow0);
    // dy tile: 128 pixels x 64 channels, 16-byte chunks (zero for pixels outside the image)
    uint4 dreg[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = tid + 256 * it;
      const int pl = e >> 3, ch = e & 7;
      const int oh = oh0 + pl / kTW, ow = ow0 + (pl % kTW);
      dreg[it] = make_uint4(0, 0, 0, 0);
      if (oh < g.Ho && ow < g.Wo)
        dreg[it] = *reinterpret_cast<const uint4*>(dy + ((static_cast<int64_t>(n) * g.Ho + oh) * g.Wo + ow) * 64 +
                                                   ch * 8);
    }
    __syncthreads();
    store_patch(patch, tid, preg);
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = tid + 256 * it;
      *reinterpret_cast<uint4*>(dyimg + (e >> 3) * kDyPitch + (e & 7) * 16) = dreg[it];
    }
    __syncthreads();
    const int next = tile + gridDim.x;
    if (next < g.ntiles) fetch_patch(x, g, next, tid, preg);

    const uint16_t* dyh = reinterpret_cast<const uint16_t*>(dyimg);
    const uint16_t* ph = reinterpret_cast<const uint16_t*>(patch);
    // 4 K-steps of 32 pixels; lane's 8 pixels: p = 32 ks + 4 j + fg (any pixel order inside a K-step
    // works as long as both operands use it; this one puts the four lane groups of a 16-bit LDS read on
    // neighbouring pixels -- distinct banks -- where 8 fg + j put them 8 pixels = 0 mod 32 banks apart)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      u32x4 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint16_t e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int p = 32 * ks + 4 * j + fg;
          e[j] = dyh[(p * kDyPitch) / 2 + 16 * i + fr];
        }
        af[i] = u32x4{static_cast<uint32_t>(e[0]) | (static_cast<uint32_t>(e[1]) << 16),
                      static_cast<uint32_t>(e[2]) | (static_cast<uint32_t>(e[3]) << 16),
                      static_cast<uint32_t>(e[4]) | (static_cast<uint32_t>(e[5]) << 16),
                      static_cast<uint32_t>(e[6]) | (static_cast<uint32_t>(e[7]) << 16)};
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int tf = wv + 4 * t;
        if (tf < nfr) {
          // tap column (tf * 16 + fr) = (r * 8 + s) * 4 + c
          const int tap = tf * 16 + fr;
          const int r = tap >> 5, s = (tap >> 2) & 7, c = tap & 3;
          uint16_t e[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int p = 32 * ks + 4 * j + fg;
            const int ohl = p / kTW, owl = p % kTW;
            e[j] = ph[((2 * ohl + r) * kPW + 2 * owl + s) * 4 + c];
          }
          const u32x4 bfr{static_cast<uint32_t>(e[0]) | (static_cast<uint32_t>(e[1]) << 16),
                          static_cast<uint32_t>(e[2]) | (static_cast<uint32_t>(e[3]) << 16),
                          static_cast<uint32_t>(e[4]) | (static_cast<uint32_t>(e[5]) << 16),
                          static_cast<uint32_t>(e[6]) | (static_cast<uint32_t>(e[7]) << 16)};
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][t] = StemMfma<T>::run(af[i], bfr, acc[i][t]);
        }
      }
    }
  }
  // slab [block][64 channels][256 tap columns]: lane holds channels 16i + 4fg + q of tap column tf*16 + fr
  float* sb = slab + static_cast<int64_t>(blockIdx.x) * 64 * 256;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int tf = wv + 4 * t;
    if (tf < kTapFrags) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) sb[(16 * i + 4 * fg + q) * 256 + tf * 16 + fr] = tf < nfr ? acc[i][t][q] : 0.f;
    }
  }
}

// dW[k][r][s][c] (+)= sum over slabs b (in order) of slab[b][k][(r * 8 + s) * 4 + c]; one block per
// (k, r): 8 slices of the slab range per tap column, combined in a fixed order
template <typename TO>
__global__ void __launch_bounds__(256) stem_wgrad_reduce_kernel(const float* __restrict__ slab, int nslab,
                                                                TO* __restrict__ out, int R, int S, int C,
                                                                int accum) {
  const int k = blockIdx.x / R, r = blockIdx.x % R;
  const int tcol = threadIdx.x & 31, slice = threadIdx.x >> 5;
  const int64_t col = static_cast<int64_t>(k) * 256 + r * 32 + tcol;
  float a = 0.f;
  for (int b = slice; b < nslab; b += 8) a += slab[static_cast<int64_t>(b) * 64 * 256 + col];
  __shared__ float red[8][32];
  red[slice][tcol] = a;
  __syncthreads();
  if (slice == 0) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += red[q][tcol];
    const int s = tcol >> 2, c = tcol & 3;
    if (s < S && c < C) {
      TO* o = out + ((static_cast<int64_t>(k) * R + r) * S + s) * C + c;
      const float prev = accum ? static_cast<float>(*o) : 0.f;
      *o = static_cast<TO>(prev + t);
    }
  }
}

StemGeom stem_geom(int N, int H, int W, int C, int K, int R, int S, int ph, int pw) {
  StemGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S; g.ph = ph; g.pw = pw;
  g.Ho = (H + 2 * ph - R) / 2 + 1;
  g.Wo = (W + 2 * pw - S) / 2 + 1;
  g.tiles_w = (g.Wo + kTW - 1) / kTW;
  g.tiles_per_img = ((g.Ho + kTH - 1) / kTH) * g.tiles_w;
  g.ntiles = N * g.tiles_per_img;
  return g;
}

void stem_check(int C, int K, int R, int S, int sh, int sw) {
  MXAMD_HOST_CHECK(C >= 1 && C <= 4, "conv_stem: input channels must be 1..4");
  MXAMD_HOST_CHECK(K == 64, "conv_stem: 64 output channels");
  MXAMD_HOST_CHECK(R >= 1 && R <= 8 && S >= 1 && S <= 8, "conv_stem: kernel up to 8x8");
  MXAMD_HOST_CHECK(sh == 2 && sw == 2, "conv_stem: stride 2");
}

}  // namespace

// forward: three resident workgroups per CU (53 KB of LDS each), persistent
int conv_stem_grid(int N, int H, int W, int R, int S, int ph, int pw) {
  const StemGeom g = stem_geom(N, H, W, 1, 64, R, S, ph, pw);
  return g.ntiles < 768 ? g.ntiles : 768;
}

// weight gradient: three resident workgroups per CU (148 registers, 25 KB LDS), one fp32 slab each
static int stem_wgrad_grid(int N, int H, int W, int R, int S, int ph, int pw) {
  const StemGeom g = stem_geom(N, H, W, 1, 64, R, S, ph, pw);
  return g.ntiles < 768 ? g.ntiles : 768;
}

void conv_stem_fwd(int dtype, const void* x, const void* w, void* y, int N, int H, int W, int C, int K, int R, int S,
                   int sh, int sw, int ph, int pw, float* part, int nparts, hipStream_t s) {
  stem_check(C, K, R, S, sh, sw);
  const StemGeom g = stem_geom(N, H, W, C, K, R, S, ph, pw);
  const int grid = conv_stem_grid(N, H, W, R, S, ph, pw);
  MXAMD_HOST_CHECK(part == nullptr || nparts == grid * 4, "conv_stem_fwd: nparts must be 4 * grid");
  MXAMD_HOST_CHECK(static_cast<int64_t>(N) * g.Ho * g.Wo * 64 < (int64_t(1) << 40), "conv_stem_fwd: too large");
  if (g.ntiles == 0) return;
  if (dtype == kF16)
    hipLaunchKernelGGL(conv_stem_fwd_kernel<__half>, dim3(grid), dim3(256), 0, s, static_cast<const __half*>(x),
                       static_cast<const __half*>(w), static_cast<__half*>(y), g, part, nparts);
  else if (dtype == kBF16)
    hipLaunchKernelGGL(conv_stem_fwd_kernel<__hip_bfloat16>, dim3(grid), dim3(256), 0, s,
                       static_cast<const __hip_bfloat16*>(x), static_cast<const __hip_bfloat16*>(w),
                       static_cast<__hip_bfloat16*>(y), g, part, nparts);
  else
    throw std::runtime_error("conv_stem_fwd: f16 / bf16 only");
}

int64_t conv_stem_wgrad_workspace(int N, int H, int W, int R, int S, int ph, int pw) {
  return static_cast<int64_t>(stem_wgrad_grid(N, H, W, R, S, ph, pw)) * 64 * 256;
}

void conv_stem_wgrad(int dtype, const void* x, const void* dy, float* slab, int out_dtype, void* out, int accum, int N,
                     int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, hipStream_t s) {
  stem_check(C, K, R, S, sh, sw);
  const StemGeom g = stem_geom(N, H, W, C, K, R, S, ph, pw);
  const int grid = stem_wgrad_grid(N, H, W, R, S, ph, pw);
  if (g.ntiles == 0) return;
  if (dtype == kF16)
    hipLaunchKernelGGL(conv_stem_wgrad_kernel<__half>, dim3(grid), dim3(256), 0, s, static_cast<const __half*>(x),
                       static_cast<const __half*>(dy), slab, g);
  else if (dtype == kBF16)
    hipLaunchKernelGGL(conv_stem_wgrad_kernel<__hip_bfloat16>, dim3(grid), dim3(256), 0, s,
                       static_cast<const __hip_bfloat16*>(x), static_cast<const __hip_bfloat16*>(dy), slab, g);
  else
    throw std::runtime_error("conv_stem_wgrad: f16 / bf16 only");
  const dim3 rgrid(64 * R);
  if (out_dtype == kF16)
    hipLaunchKernelGGL(stem_wgrad_reduce_kernel<__half>, rgrid, dim3(256), 0, s, slab, grid,
                       static_cast<__half*>(out), R, S, C, accum);
  else if (out_dtype == kBF16)
    hipLaunchKernelGGL(stem_wgrad_reduce_kernel<__hip_bfloat16>, rgrid, dim3(256), 0, s, slab, grid,
                       static_cast<__hip_bfloat16*>(out), R, S, C, accum);
  else
    hipLaunchKernelGGL(stem_wgrad_reduce_kernel<float>, rgrid, dim3(256), 0, s, slab, grid,
                       static_cast<float*>(out), R, S, C, accum);
}

}  // namespace mxamd
