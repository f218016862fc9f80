// Channel-last (NHWC) BatchNorm for gfx950: training statistics, fused
// apply (+residual add, +ReLU) and fused backward.
//
// Parity: src/operator/nn/batch_norm.cu / cudnn_batch_norm (forward with
// moving statistics, fix_gamma, use_global_stats), contrib BatchNormWithReLU
// and the "BatchNormAddReLU" residual tail used by MXNet's NHWC ResNet.
//
// Design (memory-bound op, so everything is about HBM passes):
//   forward : 1 read pass for shifted sums (sum(x-k), sum((x-k)^2), k = running
//             mean: no catastrophic cancellation), 1 read + 1 write pass for
//             y = x*scale + shift (+addend) (relu).
//   backward: 1 read pass over (dy, x[, y]) for sum(dz), sum(dz*(x-mean)) where
//             dz = relu ? dy*mask : dy, then 1 pass writing
//             dx = A*dz + B*x + C (and d_addend = dz for the residual branch).
//             The ReLU mask of a plain BN+ReLU is recomputed from x and the
//             forward's (scale, shift) -- (x*scale + shift > 0) -- so y is never
//             saved or re-read (one pass fewer in each backward kernel); only the
//             residual tail, whose mask also depends on the addend, reads y.
//             dgamma/dbeta can be accumulated straight into the parameters'
//             fp32 gradient buffers (no separate accumulate kernels).
// Every thread moves 16 bytes (8 x fp16/bf16) per access; a row of C channels
// is covered by C/8 lanes so loads are fully coalesced for any C % 8 == 0.
// Reductions: per-thread fp32 registers -> LDS tree -> per-block partials ->
// one block per channel combines the (channel-major) partials in fp64.
#include <cstdlib>
#include <stdexcept>

#include <algorithm>

#include "common.h"

namespace mxamd {

constexpr int kBnThreads = 256;

struct BnGeom {
  int tpr;   // threads per row (each covers 8 channels)
  int cb;    // channels per block (= tpr * 8)
  int rpi;   // rows per iteration of the block
};

static inline BnGeom bn_geom(int C) {
  BnGeom g;
  // threads per row: all C/8 channel groups when they fit in a block, else the largest divisor of
  // C/8 that does (C = 3072 -> 192), so every block covers whole channel groups
  int v = C / 8;
  g.tpr = v;
  if (v > kBnThreads)
    for (g.tpr = kBnThreads; v % g.tpr != 0; --g.tpr) {
    }
  g.cb = g.tpr * 8;
  g.rpi = kBnThreads / g.tpr;
  return g;
}

// ReLU mask source in the backward kernels
constexpr int kReluNone = 0;   // no ReLU
constexpr int kReluFromY = 1;  // mask = y > 0 (residual tail: y depends on the addend)
constexpr int kReluFromX = 2;  // mask = x*scale + shift > 0 (recomputed, y not needed)
constexpr int kReluFromMask = 3;  // residual tail: 1 bit per element written by the forward (y not kept)

// MODE 0: forward sums of (x - shift) and (x - shift)^2
// MODE 1: backward sums of dz and dz * (x - mean), dz = dy * mask (RELU != kReluNone)
template <typename T, int MODE, int RELU>
__global__ void __launch_bounds__(kBnThreads) bn_reduce_kernel(
    const T* __restrict__ x, const T* __restrict__ dy, const T* __restrict__ y, const uint8_t* __restrict__ mask,
    const float* __restrict__ center, const float* __restrict__ fscale, const float* __restrict__ fshift,
    float* __restrict__ part1, float* __restrict__ part2, int64_t R, int C, int tpr, int rpi,
    int64_t rows_per_block) {
  const int tid = threadIdx.x;
  const int lane_c = tid % tpr;   // which 8-channel group inside the block's channel slice
  const int lane_r = tid / tpr;   // row offset within an iteration
  const int cbase = blockIdx.y * tpr * 8 + lane_c * 8;
  float s1[8], s2[8], k[8], fs[8], fh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s1[i] = 0.f;
    s2[i] = 0.f;
    k[i] = center[cbase + i];
    if (RELU == kReluFromX) {
      fs[i] = fscale[cbase + i];
      fh[i] = fshift[cbase + i];
    }
  }
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  int64_t r1 = r0 + rows_per_block;
  if (r1 > R) r1 = R;
  // when tpr does not divide the block (C/8 not a power of two, e.g. C = 96 or 768) the last
  // tid / tpr == rpi lanes are spare: they load nothing and stay out of the LDS reduction
  const bool spare = lane_r >= rpi;
  if (spare) r1 = r0;
  // rows are consumed UNR at a time: all loads of a batch are issued before any
  // accumulation, so each thread keeps UNR (x3 in backward) 16-byte loads in flight
  constexpr int UNR = 4;
  auto accum = [&](const Vec8<T>& vx, const Vec8<T>& vdy, const Vec8<T>& vy, uint32_t mb) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (MODE == 0) {
        float d = vx.get(i) - k[i];
        s1[i] += d;
        s2[i] += d * d;
      } else {
        float dz = vdy.get(i);
        const float xi = vx.get(i);
        if (RELU == kReluFromY) dz = vy.get(i) > 0.f ? dz : 0.f;
        if (RELU == kReluFromX) dz = fmaf(xi, fs[i], fh[i]) > 0.f ? dz : 0.f;
        if (RELU == kReluFromMask) dz = ((mb >> i) & 1u) ? dz : 0.f;
        s1[i] += dz;
        s2[i] += dz * (xi - k[i]);
      }
    }
  };
  int64_t r = r0 + lane_r;
  for (; r + (UNR - 1) * rpi < r1; r += UNR * rpi) {
    Vec8<T> vx[UNR], vdy[UNR], vy[UNR];
    uint32_t vm[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t off = (r + u * rpi) * C + cbase;
      vx[u].load(x + off);
      if (MODE == 1) vdy[u].load(dy + off);
      if (MODE == 1 && RELU == kReluFromY) vy[u].load(y + off);
      vm[u] = (MODE == 1 && RELU == kReluFromMask) ? mask[off >> 3] : 0u;
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) accum(vx[u], vdy[u], vy[u], vm[u]);
  }
  for (; r < r1; r += rpi) {
    const int64_t off = r * C + cbase;
    Vec8<T> vx, vdy, vy;
    vx.load(x + off);
    if (MODE == 1) vdy.load(dy + off);
    if (MODE == 1 && RELU == kReluFromY) vy.load(y + off);
    accum(vx, vdy, vy, (MODE == 1 && RELU == kReluFromMask) ? mask[off >> 3] : 0u);
  }
  // reduce the rpi row-lanes that share a channel group through LDS
  __shared__ float sh1[kBnThreads * 8];
  __shared__ float sh2[kBnThreads * 8];
  const int cb = tpr * 8;
  if (!spare) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sh1[lane_r * cb + lane_c * 8 + i] = s1[i];
      sh2[lane_r * cb + lane_c * 8 + i] = s2[i];
    }
  }
  __syncthreads();
  for (int c = tid; c < cb; c += kBnThreads) {
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < rpi; ++rr) {
      a += sh1[rr * cb + c];
      b += sh2[rr * cb + c];
    }
    // channel-major partials [C][nblk]: the finalize reads each channel's
    // partials contiguously
    const int64_t o = static_cast<int64_t>(blockIdx.y * cb + c) * gridDim.x + blockIdx.x;
    part1[o] = a;
    part2[o] = b;
  }
}

// One wave per channel (four channels per 256-thread block): combine the channel's per-block partials
// (contiguous, channel-major) in fp64 and emit statistics -- a wave-level shuffle reduction, no LDS or
// block barrier, and C / 4 workgroups to dispatch (these launches run ~100 times per ResNet-50 step).
// MODE 0 (forward): out mean, invstd, var(biased); scale = g*invstd, shift = b - mean*scale
// MODE 1 (backward): dgamma, dbeta and the dx coefficients A, B, Cc
constexpr int kFinThreads = 256;
constexpr int kFinPerBlock = kFinThreads / 64;
template <int MODE>
__global__ void __launch_bounds__(kFinThreads) bn_finalize_kernel(
    const float* __restrict__ part1, const float* __restrict__ part2, int nblk, int C, int64_t R,
    const float* __restrict__ center, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ invstd_in, float eps, float* __restrict__ o0, float* __restrict__ o1,
    float* __restrict__ o2, float* __restrict__ o3, float* __restrict__ o4, float* __restrict__ o5,
    int fix_gamma, int training, float momentum, float* __restrict__ mm_upd, float* __restrict__ mv_upd,
    int accum) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * kFinPerBlock + (threadIdx.x >> 6);
  if (c >= C) return;   // whole waves only
  const float* p1 = part1 + static_cast<int64_t>(c) * nblk;
  const float* p2 = part2 + static_cast<int64_t>(c) * nblk;
  double a = 0.0, b = 0.0;
  // 16-byte loads where the channel's partial row is aligned: 4x fewer dependent load rounds
  const int nv = ((reinterpret_cast<uintptr_t>(p1) | reinterpret_cast<uintptr_t>(p2)) & 15) == 0 ? nblk / 4 : 0;
  for (int i = lane; i < nv; i += 64) {
    const float4 x = reinterpret_cast<const float4*>(p1)[i];
    const float4 y = reinterpret_cast<const float4*>(p2)[i];
    a += static_cast<double>(x.x) + static_cast<double>(x.y) + static_cast<double>(x.z) + static_cast<double>(x.w);
    b += static_cast<double>(y.x) + static_cast<double>(y.y) + static_cast<double>(y.z) + static_cast<double>(y.w);
  }
  for (int i = nv * 4 + lane; i < nblk; i += 64) {
    a += p1[i];
    b += p2[i];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  if (lane != 0) return;
  const double n = static_cast<double>(R);
  const float g = fix_gamma ? 1.f : gamma[c];
  if (MODE == 0) {
    double m1 = a / n;
    double var = b / n - m1 * m1;
    if (var < 0) var = 0;
    double mean = center[c] + m1;
    float inv = static_cast<float>(1.0 / sqrt(var + eps));
    o0[c] = static_cast<float>(mean);
    o1[c] = inv;
    o2[c] = static_cast<float>(var);
    float sc = g * inv;
    o3[c] = sc;
    o4[c] = beta[c] - static_cast<float>(mean) * sc;
    // moving statistics (MXNet: moving = moving * momentum + batch * (1 - momentum), biased var)
    if (mm_upd) mm_upd[c] = mm_upd[c] * momentum + static_cast<float>(mean) * (1.f - momentum);
    if (mv_upd) mv_upd[c] = mv_upd[c] * momentum + static_cast<float>(var) * (1.f - momentum);
  } else {
    // a = sum(dz), b = sum(dz * (x - mean)); center = mean, invstd_in = invstd
    const float inv = invstd_in[c];
    const double dbeta = a;
    const double dgamma = b * inv;
    // accum: o0/o1 are the parameters' gradient buffers (grad_req write was zeroed, add accumulates)
    if (accum) {
      o0[c] += static_cast<float>(dgamma);
      o1[c] += static_cast<float>(dbeta);
    } else {
      o0[c] = static_cast<float>(dgamma);
      o1[c] = static_cast<float>(dbeta);
    }
    const double A = static_cast<double>(g) * inv;
    const double B = training ? -A * inv * dgamma / n : 0.0;
    const double Cc = training ? A * (static_cast<double>(center[c]) * inv * dgamma / n - dbeta / n) : 0.0;
    o2[c] = static_cast<float>(A);
    o3[c] = static_cast<float>(B);
    o4[c] = static_cast<float>(Cc);
  }
}

typedef unsigned int bn_u32x4 __attribute__((ext_vector_type(4)));

// tensor loads / stores of the apply kernels; nt = 1: non-temporal loads (each input is read once),
// nt = 2: non-temporal stores as well (MXAMD_BN_NT)
template <typename T>
__device__ __forceinline__ void vload(Vec8<T>& v, const T* p, int nt) {
  if constexpr (sizeof(T) == 2) {
    if (nt) {
      const bn_u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const bn_u32x4*>(p));
      v.raw = make_uint4(r.x, r.y, r.z, r.w);
      return;
    }
  }
  v.load(p);
}

template <typename T>
__device__ __forceinline__ void vstore(const Vec8<T>& v, T* p, int nt) {
  if constexpr (sizeof(T) == 2) {
    if (nt > 1) {
      const bn_u32x4 r = {v.raw.x, v.raw.y, v.raw.z, v.raw.w};
      __builtin_nontemporal_store(r, reinterpret_cast<bn_u32x4*>(p));
      return;
    }
  }
  v.store(p);
}

__device__ __forceinline__ void load8f(const float* __restrict__ p, float* o) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

// The apply kernels stream 8-element vectors with a grid-stride loop.  When the stride (blocks x 256
// threads x 8 elements, a multiple of 2048) is a multiple of C -- every C dividing 2048, i.e. all of
// ResNet's -- each thread keeps one channel group for its whole life: its per-channel coefficients are
// loaded once into registers instead of per vector (they were 2-5 extra 32-byte cache loads per 16-byte
// tensor load, L1 traffic that held these kernels near 5 TB/s), and two vectors per iteration are in
// flight.  Other C fall back to per-vector coefficient loads.

// y = x * scale + shift (+ addend) (relu)
// MASK: also write the ReLU mask, one byte per 8-element vector (bit i = y[8v+i] > 0)
template <typename T, bool ADD, bool RELU, bool MASK>
__global__ void __launch_bounds__(kBnThreads) bn_apply_kernel(
    const T* __restrict__ x, const T* __restrict__ addend, const float* __restrict__ scale,
    const float* __restrict__ shift, T* __restrict__ y, uint8_t* __restrict__ mask, int64_t nvec, int C, int nt) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  // channel of this thread's first vector; advancing by `stride` vectors moves
  // the channel by a fixed step (< C), so no per-iteration 64-bit modulo.
  int c = static_cast<int>((v * 8) % C);
  const int cstep = static_cast<int>((stride * 8) % C);
  float sc[8], sh[8];
  auto compute = [&](const Vec8<T>& vx, const Vec8<T>& va, int64_t vv) {
    Vec8<T> out;
    uint32_t bits = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float r = vx.get(i) * sc[i] + sh[i];
      if (ADD) r += va.get(i);
      if (MASK) bits |= (r > 0.f ? 1u : 0u) << i;
      if (RELU) r = r > 0.f ? r : 0.f;
      out.set(i, r);
    }
    vstore(out, y + vv * 8, nt == 2 ? 2 : 0);
    if (MASK) mask[vv] = static_cast<uint8_t>(bits);
  };
  if (cstep == 0) {
    load8f(scale + c, sc);
    load8f(shift + c, sh);
    for (; v + stride < nvec; v += 2 * stride) {
      Vec8<T> vx0, vx1, va0, va1;
      vload(vx0, x + v * 8, nt);
      vload(vx1, x + (v + stride) * 8, nt);
      if (ADD) {
        vload(va0, addend + v * 8, nt);
        vload(va1, addend + (v + stride) * 8, nt);
      }
      compute(vx0, va0, v);
      compute(vx1, va1, v + stride);
    }
    if (v < nvec) {
      Vec8<T> vx, va;
      vload(vx, x + v * 8, nt);
      if (ADD) vload(va, addend + v * 8, nt);
      compute(vx, va, v);
    }
    return;
  }
  for (; v < nvec; v += stride, c = (c + cstep >= C) ? c + cstep - C : c + cstep) {
    Vec8<T> vx, va;
    vload(vx, x + v * 8, nt);
    if (ADD) vload(va, addend + v * 8, nt);
    load8f(scale + c, sc);
    load8f(shift + c, sh);
    compute(vx, va, v);
  }
}

// dx = A*dz + B*x + Cc, dz = dy * mask (see RELU modes); optionally d_addend = dz
template <typename T, int RELU, bool WRITE_DZ>
__global__ void __launch_bounds__(kBnThreads) bn_bwd_apply_kernel(
    const T* __restrict__ x, const T* __restrict__ dy, const T* __restrict__ y, const uint8_t* __restrict__ mask,
    const float* __restrict__ A, const float* __restrict__ B, const float* __restrict__ Cc,
    const float* __restrict__ fscale, const float* __restrict__ fshift,
    T* __restrict__ dx, T* __restrict__ dz_out, int64_t nvec, int C, int nt) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  int c = static_cast<int>((v * 8) % C);
  const int cstep = static_cast<int>((stride * 8) % C);
  float fs[8], fh[8], ka[8], kb[8], kc[8];
  auto coef = [&](int cc) {
    if (RELU == kReluFromX) {
      load8f(fscale + cc, fs);
      load8f(fshift + cc, fh);
    }
    load8f(A + cc, ka);
    load8f(B + cc, kb);
    load8f(Cc + cc, kc);
  };
  struct In {
    Vec8<T> x, dy, y;
    uint32_t mb;
  };
  auto load = [&](In& in, int64_t vv) {
    vload(in.x, x + vv * 8, nt);
    vload(in.dy, dy + vv * 8, nt);
    if (RELU == kReluFromY) vload(in.y, y + vv * 8, nt);
    in.mb = RELU == kReluFromMask ? mask[vv] : 0u;
  };
  auto compute = [&](const In& in, int64_t vv) {
    Vec8<T> out, dz;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float d = in.dy.get(i);
      if (RELU == kReluFromY) d = in.y.get(i) > 0.f ? d : 0.f;
      if (RELU == kReluFromX) d = fmaf(in.x.get(i), fs[i], fh[i]) > 0.f ? d : 0.f;
      if (RELU == kReluFromMask) d = ((in.mb >> i) & 1u) ? d : 0.f;
      if (WRITE_DZ) dz.set(i, d);
      out.set(i, ka[i] * d + kb[i] * in.x.get(i) + kc[i]);
    }
    vstore(out, dx + vv * 8, nt == 2 ? 2 : 0);
    if (WRITE_DZ) vstore(dz, dz_out + vv * 8, nt >= 2 ? 2 : 0);
  };
  if (cstep == 0) {
    coef(c);
    for (; v + stride < nvec; v += 2 * stride) {
      In i0, i1;
      load(i0, v);
      load(i1, v + stride);
      compute(i0, v);
      compute(i1, v + stride);
    }
    if (v < nvec) {
      In i0;
      load(i0, v);
      compute(i0, v);
    }
    return;
  }
  for (; v < nvec; v += stride, c = (c + cstep >= C) ? c + cstep - C : c + cstep) {
    In i0;
    load(i0, v);
    coef(c);
    compute(i0, v);
  }
}

// Residual-tail backward apply (mask from the forward's bits) that also reduces the statistics of
// the BatchNorm that produced the tail's addend (a projection shortcut's BN, no ReLU): its incoming
// gradient is exactly dz, so sum(dz) and sum(dz * (z_ds - mean_ds)) are accumulated here while dz is
// in registers -- the shortcut BN's own reduction pass (a re-read of dz and z_ds) is not run.
// Geometry of bn_reduce_kernel (fixed 8-channel group per thread, rows strided by rpi).
template <typename T>
__global__ void __launch_bounds__(kBnThreads) bn_tail_bwd_ds_kernel(
    const T* __restrict__ x, const T* __restrict__ dy, const uint8_t* __restrict__ mask,
    const float* __restrict__ A, const float* __restrict__ B, const float* __restrict__ Cc, T* __restrict__ dx,
    T* __restrict__ dz_out, const T* __restrict__ zds, const float* __restrict__ mean_ds, float* __restrict__ part1,
    float* __restrict__ part2, int64_t R, int C, int tpr, int rpi, int64_t rows_per_block, int nt) {
  const int tid = threadIdx.x;
  const int lane_c = tid % tpr;
  const int lane_r = tid / tpr;
  const int cbase = blockIdx.y * tpr * 8 + lane_c * 8;
  float s1[8], s2[8], ka[8], kb[8], kc[8], km[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s1[i] = 0.f;
    s2[i] = 0.f;
    ka[i] = A[cbase + i];
    kb[i] = B[cbase + i];
    kc[i] = Cc[cbase + i];
    km[i] = mean_ds[cbase + i];
  }
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  int64_t r1 = r0 + rows_per_block;
  if (r1 > R) r1 = R;
  const bool spare = lane_r >= rpi;
  if (spare) r1 = r0;
  constexpr int UNR = 2;
  auto body = [&](const Vec8<T>& vx, const Vec8<T>& vdy, const Vec8<T>& vz, uint32_t mb, int64_t off) {
    Vec8<T> out, dz;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = ((mb >> i) & 1u) ? vdy.get(i) : 0.f;
      dz.set(i, d);
      out.set(i, ka[i] * d + kb[i] * vx.get(i) + kc[i]);
      s1[i] += d;
      s2[i] += d * (vz.get(i) - km[i]);
    }
    out.store(dx + off);
    if (dz_out != nullptr) vstore(dz, dz_out + off, nt >= 2 ? 2 : 0);   // null: the shortcut gradient stays lazy
  };
  int64_t r = r0 + lane_r;
  for (; r + (UNR - 1) * rpi < r1; r += UNR * rpi) {
    Vec8<T> vx[UNR], vdy[UNR], vz[UNR];
    uint32_t vm[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t off = (r + u * rpi) * C + cbase;
      vload(vx[u], x + off, nt);
      vload(vdy[u], dy + off, nt);
      vload(vz[u], zds + off, nt);
      vm[u] = mask[off >> 3];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) body(vx[u], vdy[u], vz[u], vm[u], (r + u * rpi) * C + cbase);
  }
  for (; r < r1; r += rpi) {
    const int64_t off = r * C + cbase;
    Vec8<T> vx, vdy, vz;
    vload(vx, x + off, nt);
    vload(vdy, dy + off, nt);
    vload(vz, zds + off, nt);
    body(vx, vdy, vz, mask[off >> 3], off);
  }
  __shared__ float sh1[kBnThreads * 8];
  __shared__ float sh2[kBnThreads * 8];
  const int cb = tpr * 8;
  if (!spare) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sh1[lane_r * cb + lane_c * 8 + i] = s1[i];
      sh2[lane_r * cb + lane_c * 8 + i] = s2[i];
    }
  }
  __syncthreads();
  for (int c = tid; c < cb; c += kBnThreads) {
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < rpi; ++rr) {
      a += sh1[rr * cb + c];
      b += sh2[rr * cb + c];
    }
    const int64_t o = static_cast<int64_t>(blockIdx.y * cb + c) * gridDim.x + blockIdx.x;
    part1[o] = a;
    part2[o] = b;
  }
}

// ---------------------------------------------------------------- launchers

// non-temporal policy of the apply kernels: their inputs are dead once applied in the step's order, so
// non-temporal loads keep them out of the Infinity Cache and leave it to the convolutions (ResNet-50 b256
// 11,308 -> 11,658 img/s in one same-box A/B, profiles/r5v_*); non-temporal stores as well measured
// as noise (profiles/r5aa_*), so the stores stay cached
static int bn_nt() { return 1; }

// workgroups of the reduction-geometry kernels (bn_reduce, bn_tail_bwd_ds): ~2 per CU (512 / 1024
// measured within noise, profiles/r5s_*)
static int bn_total_blocks() { return 512; }

static inline int64_t bn_rows_per_block(int64_t R, int C, const BnGeom& g, int* nblk,
                                        int total_blocks = bn_total_blocks(), int min_rows = 0) {
  const int cblocks = C / g.cb;
  int64_t target = total_blocks / cblocks;   // default ~2 blocks per CU; partial rows stay few
  if (target < 8) target = 8;
  int64_t rpb = (R + target - 1) / target;
  rpb = (rpb + g.rpi - 1) / g.rpi * g.rpi;
  if (rpb < g.rpi * 4) rpb = g.rpi * 4;
  if (rpb < min_rows) rpb = (min_rows + g.rpi - 1) / g.rpi * g.rpi;
  *nblk = static_cast<int>((R + rpb - 1) / rpb);
  return rpb;
}

// the residual-tail kernel with the shortcut statistics streams 4 tensors in and 2 out: it wants a
// larger grid than the 2-input reductions (measured: 1.06 -> 0.76 ms/step for 4 calls at 512 -> 1024);
// at least 64 rows per block keeps the partials small for wide layers (C = 2048: 1 block column)
static int bn_tail_blocks() { return 1024; }

int bn_tail_ds_rows(int64_t R, int C) {
  BnGeom g = bn_geom(C);
  int nblk;
  bn_rows_per_block(R, C, g, &nblk, bn_tail_blocks(), 64);
  return nblk;
}

int bn_partials_rows(int64_t R, int C) {
  BnGeom g = bn_geom(C);
  int nblk;
  bn_rows_per_block(R, C, g, &nblk);
  return nblk;
}

template <typename T>
static void bn_forward_impl(const void* x, const void* addend, void* y, uint8_t* mask, const float* gamma,
                            const float* beta, const float* center, float* part, float* mean, float* invstd,
                            float* var, float* scale, float* shift, int64_t R, int C, float eps, int training,
                            int relu, int fix_gamma, float momentum, float* mm_upd, float* mv_upd, int ext_nblk,
                            hipStream_t s) {
  MXAMD_HOST_CHECK(C % 8 == 0, "bn_nhwc: channels must be a multiple of 8");
  BnGeom g = bn_geom(C);
  MXAMD_HOST_CHECK(C % g.cb == 0, "bn_nhwc: unsupported channel count");
  if (training) {
    int nblk;
    float* p1 = part;
    if (ext_nblk > 0) {
      // statistics partials already produced by the convolution epilogue (conv_big.hip):
      // channel-major sum(x) / sum(x^2), center must be zero
      nblk = ext_nblk;
    } else {
      int64_t rpb = bn_rows_per_block(R, C, g, &nblk);
      dim3 grid(nblk, C / g.cb);
      float* p2r = part + static_cast<int64_t>(nblk) * C;
      hipLaunchKernelGGL((bn_reduce_kernel<T, 0, kReluNone>), grid, dim3(kBnThreads), 0, s,
                         static_cast<const T*>(x), nullptr, nullptr, nullptr, center, nullptr, nullptr, p1, p2r, R, C,
                         g.tpr, g.rpi, rpb);
    }
    float* p2 = part + static_cast<int64_t>(nblk) * C;
    hipLaunchKernelGGL((bn_finalize_kernel<0>), dim3((C + kFinPerBlock - 1) / kFinPerBlock), dim3(kFinThreads), 0, s, p1, p2, nblk, C, R, center, gamma,
                       beta, nullptr, eps, mean, invstd, var, scale, shift, nullptr, fix_gamma, 1, momentum, mm_upd,
                       mv_upd, 0);
  }
  // y == nullptr: statistics (and scale / shift) only -- the consumer applies them (the stem's BN + ReLU
  // folded into the max pooling, pool_nhwc.hip)
  if (y == nullptr) return;
  const int64_t nvec = R * C / 8;
  int blocks = static_cast<int>((nvec + kBnThreads - 1) / kBnThreads);
  if (blocks > 256 * 16) blocks = 256 * 16;
  const T* xa = static_cast<const T*>(x);
  const T* aa = static_cast<const T*>(addend);
  T* ya = static_cast<T*>(y);
#define APPLY(ADD, RELU, MASK)                                                                              \
  hipLaunchKernelGGL((bn_apply_kernel<T, ADD, RELU, MASK>), dim3(blocks), dim3(kBnThreads), 0, s, xa, aa, scale, \
                     shift, ya, mask, nvec, C, bn_nt())
  MXAMD_HOST_CHECK(mask == nullptr || (addend && relu), "bn_nhwc_forward: mask output only for add+relu");
  if (addend) {
    if (relu) {
      if (mask) APPLY(true, true, true); else APPLY(true, true, false);
    } else {
      APPLY(true, false, false);
    }
  } else {
    if (relu) APPLY(false, true, false); else APPLY(false, false, false);
  }
#undef APPLY
}

template <typename T>
static void bn_backward_impl(const void* x, const void* dy, const void* y, const uint8_t* mask, void* dx, void* dz,
                             const float* gamma, const float* mean, const float* invstd, const float* fscale,
                             const float* fshift, float* part, float* dgamma, float* dbeta, float* coef, int64_t R,
                             int C, int relu_mode, int fix_gamma, int training, int accum, hipStream_t s,
                             int ext_nblk, const void* ds_z, const float* ds_mean, float* ds_part) {
  BnGeom g = bn_geom(C);
  int nblk;
  int64_t rpb = bn_rows_per_block(R, C, g, &nblk);
  if (ext_nblk > 0) nblk = ext_nblk;   // sum(dz) / sum(dz*(x-mean)) partials came from the dgrad epilogue
  dim3 grid(nblk, C / g.cb);
  float* p1 = part;
  float* p2 = part + static_cast<int64_t>(nblk) * C;
  const T* xa = static_cast<const T*>(x);
  const T* dya = static_cast<const T*>(dy);
  const T* ya = static_cast<const T*>(y);
  MXAMD_HOST_CHECK(relu_mode != kReluFromY || y != nullptr, "bn_nhwc_backward: relu mask from y needs y");
  MXAMD_HOST_CHECK(relu_mode != kReluFromX || (fscale && fshift), "bn_nhwc_backward: relu-from-x needs scale/shift");
  MXAMD_HOST_CHECK(relu_mode != kReluFromMask || mask != nullptr, "bn_nhwc_backward: relu-from-mask needs the mask");
#define RED(RL)                                                                                                \
  hipLaunchKernelGGL((bn_reduce_kernel<T, 1, RL>), grid, dim3(kBnThreads), 0, s, xa, dya, ya, mask, mean, fscale, \
                     fshift,                                                                                         \
                     p1, p2, R, C, g.tpr, g.rpi, rpb)
  if (ext_nblk > 0) {
  } else if (relu_mode == kReluFromY) RED(kReluFromY);
  else if (relu_mode == kReluFromX) RED(kReluFromX);
  else if (relu_mode == kReluFromMask) RED(kReluFromMask);
  else RED(kReluNone);
#undef RED
  float* A = coef;
  float* B = coef + C;
  float* Cc = coef + 2 * C;
  hipLaunchKernelGGL((bn_finalize_kernel<1>), dim3((C + kFinPerBlock - 1) / kFinPerBlock), dim3(kFinThreads), 0, s, p1, p2, nblk, C, R, mean, gamma, nullptr,
                     invstd, 0.f, dgamma, dbeta, A, B, Cc, nullptr, fix_gamma, training, 0.f, nullptr,
                     nullptr, accum);
  const int64_t nvec = R * C / 8;
  int blocks = static_cast<int>((nvec + kBnThreads - 1) / kBnThreads);
  if (blocks > 256 * 16) blocks = 256 * 16;
  T* dxa = static_cast<T*>(dx);
  T* dza = static_cast<T*>(dz);
  if (ds_z) {
    // residual tail whose addend came from a shortcut BatchNorm: its backward statistics ride along
    MXAMD_HOST_CHECK(relu_mode == kReluFromMask && ds_mean && ds_part,
                     "bn_nhwc_backward: shortcut statistics need the tail's mask mode and the BN's mean");
    int dnblk;
    const int64_t drpb = bn_rows_per_block(R, C, g, &dnblk, bn_tail_blocks(), 64);
    hipLaunchKernelGGL((bn_tail_bwd_ds_kernel<T>), dim3(dnblk, C / g.cb), dim3(kBnThreads), 0, s, xa, dya, mask, A, B,
                       Cc, dxa, dza, static_cast<const T*>(ds_z), ds_mean, ds_part,
                       ds_part + static_cast<int64_t>(dnblk) * C, R, C, g.tpr, g.rpi, drpb, bn_nt());
    return;
  }
#define BWD(RL, WD)                                                                                      \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, RL, WD>), dim3(blocks), dim3(kBnThreads), 0, s, xa, dya, ya, mask, A, B, \
                     Cc, fscale, fshift, dxa, dza, nvec, C, bn_nt())
  if (relu_mode == kReluFromY) {
    if (dz) BWD(kReluFromY, true); else BWD(kReluFromY, false);
  } else if (relu_mode == kReluFromX) {
    if (dz) BWD(kReluFromX, true); else BWD(kReluFromX, false);
  } else if (relu_mode == kReluFromMask) {
    if (dz) BWD(kReluFromMask, true); else BWD(kReluFromMask, false);
  } else {
    if (dz) BWD(kReluNone, true); else BWD(kReluNone, false);
  }
#undef BWD
}

// Statistics pass only (per-channel partial sums of x - center): lets the conv autotuner charge a
// candidate that cannot emit BN partials from its epilogue with the pass it leaves to BatchNorm.
int bn_nhwc_stats(int dtype, const void* x, const float* center, float* part, int64_t R, int C, hipStream_t s,
                  int total_blocks) {
  MXAMD_HOST_CHECK(C % 8 == 0, "bn_nhwc: channels must be a multiple of 8");
  BnGeom g = bn_geom(C);
  MXAMD_HOST_CHECK(C % g.cb == 0, "bn_nhwc: unsupported channel count");
  int nblk;
  int64_t rpb = bn_rows_per_block(R, C, g, &nblk, total_blocks);
  dim3 grid(nblk, C / g.cb);
  float* p2 = part + static_cast<int64_t>(nblk) * C;
#define STATS(T)                                                                                              \
  hipLaunchKernelGGL((bn_reduce_kernel<T, 0, kReluNone>), grid, dim3(kBnThreads), 0, s, static_cast<const T*>(x), \
                     nullptr, nullptr, nullptr, center, nullptr, nullptr, part, p2, R, C, g.tpr, g.rpi, rpb)
  if (dtype == kF16) STATS(__half); else if (dtype == kBF16) STATS(__hip_bfloat16); else STATS(float);
#undef STATS
  return nblk;
}

// Column sums of a row-major [R][C] matrix (bias gradient of a FullyConnected layer).
// Pass 1: grid (C/64 column strips) x (row chunks), ~768 blocks even for a 4096 x 768 gradient;
// each block = 8 column vectors (16-byte loads, 64 columns) x 32 row lanes, LDS combine of the row
// lanes, one fp32 partial row per chunk.  Pass 2: per 64 columns, 4 lanes per column sum the chunks
// (coalesced rows of the partials) and write / accumulate the parameter gradient in its dtype.
namespace {
constexpr int kColsumTargetBlocks = 768;

inline void colsum_geom(int64_t R, int C, int* nchunk, int* rows_per) {
  const int strips = (C + 63) / 64;
  int64_t n = (kColsumTargetBlocks + strips - 1) / strips;
  n = std::max<int64_t>(1, std::min<int64_t>(n, (R + 31) / 32));
  int64_t rp = (R + n - 1) / n;
  rp = (rp + 31) / 32 * 32;
  *rows_per = static_cast<int>(rp);
  *nchunk = static_cast<int>((R + rp - 1) / rp);
}

template <typename T>
__global__ void __launch_bounds__(256) colsum_part_kernel(const T* __restrict__ x, int64_t R, int C, int rows_per,
                                                          float* __restrict__ part) {
  __shared__ float red[32][64 + 1];
  const int cv = threadIdx.x & 7, ty = threadIdx.x >> 3;
  const int c0 = (blockIdx.x * 8 + cv) * 8;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * rows_per;
  const int64_t r1 = r0 + rows_per < R ? r0 + rows_per : R;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < C) {
    for (int64_t r = r0 + ty; r < r1; r += 32) {
      Vec8<T> v;
      v.load(x + r * C + c0);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] += v.get(i);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[ty][cv * 8 + i] = a[i];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int col = threadIdx.x;
    float t = 0.f;
#pragma unroll 8
    for (int j = 0; j < 32; ++j) t += red[j][col];
    const int c = blockIdx.x * 64 + col;
    if (c < C) part[static_cast<int64_t>(blockIdx.y) * C + c] = t;
  }
}

template <typename TO>
__global__ void __launch_bounds__(256) colsum_fin_kernel(const float* __restrict__ part, int nchunk, int C,
                                                         TO* __restrict__ out, int accum) {
  // 16 columns x 16 lanes: each lane sums every 16th chunk (4 independent loads in flight per step)
  __shared__ float red[16][17];
  const int col = threadIdx.x & 15, l16 = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + col;
  float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
  if (c < C) {
    int i = l16;
    for (; i + 48 < nchunk; i += 64) {
      t0 += part[static_cast<int64_t>(i) * C + c];
      t1 += part[static_cast<int64_t>(i + 16) * C + c];
      t2 += part[static_cast<int64_t>(i + 32) * C + c];
      t3 += part[static_cast<int64_t>(i + 48) * C + c];
    }
    for (; i < nchunk; i += 16) t0 += part[static_cast<int64_t>(i) * C + c];
  }
  red[l16][col] = (t0 + t1) + (t2 + t3);
  __syncthreads();
  if (l16 == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) t += red[j][col];
    if (accum) t += static_cast<float>(out[c]);
    out[c] = static_cast<TO>(t);
  }
}
}  // namespace

int64_t colsum_partials(int64_t R, int C) {
  int nchunk, rows_per;
  colsum_geom(R, C, &nchunk, &rows_per);
  return static_cast<int64_t>(nchunk) * C;
}

// (A single-launch variant -- the last block of each column strip finalising after a device-scope
// fence + counter -- measured 57 us per BERT bias gradient vs ~10 us for these two launches: on a
// multi-XCD part every block's agent-scope release writes back its XCD's L2.)
void colsum_rows(int dtype, const void* x, const float* zeros, float* part, int64_t R, int C, int out_dtype,
                 void* out, int accum, hipStream_t s) {
  (void)zeros;
  MXAMD_HOST_CHECK(C % 8 == 0, "colsum_rows: columns must be a multiple of 8");
  int nchunk, rows_per;
  colsum_geom(R, C, &nchunk, &rows_per);
  const dim3 grid((C + 63) / 64, nchunk);
  if (dtype == kF16)
    hipLaunchKernelGGL(colsum_part_kernel<__half>, grid, dim3(256), 0, s, static_cast<const __half*>(x), R, C,
                       rows_per, part);
  else if (dtype == kBF16)
    hipLaunchKernelGGL(colsum_part_kernel<__hip_bfloat16>, grid, dim3(256), 0, s,
                       static_cast<const __hip_bfloat16*>(x), R, C, rows_per, part);
  else
    hipLaunchKernelGGL(colsum_part_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(x), R, C,
                       rows_per, part);
  const dim3 g2((C + 15) / 16);
  if (out_dtype == kF16)
    hipLaunchKernelGGL(colsum_fin_kernel<__half>, g2, dim3(256), 0, s, part, nchunk, C, static_cast<__half*>(out),
                       accum);
  else if (out_dtype == kBF16)
    hipLaunchKernelGGL(colsum_fin_kernel<__hip_bfloat16>, g2, dim3(256), 0, s, part, nchunk, C,
                       static_cast<__hip_bfloat16*>(out), accum);
  else
    hipLaunchKernelGGL(colsum_fin_kernel<float>, g2, dim3(256), 0, s, part, nchunk, C, static_cast<float*>(out),
                       accum);
}

void bn_nhwc_forward(int dtype, const void* x, const void* addend, void* y, uint8_t* mask, const float* gamma,
                     const float* beta,
                     const float* center, float* part, float* mean, float* invstd, float* var, float* scale,
                     float* shift, int64_t R, int C, float eps, int training, int relu, int fix_gamma,
                     float momentum, float* mm_upd, float* mv_upd, int ext_nblk, hipStream_t s) {
  switch (dtype) {
    case kF16:
      bn_forward_impl<__half>(x, addend, y, mask, gamma, beta, center, part, mean, invstd, var, scale, shift, R, C, eps,
                              training, relu, fix_gamma, momentum, mm_upd, mv_upd, ext_nblk, s);
      break;
    case kBF16:
      bn_forward_impl<__hip_bfloat16>(x, addend, y, mask, gamma, beta, center, part, mean, invstd, var, scale, shift, R,
                                      C, eps, training, relu, fix_gamma, momentum, mm_upd, mv_upd, ext_nblk, s);
      break;
    default:
      bn_forward_impl<float>(x, addend, y, mask, gamma, beta, center, part, mean, invstd, var, scale, shift, R, C, eps,
                             training, relu, fix_gamma, momentum, mm_upd, mv_upd, ext_nblk, s);
  }
}

// Backward finalize from channel-major partials part[2][C][nblk] of sum(dz), sum(dz * (x - mean)) produced by
// another kernel (the stem's fused pooling backward, pool_nhwc.hip): dgamma / dbeta (accumulated when
// accum) and the dx coefficients coef[3][C].
void bn_finalize_backward(const float* part, int nblk, int C, int64_t R, const float* mean, const float* gamma,
                          const float* invstd, float* dgamma, float* dbeta, float* coef, int fix_gamma, int training,
                          int accum, hipStream_t s) {
  hipLaunchKernelGGL((bn_finalize_kernel<1>), dim3((C + kFinPerBlock - 1) / kFinPerBlock), dim3(kFinThreads), 0, s, part,
                     part + static_cast<int64_t>(nblk) * C, nblk, C, R, mean, gamma, nullptr, invstd, 0.f, dgamma,
                     dbeta, coef, coef + C, coef + 2 * C, nullptr, fix_gamma, training, 0.f, nullptr, nullptr, accum);
}

void bn_nhwc_backward(int dtype, const void* x, const void* dy, const void* y, const uint8_t* mask, void* dx,
                      void* dz,
                      const float* gamma, const float* mean, const float* invstd, const float* fscale,
                      const float* fshift, float* part, float* dgamma, float* dbeta, float* coef, int64_t R, int C,
                      int relu_mode, int fix_gamma, int training, int accum, hipStream_t s, int ext_nblk,
                      const void* ds_z, const float* ds_mean, float* ds_part) {
  switch (dtype) {
    case kF16:
      bn_backward_impl<__half>(x, dy, y, mask, dx, dz, gamma, mean, invstd, fscale, fshift, part, dgamma, dbeta, coef, R,
                               C, relu_mode, fix_gamma, training, accum, s, ext_nblk, ds_z, ds_mean, ds_part);
      break;
    case kBF16:
      bn_backward_impl<__hip_bfloat16>(x, dy, y, mask, dx, dz, gamma, mean, invstd, fscale, fshift, part, dgamma, dbeta,
                                       coef, R, C, relu_mode, fix_gamma, training, accum, s, ext_nblk, ds_z, ds_mean,
                                       ds_part);
      break;
    default:
      bn_backward_impl<float>(x, dy, y, mask, dx, dz, gamma, mean, invstd, fscale, fshift, part, dgamma, dbeta, coef, R,
                              C, relu_mode, fix_gamma, training, accum, s, ext_nblk, ds_z, ds_mean, ds_part);
  }
}

}  // namespace mxamd
