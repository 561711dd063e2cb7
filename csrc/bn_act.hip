// Fused BatchNorm + (residual add) + (ReLU) for NHWC activations on gfx950.
//
// An NHWC activation is a row-major [M, C] matrix (M = N*H*W).  Every kernel
// uses the same thread tiling: a 256-thread block covers TPR channel groups
// (VEC channels per lane = one 16-byte load) by RPI rows per iteration, so
// loads are 16-byte vectors along the contiguous C axis and a lane's
// channels (hence its per-channel coefficients) never change.
//
// Three kernels per direction, no host-side memsets:
//
//   forward  (training): stats    -- per-block shifted sums  sum(x-K), sum((x-K)^2)
//                                    (K = x[0,c], one global shift per channel, so
//                                    |mean| >> std does not cancel), folded in LDS
//                                    and added with no-return fp32 atomics into one
//                                    of kReplicas copies of a [2, C] accumulator
//                                    (block b -> replica b % kReplicas: every
//                                    address sees P/kReplicas adds, not P --
//                                    MI355X_MICROARCH.md "Global float atomics":
//                                    all blocks on ONE row is 14x slower);
//                        finalize -- one thread per channel sums the replicas,
//                                    writes scale/shift, save_mean/invstd, the
//                                    running-stat update, and re-zeroes the
//                                    replicas (the workspace is self-cleaning);
//                        apply    -- y = act(x*scale + shift [+ r]).
//   backward:            reduce   -- sum(dz), sum(dz*(x-mean)) the same way; the
//                                    ReLU mask comes from the saved output y when
//                                    there is a residual and is recomputed from x
//                                    (x*scale+shift > 0, the forward's fp32
//                                    expression) when there is not, which saves
//                                    one activation read per pass;
//                        finalize -- dgamma/dbeta + the affine dx coefficients;
//                        apply    -- dx = k*dz + c1*x + c0, d(residual) = dz.
//
// Workspace per BN layer (fp32, zero on first use, kept zero by finalize):
//   [kReplicas][2C] forward accumulators | [kReplicas][2C] backward | [2C] forward coefs (scale, shift) | [3C] backward coefs (k, c1, c0).
// History (profiles/): v0 wrote [P][C] partials and finalised them with a
// single-block serial loop (65-73 us per launch, 7.3 ms/step); v1 put all P
// blocks' atomics on one [2C] row (165 us per stats launch: same-address
// atomics serialise at the memory side).
//
// The reference has no kernels; this is the data-plane op
// the PyTorchJob ResNet-50 worker spends most of its non-conv time in.
#include <cstdlib>

#include "bn_fin.h"
#include "common.h"
#include "kdl_api.h"
#include "tune.h"

namespace kdl {
namespace {

constexpr int kBlock = 256;
constexpr int kReplicas = 32;

template <typename PT> __device__ __forceinline__ float ldp(const PT* p, int i);
template <> __device__ __forceinline__ float ldp<float>(const float* p, int i) { return p[i]; }
template <> __device__ __forceinline__ float ldp<bf16_t>(const bf16_t* p, int i) { return bf16_to_f32(p[i]); }
template <typename PT> __device__ __forceinline__ void stp(PT* p, int i, float v);
template <> __device__ __forceinline__ void stp<float>(float* p, int i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void stp<bf16_t>(bf16_t* p, int i, float v) { p[i] = f32_to_bf16(v); }

struct Tiling {
  int TPR, RPI, gy;
};

// At most 32 lanes (512 contiguous bytes) along C per row: wide layers split
// their channels over gy blocks instead of over rows, which is what keeps the
// reduction kernels' atomics per byte low when M is small (C=2048 at 7x7).
constexpr int kMaxTPR = 32;

__host__ Tiling make_tiling(int C, int VEC) {
  int CG = C / VEC;
  Tiling t;
  t.TPR = CG < kMaxTPR ? CG : kMaxTPR;
  t.RPI = kBlock / t.TPR;
  t.gy = (CG + t.TPR - 1) / t.TPR;
  return t;
}

// workspace views
__host__ __device__ __forceinline__ float* ws_acc_fwd(float* ws, int C) { return ws; }
__host__ __device__ __forceinline__ float* ws_acc_bwd(float* ws, int C) {
  return ws + static_cast<int64_t>(kReplicas) * 2 * C;
}
__host__ __device__ __forceinline__ float* ws_coef(float* ws, int C) {
  return ws + static_cast<int64_t>(kReplicas) * 4 * C;
}
// backward coefficients (k, c1, c0) live beside the forward ones (scale, shift),
// so a weight gradient that re-applies the forward BN (GEMM prologue) may run on
// a side stream while the backward finalize of the same BN runs on the main one
__host__ __device__ __forceinline__ float* ws_bcoef(float* ws, int C) { return ws_coef(ws, C) + 2 * C; }

__device__ __forceinline__ void atomic_add_f32(float* p, float v) {
  // no-return fp32 atomic (global_atomic_add_f32 with -munsafe-fp-atomics),
  // executed at the memory side.
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Block-level fold of per-lane VEC-wide sums over the RPI row groups, then one
// atomic per channel (and per sum) from the r0 == 0 lanes into the block's replica.
template <int VEC>
__device__ __forceinline__ void block_fold_atomic(float (&a)[VEC], float (&b)[VEC], float* sh,
                                                  int t, int lc, int r0, int TPR, int RPI,
                                                  bool active, float* acc_a, float* acc_b) {
  float* sh1 = sh;
  float* sh2 = sh + kBlock * VEC;
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sh1[t * VEC + i] = a[i]; sh2[t * VEC + i] = b[i]; }
  __syncthreads();
  if (active && r0 == 0) {
    for (int rr = 1; rr < RPI; ++rr) {
      const int o = (rr * TPR + lc) * VEC;
#pragma unroll
      for (int i = 0; i < VEC; ++i) { a[i] += sh1[o + i]; b[i] += sh2[o + i]; }
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      atomic_add_f32(acc_a + i, a[i]);
      atomic_add_f32(acc_b + i, b[i]);
    }
  }
}

// ---------------------------------------------------------------- forward stats
template <typename T, int VEC>
__global__ __launch_bounds__(kBlock) void bn_fwd_stats_kernel(
    const T* __restrict__ x, int64_t M, int C, int TPR, int RPI, float* __restrict__ acc) {
  __shared__ float sh[2 * kBlock * VEC];
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int CG = C / VEC;
  const int cg = blockIdx.y * TPR + lc;
  const bool active = (r0 < RPI) && (cg < CG);
  // grid-stride rows: at any moment the whole grid streams one contiguous
  // window of the activation (DRAM-page / TLB friendly), instead of every
  // block walking its own distant chunk.
  const int64_t step = static_cast<int64_t>(gridDim.x) * RPI;
  const int c0 = cg * VEC;
  float K[VEC], s1[VEC], s2[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { K[i] = 0.f; s1[i] = 0.f; s2[i] = 0.f; }
  if (active) {
    VecIO<T, VEC>::load(x + c0, K);  // global per-channel shift K = x[0, c]
    int64_t r = static_cast<int64_t>(blockIdx.x) * RPI + r0;
    for (; r + 3 * step < M; r += 4 * step) {
      float v0[VEC], v1[VEC], v2[VEC], v3[VEC];
      VecIO<T, VEC>::load(x + r * C + c0, v0);
      VecIO<T, VEC>::load(x + (r + step) * C + c0, v1);
      VecIO<T, VEC>::load(x + (r + 2 * step) * C + c0, v2);
      VecIO<T, VEC>::load(x + (r + 3 * step) * C + c0, v3);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        float d0 = v0[i] - K[i], d1 = v1[i] - K[i], d2 = v2[i] - K[i], d3 = v3[i] - K[i];
        s1[i] += (d0 + d1) + (d2 + d3);
        s2[i] += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
      }
    }
    for (; r < M; r += step) {
      float v[VEC];
      VecIO<T, VEC>::load(x + r * C + c0, v);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        float d = v[i] - K[i];
        s1[i] += d;
        s2[i] += d * d;
      }
    }
  }
  float* rep = acc + static_cast<int64_t>(blockIdx.x % kReplicas) * 2 * C;
  block_fold_atomic<VEC>(s1, s2, sh, t, lc, r0, TPR, RPI, active, rep + c0, rep + C + c0);
}

// ---------------------------------------------------------------- forward finalize
// One thread per channel: sum the replicas, re-zero them, publish coefficients.
template <typename T, typename PT>
__global__ __launch_bounds__(kBlock) void bn_fwd_finalize_kernel(
    const T* __restrict__ x, float* __restrict__ acc, int C, float Mf, const PT* __restrict__ gamma,
    const PT* __restrict__ beta, float* __restrict__ rm, float* __restrict__ rv, float momentum,
    float eps, float* __restrict__ save_mean, float* __restrict__ save_invstd,
    float* __restrict__ coef, const float* __restrict__ ext_shift = nullptr) {
  const int ch = blockIdx.x * kBlock + threadIdx.x;
  if (ch >= C) return;
  // sums were taken around K = ext_shift[c] (GEMM-epilogue stats; may alias rm,
  // which is read here before this thread updates it) or x[0, c] (stats kernel)
  const float K = ext_shift ? ext_shift[ch] : Vec1<T>::ld(x + ch);
  // all 2 x kReplicas loads issued before any add: ONE memory round trip per
  // thread (the 8-deep unroll took four, ~5.5 us per launch, x ~53 per step)
  float va[kReplicas], vb[kReplicas];
#pragma unroll
  for (int r = 0; r < kReplicas; ++r) {
    const float* row = acc + static_cast<int64_t>(r) * 2 * C;
    va[r] = row[ch];
    vb[r] = row[C + ch];
  }
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int r = 0; r < kReplicas; ++r) {
    s1 += va[r];
    s2 += vb[r];
    float* row = acc + static_cast<int64_t>(r) * 2 * C;
    row[ch] = 0.f;
    row[C + ch] = 0.f;
  }
  const float inv_m = 1.f / Mf;
  const float m1 = s1 * inv_m;
  float var = s2 * inv_m - m1 * m1;
  var = var > 0.f ? var : 0.f;
  const float mean = K + m1;
  const float invstd = rsqrtf(var + eps);
  save_mean[ch] = mean;
  save_invstd[ch] = invstd;
  if (rm != nullptr) {
    const float unbiased = Mf > 1.f ? var * Mf / (Mf - 1.f) : var;
    rm[ch] = (1.f - momentum) * rm[ch] + momentum * mean;
    rv[ch] = (1.f - momentum) * rv[ch] + momentum * unbiased;
  }
  const float g = gamma ? ldp<PT>(gamma, ch) : 1.f;
  const float b = beta ? ldp<PT>(beta, ch) : 0.f;
  const float sc = g * invstd;
  coef[ch] = sc;
  coef[C + ch] = b - mean * sc;
}

template <typename PT>
__global__ void bn_eval_prep_kernel(int C, const PT* __restrict__ gamma, const PT* __restrict__ beta,
                                    const float* __restrict__ rm, const float* __restrict__ rv,
                                    float eps, float* __restrict__ save_mean,
                                    float* __restrict__ save_invstd, float* __restrict__ coef) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= C) return;
  const float invstd = rsqrtf(rv[ch] + eps);
  const float g = gamma ? ldp<PT>(gamma, ch) : 1.f;
  const float b = beta ? ldp<PT>(beta, ch) : 0.f;
  save_mean[ch] = rm[ch];
  save_invstd[ch] = invstd;
  coef[ch] = g * invstd;
  coef[C + ch] = b - rm[ch] * g * invstd;
}

// ---------------------------------------------------------------- forward apply
template <typename T, int VEC, bool RELU, bool RES, bool MOUT>
__global__ __launch_bounds__(kBlock) void bn_fwd_apply_kernel(
    const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y,
    uint8_t* __restrict__ mbits, const float* __restrict__ coef, int64_t M, int C, int TPR,
    int RPI) {
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int cg = blockIdx.y * TPR + lc;
  if (r0 >= RPI || cg >= C / VEC) return;
  const int c0 = cg * VEC;
  float sc[VEC], sf[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sc[i] = coef[c0 + i]; sf[i] = coef[C + c0 + i]; }
  const int64_t step = static_cast<int64_t>(gridDim.x) * RPI;
  int64_t r = static_cast<int64_t>(blockIdx.x) * RPI + r0;
  auto body = [&](int64_t row) {
    float v[VEC];
    VecIO<T, VEC>::load(x + row * C + c0, v);
    float rr[VEC];
    if constexpr (RES) VecIO<T, VEC>::load(res + row * C + c0, rr);
    uint32_t bits = 0;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float o = fmaf(v[i], sc[i], sf[i]);
      if constexpr (RES) o += rr[i];
      if constexpr (MOUT) bits |= (o > 0.f ? 1u : 0u) << i;
      if constexpr (RELU) o = o > 0.f ? o : 0.f;
      v[i] = o;
    }
    VecIO<T, VEC>::store(y + row * C + c0, v);
    // 1 bit per channel (VEC == 8: one byte per lane) = the ReLU mask the
    // backward needs, at 1/16 of the bytes of re-reading y.
    if constexpr (MOUT) mbits[row * (C / VEC) + cg] = static_cast<uint8_t>(bits);
  };
  for (; r + step < M; r += 2 * step) {  // two rows in flight per lane
    body(r);
    body(r + step);
  }
  if (r < M) body(r);
}

// ReLU-mask modes for the backward passes.
constexpr int kMaskNone = 0;  // no activation
constexpr int kMaskY = 1;     // mask = y > 0 (residual case: y saw the residual)
constexpr int kMaskX = 2;     // mask = x*scale + shift > 0 (recomputed, saves reading y)
constexpr int kMaskBits = 3;  // mask = bit i of the forward's packed byte (residual case, VEC 8)

template <typename PT, int VEC>
__device__ __forceinline__ void mask_coeffs(const PT* __restrict__ gamma, const PT* __restrict__ beta,
                                            const float* __restrict__ mean,
                                            const float* __restrict__ invstd, int c0,
                                            float (&sc)[VEC], float (&sf)[VEC]) {
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const float g = gamma ? ldp<PT>(gamma, c0 + i) : 1.f;
    const float b = beta ? ldp<PT>(beta, c0 + i) : 0.f;
    sc[i] = g * invstd[c0 + i];  // identical fp32 expressions to the forward finalize
    sf[i] = b - mean[c0 + i] * sc[i];
  }
}

// ---------------------------------------------------------------- backward reduce
template <typename T, typename PT, int VEC, int MASK>
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce_kernel(
    const T* __restrict__ dy, const T* __restrict__ y, const uint8_t* __restrict__ mbits,
    const T* __restrict__ x,
    const PT* __restrict__ gamma, const PT* __restrict__ beta, const float* __restrict__ mean,
    const float* __restrict__ invstd, int64_t M, int C, int TPR, int RPI, float* __restrict__ acc) {
  __shared__ float sh[2 * kBlock * VEC];
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int CG = C / VEC;
  const int cg = blockIdx.y * TPR + lc;
  const bool active = (r0 < RPI) && (cg < CG);
  const int64_t step = static_cast<int64_t>(gridDim.x) * RPI;  // grid-stride, as the stats kernel
  const int c0 = cg * VEC;
  float mu[VEC], sa[VEC], sb[VEC], sc[VEC], sf[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sa[i] = 0.f; sb[i] = 0.f; mu[i] = 0.f; sc[i] = 0.f; sf[i] = 0.f; }
  if (active) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) mu[i] = mean[c0 + i];
    if constexpr (MASK == kMaskX) mask_coeffs<PT, VEC>(gamma, beta, mean, invstd, c0, sc, sf);
    int64_t r = static_cast<int64_t>(blockIdx.x) * RPI + r0;
    auto body = [&](int64_t row) {
      float g[VEC], xv[VEC];
      VecIO<T, VEC>::load(dy + row * C + c0, g);
      VecIO<T, VEC>::load(x + row * C + c0, xv);
      if constexpr (MASK == kMaskY) {
        float yv[VEC];
        VecIO<T, VEC>::load(y + row * C + c0, yv);
#pragma unroll
        for (int i = 0; i < VEC; ++i) g[i] = yv[i] > 0.f ? g[i] : 0.f;
      } else if constexpr (MASK == kMaskX) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) g[i] = fmaf(xv[i], sc[i], sf[i]) > 0.f ? g[i] : 0.f;
      } else if constexpr (MASK == kMaskBits) {
        const uint32_t m = mbits[row * (C / VEC) + cg];
#pragma unroll
        for (int i = 0; i < VEC; ++i) g[i] = (m >> i) & 1u ? g[i] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        sa[i] += g[i];
        sb[i] = fmaf(g[i], xv[i] - mu[i], sb[i]);
      }
    };
    for (; r + step < M; r += 2 * step) {
      body(r);
      body(r + step);
    }
    if (r < M) body(r);
  }
  float* rep = acc + static_cast<int64_t>(blockIdx.x % kReplicas) * 2 * C;
  block_fold_atomic<VEC>(sa, sb, sh, t, lc, r0, TPR, RPI, active, rep + c0, rep + C + c0);
}

// ---------------------------------------------------------------- backward finalize
template <typename PT>
__global__ __launch_bounds__(kBlock) void bn_bwd_finalize_kernel(
    float* __restrict__ acc, int C, float Mf, const PT* __restrict__ gamma,
    const float* __restrict__ mean, const float* __restrict__ invstd, bool training,
    PT* __restrict__ dgamma, PT* __restrict__ dbeta, float* __restrict__ coef) {
  const int ch = blockIdx.x * kBlock + threadIdx.x;
  if (ch >= C) return;
  float va[kReplicas], vb[kReplicas];  // one round trip, as the forward finalize
#pragma unroll
  for (int r = 0; r < kReplicas; ++r) {
    const float* row = acc + static_cast<int64_t>(r) * 2 * C;
    va[r] = row[ch];
    vb[r] = row[C + ch];
  }
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int r = 0; r < kReplicas; ++r) {
    a += va[r];
    b += vb[r];
    float* row = acc + static_cast<int64_t>(r) * 2 * C;
    row[ch] = 0.f;
    row[C + ch] = 0.f;
  }
  const float is = invstd[ch];
  const float db = a;
  const float dg = b * is;
  if (dgamma) stp<PT>(dgamma, ch, dg);
  if (dbeta) stp<PT>(dbeta, ch, db);
  const float g = gamma ? ldp<PT>(gamma, ch) : 1.f;
  const float k = g * is;
  float c1 = 0.f, c0 = 0.f;
  if (training) {
    c1 = -k * is * dg / Mf;
    c0 = -k * db / Mf - c1 * mean[ch];
  }
  coef[ch] = k;
  coef[C + ch] = c1;
  coef[2 * C + ch] = c0;
}

// ---------------------------------------------------------------- backward apply
template <typename T, typename PT, int VEC, int MASK, bool RES>
__global__ __launch_bounds__(kBlock) void bn_bwd_apply_kernel(
    const T* __restrict__ dy, const T* __restrict__ y, const uint8_t* __restrict__ mbits,
    const T* __restrict__ x,
    const PT* __restrict__ gamma, const PT* __restrict__ beta, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ coef, T* __restrict__ dx,
    T* __restrict__ dres, int64_t M, int C, int TPR, int RPI) {
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int cg = blockIdx.y * TPR + lc;
  if (r0 >= RPI || cg >= C / VEC) return;
  const int c0 = cg * VEC;
  float k[VEC], c1[VEC], c0v[VEC], sc[VEC], sf[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    k[i] = coef[c0 + i];
    c1[i] = coef[C + c0 + i];
    c0v[i] = coef[2 * C + c0 + i];
    sc[i] = 0.f;
    sf[i] = 0.f;
  }
  if constexpr (MASK == kMaskX) mask_coeffs<PT, VEC>(gamma, beta, mean, invstd, c0, sc, sf);
  const int64_t step = static_cast<int64_t>(gridDim.x) * RPI;
  auto body = [&](int64_t row) {
    float g[VEC], xv[VEC];
    VecIO<T, VEC>::load(dy + row * C + c0, g);
    VecIO<T, VEC>::load(x + row * C + c0, xv);
    if constexpr (MASK == kMaskY) {
      float yv[VEC];
      VecIO<T, VEC>::load(y + row * C + c0, yv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) g[i] = yv[i] > 0.f ? g[i] : 0.f;
    } else if constexpr (MASK == kMaskX) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) g[i] = fmaf(xv[i], sc[i], sf[i]) > 0.f ? g[i] : 0.f;
    } else if constexpr (MASK == kMaskBits) {
      const uint32_t m = mbits[row * (C / VEC) + cg];
#pragma unroll
      for (int i = 0; i < VEC; ++i) g[i] = (m >> i) & 1u ? g[i] : 0.f;
    }
    if constexpr (RES) VecIO<T, VEC>::store(dres + row * C + c0, g);
#pragma unroll
    for (int i = 0; i < VEC; ++i) xv[i] = fmaf(k[i], g[i], fmaf(c1[i], xv[i], c0v[i]));
    VecIO<T, VEC>::store(dx + row * C + c0, xv);
  };
  int64_t r = static_cast<int64_t>(blockIdx.x) * RPI + r0;
  for (; r + step < M; r += 2 * step) {
    body(r);
    body(r + step);
  }
  if (r < M) body(r);
}

// ---------------------------------------------------------------- stem: BN + ReLU + max-pool 3x3/s2/p1
// The ResNet stem's BN output is only ever read by the max-pool, so it is
// never materialised: the forward writes the pooled map plus a 1-byte
// in-window argmax per channel (first maximum in (kh, kw) scan order, the
// tie rule of torch's NHWC max-pool, on the bf16-rounded ReLU output); the
// backward rebuilds d(relu output) at each input pixel from the <= 2x2
// windows that contain it and feeds it straight into the BN reduce/apply.
// Saves the full-resolution y write + re-read in the forward and the
// full-resolution d(y) write + two re-reads in the backward.
__device__ __forceinline__ float bf16_round(float v) { return bf16_to_f32(f32_to_bf16(v)); }

template <int VEC>
// xam (optional): the BN input x at each window's argmax -- the backward's
// BN sums then run over the pooled cells (dp * mask(xam), dp * mask * (xam -
// mean)) instead of gathering every full-resolution pixel's windows.
__global__ __launch_bounds__(kBlock) void bn_pool_fwd_kernel(
    const bf16_t* __restrict__ x, bf16_t* __restrict__ y, uint8_t* __restrict__ idx,
    const float* __restrict__ coef, int64_t MP, int C, int H, int W, int PH, int PW, int TPR,
    int RPI, bf16_t* __restrict__ xam) {
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int cg = blockIdx.y * TPR + lc;
  if (r0 >= RPI || cg >= C / VEC) return;
  const int c0 = cg * VEC;
  float sc[VEC], sf[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sc[i] = coef[c0 + i]; sf[i] = coef[C + c0 + i]; }
  const int64_t step = static_cast<int64_t>(gridDim.x) * RPI;
  for (int64_t p = static_cast<int64_t>(blockIdx.x) * RPI + r0; p < MP; p += step) {
    // 32-bit index math (host guarantees MP < 2^31): a 64-bit division per
    // element made these passes VALU-bound
    const uint32_t pu = static_cast<uint32_t>(p), phw = static_cast<uint32_t>(PH * PW);
    const int n = static_cast<int>(pu / phw);
    const int rem = static_cast<int>(pu - static_cast<uint32_t>(n) * phw);
    const int ph = rem / PW, pw = rem - (rem / PW) * PW;
    float best[VEC], bx[VEC];
    uint32_t bi[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) { best[i] = -__builtin_inff(); bi[i] = 0; bx[i] = 0.f; }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * ph - 1 + kh;
      if (ih < 0 || ih >= H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * pw - 1 + kw;
        if (iw < 0 || iw >= W) continue;
        float v[VEC];
        VecIO<bf16_t, VEC>::load(x + static_cast<int64_t>((n * H + ih) * W + iw) * C + c0, v);
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          float z = fmaf(v[i], sc[i], sf[i]);
          z = bf16_round(z > 0.f ? z : 0.f);
          if (z > best[i]) { best[i] = z; bi[i] = kh * 3 + kw; bx[i] = v[i]; }
        }
      }
    }
    VecIO<bf16_t, VEC>::store(y + p * C + c0, best);
    if (xam) VecIO<bf16_t, VEC>::store(xam + p * C + c0, bx);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      if (i < 4) lo |= bi[i] << (8 * i);
      else hi |= bi[i] << (8 * (i - 4));
    }
    if constexpr (VEC == 8) {
      *reinterpret_cast<uint2*>(idx + p * C + c0) = make_uint2(lo, hi);
    } else {
#pragma unroll
      for (int i = 0; i < VEC; ++i) idx[p * C + c0 + i] = static_cast<uint8_t>(bi[i]);
    }
  }
}

// d(relu output) at input pixel (n, h, w), channels c0..c0+VEC: the pooled
// gradients of the windows whose argmax is this pixel.
template <int VEC>
__device__ __forceinline__ void pool_grad_at(const bf16_t* __restrict__ dyp,
                                             const uint8_t* __restrict__ idx, int n, int h,
                                             int w, int C, int c0, int PH, int PW, float (&g)[VEC]) {
#pragma unroll
  for (int i = 0; i < VEC; ++i) g[i] = 0.f;
#pragma unroll
  for (int dh = 0; dh < 2; ++dh) {
    const int ph = (h + 1) / 2 - dh;
    const int kh = h + 1 - 2 * ph;
    if (ph < 0 || ph >= PH || kh > 2) continue;
#pragma unroll
    for (int dw = 0; dw < 2; ++dw) {
      const int pw = (w + 1) / 2 - dw;
      const int kw = w + 1 - 2 * pw;
      if (pw < 0 || pw >= PW || kw > 2) continue;
      const uint32_t pos = kh * 3 + kw;
      const int64_t p = static_cast<int64_t>((n * PH + ph) * PW + pw);
      uint8_t ib[VEC];
      if constexpr (VEC == 8) {
        const uint2 u = *reinterpret_cast<const uint2*>(idx + p * C + c0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          ib[i] = static_cast<uint8_t>(u.x >> (8 * i));
          ib[i + 4] = static_cast<uint8_t>(u.y >> (8 * i));
        }
      } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) ib[i] = idx[p * C + c0 + i];
      }
      float d[VEC];
      VecIO<bf16_t, VEC>::load(dyp + p * C + c0, d);
#pragma unroll
      for (int i = 0; i < VEC; ++i) g[i] += (ib[i] == pos) ? d[i] : 0.f;
    }
  }
}

template <typename PT, int VEC>
__global__ __launch_bounds__(kBlock) void bn_pool_bwd_reduce_kernel(
    const bf16_t* __restrict__ dyp, const uint8_t* __restrict__ idx, const bf16_t* __restrict__ x,
    const PT* __restrict__ gamma, const PT* __restrict__ beta, const float* __restrict__ mean,
    const float* __restrict__ invstd, int64_t M, int C, int H, int W, int PH, int PW, int TPR,
    int RPI, float* __restrict__ acc) {
  __shared__ float sh[2 * kBlock * VEC];
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int cg = blockIdx.y * TPR + lc;
  const bool active = (r0 < RPI) && (cg < C / VEC);
  const int64_t step = static_cast<int64_t>(gridDim.x) * RPI;
  const int c0 = cg * VEC;
  float mu[VEC], sa[VEC], sb[VEC], sc[VEC], sf[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sa[i] = 0.f; sb[i] = 0.f; mu[i] = 0.f; sc[i] = 0.f; sf[i] = 0.f; }
  if (active) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) mu[i] = mean[c0 + i];
    mask_coeffs<PT, VEC>(gamma, beta, mean, invstd, c0, sc, sf);
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * RPI + r0; r < M; r += step) {
      const uint32_t ru = static_cast<uint32_t>(r), hw = static_cast<uint32_t>(H * W);
      const int n = static_cast<int>(ru / hw);
      const int rem = static_cast<int>(ru - static_cast<uint32_t>(n) * hw);
      const int h = rem / W;
      float g[VEC], xv[VEC];
      VecIO<bf16_t, VEC>::load(x + r * C + c0, xv);
      pool_grad_at<VEC>(dyp, idx, n, h, rem - h * W, C, c0, PH, PW, g);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        const float gi = fmaf(xv[i], sc[i], sf[i]) > 0.f ? g[i] : 0.f;
        sa[i] += gi;
        sb[i] = fmaf(gi, xv[i] - mu[i], sb[i]);
      }
    }
  }
  float* rep = acc + static_cast<int64_t>(blockIdx.x % kReplicas) * 2 * C;
  block_fold_atomic<VEC>(sa, sb, sh, t, lc, r0, TPR, RPI, active, rep + c0, rep + C + c0);
}

template <typename PT, int VEC>
__global__ __launch_bounds__(kBlock) void bn_pool_bwd_apply_kernel(
    const bf16_t* __restrict__ dyp, const uint8_t* __restrict__ idx, const bf16_t* __restrict__ x,
    const PT* __restrict__ gamma, const PT* __restrict__ beta, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ coef, bf16_t* __restrict__ dx,
    int64_t M, int C, int H, int W, int PH, int PW, int TPR, int RPI) {
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int cg = blockIdx.y * TPR + lc;
  if (r0 >= RPI || cg >= C / VEC) return;
  const int c0 = cg * VEC;
  float k[VEC], c1[VEC], c0v[VEC], sc[VEC], sf[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    k[i] = coef[c0 + i];
    c1[i] = coef[C + c0 + i];
    c0v[i] = coef[2 * C + c0 + i];
  }
  mask_coeffs<PT, VEC>(gamma, beta, mean, invstd, c0, sc, sf);
  const int64_t step = static_cast<int64_t>(gridDim.x) * RPI;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * RPI + r0; r < M; r += step) {
    const uint32_t ru = static_cast<uint32_t>(r), hw = static_cast<uint32_t>(H * W);
    const int n = static_cast<int>(ru / hw);
    const int rem = static_cast<int>(ru - static_cast<uint32_t>(n) * hw);
    const int h = rem / W;
    float g[VEC], xv[VEC];
    VecIO<bf16_t, VEC>::load(x + r * C + c0, xv);
    pool_grad_at<VEC>(dyp, idx, n, h, rem - h * W, C, c0, PH, PW, g);
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const float gi = fmaf(xv[i], sc[i], sf[i]) > 0.f ? g[i] : 0.f;
      xv[i] = fmaf(k[i], gi, fmaf(c1[i], xv[i], c0v[i]));
    }
    VecIO<bf16_t, VEC>::store(dx + r * C + c0, xv);
  }
}

// ---------------------------------------------------------------- staged entry points (engine)
// The explicit ResNet engine (kubedl_amd/models/resnet_engine.py) splits BN into
// stages so the 1x1-conv GEMMs (conv1x1.hip) can own the reductions: the
// kernels below are the pieces the GEMM epilogues do not cover.

// out = relu(x*sc + sf + xd*scd + sfd) (+ packed mask): bottleneck output with
// the downsample branch's BN applied on the fly (its output never hits HBM).
__global__ __launch_bounds__(kBlock) void bn_fwd_apply_dual_kernel(
    const bf16_t* __restrict__ x, const float* __restrict__ coef, const bf16_t* __restrict__ xd,
    const float* __restrict__ coefd, bf16_t* __restrict__ y, uint8_t* __restrict__ mbits, int64_t M, int C,
    int TPR, int RPI) {
  constexpr int VEC = 8;
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int cg = blockIdx.y * TPR + lc;
  if (r0 >= RPI || cg >= C / VEC) return;
  const int c0 = cg * VEC;
  float sc[VEC], sf[VEC], sd[VEC], fd[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    sc[i] = coef[c0 + i]; sf[i] = coef[C + c0 + i];
    sd[i] = coefd[c0 + i]; fd[i] = coefd[C + c0 + i];
  }
  const int64_t step = static_cast<int64_t>(gridDim.x) * RPI;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * RPI + r0; r < M; r += step) {
    float v[VEC], w[VEC];
    VecIO<bf16_t, VEC>::load(x + r * C + c0, v);
    VecIO<bf16_t, VEC>::load(xd + r * C + c0, w);
    uint32_t bits = 0;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const float o = fmaf(v[i], sc[i], sf[i]) + fmaf(w[i], sd[i], fd[i]);
      bits |= (o > 0.f ? 1u : 0u) << i;
      v[i] = o > 0.f ? o : 0.f;
    }
    VecIO<bf16_t, VEC>::store(y + r * C + c0, v);
    if (mbits) mbits[r * (C / VEC) + cg] = static_cast<uint8_t>(bits);
  }
}

// dx = k g + c1 x + c0 and dxd = kd g + c1d xd + c0d: backward of the dual apply
// (g already masked), reading g once for both BN branches.
__global__ __launch_bounds__(kBlock) void bn_bwd_apply_dual_kernel(
    const bf16_t* __restrict__ g, const bf16_t* __restrict__ x, const float* __restrict__ coef,
    bf16_t* __restrict__ dx, const bf16_t* __restrict__ xd, const float* __restrict__ coefd,
    bf16_t* __restrict__ dxd, int64_t M, int C, int TPR, int RPI) {
  constexpr int VEC = 8;
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int cg = blockIdx.y * TPR + lc;
  if (r0 >= RPI || cg >= C / VEC) return;
  const int c0 = cg * VEC;
  float k[VEC], c1[VEC], cz[VEC], kd[VEC], c1d[VEC], czd[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    k[i] = coef[c0 + i]; c1[i] = coef[C + c0 + i]; cz[i] = coef[2 * C + c0 + i];
    kd[i] = coefd[c0 + i]; c1d[i] = coefd[C + c0 + i]; czd[i] = coefd[2 * C + c0 + i];
  }
  const int64_t step = static_cast<int64_t>(gridDim.x) * RPI;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * RPI + r0; r < M; r += step) {
    float gv[VEC], xv[VEC], wv[VEC];
    VecIO<bf16_t, VEC>::load(g + r * C + c0, gv);
    VecIO<bf16_t, VEC>::load(x + r * C + c0, xv);
    VecIO<bf16_t, VEC>::load(xd + r * C + c0, wv);
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      xv[i] = fmaf(k[i], gv[i], fmaf(c1[i], xv[i], cz[i]));
      wv[i] = fmaf(kd[i], gv[i], fmaf(c1d[i], wv[i], czd[i]));
    }
    VecIO<bf16_t, VEC>::store(dx + r * C + c0, xv);
    VecIO<bf16_t, VEC>::store(dxd + r * C + c0, wv);
  }
}

// g = dy * mask-bit, written out, plus sum(g), sum(g (x - mean)) into the
// backward replicas (standalone form of the conv1x1 RESBITS epilogue, for the
// last bottleneck whose gradient comes from the pooling head).  dy may be a
// per-image broadcast: dy_rows_per_img > 0 means dy is [M / rows, C] scaled by
// dy_scale (global average pool backward folded in).
__global__ __launch_bounds__(kBlock) void bn_bwd_mask_reduce_kernel(
    const bf16_t* __restrict__ dy, int dy_rows_per_img, float dy_scale, const uint8_t* __restrict__ mbits,
    const bf16_t* __restrict__ x, const float* __restrict__ mean, bf16_t* __restrict__ gout, int64_t M, int C,
    int TPR, int RPI, float* __restrict__ acc, const bf16_t* __restrict__ x2, const float* __restrict__ mean2,
    float* __restrict__ acc2) {
  constexpr int VEC = 8;
  __shared__ float sh[2 * kBlock * VEC];
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int CG = C / VEC;
  const int cg = blockIdx.y * TPR + lc;
  const bool active = (r0 < RPI) && (cg < CG);
  const int64_t step = static_cast<int64_t>(gridDim.x) * RPI;
  const int c0 = cg * VEC;
  float mu[VEC], sa[VEC], sb[VEC], mu2[VEC], sb2[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sa[i] = 0.f; sb[i] = 0.f; mu[i] = 0.f; mu2[i] = 0.f; sb2[i] = 0.f; }
  if (active) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      mu[i] = mean[c0 + i];
      if (x2) mu2[i] = mean2[c0 + i];
    }
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * RPI + r0; r < M; r += step) {
      float g[VEC], xv[VEC];
      if (dy_rows_per_img > 0) {
        VecIO<bf16_t, VEC>::load(dy + (r / dy_rows_per_img) * C + c0, g);
#pragma unroll
        for (int i = 0; i < VEC; ++i) g[i] = bf16_to_f32(f32_to_bf16(g[i] * dy_scale));
      } else {
        VecIO<bf16_t, VEC>::load(dy + r * C + c0, g);
      }
      VecIO<bf16_t, VEC>::load(x + r * C + c0, xv);
      const uint32_t m = mbits[r * CG + cg];
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        g[i] = (m >> i) & 1u ? g[i] : 0.f;
        sa[i] += g[i];
        sb[i] = fmaf(g[i], xv[i] - mu[i], sb[i]);
      }
      VecIO<bf16_t, VEC>::store(gout + r * C + c0, g);
      if (x2) {  // second BN fed by the same gradient (downsample branch)
        float xw[VEC];
        VecIO<bf16_t, VEC>::load(x2 + r * C + c0, xw);
#pragma unroll
        for (int i = 0; i < VEC; ++i) sb2[i] = fmaf(g[i], xw[i] - mu2[i], sb2[i]);
      }
    }
  }
  float* rep = acc + static_cast<int64_t>(blockIdx.x % kReplicas) * 2 * C;
  if (x2) {
    float* rep2 = acc2 + static_cast<int64_t>(blockIdx.x % kReplicas) * 2 * C;
    float sa2[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) sa2[i] = sa[i];
    block_fold_atomic<VEC>(sa2, sb2, sh, t, lc, r0, TPR, RPI, active, rep2 + c0, rep2 + C + c0);
    __syncthreads();
  }
  block_fold_atomic<VEC>(sa, sb, sh, t, lc, r0, TPR, RPI, active, rep + c0, rep + C + c0);
}

// ---------------------------------------------------------------- host side
struct ReducePlan {
  Tiling tl;
  int gx;
  int64_t rows_per_block;
};

// Up to 1024 blocks to fill 256 CUs several times (Guideline 11), but every
// block covers >= kMinRows rows: a block issues 2 atomics per channel it owns, so
// rows-per-block IS the bytes-per-atomic ratio (v3 used 16 rows per lane:
// C=2048 at 7x7 ran at 0.5 TB/s, bound by 3.2M memory-side atomics).
ReducePlan plan_reduce(int64_t M, int C, int VEC) {
  ReducePlan p;
  p.tl = make_tiling(C, VEC);
  int64_t target = 1024 / p.tl.gy;
  if (target < 1) target = 1;
  static const int64_t kMinRows = tune_int("bn_min_rows", 128);  // sweep knob; default measured best
  int64_t min_rows = static_cast<int64_t>(p.tl.RPI) * 16;
  if (min_rows < kMinRows) min_rows = kMinRows;
  int64_t gx = (M + min_rows - 1) / min_rows;
  if (gx > target) gx = target;
  if (gx < 1) gx = 1;
  int64_t rpb = (M + gx - 1) / gx;
  rpb = ((rpb + p.tl.RPI - 1) / p.tl.RPI) * p.tl.RPI;
  if (rpb < 1) rpb = 1;
  p.rows_per_block = rpb;
  p.gx = static_cast<int>((M + rpb - 1) / rpb);
  if (p.gx < 1) p.gx = 1;
  return p;
}

int apply_gx(int64_t M, const Tiling& tl) {
  int64_t rows_per_it = tl.RPI;
  int64_t cap = 2048 / tl.gy;
  if (cap < 1) cap = 1;
  int64_t gx = (M + rows_per_it * 2 - 1) / (rows_per_it * 2);
  if (gx > cap) gx = cap;
  if (gx < 1) gx = 1;
  return static_cast<int>(gx);
}

template <typename T, int VEC, typename PT>
hipError_t fwd_impl(const T* x, const T* res, T* y, uint8_t* mbits, const PT* gamma, const PT* beta, float* rm,
                    float* rv, float* save_mean, float* save_invstd, float* ws, int64_t M, int C,
                    bool relu, bool training, float momentum, float eps, hipStream_t s) {
  ReducePlan rp = plan_reduce(M, C, VEC);
  float* acc = ws_acc_fwd(ws, C);
  float* coef = ws_coef(ws, C);
  const int fin_grid = (C + kBlock - 1) / kBlock;
  if (training) {
    hipLaunchKernelGGL((bn_fwd_stats_kernel<T, VEC>), dim3(rp.gx, rp.tl.gy), dim3(kBlock), 0, s,
                       x, M, C, rp.tl.TPR, rp.tl.RPI, acc);
    hipLaunchKernelGGL((bn_fwd_finalize_kernel<T, PT>), dim3(fin_grid), dim3(kBlock), 0, s, x, acc,
                       C, static_cast<float>(M), gamma, beta, rm, rv, momentum, eps, save_mean,
                       save_invstd, coef);
  } else {
    hipLaunchKernelGGL((bn_eval_prep_kernel<PT>), dim3(fin_grid), dim3(kBlock), 0, s, C, gamma,
                       beta, rm, rv, eps, save_mean, save_invstd, coef);
  }
  dim3 grid(apply_gx(M, rp.tl), rp.tl.gy);
#define BN_LAUNCH_FWD_APPLY(R, S, MO)                                                             \
  hipLaunchKernelGGL((bn_fwd_apply_kernel<T, VEC, R, S, MO>), grid, dim3(kBlock), 0, s, x, res, \
                     y, mbits, coef, M, C, rp.tl.TPR, rp.tl.RPI)
  if constexpr (VEC == 8) {
    if (relu && res && mbits) {
      BN_LAUNCH_FWD_APPLY(true, true, true);
      return hipGetLastError();
    }
  }
  if (relu && res) BN_LAUNCH_FWD_APPLY(true, true, false);
  else if (relu) BN_LAUNCH_FWD_APPLY(true, false, false);
  else if (res) BN_LAUNCH_FWD_APPLY(false, true, false);
  else BN_LAUNCH_FWD_APPLY(false, false, false);
#undef BN_LAUNCH_FWD_APPLY
  return hipGetLastError();
}

template <typename T, int VEC, typename PT, int MASK>
void bwd_launch(const ReducePlan& rp, const T* dy, const T* y, const uint8_t* mbits, const T* x, const PT* gamma,
                const PT* beta, const float* mean, const float* invstd, T* dx, T* dres, PT* dgamma,
                PT* dbeta, float* ws, int64_t M, int C, bool training, hipStream_t s) {
  float* acc = ws_acc_bwd(ws, C);
  float* coef = ws_bcoef(ws, C);
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, PT, VEC, MASK>), dim3(rp.gx, rp.tl.gy), dim3(kBlock),
                     0, s, dy, y, mbits, x, gamma, beta, mean, invstd, M, C, rp.tl.TPR, rp.tl.RPI, acc);
  hipLaunchKernelGGL((bn_bwd_finalize_kernel<PT>), dim3((C + kBlock - 1) / kBlock), dim3(kBlock), 0,
                     s, acc, C, static_cast<float>(M), gamma, mean, invstd, training, dgamma, dbeta,
                     coef);
  dim3 grid(apply_gx(M, rp.tl), rp.tl.gy);
  if (dres)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, PT, VEC, MASK, true>), grid, dim3(kBlock), 0, s, dy,
                       y, mbits, x, gamma, beta, mean, invstd, coef, dx, dres, M, C, rp.tl.TPR, rp.tl.RPI);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, PT, VEC, MASK, false>), grid, dim3(kBlock), 0, s,
                       dy, y, mbits, x, gamma, beta, mean, invstd, coef, dx, dres, M, C, rp.tl.TPR,
                       rp.tl.RPI);
}

template <typename T, int VEC, typename PT>
hipError_t bwd_impl(const T* dy, const T* y, const uint8_t* mbits, const T* x, const PT* gamma, const PT* beta,
                    const float* mean, const float* invstd, T* dx, T* dres, PT* dgamma, PT* dbeta,
                    float* ws, int64_t M, int C, bool relu, bool training, hipStream_t s) {
  ReducePlan rp = plan_reduce(M, C, VEC);
#define BN_LAUNCH_BWD(MODE)                                                                        \
  bwd_launch<T, VEC, PT, MODE>(rp, dy, y, mbits, x, gamma, beta, mean, invstd, dx, dres, dgamma, \
                               dbeta, ws, M, C, training, s)
  if (!relu) BN_LAUNCH_BWD(kMaskNone);
  else if (mbits != nullptr && VEC == 8) BN_LAUNCH_BWD(kMaskBits);
  // with a residual the mask must come from y (it saw the residual); without
  // one it is recomputed from x (y is not read)
  else if (dres == nullptr && beta != nullptr) BN_LAUNCH_BWD(kMaskX);
  else if (y != nullptr) BN_LAUNCH_BWD(kMaskY);
  else return hipErrorInvalidValue;
#undef BN_LAUNCH_BWD
  return hipGetLastError();
}

}  // namespace

int64_t bn_workspace_floats(int C) {  // + the folded-finalize descriptor and tile counters (bn_fin.h)
  return static_cast<int64_t>(kReplicas) * 4 * C + 5 * static_cast<int64_t>(C) + kFinDescFloats + kFinCounters;
}

#define BN_DISPATCH_PT(pdtype, ...)              \
  do {                                           \
    if ((pdtype) == 1) {                         \
      using PT = bf16_t;                         \
      __VA_ARGS__;                               \
    } else {                                     \
      using PT = float;                          \
      __VA_ARGS__;                               \
    }                                            \
  } while (0)

#define BN_DISPATCH_T(dtype, C, ...)                                      \
  do {                                                                     \
    if ((dtype) == 1) {                                                    \
      using T = bf16_t;                                                    \
      if ((C) % 8 == 0) { constexpr int VEC = 8; __VA_ARGS__; }            \
      else { constexpr int VEC = 1; __VA_ARGS__; }                         \
    } else {                                                               \
      using T = float;                                                     \
      if ((C) % 4 == 0) { constexpr int VEC = 4; __VA_ARGS__; }            \
      else { constexpr int VEC = 1; __VA_ARGS__; }                         \
    }                                                                      \
  } while (0)

hipError_t bn_act_forward(const void* x, const void* res, void* y, uint8_t* mbits, const void* gamma,
                          const void* beta, float* rm, float* rv, float* save_mean,
                          float* save_invstd, float* ws, int64_t M, int C, int dtype, int pdtype,
                          bool relu, bool training, float momentum, float eps, hipStream_t s) {
  if (M <= 0 || C <= 0) return hipSuccess;
  hipError_t e = hipSuccess;
  BN_DISPATCH_PT(pdtype, BN_DISPATCH_T(dtype, C, {
    e = fwd_impl<T, VEC, PT>(static_cast<const T*>(x), static_cast<const T*>(res),
                             static_cast<T*>(y), mbits, static_cast<const PT*>(gamma),
                             static_cast<const PT*>(beta), rm, rv, save_mean, save_invstd, ws, M,
                             C, relu, training, momentum, eps, s);
  }));
  return e;
}

hipError_t bn_act_backward(const void* dy, const void* y, const uint8_t* mbits, const void* x, const void* gamma,
                           const void* beta, const float* mean, const float* invstd, void* dx,
                           void* dres, void* dgamma, void* dbeta, float* ws, int64_t M, int C,
                           int dtype, int pdtype, bool relu, bool training, hipStream_t s) {
  if (M <= 0 || C <= 0) return hipSuccess;
  hipError_t e = hipSuccess;
  BN_DISPATCH_PT(pdtype, BN_DISPATCH_T(dtype, C, {
    e = bwd_impl<T, VEC, PT>(static_cast<const T*>(dy), static_cast<const T*>(y), mbits,
                             static_cast<const T*>(x), static_cast<const PT*>(gamma),
                             static_cast<const PT*>(beta), mean, invstd, static_cast<T*>(dx),
                             static_cast<T*>(dres), static_cast<PT*>(dgamma),
                             static_cast<PT*>(dbeta), ws, M, C, relu, training, s);
  }));
  return e;
}


hipError_t bn_pool_forward(const void* x, void* y, uint8_t* idx, const void* gamma, const void* beta,
                           float* rm, float* rv, float* save_mean, float* save_invstd, float* ws,
                           int N, int H, int W, int C, int pdtype, bool training, float momentum,
                           float eps, hipStream_t s, bool gemm_stats, void* xam) {
  if (N <= 0 || C <= 0 || C % 8 != 0) return hipErrorInvalidValue;
  constexpr int VEC = 8;
  const int64_t M = static_cast<int64_t>(N) * H * W;
  if (M >= (int64_t(1) << 31)) return hipErrorInvalidValue;  // 32-bit pixel index math
  const int PH = (H - 1) / 2 + 1, PW = (W - 1) / 2 + 1;  // k3 s2 p1
  const int64_t MP = static_cast<int64_t>(N) * PH * PW;
  ReducePlan rp = plan_reduce(M, C, VEC);
  float* acc = ws_acc_fwd(ws, C);
  float* coef = ws_coef(ws, C);
  const int fin_grid = (C + kBlock - 1) / kBlock;
  const bf16_t* xb = static_cast<const bf16_t*>(x);
  BN_DISPATCH_PT(pdtype, {
    if (training && gemm_stats) {  // sums around rm already in acc (conv epilogue, csrc/stem.hip)
      hipLaunchKernelGGL((bn_fwd_finalize_kernel<bf16_t, PT>), dim3(fin_grid), dim3(kBlock), 0, s,
                         static_cast<const bf16_t*>(nullptr), acc, C, static_cast<float>(M),
                         static_cast<const PT*>(gamma), static_cast<const PT*>(beta), rm, rv, momentum, eps,
                         save_mean, save_invstd, coef, rm);
    } else if (training) {
      hipLaunchKernelGGL((bn_fwd_stats_kernel<bf16_t, VEC>), dim3(rp.gx, rp.tl.gy), dim3(kBlock), 0, s,
                         xb, M, C, rp.tl.TPR, rp.tl.RPI, acc);
      hipLaunchKernelGGL((bn_fwd_finalize_kernel<bf16_t, PT>), dim3(fin_grid), dim3(kBlock), 0, s, xb,
                         acc, C, static_cast<float>(M), static_cast<const PT*>(gamma),
                         static_cast<const PT*>(beta), rm, rv, momentum, eps, save_mean, save_invstd,
                         coef);
    } else {
      hipLaunchKernelGGL((bn_eval_prep_kernel<PT>), dim3(fin_grid), dim3(kBlock), 0, s, C,
                         static_cast<const PT*>(gamma), static_cast<const PT*>(beta), rm, rv, eps,
                         save_mean, save_invstd, coef);
    }
  });
  dim3 grid(apply_gx(MP, rp.tl), rp.tl.gy);
  hipLaunchKernelGGL((bn_pool_fwd_kernel<VEC>), grid, dim3(kBlock), 0, s, xb,
                     static_cast<bf16_t*>(y), idx, coef, MP, C, H, W, PH, PW, rp.tl.TPR, rp.tl.RPI,
                     static_cast<bf16_t*>(xam));
  return hipGetLastError();
}

hipError_t bn_pool_backward(const void* dyp, const uint8_t* idx, const void* x, const void* gamma,
                            const void* beta, const float* mean, const float* invstd, void* dx,
                            void* dgamma, void* dbeta, float* ws, int N, int H, int W, int C,
                            int pdtype, bool training, hipStream_t s, bool with_dx) {
  if (N <= 0 || C <= 0 || C % 8 != 0) return hipErrorInvalidValue;
  constexpr int VEC = 8;
  const int64_t M = static_cast<int64_t>(N) * H * W;
  if (M >= (int64_t(1) << 31)) return hipErrorInvalidValue;  // 32-bit pixel index math
  const int PH = (H - 1) / 2 + 1, PW = (W - 1) / 2 + 1;
  ReducePlan rp = plan_reduce(M, C, VEC);
  float* acc = ws_acc_bwd(ws, C);
  float* coef = ws_bcoef(ws, C);
  const bf16_t* db = static_cast<const bf16_t*>(dyp);
  const bf16_t* xb = static_cast<const bf16_t*>(x);
  BN_DISPATCH_PT(pdtype, {
    const PT* g = static_cast<const PT*>(gamma);
    const PT* b = static_cast<const PT*>(beta);
    hipLaunchKernelGGL((bn_pool_bwd_reduce_kernel<PT, VEC>), dim3(rp.gx, rp.tl.gy), dim3(kBlock), 0, s,
                       db, idx, xb, g, b, mean, invstd, M, C, H, W, PH, PW, rp.tl.TPR, rp.tl.RPI, acc);
    hipLaunchKernelGGL((bn_bwd_finalize_kernel<PT>), dim3((C + kBlock - 1) / kBlock), dim3(kBlock), 0,
                       s, acc, C, static_cast<float>(M), g, mean, invstd, training,
                       static_cast<PT*>(dgamma), static_cast<PT*>(dbeta), coef);
    if (with_dx) {  // else the consumer applies the coefficients itself (csrc/stem.hip)
      dim3 grid(apply_gx(M, rp.tl), rp.tl.gy);
      hipLaunchKernelGGL((bn_pool_bwd_apply_kernel<PT, VEC>), grid, dim3(kBlock), 0, s, db, idx, xb, g, b,
                         mean, invstd, coef, static_cast<bf16_t*>(dx), M, C, H, W, PH, PW, rp.tl.TPR,
                         rp.tl.RPI);
    }
  });
  return hipGetLastError();
}


// ---------------------------------------------------------------- staged host entry points (bf16 NHWC, C % 8 == 0)
hipError_t bn_stage_fwd_stats(const void* x, float* ws, int64_t M, int C, hipStream_t s) {
  if (M <= 0 || C % 8) return hipErrorInvalidValue;
  ReducePlan rp = plan_reduce(M, C, 8);
  hipLaunchKernelGGL((bn_fwd_stats_kernel<bf16_t, 8>), dim3(rp.gx, rp.tl.gy), dim3(kBlock), 0, s,
                     static_cast<const bf16_t*>(x), M, C, rp.tl.TPR, rp.tl.RPI, ws_acc_fwd(ws, C));
  return hipGetLastError();
}

hipError_t bn_stage_fwd_finalize(const void* x, const float* shift, float* ws, int64_t M, int C, const void* gamma,
                                 const void* beta, float* rm, float* rv, float* save_mean, float* save_invstd,
                                 int pdtype, bool training, float momentum, float eps, hipStream_t s) {
  const int fin_grid = (C + kBlock - 1) / kBlock;
  float* coef = ws_coef(ws, C);
  BN_DISPATCH_PT(pdtype, {
    if (training)
      hipLaunchKernelGGL((bn_fwd_finalize_kernel<bf16_t, PT>), dim3(fin_grid), dim3(kBlock), 0, s,
                         static_cast<const bf16_t*>(x), ws_acc_fwd(ws, C), C, static_cast<float>(M),
                         static_cast<const PT*>(gamma), static_cast<const PT*>(beta), rm, rv, momentum, eps,
                         save_mean, save_invstd, coef, shift);
    else
      hipLaunchKernelGGL((bn_eval_prep_kernel<PT>), dim3(fin_grid), dim3(kBlock), 0, s, C,
                         static_cast<const PT*>(gamma), static_cast<const PT*>(beta), rm, rv, eps, save_mean,
                         save_invstd, coef);
  });
  return hipGetLastError();
}

const float* bn_stage_coef(const float* ws, int C) { return ws + static_cast<int64_t>(kReplicas) * 4 * C; }

hipError_t bn_stage_fwd_apply(const void* x, const float* ws, const void* res, const void* xd, const float* wsd,
                              void* y, uint8_t* mbits, int64_t M, int C, bool relu, hipStream_t s) {
  if (M <= 0 || C % 8) return hipErrorInvalidValue;
  const Tiling tl = make_tiling(C, 8);
  dim3 grid(apply_gx(M, tl), tl.gy);
  const bf16_t* xb = static_cast<const bf16_t*>(x);
  bf16_t* yb = static_cast<bf16_t*>(y);
  const float* coef = ws_coef(const_cast<float*>(ws), C);
  if (xd) {
    if (!relu) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_fwd_apply_dual_kernel, grid, dim3(kBlock), 0, s, xb, coef,
                       static_cast<const bf16_t*>(xd), ws_coef(const_cast<float*>(wsd), C), yb, mbits, M, C,
                       tl.TPR, tl.RPI);
    return hipGetLastError();
  }
  const bf16_t* rb = static_cast<const bf16_t*>(res);
#define BN_LAUNCH_APPLY(R, S, MO)                                                                              \
  hipLaunchKernelGGL((bn_fwd_apply_kernel<bf16_t, 8, R, S, MO>), grid, dim3(kBlock), 0, s, xb, rb, yb, mbits, \
                     coef, M, C, tl.TPR, tl.RPI)
  if (relu && rb && mbits) BN_LAUNCH_APPLY(true, true, true);
  else if (relu && rb) BN_LAUNCH_APPLY(true, true, false);
  else if (relu) BN_LAUNCH_APPLY(true, false, false);
  else if (rb) BN_LAUNCH_APPLY(false, true, false);
  else BN_LAUNCH_APPLY(false, false, false);
#undef BN_LAUNCH_APPLY
  return hipGetLastError();
}

hipError_t bn_stage_bwd_mask_reduce(const void* dy, int dy_rows_per_img, float dy_scale, const uint8_t* mbits,
                                    const void* x, const float* mean, void* gout, float* ws, int64_t M, int C,
                                    const void* x2, const float* mean2, float* ws2, hipStream_t s) {
  if (M <= 0 || C % 8) return hipErrorInvalidValue;
  ReducePlan rp = plan_reduce(M, C, 8);
  hipLaunchKernelGGL(bn_bwd_mask_reduce_kernel, dim3(rp.gx, rp.tl.gy), dim3(kBlock), 0, s,
                     static_cast<const bf16_t*>(dy), dy_rows_per_img, dy_scale, mbits,
                     static_cast<const bf16_t*>(x), mean, static_cast<bf16_t*>(gout), M, C, rp.tl.TPR, rp.tl.RPI,
                     ws_acc_bwd(ws, C), static_cast<const bf16_t*>(x2), mean2, x2 ? ws_acc_bwd(ws2, C) : nullptr);
  return hipGetLastError();
}

hipError_t bn_stage_bwd_reduce(const void* dy, const void* x, const void* gamma, const void* beta, const float* mean,
                               const float* invstd, float* ws, int64_t M, int C, bool relu_mask_x, int pdtype,
                               hipStream_t s) {
  if (M <= 0 || C % 8) return hipErrorInvalidValue;
  ReducePlan rp = plan_reduce(M, C, 8);
  BN_DISPATCH_PT(pdtype, {
    const PT* g = static_cast<const PT*>(gamma);
    const PT* b = static_cast<const PT*>(beta);
    if (relu_mask_x)
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<bf16_t, PT, 8, kMaskX>), dim3(rp.gx, rp.tl.gy), dim3(kBlock), 0, s,
                         static_cast<const bf16_t*>(dy), nullptr, nullptr, static_cast<const bf16_t*>(x), g, b, mean,
                         invstd, M, C, rp.tl.TPR, rp.tl.RPI, ws_acc_bwd(ws, C));
    else
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<bf16_t, PT, 8, kMaskNone>), dim3(rp.gx, rp.tl.gy), dim3(kBlock), 0, s,
                         static_cast<const bf16_t*>(dy), nullptr, nullptr, static_cast<const bf16_t*>(x), g, b, mean,
                         invstd, M, C, rp.tl.TPR, rp.tl.RPI, ws_acc_bwd(ws, C));
  });
  return hipGetLastError();
}

hipError_t bn_stage_bwd_apply_maskx(const void* dy, const void* x, const void* gamma, const void* beta,
                                    const float* mean, const float* invstd, const float* ws, void* dx, int64_t M,
                                    int C, int pdtype, hipStream_t s) {
  if (M <= 0 || C % 8) return hipErrorInvalidValue;
  const Tiling tl = make_tiling(C, 8);
  dim3 grid(apply_gx(M, tl), tl.gy);
  const float* coef = ws_bcoef(const_cast<float*>(ws), C);
  BN_DISPATCH_PT(pdtype, {
    hipLaunchKernelGGL((bn_bwd_apply_kernel<bf16_t, PT, 8, kMaskX, false>), grid, dim3(kBlock), 0, s,
                       static_cast<const bf16_t*>(dy), nullptr, nullptr, static_cast<const bf16_t*>(x),
                       static_cast<const PT*>(gamma), static_cast<const PT*>(beta), mean, invstd, coef,
                       static_cast<bf16_t*>(dx), nullptr, M, C, tl.TPR, tl.RPI);
  });
  return hipGetLastError();
}

hipError_t bn_stage_bwd_finalize(float* ws, int64_t M, int C, const void* gamma, const float* mean,
                                 const float* invstd, void* dgamma, void* dbeta, int pdtype, bool training,
                                 hipStream_t s) {
  BN_DISPATCH_PT(pdtype, {
    hipLaunchKernelGGL((bn_bwd_finalize_kernel<PT>), dim3((C + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                       ws_acc_bwd(ws, C), C, static_cast<float>(M), static_cast<const PT*>(gamma), mean, invstd,
                       training, static_cast<PT*>(dgamma), static_cast<PT*>(dbeta), ws_bcoef(ws, C));
  });
  return hipGetLastError();
}

hipError_t bn_stage_bwd_apply(const void* g, const void* x, const float* ws, void* dx, const void* xd,
                              const float* wsd, void* dxd, int64_t M, int C, hipStream_t s) {
  if (M <= 0 || C % 8) return hipErrorInvalidValue;
  const Tiling tl = make_tiling(C, 8);
  dim3 grid(apply_gx(M, tl), tl.gy);
  const float* coef = ws_bcoef(const_cast<float*>(ws), C);
  if (xd) {
    hipLaunchKernelGGL(bn_bwd_apply_dual_kernel, grid, dim3(kBlock), 0, s, static_cast<const bf16_t*>(g),
                       static_cast<const bf16_t*>(x), coef, static_cast<bf16_t*>(dx),
                       static_cast<const bf16_t*>(xd), ws_bcoef(const_cast<float*>(wsd), C),
                       static_cast<bf16_t*>(dxd), M, C, tl.TPR, tl.RPI);
  } else {
    hipLaunchKernelGGL((bn_bwd_apply_kernel<bf16_t, bf16_t, 8, kMaskNone, false>), grid, dim3(kBlock), 0, s,
                       static_cast<const bf16_t*>(g), nullptr, nullptr, static_cast<const bf16_t*>(x), nullptr,
                       nullptr, nullptr, nullptr, coef, static_cast<bf16_t*>(dx), nullptr, M, C, tl.TPR, tl.RPI);
  }
  return hipGetLastError();
}

}  // namespace kdl
