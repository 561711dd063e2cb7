// Fused BatchNorm + (residual add) + (ReLU) for NHWC activations on gfx950.
//
// An NHWC activation is a row-major [M, C] matrix (M = N*H*W).  Every kernel
// here uses the same thread tiling: a 256-thread block covers TPR channel
// groups (VEC channels per lane, 16 bytes per load) by RPI rows per
// iteration, so loads are 16-byte vectors along the contiguous C axis and a
// lane's channels (hence its per-channel coefficients) never change.
//
// Forward (training):  stats partials (shifted sums per block, merged across
//   blocks with Chan's parallel variance formula) -> finalize (mean, invstd,
//   running-stat update, scale/shift) -> apply (y = act(x*scale+shift [+r])).
// Backward: reduce partials of sum(dz), sum(dz*(x-mean)) with the ReLU mask
//   taken from the saved output y -> finalize (dgamma, dbeta, affine dx
//   coefficients) -> apply (dx = a*dz + c1*x + c0, d(residual) = dz).
//
// The reference has no kernels; this is the data-plane op
// the PyTorchJob ResNet-50 worker spends most of its non-conv time in.
#include "common.h"
#include "kdl_api.h"

#include <tuple>

namespace kdl {
namespace {

constexpr int kBlock = 256;

template <typename PT> __device__ __forceinline__ float ldp(const PT* p, int i);
template <> __device__ __forceinline__ float ldp<float>(const float* p, int i) { return p[i]; }
template <> __device__ __forceinline__ float ldp<bf16_t>(const bf16_t* p, int i) { return bf16_to_f32(p[i]); }
template <typename PT> __device__ __forceinline__ void stp(PT* p, int i, float v);
template <> __device__ __forceinline__ void stp<float>(float* p, int i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void stp<bf16_t>(bf16_t* p, int i, float v) { p[i] = f32_to_bf16(v); }

struct Tiling {
  int TPR, RPI, gy;
};

__host__ Tiling make_tiling(int C, int VEC) {
  int CG = C / VEC;
  Tiling t;
  t.TPR = CG < kBlock ? CG : kBlock;
  t.RPI = kBlock / t.TPR;
  t.gy = (CG + t.TPR - 1) / t.TPR;
  return t;
}

// ---------------------------------------------------------------- forward stats
template <typename T, int VEC>
__global__ __launch_bounds__(kBlock) void bn_fwd_stats_kernel(
    const T* __restrict__ x, int64_t M, int C, int TPR, int RPI, int64_t rows_per_block,
    float* __restrict__ part_mean, float* __restrict__ part_m2, float* __restrict__ part_n) {
  __shared__ float sh1[kBlock * VEC];
  __shared__ float sh2[kBlock * VEC];
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int CG = C / VEC;
  const int cg = blockIdx.y * TPR + lc;
  const bool active = (r0 < RPI) && (cg < CG);
  const int64_t rb = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t re = (rb + rows_per_block < M) ? rb + rows_per_block : M;
  const int c0 = cg * VEC;
  float K[VEC], s1[VEC], s2[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { K[i] = 0.f; s1[i] = 0.f; s2[i] = 0.f; }
  if (active && rb < re) {
    VecIO<T, VEC>::load(x + rb * C + c0, K);  // per-block shift: kills cancellation
    int64_t r = rb + r0;
    for (; r + 3 * RPI < re; r += 4 * RPI) {
      float v0[VEC], v1[VEC], v2[VEC], v3[VEC];
      VecIO<T, VEC>::load(x + r * C + c0, v0);
      VecIO<T, VEC>::load(x + (r + RPI) * C + c0, v1);
      VecIO<T, VEC>::load(x + (r + 2 * RPI) * C + c0, v2);
      VecIO<T, VEC>::load(x + (r + 3 * RPI) * C + c0, v3);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        float d0 = v0[i] - K[i], d1 = v1[i] - K[i], d2 = v2[i] - K[i], d3 = v3[i] - K[i];
        s1[i] += (d0 + d1) + (d2 + d3);
        s2[i] += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
      }
    }
    for (; r < re; r += RPI) {
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
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sh1[t * VEC + i] = s1[i]; sh2[t * VEC + i] = s2[i]; }
  __syncthreads();
  if (active && r0 == 0 && rb < re) {
    for (int rr = 1; rr < RPI; ++rr) {
      const int o = (rr * TPR + lc) * VEC;
#pragma unroll
      for (int i = 0; i < VEC; ++i) { s1[i] += sh1[o + i]; s2[i] += sh2[o + i]; }
    }
    const float n = static_cast<float>(re - rb);
    const float inv_n = 1.f / n;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      part_mean[blockIdx.x * static_cast<int64_t>(C) + c0 + i] = K[i] + s1[i] * inv_n;
      float m2 = s2[i] - s1[i] * s1[i] * inv_n;
      part_m2[blockIdx.x * static_cast<int64_t>(C) + c0 + i] = m2 > 0.f ? m2 : 0.f;
    }
    if (blockIdx.y == 0 && t == 0) part_n[blockIdx.x] = n;
  }
}

// Chan et al. merge of (n, mean, M2) partials; 4 partial-lanes per channel.
template <typename PT>
__global__ __launch_bounds__(kBlock) void bn_fwd_finalize_kernel(
    const float* __restrict__ part_mean, const float* __restrict__ part_m2,
    const float* __restrict__ part_n, int P, int C, const PT* __restrict__ gamma,
    const PT* __restrict__ beta, float* __restrict__ running_mean, float* __restrict__ running_var,
    float momentum, float eps, float* __restrict__ save_mean, float* __restrict__ save_invstd,
    float* __restrict__ scale, float* __restrict__ shift) {
  __shared__ float shn[kBlock], shm[kBlock], shq[kBlock];
  const int t = threadIdx.x;
  const int ch = blockIdx.x * 64 + (t & 63);
  const int sub = t >> 6;
  float n = 0.f, mean = 0.f, m2 = 0.f;
  if (ch < C) {
    for (int p = sub; p < P; p += 4) {
      const float nb = part_n[p];
      const float mb = part_mean[static_cast<int64_t>(p) * C + ch];
      const float qb = part_m2[static_cast<int64_t>(p) * C + ch];
      const float nn = n + nb;
      const float d = mb - mean;
      const float f = nb / nn;
      mean += d * f;
      m2 += qb + d * d * n * f;
      n = nn;
    }
  }
  shn[t] = n; shm[t] = mean; shq[t] = m2;
  __syncthreads();
  if (sub == 0 && ch < C) {
    for (int s = 1; s < 4; ++s) {
      const float nb = shn[t + 64 * s], mb = shm[t + 64 * s], qb = shq[t + 64 * s];
      if (nb == 0.f) continue;
      const float nn = n + nb;
      const float d = mb - mean;
      const float f = nb / nn;
      mean += d * f;
      m2 += qb + d * d * n * f;
      n = nn;
    }
    const float var = m2 / n;
    const float invstd = rsqrtf(var + eps);
    if (running_mean != nullptr) {
      const float unbiased = n > 1.f ? m2 / (n - 1.f) : var;
      running_mean[ch] = (1.f - momentum) * running_mean[ch] + momentum * mean;
      running_var[ch] = (1.f - momentum) * running_var[ch] + momentum * unbiased;
    }
    save_mean[ch] = mean;
    save_invstd[ch] = invstd;
    const float g = gamma ? ldp<PT>(gamma, ch) : 1.f;
    const float b = beta ? ldp<PT>(beta, ch) : 0.f;
    scale[ch] = g * invstd;
    shift[ch] = b - mean * g * invstd;
  }
}

template <typename PT>
__global__ void bn_eval_prep_kernel(int C, const PT* __restrict__ gamma, const PT* __restrict__ beta,
                                    const float* __restrict__ rm, const float* __restrict__ rv,
                                    float eps, float* __restrict__ save_mean,
                                    float* __restrict__ save_invstd, float* __restrict__ scale,
                                    float* __restrict__ shift) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= C) return;
  const float invstd = rsqrtf(rv[ch] + eps);
  const float g = gamma ? ldp<PT>(gamma, ch) : 1.f;
  const float b = beta ? ldp<PT>(beta, ch) : 0.f;
  save_mean[ch] = rm[ch];
  save_invstd[ch] = invstd;
  scale[ch] = g * invstd;
  shift[ch] = b - rm[ch] * g * invstd;
}

// ---------------------------------------------------------------- forward apply
template <typename T, int VEC, bool RELU, bool RES>
__global__ __launch_bounds__(kBlock) void bn_fwd_apply_kernel(
    const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y,
    const float* __restrict__ scale, const float* __restrict__ shift, int64_t M, int C, int TPR,
    int RPI) {
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int cg = blockIdx.y * TPR + lc;
  if (r0 >= RPI || cg >= C / VEC) return;
  const int c0 = cg * VEC;
  float sc[VEC], sf[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sc[i] = scale[c0 + i]; sf[i] = shift[c0 + i]; }
  const int64_t step = static_cast<int64_t>(gridDim.x) * RPI;
  int64_t r = static_cast<int64_t>(blockIdx.x) * RPI + r0;
  auto body = [&](int64_t row) {
    float v[VEC];
    VecIO<T, VEC>::load(x + row * C + c0, v);
    float rv[VEC];
    if constexpr (RES) VecIO<T, VEC>::load(res + row * C + c0, rv);
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float o = fmaf(v[i], sc[i], sf[i]);
      if constexpr (RES) o += rv[i];
      if constexpr (RELU) o = o > 0.f ? o : 0.f;
      v[i] = o;
    }
    VecIO<T, VEC>::store(y + row * C + c0, v);
  };
  for (; r + step < M; r += 2 * step) {  // two rows in flight per lane
    body(r);
    body(r + step);
  }
  if (r < M) body(r);
}

// ---------------------------------------------------------------- backward reduce
template <typename T, int VEC, bool RELU>
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce_kernel(
    const T* __restrict__ dy, const T* __restrict__ y, const T* __restrict__ x,
    const float* __restrict__ mean, int64_t M, int C, int TPR, int RPI, int64_t rows_per_block,
    float* __restrict__ part_a, float* __restrict__ part_b) {
  __shared__ float sh1[kBlock * VEC];
  __shared__ float sh2[kBlock * VEC];
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int CG = C / VEC;
  const int cg = blockIdx.y * TPR + lc;
  const bool active = (r0 < RPI) && (cg < CG);
  const int64_t rb = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t re = (rb + rows_per_block < M) ? rb + rows_per_block : M;
  const int c0 = cg * VEC;
  float mu[VEC], sa[VEC], sb[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sa[i] = 0.f; sb[i] = 0.f; mu[i] = 0.f; }
  if (active) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) mu[i] = mean[c0 + i];
    int64_t r = rb + r0;
    auto body = [&](int64_t row) {
      float g[VEC], xv[VEC];
      VecIO<T, VEC>::load(dy + row * C + c0, g);
      VecIO<T, VEC>::load(x + row * C + c0, xv);
      if constexpr (RELU) {
        float yv[VEC];
        VecIO<T, VEC>::load(y + row * C + c0, yv);
#pragma unroll
        for (int i = 0; i < VEC; ++i) g[i] = yv[i] > 0.f ? g[i] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        sa[i] += g[i];
        sb[i] = fmaf(g[i], xv[i] - mu[i], sb[i]);
      }
    };
    for (; r + RPI < re; r += 2 * RPI) {
      body(r);
      body(r + RPI);
    }
    if (r < re) body(r);
  }
#pragma unroll
  for (int i = 0; i < VEC; ++i) { sh1[t * VEC + i] = sa[i]; sh2[t * VEC + i] = sb[i]; }
  __syncthreads();
  if (active && r0 == 0) {
    for (int rr = 1; rr < RPI; ++rr) {
      const int o = (rr * TPR + lc) * VEC;
#pragma unroll
      for (int i = 0; i < VEC; ++i) { sa[i] += sh1[o + i]; sb[i] += sh2[o + i]; }
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      part_a[blockIdx.x * static_cast<int64_t>(C) + c0 + i] = sa[i];
      part_b[blockIdx.x * static_cast<int64_t>(C) + c0 + i] = sb[i];
    }
  }
}

template <typename PT>
__global__ __launch_bounds__(kBlock) void bn_bwd_finalize_kernel(
    const float* __restrict__ part_a, const float* __restrict__ part_b, int P, int C, float Mf,
    const PT* __restrict__ gamma, const float* __restrict__ mean, const float* __restrict__ invstd,
    bool training, PT* __restrict__ dgamma, PT* __restrict__ dbeta, float* __restrict__ coef) {
  __shared__ float sha[kBlock], shb[kBlock];
  const int t = threadIdx.x;
  const int ch = blockIdx.x * 64 + (t & 63);
  const int sub = t >> 6;
  float a = 0.f, b = 0.f;
  if (ch < C) {
    for (int p = sub; p < P; p += 4) {
      a += part_a[static_cast<int64_t>(p) * C + ch];
      b += part_b[static_cast<int64_t>(p) * C + ch];
    }
  }
  sha[t] = a; shb[t] = b;
  __syncthreads();
  if (sub == 0 && ch < C) {
    a += sha[t + 64] + sha[t + 128] + sha[t + 192];
    b += shb[t + 64] + shb[t + 128] + shb[t + 192];
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
}

template <typename T, int VEC, bool RELU, bool RES>
__global__ __launch_bounds__(kBlock) void bn_bwd_apply_kernel(
    const T* __restrict__ dy, const T* __restrict__ y, const T* __restrict__ x,
    const float* __restrict__ coef, T* __restrict__ dx, T* __restrict__ dres, int64_t M, int C,
    int TPR, int RPI) {
  const int t = threadIdx.x;
  const int lc = t % TPR, r0 = t / TPR;
  const int cg = blockIdx.y * TPR + lc;
  if (r0 >= RPI || cg >= C / VEC) return;
  const int c0 = cg * VEC;
  float k[VEC], c1[VEC], c0v[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    k[i] = coef[c0 + i];
    c1[i] = coef[C + c0 + i];
    c0v[i] = coef[2 * C + c0 + i];
  }
  const int64_t step = static_cast<int64_t>(gridDim.x) * RPI;
  auto body = [&](int64_t row) {
    float g[VEC], xv[VEC];
    VecIO<T, VEC>::load(dy + row * C + c0, g);
    VecIO<T, VEC>::load(x + row * C + c0, xv);
    if constexpr (RELU) {
      float yv[VEC];
      VecIO<T, VEC>::load(y + row * C + c0, yv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) g[i] = yv[i] > 0.f ? g[i] : 0.f;
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

// ---------------------------------------------------------------- host side
struct ReducePlan {
  Tiling tl;
  int gx;
  int64_t rows_per_block;
};

ReducePlan plan_reduce(int64_t M, int C, int VEC) {
  ReducePlan p;
  p.tl = make_tiling(C, VEC);
  int64_t target = 1024 / p.tl.gy;
  if (target < 1) target = 1;
  int64_t min_rows = static_cast<int64_t>(p.tl.RPI) * 8;  // >= 8 rows per lane
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

template <typename T>
constexpr int full_vec() { return 16 / sizeof(T); }

template <typename T, int VEC, typename PT>
hipError_t fwd_impl(const T* x, const T* res, T* y, const PT* gamma, const PT* beta, float* rm,
                    float* rv, float* save_mean, float* save_invstd, float* ws, int64_t M, int C,
                    bool relu, bool training, float momentum, float eps, hipStream_t s) {
  ReducePlan rp = plan_reduce(M, C, VEC);
  float* scale = ws;
  float* shift = ws + C;
  if (training) {
    float* pm = ws + 2 * C;
    float* pq = pm + static_cast<int64_t>(rp.gx) * C;
    float* pn = pq + static_cast<int64_t>(rp.gx) * C;
    hipLaunchKernelGGL((bn_fwd_stats_kernel<T, VEC>), dim3(rp.gx, rp.tl.gy), dim3(kBlock), 0, s,
                       x, M, C, rp.tl.TPR, rp.tl.RPI, rp.rows_per_block, pm, pq, pn);
    hipLaunchKernelGGL((bn_fwd_finalize_kernel<PT>), dim3((C + 63) / 64), dim3(kBlock), 0, s, pm,
                       pq, pn, rp.gx, C, gamma, beta, rm, rv, momentum, eps, save_mean,
                       save_invstd, scale, shift);
  } else {
    hipLaunchKernelGGL((bn_eval_prep_kernel<PT>), dim3((C + 255) / 256), dim3(256), 0, s, C, gamma,
                       beta, rm, rv, eps, save_mean, save_invstd, scale, shift);
  }
  dim3 grid(apply_gx(M, rp.tl), rp.tl.gy);
#define KDL_FWD_APPLY(R, S)                                                                  \
  hipLaunchKernelGGL((bn_fwd_apply_kernel<T, VEC, R, S>), grid, dim3(kBlock), 0, s, x, res, y, \
                     scale, shift, M, C, rp.tl.TPR, rp.tl.RPI)
  if (relu && res) KDL_FWD_APPLY(true, true);
  else if (relu) KDL_FWD_APPLY(true, false);
  else if (res) KDL_FWD_APPLY(false, true);
  else KDL_FWD_APPLY(false, false);
#undef KDL_FWD_APPLY
  return hipGetLastError();
}

template <typename T, int VEC, typename PT>
hipError_t bwd_impl(const T* dy, const T* y, const T* x, const PT* gamma, const float* mean,
                    const float* invstd, T* dx, T* dres, PT* dgamma, PT* dbeta, float* ws,
                    int64_t M, int C, bool relu, bool training, hipStream_t s) {
  ReducePlan rp = plan_reduce(M, C, VEC);
  float* coef = ws;
  float* pa = ws + 3 * C;
  float* pb = pa + static_cast<int64_t>(rp.gx) * C;
  if (relu)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, VEC, true>), dim3(rp.gx, rp.tl.gy), dim3(kBlock),
                       0, s, dy, y, x, mean, M, C, rp.tl.TPR, rp.tl.RPI, rp.rows_per_block, pa, pb);
  else
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, VEC, false>), dim3(rp.gx, rp.tl.gy), dim3(kBlock),
                       0, s, dy, y, x, mean, M, C, rp.tl.TPR, rp.tl.RPI, rp.rows_per_block, pa, pb);
  hipLaunchKernelGGL((bn_bwd_finalize_kernel<PT>), dim3((C + 63) / 64), dim3(kBlock), 0, s, pa, pb,
                     rp.gx, C, static_cast<float>(M), gamma, mean, invstd, training, dgamma, dbeta,
                     coef);
  dim3 grid(apply_gx(M, rp.tl), rp.tl.gy);
#define KDL_BWD_APPLY(R, S)                                                                   \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, VEC, R, S>), grid, dim3(kBlock), 0, s, dy, y, x, \
                     coef, dx, dres, M, C, rp.tl.TPR, rp.tl.RPI)
  if (relu && dres) KDL_BWD_APPLY(true, true);
  else if (relu) KDL_BWD_APPLY(true, false);
  else if (dres) KDL_BWD_APPLY(false, true);
  else KDL_BWD_APPLY(false, false);
#undef KDL_BWD_APPLY
  return hipGetLastError();
}

}  // namespace

// dtype codes: 0 = f32, 1 = bf16
int64_t bn_workspace_floats(int64_t M, int C, int dtype) {
  const int vec = (dtype == 1) ? ((C % 8 == 0) ? 8 : 1) : ((C % 4 == 0) ? 4 : 1);
  ReducePlan rp = plan_reduce(M, C, vec);
  const int64_t fwd = 2 * C + 2 * static_cast<int64_t>(rp.gx) * C + rp.gx;
  const int64_t bwd = 3 * C + 2 * static_cast<int64_t>(rp.gx) * C;
  return fwd > bwd ? fwd : bwd;
}

#define KDL_DISPATCH_PT(pdtype, ...)              \
  do {                                           \
    if ((pdtype) == 1) {                         \
      using PT = bf16_t;                         \
      __VA_ARGS__;                               \
    } else {                                     \
      using PT = float;                          \
      __VA_ARGS__;                               \
    }                                            \
  } while (0)

hipError_t bn_act_forward(const void* x, const void* res, void* y, const void* gamma,
                          const void* beta, float* rm, float* rv, float* save_mean,
                          float* save_invstd, float* ws, int64_t M, int C, int dtype, int pdtype,
                          bool relu, bool training, float momentum, float eps, hipStream_t s) {
  if (M <= 0 || C <= 0) return hipSuccess;
  hipError_t e = hipSuccess;
  if (dtype == 1) {
    using T = bf16_t;
    auto* xp = static_cast<const T*>(x);
    auto* rp = static_cast<const T*>(res);
    auto* yp = static_cast<T*>(y);
    KDL_DISPATCH_PT(pdtype, {
      auto* g = static_cast<const PT*>(gamma);
      auto* b = static_cast<const PT*>(beta);
      e = (C % 8 == 0) ? fwd_impl<T, 8, PT>(xp, rp, yp, g, b, rm, rv, save_mean, save_invstd, ws, M,
                                            C, relu, training, momentum, eps, s)
                       : fwd_impl<T, 1, PT>(xp, rp, yp, g, b, rm, rv, save_mean, save_invstd, ws, M,
                                            C, relu, training, momentum, eps, s);
    });
  } else {
    using T = float;
    auto* xp = static_cast<const T*>(x);
    auto* rp = static_cast<const T*>(res);
    auto* yp = static_cast<T*>(y);
    KDL_DISPATCH_PT(pdtype, {
      auto* g = static_cast<const PT*>(gamma);
      auto* b = static_cast<const PT*>(beta);
      e = (C % 4 == 0) ? fwd_impl<T, 4, PT>(xp, rp, yp, g, b, rm, rv, save_mean, save_invstd, ws, M,
                                            C, relu, training, momentum, eps, s)
                       : fwd_impl<T, 1, PT>(xp, rp, yp, g, b, rm, rv, save_mean, save_invstd, ws, M,
                                            C, relu, training, momentum, eps, s);
    });
  }
  return e;
}

hipError_t bn_act_backward(const void* dy, const void* y, const void* x, const void* gamma,
                           const float* mean, const float* invstd, void* dx, void* dres,
                           void* dgamma, void* dbeta, float* ws, int64_t M, int C, int dtype,
                           int pdtype, bool relu, bool training, hipStream_t s) {
  if (M <= 0 || C <= 0) return hipSuccess;
  hipError_t e = hipSuccess;
  if (dtype == 1) {
    using T = bf16_t;
    KDL_DISPATCH_PT(pdtype, {
      auto args = std::make_tuple(static_cast<const T*>(dy), static_cast<const T*>(y),
                                  static_cast<const T*>(x), static_cast<const PT*>(gamma));
      e = (C % 8 == 0)
              ? bwd_impl<T, 8, PT>(std::get<0>(args), std::get<1>(args), std::get<2>(args),
                                   std::get<3>(args), mean, invstd, static_cast<T*>(dx),
                                   static_cast<T*>(dres), static_cast<PT*>(dgamma),
                                   static_cast<PT*>(dbeta), ws, M, C, relu, training, s)
              : bwd_impl<T, 1, PT>(std::get<0>(args), std::get<1>(args), std::get<2>(args),
                                   std::get<3>(args), mean, invstd, static_cast<T*>(dx),
                                   static_cast<T*>(dres), static_cast<PT*>(dgamma),
                                   static_cast<PT*>(dbeta), ws, M, C, relu, training, s);
    });
  } else {
    using T = float;
    KDL_DISPATCH_PT(pdtype, {
      auto args = std::make_tuple(static_cast<const T*>(dy), static_cast<const T*>(y),
                                  static_cast<const T*>(x), static_cast<const PT*>(gamma));
      e = (C % 4 == 0)
              ? bwd_impl<T, 4, PT>(std::get<0>(args), std::get<1>(args), std::get<2>(args),
                                   std::get<3>(args), mean, invstd, static_cast<T*>(dx),
                                   static_cast<T*>(dres), static_cast<PT*>(dgamma),
                                   static_cast<PT*>(dbeta), ws, M, C, relu, training, s)
              : bwd_impl<T, 1, PT>(std::get<0>(args), std::get<1>(args), std::get<2>(args),
                                   std::get<3>(args), mean, invstd, static_cast<T*>(dx),
                                   static_cast<T*>(dres), static_cast<PT*>(dgamma),
                                   static_cast<PT*>(dbeta), ws, M, C, relu, training, s);
    });
  }
  return e;
}

}  // namespace kdl
