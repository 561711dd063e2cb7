// BatchNorm finalize folded into the GEMM that produced the sums (gfx950).
//
// The conv GEMM epilogues (gemm_epi.h STATS / MASKX / RESBITS) add their
// per-channel sums into the BN workspace replicas; a separate finalize kernel
// then turned the replicas into the layer's coefficients -- ~106 launches of
// ~5 us per ResNet-50 step, each behind a kernel boundary.  Here the LAST
// block of each output-channel tile to finish (an arrival counter per tile in
// the workspace tail, device-scope acq_rel) finalizes that tile's channels:
//
//   writer blocks:  replica atomics -> __threadfence -> counter += 1
//   last arriver:   __threadfence (acquire) -> agent-scope loads of the 32
//                   replicas -> zero them -> coefficients / running stats /
//                   dgamma, dbeta -> counter = 0
//
// Each tile's last block handles <= 256 channels (one memory round trip), so
// the tail it adds is shorter than the launch it replaces.  The pointers a
// finalize needs are the layer's and stable across steps: the host writes them
// once into the workspace tail (BnFinDesc, bn_fin_desc in bindings.cpp).
//
// Workspace (fp32 elements, bn_workspace_floats):
//   [32][2C] forward replicas | [32][2C] backward | [2C] scale, shift |
//   [3C] k, c1, c0 | [32] BnFinDesc | [64] tile counters (fwd 0..31, bwd 32..63)
#pragma once

#include "common.h"

namespace kdl {

constexpr int kFinReplicas = 32;
constexpr int kFinDescFloats = 32;
constexpr int kFinCounters = 64;

struct BnFinDesc {
  const void* gamma;
  const void* beta;
  float* rm;
  float* rv;
  float* save_mean;
  float* save_invstd;
  void* dgamma;
  void* dbeta;
  float momentum, eps;
  int C, pt_bf16;  // parameter dtype: 1 bf16, 0 fp32
};
static_assert(sizeof(BnFinDesc) <= kFinDescFloats * 4, "descriptor fits its slot");

__host__ __device__ __forceinline__ int64_t fin_desc_off(int C) {
  return static_cast<int64_t>(kFinReplicas) * 4 * C + 5 * static_cast<int64_t>(C);
}

__device__ __forceinline__ float fin_ldp(const void* p, int bf, int i) {
  return bf ? bf16_to_f32(static_cast<const bf16_t*>(p)[i]) : static_cast<const float*>(p)[i];
}
__device__ __forceinline__ void fin_stp(void* p, int bf, int i, float v) {
  if (bf)
    static_cast<bf16_t*>(p)[i] = f32_to_bf16(v);
  else
    static_cast<float*>(p)[i] = v;
}

// sum the 32 replicas of (row[c], row[C + c]) with agent-scope loads (the adds
// came from blocks on every XCD) and re-zero them.  Eight replicas per batch of
// loads: all 64 values at once cost the host GEMM kernels ~90 spilled VGPRs
// (this tail is inlined into their epilogues); the sum order is unchanged.
__device__ __forceinline__ void fin_sum(float* acc, int C, int c, float& s1, float& s2) {
  constexpr int kB = 8;
  s1 = 0.f;
  s2 = 0.f;
#pragma unroll 1
  for (int r0 = 0; r0 < kFinReplicas; r0 += kB) {
    float va[kB], vb[kB];
#pragma unroll
    for (int r = 0; r < kB; ++r) {
      float* row = acc + static_cast<int64_t>(r0 + r) * 2 * C;
      va[r] = __hip_atomic_load(row + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      vb[r] = __hip_atomic_load(row + C + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int r = 0; r < kB; ++r) {
      s1 += va[r];
      s2 += vb[r];
      float* row = acc + static_cast<int64_t>(r0 + r) * 2 * C;
      row[c] = 0.f;
      row[C + c] = 0.f;
    }
  }
}

// forward (training): sums taken around running_mean (the GEMM epilogue's shift),
// the same fp32 expressions as bn_act.hip bn_fwd_finalize_kernel
__device__ __forceinline__ void fin_fwd_channel(const BnFinDesc& d, float* ws, int c, float Mf) {
  const int C = d.C;
  const float K = d.rm[c];  // read before this thread updates it
  float s1, s2;
  fin_sum(ws, C, c, s1, s2);
  const float inv_m = 1.f / Mf;
  const float m1 = s1 * inv_m;
  float var = s2 * inv_m - m1 * m1;
  var = var > 0.f ? var : 0.f;
  const float mean = K + m1;
  const float invstd = rsqrtf(var + d.eps);
  d.save_mean[c] = mean;
  d.save_invstd[c] = invstd;
  const float unbiased = Mf > 1.f ? var * Mf / (Mf - 1.f) : var;
  d.rm[c] = (1.f - d.momentum) * d.rm[c] + d.momentum * mean;
  d.rv[c] = (1.f - d.momentum) * d.rv[c] + d.momentum * unbiased;
  const float g = d.gamma ? fin_ldp(d.gamma, d.pt_bf16, c) : 1.f;
  const float b = d.beta ? fin_ldp(d.beta, d.pt_bf16, c) : 0.f;
  const float sc = g * invstd;
  float* coef = ws + static_cast<int64_t>(kFinReplicas) * 4 * C;
  coef[c] = sc;
  coef[C + c] = b - mean * sc;
}

// backward (training): bn_act.hip bn_bwd_finalize_kernel's expressions
__device__ __forceinline__ void fin_bwd_channel(const BnFinDesc& d, float* ws, int c, float Mf) {
  const int C = d.C;
  float a, b;
  fin_sum(ws + static_cast<int64_t>(kFinReplicas) * 2 * C, C, c, a, b);
  const float is = d.save_invstd[c];
  const float db = a;
  const float dg = b * is;
  if (d.dgamma) fin_stp(d.dgamma, d.pt_bf16, c, dg);
  if (d.dbeta) fin_stp(d.dbeta, d.pt_bf16, c, db);
  const float g = d.gamma ? fin_ldp(d.gamma, d.pt_bf16, c) : 1.f;
  const float k = g * is;
  const float c1 = -k * is * dg / Mf;
  const float c0 = -k * db / Mf - c1 * d.save_mean[c];
  float* bcoef = ws + static_cast<int64_t>(kFinReplicas) * 4 * C + 2 * C;
  bcoef[c] = k;
  bcoef[C + c] = c1;
  bcoef[2 * C + c] = c0;
}

}  // namespace kdl
