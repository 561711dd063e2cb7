// BatchNorm folded through the bottleneck's closing 1x1 conv (gfx950).
//
// A bottleneck ends with c3 = a2 W3^T (a2 = ReLU(BN2(c2)), [M, C]; W3 [4C, C])
// and y = BN3(c3).  At the 56x56 / 28x28 stages c3 is the widest tensor of the
// step (4C channels), so the ResNet engine can run those blocks without ever
// storing it (kubedl_amd/models/resnet_engine.py, "recompute" blocks): the
// forward recomputes c3 inside the GEMM that applies BN3 + residual + ReLU
// (csrc/gemm_epi.h APPLY), the next block's conv1 data gradient recomputes it
// for the BN3 backward sums (csrc/conv1x1.hip PRO_RECOMP), and the two
// consumers of the BN3 backward apply dc3 = k g + c1 c3 + c0 take it in
// algebraic form, because c3 is linear in a2:
//
//   conv3 data gradient   dc3 W3 = (diag(k) g) W3 + a2 S + 1 b^T,
//                         S = W3^T diag(c1) W3 [C, C],  b = W3^T c0 [C]
//     -> one two-segment GEMM [k g | a2 | a2] . [W3 ; S_hi ; S_lo] (csrc/conv1x1.hip
//        PRO_SEG: k applied per element while staging g -- random rounding, as
//        the materialised dc3 had --, S as a bf16 hi + lo pair, bias in the
//        MASKX epilogue): S_hi | S_lo and b from fold_dgrad below;
//   conv3 weight gradient dW3 = dc3^T a2 = diag(k) G + diag(c1) W3 Q + c0 sum(a2)^T,
//                         G = g^T a2, Q = a2^T a2 (both split-M MFMA GEMMs on
//                         the LDS-DMA weight-gradient kernel, Q with the GRELU
//                         G prologue) -> fold_wgrad below.
//
// Every kernel here is O(C^2 * 4C) fp32 work on L2-resident operands (at most
// a few microseconds); no atomics, fixed summation orders (deterministic).
//
// The reference has no kernels; this serves the PyTorchJob
// ResNet-50 worker (BASELINE.json config 2).
#include "common.h"
#include "kdl_api.h"

namespace kdl {
namespace {

constexpr int kFoldThreads = 256;

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }

// Small fp32 GEMM tiles out[m][n] = sum_k a(m, k) b(k, n) over 16 x 16 output
// tiles, one output per thread.  The whole K range (<= kMaxK) of both operand
// panels is staged through LDS in one pass -- every load of the block issued
// back to back, one memory latency instead of one per K chunk -- then summed in
// a fixed order.
constexpr int kT = 16, kMaxK = 512;

template <typename FA, typename FB>
__device__ __forceinline__ float tile_dot(int K, int m0, int n0, FA a, FB b, float (*as)[kT + 1],
                                          float (*bs)[kT + 1]) {
  const int t = threadIdx.x, tm = t / kT, tn = t % kT;
  for (int e = t; e < K * kT; e += kFoldThreads) {  // e = k * 16 + i
    const int k = e / kT, i = e % kT;
    as[k][i] = a(m0 + i, k);
    bs[k][i] = b(k, n0 + i);
  }
  __syncthreads();
  float acc = 0.f;
#pragma unroll 16
  for (int k = 0; k < K; ++k) acc = fmaf(as[k][tm], bs[k][tn], acc);
  __syncthreads();
  return acc;
}

// Blocks [0, (C/16)^2): tiles of S = W3^T diag(c1) W3 [C, C] as a bf16 hi + lo
// pair, S2[j][l] = bf16(S[l][j]), S2[j][C + l] = bf16(S[l][j] - S2[j][l]) (~16
// significant bits: S multiplies every pixel's a2, so a plain bf16 rounding of
// it would be one systematic error repeated across the whole batch).  Blocks
// past them: 16 columns j each, bias[j] = sum_c c0_c W3[c][j] (fp32).
__global__ __launch_bounds__(kFoldThreads) void fold_dgrad_kernel(const uint16_t* __restrict__ w3,
                                                                  const float* __restrict__ bcoef, int N4, int C,
                                                                  uint16_t* __restrict__ s2, float* __restrict__ bias) {
  __shared__ float as[kMaxK][kT + 1], bs[kMaxK][kT + 1];
  const float* c1 = bcoef + N4;
  const float* c0 = bcoef + 2 * N4;
  const int tiles = C / kT, t = threadIdx.x;
  if (static_cast<int>(blockIdx.x) < tiles * tiles) {
    const int l0 = (blockIdx.x / tiles) * kT, j0 = (blockIdx.x % tiles) * kT;
    const float s = tile_dot(
        N4, l0, j0, [&](int l, int c) { return bf2f(w3[static_cast<int64_t>(c) * C + l]); },
        [&](int c, int j) { return c1[c] * bf2f(w3[static_cast<int64_t>(c) * C + j]); }, as, bs);
    const int l = l0 + t / kT, j = j0 + t % kT;
    const uint16_t hi = f32_to_bf16(s);
    s2[static_cast<int64_t>(j) * 2 * C + l] = hi;
    s2[static_cast<int64_t>(j) * 2 * C + C + l] = f32_to_bf16(s - bf2f(hi));
    return;
  }
  const int j0 = (blockIdx.x - tiles * tiles) * kT;
  float b[kT];
#pragma unroll
  for (int i = 0; i < kT; ++i) b[i] = 0.f;
  for (int c = t; c < N4; c += kFoldThreads) {
    const float cc = c0[c];
#pragma unroll
    for (int i = 0; i < kT; ++i) b[i] = fmaf(cc, bf2f(w3[static_cast<int64_t>(c) * C + j0 + i]), b[i]);
  }
  float* red = &as[0][0];  // [kT][kFoldThreads / 64] wave partials
#pragma unroll
  for (int i = 0; i < kT; ++i) {
    float v = b[i];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((t & 63) == 0) red[i * (kFoldThreads / 64) + (t >> 6)] = v;
  }
  __syncthreads();
  if (t < kT) {
    float v = 0.f;
    for (int w = 0; w < kFoldThreads / 64; ++w) v += red[t * (kFoldThreads / 64) + w];  // fixed order
    bias[j0 + t] = v;
  }
}

// Column sums of relu(x * scale + shift), x [M, C] bf16 -> part[block][C]
// (each block a contiguous row range; 8 channels per thread, row groups folded
// in LDS in a fixed order).
__global__ __launch_bounds__(kFoldThreads) void relu_colsum_kernel(const uint16_t* __restrict__ x,
                                                                   const float* __restrict__ coef, int64_t M, int C,
                                                                   int64_t rows_per_block, float* __restrict__ part) {
  extern __shared__ float sm[];  // [groups][C]
  const int cpr = C / 8;
  const int t = threadIdx.x;
  const int groups = kFoldThreads / cpr;
  const int g = t / cpr, cc = (t % cpr) * 8;
  float sc[8], sf[8], a[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = coef[cc + e];
    sf[e] = coef[C + cc + e];
    a[e] = 0.f;
  }
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < M ? r0 + rows_per_block : M;
  if (g < groups) {
    for (int64_t r = r0 + g; r < r1; r += groups) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + r * C + cc);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = __uint_as_float(w[e] << 16), hi = __uint_as_float(w[e] & 0xffff0000u);
        const float o0 = fmaf(lo, sc[2 * e], sf[2 * e]), o1 = fmaf(hi, sc[2 * e + 1], sf[2 * e + 1]);
        a[2 * e] += o0 > 0.f ? o0 : 0.f;
        a[2 * e + 1] += o1 > 0.f ? o1 : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) sm[g * C + cc + e] = a[e];
  }
  __syncthreads();
  for (int c = t; c < C; c += kFoldThreads) {
    float s = 0.f;
    for (int q = 0; q < groups; ++q) s += sm[q * C + c];
    part[static_cast<int64_t>(blockIdx.x) * C + c] = s;
  }
}

// 16 x 16 tiles of dW3 [N4][C]:
//   dW3[c][j] = k_c G[c][j] + c1_c sum_l W3[c][l] Q[l][j] + c0_c asum[j],
//   asum[j] = sum_p part[p][j]  (fixed order)
__global__ __launch_bounds__(kFoldThreads) void fold_wgrad_kernel(const uint16_t* __restrict__ w3,
                                                                  const float* __restrict__ bcoef,
                                                                  const float* __restrict__ G,
                                                                  const float* __restrict__ Q,
                                                                  const float* __restrict__ part, int nparts, int N4,
                                                                  int C, uint16_t* __restrict__ dw) {
  __shared__ float as[kMaxK][kT + 1], bs[kMaxK][kT + 1];
  const int tj = C / kT;
  const int c0i = (blockIdx.x / tj) * kT, j0 = (blockIdx.x % tj) * kT;
  const float q = tile_dot(
      C, c0i, j0, [&](int c, int l) { return bf2f(w3[static_cast<int64_t>(c) * C + l]); },
      [&](int l, int j) { return Q[static_cast<int64_t>(l) * C + j]; }, as, bs);
  const int c = c0i + threadIdx.x / kT, j = j0 + threadIdx.x % kT;
  float asum = 0.f;
  for (int p = 0; p < nparts; ++p) asum += part[static_cast<int64_t>(p) * C + j];
  const float k = bcoef[c], c1 = bcoef[N4 + c], c0 = bcoef[2 * N4 + c];
  const float v = fmaf(k, G[static_cast<int64_t>(c) * C + j], fmaf(c1, q, c0 * asum));
  dw[static_cast<int64_t>(c) * C + j] = f32_to_bf16(v);
}

}  // namespace

hipError_t bn_fold_dgrad(const void* w3, const float* bcoef, int N4, int C, void* bp, float* bias, hipStream_t s) {
  if (N4 <= 0 || C <= 0 || C % kT || N4 % kT || N4 > kMaxK) return hipErrorInvalidValue;
  const int tiles = C / kT;
  hipLaunchKernelGGL(fold_dgrad_kernel, dim3(tiles * tiles + tiles), dim3(kFoldThreads), 0, s,
                     static_cast<const uint16_t*>(w3), bcoef, N4, C, static_cast<uint16_t*>(bp), bias);
  return hipGetLastError();
}

int relu_colsum_parts(int64_t M) { return M >= 256 * 64 ? 256 : static_cast<int>((M + 63) / 64); }

hipError_t relu_colsum(const void* x, const float* coef, int64_t M, int C, float* part, hipStream_t s) {
  if (M <= 0 || C % 8 || C / 8 > kFoldThreads) return hipErrorInvalidValue;
  const int parts = relu_colsum_parts(M);
  const int64_t rpb = (M + parts - 1) / parts;
  const int groups = kFoldThreads / (C / 8);
  hipLaunchKernelGGL(relu_colsum_kernel, dim3(parts), dim3(kFoldThreads), groups * C * sizeof(float), s,
                     static_cast<const uint16_t*>(x), coef, M, C, rpb, part);
  return hipGetLastError();
}

hipError_t bn_fold_wgrad(const void* w3, const float* bcoef, const float* G, const float* Q, const float* part,
                         int nparts, int N4, int C, void* dw, hipStream_t s) {
  if (N4 <= 0 || C <= 0 || nparts <= 0 || C % kT || N4 % kT || C > kMaxK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fold_wgrad_kernel, dim3((N4 / kT) * (C / kT)), dim3(kFoldThreads), 0, s,
                     static_cast<const uint16_t*>(w3), bcoef, G, Q, part, nparts, N4, C, static_cast<uint16_t*>(dw));
  return hipGetLastError();
}

}  // namespace kdl
