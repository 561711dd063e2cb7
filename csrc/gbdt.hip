// Histogram GBDT kernels for the XGBoostJob worker (gfx950).
//
// Data layout: quantised features ``bins`` are uint8 row-major [N, F] (<= 256
// bins per feature).  Rows are kept grouped by tree node: ``rows`` holds row
// ids ordered by node, node n owning rows[seg[n] .. seg[n+1]).
//
// hist_build: one wave handles one row at a time with LANE = FEATURE, so the
//   row's F bin codes are one coalesced load and the 64 lanes update 64
//   DIFFERENT per-feature histograms in LDS (ds_add_f32; lanes never collide
//   on an address, only on banks).  g/h of the row are wave-uniform.  A block
//   (4 waves) accumulates [F_TILE][B][2] in LDS (F_TILE=64, B=256 -> 128 KiB of
//   the CU's 160 KiB LDS), then flushes with no-return fp32 global atomics
//   into the node's [F][B][2] histogram; the grid is (row chunks, nodes,
//   feature tiles) with >= 2048 rows per block so that flush atomics are a
//   small fraction of the traffic.
// split_find: one 256-thread block per (node, feature), thread = bin:
//   block-wide inclusive scan of (G, H) over bins (wave scan with DPP-free
//   __shfl_up over 64 lanes + LDS carry), XGBoost gain
//     GL^2/(HL+l) + GR^2/(HR+l) - G^2/(H+l)
//   subject to min_child_weight on both sides, block argmax -> best split.
//
// The reference runs XGBoost/rabit inside a user image; the
// distributed part here is an RCCL all-reduce of the level's histograms.
#include "common.h"
#include "kdl_api.h"

namespace kdl {
namespace {

constexpr int kHistBlock = 256;
constexpr int kFTile = 64;  // features per block = wave width

// ``fp`` = features per row slot (power of two >= the tile's feature count, <= 64):
// a wave covers 64 / fp rows per step (F = 28 -> two rows per wave, no idle
// half-wave), and the LDS tile is [fp][B][2] (64 KiB at F <= 32 -> two blocks
// per CU).  Blocks past their node's last row exit before touching LDS (the
// grid is sized by the largest node of the level).
__global__ __launch_bounds__(kHistBlock) void hist_build_kernel(
    const uint8_t* __restrict__ bins, const float* __restrict__ grad, const float* __restrict__ hess,
    int64_t gh_stride, const int32_t* __restrict__ rows, const int32_t* __restrict__ seg, int F, int B,
    int rows_per_block, int fp, float* __restrict__ hist) {
  extern __shared__ float lds[];  // [fp][B][2]
  const int node = blockIdx.y;
  const int s0 = seg[node], s1 = seg[node + 1];
  const int r0 = s0 + blockIdx.x * rows_per_block;
  if (r0 >= s1) return;  // block-uniform
  const int r1 = (r0 + rows_per_block) < s1 ? (r0 + rows_per_block) : s1;
  const int f0 = blockIdx.z * fp;
  const int nf = (F - f0) < fp ? (F - f0) : fp;
  const int t = threadIdx.x;
  for (int i = t; i < nf * B * 2; i += kHistBlock) lds[i] = 0.f;
  __syncthreads();
  const int lane = t & 63, wave = t >> 6;
  const int rpw = 64 / fp;                 // rows per wave step
  const int sub = lane / fp, fl = lane - sub * fp;
  for (int r = r0 + wave * rpw + sub; r < r1; r += (kHistBlock / 64) * rpw) {
    const int row = rows[r];
    const float g = grad[static_cast<int64_t>(row) * gh_stride];
    const float h = hess[static_cast<int64_t>(row) * gh_stride];
    if (fl < nf) {
      const int b = bins[static_cast<int64_t>(row) * F + f0 + fl];
      float* p = lds + (fl * B + b) * 2;
      atomicAdd(p, g);
      atomicAdd(p + 1, h);
    }
  }
  __syncthreads();
  float* out = hist + (static_cast<int64_t>(node) * F + f0) * B * 2;
  for (int i = t; i < nf * B * 2; i += kHistBlock) {
    const float v = lds[i];
    if (v != 0.f) __hip_atomic_fetch_add(out + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Wave-level inclusive scan over 64 lanes.
__device__ __forceinline__ float wave_incl_scan(float v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

__global__ __launch_bounds__(256) void split_find_kernel(
    const float* __restrict__ hist, int F, int B, float lambda, float min_child_weight,
    float* __restrict__ best_gain, int32_t* __restrict__ best_bin, float* __restrict__ best_gl,
    float* __restrict__ best_hl) {
  __shared__ float carry_g[4], carry_h[4];
  __shared__ float red_gain[4];
  __shared__ int red_bin[4];
  const int node = blockIdx.y, f = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const float* hp = hist + ((static_cast<int64_t>(node) * F + f) * B) * 2;
  float g = 0.f, h = 0.f;
  if (t < B) {
    g = hp[2 * t];
    h = hp[2 * t + 1];
  }
  float sg = wave_incl_scan(g), sh = wave_incl_scan(h);
  if (lane == 63) {
    carry_g[wave] = sg;
    carry_h[wave] = sh;
  }
  __syncthreads();
  float tot_g = 0.f, tot_h = 0.f, pre_g = 0.f, pre_h = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    if (w < wave) {
      pre_g += carry_g[w];
      pre_h += carry_h[w];
    }
    tot_g += carry_g[w];
    tot_h += carry_h[w];
  }
  const float gl = sg + pre_g, hl = sh + pre_h;  // rows with bin <= t go left
  const float gr = tot_g - gl, hr = tot_h - hl;
  float gain = -INFINITY;
  if (t < B - 1 && hl >= min_child_weight && hr >= min_child_weight) {
    gain = gl * gl / (hl + lambda) + gr * gr / (hr + lambda) - tot_g * tot_g / (tot_h + lambda);
  }
  int bin = t;
  // wave argmax (ties -> lower bin)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float og = __shfl_xor(gain, o, 64);
    const int ob = __shfl_xor(bin, o, 64);
    if (og > gain || (og == gain && ob < bin)) {
      gain = og;
      bin = ob;
    }
  }
  if (lane == 0) {
    red_gain[wave] = gain;
    red_bin[wave] = bin;
  }
  __syncthreads();
  if (t == 0) {
    float bg = red_gain[0];
    int bb = red_bin[0];
    for (int w = 1; w < 4; ++w)
      if (red_gain[w] > bg || (red_gain[w] == bg && red_bin[w] < bb)) {
        bg = red_gain[w];
        bb = red_bin[w];
      }
    red_gain[0] = bg;
    red_bin[0] = bb;
  }
  __syncthreads();
  // the thread owning the winning bin publishes its left sums
  if (t == red_bin[0]) {
    const int64_t o = static_cast<int64_t>(node) * F + f;
    best_gain[o] = red_gain[0];
    best_bin[o] = red_bin[0];
    best_gl[o] = gl;
    best_hl[o] = hl;
  }
  if (t == 0 && red_gain[0] == -INFINITY) {
    const int64_t o = static_cast<int64_t>(node) * F + f;
    best_gain[o] = -INFINITY;
    best_bin[o] = -1;
    best_gl[o] = 0.f;
    best_hl[o] = 0.f;
  }
}

// Row routing: 1 = right child, per row of every splitting node.
__global__ __launch_bounds__(256) void route_rows_kernel(
    const uint8_t* __restrict__ bins, const int32_t* __restrict__ rows, const int32_t* __restrict__ row_node,
    const int32_t* __restrict__ split_feat, const int32_t* __restrict__ split_bin, int F, int n,
    int32_t* __restrict__ go_right) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int row = rows[i];
  const int node = row_node[i];
  const int f = split_feat[node];
  int r = 0;
  if (f >= 0) r = bins[static_cast<int64_t>(row) * F + f] > split_bin[node] ? 1 : 0;
  go_right[i] = r;
}

}  // namespace

hipError_t gbdt_hist_build(const uint8_t* bins, const float* grad, const float* hess, int64_t gh_stride,
                           const int32_t* rows, const int32_t* seg, int num_nodes, int max_rows_per_node,
                           int F, int B, float* hist, hipStream_t s) {
  if (num_nodes <= 0 || F <= 0) return hipSuccess;
  const int rows_per_block = 2048;
  int chunks = (max_rows_per_node + rows_per_block - 1) / rows_per_block;
  if (chunks < 1) chunks = 1;
  int fp = 1;
  while (fp < F && fp < kFTile) fp <<= 1;  // features per row slot
  dim3 grid(chunks, num_nodes, (F + fp - 1) / fp);
  const size_t lds = static_cast<size_t>(fp) * B * 2 * sizeof(float);
  static bool attr_set = false;  // > 64 KiB of dynamic LDS must be opted into once
  if (!attr_set) {
    KDL_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(hist_build_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      static_cast<int>(kFTile * 256 * 2 * sizeof(float))));
    attr_set = true;
  }
  hipLaunchKernelGGL(hist_build_kernel, grid, dim3(kHistBlock), lds, s, bins, grad, hess, gh_stride, rows,
                     seg, F, B, rows_per_block, fp, hist);
  return hipGetLastError();
}

hipError_t gbdt_split_find(const float* hist, int num_nodes, int F, int B, float lambda,
                           float min_child_weight, float* best_gain, int32_t* best_bin, float* best_gl,
                           float* best_hl, hipStream_t s) {
  if (num_nodes <= 0 || F <= 0) return hipSuccess;
  hipLaunchKernelGGL(split_find_kernel, dim3(F, num_nodes), dim3(256), 0, s, hist, F, B, lambda,
                     min_child_weight, best_gain, best_bin, best_gl, best_hl);
  return hipGetLastError();
}

hipError_t gbdt_route_rows(const uint8_t* bins, const int32_t* rows, const int32_t* row_node,
                           const int32_t* split_feat, const int32_t* split_bin, int F, int n,
                           int32_t* go_right, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(route_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, s, bins, rows, row_node,
                     split_feat, split_bin, F, n, go_right);
  return hipGetLastError();
}

}  // namespace kdl
