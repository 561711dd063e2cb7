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
// Device-resident tree growth (no host round trip inside a tree; the host only
// enqueues a fixed kernel sequence per level):
//   nodes live in heap order (level d = heap ids [2^d-1, 2^(d+1)-1)); ``rows``
//   keeps rows grouped by node, node i of the level owning rows[lo[i] .. hi[i]),
//   and ``node_pos`` holds the heap node id of the row at each position (moved
//   with the rows; the row-indexed ``node_of_row`` is written at the tree's end).  Per level:
//   split_find -> gbdt_decide (argmax over features, leaf weight, tree arrays)
//   -> gbdt_route_flags (1 = goes right) -> inclusive scan of the flags
//   -> gbdt_partition (stable in-segment partition: left rows keep their
//   order, then right rows; node ids advanced to 2h+1 / 2h+2)
//   -> gbdt_children (child segments; the smaller child by row count is the
//   one whose histogram gets built) -> gbdt_hist_plan (chunks per built node,
//   exclusive prefix) -> hist_build_wq (work-queue grid: block -> (node,
//   chunk) by binary search over the prefix) -> gbdt_subtract (sibling =
//   parent - built).  With > 1 rank the child counts and the built histograms
//   are all-reduced between these kernels (RCCL), nothing else.
// gbdt_quantise: bins = number of cuts < x (torch.bucketize right=False), one
//   thread per element, binary search over the feature's cut row.
//
// The reference runs XGBoost/rabit inside a user image; the
// distributed part here is an RCCL all-reduce of the level's histograms.
#include "common.h"
#include "kdl_api.h"
#include "tune.h"

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
    float* __restrict__ best_hl, float* __restrict__ node_tot) {
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
  if (node_tot != nullptr && f == 0 && t == 0) {
    node_tot[2 * node] = tot_g;
    node_tot[2 * node + 1] = tot_h;
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

// ---------------------------------------------------------------- device-resident growth
// Work-queue histogram build: block c of the grid works on chunk c of the
// concatenated chunk lists of the ``nb`` built nodes (chunk_off = exclusive
// prefix of ceil(size / rpb), chunk_off[nb] = total).  Each wave keeps UNROLL
// row slots in flight (row ids, g/h and bin codes loaded before any LDS
// atomic) so the dependent global loads overlap.
// Quantised gradients (XGBoost's GPU-hist idea, here for the LDS rate): float
// LDS atomics are the slow path on gfx950 -- the same round with the h
// ds_add_f32 dropped ran 2.9x faster, and with both adds as ds_add_u32 as fast
// as with no atomics at all (383 -> 1446 rounds/s, KDL_TUNE-priced variants,
// profiles/r05_gbdt_price.txt).  So each block accumulates fixed-point
// integers: q = rint(g * sg) with sg = 2^30 / (rpb * max|g|) -- a block sums
// at most rpb rows, so |sum| <= 2^30 never overflows, and a row's rounding
// error is <= 2^-31 rpb max|g| (~1e-6 max|g| at 2048 rows per chunk).  The
// block's exact integer sums are converted back (/ sg) when flushed into the
// node's fp32 histogram.  ``gh_max`` = {max |g|, max h} of the tree's rows
// (gbdt_gh_absmax).
constexpr float kQuantRange = 1073741824.f;  // 2^30

template <int UNROLL>
__global__ __launch_bounds__(kHistBlock) void hist_build_wq_kernel(
    const uint8_t* __restrict__ bins, const float* __restrict__ grad, const float* __restrict__ hess,
    int64_t gh_stride, const int32_t* __restrict__ rows, const int32_t* __restrict__ blo,
    const int32_t* __restrict__ bhi, const int32_t* __restrict__ chunk_off, int nb, int F, int B, int rpb, int fp,
    const float* __restrict__ gh_max, float* __restrict__ hist) {
  // LDS: two int planes, g [fp][B] then h [fp][B]
  extern __shared__ int qlds[];
  int* qh_pl = qlds + fp * B;
  const int c = blockIdx.x;
  if (c >= chunk_off[nb]) return;  // block-uniform
  int a = 0, z = nb;               // last j with chunk_off[j] <= c
  while (z - a > 1) {
    const int m = (a + z) >> 1;
    if (chunk_off[m] <= c) a = m; else z = m;
  }
  const int j = a;
  const int r0 = blo[j] + (c - chunk_off[j]) * rpb;
  const int r1 = (r0 + rpb) < bhi[j] ? (r0 + rpb) : bhi[j];
  const int f0 = blockIdx.y * fp;
  const int nf = (F - f0) < fp ? (F - f0) : fp;
  const int t = threadIdx.x;
  const float mg = gh_max[0], mh = gh_max[1];
  const float sg = mg > 0.f ? kQuantRange / (static_cast<float>(rpb) * mg) : 0.f;
  const float sh = mh > 0.f ? kQuantRange / (static_cast<float>(rpb) * mh) : 0.f;
  for (int i = t; i < 2 * fp * B; i += kHistBlock) qlds[i] = 0;
  __syncthreads();
  const int lane = t & 63, wave = t >> 6;
  const int rpw = 64 / fp;
  const int sub = lane / fp, fl = lane - sub * fp;
  const int step = (kHistBlock / 64) * rpw;  // rows per block-wide slot
  for (int base = r0 + wave * rpw + sub; base < r1; base += step * UNROLL) {
    int row[UNROLL];
    float g[UNROLL], h[UNROLL];
    int b[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int r = base + u * step;
      row[u] = r < r1 ? rows[r] : -1;
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (row[u] >= 0) {
        g[u] = grad[static_cast<int64_t>(row[u]) * gh_stride];
        h[u] = hess[static_cast<int64_t>(row[u]) * gh_stride];
        b[u] = fl < nf ? bins[static_cast<int64_t>(row[u]) * F + f0 + fl] : 0;
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (row[u] >= 0 && fl < nf) {
        const int e = fl * B + b[u];
        atomicAdd(qlds + e, __float2int_rn(g[u] * sg));
        atomicAdd(qh_pl + e, __float2int_rn(h[u] * sh));
      }
    }
  }
  __syncthreads();
  float* out = hist + (static_cast<int64_t>(j) * F + f0) * B * 2;
  const float ig = sg > 0.f ? 1.f / sg : 0.f, ih = sh > 0.f ? 1.f / sh : 0.f;
  for (int i = t; i < nf * B; i += kHistBlock) {
    const int vg = qlds[i], vh = qh_pl[i];
    if (vg != 0) __hip_atomic_fetch_add(out + 2 * i, static_cast<float>(vg) * ig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (vh != 0) __hip_atomic_fetch_add(out + 2 * i + 1, static_cast<float>(vh) * ih, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Row-per-lane variant (F % 4 == 0): each lane owns whole rows -- its row
// index, g / h quantised once per row, and the row's fp bin codes as NW = fp / 4
// dword loads -- so a wave's memory instructions cover 64 rows x fp features;
// the slot kernel above issues a row-index, g, h and a byte load per 64
// (row, feature) pairs.  Same chunks, same fixed-point values, same integer
// block sums (exact, so order-free): the flushed histogram equals the slot
// kernel's up to the order of the fp32 flush atomics.  LDS holds nf = min(fp, F - f0)
// feature planes (g [nf][B] then h [nf][B]).
// The chunk plan (hist_plan_kernel's prefix of ceil(size / rpb) over the nb
// built nodes) is computed by wave 0 of every block into LDS: no plan launch
// per level (nb <= kPlanMax).
constexpr int kPlanMax = 1024;

// P64: g and h packed into one 64-bit LDS add (ds_add_u64): g's fixed-point
// value in the high word (two's complement, |block sum| < 2^31), h's in the low
// word (non-negative, block sum <= 2^30: no carry into g) -- half the LDS atomics
template <int U, int NW, bool P64 = false>
__global__ __launch_bounds__(kHistBlock) void hist_build_rows_kernel(
    const uint8_t* __restrict__ bins, const float* __restrict__ grad, const float* __restrict__ hess,
    int64_t gh_stride, const int32_t* __restrict__ rows, const int32_t* __restrict__ blo,
    const int32_t* __restrict__ bhi, int nb, int F, int B, int rpb, int fp,
    const float* __restrict__ gh_max, float* __restrict__ hist, int flush) {
  // 16-B aligned: the dynamic planes start after the static s_off, and P64's
  // 8-byte LDS atomics fault on a 4-byte-aligned address
  extern __shared__ __attribute__((aligned(16))) int qlds[];
  __shared__ __attribute__((aligned(16))) int s_off[kPlanMax + 4];
  const int t = threadIdx.x;
  if (t < 64) {  // wave 0: inclusive wave scans, 64 nodes at a time
    int carry = 0;
    if (t == 0) s_off[0] = 0;
    for (int j0 = 0; j0 < nb; j0 += 64) {
      const int jj = j0 + t;
      int n = 0;
      if (jj < nb) {
        const int sz = bhi[jj] - blo[jj];
        n = sz > 0 ? (sz + rpb - 1) / rpb : 0;
      }
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(n, o, 64);
        if (t >= o) n += u;
      }
      if (jj < nb) s_off[jj + 1] = carry + n;
      carry += __shfl(n, 63, 64);
    }
  }
  __syncthreads();
  const int c = blockIdx.x;
  if (c >= s_off[nb]) return;  // block-uniform
  int a = 0, z = nb;
  while (z - a > 1) {
    const int m = (a + z) >> 1;
    if (s_off[m] <= c) a = m; else z = m;
  }
  const int j = a;
  const int r0 = blo[j] + (c - s_off[j]) * rpb;
  const int r1 = (r0 + rpb) < bhi[j] ? (r0 + rpb) : bhi[j];
  const int f0 = blockIdx.y * fp;
  const int nf = (F - f0) < fp ? (F - f0) : fp;  // a multiple of 4 (F % 4 == 0, fp % 4 == 0)
  int* qh_pl = qlds + nf * B;
  const float mg = gh_max[0], mh = gh_max[1];
  const float sg = mg > 0.f ? kQuantRange / (static_cast<float>(rpb) * mg) : 0.f;
  const float sh = mh > 0.f ? kQuantRange / (static_cast<float>(rpb) * mh) : 0.f;
  for (int i = t; i < 2 * nf * B; i += kHistBlock) qlds[i] = 0;
  __syncthreads();
  const int nw = nf >> 2;
  for (int base = r0 + t; base < r1; base += kHistBlock * U) {
    int row[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = base + u * kHistBlock;
      row[u] = r < r1 ? rows[r] : -1;
    }
    int qg[U], qh[U];
    uint32_t w[U][NW];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t rr = row[u] >= 0 ? row[u] : 0;  // unconditional loads (row 0 for an idle slot)
      qg[u] = __float2int_rn(grad[rr * gh_stride] * sg);
      qh[u] = __float2int_rn(hess[rr * gh_stride] * sh);
      const uint32_t* bw = reinterpret_cast<const uint32_t*>(bins + rr * F + f0);
#pragma unroll
      for (int k = 0; k < NW; ++k) w[u][k] = k < nw ? bw[k] : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (row[u] < 0) continue;
#pragma unroll
      for (int k = 0; k < NW; ++k) {
        if (k >= nw) break;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = (4 * k + q) * B + ((w[u][k] >> (8 * q)) & 255u);
          if constexpr (P64) {
            // (a negative hessian -- no objective here produces one -- is clamped to 0
            // rather than borrowing from g's word)
            atomicAdd(reinterpret_cast<unsigned long long*>(qlds) + e,
                      (static_cast<unsigned long long>(static_cast<uint32_t>(qg[u])) << 32) |
                          static_cast<uint32_t>(qh[u] > 0 ? qh[u] : 0));
          } else {
            atomicAdd(qlds + e, qg[u]);
            atomicAdd(qh_pl + e, qh[u]);
          }
        }
      }
    }
  }
  __syncthreads();
  if (!flush) {  // timing only (KDL_TUNE gbdt_price_noflush): keep the sums alive, skip the atomics
    if (t == 0 && qlds[0] == 0x7fffffff) hist[0] = 0.f;
    return;
  }
  float* out = hist + (static_cast<int64_t>(j) * F + f0) * B * 2;
  const float ig = sg > 0.f ? 1.f / sg : 0.f, ih = sh > 0.f ? 1.f / sh : 0.f;
  for (int i = t; i < nf * B; i += kHistBlock) {
    int vg, vh;
    if constexpr (P64) {
      const unsigned long long v = reinterpret_cast<const unsigned long long*>(qlds)[i];
      vg = static_cast<int>(static_cast<uint32_t>(v >> 32));
      vh = static_cast<int>(static_cast<uint32_t>(v));
    } else {
      vg = qlds[i];
      vh = qh_pl[i];
    }
    if (vg != 0) __hip_atomic_fetch_add(out + 2 * i, static_cast<float>(vg) * ig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (vh != 0) __hip_atomic_fetch_add(out + 2 * i + 1, static_cast<float>(vh) * ih, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// {max |g|, max h} over n rows into out[2] (zeroed by the caller): a block max,
// then one integer atomicMax per value (non-negative floats order as their bits)
// (n4 > 0: g and h 16-B aligned, read as float4 up to 4 n4, the tail as floats)
__global__ __launch_bounds__(256) void gh_absmax_kernel(const float* __restrict__ g, const float* __restrict__ h,
                                                        int n, int n4, unsigned* __restrict__ out) {
  float mg = 0.f, mh = 0.f;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const float4* h4 = reinterpret_cast<const float4*>(h);
#pragma unroll 4
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) {
    const float4 a = g4[i], b = h4[i];
    mg = fmaxf(mg, fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))));
    mh = fmaxf(mh, fmaxf(fmaxf(fabsf(b.x), fabsf(b.y)), fmaxf(fabsf(b.z), fabsf(b.w))));
  }
  for (int i = 4 * n4 + blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    mg = fmaxf(mg, fabsf(g[i]));
    mh = fmaxf(mh, fabsf(h[i]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mg = fmaxf(mg, __shfl_xor(mg, o));
    mh = fmaxf(mh, __shfl_xor(mh, o));
  }
  __shared__ float sm[2][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { sm[0][w] = mg; sm[1][w] = mh; }
  __syncthreads();
  if (threadIdx.x == 0) {
    mg = fmaxf(fmaxf(sm[0][0], sm[0][1]), fmaxf(sm[0][2], sm[0][3]));
    mh = fmaxf(fmaxf(sm[1][0], sm[1][1]), fmaxf(sm[1][2], sm[1][3]));
    atomicMax(out, __float_as_uint(mg));
    atomicMax(out + 1, __float_as_uint(mh));
  }
}

// one thread: chunk_off[j+1] = chunk_off[j] + ceil((bhi[j] - blo[j]) / rpb)
__global__ void hist_plan_kernel(const int32_t* __restrict__ blo, const int32_t* __restrict__ bhi, int nb, int rpb,
                                 int32_t* __restrict__ chunk_off) {
  if (threadIdx.x != 0) return;
  int acc = 0;
  chunk_off[0] = 0;
  for (int j = 0; j < nb; ++j) {
    const int n = bhi[j] - blo[j];
    acc += n > 0 ? (n + rpb - 1) / rpb : 0;
    chunk_off[j + 1] = acc;
  }
}

// thread per level node i (heap id h0 + i): best feature (ties -> lower id),
// split decision, leaf weight, tree arrays; split[i] and the children's
// existence for the next level.
__global__ __launch_bounds__(256) void decide_kernel(
    const float* __restrict__ gain, const int32_t* __restrict__ sbin, const float* __restrict__ tot,
    const float* __restrict__ cuts, const int32_t* __restrict__ exists, int L, int F, int ncut, int h0,
    int can_split, float lambda, float gamma, float lr, int32_t* __restrict__ t_feat,
    int32_t* __restrict__ t_bin, float* __restrict__ t_thr, float* __restrict__ t_val, int32_t* __restrict__ split,
    int32_t* __restrict__ exists_next) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= L) return;
  const int h = h0 + i;
  const bool ex = exists[i] != 0;
  float bg = -INFINITY;
  int bf = -1;
  for (int f = 0; f < F; ++f) {
    const float v = gain[static_cast<int64_t>(i) * F + f];
    if (v > bg) {
      bg = v;
      bf = f;
    }
  }
  const bool sp = ex && can_split && bf >= 0 && bg > gamma && bg < INFINITY;
  const int bb = sp ? sbin[static_cast<int64_t>(i) * F + bf] : -1;
  t_feat[h] = sp ? bf : -1;
  t_bin[h] = bb;
  t_thr[h] = sp ? (bb < ncut ? cuts[static_cast<int64_t>(bf) * ncut + bb] : INFINITY) : 0.f;
  t_val[h] = ex ? -tot[2 * i] / (tot[2 * i + 1] + lambda) * lr : 0.f;
  split[i] = sp ? 1 : 0;
  if (exists_next != nullptr) {
    exists_next[2 * i] = sp ? 1 : 0;
    exists_next[2 * i + 1] = sp ? 1 : 0;
  }
}

// flag[p] = 1 when the row at position p belongs to a splitting node of the
// level and goes right.  ``node_pos`` is POSITION-indexed (the heap node of the
// row at position p, moved with the rows by partition_kernel): a coalesced read
// where a row-indexed node id was a dependent random gather (both kernels are
// latency-bound: waves parked ~90 % of their cycles, scripts/gpu_r06_gbdt_pmc.sh).
// kRouteItems positions per thread (strided by the block width: coalesced), every
// level of the dependent load chain (row / node -> split, feature, bin -> the
// row's bin code) issued for all items before the next level is used
constexpr int kRouteItems = 4;

// The bin code of (row, f) is bins[row * rs + f * fs]: row-major [N, F] (rs = F,
// fs = 1) or the grower's feature-major copy [F, N] (rs = 1, fs = N) -- a node's
// rows keep their original order (stable partitions), so at shallow levels
// consecutive positions read nearby bytes of one feature's column instead of
// one 64-B sector per position.
__global__ __launch_bounds__(256) void route_flags_kernel(
    const uint8_t* __restrict__ bins, const int32_t* __restrict__ rows, const int32_t* __restrict__ node_pos,
    const int32_t* __restrict__ split, const int32_t* __restrict__ t_feat, const int32_t* __restrict__ t_bin,
    int64_t rs, int64_t fs, int n, int h0, int L, int32_t* __restrict__ flag) {
  const int p0 = blockIdx.x * 256 * kRouteItems + threadIdx.x;
  int row[kRouteItems], i[kRouteItems], sp[kRouteItems], fe[kRouteItems], tb[kRouteItems];
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    const int p = p0 + k * 256;
    row[k] = p < n ? rows[p] : 0;
    i[k] = p < n ? node_pos[p] - h0 : -1;
  }
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    const bool in = i[k] >= 0 && i[k] < L;
    sp[k] = in ? split[i[k]] : 0;
    fe[k] = in ? t_feat[h0 + i[k]] : 0;
    tb[k] = in ? t_bin[h0 + i[k]] : 0;
  }
  int b[kRouteItems];
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) b[k] = sp[k] ? bins[row[k] * rs + fe[k] * fs] : 0;
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    const int p = p0 + k * 256;
    if (p < n) flag[p] = (sp[k] && b[k] > tb[k]) ? 1 : 0;
  }
}

// Route + inclusive scan of the flags in one launch (replaces route_flags_kernel
// and a two-launch device scan): single-pass scan with decoupled look-back.
// A block takes the next tile of kScanTile positions from a ticket (tiles are
// handed out in start order, so a block only ever waits on tiles of blocks
// that are already running), routes its 8 positions per thread with every
// load issued first, scans the tile in registers / LDS, publishes its
// aggregate, looks back over its predecessors' words 64 at a time (wave 0)
// until one holds an inclusive prefix, and publishes its own.  A status word
// is one 8-B agent-scope atomic: epoch (31 bits) | state (2: aggregate,
// prefix) | value (31 bits) -- the payload travels in the flag word, and a
// word of an earlier launch (older epoch) reads as not ready, so the array is
// never reset.  A poll that does not become ready within kScanSpins (a
// protocol bug, never expected) records a fault instead of hanging the GPU.
constexpr int kScanItems = 8;
constexpr int kScanTile = 256 * kScanItems;
constexpr int kScanSpins = 1 << 22;

__device__ __forceinline__ unsigned long long scan_word(uint32_t epoch, uint32_t state, uint32_t v) {
  return (static_cast<unsigned long long>(epoch) << 33) | (static_cast<unsigned long long>(state) << 31) | v;
}

__global__ __launch_bounds__(256) void route_scan_kernel(
    const uint8_t* __restrict__ bins, const int32_t* __restrict__ rows, const int32_t* __restrict__ node_pos,
    const int32_t* __restrict__ split, const int32_t* __restrict__ t_feat, const int32_t* __restrict__ t_bin,
    int F, int n, int h0, int L, int32_t* __restrict__ flag, int32_t* __restrict__ sc,
    unsigned long long* __restrict__ status, unsigned* __restrict__ ticket, uint32_t epoch, int* __restrict__ fault) {
  __shared__ int s_tile, s_excl;
  __shared__ int s_wsum[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) s_tile = static_cast<int>(__hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  __syncthreads();
  const int tile = s_tile;
  const int p0 = tile * kScanTile + t * kScanItems;
  int row[kScanItems], hn[kScanItems];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int p = p0 + k;
    row[k] = p < n ? rows[p] : 0;
    hn[k] = p < n ? node_pos[p] : -1;
  }
  int f[kScanItems];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int i = hn[k] - h0;
    f[k] = (i >= 0 && i < L && split[i]) ? 1 : 0;
    if (f[k]) {
      const int h = hn[k];
      f[k] = bins[static_cast<int64_t>(row[k]) * F + t_feat[h]] > t_bin[h] ? 1 : 0;
    }
  }
  int incl[kScanItems];
  int run = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    run += f[k];
    incl[k] = run;
    if (p0 + k < n) flag[p0 + k] = f[k];
  }
  // block scan of the thread totals
  int x = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(x, o, 64);
    if (lane >= o) x += u;
  }
  if (lane == 63) s_wsum[w] = x;
  __syncthreads();
  int wexcl = 0, agg = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < w) wexcl += s_wsum[k];
    agg += s_wsum[k];
  }
  const int texcl = wexcl + x - run;  // positions of earlier threads in this tile
  if (w == 0) {
    int excl = 0;
    if (tile == 0) {
      if (lane == 0)
        __hip_atomic_store(status, scan_word(epoch, 2u, static_cast<uint32_t>(agg)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0)
        __hip_atomic_store(status + tile, scan_word(epoch, 1u, static_cast<uint32_t>(agg)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      int j = tile - 1;
      bool bad = false;
      while (true) {
        const int jj = j - lane;
        uint32_t state = 2u, val = 0u;  // past tile 0: a virtual zero prefix
        if (jj >= 0) {
          int spins = 0;
          do {
            const unsigned long long wd = __hip_atomic_load(status + jj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            state = static_cast<uint32_t>(wd >> 33) == epoch ? static_cast<uint32_t>((wd >> 31) & 3u) : 0u;
            val = static_cast<uint32_t>(wd & 0x7fffffffu);
          } while (state == 0u && ++spins < kScanSpins);
          if (state == 0u) {
            bad = true;
            state = 2u;
            val = 0u;
          }
        }
        const unsigned long long pm = __ballot(state == 2u);
        const int stop = pm ? __ffsll(static_cast<long long>(pm)) - 1 : 64;
        int c = lane <= stop ? static_cast<int>(val) : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        excl += c;
        if (pm) break;
        j -= 64;
      }
      if (__ballot(bad) && lane == 0) atomicAdd(fault, 1);
      if (lane == 0)
        __hip_atomic_store(status + tile, scan_word(epoch, 2u, static_cast<uint32_t>(excl + agg)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) s_excl = excl;
  }
  __syncthreads();
  const int base = s_excl + texcl;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (p0 + k < n) sc[p0 + k] = base + incl[k];
  // every block has drawn its ticket once the last tile is handed out: re-arm
  if (t == 0 && tile == static_cast<int>(gridDim.x) - 1)
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// stable in-segment partition by flag (sc = inclusive scan of flag over all
// positions): left rows first, then right rows, each in their old order.
// (kRouteItems positions per thread, each load level issued for all of them first)
__global__ __launch_bounds__(256) void partition_kernel(
    const int32_t* __restrict__ rows, const int32_t* __restrict__ node_pos, const int32_t* __restrict__ split,
    const int32_t* __restrict__ lo, const int32_t* __restrict__ hi, const int32_t* __restrict__ flag,
    const int32_t* __restrict__ sc, int n, int h0, int L, int32_t* __restrict__ rows_next,
    int32_t* __restrict__ node_pos_next) {
  const int p0 = blockIdx.x * 256 * kRouteItems + threadIdx.x;
  int row[kRouteItems], hn[kRouteItems], fl[kRouteItems], scp[kRouteItems];
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    const int p = p0 + k * 256;
    const bool ok = p < n;
    row[k] = ok ? rows[p] : 0;
    hn[k] = ok ? node_pos[p] : -1;
    fl[k] = ok ? flag[p] : 0;
    scp[k] = ok ? sc[p] : 0;
  }
  int s0[kRouteItems], s1[kRouteItems], sp[kRouteItems];
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    const int i = hn[k] - h0;
    const bool in = i >= 0 && i < L;
    sp[k] = in ? split[i] : 0;
    s0[k] = in ? lo[i] : 0;
    s1[k] = in ? hi[i] : 0;
  }
  int base[kRouteItems], tot[kRouteItems];
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    base[k] = (sp[k] && s0[k] > 0) ? sc[s0[k] - 1] : 0;
    tot[k] = sp[k] ? sc[s1[k] - 1] : 0;
  }
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    const int p = p0 + k * 256;
    if (p >= n) continue;
    if (sp[k]) {
      const int rb = scp[k] - fl[k] - base[k];  // right rows before p in the segment
      const int nl = (s1[k] - s0[k]) - (tot[k] - base[k]);
      const int np = fl[k] ? s0[k] + nl + rb : s0[k] + (p - s0[k] - rb);
      rows_next[np] = row[k];
      node_pos_next[np] = fl[k] ? 2 * hn[k] + 2 : 2 * hn[k] + 1;
    } else {
      rows_next[p] = row[k];
      node_pos_next[p] = hn[k];
    }
  }
}

// ---- one level's routing + stable partition in three launches: route_count
// routes each tile of kTilePos positions and writes, besides the flags, the
// tile-local inclusive scan of the flags and the tile's total; level_plan (one
// block) scans the tile totals into tile offsets, so the global count of
// right-goers before position x is P(x) = tile_off[tile(x - 1)] + tincl[x - 1],
// and takes each node's right count P(hi) - P(lo) and base P(lo) from its
// segment ends, then writes the child segments (children_kernel's outputs);
// partition places every row as partition_kernel does, from tile_off + tincl.
// Replaces route_flags, the two-launch device scan, partition and children.
constexpr int kTilePos = 256 * kRouteItems;  // positions per tile (one block)

__device__ __forceinline__ int block_incl_scan256(int v, int* wsum) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(x, o, 64);
    if (lane >= o) x += u;
  }
  __syncthreads();  // wsum reuse across calls
  if (lane == 63) wsum[w] = x;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (k < w) x += wsum[k];
  return x;  // inclusive; wsum[0..3] hold the wave totals (block total = their sum)
}

__global__ __launch_bounds__(256) void route_count_kernel(
    const uint8_t* __restrict__ bins, const int32_t* __restrict__ rows, const int32_t* __restrict__ node_pos,
    const int32_t* __restrict__ split, const int32_t* __restrict__ t_feat, const int32_t* __restrict__ t_bin,
    int64_t rs, int64_t fs, int n, int h0, int L, int32_t* __restrict__ flag, int32_t* __restrict__ tincl,
    int32_t* __restrict__ tile_cnt) {
  __shared__ int wsum[4];
  const int p0 = blockIdx.x * kTilePos + threadIdx.x;
  int row[kRouteItems], i[kRouteItems], sp[kRouteItems], fe[kRouteItems], tb[kRouteItems];
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    const int p = p0 + k * 256;
    row[k] = p < n ? rows[p] : 0;
    i[k] = p < n ? node_pos[p] - h0 : -1;
  }
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    const bool in = i[k] >= 0 && i[k] < L;
    sp[k] = in ? split[i[k]] : 0;
    fe[k] = in ? t_feat[h0 + i[k]] : 0;
    tb[k] = in ? t_bin[h0 + i[k]] : 0;
  }
  int b[kRouteItems];
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) b[k] = sp[k] ? bins[row[k] * rs + fe[k] * fs] : 0;
  int before = 0;  // right-goers of this tile before position p0 + 256 k (k-major, then thread order)
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    const int p = p0 + k * 256;
    const int f = (sp[k] && b[k] > tb[k]) ? 1 : 0;
    const int incl = before + block_incl_scan256(f, wsum);
    before += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (p < n) {
      flag[p] = f;
      tincl[p] = incl;
    }
  }
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = before;
}

// one block of 1024 threads: tile offsets (exclusive scan of tile_cnt), each
// node's base P(lo) and right count P(hi) - P(lo), the children's segments /
// counts / built-child choice as children_kernel
__global__ __launch_bounds__(1024) void level_plan_kernel(
    const int32_t* __restrict__ tile_cnt, int ntiles, int32_t* __restrict__ tile_off, const int32_t* __restrict__ tincl,
    const int32_t* __restrict__ split, const int32_t* __restrict__ lo, const int32_t* __restrict__ hi, int L,
    int32_t* __restrict__ node_base, int32_t* __restrict__ node_r, int32_t* __restrict__ lo_next,
    int32_t* __restrict__ hi_next, float* __restrict__ cnt, int pick, int32_t* __restrict__ build_child,
    int32_t* __restrict__ blo, int32_t* __restrict__ bhi) {
  __shared__ int wsum[16];
  __shared__ int s_carry;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) s_carry = 0;
  __syncthreads();
  for (int b0 = 0; b0 < ntiles; b0 += 1024) {
    const int j = b0 + t;
    const int v = j < ntiles ? tile_cnt[j] : 0;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(x, o, 64);
      if (lane >= o) x += u;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int pre = s_carry, tot = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (k < w) pre += wsum[k];
      tot += wsum[k];
    }
    if (j < ntiles) tile_off[j] = pre + x - v;
    __syncthreads();
    if (t == 0) s_carry += tot;
    __syncthreads();
  }
  // (tile_off is read back below by other threads: the loop's last barrier orders it)
  auto P = [&](int x) {  // right-goers in positions [0, x)
    if (x <= 0) return 0;
    return tile_off[(x - 1) / kTilePos] + tincl[x - 1];
  };
  for (int i = t; i < L; i += 1024) {
    int a0 = 0, a1 = 0, b0 = 0, b1 = 0, base = 0, r = 0;
    if (split[i] && hi[i] > lo[i]) {  // a node split on the global histogram may own no rows here
      const int s0 = lo[i], s1 = hi[i];
      base = P(s0);
      r = P(s1) - base;
      const int nl = (s1 - s0) - r;
      a0 = s0;
      a1 = s0 + nl;
      b0 = s0 + nl;
      b1 = s1;
    }
    node_base[i] = base;
    node_r[i] = r;
    lo_next[2 * i] = a0;
    hi_next[2 * i] = a1;
    lo_next[2 * i + 1] = b0;
    hi_next[2 * i + 1] = b1;
    cnt[2 * i] = static_cast<float>(a1 - a0);
    cnt[2 * i + 1] = static_cast<float>(b1 - b0);
    if (pick) {
      const int c = (a1 - a0) <= (b1 - b0) ? 0 : 1;
      build_child[i] = 2 * i + c;
      blo[i] = c ? b0 : a0;
      bhi[i] = c ? b1 : a1;
    }
  }
}

__global__ __launch_bounds__(256) void partition_tiles_kernel(
    const int32_t* __restrict__ rows, const int32_t* __restrict__ node_pos, const int32_t* __restrict__ split,
    const int32_t* __restrict__ lo, const int32_t* __restrict__ hi, const int32_t* __restrict__ flag,
    const int32_t* __restrict__ tincl, const int32_t* __restrict__ tile_off, const int32_t* __restrict__ node_base,
    const int32_t* __restrict__ node_r, int n, int h0, int L, int32_t* __restrict__ rows_next,
    int32_t* __restrict__ node_pos_next) {
  const int p0 = blockIdx.x * kTilePos + threadIdx.x;
  const int toff = tile_off[blockIdx.x];
  int row[kRouteItems], hn[kRouteItems], fl[kRouteItems], inc[kRouteItems];
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    const int p = p0 + k * 256;
    const bool ok = p < n;
    row[k] = ok ? rows[p] : 0;
    hn[k] = ok ? node_pos[p] : -1;
    fl[k] = ok ? flag[p] : 0;
    inc[k] = ok ? tincl[p] : 0;
  }
  int s0[kRouteItems], s1[kRouteItems], sp[kRouteItems], nb[kRouteItems], nr[kRouteItems];
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    const int i = hn[k] - h0;
    const bool in = i >= 0 && i < L;
    sp[k] = in ? split[i] : 0;
    s0[k] = sp[k] ? lo[i] : 0;
    s1[k] = sp[k] ? hi[i] : 0;
    nb[k] = sp[k] ? node_base[i] : 0;
    nr[k] = sp[k] ? node_r[i] : 0;
  }
#pragma unroll
  for (int k = 0; k < kRouteItems; ++k) {
    const int p = p0 + k * 256;
    if (p >= n) continue;
    if (sp[k]) {
      const int r_in = toff + inc[k] - fl[k] - nb[k];  // right rows before p in the segment
      const int nl = (s1[k] - s0[k]) - nr[k];
      const int np = fl[k] ? s0[k] + nl + r_in : s0[k] + (p - s0[k] - r_in);
      rows_next[np] = row[k];
      node_pos_next[np] = fl[k] ? 2 * hn[k] + 2 : 2 * hn[k] + 1;
    } else {
      rows_next[p] = row[k];
      node_pos_next[p] = hn[k];
    }
  }
}

// thread per parent i: child segments and counts; when ``pick`` (counts are
// already global) also the built (smaller) child and its segment.
__global__ __launch_bounds__(256) void children_kernel(
    const int32_t* __restrict__ split, const int32_t* __restrict__ lo, const int32_t* __restrict__ hi,
    const int32_t* __restrict__ sc, int L, int32_t* __restrict__ lo_next, int32_t* __restrict__ hi_next,
    float* __restrict__ cnt, int pick, int32_t* __restrict__ build_child, int32_t* __restrict__ blo,
    int32_t* __restrict__ bhi) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= L) return;
  int a0 = 0, a1 = 0, b0 = 0, b1 = 0;
  // a node split on the global histogram may own no rows on this rank
  if (split[i] && hi[i] > lo[i]) {
    const int s0 = lo[i], s1 = hi[i];
    const int base = s0 > 0 ? sc[s0 - 1] : 0;
    const int nl = (s1 - s0) - (sc[s1 - 1] - base);
    a0 = s0;
    a1 = s0 + nl;
    b0 = s0 + nl;
    b1 = s1;
  }
  lo_next[2 * i] = a0;
  hi_next[2 * i] = a1;
  lo_next[2 * i + 1] = b0;
  hi_next[2 * i + 1] = b1;
  cnt[2 * i] = static_cast<float>(a1 - a0);
  cnt[2 * i + 1] = static_cast<float>(b1 - b0);
  if (pick) {
    const int c = (a1 - a0) <= (b1 - b0) ? 0 : 1;
    build_child[i] = 2 * i + c;
    blo[i] = c ? b0 : a0;
    bhi[i] = c ? b1 : a1;
  }
}

__global__ __launch_bounds__(256) void pick_small_kernel(const float* __restrict__ cnt,
                                                         const int32_t* __restrict__ lo_next,
                                                         const int32_t* __restrict__ hi_next, int L,
                                                         int32_t* __restrict__ build_child, int32_t* __restrict__ blo,
                                                         int32_t* __restrict__ bhi) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= L) return;
  const int c = 2 * i + (cnt[2 * i] <= cnt[2 * i + 1] ? 0 : 1);
  build_child[i] = c;
  blo[i] = lo_next[c];
  bhi[i] = hi_next[c];
}

// hist_next[build_child[i]] = built[i]; hist_next[sibling] = parent[i] - built[i]
// (zero below a non-split parent).  float4 per thread over [L][F*B*2].  built[i]
// is zeroed once read: the next level's build accumulates into a zeroed buffer
// without a fill launch (the grower's built_ starts zeroed; a complete tree's
// last level leaves all of it zero).
__global__ __launch_bounds__(256) void subtract_kernel(const float4* __restrict__ parent,
                                                       float4* __restrict__ built,
                                                       const int32_t* __restrict__ split,
                                                       const int32_t* __restrict__ build_child, int L, int per_node4,
                                                       float4* __restrict__ next) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= static_cast<int64_t>(L) * per_node4) return;
  const int i = static_cast<int>(e / per_node4);
  const int64_t k = e - static_cast<int64_t>(i) * per_node4;
  const int c = build_child[i];
  const float4 b = built[e];
  built[e] = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 sib = make_float4(0.f, 0.f, 0.f, 0.f);
  if (split[i]) {
    const float4 pa = parent[e];
    sib = make_float4(pa.x - b.x, pa.y - b.y, pa.z - b.z, pa.w - b.w);
  }
  next[static_cast<int64_t>(c) * per_node4 + k] = b;
  next[static_cast<int64_t>(c ^ 1) * per_node4 + k] = sib;
}

__global__ __launch_bounds__(256) void quantise_kernel(const float* __restrict__ X, const float* __restrict__ cuts,
                                                       int64_t n, int F, int ncut, int max_code,
                                                       uint8_t* __restrict__ out) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= n * F) return;
  const int f = static_cast<int>(e % F);
  const float x = X[e];
  const float* c = cuts + static_cast<int64_t>(f) * ncut;
  int a = 0, z = ncut;  // first index with c[idx] >= x
  while (a < z) {
    const int m = (a + z) >> 1;
    if (c[m] < x) a = m + 1; else z = m;
  }
  out[e] = static_cast<uint8_t>(a < max_code ? a : max_code);
}

// Gradient / hessian of a boosting round in one pass over (pred, y):
//   obj 0 reg:squarederror   g = p - y,            h = 1
//   obj 1 binary:logistic    s = 1 / (1 + e^-p),   g = s - y,     h = max(s (1 - s), 1e-16)
//   obj 2 multi:softprob     s = softmax_k(p),     g = s - [y == k], h = max(2 s (1 - s), 1e-16)
// pred / g / h are [n, K] row-major (K = 1 except multi); one thread per row.
// The same fp32 expressions as the torch composition (models/gbdt.py) -- one
// launch instead of ~5 elementwise kernels per round.
__global__ __launch_bounds__(256) void grad_hess_kernel(const float* __restrict__ pred, const float* __restrict__ y,
                                                        int64_t n, int K, int obj, float* __restrict__ g,
                                                        float* __restrict__ h) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const float yi = y[i];
  if (obj == 0) {
    for (int k = 0; k < K; ++k) {
      g[i * K + k] = pred[i * K + k] - yi;
      h[i * K + k] = 1.f;
    }
  } else if (obj == 1) {
    const float s = 1.f / (1.f + expf(-pred[i]));
    g[i] = s - yi;
    h[i] = fmaxf(s * (1.f - s), 1e-16f);
  } else {
    float mx = -INFINITY;
    for (int k = 0; k < K; ++k) mx = fmaxf(mx, pred[i * K + k]);
    float z = 0.f;
    for (int k = 0; k < K; ++k) z += expf(pred[i * K + k] - mx);
    const int cls = static_cast<int>(yi);
    for (int k = 0; k < K; ++k) {
      const float s = expf(pred[i * K + k] - mx) / z;
      g[i * K + k] = s - (k == cls ? 1.f : 0.f);
      h[i * K + k] = fmaxf(2.f * s * (1.f - s), 1e-16f);
    }
  }
}

// A tree's state reset in one launch (was eight torch fills / copies per tree):
// rows = iota, every row at the root, empty heap arrays, the root's bounds and
// zeroed root histogram.
__global__ __launch_bounds__(256) void tree_init_kernel(int32_t* __restrict__ rows, int32_t* __restrict__ node_pos,
                                                        int N, int32_t* __restrict__ feat, int32_t* __restrict__ tbin,
                                                        float* __restrict__ thr, float* __restrict__ val, int heap,
                                                        int32_t* __restrict__ exists0, int32_t* __restrict__ lo0,
                                                        int32_t* __restrict__ hi0, float* __restrict__ root,
                                                        int root_n) {
  const int stride = gridDim.x * 256;
  const int t0 = blockIdx.x * 256 + threadIdx.x;
  for (int i = t0; i < N; i += stride) {
    rows[i] = i;
    node_pos[i] = 0;
  }
  for (int i = t0; i < heap; i += stride) {
    feat[i] = -1;
    tbin[i] = -1;
    thr[i] = 0.f;
    val[i] = 0.f;
  }
  for (int i = t0; i < root_n; i += stride) root[i] = 0.f;
  if (t0 == 0) {
    exists0[0] = 1;
    lo0[0] = 0;
    hi0[0] = N;
  }
}

// the row-indexed leaf of every row: node_of_row[rows[p]] = node_pos[p] (a
// scatter of plain stores), then pred[r * ld + k] += val[node_of_row[r]] with
// coalesced margins -- one position-ordered read-modify-write of pred measured
// 50 us per tree against ~20 for the pair
__global__ __launch_bounds__(256) void leaf_scatter_kernel(const int32_t* __restrict__ rows,
                                                           const int32_t* __restrict__ node_pos, int N,
                                                           int32_t* __restrict__ node_of_row) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p < N) node_of_row[rows[p]] = node_pos[p];
}

__global__ __launch_bounds__(256) void leaf_add_kernel(float* __restrict__ pred, int ld, int k,
                                                       const float* __restrict__ val,
                                                       const int32_t* __restrict__ node_of_row, int N) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r < N) pred[static_cast<int64_t>(r) * ld + k] += val[node_of_row[r]];
}

// [4, heap] fp32 (feature, split bin, threshold, value) of the current tree
__global__ __launch_bounds__(256) void heap_pack_kernel(const int32_t* __restrict__ feat,
                                                        const int32_t* __restrict__ tbin,
                                                        const float* __restrict__ thr, const float* __restrict__ val,
                                                        int heap, float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= heap) return;
  out[i] = static_cast<float>(feat[i]);
  out[heap + i] = static_cast<float>(tbin[i]);
  out[2 * heap + i] = thr[i];
  out[3 * heap + i] = val[i];
}

}  // namespace

hipError_t gbdt_grad_hess(const float* pred, const float* y, int64_t n, int K, int obj, float* g, float* h,
                          hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (obj < 0 || obj > 2 || K < 1 || (obj == 1 && K != 1)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(grad_hess_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, pred, y, n, K,
                     obj, g, h);
  return hipGetLastError();
}

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
    RETURN_IF_HIP_ERR(hipFuncSetAttribute(reinterpret_cast<const void*>(hist_build_kernel),
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
                           float* best_hl, float* node_tot, hipStream_t s) {
  if (num_nodes <= 0 || F <= 0) return hipSuccess;
  hipLaunchKernelGGL(split_find_kernel, dim3(F, num_nodes), dim3(256), 0, s, hist, F, B, lambda,
                     min_child_weight, best_gain, best_bin, best_gl, best_hl, node_tot);
  return hipGetLastError();
}

// features per block of the quantised build (a power of two up to the wave
// width); KDL_TUNE gbdt_ftile caps it below F: more, smaller blocks (LDS fp x B
// x 8 bytes each, more resident per CU) at the price of re-reading each row's
// index and g / h once per feature tile
static int hist_fp(int F) {
  static const int cap = [] { const int v = tune_int("gbdt_ftile", kFTile); return v < 1 ? 1 : v > kFTile ? kFTile : v; }();
  int fp = 1;
  while (fp < F && fp < cap) fp <<= 1;
  return fp;
}

static hipError_t hist_lds_attr() {
  static bool attr_set = false;
  if (!attr_set) {
    const int bytes = static_cast<int>(kFTile * 256 * 2 * sizeof(float));
    RETURN_IF_HIP_ERR(hipFuncSetAttribute(reinterpret_cast<const void*>(hist_build_wq_kernel<4>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    RETURN_IF_HIP_ERR(hipFuncSetAttribute(reinterpret_cast<const void*>(hist_build_wq_kernel<8>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    RETURN_IF_HIP_ERR(hipFuncSetAttribute(reinterpret_cast<const void*>(hist_build_wq_kernel<16>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    attr_set = true;
  }
  return hipSuccess;
}

template <int U, int NW, bool P64>
static hipError_t rows_lds_attr() {
  static bool attr_set = false;
  if (!attr_set) {
    RETURN_IF_HIP_ERR(hipFuncSetAttribute(reinterpret_cast<const void*>(hist_build_rows_kernel<U, NW, P64>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize,
                                          static_cast<int>(kFTile * 256 * 2 * sizeof(int))));
    attr_set = true;
  }
  return hipSuccess;
}

hipError_t gbdt_gh_absmax(const float* grad, const float* hess, int n, float* out, hipStream_t s) {
  RETURN_IF_HIP_ERR(hipMemsetAsync(out, 0, 2 * sizeof(float), s));
  if (n <= 0) return hipSuccess;
  // 128 blocks: each ends in two device-scope atomicMax on the same two words,
  // which serialise (1024 blocks: 27 us for 2M rows, the atomics not the 16 MB read)
  int blocks = (n + 1023) / 1024;
  if (blocks > 128) blocks = 128;
  const bool vec = ((reinterpret_cast<uintptr_t>(grad) | reinterpret_cast<uintptr_t>(hess)) & 15) == 0;
  hipLaunchKernelGGL(gh_absmax_kernel, dim3(blocks), dim3(256), 0, s, grad, hess, n, vec ? n / 4 : 0,
                     reinterpret_cast<unsigned*>(out));
  return hipGetLastError();
}

static int g_hist_rows = -2;  // -2: KDL_TUNE gbdt_hist_rows
void set_gbdt_hist_rows(int u) { g_hist_rows = u; }
static int g_pack64 = -1;  // -1: KDL_TUNE gbdt_pack64
void set_gbdt_pack64(int p) { g_pack64 = p < 0 ? -1 : (p != 0 ? 1 : 0); }

hipError_t gbdt_hist_wq(const uint8_t* bins, const float* grad, const float* hess, int64_t gh_stride,
                        const int32_t* rows, const int32_t* blo, const int32_t* bhi, int32_t* chunk_off, int nb,
                        int max_chunks, int rpb, int F, int B, const float* gh_max, float* hist, hipStream_t s) {
  if (nb <= 0 || F <= 0 || max_chunks <= 0) return hipSuccess;
  const int fp = hist_fp(F);
  RETURN_IF_HIP_ERR(hist_lds_attr());
  dim3 grid(max_chunks, (F + fp - 1) / fp);
  const size_t lds = static_cast<size_t>(fp) * B * 2 * sizeof(int);
  // row slots in flight per thread (KDL_TUNE gbdt_unroll: 4 | 8 | 16): the build waits on its
  // dependent row -> bins / g / h loads (PMC: waves parked 58 % of their cycles at 4); 2M x 28,
  // depth 6: 637-642 / 680-694 / 701-712 boosting rounds/s at 4 / 8 / 16, and 32 slots or 1024 /
  // 4096 rows per chunk no better than 16 (profiles/r06_gbdt_unroll.txt)
  static const int unroll = tune_int("gbdt_unroll", 16);
  // row-per-lane build (KDL_TUNE gbdt_hist_rows: 0 = slot kernel only; else its rows in flight per lane, 4 | 8)
  if (g_hist_rows == -2) g_hist_rows = tune_int("gbdt_hist_rows", 4);
  const int rows_u = g_hist_rows;
  static const bool noflush = tune_int("gbdt_price_noflush", 0) != 0;
  if (rows_u > 0 && F % 4 == 0 && fp >= 4 && nb <= kPlanMax) {
    const int nf0 = F < fp ? F : fp;  // the first (largest) tile's planes
    const size_t lds_r = static_cast<size_t>(nf0) * B * 2 * sizeof(int);
#define HIST_ROWS_LAUNCH(U, NW, P)                                                                                     \
  RETURN_IF_HIP_ERR((rows_lds_attr<U, NW, P>()));                                                                     \
  hipLaunchKernelGGL((hist_build_rows_kernel<U, NW, P>), grid, dim3(kHistBlock), lds_r, s, bins, grad, hess,         \
                     gh_stride, rows, blo, bhi, nb, F, B, rpb, fp, gh_max, hist, noflush ? 0 : 1)
#define HIST_ROWS_BY_U(U, P)                  \
  switch (fp / 4) {                            \
    case 1: HIST_ROWS_LAUNCH(U, 1, P); break;     \
    case 2: HIST_ROWS_LAUNCH(U, 2, P); break;     \
    case 4: HIST_ROWS_LAUNCH(U, 4, P); break;     \
    case 8: HIST_ROWS_LAUNCH(U, 8, P); break;     \
    default: HIST_ROWS_LAUNCH(U, 16, P); break;   \
  }
    // g and h in one 64-bit LDS add (the hessians of every objective here
    // are >= 0, as P64 needs): 1,500-1,501 -> 1,564-1,568 boosting rounds/s at 2M x 28
    // (profiles/r06_gbdt_pack64.txt); KDL_TUNE gbdt_pack64=0: two 32-bit adds
    if (g_pack64 < 0) g_pack64 = tune_int("gbdt_pack64", 1) != 0 ? 1 : 0;
    const bool pack64 = g_pack64 != 0;
    if (pack64 && rows_u >= 8) { HIST_ROWS_BY_U(8, true) }
    else if (pack64) { HIST_ROWS_BY_U(4, true) }
    else if (rows_u >= 8) { HIST_ROWS_BY_U(8, false) }
    else { HIST_ROWS_BY_U(4, false) }
#undef HIST_ROWS_BY_U
#undef HIST_ROWS_LAUNCH
    return hipGetLastError();
  }
  hipLaunchKernelGGL(hist_plan_kernel, dim3(1), dim3(64), 0, s, blo, bhi, nb, rpb, chunk_off);
#define HIST_WQ_LAUNCH(U)                                                                                         \
  hipLaunchKernelGGL((hist_build_wq_kernel<U>), grid, dim3(kHistBlock), lds, s, bins, grad, hess, gh_stride, rows, \
                     blo, bhi, chunk_off, nb, F, B, rpb, fp, gh_max, hist)
  if (unroll >= 16) HIST_WQ_LAUNCH(16);
  else if (unroll >= 8) HIST_WQ_LAUNCH(8);
  else HIST_WQ_LAUNCH(4);
#undef HIST_WQ_LAUNCH
  return hipGetLastError();
}

hipError_t gbdt_decide(const float* gain, const int32_t* sbin, const float* tot, const float* cuts,
                       const int32_t* exists, int L, int F, int ncut, int h0, int can_split, float lambda,
                       float gamma, float lr, int32_t* t_feat, int32_t* t_bin, float* t_thr, float* t_val,
                       int32_t* split, int32_t* exists_next, hipStream_t s) {
  if (L <= 0) return hipSuccess;
  hipLaunchKernelGGL(decide_kernel, dim3((L + 255) / 256), dim3(256), 0, s, gain, sbin, tot, cuts, exists, L, F,
                     ncut, h0, can_split, lambda, gamma, lr, t_feat, t_bin, t_thr, t_val, split, exists_next);
  return hipGetLastError();
}

hipError_t gbdt_route_flags(const uint8_t* bins, const int32_t* rows, const int32_t* node_pos,
                            const int32_t* split, const int32_t* t_feat, const int32_t* t_bin, int F, int n, int h0,
                            int L, int32_t* flag, hipStream_t s, bool feature_major) {
  if (n <= 0) return hipSuccess;
  const int64_t rs = feature_major ? 1 : F, fs = feature_major ? n : 1;
  hipLaunchKernelGGL(route_flags_kernel, dim3((n + 256 * kRouteItems - 1) / (256 * kRouteItems)), dim3(256), 0, s,
                     bins, rows, node_pos, split, t_feat, t_bin, rs, fs, n, h0, L, flag);
  return hipGetLastError();
}

int gbdt_route_scan_tiles(int n) { return (n + kScanTile - 1) / kScanTile; }

hipError_t gbdt_route_scan(const uint8_t* bins, const int32_t* rows, const int32_t* node_pos, const int32_t* split,
                           const int32_t* t_feat, const int32_t* t_bin, int F, int n, int h0, int L, int32_t* flag,
                           int32_t* sc, unsigned long long* status, unsigned* ticket, uint32_t epoch, int* fault,
                           hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (epoch == 0 || epoch >= (1u << 31)) return hipErrorInvalidValue;  // 0: the zeroed array's epoch
  hipLaunchKernelGGL(route_scan_kernel, dim3(gbdt_route_scan_tiles(n)), dim3(256), 0, s, bins, rows, node_pos, split,
                     t_feat, t_bin, F, n, h0, L, flag, sc, status, ticket, epoch, fault);
  return hipGetLastError();
}

hipError_t gbdt_partition(const int32_t* rows, const int32_t* node_pos, const int32_t* split, const int32_t* lo,
                          const int32_t* hi, const int32_t* flag, const int32_t* sc, int n, int h0, int L,
                          int32_t* rows_next, int32_t* node_pos_next, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(partition_kernel, dim3((n + 256 * kRouteItems - 1) / (256 * kRouteItems)), dim3(256), 0, s, rows,
                     node_pos, split, lo, hi, flag, sc, n, h0, L, rows_next, node_pos_next);
  return hipGetLastError();
}

int gbdt_level_tiles(int n) { return (n + kTilePos - 1) / kTilePos; }

hipError_t gbdt_route_partition(const uint8_t* bins, bool feature_major, int F, const int32_t* rows,
                                const int32_t* node_pos, const int32_t* split, const int32_t* t_feat,
                                const int32_t* t_bin, const int32_t* lo, const int32_t* hi, int n, int h0, int L,
                                int32_t* flag, int32_t* tincl, int32_t* tile_cnt, int32_t* tile_off,
                                int32_t* node_base, int32_t* node_r, int32_t* rows_next, int32_t* node_pos_next,
                                int32_t* lo_next, int32_t* hi_next, float* cnt, int pick, int32_t* build_child,
                                int32_t* blo, int32_t* bhi, hipStream_t s) {
  if (n <= 0 || L <= 0) return hipSuccess;
  const int nt = gbdt_level_tiles(n);
  const int64_t rs = feature_major ? 1 : F, fs = feature_major ? n : 1;
  hipLaunchKernelGGL(route_count_kernel, dim3(nt), dim3(256), 0, s, bins, rows, node_pos, split, t_feat, t_bin, rs, fs,
                     n, h0, L, flag, tincl, tile_cnt);
  hipLaunchKernelGGL(level_plan_kernel, dim3(1), dim3(1024), 0, s, tile_cnt, nt, tile_off, tincl, split, lo, hi, L,
                     node_base, node_r, lo_next, hi_next, cnt, pick, build_child, blo, bhi);
  hipLaunchKernelGGL(partition_tiles_kernel, dim3(nt), dim3(256), 0, s, rows, node_pos, split, lo, hi, flag, tincl,
                     tile_off, node_base, node_r, n, h0, L, rows_next, node_pos_next);
  return hipGetLastError();
}

hipError_t gbdt_children(const int32_t* split, const int32_t* lo, const int32_t* hi, const int32_t* sc, int L,
                         int32_t* lo_next, int32_t* hi_next, float* cnt, int pick, int32_t* build_child,
                         int32_t* blo, int32_t* bhi, hipStream_t s) {
  if (L <= 0) return hipSuccess;
  hipLaunchKernelGGL(children_kernel, dim3((L + 255) / 256), dim3(256), 0, s, split, lo, hi, sc, L, lo_next,
                     hi_next, cnt, pick, build_child, blo, bhi);
  return hipGetLastError();
}

hipError_t gbdt_pick_small(const float* cnt, const int32_t* lo_next, const int32_t* hi_next, int L,
                           int32_t* build_child, int32_t* blo, int32_t* bhi, hipStream_t s) {
  if (L <= 0) return hipSuccess;
  hipLaunchKernelGGL(pick_small_kernel, dim3((L + 255) / 256), dim3(256), 0, s, cnt, lo_next, hi_next, L,
                     build_child, blo, bhi);
  return hipGetLastError();
}

hipError_t gbdt_subtract(const float* parent, float* built, const int32_t* split, const int32_t* build_child,
                         int L, int per_node, float* next, hipStream_t s) {
  if (L <= 0) return hipSuccess;
  const int per4 = per_node / 4;
  const int64_t n = static_cast<int64_t>(L) * per4;
  hipLaunchKernelGGL(subtract_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(parent), reinterpret_cast<float4*>(built), split,
                     build_child, L, per4, reinterpret_cast<float4*>(next));
  return hipGetLastError();
}

hipError_t gbdt_quantise(const float* X, const float* cuts, int64_t n, int F, int ncut, int max_code, uint8_t* out,
                         hipStream_t s) {
  if (n <= 0 || F <= 0) return hipSuccess;
  const int64_t tot = n * F;
  hipLaunchKernelGGL(quantise_kernel, dim3(static_cast<unsigned>((tot + 255) / 256)), dim3(256), 0, s, X, cuts, n,
                     F, ncut, max_code, out);
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

hipError_t gbdt_tree_init(int32_t* rows, int32_t* node_pos, int N, int32_t* feat, int32_t* tbin, float* thr,
                          float* val, int heap, int32_t* exists0, int32_t* lo0, int32_t* hi0, float* root, int root_n,
                          hipStream_t s) {
  if (N < 0 || heap < 0 || root_n < 0) return hipErrorInvalidValue;
  int m = N > heap ? N : heap;
  if (root_n > m) m = root_n;
  int blocks = (m + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(tree_init_kernel, dim3(blocks), dim3(256), 0, s, rows, node_pos, N, feat, tbin, thr, val, heap,
                     exists0, lo0, hi0, root, root_n);
  return hipGetLastError();
}

hipError_t gbdt_leaf_add(float* pred, int ld, int k, const float* val, const int32_t* rows, const int32_t* node_pos,
                         int N, int32_t* node_of_row, hipStream_t s) {
  if (N <= 0) return hipSuccess;
  if (ld < 1 || k < 0 || k >= ld) return hipErrorInvalidValue;
  if (node_of_row == nullptr) return hipErrorInvalidValue;
  hipLaunchKernelGGL(leaf_scatter_kernel, dim3((N + 255) / 256), dim3(256), 0, s, rows, node_pos, N, node_of_row);
  hipLaunchKernelGGL(leaf_add_kernel, dim3((N + 255) / 256), dim3(256), 0, s, pred, ld, k, val, node_of_row, N);
  return hipGetLastError();
}

hipError_t gbdt_heap_pack(const int32_t* feat, const int32_t* tbin, const float* thr, const float* val, int heap,
                          float* out, hipStream_t s) {
  if (heap <= 0) return hipSuccess;
  hipLaunchKernelGGL(heap_pack_kernel, dim3((heap + 255) / 256), dim3(256), 0, s, feat, tbin, thr, val, heap, out);
  return hipGetLastError();
}

}  // namespace kdl
