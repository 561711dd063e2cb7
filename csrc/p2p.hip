// Peer-to-peer all-reduce over IPC-mapped device memory (xGMI on an MI355X node).
//
// Why not only RCCL: an 8-GPU MI355X node is a full mesh of point-to-point
// xGMI links (7 per GPU).  A ring all-reduce drives one link in each direction
// per step and pays 2(W-1) dependent steps of latency; reading all peers at
// once drives all 7 links concurrently and needs two dependent phases:
//
//   phase 1 (reduce-scatter, in place): rank r sums its chunk r of the bucket
//            over every rank's buffer (W loads in flight per 16-B unit, fp32
//            accumulation) and writes the sum into its own buffer;
//   phase 2 (all-gather, in place): rank r copies chunk j from rank j for all
//            j != r.
//
// Each phase is preceded by a cross-GPU barrier and the kernel ends with one,
// so no rank reuses its buffer while a peer may still read it.
//
// Barriers are per block: block b of rank r signals block b of every rank
// and waits for their signals.  The element -> (chunk, block) mapping is the
// same on every rank, so block b only ever reads bytes that block b of the
// owning rank wrote (or that were final before the kernel started).
// Signals are monotone epochs (one per call, same sequence on every rank) in
// [phase][block][src] slots of an uncached signal buffer per rank, so nothing
// is ever reset.  Stores become visible system-wide through a system-scope
// release (L2 write-back) in the signalling lane after every wave drained its
// stores; peer data is always read with sc0|sc1 (system-coherent) buffer loads,
// so no stale line of a previous call can be served from this GPU's caches.
//
// Small buckets take a one-shot path (each rank sums the whole bucket from all
// peers, two barriers); the caller picks it by size, identically on every rank.
//
// Every wait is bounded by the wall clock (s_memrealtime, 100 MHz): a peer
// that never arrives sets a bit in a host-mapped error word and the kernel
// drains instead of hanging the GPU.
//
// The reference has no collective code at all (discovery only,
// reference pkg/job_controller/service.go:263-276 gives the stable peer
// addresses); this is the MI355X transport SURVEY.md §5 asks for next to RCCL.
#include "common.h"
#include "kdl_api.h"

namespace kdl {
namespace {

constexpr int kP2PThreads = 256;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t p2p_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}

// sc0 | sc1: system-coherent load (misses every cache level that could hold a
// stale copy of the peer's line)
__device__ __forceinline__ uint4 p2p_load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 17);
  return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void p2p_barrier(const P2PArgs& a, int phase) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores have left the CU
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world) {
    const int slot = (phase * kP2PMaxBlocks + static_cast<int>(blockIdx.x)) * kP2PMaxRanks;
    // release (system): writes back this XCD's L2 before the flag lands on rank t
    __hip_atomic_store(a.sig[t] + slot + a.rank, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* mine = a.sig[a.rank] + slot + t;
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - a.epoch > 0x7fffffffu) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > a.timeout_ticks) {
        __hip_atomic_fetch_or(a.err, 1u << phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
}

// 16-byte unit = 8 bf16 or 4 fp32
template <bool BF16>
__device__ __forceinline__ void acc_unit(float (&s)[8], uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  if constexpr (BF16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s[2 * i] += __uint_as_float(w[i] << 16);
      s[2 * i + 1] += __uint_as_float(w[i] & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] += __uint_as_float(w[i]);
  }
}

template <bool BF16>
__device__ __forceinline__ uint4 pack_unit(const float (&s)[8], float scale) {
  if constexpr (BF16) {
    return make_uint4(pack_bf16x2(s[0] * scale, s[1] * scale), pack_bf16x2(s[2] * scale, s[3] * scale),
                      pack_bf16x2(s[4] * scale, s[5] * scale), pack_bf16x2(s[6] * scale, s[7] * scale));
  } else {
    return make_uint4(__float_as_uint(s[0] * scale), __float_as_uint(s[1] * scale),
                      __float_as_uint(s[2] * scale), __float_as_uint(s[3] * scale));
  }
}

template <bool BF16>
__global__ __launch_bounds__(kP2PThreads) void p2p_allreduce_kernel(P2PArgs a) {
  const int W = a.world, r = a.rank;
  const uint32_t units = a.units;                     // 16-B units in the bucket
  const uint32_t cs = (units + W - 1) / W;            // units per chunk
  const uint32_t step = gridDim.x * kP2PThreads;
  const uint32_t first = blockIdx.x * kP2PThreads + threadIdx.x;
  const uint32_t bytes = units * 16u;
  __amdgpu_buffer_rsrc_t rs[kP2PMaxRanks];
#pragma unroll
  for (int j = 0; j < kP2PMaxRanks; ++j) rs[j] = p2p_rsrc(a.buf[j < W ? j : 0], bytes);
  uint4* own = reinterpret_cast<uint4*>(a.buf[r]);

  p2p_barrier(a, 0);  // every rank's input is final
  {
    const uint32_t lo = r * cs, hi = min(units, lo + cs);
    for (uint32_t u = lo + first; u < hi; u += step) {
      uint4 v[kP2PMaxRanks];
#pragma unroll
      for (int j = 0; j < kP2PMaxRanks; ++j)
        if (j < W) v[j] = p2p_load(rs[j], u * 16u);
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < kP2PMaxRanks; ++j)
        if (j < W) acc_unit<BF16>(s, v[j]);
      own[u] = pack_unit<BF16>(s, a.scale);
    }
  }
  p2p_barrier(a, 1);  // every chunk is reduced
  for (int jj = 1; jj < W; ++jj) {
    const int j = (r + jj) % W;  // stagger the source rank so the links load evenly
    const uint32_t lo = j * cs, hi = min(units, lo + cs);
    constexpr int U = 4;  // 4 loads in flight per lane
    uint32_t u = lo + first;
    for (; u + (U - 1) * step < hi; u += U * step) {
      uint4 v[U];
#pragma unroll
      for (int i = 0; i < U; ++i) v[i] = p2p_load(rs[j], (u + i * step) * 16u);
#pragma unroll
      for (int i = 0; i < U; ++i) own[u + i * step] = v[i];
    }
    for (; u < hi; u += step) own[u] = p2p_load(rs[j], u * 16u);
  }
  p2p_barrier(a, 2);  // nobody reads this rank's buffer any more
}

// One-shot variant for small buckets (latency-bound): every rank sums the
// WHOLE bucket from all peers into registers (at most kOneShotUnits units per
// thread), waits until every rank has read every buffer, then writes its sums
// in place.  Two barriers and one round of peer reads instead of three and two.
constexpr int kOneShotUnits = 4;

template <bool BF16>
__global__ __launch_bounds__(kP2PThreads) void p2p_allreduce_oneshot_kernel(P2PArgs a) {
  const int W = a.world;
  const uint32_t units = a.units;
  const uint32_t step = gridDim.x * kP2PThreads;
  const uint32_t first = blockIdx.x * kP2PThreads + threadIdx.x;
  const uint32_t bytes = units * 16u;
  __amdgpu_buffer_rsrc_t rs[kP2PMaxRanks];
#pragma unroll
  for (int j = 0; j < kP2PMaxRanks; ++j) rs[j] = p2p_rsrc(a.buf[j < W ? j : 0], bytes);
  uint4* own = reinterpret_cast<uint4*>(a.buf[a.rank]);

  p2p_barrier(a, 0);
  uint4 out[kOneShotUnits];
#pragma unroll
  for (int i = 0; i < kOneShotUnits; ++i) {
    const uint32_t u = first + i * step;
    out[i] = make_uint4(0, 0, 0, 0);
    if (u < units) {  // the buffer descriptor range-checks the rest anyway
      uint4 v[kP2PMaxRanks];
#pragma unroll
      for (int j = 0; j < kP2PMaxRanks; ++j)
        if (j < W) v[j] = p2p_load(rs[j], u * 16u);
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < kP2PMaxRanks; ++j)
        if (j < W) acc_unit<BF16>(s, v[j]);
      out[i] = pack_unit<BF16>(s, a.scale);
    }
  }
  p2p_barrier(a, 1);  // every rank has read every buffer: overwrite in place
#pragma unroll
  for (int i = 0; i < kOneShotUnits; ++i) {
    const uint32_t u = first + i * step;
    if (u < units) own[u] = out[i];
  }
}

}  // namespace

int p2p_oneshot_max_units() { return kP2PMaxBlocks * kP2PThreads * kOneShotUnits; }

int p2p_blocks(int64_t units, int world) {
  const int64_t per_rank = (units + world - 1) / world;
  int64_t b = (per_rank + kP2PThreads * 4 - 1) / (kP2PThreads * 4);
  if (b < 1) b = 1;
  if (b > kP2PMaxBlocks) b = kP2PMaxBlocks;
  return static_cast<int>(b);
}

hipError_t p2p_allreduce(const P2PArgs& a, bool bf16, bool oneshot, hipStream_t s) {
  if (a.world < 1 || a.world > kP2PMaxRanks || a.units == 0) return hipErrorInvalidValue;
  if (oneshot) {
    if (a.units > static_cast<uint32_t>(p2p_oneshot_max_units())) return hipErrorInvalidValue;
    int blocks = static_cast<int>((a.units + kP2PThreads * kOneShotUnits - 1) / (kP2PThreads * kOneShotUnits));
    if (blocks < 1) blocks = 1;
    if (bf16)
      hipLaunchKernelGGL(p2p_allreduce_oneshot_kernel<true>, dim3(blocks), dim3(kP2PThreads), 0, s, a);
    else
      hipLaunchKernelGGL(p2p_allreduce_oneshot_kernel<false>, dim3(blocks), dim3(kP2PThreads), 0, s, a);
    return hipGetLastError();
  }
  const int blocks = p2p_blocks(a.units, a.world);
  if (bf16)
    hipLaunchKernelGGL(p2p_allreduce_kernel<true>, dim3(blocks), dim3(kP2PThreads), 0, s, a);
  else
    hipLaunchKernelGGL(p2p_allreduce_kernel<false>, dim3(blocks), dim3(kP2PThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace kdl
