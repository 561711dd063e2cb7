// CTR (XDLJob) data-plane kernels for gfx950: MFMA GEMM with fused bias+ReLU,
// embedding row gather, and sort-based sparse gradient reduction fused with
// the Adagrad update (no atomics: deterministic).
//
// gemm_bias_act:  C[M,N] = act(A[M,K] . B[N,K]^T + bias[N]) in bf16, fp32
//   accumulation on v_mfma_f32_32x32x16_bf16.  Both operands are K-contiguous
//   (A row-major activations, B = nn.Linear weight [out, in]), so every MFMA
//   fragment row (8 consecutive k of one row) is one 16-byte LDS read.
//   Tile 128x128x64, 256 threads = 4 waves as 2x2, each wave 64x64 = 2x2
//   MFMA 32x32 blocks (4 x 16 accumulator VGPRs).  Register-staged double
//   buffering: the next k-tile's global loads are issued before the MFMAs
//   of the current one and written to the other LDS buffer after them.
//   LDS rows are padded to 72 bf16 (144 B): lanes 0..31 of a 32x32 fragment
//   read rows r with bank slot 9r mod 16 -> every 16-lane ds_read_b128 group
//   hits 16 distinct slots (conflict-free) without breaking 16-B alignment.
//   The blockIdx -> tile map keeps 8 consecutive N-tiles of one M-row panel
//   on consecutive block ids (the A panel is re-read from L2 by its N-tiles).
// embed_gather:   out[b, col0 + f*D : +D] = table[idx[b*F+f], :] (bf16 / f32),
//   one wave per output row, 16-byte vector loads.
// segment_reduce / segment_adagrad: rows sorted by key; one wave per unique
//   key sums its segment (fixed order -> bitwise reproducible) and either
//   writes the sum or applies Adagrad to the owned table row in place.
// head_bce_fwd / head_bce_bwd: the tower's 1-wide logit layer fused with the
//   sigmoid-BCE loss.  A [K] -> 1 projection is a GEMV (no MFMA shape), so it
//   runs as one wave per row (dot product in registers + DPP reduction), the
//   loss and dlogit computed in the same pass; the backward writes
//   dx = dlogit * w and per-block fp32 partials of dw / db (reduced in fixed
//   order by the caller) -- no vendor GEMM for the N=1 layer.
#include "common.h"
#include "gemm_epi.h"
#include "kdl_api.h"
#include "tune.h"

namespace kdl {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;

// ds_read_b64_tr_b16: per 16-lane group a 4-row x 16-column block, lane i gets
// column i's 4 rows (device pass only: the host pass has no such builtin)
__device__ __forceinline__ v4s_t tr_read(const bf16_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(p));
#else
  return v4s_t{};
#endif
}

constexpr int BK = 64;
constexpr int LDA = BK + 8;  // padded LDS row (bf16 elements)
constexpr int kThreads = 256;

// Sum of part[r * stride] for r in [0, n), in r order; 16 loads in flight per
// round (one dependent load per partial made the last block's sum the
// kernel's critical path: 64 partials x L2 latency)
__device__ __forceinline__ float ordered_sum(const float* __restrict__ part, int n, int64_t stride) {
  float a = 0.f;
  for (int r0 = 0; r0 < n; r0 += 16) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = r0 + j < n ? part[static_cast<int64_t>(r0 + j) * stride] : 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) a += v[j];
  }
  return a;
}

// Ticketed hand-off of per-block partials to the last block to arrive (the
// in-launch split reductions below).  sc1 = 0: plain partial stores, an agent
// release fence before the ticket and an acquire in the last block -- the
// release writes back every dirty line of the XCD's L2, ~6.5 us per block with
// a freshly stored output tile (MI355X_MICROARCH.md).  sc1 = 1: partials stored
// and read with agent-scope relaxed atomics (global_store / global_load sc1:
// written through, read past L1), the ticket add after every storing wave's
// vmcnt(0) and a barrier, no fence (the hand-off table's row 1; that row was
// measured at one workgroup per CU, these kernels run two or more: the CTR GPU
// tests -- bitwise / fp32-truth checks of every reduction, repeated launches --
// pass under it, and KDL_TUNE ctr_handoff=0 restores the fenced form).
__device__ __forceinline__ void part_store(float* p, float v, int sc1) {
  if (sc1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

__device__ __forceinline__ float part_sum(const float* __restrict__ part, int n, int64_t stride, int sc1) {
  if (!sc1) return ordered_sum(part, n, stride);
  float a = 0.f;
  for (int r0 = 0; r0 < n; r0 += 16) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j)
      v[j] = r0 + j < n ? __hip_atomic_load(const_cast<float*>(part) + static_cast<int64_t>(r0 + j) * stride,
                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) a += v[j];
  }
  return a;
}

// every thread, after its partial stores: true in the block that arrived last
__device__ __forceinline__ bool handoff_last(unsigned* cnt, unsigned arrivals, int sc1, int* last) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (!sc1) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const bool l = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == arrivals - 1;
    if (l && !sc1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *last = l;
  }
  __syncthreads();
  return *last != 0;
}

// 8 bf16 <-> 8 fp32 through one 16-B register
__device__ __forceinline__ void u4_to_f8(const uint4 v, float (&o)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 f8_to_u4(const float (&o)[8]) {
  return make_uint4(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]), pack_bf16x2(o[4], o[5]), pack_bf16x2(o[6], o[7]));
}

// BM_ x BN_ tile (128x128, 128x64 or 64x64): 4 waves as 2x2, each wave
// (BM_/2) x (BN_/2) = I x J MFMA 32x32 blocks.  A 4096-row batch gives a
// 128x128 tiling only 64-256 tiles on 256 CUs (one wave per SIMD, nothing to
// hide the LDS and barrier latency); the smaller tiles trade MFMA-per-LDS-read
// for two or more resident blocks per CU (the host picks, gemm_bias_act).
//
// BT: B is [K][N] (N contiguous: the data gradient dX = dZ W reads the
// nn.Linear weight as it is, no per-step transpose).  Its tile is staged as
// [BK k][BN_ + 32] (16-B chunks along n, as loaded) and read with
// ds_read_b64_tr_b16: a 32x32x16 B fragment (8 k of one n per lane) is two
// transposed reads 4 rows apart.  Row stride 2*BN_ + 64 bytes = 64 or 192 mod 256:
// the 4 rows of a read land on 4 distinct 16-bank quarters (conflict-free).
//
// DM (data gradient through the previous layer's ReLU, BT only): C = bf16(acc)
// masked by ymask > 0 (that layer's output), and that layer's bias gradient
// db[n] = sum_m C[m, n] -- per-tile column sums into part[tile_m][N], the last
// block of each column of tiles summing them in tile order (deterministic);
// replaces a separate ReLU-backward + dbias pass over dy (relu_bwd_dbias).
template <bool RELU, int BM_, int BN_, bool BT, bool DM = false>
__global__ __launch_bounds__(kThreads, 2) void gemm_bias_act_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, const float* __restrict__ bias32,
    const bf16_t* __restrict__ bias16, bf16_t* __restrict__ C, int M, int N, int K, int tiles_n,
    const bf16_t* __restrict__ ymask = nullptr, float* __restrict__ part = nullptr, unsigned* __restrict__ cnt = nullptr,
    bf16_t* __restrict__ db = nullptr, int sc1 = 0) {
  constexpr int I = BM_ / 64, J = BN_ / 64;
  constexpr int SA = BM_ / 32, SB = BN_ / 32;  // 16-B chunks per thread per k-tile (rows x 8 chunks / 256)
  constexpr int SBT = BN_ + 32;                // BT: B image row (elements)
  constexpr int BOFF = BM_ * LDA;              // B image offset in a buffer
  constexpr int BSZ = BT ? BK * SBT : BN_ * LDA;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2][BOFF + BSZ];  // [buf][A rows | B image]
  // block -> (tile_m, tile_n): groups of 8 N-tiles share one A panel
  const int bid = blockIdx.x;
  const int group = 8;
  const int tiles_m = (M + BM_ - 1) / BM_;
  const int per_group = group * tiles_m;
  const int g = bid / per_group;
  const int first_n = g * group;
  const int gsize = (tiles_n - first_n) < group ? (tiles_n - first_n) : group;
  const int in_g = bid % per_group;
  const int tile_m = in_g / gsize;
  const int tile_n = first_n + in_g % gsize;
  const int m0 = tile_m * BM_, n0 = tile_n * BN_;

  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int wm = (wave >> 1) * (BM_ / 2), wn = (wave & 1) * (BN_ / 2);

  uint4 ra[SA], rb[SB];
  const int nk = (K + BK - 1) / BK;

  // Loads are unconditional (no load behind an exec branch, which makes hipcc
  // drain vmcnt before the next tile's MFMAs): rows past M / N re-read row 0
  // (their outputs are never stored), and K-tail chunks re-read chunk 0 and are
  // zeroed when staged (they would otherwise feed valid outputs).
  uint32_t koka = 0, kokb = 0;
  auto gload = [&](int kt) {
    const int k0 = kt * BK;
    koka = kokb = 0;
#pragma unroll
    for (int i = 0; i < SA; ++i) {
      const int cidx = t + i * kThreads, row = cidx >> 3, kk = k0 + (cidx & 7) * 8;
      const bool kin = kk < K;
      koka |= kin ? (1u << i) : 0u;
      const int am = m0 + row < M ? m0 + row : 0;
      ra[i] = *reinterpret_cast<const uint4*>(A + static_cast<int64_t>(am) * K + (kin ? kk : 0));
    }
#pragma unroll
    for (int i = 0; i < SB; ++i) {
      const int cidx = t + i * kThreads;
      if constexpr (BT) {
        // 64 k rows x BN_/8 chunks of 8 n; columns past N re-read column 0 (never stored)
        const int kk = k0 + cidx / (BN_ / 8), n = n0 + (cidx % (BN_ / 8)) * 8;
        const bool kin = kk < K;
        kokb |= kin ? (1u << i) : 0u;
        rb[i] = *reinterpret_cast<const uint4*>(B + static_cast<int64_t>(kin ? kk : 0) * N + (n < N ? n : 0));
      } else {
        const int row = cidx >> 3, kk = k0 + (cidx & 7) * 8;
        const bool kin = kk < K;
        kokb |= kin ? (1u << i) : 0u;
        const int bn = n0 + row < N ? n0 + row : 0;
        rb[i] = *reinterpret_cast<const uint4*>(B + static_cast<int64_t>(bn) * K + (kin ? kk : 0));
      }
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < SA; ++i) {
      const int cidx = t + i * kThreads;
      *reinterpret_cast<uint4*>(&lds[buf][(cidx >> 3) * LDA + (cidx & 7) * 8]) =
          (koka >> i) & 1u ? ra[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < SB; ++i) {
      const int cidx = t + i * kThreads;
      const int off = BT ? (cidx / (BN_ / 8)) * SBT + (cidx % (BN_ / 8)) * 8 : (cidx >> 3) * LDA + (cidx & 7) * 8;
      *reinterpret_cast<uint4*>(&lds[buf][BOFF + off]) = (kokb >> i) & 1u ? rb[i] : make_uint4(0, 0, 0, 0);
    }
  };

  f32x16_t acc[I][J];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  gload(0);
  swrite(0);
  __syncthreads();
  const int fr = lane & 31, fh = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8_t af[I], bfr[J];
#pragma unroll
      for (int i = 0; i < I; ++i) {
        const uint4 v = *reinterpret_cast<const uint4*>(&lds[cur][(wm + i * 32 + fr) * LDA + s * 16 + fh * 8]);
        af[i] = __builtin_bit_cast(bf16x8_t, v);
      }
#pragma unroll
      for (int j = 0; j < J; ++j) {
        if constexpr (BT) {
          // lane 4q+p of 16-lane group g: row k = s*16 + fh*8 + q (+4), columns 16(g&1) + 4p..+3
          const bf16_t* b = &lds[cur][BOFF + (s * 16 + fh * 8 + ((lane & 15) >> 2)) * SBT + wn + j * 32 +
                                      ((lane >> 4) & 1) * 16 + (lane & 3) * 4];
          const uint2 lo = __builtin_bit_cast(uint2, tr_read(b)), hi = __builtin_bit_cast(uint2, tr_read(b + 4 * SBT));
          bfr[j] = __builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
        } else {
          const uint4 v = *reinterpret_cast<const uint4*>(&lds[cur][BOFF + (wn + j * 32 + fr) * LDA + s * 16 + fh * 8]);
          bfr[j] = __builtin_bit_cast(bf16x8_t, v);
        }
      }
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    // buf cur^1 was last read in iteration kt-1, which ended with a barrier
    if (kt + 1 < nk) swrite(cur ^ 1);
    __syncthreads();
  }
  // epilogue: C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  // N % 8 == 0 (every DM / BT launch): the tile goes through LDS (the K-loop
  // buffers are free: the last iteration ended in a barrier) and leaves as
  // 16-B row chunks -- the lanes of a 32x32 block hold one column each, so a
  // direct store is a 2-byte store per element (and DM's mask a 2-byte load).
  const bool vec = (N & 7) == 0;
  if (vec) {
    constexpr int LDC = BN_ + 8;
    static_assert(BM_ * LDC <= 2 * (BOFF + BSZ), "C tile fits the K-loop buffers");
    bf16_t* Cs = &lds[0][0];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int cl = wn + j * 32 + fr;
      float bv = 0.f;
      if constexpr (!DM) {
        if (n0 + cl < N) bv = bias32 ? bias32[n0 + cl] : bias16 ? bf16_to_f32(bias16[n0 + cl]) : 0.f;
      }
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = acc[i][j][r] + bv;  // one rounding, after bias and ReLU (as the direct path)
          if (RELU) v = v > 0.f ? v : 0.f;
          Cs[(wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh) * LDC + cl] = f32_to_bf16(v);
        }
    }
    __syncthreads();
    constexpr int CPR = BN_ / 8, RPP = kThreads / CPR, NP = BM_ / RPP;
    const int ec = t % CPR, er0 = t / CPR;
    const int col = n0 + ec * 8;
    uint4 yv[NP];
    if constexpr (DM) {
#pragma unroll
      for (int ps = 0; ps < NP; ++ps) {
        const int row = m0 + ps * RPP + er0;
        yv[ps] = (row < M && col < N) ? *reinterpret_cast<const uint4*>(ymask + static_cast<int64_t>(row) * N + col)
                                      : make_uint4(0, 0, 0, 0);
      }
    }
    float cs8[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) cs8[k] = 0.f;
#pragma unroll
    for (int ps = 0; ps < NP; ++ps) {
      const int rl = ps * RPP + er0, row = m0 + rl;
      if (row < M && col < N) {
        uint4 v = *reinterpret_cast<const uint4*>(&Cs[rl * LDC + ec * 8]);
        if constexpr (DM) {
          float x[8], yy[8];
          u4_to_f8(v, x);
          u4_to_f8(yv[ps], yy);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            x[k] = yy[k] > 0.f ? x[k] : 0.f;
            cs8[k] += x[k];
          }
          v = f8_to_u4(x);
        }
        *reinterpret_cast<uint4*>(C + static_cast<int64_t>(row) * N + col) = v;
      }
    }
    if constexpr (DM) {
      // column sums: the RPP row groups folded in order through LDS (after
      // every thread's tile reads), then the ticketed cross-tile reduction
      __shared__ int last;
      float* red = reinterpret_cast<float*>(&lds[0][0]);  // [RPP][BN_]
      static_assert(RPP * BN_ * 4 <= 2 * (BOFF + BSZ) * 2, "column-sum scratch fits");
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 8; ++k) red[er0 * BN_ + ec * 8 + k] = cs8[k];
      __syncthreads();
      if (t < BN_ && n0 + t < N) {
        float a = 0.f;
        for (int rr = 0; rr < RPP; ++rr) a += red[rr * BN_ + t];
        part_store(part + static_cast<int64_t>(tile_m) * N + n0 + t, a, sc1);
      }
      if (!handoff_last(cnt + tile_n, static_cast<unsigned>(tiles_m), sc1, &last)) return;
      if (t < BN_ && n0 + t < N) db[n0 + t] = f32_to_bf16(part_sum(part + n0 + t, tiles_m, N, sc1));  // tile order
      if (t == 0) __hip_atomic_store(cnt + tile_n, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if constexpr (!DM) {  // ragged N (the forward path only): element stores
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int col = n0 + wn + j * 32 + fr;
      float bv = 0.f;
      if (col < N) bv = bias32 ? bias32[col] : bias16 ? bf16_to_f32(bias16[col]) : 0.f;
#pragma unroll
      for (int i = 0; i < I; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          if (row < M && col < N) {
            float v = acc[i][j][r] + bv;
            if (RELU) v = v > 0.f ? v : 0.f;
            C[static_cast<int64_t>(row) * N + col] = f32_to_bf16(v);
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------- ReLU backward + dbias
// dz = dy * (y > 0) (bf16 out), dbias[n] += sum_m dz[m, n]; 16 B along N per lane.
// 8 bf16 <-> 8 fp32 through one 16-B register (the loads of a round are raw
// uint4 so every one is issued before the first conversion)

// Row-block partial column sums go to part[blockIdx.x][N]; the last block of a
// column block to arrive (agent-scope release + ticket; acquire in the
// reducer: the in-launch split reduction of cdna_hip_programming.md) sums them
// in row-block order -- deterministic, no zero-fill, no separate conversion --
// and writes db as bf16 (db16) or fp32 (db32), then re-arms its ticket.
__global__ __launch_bounds__(256) void relu_bwd_dbias_kernel(const bf16_t* __restrict__ dy,
                                                             const bf16_t* __restrict__ y,
                                                             bf16_t* __restrict__ dz, float* __restrict__ part,
                                                             unsigned* __restrict__ cnt, bf16_t* __restrict__ db16,
                                                             float* __restrict__ db32, int M, int N,
                                                             int rows_per_block, int sc1) {
  __shared__ float red[8][32 * 8];
  __shared__ int last;
  const int cl = threadIdx.x & 31;        // column group within the block
  const int cg = blockIdx.y * 32 + cl;    // 8-column group
  const int r0 = threadIdx.x >> 5;        // 8 row lanes
  float s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = 0.f;
  if (cg * 8 < N) {
    const int mb = blockIdx.x * rows_per_block;
    const int me = (mb + rows_per_block) < M ? (mb + rows_per_block) : M;
    // 8 rows per thread per round, every load of the round issued before the
    // first use (one dependent load chain per thread was latency-bound: 25 us
    // for a 4096 x 1024 layer)
    for (int m0 = mb + r0; m0 < me; m0 += 64) {
      uint4 gv[8], yv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = m0 + 8 * j;
        const int64_t o = static_cast<int64_t>(m < me ? m : m0) * N + cg * 8;
        gv[j] = *reinterpret_cast<const uint4*>(dy + o);
        if (y != nullptr) yv[j] = *reinterpret_cast<const uint4*>(y + o);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = m0 + 8 * j;
        if (m >= me) break;
        float g[8];
        u4_to_f8(gv[j], g);
        if (y != nullptr) {
          float yy[8];
          u4_to_f8(yv[j], yy);
#pragma unroll
          for (int i = 0; i < 8; ++i) g[i] = yy[i] > 0.f ? g[i] : 0.f;
          *reinterpret_cast<uint4*>(dz + static_cast<int64_t>(m) * N + cg * 8) = f8_to_u4(g);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) s[i] += g[i];
      }
    }
  }
  // the 8 row lanes folded in LDS, in order: this block's 256 column sums
#pragma unroll
  for (int i = 0; i < 8; ++i) red[r0][cl * 8 + i] = s[i];
  __syncthreads();
  const int c = threadIdx.x;
  const int col = blockIdx.y * 256 + c;
  if (col < N) {
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) a += red[r][c];
    part_store(part + static_cast<int64_t>(blockIdx.x) * N + col, a, sc1);
  }
  if (!handoff_last(cnt + blockIdx.y, gridDim.x, sc1, &last)) return;
  if (col < N) {
    const float a = part_sum(part + col, static_cast<int>(gridDim.x), N, sc1);
    if (db16) db16[col] = f32_to_bf16(a);
    else db32[col] = a;
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt + blockIdx.y, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- embeddings
constexpr int kGatherRows = 1;
template <typename T>
__global__ __launch_bounds__(256) void embed_gather_kernel(const T* __restrict__ table, const int64_t* __restrict__ idx,
                                                           int n, int F, int D, T* __restrict__ out, int ld_out,
                                                           int col0, int lg) {
  // a group of 2^lg lanes per row (16 B each; one wave per 128-256 B row left
  // 48-56 of 64 lanes idle: 20 -> 11 us for the fp32 pull at batch 4096).
  // kGatherRows > 1 walks that many rows per group with every load issued
  // before the first store: measured slower at 4 (30 us), so 1.
  constexpr int VEC = 16 / sizeof(T);
  const int g = (blockIdx.x * 256 + threadIdx.x) >> lg;
  const int gl = threadIdx.x & ((1 << lg) - 1);
  const int r0 = g * kGatherRows;
  if (r0 >= n) return;
  for (int c = gl * VEC; c < D; c += VEC << lg) {
    const bool full = c + VEC <= D;
    uint4 v[kGatherRows];
    const T* src[kGatherRows];
#pragma unroll
    for (int i = 0; i < kGatherRows; ++i) {
      const int r = r0 + i < n ? r0 + i : r0;
      src[i] = table + idx[r] * static_cast<int64_t>(D);
      if (full) v[i] = *reinterpret_cast<const uint4*>(src[i] + c);
    }
#pragma unroll
    for (int i = 0; i < kGatherRows; ++i) {
      const int r = r0 + i;
      if (r >= n) break;
      const int b = r / F, f = r - b * F;
      T* dst = out + static_cast<int64_t>(b) * ld_out + col0 + f * D;
      if (full) {
        *reinterpret_cast<uint4*>(dst + c) = v[i];
      } else {
        for (int k = c; k < D; ++k) dst[k] = src[i][k];
      }
    }
  }
}

// Fused pull for one owner: out[b, col0 + f*D : +D] = bf16(table[uniq[inv[r]], :]),
// r = b*F + f -- the fp32 table rows go straight into the bf16 tower input
// (no [n, D] fp32 gather and no cast pass in between).  A group of 2^lg lanes
// per row, 8 elements (two 16-B loads, one 16-B store) per lane; D % 8 == 0 and
// 16-B aligned rows (host-checked).  T = bf16: the rows are already bf16 (the
// fixed exchange's received rows, rounded once by their owner): one 16-B copy.
template <typename T>
// tail > 0 (the CTR tower input): the last field's lane group of each row also
// writes the row's next ``tail`` columns -- the nd dense features (fp32 ->
// bf16) then zeros up to the padded width -- so the input is built in one
// launch (no torch fill of the pad, no cast-copy of the dense block).
__global__ __launch_bounds__(256) void embed_gather_cast_kernel(const T* __restrict__ table,
                                                                const int64_t* __restrict__ uniq,
                                                                const int64_t* __restrict__ inv, int n, int F, int D,
                                                                bf16_t* __restrict__ out, int ld_out, int col0,
                                                                int lg, const float* __restrict__ dense = nullptr,
                                                                int nd = 0, int tail = 0) {
  const int r = (blockIdx.x * 256 + threadIdx.x) >> lg;
  const int gl = threadIdx.x & ((1 << lg) - 1);
  if (r >= n) return;
  const T* src = table + uniq[inv[r]] * static_cast<int64_t>(D);
  const int b = r / F, f = r - b * F;
  bf16_t* dst = out + static_cast<int64_t>(b) * ld_out + col0 + static_cast<int64_t>(f) * D;
  if (tail > 0 && f == F - 1) {
    bf16_t* tdst = dst + D;
    const float* dsrc = dense + static_cast<int64_t>(b) * nd;
    for (int c = gl * 8; c < tail; c += 8 << lg) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = c + e < nd ? dsrc[c + e] : 0.f;
      *reinterpret_cast<uint4*>(tdst + c) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                                       pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
    }
  }
  for (int c = gl * 8; c < D; c += 8 << lg) {
    if constexpr (sizeof(T) == 2) {
      *reinterpret_cast<uint4*>(dst + c) = *reinterpret_cast<const uint4*>(src + c);
    } else {
      const float4 v0 = *reinterpret_cast<const float4*>(src + c);
      const float4 v1 = *reinterpret_cast<const float4*>(src + c + 4);
      *reinterpret_cast<uint4*>(dst + c) = make_uint4(pack_bf16x2(v0.x, v0.y), pack_bf16x2(v0.z, v0.w),
                                                      pack_bf16x2(v1.x, v1.y), pack_bf16x2(v1.z, v1.w));
    }
  }
}

// 4 consecutive elements -> fp32: one 8-B (bf16) / 16-B (fp32) load when V4
// (row base and column aligned, host-checked), else element by element up to n
template <typename T, bool V4>
__device__ __forceinline__ void ld4(const T* p, int n, float (&o)[4]) {
  if constexpr (V4) {
    if constexpr (sizeof(T) == 2) {
      const uint2 v = *reinterpret_cast<const uint2*>(p);
      o[0] = __uint_as_float(v.x << 16);
      o[1] = __uint_as_float(v.x & 0xffff0000u);
      o[2] = __uint_as_float(v.y << 16);
      o[3] = __uint_as_float(v.y & 0xffff0000u);
    } else {
      const float4 v = *reinterpret_cast<const float4*>(p);
      o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = k < n ? Vec1<T>::ld(p + k) : 0.f;
  }
}

// Row j = b*F + f of a [B, ld] activation-gradient matrix lives at
// rows + b*ld + col0 + f*D (the layout embed_gather wrote).  Rows order[j]
// are summed per segment [seg[u], seg[u+1]), in j order, by a group of G =
// 2^lg lanes (G*4 >= D when D <= 256: a wave per segment left 48 of 64 lanes
// idle at D = 64), kSegFly rows' loads in flight per step on long segments.
// (Four segments per group in lock step measured slower: 63 vs 33 us at batch 4096.)
// j / F as umulhi(j, mF), mF = ceil(2^32 / F): exact while j * F < 2^32 (host
// check; mF = 0 selects the 64-bit division) -- no 64-bit division sequence per row.
// ``ucount`` (optional): the live segment count on the device (U is then the
// capacity the grid was sized for) -- no host round trip for data-dependent U.
template <typename T, bool V4>
__device__ __forceinline__ void seg_row(const T* rows, int64_t jj, uint32_t F, uint32_t mF, int ld, int col0, int D,
                                        int c, int n, float (&v)[4]) {
  int64_t bi, f;
  if (mF != 0) {  // grid-uniform: the umulhi form is exact for this launch
    const uint32_t j = static_cast<uint32_t>(jj);
    const uint32_t q = __umulhi(j, mF);
    bi = q;
    f = j - q * F;
  } else {  // j * F may reach 2^32: 64-bit division
    bi = jj / F;
    f = jj - bi * F;
  }
  ld4<T, V4>(rows + bi * ld + col0 + f * D + c, n, v);
}

constexpr int kSegFly = 8;  // rows in flight per lane group on a long segment (16: 39.9 vs 34.5 us)

// Sum of the rows order[s0 .. s1) of one segment, columns [c, c + n), in j
// order.  Hot ids: a long segment is a serial chain (index load -> row load ->
// add), and the longest one sets the launch's time -- keep kSegFly rows' loads
// in flight, then add them in j order (the same sums, bit for bit).
template <typename T, bool V4>
__device__ __forceinline__ void seg_sum(const T* rows, const int64_t* order, int64_t s0, int64_t s1, uint32_t F,
                                        uint32_t mF, int ld, int col0, int D, int c, int n, float (&a)[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) a[k] = 0.f;
  int64_t j = s0;
  for (; j + kSegFly <= s1; j += kSegFly) {
    int64_t jj[kSegFly];
    float v[kSegFly][4];
#pragma unroll
    for (int r = 0; r < kSegFly; ++r) jj[r] = order[j + r];
#pragma unroll
    for (int r = 0; r < kSegFly; ++r) seg_row<T, V4>(rows, jj[r], F, mF, ld, col0, D, c, n, v[r]);
#pragma unroll
    for (int r = 0; r < kSegFly; ++r)
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] += v[r][k];
  }
  for (; j + 1 < s1; j += 2) {
    const int64_t j0 = order[j], j1 = order[j + 1];
    float v0[4], v1[4];
    seg_row<T, V4>(rows, j0, F, mF, ld, col0, D, c, n, v0);
    seg_row<T, V4>(rows, j1, F, mF, ld, col0, D, c, n, v1);
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = (a[k] + v0[k]) + v1[k];
  }
  if (j < s1) {
    float v0[4];
    seg_row<T, V4>(rows, order[j], F, mF, ld, col0, D, c, n, v0);
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] += v0[k];
  }
}

template <typename T, bool V4>
__global__ __launch_bounds__(256) void segment_reduce_kernel(const T* __restrict__ rows, int F, uint32_t mF, int ld,
                                                             int col0, const int64_t* __restrict__ order,
                                                             const int64_t* __restrict__ seg, int U, int D, int lg,
                                                             float* __restrict__ out, const int* __restrict__ ucount,
                                                             const int64_t* __restrict__ out_row, int64_t out_lim) {
  const int u = (blockIdx.x * 256 + threadIdx.x) >> lg;
  const int gl = threadIdx.x & ((1 << lg) - 1);
  if (u >= (ucount ? *ucount : U)) return;
  // out_row: segment u's sum goes to row out_row[u] of the exchange send buffer
  // (rows >= out_lim: the id did not fit the capacity -- nothing to send)
  const int64_t orow = out_row ? out_row[u] : u;
  if (orow >= out_lim) return;
  const int64_t s0 = seg[u], s1 = seg[u + 1];
  for (int c = gl * 4; c < D; c += 4 << lg) {
    const int n = D - c < 4 ? D - c : 4;
    float a[4];
    seg_sum<T, V4>(rows, order, s0, s1, F, mF, ld, col0, D, c, n, a);
    float* o = out + orow * D + c;
    if (V4) {
      *reinterpret_cast<float4*>(o) = make_float4(a[0], a[1], a[2], a[3]);
    } else {
      for (int k = 0; k < n; ++k) o[k] = a[k];
    }
  }
}

// One owner, sync-free push (world 1): segment u's summed gradient is applied
// straight to table row rows_local[u] -- segment_reduce_kernel followed by a
// one-row-per-segment segment_adagrad_kernel, without the [U, D] fp32 rows
// between them (written once, read once) or the second launch.  Same
// arithmetic in the same order: bitwise those two launches.
template <typename T, bool V4>
__global__ __launch_bounds__(256) void segment_reduce_adagrad_kernel(
    const T* __restrict__ rows, int F, uint32_t mF, int ld, int col0, const int64_t* __restrict__ order,
    const int64_t* __restrict__ seg, int U, int D, int lg, const int* __restrict__ ucount,
    const int64_t* __restrict__ rows_local, int64_t nrows, float* __restrict__ table, float* __restrict__ accum,
    float lr, float eps, float scale) {
  const int u = (blockIdx.x * 256 + threadIdx.x) >> lg;
  const int gl = threadIdx.x & ((1 << lg) - 1);
  if (u >= (ucount ? *ucount : U)) return;
  const int64_t row = rows_local[u];
  if (row < 0 || row >= nrows) return;
  const int64_t s0 = seg[u], s1 = seg[u + 1];
  float* w = table + row * static_cast<int64_t>(D);
  float* ac = accum + row * static_cast<int64_t>(D);
  for (int c = gl * 4; c < D; c += 4 << lg) {
    const int n = D - c < 4 ? D - c : 4;
    float wv[4], av[4], a[4];
    ld4<float, V4>(w + c, n, wv);  // issued before the gradient rows
    ld4<float, V4>(ac + c, n, av);
    seg_sum<T, V4>(rows, order, s0, s1, F, mF, ld, col0, D, c, n, a);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = (0.f + a[k]) * scale;  // segment_adagrad's one-row sum: 0 + g
      av[k] += gk * gk;
      wv[k] -= lr * gk / (sqrtf(av[k]) + eps);
    }
    if (V4) {
      *reinterpret_cast<float4*>(ac + c) = make_float4(av[0], av[1], av[2], av[3]);
      *reinterpret_cast<float4*>(w + c) = make_float4(wv[0], wv[1], wv[2], wv[3]);
    } else {
      for (int k = 0; k < n; ++k) {
        ac[c + k] = av[k];
        w[c + k] = wv[k];
      }
    }
  }
}

// Owner side: sum the received gradient rows of each unique local row and
// apply Adagrad in place: acc += g^2; w -= lr * g / (sqrt(acc) + eps).  Same
// lane groups as segment_reduce_kernel; V4 when D % 4 == 0 (all rows 16-B aligned).
template <bool V4>
__global__ __launch_bounds__(256) void segment_adagrad_kernel(const float* __restrict__ grads,
                                                              const int64_t* __restrict__ order,
                                                              const int64_t* __restrict__ seg,
                                                              const int64_t* __restrict__ rows_local, int U, int D,
                                                              int lg, float* __restrict__ table,
                                                              float* __restrict__ accum, float lr, float eps,
                                                              float scale, const int* __restrict__ ucount,
                                                              int64_t nrows) {
  const int u = (blockIdx.x * 256 + threadIdx.x) >> lg;
  const int gl = threadIdx.x & ((1 << lg) - 1);
  if (u >= (ucount ? *ucount : U)) return;
  const int64_t s0 = seg[u], s1 = seg[u + 1];
  const int64_t row = rows_local[u];
  // rows outside the shard are exchange padding (distinct negative sentinels,
  // models/ctr.py _push_fixed): nothing to update
  if (row < 0 || row >= nrows) return;
  float* w = table + row * static_cast<int64_t>(D);
  float* a = accum + row * static_cast<int64_t>(D);
  for (int c = gl * 4; c < D; c += 4 << lg) {
    const int n = D - c < 4 ? D - c : 4;
    float wv[4], av[4], g[4] = {0.f, 0.f, 0.f, 0.f};
    ld4<float, V4>(w + c, n, wv);  // issued before the gradient rows
    ld4<float, V4>(a + c, n, av);
    int64_t j = s0;
    for (; j + 1 < s1; j += 2) {
      const int64_t j0 = order[j], j1 = order[j + 1];
      float v0[4], v1[4];
      ld4<float, V4>(grads + j0 * static_cast<int64_t>(D) + c, n, v0);
      ld4<float, V4>(grads + j1 * static_cast<int64_t>(D) + c, n, v1);
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] = (g[k] + v0[k]) + v1[k];
    }
    if (j < s1) {
      float v0[4];
      ld4<float, V4>(grads + order[j] * static_cast<int64_t>(D) + c, n, v0);
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] += v0[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = g[k] * scale;
      av[k] += gk * gk;
      wv[k] -= lr * gk / (sqrtf(av[k]) + eps);
    }
    if (V4) {
      *reinterpret_cast<float4*>(a + c) = make_float4(av[0], av[1], av[2], av[3]);
      *reinterpret_cast<float4*>(w + c) = make_float4(wv[0], wv[1], wv[2], wv[3]);
    } else {
      for (int k = 0; k < n; ++k) {
        a[c + k] = av[k];
        w[c + k] = wv[k];
      }
    }
  }
}

// Owner side of a fixed exchange without a de-duplication pass.  The received
// gradient blocks are W senders x cap slots (slot s = w * cap + k, local row
// local[s], padding < 0), and a sender routes each of its UNIQUE ids once, so a
// row repeats only across senders.  Each slot stamps slotmap[row * W + w] =
// (call << 32) | s -- one plain store, no atomics, nothing to clear: an entry
// is live only while its stamp equals the current call.
__global__ __launch_bounds__(256) void a2a_stamp_kernel(const int64_t* __restrict__ local, int S, int cap, int W,
                                                        int64_t nrows, int64_t* __restrict__ slotmap, int64_t call) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= S) return;
  const int64_t r = local[s];
  if (r < 0 || r >= nrows) return;
  slotmap[r * W + s / cap] = (call << 32) | static_cast<int64_t>(s);
}

// One lane group per slot; the row's leader is its lowest stamping sender.  It
// sums the row's live senders' gradient rows in sender (= slot) order --
// bitwise segment_adagrad's position order -- and applies Adagrad in place.
template <bool V4>
__global__ __launch_bounds__(256) void a2a_adagrad_kernel(const float* __restrict__ grads,
                                                          const int64_t* __restrict__ local, int S, int cap, int D,
                                                          int lg, int W, int64_t nrows,
                                                          const int64_t* __restrict__ slotmap, int64_t call,
                                                          float* __restrict__ table, float* __restrict__ accum,
                                                          float lr, float eps, float scale) {
  const int s = (blockIdx.x * 256 + threadIdx.x) >> lg;
  const int gl = threadIdx.x & ((1 << lg) - 1);
  if (s >= S) return;
  const int64_t row = local[s];
  if (row < 0 || row >= nrows) return;
  const int w0 = s / cap;
  const int64_t* sm = slotmap + row * W;
  for (int w = 0; w < w0; ++w)
    if ((sm[w] >> 32) == call) return;  // a lower sender holds this row: it updates it
  float* wt = table + row * static_cast<int64_t>(D);
  float* a = accum + row * static_cast<int64_t>(D);
  for (int c = gl * 4; c < D; c += 4 << lg) {
    const int n = D - c < 4 ? D - c : 4;
    float wv[4], av[4], g[4] = {0.f, 0.f, 0.f, 0.f};
    ld4<float, V4>(wt + c, n, wv);
    ld4<float, V4>(a + c, n, av);
    for (int w = w0; w < W; ++w) {
      const int64_t e = w == w0 ? ((call << 32) | s) : sm[w];
      if ((e >> 32) != call) continue;
      float v[4];
      ld4<float, V4>(grads + (e & 0xffffffffll) * D + c, n, v);
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] += v[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = g[k] * scale;
      av[k] += gk * gk;
      wv[k] -= lr * gk / (sqrtf(av[k]) + eps);
    }
    if (V4) {
      *reinterpret_cast<float4*>(a + c) = make_float4(av[0], av[1], av[2], av[3]);
      *reinterpret_cast<float4*>(wt + c) = make_float4(wv[0], wv[1], wv[2], wv[3]);
    } else {
      for (int k = 0; k < n; ++k) {
        a[c + k] = av[k];
        wt[c + k] = wv[k];
      }
    }
  }
}

// ---------------------------------------------------------------- logit head + BCE
// 8 rows per wave (32 per block): logit = x[m,:] . w + b; loss_m = softplus(l) - y l;
// dlogit_m = sigmoid(l) - y.  Each block writes the sum of its rows' losses
// (row order).  The last block to arrive (agent release / ticket / acquire)
// sums the block partials in order into the mean loss[0] and re-arms its
// ticket.  One row per wave made 1024 blocks, i.e. 1024 ticket atomics on one
// address: 22 us for a 4096 x 256 head.  b: the bias, bf16 (b16) or fp32.
constexpr int kHeadRowsPerWave = 8;
__global__ __launch_bounds__(256) void head_bce_fwd_kernel(const bf16_t* __restrict__ x,
                                                           const bf16_t* __restrict__ w, const float* __restrict__ b,
                                                           const bf16_t* __restrict__ b16,
                                                           const float* __restrict__ y, int M, int K,
                                                           float* __restrict__ logit, float* __restrict__ dlogit,
                                                           float* __restrict__ loss_part, unsigned* __restrict__ cnt,
                                                           float* __restrict__ loss, int sc1) {
  constexpr int R = kHeadRowsPerWave;
  __shared__ float wave_loss[4];
  __shared__ int last;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int mb = (blockIdx.x * 4 + wv) * R;
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.f;
  for (int k = lane * 8; k < K; k += 512) {
    float wv8[8];
    Vec<bf16_t, 8>::load(w + k, wv8);
    uint4 xr[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {  // every row's load issued before the first use (rows past M re-read row 0)
      const int m = mb + r < M ? mb + r : 0;
      xr[r] = *reinterpret_cast<const uint4*>(x + static_cast<int64_t>(m) * K + k);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float xv[8];
      u4_to_f8(xr[r], xv);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[r] += xv[i] * wv8[i];
    }
  }
  const float bias = b16 ? __uint_as_float(static_cast<uint32_t>(b16[0]) << 16) : b[0];
  float l = 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float a = acc[r];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, 64);
    const int m = mb + r;
    if (m < M) {
      const float z = a + bias;
      const float t = y[m];
      // softplus(z) - t z, stable for both signs
      l += fmaxf(z, 0.f) - t * z + log1pf(__expf(-fabsf(z)));
      if (lane == r) {
        logit[m] = z;
        dlogit[m] = 1.f / (1.f + __expf(-z)) - t;
      }
    }
  }
  if (lane == 0) wave_loss[wv] = l;
  __syncthreads();
  // the hand-off of the block sums (handoff_last: with sc1 no release fence, which
  // wrote back the L2 lines the logit / dlogit stores had just dirtied)
  if (threadIdx.x == 0)
    part_store(loss_part + blockIdx.x, (wave_loss[0] + wave_loss[1]) + (wave_loss[2] + wave_loss[3]), sc1);
  if (!handoff_last(cnt, gridDim.x, sc1, &last)) return;
  // fixed order: 256 strided partial sums, then the 4 waves' in LDS order
  float a = 0.f;
  for (int i = threadIdx.x; i < static_cast<int>(gridDim.x); i += 256)
    a += sc1 ? __hip_atomic_load(loss_part + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : loss_part[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, 64);
  if (lane == 0) wave_loss[wv] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    loss[0] = ((wave_loss[0] + wave_loss[1]) + (wave_loss[2] + wave_loss[3])) / static_cast<float>(M);
    __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// block = 256 threads = 8 row lanes x 32 column groups of 8 (K <= 256 per
// pass, looped for wider K); rows [blockIdx.x*rpb, +rpb).  dx = g*w (bf16),
// dw partial[block, k] = sum g*x, db partial[block] = sum g; g = dlogit*scale.
// MASK: x is the previous layer's ReLU output -- dx = g*w*[x > 0] (the gradient
// into that layer's pre-activation) and that layer's bias gradient
// dbx[k] = sum_m bf16(dx[m, k]) from per-block partials dbx_part (replaces a
// relu_bwd_dbias pass over dx).
template <bool MASK>
__global__ __launch_bounds__(256) void head_bce_bwd_kernel(const bf16_t* __restrict__ x,
                                                           const bf16_t* __restrict__ w,
                                                           const float* __restrict__ dlogit, float scale,
                                                           const float* __restrict__ gscale, int M,
                                                           int K, int rpb, bf16_t* __restrict__ dx,
                                                           float* __restrict__ dw_part, float* __restrict__ db_part,
                                                           unsigned* __restrict__ cnt, bf16_t* __restrict__ dw,
                                                           bf16_t* __restrict__ db, float* __restrict__ dbx_part,
                                                           bf16_t* __restrict__ dbx, int sc1) {
  // per-row-lane partials, column c at hidx(c): a lane's 8 columns leave as two
  // 16-B writes into contiguous runs (the half-columns 4..7 a 32-bank offset away),
  // where 8 scalar writes at a 32-B lane stride conflicted 8 ways; [288] = g sum
  constexpr int kRS = 292;
  __shared__ __attribute__((aligned(16))) float red[8][kRS];
  __shared__ __attribute__((aligned(16))) float redx[MASK ? 8 : 1][MASK ? kRS : 4];
  __shared__ int last;
  auto hidx = [](int c) { return ((c & 7) >> 2) * 160 + (c >> 3) * 4 + (c & 3); };
  if (gscale != nullptr) scale *= gscale[0];  // upstream gradient of the loss, read on the device
  const int rl = threadIdx.x >> 5, cg = threadIdx.x & 31;
  const int m0 = blockIdx.x * rpb;
  const int m1 = (m0 + rpb) < M ? (m0 + rpb) : M;
  float gsum = 0.f;
  for (int kb = 0; kb < K; kb += 256) {
    const int k = kb + cg * 8;
    const bool on = k < K;
    float wv8[8], s[8], sx[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { s[i] = 0.f; sx[i] = 0.f; }
    if (on) Vec<bf16_t, 8>::load(w + k, wv8);
    // RB of the thread's rows (stride 8) per batch, every row's dlogit and x loads
    // issued before the first use: one memory latency per batch, not one per row
    // (a 64-row block is one batch; the row-serial loop took 16 us for 4096 x 256)
    constexpr int RB = 8;
    for (int mb = m0 + rl; mb < m1; mb += 8 * RB) {
      float gr[RB];
      uint4 xr[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int m = mb + 8 * r;
        const bool ok = m < m1;
        gr[r] = ok ? dlogit[m] : 0.f;
        xr[r] = (ok && on) ? *reinterpret_cast<const uint4*>(x + static_cast<int64_t>(m) * K + k) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int m = mb + 8 * r;
        if (m >= m1) break;  // (rows ascend: the rest of the batch is past the block)
        const float g = gr[r] * scale;
        if (kb == 0 && cg == 0) gsum += g;
        if (!on) continue;
        float xv[8], d[8];
        u4_to_f8(xr[r], xv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          s[i] += g * xv[i];
          d[i] = g * wv8[i];
          if constexpr (MASK) {
            d[i] = xv[i] > 0.f ? bf16_to_f32(f32_to_bf16(d[i])) : 0.f;  // the stored (rounded) value
            sx[i] += d[i];
          }
        }
        Vec<bf16_t, 8>::store(dx + static_cast<int64_t>(m) * K + k, d);
      }
    }
    *reinterpret_cast<float4*>(&red[rl][cg * 4]) = make_float4(s[0], s[1], s[2], s[3]);
    *reinterpret_cast<float4*>(&red[rl][160 + cg * 4]) = make_float4(s[4], s[5], s[6], s[7]);
    if constexpr (MASK) {
      *reinterpret_cast<float4*>(&redx[rl][cg * 4]) = make_float4(sx[0], sx[1], sx[2], sx[3]);
      *reinterpret_cast<float4*>(&redx[rl][160 + cg * 4]) = make_float4(sx[4], sx[5], sx[6], sx[7]);
    }
    if (kb == 0 && cg == 0) red[rl][288] = gsum;
    __syncthreads();
    // fixed-order sum over the 8 row lanes
    const int c = threadIdx.x;  // 0..255 -> column kb + c
    if (kb + c < K) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) t += red[r][hidx(c)];
      part_store(dw_part + static_cast<int64_t>(blockIdx.x) * K + kb + c, t, sc1);
      if constexpr (MASK) {
        float tx = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r) tx += redx[r][hidx(c)];
        part_store(dbx_part + static_cast<int64_t>(blockIdx.x) * K + kb + c, tx, sc1);
      }
    }
    if (kb == 0 && threadIdx.x == 0) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) t += red[r][288];
      part_store(db_part + blockIdx.x, t, sc1);
    }
    __syncthreads();
  }
  if (dw == nullptr) return;  // partials only (the caller sums them)
  // the last block to arrive sums the partials in block order into bf16 dw / db
  if (!handoff_last(cnt, gridDim.x, sc1, &last)) return;
  for (int k = threadIdx.x; k < K; k += 256) {
    const float t = part_sum(dw_part + k, static_cast<int>(gridDim.x), K, sc1);
    dw[k] = f32_to_bf16(t);
    if constexpr (MASK) dbx[k] = f32_to_bf16(part_sum(dbx_part + k, static_cast<int>(gridDim.x), K, sc1));
  }
  if (threadIdx.x == 0) {
    const float t = part_sum(db_part, static_cast<int>(gridDim.x), 1, sc1);
    db[0] = f32_to_bf16(t);
    __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

// the split reductions' hand-off (handoff_last): KDL_TUNE ctr_handoff 1 (default) = sc1
// partials, no fences; 0 = release / acquire fences.  CTR step 11.34-11.38 -> 11.43-11.47 M
// samples/s, and with the fused ReLU backward 11.54-11.58 (profiles/r06_ctr_handoff.txt)
static int g_handoff = -1;  // -1: the KDL_TUNE value (read once); set_ctr_handoff overrides
static int handoff_sc1() {
  if (g_handoff < 0) g_handoff = tune_int("ctr_handoff", 1) != 0 ? 1 : 0;
  return g_handoff;
}
void set_ctr_handoff(int sc1) { g_handoff = sc1 < 0 ? -1 : (sc1 != 0 ? 1 : 0); }

int head_bce_fwd_blocks(int M) { return (M + 4 * kHeadRowsPerWave - 1) / (4 * kHeadRowsPerWave); }

hipError_t head_bce_fwd(const void* x, const void* w, const void* b, bool b_bf16, const float* y, int M, int K,
                        float* logit, float* dlogit, float* loss_part, unsigned* cnt, float* loss, hipStream_t s) {
  if (M <= 0) return hipSuccess;
  hipLaunchKernelGGL(head_bce_fwd_kernel, dim3(head_bce_fwd_blocks(M)), dim3(256), 0, s, static_cast<const bf16_t*>(x),
                     static_cast<const bf16_t*>(w), b_bf16 ? nullptr : static_cast<const float*>(b),
                     b_bf16 ? static_cast<const bf16_t*>(b) : nullptr, y, M, K, logit, dlogit, loss_part, cnt, loss,
                     handoff_sc1());
  return hipGetLastError();
}

int head_bce_bwd_blocks(int M) {
  // 128 rows per block, at most 1024 partials (KDL_TUNE ctr_head_rpb: with the batched row
  // loads 128 rows measured +0.3 % per CTR step over 64 and 32 rows -2 to -9 %: more blocks,
  // more ticket atomics on one word; profiles/r06_ctr_rpb2.txt, r06_ctr_small.txt)
  static const int rpb = [] { const int v = tune_int("ctr_head_rpb", 128); return v < 8 ? 8 : v; }();
  int nb = (M + rpb - 1) / rpb;
  return nb < 1024 ? nb : 1024;
}

hipError_t head_bce_bwd(const void* x, const void* w, const float* dlogit, float scale, const float* gscale, int M,
                        int K, void* dx, float* dw_part, float* db_part, unsigned* cnt, void* dw, void* db,
                        hipStream_t s, float* dbx_part, void* dbx) {
  if (M <= 0) return hipSuccess;
  if ((dbx != nullptr) && (dw == nullptr || dbx_part == nullptr)) return hipErrorInvalidValue;
  const int nb = head_bce_bwd_blocks(M);
  const int rpb = (M + nb - 1) / nb;
  if (dbx != nullptr)
    hipLaunchKernelGGL(head_bce_bwd_kernel<true>, dim3(nb), dim3(256), 0, s, static_cast<const bf16_t*>(x),
                       static_cast<const bf16_t*>(w), dlogit, scale, gscale, M, K, rpb, static_cast<bf16_t*>(dx),
                       dw_part, db_part, cnt, static_cast<bf16_t*>(dw), static_cast<bf16_t*>(db), dbx_part,
                       static_cast<bf16_t*>(dbx), handoff_sc1());
  else
    hipLaunchKernelGGL(head_bce_bwd_kernel<false>, dim3(nb), dim3(256), 0, s, static_cast<const bf16_t*>(x),
                       static_cast<const bf16_t*>(w), dlogit, scale, gscale, M, K, rpb, static_cast<bf16_t*>(dx),
                       dw_part, db_part, cnt, static_cast<bf16_t*>(dw), static_cast<bf16_t*>(db), nullptr, nullptr,
                       handoff_sc1());
  return hipGetLastError();
}

static int g_ctr_tile = -2;  // -2: KDL_TUNE ctr_tile, -1: by shape, 0/1/2: 128x128 / 128x64 / 64x64

void set_ctr_tile(int t) { g_ctr_tile = t; }

// the largest tile with >= 1.5 blocks per CU (384 tiles), else the smallest
// (batch 4096: 1728-wide dX 128x128 31.7 us vs 128x64 36.9; 1024-wide forward
// 128x64 30.1 vs 128x128 35.3; 512 / 256 wide 64x64; profiles/r04_ctr_tile_probe.txt)
int ctr_tile_for(int M, int N) {
  if (g_ctr_tile == -2) g_ctr_tile = tune_int("ctr_tile", -1);
  if (g_ctr_tile >= 0) return g_ctr_tile;
  const int bm[3] = {128, 128, 64}, bn[3] = {128, 64, 64};
  for (int c = 0; c < 3; ++c)
    if (static_cast<int64_t>((M + bm[c] - 1) / bm[c]) * ((N + bn[c] - 1) / bn[c]) >= 384) return c;
  return 2;
}

static int g_ctr_igemm = -2;  // -2: KDL_TUNE ctr_igemm; 0 off, 1 by tile count, 2 every K % 64 / N % 64 shape
static int g_ctr_igemm_cfg = -2;

void set_ctr_igemm(int mode, int cfg) { g_ctr_igemm = mode; g_ctr_igemm_cfg = cfg; }

// The LDS-DMA implicit-GEMM main loop (csrc/igemm.hip, DMA issued in the MFMA
// shadow) for the forward layers (B = [N, K]) with at least 128 128x128 tiles:
// at batch 4096 the 1728 -> 1024 layer 32.6 -> 22.4 us and the 1024 -> 512 one
// 14.2 -> 11.3 us against the register-staged kernel below; the 512 -> 256 layer
// (64 tiles) stays there (7.0 vs 8.0 us; profiles/r06_ctr_igemm_probe.txt).
// -1: not served.
int ctr_igemm_cfg_for(int M, int N, int K) {
  if (g_ctr_igemm == -2) g_ctr_igemm = tune_int("ctr_igemm", 1);
  if (g_ctr_igemm_cfg == -2) g_ctr_igemm_cfg = tune_int("ctr_igemm_cfg", -1);
  if (g_ctr_igemm <= 0 || K % 64 || N % 64 || M <= 0) return -1;
  if (g_ctr_igemm_cfg >= 0) return g_ctr_igemm_cfg;
  if (g_ctr_igemm == 2) return N % 128 == 0 ? 2 : 3;
  const int64_t t128 = N % 128 == 0 ? static_cast<int64_t>((M + 127) / 128) * (N / 128) : 0;
  return t128 >= 128 ? 2 : -1;
}

hipError_t gemm_bias_act(const void* A, const void* B, const void* bias, bool bias_bf16, void* C, int M, int N, int K,
                         bool relu, bool b_kn, hipStream_t s) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (b_kn && N % 8) return hipErrorInvalidValue;  // 16-B chunks along N
  if (!b_kn) {
    const int icfg = ctr_igemm_cfg_for(M, N, K);
    if (icfg >= 0) {
      gemm::GemmParams p{};
      p.A = static_cast<const bf16_t*>(A);
      p.B = static_cast<const bf16_t*>(B);
      p.C = static_cast<bf16_t*>(C);
      p.M = M;
      p.N = N;
      p.K = K;
      p.a_rows = M;
      p.shift = bias_bf16 ? nullptr : static_cast<const float*>(bias);
      p.bias16 = bias_bf16 ? static_cast<const bf16_t*>(bias) : nullptr;
      const hipError_t e = gemm::igemm(p, relu ? gemm::EPI_BIAS_RELU : gemm::EPI_BIAS, gemm::G_DENSE, icfg, s);
      if (e != hipErrorInvalidValue) return e;  // InvalidValue: a shape igemm does not take; the kernel below does
    }
  }
  auto a = static_cast<const bf16_t*>(A);
  auto b = static_cast<const bf16_t*>(B);
  auto c = static_cast<bf16_t*>(C);
  const float* b32 = bias_bf16 ? nullptr : static_cast<const float*>(bias);
  const bf16_t* b16 = bias_bf16 ? static_cast<const bf16_t*>(bias) : nullptr;
  const int cfg = ctr_tile_for(M, N);
#define CTR_LAUNCH_GBA(R, TM, TN, T)                                                                                \
  do {                                                                                                       \
    const int tn = (N + TN - 1) / TN, tm = (M + TM - 1) / TM;                                                \
    hipLaunchKernelGGL((gemm_bias_act_kernel<R, TM, TN, T>), dim3(tn * tm), dim3(kThreads), 0, s, a, b, b32, b16, \
                       c, M, N, K, tn);                                                                      \
  } while (0)
#define CTR_LAUNCH_GBA_T(R, T)                 \
  if (cfg == 0) CTR_LAUNCH_GBA(R, 128, 128, T); \
  else if (cfg == 1) CTR_LAUNCH_GBA(R, 128, 64, T); \
  else CTR_LAUNCH_GBA(R, 64, 64, T)
  if (relu) {
    if (b_kn) { CTR_LAUNCH_GBA_T(true, true); }
    else { CTR_LAUNCH_GBA_T(true, false); }
  } else {
    if (b_kn) { CTR_LAUNCH_GBA_T(false, true); }
    else { CTR_LAUNCH_GBA_T(false, false); }
  }
#undef CTR_LAUNCH_GBA_T
#undef CTR_LAUNCH_GBA
  return hipGetLastError();
}

hipError_t gemm_dgrad_relu(const void* A, const void* B, const void* y, void* C, float* part, unsigned* cnt, void* db,
                           int M, int N, int K, hipStream_t s) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (N % 8) return hipErrorInvalidValue;  // B = W [K, N]: 16-B chunks along N
  auto a = static_cast<const bf16_t*>(A);
  auto b = static_cast<const bf16_t*>(B);
  auto ym = static_cast<const bf16_t*>(y);
  auto c = static_cast<bf16_t*>(C);
  auto d = static_cast<bf16_t*>(db);
  const int cfg = ctr_tile_for(M, N);
#define CTR_LAUNCH_DM(TM, TN)                                                                                    \
  do {                                                                                                           \
    const int tn = (N + TN - 1) / TN, tm = (M + TM - 1) / TM;                                                    \
    hipLaunchKernelGGL((gemm_bias_act_kernel<false, TM, TN, true, true>), dim3(tn * tm), dim3(kThreads), 0, s, a, b, \
                       nullptr, nullptr, c, M, N, K, tn, ym, part, cnt, d, handoff_sc1());                       \
  } while (0)
  if (cfg == 0) CTR_LAUNCH_DM(128, 128);
  else if (cfg == 1) CTR_LAUNCH_DM(128, 64);
  else CTR_LAUNCH_DM(64, 64);
#undef CTR_LAUNCH_DM
  return hipGetLastError();
}

int gemm_dgrad_relu_tiles_m(int M, int N) {
  const int bm = ctr_tile_for(M, N) == 2 ? 64 : 128;
  return (M + bm - 1) / bm;
}

int relu_bwd_dbias_rows(int M, int N) {
  // ~256 blocks of 64+ rows (a 4096 x 1024 layer at 256 rows per block was 64
  // blocks on 256 CUs, 44 us)
  const int ncg = (N / 8 + 31) / 32;
  int rows_per_block = static_cast<int>((static_cast<int64_t>(M) * ncg + 255) / 256);
  rows_per_block = (rows_per_block + 7) / 8 * 8;
  return rows_per_block < 64 ? 64 : rows_per_block;
}

int relu_bwd_dbias_parts(int M, int N) {
  const int rpb = relu_bwd_dbias_rows(M, N);
  return (M + rpb - 1) / rpb;
}

hipError_t relu_bwd_dbias(const void* dy, const void* y, void* dz, float* part, unsigned* cnt, void* db, bool db_bf16,
                          int M, int N, hipStream_t s) {
  if (M <= 0 || N <= 0) return hipSuccess;
  const int ncg = (N / 8 + 31) / 32;
  const int rows_per_block = relu_bwd_dbias_rows(M, N);
  dim3 grid((M + rows_per_block - 1) / rows_per_block, ncg);
  hipLaunchKernelGGL(relu_bwd_dbias_kernel, grid, dim3(256), 0, s, static_cast<const bf16_t*>(dy),
                     static_cast<const bf16_t*>(y), static_cast<bf16_t*>(dz), part, cnt,
                     db_bf16 ? static_cast<bf16_t*>(db) : nullptr, db_bf16 ? nullptr : static_cast<float*>(db), M, N,
                     rows_per_block, handoff_sc1());
  return hipGetLastError();
}

hipError_t embed_gather(const void* table, int dtype, const int64_t* idx, int n, int F, int D, void* out, int ld_out,
                        int col0, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int vec = dtype == 1 ? 8 : 4;  // elements per 16-B lane piece
  int lg = 0;
  while (lg < 6 && (vec << lg) < D) ++lg;
  const int64_t groups = (n + kGatherRows - 1) / kGatherRows;
  dim3 grid(static_cast<unsigned>(((groups << lg) + 255) / 256));
  if (dtype == 1)
    hipLaunchKernelGGL((embed_gather_kernel<bf16_t>), grid, dim3(256), 0, s, static_cast<const bf16_t*>(table), idx,
                       n, F, D, static_cast<bf16_t*>(out), ld_out, col0, lg);
  else
    hipLaunchKernelGGL((embed_gather_kernel<float>), grid, dim3(256), 0, s, static_cast<const float*>(table), idx, n,
                       F, D, static_cast<float*>(out), ld_out, col0, lg);
  return hipGetLastError();
}

hipError_t embed_gather_cast(const void* table, bool table_bf16, const int64_t* uniq, const int64_t* inv, int n,
                             int F, int D, void* out, int ld_out, int col0, hipStream_t s, const float* dense, int nd,
                             int tail) {
  if (n <= 0) return hipSuccess;
  if (D % 8 || ld_out % 8 || col0 % 8 || tail % 8 || tail < 0 || nd > tail || (nd > 0 && dense == nullptr))
    return hipErrorInvalidValue;
  int lg = 0;
  while (lg < 6 && (8 << lg) < D) ++lg;
  dim3 grid(static_cast<unsigned>(((static_cast<int64_t>(n) << lg) + 255) / 256));
  if (table_bf16)
    hipLaunchKernelGGL(embed_gather_cast_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(table),
                       uniq, inv, n, F, D, static_cast<bf16_t*>(out), ld_out, col0, lg, dense, nd, tail);
  else
    hipLaunchKernelGGL(embed_gather_cast_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(table), uniq,
                       inv, n, F, D, static_cast<bf16_t*>(out), ld_out, col0, lg, dense, nd, tail);
  return hipGetLastError();
}

// lanes per segment: the power of two G with G*4 >= D (capped at a wave)
static int seg_lanes_log2(int D) {
  int lg = 0;
  while (lg < 6 && (4 << lg) < D) ++lg;
  return lg;
}

hipError_t segment_reduce(const void* rows, int dtype, int F, int ld, int col0, const int64_t* order,
                          const int64_t* seg, int U, int D, float* out, hipStream_t s, const int* ucount,
                          int64_t nrows, const int64_t* out_row, int64_t out_lim) {
  if (U <= 0 || nrows <= 0) return hipSuccess;
  if (!out_row) out_lim = U;
  const int lg = seg_lanes_log2(D);
  dim3 grid(static_cast<unsigned>(((static_cast<int64_t>(U) << lg) + 255) / 256));
  const size_t esz = dtype == 1 ? 2 : 4;
  const bool v4 = D % 4 == 0 && ld % 4 == 0 && col0 % 4 == 0 && reinterpret_cast<uintptr_t>(rows) % (4 * esz) == 0 &&
                  reinterpret_cast<uintptr_t>(out) % 16 == 0;
  // rows j < n = B * F; umulhi division exact while j * F < 2^32
  // (mF = 0 when j * F can reach 2^32: the kernel divides in 64 bits instead)
  const bool fast = static_cast<uint64_t>(nrows) * static_cast<uint64_t>(F) < (uint64_t(1) << 32);
  const uint32_t mF = fast ? static_cast<uint32_t>(((uint64_t(1) << 32) + F - 1) / F) : 0u;
#define CTR_LAUNCH_SEGRED(T, V)                                                                                      \
  hipLaunchKernelGGL((segment_reduce_kernel<T, V>), grid, dim3(256), 0, s, static_cast<const T*>(rows), F, mF, \
                     ld, col0, order, seg, U, D, lg, out, ucount, out_row, out_lim)
  if (dtype == 1) {
    if (v4) CTR_LAUNCH_SEGRED(bf16_t, true);
    else CTR_LAUNCH_SEGRED(bf16_t, false);
  } else {
    if (v4) CTR_LAUNCH_SEGRED(float, true);
    else CTR_LAUNCH_SEGRED(float, false);
  }
#undef CTR_LAUNCH_SEGRED
  return hipGetLastError();
}

hipError_t segment_reduce_adagrad(const void* rows, int dtype, int F, int ld, int col0, const int64_t* order,
                                  const int64_t* seg, int U, int D, const int* ucount, int64_t nrows_in,
                                  const int64_t* rows_local, int64_t nrows, float* table, float* accum, float lr,
                                  float eps, float scale, hipStream_t s) {
  if (U <= 0 || nrows_in <= 0) return hipSuccess;
  const int lg = seg_lanes_log2(D);
  dim3 grid(static_cast<unsigned>(((static_cast<int64_t>(U) << lg) + 255) / 256));
  const size_t esz = dtype == 1 ? 2 : 4;
  const bool v4 = D % 4 == 0 && ld % 4 == 0 && col0 % 4 == 0 && reinterpret_cast<uintptr_t>(rows) % (4 * esz) == 0 &&
                  reinterpret_cast<uintptr_t>(table) % 16 == 0 && reinterpret_cast<uintptr_t>(accum) % 16 == 0;
  const bool fast = static_cast<uint64_t>(nrows_in) * static_cast<uint64_t>(F) < (uint64_t(1) << 32);
  const uint32_t mF = fast ? static_cast<uint32_t>(((uint64_t(1) << 32) + F - 1) / F) : 0u;
#define CTR_LAUNCH_SRA(T, V)                                                                                       \
  hipLaunchKernelGGL((segment_reduce_adagrad_kernel<T, V>), grid, dim3(256), 0, s, static_cast<const T*>(rows), F, \
                     mF, ld, col0, order, seg, U, D, lg, ucount, rows_local, nrows, table, accum, lr, eps, scale)
  if (dtype == 1) {
    if (v4) CTR_LAUNCH_SRA(bf16_t, true);
    else CTR_LAUNCH_SRA(bf16_t, false);
  } else {
    if (v4) CTR_LAUNCH_SRA(float, true);
    else CTR_LAUNCH_SRA(float, false);
  }
#undef CTR_LAUNCH_SRA
  return hipGetLastError();
}

hipError_t segment_adagrad(const float* grads, const int64_t* order, const int64_t* seg, const int64_t* rows_local,
                           int U, int D, int64_t nrows, float* table, float* accum, float lr, float eps, float scale,
                           hipStream_t s, const int* ucount) {
  if (U <= 0) return hipSuccess;
  const int lg = seg_lanes_log2(D);
  dim3 grid(static_cast<unsigned>((static_cast<int64_t>(U) << lg) + 255) / 256);
  const bool v4 = D % 4 == 0 && reinterpret_cast<uintptr_t>(grads) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(table) % 16 == 0 && reinterpret_cast<uintptr_t>(accum) % 16 == 0;
  if (v4)
    hipLaunchKernelGGL(segment_adagrad_kernel<true>, grid, dim3(256), 0, s, grads, order, seg, rows_local, U, D, lg,
                       table, accum, lr, eps, scale, ucount, nrows);
  else
    hipLaunchKernelGGL(segment_adagrad_kernel<false>, grid, dim3(256), 0, s, grads, order, seg, rows_local, U, D, lg,
                       table, accum, lr, eps, scale, ucount, nrows);
  return hipGetLastError();
}

hipError_t a2a_owner_update(const float* grads, const int64_t* local, int S, int cap, int W, int D, int64_t nrows,
                            int64_t* slotmap, int64_t call, float* table, float* accum, float lr, float eps,
                            float scale, hipStream_t s, bool stamped) {
  if (S <= 0 || cap <= 0 || W < 1 || call < 1 || call >= (int64_t(1) << 31)) return hipErrorInvalidValue;
  if (!stamped) {
    hipLaunchKernelGGL(a2a_stamp_kernel, dim3((S + 255) / 256), dim3(256), 0, s, local, S, cap, W, nrows, slotmap,
                       call);
    RETURN_IF_HIP_ERR(hipGetLastError());
  }
  const int lg = seg_lanes_log2(D);
  dim3 grid(static_cast<unsigned>((static_cast<int64_t>(S) << lg) + 255) / 256);
  const bool v4 = D % 4 == 0 && reinterpret_cast<uintptr_t>(grads) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(table) % 16 == 0 && reinterpret_cast<uintptr_t>(accum) % 16 == 0;
  if (v4)
    hipLaunchKernelGGL(a2a_adagrad_kernel<true>, grid, dim3(256), 0, s, grads, local, S, cap, D, lg, W, nrows,
                       slotmap, call, table, accum, lr, eps, scale);
  else
    hipLaunchKernelGGL(a2a_adagrad_kernel<false>, grid, dim3(256), 0, s, grads, local, S, cap, D, lg, W, nrows,
                       slotmap, call, table, accum, lr, eps, scale);
  return hipGetLastError();
}

// ---------------------------------------------------------------- sync-free dedup + CSR
// torch.unique / argsort / bincount of the embedding exchange return
// data-dependent sizes, i.e. a device -> host copy every step, and run as
// rocprim merge sorts.  Here every size is a CAPACITY (n ids -> at most n
// unique ids) and the live count stays on the device:
//
//   insert   open-addressing hash table (T = pow2 >= 2n slots of int64 keys,
//            empty = -1, linear probing, 64-bit atomicCAS): slot_of[i]
//   count    occupied slots per 1024-slot chunk
//   assign   unique id of each occupied slot = its rank in slot order
//            (chunk prefix + in-chunk scan): uniq[uid] = key; the key is reset
//            to empty (the table cleans itself for the next call); the last
//            chunk writes the count
//   inverse  inv[i] = uid of slot_of[i]; uniq[count..n) padded with uniq[0]
//            (a fixed-size gather over the capacity stays in bounds);
//            segment sizes by atomic counting
//   csr      seg = exclusive scan of the sizes (count + assign again), the
//            positions scattered into their segments (atomic cursors: any
//            order), then each segment sorted by position (one wave per
//            segment) -- the gradient sums run in position order: bitwise
//            reproducible, unlike an atomic float accumulation.
// Which slot an id lands in depends on insertion races, so unique-id ORDER is
// not reproducible; nothing numeric depends on it (per-row sums and updates).
namespace {
constexpr int kChunk = 1024;  // slots (or counts) per scan block: 256 threads x 4
constexpr long long kEmpty = -1;

__device__ __forceinline__ uint32_t hash64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return static_cast<uint32_t>(x);
}

__global__ __launch_bounds__(256) void dedup_insert_kernel(const int64_t* __restrict__ ids, int n,
                                                           unsigned long long* __restrict__ keys, uint32_t mask,
                                                           int* __restrict__ slot_of, int* __restrict__ sizes) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  // the segment sizes counted by dedup_inverse_kernel (a later launch) start
  // at zero: cleared here rather than by a runtime memset, so a captured
  // step holds kernel nodes only (docs/perf_notes.md, the CTR hipGraph fault)
  sizes[i] = 0;
  if (i == 0) sizes[n] = 0;
  const unsigned long long id = static_cast<unsigned long long>(ids[i]);
  uint32_t h = hash64(id) & mask;
  // T >= 2n: at most n keys, so a free or matching slot exists within T probes
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    const unsigned long long k = keys[h];
    if (k == id) break;
    if (k == static_cast<unsigned long long>(kEmpty)) {
      const unsigned long long prev = atomicCAS(keys + h, static_cast<unsigned long long>(kEmpty), id);
      if (prev == static_cast<unsigned long long>(kEmpty) || prev == id) break;
    }
    h = (h + 1) & mask;
  }
  slot_of[i] = static_cast<int>(h);
}

// Block b: the number of non-zero flags in [b * kChunk, +kChunk) -> bsum[b].
// mode 0: flags are occupied hash slots (keys != empty); mode 1: int counts.
__global__ __launch_bounds__(256) void chunk_count_kernel(const unsigned long long* __restrict__ keys,
                                                          const int* __restrict__ vals, int len, int mode,
                                                          int* __restrict__ bsum) {
  __shared__ int part[256];
  const int base = blockIdx.x * kChunk + threadIdx.x * 4;
  int c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = base + k;
    if (j < len) c += mode == 0 ? (keys[j] != static_cast<unsigned long long>(kEmpty)) : vals[j];
  }
  part[threadIdx.x] = c;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = part[0];
}

// exclusive prefix of this block's chunk: sum of bsum[0..b) + in-chunk scan
__device__ __forceinline__ int chunk_prefix(const int* bsum, int* part) {
  int acc = 0;
  for (int j = threadIdx.x; j < static_cast<int>(blockIdx.x); j += 256) acc += bsum[j];
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  const int pre = part[0];
  __syncthreads();
  return pre;
}

__device__ __forceinline__ int block_exclusive_scan(int v, int* part) {
  part[threadIdx.x] = v;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {  // Hillis-Steele inclusive
    const int add = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += add;
    __syncthreads();
  }
  const int incl = part[threadIdx.x];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(256) void dedup_assign_kernel(unsigned long long* __restrict__ keys, int T,
                                                           const int* __restrict__ bsum, int* __restrict__ slot_uid,
                                                           int64_t* __restrict__ uniq, int* __restrict__ count) {
  __shared__ int part[256];
  const int pre = chunk_prefix(bsum, part);
  const int base = blockIdx.x * kChunk + threadIdx.x * 4;
  unsigned long long k4[4];
  int c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = base + k;
    k4[k] = j < T ? keys[j] : static_cast<unsigned long long>(kEmpty);
    c += k4[k] != static_cast<unsigned long long>(kEmpty);
  }
  int uid = pre + block_exclusive_scan(c, part);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = base + k;
    if (k4[k] != static_cast<unsigned long long>(kEmpty)) {
      slot_uid[j] = uid;
      uniq[uid] = static_cast<int64_t>(k4[k]);
      keys[j] = static_cast<unsigned long long>(kEmpty);  // clean for the next call
      ++uid;
    }
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 255) *count = uid;
}

__global__ __launch_bounds__(256) void dedup_inverse_kernel(const int* __restrict__ slot_of, int n,
                                                            const int* __restrict__ slot_uid,
                                                            int64_t* __restrict__ inv, int64_t* __restrict__ uniq,
                                                            const int* __restrict__ count, int* __restrict__ sizes) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int u = slot_uid[slot_of[i]];
  inv[i] = u;
  atomicAdd(sizes + u, 1);
  if (i >= *count) uniq[i] = uniq[0];
}

// seg[u] = exclusive prefix of sizes (u <= n); cursor[u] = 0 for the scatter
__global__ __launch_bounds__(256) void csr_assign_kernel(const int* __restrict__ sizes, int len,
                                                         const int* __restrict__ bsum, int64_t* __restrict__ seg,
                                                         int* __restrict__ cursor, int* __restrict__ nlong) {
  __shared__ int part[256];
  if (blockIdx.x == 0 && threadIdx.x == 0) *nlong = 0;  // (read by csr_sort_kernel, a later launch)
  const int pre = chunk_prefix(bsum, part);
  const int base = blockIdx.x * kChunk + threadIdx.x * 4;
  int v[4], c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = base + k < len ? sizes[base + k] : 0;
    c += v[k];
  }
  int off = pre + block_exclusive_scan(c, part);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = base + k;
    if (j < len) {
      seg[j] = off;
      cursor[j] = 0;
    }
    off += v[k];
  }
}

__global__ __launch_bounds__(256) void csr_scatter_kernel(const int64_t* __restrict__ inv, int n,
                                                          const int64_t* __restrict__ seg, int* __restrict__ cursor,
                                                          int64_t* __restrict__ order) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int u = static_cast<int>(inv[i]);
  order[seg[u] + atomicAdd(cursor + u, 1)] = i;
}

// one wave per segment: sort its positions ascending, in place.  Segments of
// up to 64 positions are a wave bitonic sort in registers; longer ones (hot
// ids) are appended to ``list`` (counter *nlong, reset by csr_assign_kernel)
// for csr_sort_long_kernel.
__global__ __launch_bounds__(256) void csr_sort_kernel(const int64_t* __restrict__ seg, int64_t* __restrict__ order,
                                                       const int* __restrict__ count, int* __restrict__ nlong,
                                                       int* __restrict__ list) {
  const int u = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (u >= *count) return;
  const int64_t s0 = seg[u], len = seg[u + 1] - s0;
  if (len <= 1) return;
  int64_t* o = order + s0;
  if (len <= 64) {  // wave bitonic sort of one value per lane (pad: INT64_MAX)
    int64_t v = lane < len ? o[lane] : INT64_MAX;
    for (int k = 2; k <= 64; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        const int64_t w = __shfl_xor(v, j);
        const bool up = (lane & k) == 0;
        const bool lower = (lane & j) == 0;
        const int64_t lo = v < w ? v : w, hi = v < w ? w : v;
        v = (lower == up) ? lo : hi;
      }
    }
    if (lane < len) o[lane] = v;
    return;
  }
  if (lane == 0) list[atomicAdd(nlong, 1)] = u;
}

constexpr int kLongSort = 8192;                 // positions sorted in LDS by one block
constexpr int kBitWindow = kLongSort * 32;      // positions per bitmap window (same 32 KiB)

// One block per long segment (grid-stride over the list).  Up to kLongSort
// positions: block bitonic sort of int32 positions in LDS, O(L log^2 L).
// Longer: the positions are distinct integers in [0, n), so their ascending
// order is a bitmap scan -- per window of kBitWindow positions set one bit per
// member, then every thread emits the set bits of its 32 words at its scanned
// offset; O(L + n / 32) per segment, and at most n / kLongSort such segments.
__global__ __launch_bounds__(256) void csr_sort_long_kernel(const int64_t* __restrict__ seg,
                                                            int64_t* __restrict__ order,
                                                            const int* __restrict__ nlong,
                                                            const int* __restrict__ list, int* __restrict__ scratch,
                                                            int n) {
  __shared__ unsigned int buf[kLongSort];
  __shared__ int part[256];
  const int nl = *nlong;
  for (int li = blockIdx.x; li < nl; li += gridDim.x) {
    const int u = list[li];
    const int64_t s0 = seg[u];
    const int len = static_cast<int>(seg[u + 1] - s0);
    int64_t* o = order + s0;
    if (len <= kLongSort) {
      int P = 128;
      while (P < len) P <<= 1;
      for (int i = threadIdx.x; i < P; i += 256) buf[i] = i < len ? static_cast<unsigned int>(o[i]) : 0xffffffffu;
      __syncthreads();
      for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = threadIdx.x; i < P; i += 256) {
            const int l = i ^ j;
            if (l > i) {
              const unsigned int a = buf[i], b = buf[l];
              const bool up = (i & k) == 0;
              if ((a > b) == up) { buf[i] = b; buf[l] = a; }
            }
          }
          __syncthreads();
        }
      }
      for (int i = threadIdx.x; i < len; i += 256) o[i] = static_cast<int64_t>(buf[i]);
      __syncthreads();
      continue;
    }
    // bitmap scan: the members are copied to ``scratch`` (int32, this
    // segment's own range of it) so every window reads them there while the
    // sorted positions are written to o[]
    for (int i = threadIdx.x; i < len; i += 256) scratch[s0 + i] = static_cast<int>(o[i]);
    __syncthreads();
    int base = 0;  // positions emitted by earlier windows
    for (int w0 = 0; w0 < n; w0 += kBitWindow) {
      for (int i = threadIdx.x; i < kLongSort; i += 256) buf[i] = 0u;
      __syncthreads();
      for (int i = threadIdx.x; i < len; i += 256) {
        const int p = scratch[s0 + i] - w0;
        if (p >= 0 && p < kBitWindow) atomicOr(&buf[p >> 5], 1u << (p & 31));
      }
      __syncthreads();
      int c = 0;
      for (int k = 0; k < 32; ++k) c += __popc(buf[threadIdx.x * 32 + k]);
      int off = base + block_exclusive_scan(c, part);
      const int tot = part[255];  // inclusive scan: the window's member count
      for (int k = 0; k < 32; ++k) {
        unsigned int m = buf[threadIdx.x * 32 + k];
        while (m) {
          const int bit = __ffs(m) - 1;
          m &= m - 1;
          o[off++] = static_cast<int64_t>(w0 + (threadIdx.x * 32 + k) * 32 + bit);
        }
      }
      base += tot;
      __syncthreads();
    }
  }
}
// ---------------------------------------------------------------- fixed-capacity exchange (PS + worker)
// A pull of U de-duplicated ids at a capacity ``cap`` every rank agrees on
// (models/ctr.py ShardedEmbedding._pull_fixed): the send buffer holds one
// block of cap + 1 int64 slots per destination rank -- the ids owned by that
// rank (owner = owner_rank[id % n_own]) in slots [0, fill), -1 padding up to
// cap, and in slot cap the header: this sender's largest per-destination fill
// (the same value in every block).  rslot[i] = d * cap + pos names the row of
// the received [W * cap] rows that answers unique id i (W * cap = the zero
// dump row: the id did not fit, or i >= *count).  Ids keep their unique order
// within a destination (a block-stable counting sort: per-block counts, then
// every block sums the earlier blocks' counts itself), so the route is a pure
// function of uniq.  Two launches, no host sync, no one-hot [U, W + 1] matrix.
constexpr int kA2aMaxW = 64;

__global__ __launch_bounds__(256) void a2a_count_kernel(const int64_t* __restrict__ uniq,
                                                        const int* __restrict__ count, int n,
                                                        const int64_t* __restrict__ owner_rank, int n_own, int W,
                                                        int* __restrict__ cnt) {
  __shared__ int c[kA2aMaxW];
  for (int d = threadIdx.x; d < W; d += 256) c[d] = 0;
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int live = count ? *count : n;
  if (i < n && i < live) atomicAdd(&c[owner_rank[uniq[i] % n_own]], 1);  // LDS counts: order-free
  __syncthreads();
  for (int d = threadIdx.x; d < W; d += 256) cnt[blockIdx.x * W + d] = c[d];
}

__global__ __launch_bounds__(256) void a2a_route_kernel(const int64_t* __restrict__ uniq,
                                                        const int* __restrict__ count, int n,
                                                        const int64_t* __restrict__ owner_rank, int n_own, int W,
                                                        int cap, const int* __restrict__ cnt, int nblk,
                                                        int64_t* __restrict__ send, int64_t* __restrict__ rslot) {
  __shared__ int base[kA2aMaxW], tot[kA2aMaxW], wcnt[4][kA2aMaxW];
  __shared__ int red[4][2];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // totals per destination and this block's exclusive base: all threads stride
  // the per-block counts, wave sums, then the four waves in LDS
  for (int d = 0; d < W; ++d) {
    int sb = 0, st = 0;
    for (int b = t; b < nblk; b += 256) {
      const int v = cnt[b * W + d];
      st += v;
      sb += b < static_cast<int>(blockIdx.x) ? v : 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      sb += __shfl_xor(sb, o);
      st += __shfl_xor(st, o);
    }
    if (lane == 0) { red[wv][0] = sb; red[wv][1] = st; }
    __syncthreads();
    if (t == 0) {
      base[d] = red[0][0] + red[1][0] + red[2][0] + red[3][0];
      tot[d] = red[0][1] + red[1][1] + red[2][1] + red[3][1];
    }
    __syncthreads();
  }
  for (int k = t; k < 4 * kA2aMaxW; k += 256) (&wcnt[0][0])[k] = 0;
  const int i = blockIdx.x * 256 + t;
  const int live = count ? *count : n;
  const bool valid = i < n && i < live;
  const int64_t id = valid ? uniq[i] : 0;
  const int d = valid ? static_cast<int>(owner_rank[id % n_own]) : -1;
  // lanes of this wave with the same destination (stable: lane order = id order)
  uint64_t same = 0;
  uint64_t todo = __ballot(valid);
  while (todo) {
    const int leader = __ffsll(static_cast<unsigned long long>(todo)) - 1;
    const int dl = __shfl(d, leader);
    const uint64_t m = __ballot(d == dl);
    if (d == dl) same = m;
    todo &= ~m;
  }
  __syncthreads();  // wcnt zeroed
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  if (valid && (same & below) == 0) wcnt[wv][d] = __popcll(same);  // the lowest lane of its group
  __syncthreads();
  if (i < n) {
    int64_t slot = static_cast<int64_t>(W) * cap;  // dump row
    if (valid) {
      int pos = base[d] + __popcll(same & below);
      for (int w = 0; w < wv; ++w) pos += wcnt[w][d];
      if (pos < cap) {
        send[static_cast<int64_t>(d) * (cap + 1) + pos] = id;
        slot = static_cast<int64_t>(d) * cap + pos;
      }
    }
    rslot[i] = slot;
  }
  // padding and headers of every destination block, spread over the grid
  int hdr = 0;
  for (int e = 0; e < W; ++e) hdr = tot[e] > hdr ? tot[e] : hdr;
  const int64_t slots = static_cast<int64_t>(W) * (cap + 1);
  for (int64_t s = static_cast<int64_t>(blockIdx.x) * 256 + t; s < slots; s += static_cast<int64_t>(gridDim.x) * 256) {
    const int dd = static_cast<int>(s / (cap + 1));
    const int p = static_cast<int>(s - static_cast<int64_t>(dd) * (cap + 1));
    if (p == cap) send[s] = hdr;
    else if (p >= (tot[dd] < cap ? tot[dd] : cap)) send[s] = -1;
  }
}

// Owner side of a fixed exchange: the W * cap requested ids (-1 = padding) ->
// the rows to send back (padding rows zero) and the local row index of every
// slot for the push's update (padding -> distinct negative sentinels -2 - r:
// one-row segments the update skips).  One lane group of 2^lg lanes per slot.
template <typename T>
__global__ __launch_bounds__(256) void a2a_serve_kernel(const float* __restrict__ table, const int64_t* __restrict__ req,
                                                        int n, int n_own, int D, int lg, T* __restrict__ rows,
                                                        int64_t* __restrict__ local, int64_t* __restrict__ slotmap,
                                                        int64_t call, int cap, int W, int64_t nrows) {
  const int r = (blockIdx.x * 256 + threadIdx.x) >> lg;
  const int gl = threadIdx.x & ((1 << lg) - 1);
  if (r >= n) return;
  const int64_t id = req[r];
  // an id past this owner's shard (a sender's id at or beyond the vocab) is
  // served like padding -- a zero row, a negative local the update skips --
  // never read out of the table's bounds
  const int64_t row = (id >= 0 && id / n_own < nrows) ? id / n_own : -2 - static_cast<int64_t>(r);
  if (gl == 0) {
    local[r] = row;
    // the push's owner update stamp (a2a_stamp_kernel's store), here while the
    // slot's row is at hand: one launch less per step
    if (slotmap != nullptr && row >= 0) slotmap[row * W + r / cap] = (call << 32) | r;
  }
  T* dst = rows + static_cast<int64_t>(r) * D;
  const float* src = table + (row >= 0 ? row : 0) * static_cast<int64_t>(D);
  for (int c = gl * 4; c < D; c += 4 << lg) {
    const float4 v = row >= 0 ? *reinterpret_cast<const float4*>(src + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (sizeof(T) == 2)  // the bf16 rounding the tower input gets anyway, done once by the owner
      *reinterpret_cast<uint2*>(dst + c) = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
    else
      *reinterpret_cast<float4*>(dst + c) = v;
  }
}

}  // namespace

int a2a_max_world() { return kA2aMaxW; }

hipError_t a2a_route(const int64_t* uniq, const int* count, int n, const int64_t* owner_rank, int n_own, int W,
                     int cap, int* cnt, int64_t* send, int64_t* rslot, hipStream_t s) {
  if (W < 1 || W > kA2aMaxW || cap < 1 || n_own < 1 || n < 0) return hipErrorInvalidValue;
  const int nblk = n > 0 ? (n + 255) / 256 : 1;
  hipLaunchKernelGGL(a2a_count_kernel, dim3(nblk), dim3(256), 0, s, uniq, count, n, owner_rank, n_own, W, cnt);
  hipLaunchKernelGGL(a2a_route_kernel, dim3(nblk), dim3(256), 0, s, uniq, count, n, owner_rank, n_own, W, cap, cnt,
                     nblk, send, rslot);
  return hipGetLastError();
}

int a2a_route_blocks(int n) { return n > 0 ? (n + 255) / 256 : 1; }

hipError_t a2a_serve(const float* table, const int64_t* req, int n, int n_own, int D, void* rows, bool rows_bf16,
                     int64_t* local, hipStream_t s, int64_t* slotmap, int64_t call, int cap, int W, int64_t nrows) {
  if (n <= 0) return hipSuccess;
  if (D % 4 || n_own < 1) return hipErrorInvalidValue;
  if (slotmap != nullptr && (cap < 1 || W < 1 || n != W * cap || call < 1 || call >= (int64_t(1) << 31)))
    return hipErrorInvalidValue;
  const int lg = seg_lanes_log2(D);
  dim3 grid(static_cast<unsigned>(((static_cast<int64_t>(n) << lg) + 255) / 256));
  if (rows_bf16)
    hipLaunchKernelGGL(a2a_serve_kernel<bf16_t>, grid, dim3(256), 0, s, table, req, n, n_own, D, lg,
                       static_cast<bf16_t*>(rows), local, slotmap, call, cap, W, nrows);
  else
    hipLaunchKernelGGL(a2a_serve_kernel<float>, grid, dim3(256), 0, s, table, req, n, n_own, D, lg,
                       static_cast<float*>(rows), local, slotmap, call, cap, W, nrows);
  return hipGetLastError();
}

int dedup_table_slots(int n) {
  int T = 1024;
  while (T < 2 * n) T <<= 1;
  return T;
}

hipError_t dedup_ids(const int64_t* ids, int n, void* keys, int T, int* slot_of, int* slot_uid, int* bsum,
                     int64_t* uniq, int64_t* inv, int* count, int* sizes, hipStream_t s) {
  if (n <= 0 || T < 2 * n || (T & (T - 1)) || T % kChunk) return hipErrorInvalidValue;
  auto* k = static_cast<unsigned long long*>(keys);
  hipLaunchKernelGGL(dedup_insert_kernel, dim3((n + 255) / 256), dim3(256), 0, s, ids, n, k,
                     static_cast<uint32_t>(T - 1), slot_of, sizes);
  const int nb = T / kChunk;
  hipLaunchKernelGGL(chunk_count_kernel, dim3(nb), dim3(256), 0, s, k, static_cast<const int*>(nullptr), T, 0, bsum);
  hipLaunchKernelGGL(dedup_assign_kernel, dim3(nb), dim3(256), 0, s, k, T, bsum, slot_uid, uniq, count);
  hipLaunchKernelGGL(dedup_inverse_kernel, dim3((n + 255) / 256), dim3(256), 0, s, slot_of, n, slot_uid, inv, uniq,
                     count, sizes);
  return hipGetLastError();
}

int csr_bsum_slots(int n) { return (n + 1 + kChunk - 1) / kChunk + 1; }

hipError_t csr_from_inverse(const int64_t* inv, int n, int* sizes, const int* count, int* bsum, int* cursor,
                            int64_t* seg, int64_t* order, hipStream_t s) {
  if (n <= 0) return hipErrorInvalidValue;
  const int len = n + 1;
  const int nb = (len + kChunk - 1) / kChunk;
  int* nlong = bsum + nb;  // long-segment counter; the list itself reuses cursor once the scatter is done
  hipLaunchKernelGGL(chunk_count_kernel, dim3(nb), dim3(256), 0, s, static_cast<const unsigned long long*>(nullptr),
                     sizes, len, 1, bsum);
  hipLaunchKernelGGL(csr_assign_kernel, dim3(nb), dim3(256), 0, s, sizes, len, bsum, seg, cursor, nlong);
  hipLaunchKernelGGL(csr_scatter_kernel, dim3((n + 255) / 256), dim3(256), 0, s, inv, n, seg, cursor, order);
  // long segments (at most n / 65): their list reuses cursor and their
  // scratch reuses sizes -- both are dead once the scatter has run
  hipLaunchKernelGGL(csr_sort_kernel, dim3((n + 3) / 4), dim3(256), 0, s, seg, order, count, nlong, cursor);
  const int gl = std::min(n / 65 + 1, 1024);
  hipLaunchKernelGGL(csr_sort_long_kernel, dim3(gl), dim3(256), 0, s, seg, order, nlong, cursor, sizes, n);
  return hipGetLastError();
}

}  // namespace kdl
