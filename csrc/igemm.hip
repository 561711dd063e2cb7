// Long-K conv GEMMs on an LDS-DMA operand pipeline (gfx950).
//
//   C[M, N] = A[M, K] . B[N, K]^T, bf16 in, fp32 MFMA accumulation, bf16 out,
//   with the fused ResNet epilogues of csrc/gemm_epi.h.
//   A rows: dense | stride-s 1x1 gather | 3x3 pad-1 implicit GEMM (K = 9 Cin,
//   one tap per 64-deep K-step; padding taps are buffer-OOB loads, which the
//   hardware returns as zeros) | stride-2 3x3 data gradient (G_DGRAD2): dx
//   pixel (2i + py, 2j + px) only sees the taps with r = py ? {0, 2} : {1}
//   and s = px ? {0, 2} : {1}, reading dy at (i + [r == 0], j + [s == 0]);
//   the four (py, px) classes are four GEMMs of 1, 2, 2, 4 taps over the
//   dy-sized pixel grid, run as consecutive M-tile ranges of one launch with
//   the weights regrouped class-major (no zero taps, no zero-filled output;
//   the epilogue scatters rows to their dx pixels).
//
// Why a second main loop (csrc/conv1x1.hip keeps the register-staged one for
// short K and for the BN+ReLU prologue): the register-staged loop spends
// ~49 % of its wave time waiting on operands and its ds_write pass adds ~40 %
// LDS traffic on top of the fragment reads (profiles/r01_gemm_longk_pmc.txt).
// Here every operand byte goes HBM/L2 -> LDS by `buffer_load_dwordx4 ... lds`
// (no VGPRs, no ds_write), 1 KiB per wave instruction, issued one full K-step
// ahead so each 64-deep stage lands while the previous one is multiplied:
//
//   issue(stage 0)
//   for k-step t:  barrier (t landed everywhere; stage t+1 free) ;
//                  issue(t+1 -> other stage) ; fragments + MFMAs of stage t
//
// LDS image: each operand row is 64 bf16 = 128 B = 8 chunks of 16 B, chunk c
// of row r stored at chunk position c ^ ((r >> 1) & 7).  The DMA writes
// lane-linear (base + 16 * lane), so the swizzle is applied to the SOURCE
// address (guide §5.4 rule 21), and a fragment read of 32 consecutive rows at
// one logical chunk is conflict-free for every 16-lane group of
// ds_read_b128.  MFMA v_mfma_f32_32x32x16_bf16 with the weight fragment as
// the A operand (lanes index output pixels, registers 4 channel runs: the
// epilogue's LDS transpose).  Blocks are persistent over M tiles with the
// XCD-aware (tile_n, M-sequence) order of conv1x1.hip.
//
// The reference has no kernels; this serves the PyTorchJob
// ResNet-50 worker (BASELINE.json config 2).
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>

#include "common.h"
#include "gemm_epi.h"
#include "kdl_api.h"
#include "lds_dma.h"
#include "tune.h"

namespace kdl {
namespace {

using namespace gemm;

using lds_dma::lds_void_t;
using lds_dma::i32x4_t;
using lds_dma::kOOB;
using lds_dma::rsrc_words;
using lds_dma::dma16;
using lds_dma::publish_stage;

constexpr int IBK = 64;  // K per stage (one 128-B LDS row per operand row)

template <int A, int B> struct cmax { static constexpr int v = A > B ? A : B; };

template <int BM, int BN, int WM, int WN, int GATHER, int EPI, int MINB, int STAGES>
__global__ __launch_bounds__(64 * WM * WN, MINB) void igemm_kernel(GemmParams p, int GM, int tiles_m, int tiles_n) {
  static_assert(STAGES == 2 || STAGES == 3, "2 or 3 LDS stages");
  constexpr int NT = 64 * WM * WN;
  constexpr int NW = WM * WN;
  constexpr int SA = BM * 128, SB = BN * 128, STAGE = SA + SB;  // bytes per stage
  static_assert((BM + BN) % (8 * NW) == 0 && BM % 16 == 0 && BN % 16 == 0, "DMA row groups");
  constexpr int IPW = (BM + BN) / 8 / NW;  // 1-KiB DMA instructions per wave per stage
  constexpr int WTM = BM / WM, WTN = BN / WN;
  static_assert(WTM % 32 == 0 && WTN % 32 == 0, "wave tile = whole 32x32 MFMA blocks");
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int NMF = 4 * TN * TM;  // MFMAs per wave per K-step
  using Epi = Epilogue<BM, BN, NT, EPI, GATHER>;
  constexpr bool TAPS = GATHER == G_CONV3 || GATHER == G_DGRAD2;
  constexpr int LDC = Epi::LDC;
  constexpr int LDS_BYTES = cmax<cmax<STAGES * STAGE, BM * LDC * 2>::v, Epi::kScratchBytes>::v;
  // ONE __shared__ object (a second one makes hipcc drain vmcnt before ds_reads)
  __shared__ __attribute__((aligned(1024))) char lds[LDS_BYTES];

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nblk = gridDim.x, b = blockIdx.x;
  const int q = (b & 7) * (nblk >> 3) + (b >> 3);  // nblk % 8 == 0 (host)
  const int tile_n = q % tiles_n;
  const int gm = q / tiles_n;
  const int n0 = tile_n * BN;
  const int K = p.K, M = p.M;
  int nk = K / IBK;
  const int wm0 = (wave / WN) * WTM, wn0 = (wave % WN) * WTN;
  const int fr = lane & 31, fh = lane >> 5;

  // buffer resources (wave-uniform: built from kernel arguments only)
  const int lda = TAPS ? p.Cin : K;
  // (a zero-record descriptor drops that operand's loads: KDL_TUNE igemm_price timing builds)
  const int bytesA = (p.price_drop & 1) ? 0 : static_cast<int>(p.a_rows * lda * 2);
  const int bytesB = (p.price_drop & 2) ? 0 : static_cast<int>(static_cast<int64_t>(p.N) * K * 2);
  const i32x4_t wA = rsrc_words(p.A, static_cast<uint32_t>(bytesA));
  const i32x4_t wB = rsrc_words(p.B, static_cast<uint32_t>(bytesB));

  // Per DMA piece i of this wave (1 KiB: 8 operand rows x 8 16-B chunks, the
  // lane's chunk swizzled at the SOURCE): a byte offset base and an INVERTED
  // validity mask, so that every piece of every gather is issued as
  //   voffset = (base + delta) | (((inv >> bit) & 1) << 31),  soffset = soff
  // with wave-uniform (delta, bit, soff) per K-step: bit 31 puts an invalid
  // row past num_records (< 2^31) and the hardware returns zeros.  3x3 taps:
  // bit 3r + s of the mask is tap (r, s); delta = ((r Win + s) Cin + kc0) * 2
  // from the row's (ih0, iw0) pixel.  Dense / strided A rows and B rows: one
  // bit (row < M, or always), delta 0, the K column in soffset.  No per-piece
  // branch and no per-piece integer division in the main loop.
  const int lrow = lane >> 3;
  int pbase[IPW];
  uint32_t pinv[IPW];
  bool pisA[IPW];  // wave-uniform
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int g = wave * IPW + i;
    pisA[i] = g < BM / 8;
    if (!pisA[i]) {  // B (weights): row n0 + r, chunk c
      const int r = 8 * (g - BM / 8) + lrow;
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      pbase[i] = ((n0 + r) * K + 8 * c) * 2;
      pinv[i] = 0;
    }
  }
  // G_DGRAD2 (per tile, wave-uniform): sub-pixel class (py, px), its taps per
  // row-of-taps (ns) and its first K column in the class-major weight matrix
  int py = 0, px = 0, ns = 1, koff = 0;
  (void)py; (void)px; (void)ns; (void)koff;

  auto setup_rows = [&](int tm) {
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      if (!pisA[i]) continue;
      const int g = wave * IPW + i;
      const int r = 8 * g + lrow;
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int m = tm * BM + r;
      if constexpr (TAPS) {
        bool live;
        int crow, ih0, iw0;
        if constexpr (GATHER == G_DGRAD2) {
          const int cls = tm / (p.mc_pad / BM);
          const int mc = m - cls * p.mc_pad;  // row within the class
          live = mc < p.mc;
          const int hw = p.Hin * p.Win;
          const int nimg = mc / hw, rem = mc - nimg * hw;
          crow = nimg * hw;
          ih0 = rem / p.Win;
          iw0 = rem - ih0 * p.Win;
        } else {
          live = m < M;
          const int hw = p.Hout * p.Wout;
          const int nimg = m / hw, rem = m - nimg * hw;
          const int oh = rem / p.Wout, ow = rem - oh * p.Wout;
          crow = nimg * p.Hin * p.Win;
          ih0 = oh * p.stride - 1;
          iw0 = ow * p.stride - 1;
        }
        uint32_t valid = 0;
#pragma unroll
        for (int rr = 0; rr < 3; ++rr)
#pragma unroll
          for (int ss = 0; ss < 3; ++ss) {
            const bool ok = static_cast<unsigned>(ih0 + rr) < static_cast<unsigned>(p.Hin) &&
                            static_cast<unsigned>(iw0 + ss) < static_cast<unsigned>(p.Win);
            valid |= (ok ? 1u : 0u) << (3 * rr + ss);
          }
        pinv[i] = live ? ~valid : ~0u;
        pbase[i] = live ? ((crow + ih0 * p.Win + iw0) * p.Cin + 8 * c) * 2 : 0;
      } else {
        int64_t src = m;
        if constexpr (GATHER == G_STRIDED) {
          const int hw = p.Hout * p.Wout;
          const int nimg = m / hw, rem = m - nimg * hw;
          const int oh = rem / p.Wout, ow = rem - oh * p.Wout;
          src = (static_cast<int64_t>(nimg) * p.Hin + oh * p.stride) * p.Win + ow * p.stride;
        }
        pinv[i] = m < M ? 0u : ~0u;
        pbase[i] = m < M ? static_cast<int>((src * K + 8 * c) * 2) : 0;
      }
    }
  };

  // wave-uniform per K-step: (delta, bit, soffset) of its A pieces and the
  // soffset of its B pieces
  struct KStep { int delta; int bit; uint32_t soffA, soffB; };
  auto kstep_of = [&](int kt) {
    KStep s;
    const int k0 = kt * IBK;
    s.delta = 0;
    s.bit = 0;
    s.soffA = static_cast<uint32_t>(k0 * 2);
    s.soffB = static_cast<uint32_t>((koff + k0) * 2);
    if constexpr (TAPS) {
      const int tap = k0 / p.Cin;  // a 64-deep K-step never straddles taps (Cin % 64 == 0)
      const int kc0 = k0 - tap * p.Cin;
      int r3, q3;
      if constexpr (GATHER == G_DGRAD2) {
        // class tap (ri, si): dy pixel offset (di, dj) = (py && ri == 0, px && si == 0)
        const int ri = tap / ns, si = tap - ri * ns;
        r3 = (py && ri == 0) ? 1 : 0;
        q3 = (px && si == 0) ? 1 : 0;
      } else {
        r3 = tap / 3;
        q3 = tap - 3 * r3;
      }
      s.delta = ((r3 * p.Win + q3) * p.Cin + kc0) * 2;
      s.bit = 3 * r3 + q3;
      s.soffA = 0;
    }
    return s;
  };
  auto piece = [&](int i, const KStep& s, int stage) {
    const int g = wave * IPW + i;
    lds_void_t* dst = (lds_void_t*)(lds + stage * STAGE + g * 1024);
    const int delta = pisA[i] ? s.delta : 0;
    const int bit = pisA[i] ? s.bit : 0;
    const uint32_t off = static_cast<uint32_t>(pbase[i] + delta) | (((pinv[i] >> bit) & 1u) << 31);
    dma16(pisA[i] ? wA : wB, dst, off, pisA[i] ? s.soffA : s.soffB);
  };

  // fragment byte offsets within a row: logical chunk 2s + fh, swizzled by the
  // row's (r >> 1) & 7 == (fr >> 1) & 7 (fragment rows start at multiples of 16)
  uint32_t xo[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) xo[s] = static_cast<uint32_t>((((2 * s + fh) ^ ((fr >> 1) & 7))) * 16);

  Epi epi;
  epi.init(t, n0);

  int tm = gm;
  for (; tm < tiles_m; tm += GM) {
    if constexpr (GATHER == G_DGRAD2) {
      // class 0 (py, px) = (0, 0): 1 tap; 1 = (0, 1): 2; 2 = (1, 0): 2; 3 = (1, 1): 4
      const int cls = tm / (p.mc_pad / BM);
      py = cls >> 1;
      px = cls & 1;
      ns = px ? 2 : 1;
      koff = (cls == 0 ? 0 : cls == 1 ? 1 : cls == 2 ? 3 : 5) * p.Cin;
      nk = (py ? 2 : 1) * ns * (p.Cin / IBK);
    }
    setup_rows(tm);
    f32x16_t acc[TN][TM];
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = f32x16_t{};
    auto frags = [&](const char* As, int s, bf16x8_t (&wf)[TN], bf16x8_t (&xf)[TM]) {
      const char* Bs = As + SA;
#pragma unroll
      for (int i = 0; i < TN; ++i)
        wf[i] = *reinterpret_cast<const bf16x8_t*>(Bs + (wn0 + i * 32 + fr) * 128 + xo[s]);
#pragma unroll
      for (int j = 0; j < TM; ++j)
        xf[j] = *reinterpret_cast<const bf16x8_t*>(As + (wm0 + j * 32 + fr) * 128 + xo[s]);
    };
    // One K-step of MFMAs on stage `As`, fragments double-buffered (substep
    // s + 1's reads issued before substep s's MFMAs); with ISSUE, the next
    // K-step's DMA pieces are spread over the first half of the MFMAs (one
    // piece per MFMA gap at most), so their issue cost runs in the MFMA
    // shadow instead of in a burst after the barrier, and each lands about
    // half a K-step before the barrier that publishes it.
    auto compute = [&](const char* As, auto issue_tag, const KStep& ks, int nstage) {
      constexpr bool ISSUE = decltype(issue_tag)::value;
      constexpr int SPAN = NMF / 2 > IPW ? NMF / 2 : (NMF > IPW ? IPW : NMF);
      bf16x8_t wf[2][TN], xf[2][TM];
      frags(As, 0, wf[0], xf[0]);
      int done = 0;
      (void)done;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (s < 3) frags(As, s + 1, wf[(s + 1) & 1], xf[(s + 1) & 1]);
        // pin the prefetch ahead of this substep's MFMAs (the scheduler would
        // otherwise sink the reads next to their first use and expose the LDS
        // latency four times per K-step)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) {
            const int mi = (s * TN + i) * TM + j;  // MFMA index within the K-step
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[s & 1][i], xf[s & 1][j], acc[i][j], 0, 0, 0);
            if constexpr (ISSUE) {
              // pieces [mi * IPW / SPAN, (mi + 1) * IPW / SPAN) after MFMA mi (mi < SPAN)
#pragma unroll
              for (int pi = 0; pi < IPW; ++pi)
                if (pi * SPAN / IPW == mi) piece(pi, ks, nstage);
            }
          }
      }
    };
    using yes = std::integral_constant<bool, true>;
    using no = std::integral_constant<bool, false>;
    if constexpr (STAGES == 2) {
      {
        const KStep k0s = kstep_of(0);
#pragma unroll
        for (int i = 0; i < IPW; ++i) piece(i, k0s, 0);
      }
      // stage kt landed (every wave's vmcnt(0) + barrier); every wave's
      // fragment reads of stage kt - 1 retired: stage kt + 1 is free.  The
      // last K-step is peeled (no DMA): one loop body, so the accumulators
      // keep their registers (an if/else of two bodies copies them per step).
      int kt = 0;
      for (; kt + 1 < nk; ++kt) {
        publish_stage();
        compute(lds + (kt & 1) * STAGE, yes{}, kstep_of(kt + 1), (kt + 1) & 1);
      }
      publish_stage();
      compute(lds + (kt & 1) * STAGE, no{}, KStep{}, 0);
    } else {
      // three stages, two K-steps of DMA in flight across each barrier: a
      // counted vmcnt retires stage kt only (the IPW loads of stage kt+1 stay
      // in flight), a raw s_barrier publishes it (no __syncthreads: its fence
      // would drain vmcnt to 0), then stage kt+2 is issued into the buffer
      // every wave finished reading in step kt-1 (its ds_reads retired by the
      // lgkmcnt(0) before this barrier).
      {
        const KStep a = kstep_of(0);
#pragma unroll
        for (int i = 0; i < IPW; ++i) piece(i, a, 0);
      }
      if (nk > 1) {
        const KStep a = kstep_of(1);
#pragma unroll
        for (int i = 0; i < IPW; ++i) piece(i, a, 1);
      }
      int cur = 0;
      for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(IPW) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + 2 < nk) {
          const KStep a = kstep_of(kt + 2);
          const int st = cur == 0 ? 2 : cur - 1;
#pragma unroll
          for (int i = 0; i < IPW; ++i) piece(i, a, st);
        }
        compute(lds + cur * STAGE, no{}, KStep{}, 0);
        cur = cur == 2 ? 0 : cur + 1;
      }
    }
    __syncthreads();  // every wave's last fragment reads are done: the stages become the C tile
    epi.begin(p, tm);
    bf16_t* Cs = reinterpret_cast<bf16_t*>(lds);
    acc_to_lds<TN, TM>(acc, Cs, LDC, wm0, wn0, lane);
    __syncthreads();
    epi.rows(p, Cs, tm);
    __syncthreads();  // the next tile's DMA overwrites Cs
  }
  epi.finish(p, reinterpret_cast<float*>(lds), b, gm < tiles_m);
}

template <int BM, int BN, int WM, int WN, int GATHER, int EPI, int MINB, int STAGES, int BPC>
hipError_t launch(const GemmParams& p, hipStream_t s) {
  GemmParams q = p;
  if constexpr (GATHER == G_DGRAD2) {  // four classes of ceil(mc / BM) tiles each
    q.mc_pad = (p.mc + BM - 1) / BM * BM;
    q.M = 4 * q.mc_pad;
  }
  const int tiles_m = (q.M + BM - 1) / BM;
  const int tiles_n = q.N / BN;
  // one round of resident blocks (KDL_TUNE igemm_rounds > 1: that many rounds -- shorter
  // per-block tile lists, for the two-stream step's contention; A/B knob)
  static const int rounds = [] { const int v = tune_int("igemm_rounds", 1); return v < 1 ? 1 : v; }();
  const int target = 256 * BPC * rounds;
  int GM = (target + tiles_n - 1) / tiles_n;
  if (GM > tiles_m) GM = tiles_m;
  while ((GM * tiles_n) % 8) ++GM;
  hipLaunchKernelGGL((igemm_kernel<BM, BN, WM, WN, GATHER, EPI, MINB, STAGES>), dim3(GM * tiles_n), dim3(64 * WM * WN),
                     0, s, q, GM, tiles_m, tiles_n);
  return hipGetLastError();
}

// MINB: the launch bound's minimum waves per SIMD (register budget); BPC:
// resident blocks per CU the persistent grid is sized for.
template <int BM, int BN, int WM, int WN, int GATHER, int MINB, int STAGES, int BPC>
hipError_t dispatch_epi(const GemmParams& p, int epi, hipStream_t s) {
  switch (epi) {
    case EPI_PLAIN: return launch<BM, BN, WM, WN, GATHER, EPI_PLAIN, MINB, STAGES, BPC>(p, s);
    case EPI_STATS: return launch<BM, BN, WM, WN, GATHER, EPI_STATS, MINB, STAGES, BPC>(p, s);
    case EPI_MASKX: return launch<BM, BN, WM, WN, GATHER, EPI_MASKX, MINB, STAGES, BPC>(p, s);
  }
  if constexpr (GATHER == G_DENSE) {
    switch (epi) {
      case EPI_RESBITS: return launch<BM, BN, WM, WN, GATHER, EPI_RESBITS, MINB, STAGES, BPC>(p, s);
      case EPI_RES: return launch<BM, BN, WM, WN, GATHER, EPI_RES, MINB, STAGES, BPC>(p, s);
      case EPI_BIAS: return launch<BM, BN, WM, WN, GATHER, EPI_BIAS, MINB, STAGES, BPC>(p, s);
      case EPI_BIAS_RELU: return launch<BM, BN, WM, WN, GATHER, EPI_BIAS_RELU, MINB, STAGES, BPC>(p, s);
    }
  }
  return hipErrorInvalidValue;
}

template <int BM, int BN, int WM, int WN, int MINB, int STAGES = 2, int BPC = MINB>
hipError_t dispatch_gather(const GemmParams& p, int epi, int gather, hipStream_t s) {
  switch (gather) {
    case G_DENSE: return dispatch_epi<BM, BN, WM, WN, G_DENSE, MINB, STAGES, BPC>(p, epi, s);
    case G_STRIDED: return dispatch_epi<BM, BN, WM, WN, G_STRIDED, MINB, STAGES, BPC>(p, epi, s);
    case G_CONV3: return dispatch_epi<BM, BN, WM, WN, G_CONV3, MINB, STAGES, BPC>(p, epi, s);
    case G_DGRAD2:
      if constexpr (STAGES == 2) return dispatch_epi<BM, BN, WM, WN, G_DGRAD2, MINB, STAGES, BPC>(p, epi, s);
      break;
  }
  return hipErrorInvalidValue;
}

}  // namespace

// Tile configs: 0 = 256x256 (8 waves, 128x64 wave tiles, 1 block/CU);
// 1 = 256x128 (8 waves, 64x64); 2 = 128x128 (4 waves, 64x64, 2 blocks/CU);
// 3 = 256x64 (4 waves, 64x64, 2 blocks/CU); 4 = 256x128 with three stages
// (two K-steps of DMA in flight, counted vmcnt + raw barrier, 144 KiB).
// Measured on the ResNet-50 shapes (profiles/r02_igemm_small_blocks_ab.jsonl,
// docs/perf_notes.md): three stages tie two at one block per CU (4 vs 1) and
// lose badly where they cost the second resident block (128x128 / 256x64 at
// 96-120 KiB: 1.6-1.7x slower); smaller independent blocks (128x64, 64x64,
// 64x128 at 3-4 blocks/CU) lose 15-60 %.  Operand delivery into LDS, not
// latency, bounds these kernels (~7-10 TB/s of L2->LDS traffic chip-wide).
namespace {
int g_forced_cfg = tune_int("igemm_cfg", -1);
}  // namespace

void set_igemm_cfg(int cfg) { g_forced_cfg = cfg; }

namespace gemm {
bool g_forced_cfg_unset() { return g_forced_cfg < 0; }
}  // namespace gemm

namespace gemm {
int igemm_pick(int M, int N, int K) {
  const int forced = g_forced_cfg;
  if (forced >= 0 && forced <= 4) {
    const int bn = forced == 0 ? 256 : forced == 3 ? 64 : 128;
    if (N % bn == 0) return forced;
  }
  // measured on the ResNet-50 b256 shapes (profiles/r02_igemm_v1_vs_reg_vs_miopen.jsonl):
  // 256x256 wins at N = 256 (fewest operand bytes per MFMA), 128x128 at two
  // blocks per CU elsewhere (more resident waves, more tiles to fill 256 CUs)
  (void)M; (void)K;
  static const int n256 = tune_int("igemm_n256", 0);  // A/B: the tile of the N = 256 (stage-3) GEMMs
  if (N == 256) return n256 >= 0 && n256 <= 4 ? n256 : 0;
  if (N % 128 == 0) return 2;
  return 3;
}
}  // namespace gemm

namespace gemm {
hipError_t igemm(const GemmParams& p_in, int epi, int gather, int cfg, hipStream_t s) {
  // timing-only: price one operand's traffic (outputs are wrong): 1 drops A's loads, 2 B's
  static const int price = tune_int("igemm_price", 0);
  GemmParams p = p_in;
  p.price_drop = price;
  if (p.K % IBK || p.M <= 0) return hipErrorInvalidValue;
  const int lda = (gather == G_CONV3 || gather == G_DGRAD2) ? p.Cin : p.K;
  if (p.a_rows * lda * 2 >= (int64_t(1) << 31) || static_cast<int64_t>(p.N) * p.K * 2 >= (int64_t(1) << 31))
    return hipErrorInvalidValue;  // 32-bit buffer offsets
  // The stride-2 data gradient with the MASKX epilogue on the 256x256 tile
  // computes wrong rows at the ResNet-50 b256 shape (a zero dy gives nonzero dx
  // and 8 % off BN sums, 14x14 -> 28x28 x 256; scripts/maskx_probe.py) while the
  // PLAIN epilogue, the other tiles and G_CONV3 / dense MASKX on this tile are
  // exact -- the variant is the one that spills both VGPRs and SGPRs around the
  // LDS-DMA loads.  It runs on 256x128 tiles instead.
  if (gather == G_DGRAD2 && epi == EPI_MASKX && cfg == 0) cfg = 1;
  switch (cfg) {
    case 0: if (p.N % 256) break; return dispatch_gather<256, 256, 2, 4, 1>(p, epi, gather, s);
    case 1: if (p.N % 128) break; return dispatch_gather<256, 128, 4, 2, 1>(p, epi, gather, s);
    case 2: if (p.N % 128) break; return dispatch_gather<128, 128, 2, 2, 2>(p, epi, gather, s);
    case 3: if (p.N % 64) break; return dispatch_gather<256, 64, 4, 1, 2>(p, epi, gather, s);
    case 4: if (p.N % 128) break; return dispatch_gather<256, 128, 4, 2, 1, 3>(p, epi, gather, s);
  }
  return hipErrorInvalidValue;
}
}  // namespace gemm

}  // namespace kdl
