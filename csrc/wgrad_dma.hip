// Conv weight gradients on the LDS-DMA operand pipeline (gfx950).
//
//   dW[n][k] = sum_m G[m][n] * pro(A)[m][k]     (split over m, fp32 slabs)
//
// G is the layer's output gradient [M][N] and A its (row-gathered: strided 1x1,
// or 3x3 pad-1 per tap) input, both NHWC rows, so the reduction index m is the
// ROW index of both operands.  The register-staged kernel (csrc/conv1x1.hip
// wgrad1x1_kernel) transposes every staged 8x8 block in registers (v_perm) to
// give the MFMA its k-contiguous fragments; here the operands go HBM -> LDS
// untouched by `buffer_load_dwordx4 ... lds` (padding taps and rows past M are
// out-of-bounds loads = zeros) and the transpose happens in the LDS read:
// `ds_read_b64_tr_b16` hands each lane 4 consecutive rows of one column, two of
// them make the 8-element fragment of v_mfma_f32_32x32x16_bf16.
//
// LDS image per operand: 64-column panels of [64 rows][128 B], 16-B chunk c of
// row r at chunk position c ^ (((r >> 1) & 1) * 4) -- for the transposed read
// (4 rows x 32 B per 16-lane group, 8 rows x 32 B per 32-lane bank cycle) every
// bank is hit once.  The DMA writes lane-linear, so the swizzle is applied to
// the source address.  Two stages, one barrier per 64-row step (the next
// step's DMA is issued before the current step's MFMAs).
//
// The optional BN+ReLU prologue of A (``pro``: conv3's input is the
// un-normalised conv2 output) is applied to the A fragments after the read:
// each lane's fragment is one input channel, so its (scale, shift) pair is a
// per-lane constant.  Rows past the end of the M range are zeroed after the
// prologue (relu(shift) of a zero row is not zero).
//
// The reference has no kernels; this serves the PyTorchJob
// ResNet-50 worker (BASELINE.json config 2).
#include "common.h"
#include "gemm_epi.h"
#include "kdl_api.h"
#include "lds_dma.h"

#include <type_traits>

namespace kdl {
namespace gemm {
namespace {

using lds_dma::dma16;
using lds_dma::i32x4_t;
using lds_dma::kOOB;
using lds_dma::lds_void_t;
using lds_dma::publish_stage;
using lds_dma::rsrc_words;
typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;

constexpr int MK = 64;  // rows (m) per stage

// (device-pass guard: referenced in the host pass this builtin makes clang
// drop the kernel's host stub)
__device__ __forceinline__ v4s_t tr_read(const char* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(p));
#else
  return v4s_t{};
#endif
}

__device__ __forceinline__ bf16x8_t frag8(v4s_t lo, v4s_t hi) {
  const uint2 a = __builtin_bit_cast(uint2, lo), b = __builtin_bit_cast(uint2, hi);
  return __builtin_bit_cast(bf16x8_t, make_uint4(a.x, a.y, b.x, b.y));
}

// WN x WK waves: 2 x 2 (4 waves, 2 blocks/CU) for tiles up to 128 x 128; 2 x 4
// (8 waves of 128 x 64, 1 block/CU, 128 KiB) for 256 x 256 -- half the LDS-DMA
// bytes per MFMA of a 128 x 128 tile (the operand stream bounds these kernels).
//
// BWDG: G is the output of a BN-backward apply that was never written, G' =
// k[n] G + c1[n] gx + c0[n] (WgParams::gx / gcoef): gx is staged by the same
// DMA as G into PN panels of its own, read with G's transposed reads, and
// combined per fragment -- each lane's G fragment is ONE output channel n, so
// (k, c1, c0) are per-lane constants, exactly as the A prologue's (scale, shift).
template <int TN_, int TK_, int GATHER, bool PRO, int WN = 2, int WK = 2, bool BWDG = false>
__global__ __launch_bounds__(64 * WN * WK, (WN * WK == 4) ? 2 : 1) void wgrad_dma_kernel(WgParams p) {
  constexpr int NW = WN * WK;
  constexpr int PN = TN_ / 64, PK = TK_ / 64;  // 64-column panels per operand
  constexpr int PX = BWDG ? PN : 0;            // gx panels (BWDG)
  constexpr int PANEL = MK * 128;              // bytes per panel per stage
  constexpr int STAGE = (PN + PK + PX) * PANEL;
  static_assert((PN + PK + PX) * (MK / 8) % NW == 0, "every wave issues the same DMA count");
  constexpr int IPW = (PN + PK + PX) * (MK / 8) / NW;  // 1-KiB DMA instructions per wave per stage
  constexpr int TN = TN_ / WN / 32, TK = TK_ / WK / 32;  // 32x32 MFMA blocks per wave
  static_assert(TN >= 1 && TK >= 1, "wave tile = whole 32x32 MFMA blocks");
  __shared__ __attribute__((aligned(1024))) char lds[2 * STAGE];

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  // XCD-aware order (bijective): the tiles of one M-split are consecutive on one XCD
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int xq = nblk >> 3, xr = nblk & 7, xcd = bid & 7;
  const int wid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (bid >> 3);
  const int tiles = (p.N / TN_) * p.tiles_k;
  const int split = wid / tiles, tile = wid - split * tiles;
  const int tn = tile / p.tiles_k, tk = tile - tn * p.tiles_k;
  const int n0 = tn * TN_, k0 = tk * TK_;
  const int mbeg = split * p.rps;
  const int mend = min(p.M, mbeg + p.rps);
  // 3x3: this tile's K range lies in one tap (TK_ | cin)
  const int tap = GATHER == G_CONV3 ? k0 / p.cin : 0;
  const int kin0 = k0 - tap * p.cin;
  const int tr3 = tap / 3, tq3 = tap - 3 * (tap / 3);
  const int lda = GATHER == G_CONV3 ? p.cin : p.K;
  const int acol0 = GATHER == G_CONV3 ? kin0 : k0;

  const i32x4_t wG = rsrc_words(p.G, static_cast<uint32_t>(static_cast<int64_t>(p.M) * p.N * 2));
  const i32x4_t wA = rsrc_words(p.A, static_cast<uint32_t>(p.a_rows * lda * 2));
  const i32x4_t wX = rsrc_words(BWDG ? p.gx : p.G, static_cast<uint32_t>(static_cast<int64_t>(p.M) * p.N * 2));

  // DMA piece i of this wave: panel kind (0 G, 1 A, 2 gx -- wave-uniform), the
  // lane's row within the 64-row step and its 16-B chunk's byte offset in the row
  const int lrow = lane >> 3;
  uint32_t gcol[IPW];
  int prow[IPW], pkind[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int g = wave * IPW + i;
    const int panel = g / (MK / 8), r = 8 * (g % (MK / 8)) + lrow;
    const int c = (lane & 7) ^ (((r >> 1) & 1) * 4);
    prow[i] = r;
    pkind[i] = panel < PN ? 0 : panel < PN + PK ? 1 : 2;
    gcol[i] = panel < PN        ? static_cast<uint32_t>((n0 + 64 * panel + 8 * c) * 2)
              : panel < PN + PK ? static_cast<uint32_t>((acol0 + 64 * (panel - PN) + 8 * c) * 2)
                                : static_cast<uint32_t>((n0 + 64 * (panel - PN - PK) + 8 * c) * 2);
  }

  // one piece of the step at rows m0.. into `stage` (rows past M: an explicit
  // out-of-range voffset -- the range check covers the VGPR offset)
  auto piece = [&](int i, int m0, int stage) {
    const int g = wave * IPW + i;
    lds_void_t* dst = (lds_void_t*)(lds + stage * STAGE + g * 1024);
    const int m = m0 + prow[i];
    if (pkind[i] != 1) {
      dma16(pkind[i] == 0 ? wG : wX, dst, m < p.M ? static_cast<uint32_t>(m * p.N * 2) + gcol[i] : kOOB, 0);
    } else if constexpr (GATHER == G_DENSE) {
      dma16(wA, dst, m < p.M ? static_cast<uint32_t>(m * p.K * 2) + gcol[i] : kOOB, 0);
    } else {
      uint32_t off = kOOB;
      if (m < p.M) {
        const int hw = p.Hout * p.Wout;
        const int nimg = static_cast<int>(__umulhi(static_cast<uint32_t>(m), p.mg_hw));
        const int rem = m - nimg * hw;
        const int oh = static_cast<int>(__umulhi(static_cast<uint32_t>(rem), p.mg_w));
        const int ow = rem - oh * p.Wout;
        if constexpr (GATHER == G_STRIDED) {
          off = static_cast<uint32_t>(((nimg * p.Hin + oh * p.stride) * p.Win + ow * p.stride) * lda * 2) + gcol[i];
        } else {
          const int ih = oh * p.stride + tr3 - 1, iw = ow * p.stride + tq3 - 1;
          if (static_cast<unsigned>(ih) < static_cast<unsigned>(p.Hin) &&
              static_cast<unsigned>(iw) < static_cast<unsigned>(p.Win))
            off = static_cast<uint32_t>(((nimg * p.Hin + ih) * p.Win + iw) * lda * 2) + gcol[i];
        }
      }
      dma16(wA, dst, off, 0);
    }
  };
  // transposed fragment reads: lane (group g = lane >> 4, q = (lane & 15) >> 2,
  // pp = lane & 3) reads rows 16s + 8(g >> 1) + q (+4) at column
  // 16(g & 1) + 4pp of its 32-column fragment
  const int grp = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int swz = ((q >> 1) & 1) * 4;
  const int rowb = (8 * (grp >> 1) + q) * 128;
  auto frag_off = [&](int col32) {  // col32: first column of the fragment within its panel (0 or 32)
    const int chunk = (col32 + 16 * (grp & 1) + 4 * pp) >> 3;
    return rowb + 16 * (chunk ^ swz) + 8 * (pp & 1);
  };
  const int wn0 = (wave / WK) * (TN_ / WN), wk0 = (wave % WK) * (TK_ / WK);
  int goff[TN], aoff[TK];
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = wn0 + 32 * i;
    goff[i] = (n / 64) * PANEL + frag_off(n % 64);
  }
#pragma unroll
  for (int j = 0; j < TK; ++j) {
    const int k = wk0 + 32 * j;
    aoff[j] = (PN + k / 64) * PANEL + frag_off(k % 64);
  }
  // prologue coefficients: this lane's A column is channel acol0 + wk0 + 32j + (lane & 15) + 16(grp & 1)
  float psc[TK], psf[TK];
#pragma unroll
  for (int j = 0; j < TK; ++j) {
    psc[j] = 1.f;
    psf[j] = 0.f;
    if constexpr (PRO) {
      const int kc = acol0 + wk0 + 32 * j + (lane & 31);
      psc[j] = p.pro[kc];
      psf[j] = p.pro[lda + kc];
    }
  }
  (void)psc; (void)psf;
  // BWDG coefficients: this lane's G row is channel n0 + wn0 + 32i + (lane & 31)
  float gk[TN], gc1[TN], gc0[TN];
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    gk[i] = 1.f;
    gc1[i] = 0.f;
    gc0[i] = 0.f;
    if constexpr (BWDG) {
      const int n = n0 + wn0 + 32 * i + (lane & 31);
      gk[i] = p.gcoef[n];
      gc1[i] = p.gcoef[p.N + n];
      gc0[i] = p.gcoef[2 * p.N + n];
    }
  }
  (void)gk; (void)gc1; (void)gc0;

  f32x16_t acc[TN][TK];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j) acc[i][j] = f32x16_t{};

  // One 64-row step on stage S: raw fragments double-buffered (substep s + 1's
  // transposed reads issued before substep s's MFMAs, its prologue applied at
  // the top of substep s + 1), and with ISSUE the next step's DMA pieces spread
  // over the first half of the MFMAs -- their address math and issue run in the
  // MFMA shadow, not in a burst after the barrier (csrc/igemm.hip, round 6).
  constexpr int NMF = 4 * TN * TK;
  // spread the pieces only where there are at least two MFMAs per piece; the
  // small, bandwidth-bound tiles (64-wide at K or N = 64: 8 MFMAs per wave
  // for 6 pieces) keep the burst right after the barrier -- spreading their
  // loads cost 8-14 % there (profiles/r06_wgrad_probe.txt)
  constexpr int SPAN = NMF < 2 * IPW ? 1 : (NMF / 2 > IPW ? NMF / 2 : IPW);
  auto raw = [&](const char* S, int s, bf16x8_t (&gf)[TN], bf16x8_t (&xf)[TN], bf16x8_t (&af)[TK]) {
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const char* b = S + goff[i] + s * 16 * 128;
      gf[i] = frag8(tr_read(b), tr_read(b + 4 * 128));
      if constexpr (BWDG) {
        const char* bx = b + (PN + PK) * PANEL;
        xf[i] = frag8(tr_read(bx), tr_read(bx + 4 * 128));
      }
    }
#pragma unroll
    for (int j = 0; j < TK; ++j) {
      const char* b = S + aoff[j] + s * 16 * 128;
      af[j] = frag8(tr_read(b), tr_read(b + 4 * 128));
    }
  };
  auto prologue = [&](int m0, int s, bool tail, bf16x8_t (&gf)[TN], const bf16x8_t (&xf)[TN], bf16x8_t (&af)[TK]) {
    (void)m0; (void)s; (void)tail; (void)gf; (void)xf; (void)af;
    const int mrow = m0 + 16 * s + 8 * (lane >> 5);
    (void)mrow;
    if constexpr (BWDG) {
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        float f[8], x[8];
        unpack8(__builtin_bit_cast(uint4, gf[i]), f);
        unpack8(__builtin_bit_cast(uint4, xf[i]), x);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float o = fmaf(gk[i], f[e], fmaf(gc1[i], x[e], gc0[i]));  // bn_bwd_apply_kernel's nesting
          f[e] = (!tail || mrow + e < mend) ? o : 0.f;
        }
        gf[i] = __builtin_bit_cast(bf16x8_t, pack8(f));
      }
    }
    if constexpr (PRO) {
#pragma unroll
      for (int j = 0; j < TK; ++j) {
        float f[8];
        unpack8(__builtin_bit_cast(uint4, af[j]), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float o = fmaf(f[e], psc[j], psf[j]);
          f[e] = (o > 0.f && (!tail || mrow + e < mend)) ? o : 0.f;
        }
        af[j] = __builtin_bit_cast(bf16x8_t, pack8(f));
      }
    }
  };
  auto step = [&](const char* S, int m0, auto issue_tag, int next_stage) {
    constexpr bool ISSUE = decltype(issue_tag)::value;
    const bool tail = (PRO || BWDG) && m0 + MK > mend;  // rows past the range: zero after the prologue
    bf16x8_t gf[2][TN], xf[2][TN], af[2][TK];
    raw(S, 0, gf[0], xf[0], af[0]);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      prologue(m0, s, tail, gf[s & 1], xf[s & 1], af[s & 1]);
      if (s < 3) raw(S, s + 1, gf[(s + 1) & 1], xf[(s + 1) & 1], af[(s + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j) {
          const int mi = (s * TN + i) * TK + j;
          if constexpr (ISSUE && SPAN == 1) {
            if (mi == 0) {
#pragma unroll
              for (int pi = 0; pi < IPW; ++pi) piece(pi, m0 + MK, next_stage);
            }
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gf[s & 1][i], af[s & 1][j], acc[i][j], 0, 0, 0);
          if constexpr (ISSUE && SPAN > 1) {
#pragma unroll
            for (int pi = 0; pi < IPW; ++pi)
              if (pi * SPAN / IPW == mi) piece(pi, m0 + MK, next_stage);
          }
        }
    }
  };
  using yes = std::integral_constant<bool, true>;
  using no = std::integral_constant<bool, false>;
  if (mbeg < mend) {
#pragma unroll
    for (int i = 0; i < IPW; ++i) piece(i, mbeg, 0);
    int st = 0, m0 = mbeg;
    // the last step is peeled (no DMA): one loop body, the accumulators keep their registers
    for (; m0 + MK < mend; m0 += MK) {
      publish_stage();
      step(lds + st * STAGE, m0, yes{}, st ^ 1);
      st ^= 1;
    }
    publish_stage();
    step(lds + st * STAGE, m0, no{}, 0);
  }
  // D[n][k]: column k = lane & 31, rows n = (r&3) + 8(r>>2) + 4(lane>>5); this
  // split's partial tile goes to its own fp32 slab (reduced in a fixed order)
  float* slab = p.dw32 + static_cast<int64_t>(split) * p.N * p.K;
  const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        const int k = k0 + wk0 + j * 32 + fr;
        slab_store(slab + static_cast<int64_t>(n) * p.K + k, acc[i][j][r]);
      }
}

template <int TN_, int TK_, int WN = 2, int WK = 2>
void launch(const WgParams& p, int grid, hipStream_t s) {
#define WGD_LAUNCH(G, P) \
  hipLaunchKernelGGL((wgrad_dma_kernel<TN_, TK_, G, P, WN, WK>), dim3(grid), dim3(64 * WN * WK), 0, s, p)
  if (p.pro) {
    if (p.mode == G_CONV3) WGD_LAUNCH(G_CONV3, true);
    else if (p.mode == G_STRIDED) WGD_LAUNCH(G_STRIDED, true);
    else WGD_LAUNCH(G_DENSE, true);
  } else {
    if (p.mode == G_CONV3) WGD_LAUNCH(G_CONV3, false);
    else if (p.mode == G_STRIDED) WGD_LAUNCH(G_STRIDED, false);
    else WGD_LAUNCH(G_DENSE, false);
  }
#undef WGD_LAUNCH
}

// G prologue (BWDG): 1x1 weight gradients only (dense or strided A rows)
template <int TN_, int TK_, int WN, int WK>
void launch_bwdg(const WgParams& p, int grid, hipStream_t s) {
#define WGD_LAUNCH_B(G, P) \
  hipLaunchKernelGGL((wgrad_dma_kernel<TN_, TK_, G, P, WN, WK, true>), dim3(grid), dim3(64 * WN * WK), 0, s, p)
  if (p.mode == G_STRIDED) WGD_LAUNCH_B(G_STRIDED, false);  // (strided rows: the downsample conv, no A prologue)
  else if (p.pro) WGD_LAUNCH_B(G_DENSE, true);               // conv3: B2 + ReLU recomputed on A as well
  else WGD_LAUNCH_B(G_DENSE, false);
#undef WGD_LAUNCH_B
}

}  // namespace

hipError_t wgrad_dma(const WgParams& p, int nsplit, int tn, int tk, hipStream_t s) {
  const int lda = p.mode == G_CONV3 ? p.cin : p.K;
  // (a prologue over zero-padded taps would need the padding re-zeroed after it:
  // that combination stays on the register-staged kernel)
  if ((p.pro && p.mode == G_CONV3) || p.rps % MK || p.N % tn || p.K % tk || (p.mode == G_CONV3 && p.cin % tk) ||
      static_cast<int64_t>(p.M) * p.N * 2 >= (int64_t(1) << 31) || p.a_rows * lda * 2 >= (int64_t(1) << 31))
    return hipErrorInvalidValue;
  if (p.mode != G_DENSE &&
      static_cast<uint64_t>(p.M) * static_cast<uint64_t>(p.Hout * p.Wout) >= (uint64_t(1) << 32))
    return hipErrorInvalidValue;  // magic-number division range
  const int grid = nsplit * (p.N / tn) * (p.K / tk);
  if (p.gx) {  // G prologue: the wgrad_tiles(bwd) configs, gx panels beside G's
    if (!p.gcoef || p.mode == G_CONV3 || (p.pro && p.mode != G_DENSE)) return hipErrorInvalidValue;
    if (tn == 128 && tk == 256) launch_bwdg<128, 256, 2, 4>(p, grid, s);
    else if (tn == 128 && tk == 128) launch_bwdg<128, 128, 2, 4>(p, grid, s);
    else if (tn == 128 && tk == 64) launch_bwdg<128, 64, 4, 2>(p, grid, s);
    else if (tn == 64 && tk == 256) launch_bwdg<64, 256, 2, 4>(p, grid, s);
    else if (tn == 64 && tk == 128) launch_bwdg<64, 128, 2, 4>(p, grid, s);
    else if (tn == 64 && tk == 64) launch_bwdg<64, 64, 2, 2>(p, grid, s);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (tn == 256 && tk == 256) launch<256, 256, 2, 4>(p, grid, s);
  else if (tn == 128 && tk == 128) launch<128, 128>(p, grid, s);
  else if (tn == 128) launch<128, 64>(p, grid, s);
  else if (tk == 128) launch<64, 128>(p, grid, s);
  else launch<64, 64>(p, grid, s);
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace kdl
