// 1x1 convolutions of the NHWC ResNet bottleneck as MFMA GEMMs with the
// neighbouring BatchNorm work fused into their prologue / epilogue (gfx950).
//
// At batch 256 every 1x1 conv of ResNet-50 is HBM-bound on MI355X (K, N <=
// 2048, M = N*H*W up to 802,816 rows: ~64-400 FLOP per byte moved), so the
// lever is not MFMA rate but bytes: each fusion below deletes a whole pass
// over an activation tensor that the unfused step (conv -> BN stats -> BN
// apply -> conv ...) pays for separately.
//
//   gemm1x1 (forward and data-gradient):   C[M, N] = pro(A)[M, K] . B[N, K]^T
//     forward:  A = activations (row-gathered for stride-2 1x1 convs),
//               B = conv weight [Cout, Cin];
//     dgrad:    A = output gradient, B = W^T [Cin, Cout] (transposed copy).
//     prologue  PRO:      A <- relu(A * scale[k] + shift[k])  -- the BN+ReLU
//                         of the previous layer applied while staging A, so
//                         its output is never written to HBM;
//     epilogue  STATS:    per-output-channel shifted sums sum(y - s),
//                         sum((y - s)^2) of the bf16 output -> the BN
//                         forward-stats replicas (no separate stats pass);
//               MASKX:    dgrad of the layer after a BN+ReLU: g' = g *
//                         [x*scale + shift > 0] (mask recomputed from the
//                         BN input x), plus the BN backward sums sum(g'),
//                         sum(g' (x - mean)) (no separate reduce pass);
//               RESBITS:  dgrad of a bottleneck's first conv: g = dgrad +
//                         d(identity) (optionally stride-gathered from the
//                         downsample branch), masked by the previous block's
//                         packed 1-bit ReLU mask, plus the previous block's
//                         bn3 (and downsample BN) backward sums: this
//                         replaces autograd's residual-gradient add kernel
//                         AND the bn3 reduce pass;
//               RES:      g = dgrad + d(identity), no mask (network stem).
//   wgrad1x1:   dW[N, K] = sum_m G[m, N]^T pro(A)[m, K]   (split over M, fp32
//               atomics from the accumulators; a cast kernel writes the bf16
//               gradient and re-zeroes the fp32 accumulator).
//
// Tiling (gemm1x1): 256 threads = 4 waves, tile 128 (M) x BN (N in {64,
// 128}) x 64 (K).  The MFMA is v_mfma_f32_32x32x16_bf16 issued as D = W . X^T
// (weight fragment as the A operand), so a lane's accumulator registers hold
// 4 consecutive OUTPUT CHANNELS of one output row: the epilogue packs them to
// 8-byte LDS writes, and the tile is read back row-wise as 16-byte vectors
// (one thread = 8 channels of one row), which is the layout both the global
// store and the per-channel reductions want.  LDS rows are padded to 72 bf16
// (144 B): the 32 rows a fragment read touches land on distinct 16-B slots.
// Register-staged double buffering; the next tile's first K-step is fetched
// while the current tile's last K-step computes.  Blocks are persistent over
// M tiles (reduction atomics once per block, not per tile) and the block ->
// (tile_n, M-sequence) map is XCD-aware: the tile_n siblings that re-read one
// A panel are consecutive on the same XCD (shared L2).
//
// The reference has no kernels; these serve the PyTorchJob
// ResNet-50 worker (BASELINE.json config 2).
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "gemm_epi.h"
#include "kdl_api.h"
#include "tune.h"

namespace kdl {
namespace {

using namespace gemm;  // GemmParams, EPI_*, G_*, fragment types, epilogue (csrc/gemm_epi.h)

constexpr int kThreads = 256;
constexpr int BK = 64;
// PRO_BWD coefficient table capacity (channels of K) per tile width: 128-wide
// tiles stay within 80 KiB of LDS (two blocks per CU) up to K = 512, 64-wide
// tiles up to K = 2048 (the widest ResNet-50 data-gradient K)
__host__ __device__ constexpr int bwd_kmax(int bn) { return bn >= 128 ? 512 : 2048; }

// PRO: 0 none, PRO_FWD = BN+ReLU of the previous layer, PRO_BWD = BN-backward
// apply (GemmParams::bx / bcoef; dense rows only)
// PRO_RES = the previous block's closing BN + residual + ReLU, relu(A * scale +
// shift + R) with R = GemmParams::bx, written through (the blocks of output
// tile 0) as the block output and its packed ReLU mask (GemmParams::obits):
// the apply pass feeding the next block's conv1, fused into that conv
// PRO_RES2 = the same after a downsample block: R = bx * scale_d + shift_d (the
// downsample branch's BN), bn_fwd_apply_dual's expression
enum { PRO_NONE = 0, PRO_FWD = 1, PRO_BWD = 2, PRO_RES = 5, PRO_RES2 = 6 };

template <int BM, int BN, int MINB, int PRO, int GATHER, int EPI, int KBK = BK>
__global__ __launch_bounds__(kThreads, MINB) void gemm1x1_kernel(GemmParams p, int GM, int tiles_m, int tiles_n) {
  static_assert((PRO != PRO_BWD && PRO != PRO_RES && PRO != PRO_RES2) || GATHER == G_DENSE,
                "the two-input prologues read dense rows");
  constexpr bool TWO_IN = PRO == PRO_BWD || PRO == PRO_RES || PRO == PRO_RES2;  // A and a second row operand bx
  // [2 buffers][BM + BN rows][KBK]; after the K loop one buffer doubles as the
  // [BM][BN + 8] output tile and finally as the reduction scratch.  Buffers are
  // spaced as padded rows (LDK) so that output tile fits one of them as before.
  constexpr int LDK = KBK + 8;
  constexpr int CPRK = KBK / 8; // 16-B chunks per staged row
  constexpr int kBuf = (BM + BN) * LDK;
  // Staged rows are unpadded with the 16-B chunk index XORed by (row / RG): the
  // 16 lanes of one staging store (RG rows x CPRK chunks) and the 16 rows of one
  // MFMA fragment read both land on distinct bank groups.  The padded layout
  // (row stride KBK + 8) left the stores 2-way conflicted: the 32-deep-K conv3
  // forward ran 131 % LDS conflict cycles per LDS cycle, 57 % swizzled, and the
  // step 13,761-13,793 -> 13,810-13,879 img/s (profiles/r05_gemm_swizzle_ab.txt).
  constexpr int RG = 16 / CPRK;
  constexpr int ldk = KBK;
  auto soff = [](int row, int chunk) { return row * KBK + ((chunk ^ ((row / RG) & (CPRK - 1))) << 3); };
  // PRO_BWD: the backward coefficients k | c1 | c0 of every K channel, staged
  // once per block behind the operand buffers (one __shared__ array: a second
  // one can make hipcc drain the pipeline, cdna_hip_programming.md §5 item 4a)
  constexpr int KT = TWO_IN ? bwd_kmax(BN) : 0;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * kBuf + 6 * KT];
  float* coef_lds = reinterpret_cast<float*>(lds + 2 * kBuf);
  (void)coef_lds;
  constexpr int WN = (BN >= 64 && BM >= 64) ? 2 : 1;  // waves along N
  constexpr int WM = 4 / WN;                           // waves along M
  static_assert(BM % (WM * 32) == 0 && BN % (WN * 32) == 0, "wave tile must be whole 32x32 MFMA blocks");
  constexpr int WTM = BM / WM;           // wave tile (M)
  constexpr int WTN = BN / WN;           // wave tile (N) = 64
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int A_CH = BM * CPRK / kThreads;  // 16-B chunks per thread per K-step
  constexpr int B_CH = BN * CPRK / kThreads;
  constexpr int LDC = BN + 8;
  // Small K-steps (KBK = 32): the [BM][LDC] output tile does not fit one stage
  // buffer, so the next tile's first K-step stays in registers through the
  // epilogue (which then owns both buffers) and is staged after it.
  constexpr bool SPLIT_C = BM * LDC > kBuf;

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int nblk = gridDim.x;
  const int b = blockIdx.x;
  const int q = (b & 7) * (nblk >> 3) + (b >> 3);  // nblk % 8 == 0 (host)
  const int tile_n = q % tiles_n;
  const int gm = q / tiles_n;
  const int n0 = tile_n * BN;
  const int K = p.K, M = p.M, N = p.N;
  const int nk = K / KBK;
  const int wm0 = (wave / WN) * WTM, wn0 = (wave % WN) * WTN;

  // staging coordinates (fixed per thread)
  int a_row[A_CH], a_kc[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int c = t + i * kThreads;
    a_row[i] = c / CPRK;
    a_kc[i] = (c % CPRK) * 8;
  }
  int64_t a_off[A_CH];
  // 3x3 implicit GEMM: per A chunk the image base row and the top-left input
  // coordinate of its output pixel; ``ra_ok`` = chunks whose tap is inside the
  // image for the K-step held in ``ra`` (padding taps stage as zeros)
  int a_base[A_CH], a_ih[A_CH], a_iw[A_CH];
  uint32_t ra_ok = 0;
  (void)a_base; (void)a_ih; (void)a_iw; (void)ra_ok;
  uint4 ra[A_CH], rb[B_CH];
  // all A chunks of a thread share one 8-channel k-chunk ((t + i*256) & 7 == t & 7)
  float psc[8], psf[8];
  (void)psc; (void)psf;
  // PRO_BWD: the BN input rows beside A, the staged K-step's k0 and the
  // chunks whose row is < M (write-through of A')
  uint4 rx[TWO_IN ? A_CH : 1];
  int st_k0 = 0;
  uint32_t a_valid = 0;
  const bool wthru = TWO_IN && p.aout != nullptr && tile_n == 0;
  (void)rx; (void)st_k0; (void)a_valid; (void)wthru;
  if constexpr (TWO_IN) {  // PRO_BWD: k | c1 | c0; PRO_RES: scale | shift; PRO_RES2: + scale_d | shift_d
    for (int i = t; i < (PRO == PRO_BWD ? 3 : PRO == PRO_RES2 ? 4 : 2) * K / 4; i += kThreads)
      reinterpret_cast<float4*>(coef_lds)[i] = (PRO == PRO_RES2 && i >= K / 2)
                                                   ? reinterpret_cast<const float4*>(p.bcoef2)[i - K / 2]
                                                   : reinterpret_cast<const float4*>(p.bcoef)[i];
    __syncthreads();
  }
  auto setup_rows = [&](int tm) {
    a_valid = 0;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int m0 = tm * BM + a_row[i];
      a_valid |= m0 < M ? (1u << i) : 0u;
      const int m = m0 < M ? m0 : 0;  // tail rows re-read row 0 (never stored): no divergent loads
      int64_t src = m;
      if constexpr (GATHER != G_DENSE) {
        const int hw = p.Hout * p.Wout;
        const int nimg = m / hw, rem = m - nimg * hw;
        const int oh = rem / p.Wout, ow = rem - oh * p.Wout;
        if constexpr (GATHER == G_STRIDED) {
          src = (static_cast<int64_t>(nimg) * p.Hin + oh * p.stride) * p.Win + ow * p.stride;
        } else {
          a_base[i] = nimg * p.Hin * p.Win;
          a_ih[i] = oh * p.stride - 1;
          a_iw[i] = ow * p.stride - 1;
        }
      }
      a_off[i] = src * K;
    }
  };
  auto gload = [&](int kt) {
    const int k0 = kt * KBK;
    int kc0 = k0;  // channel offset of this K-step within a tap
    if constexpr (GATHER == G_CONV3) {
      const int tap = k0 / p.Cin;  // BK divides Cin: a K-step never straddles taps
      kc0 = k0 - tap * p.Cin;
      const int r = tap / 3, q = tap - 3 * (tap / 3);
      ra_ok = 0;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int ih = a_ih[i] + r, iw = a_iw[i] + q;
        const bool ok = static_cast<unsigned>(ih) < static_cast<unsigned>(p.Hin) &&
                        static_cast<unsigned>(iw) < static_cast<unsigned>(p.Win);
        const int row = ok ? a_base[i] + ih * p.Win + iw : 0;
        ra_ok |= ok ? (1u << i) : 0u;
        ra[i] = ld16(p.A + static_cast<int64_t>(row) * p.Cin + kc0 + a_kc[i]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_CH; ++i)
        ra[i] = ld16(p.A + a_off[i] + k0 + a_kc[i]);  // rows >= M read row 0: their outputs are never stored
      if constexpr (TWO_IN) {
#pragma unroll
        for (int i = 0; i < A_CH; ++i) rx[i] = ld16(p.bx + a_off[i] + k0 + a_kc[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int c = t + i * kThreads;
      rb[i] = ld16(p.B + static_cast<int64_t>(n0 + c / CPRK) * K + k0 + (c % CPRK) * 8);
    }
    if constexpr (TWO_IN) st_k0 = k0;
    if constexpr (PRO == PRO_FWD) {
      const int kcoef = GATHER == G_CONV3 ? p.Cin : K;
      const float4* sp = reinterpret_cast<const float4*>(p.pro_coef + kc0 + a_kc[0]);
      const float4* fp = reinterpret_cast<const float4*>(p.pro_coef + kcoef + kc0 + a_kc[0]);
      const float4 s0 = sp[0], s1 = sp[1], f0 = fp[0], f1 = fp[1];
      psc[0] = s0.x; psc[1] = s0.y; psc[2] = s0.z; psc[3] = s0.w;
      psc[4] = s1.x; psc[5] = s1.y; psc[6] = s1.z; psc[7] = s1.w;
      psf[0] = f0.x; psf[1] = f0.y; psf[2] = f0.z; psf[3] = f0.w;
      psf[4] = f1.x; psf[5] = f1.y; psf[6] = f1.z; psf[7] = f1.w;
    }
  };
  auto swrite = [&](int buf) {
    bf16_t* As = lds + buf * kBuf;
    bf16_t* Bs = As + BM * ldk;
    float bk[8], bc1[8], bc0[8], bd[8];  // PRO_BWD / RES / RES2: this thread's 8 channels of the staged K-step
    (void)bk; (void)bc1; (void)bc0; (void)bd;
    if constexpr (TWO_IN) {
      const int c = st_k0 + a_kc[0];
#pragma unroll
      for (int j = 0; j < 8; j += 4) {
        const float4 a = *reinterpret_cast<const float4*>(coef_lds + c + j);
        const float4 b = *reinterpret_cast<const float4*>(coef_lds + K + c + j);
        bk[j] = a.x; bk[j + 1] = a.y; bk[j + 2] = a.z; bk[j + 3] = a.w;
        bc1[j] = b.x; bc1[j + 1] = b.y; bc1[j + 2] = b.z; bc1[j + 3] = b.w;
        if constexpr (PRO == PRO_BWD || PRO == PRO_RES2) {
          const float4 z = *reinterpret_cast<const float4*>(coef_lds + 2 * K + c + j);
          bc0[j] = z.x; bc0[j + 1] = z.y; bc0[j + 2] = z.z; bc0[j + 3] = z.w;
        }
        if constexpr (PRO == PRO_RES2) {
          const float4 z = *reinterpret_cast<const float4*>(coef_lds + 3 * K + c + j);
          bd[j] = z.x; bd[j + 1] = z.y; bd[j + 2] = z.z; bd[j + 3] = z.w;
        }
      }
    }
    constexpr bool fwd_pro = PRO == PRO_FWD;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      uint4 v = ra[i];
      if constexpr (fwd_pro) {
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float o = fmaf(f[j], psc[j], psf[j]);
          f[j] = o > 0.f ? o : 0.f;
        }
        v = pack8(f);
      } else if constexpr (PRO == PRO_BWD) {
        float f[8], x[8];
        unpack8(v, f);
        unpack8(rx[i], x);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaf(bk[j], f[j], fmaf(bc1[j], x[j], bc0[j]));
        v = pack8(f);
        if (wthru && ((a_valid >> i) & 1u))
          *reinterpret_cast<uint4*>(p.aout + a_off[i] + st_k0 + a_kc[i]) = v;
      } else if constexpr (PRO == PRO_RES || PRO == PRO_RES2) {
        // bn_fwd_apply('s dual) expression order: fmaf, + residual (its own fmaf), mask, ReLU
        float f[8], r[8];
        unpack8(v, f);
        unpack8(rx[i], r);
        uint32_t bits = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float o = fmaf(f[j], bk[j], bc1[j]) + (PRO == PRO_RES2 ? fmaf(r[j], bc0[j], bd[j]) : r[j]);
          bits |= (o > 0.f ? 1u : 0u) << j;
          f[j] = o > 0.f ? o : 0.f;
        }
        v = pack8(f);
        if (wthru && ((a_valid >> i) & 1u)) {
          const int64_t e = a_off[i] + st_k0 + a_kc[i];
          *reinterpret_cast<uint4*>(p.aout + e) = v;
          p.obits[e >> 3] = static_cast<uint8_t>(bits);
        }
      }
      if constexpr (GATHER == G_CONV3) {
        if (!((ra_ok >> i) & 1u)) v = make_uint4(0, 0, 0, 0);  // zero padding (after BN+ReLU)
      }
      *reinterpret_cast<uint4*>(&As[soff(a_row[i], a_kc[i] >> 3)]) = v;
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int c = t + i * kThreads;
      *reinterpret_cast<uint4*>(&Bs[soff(c / CPRK, c % CPRK)]) = rb[i];
    }
  };

  Epilogue<BM, BN, kThreads, EPI, G_DENSE> epi;
  epi.init(t, n0);
  int tm = gm;
  if (tm < tiles_m) {
    setup_rows(tm);
    gload(0);
    swrite(0);
  }
  __syncthreads();
  int cur = 0;
  const int fr = lane & 31, fh = lane >> 5;
  for (; tm < tiles_m; tm += GM) {
    f32x16_t acc[TN][TM];
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = f32x16_t{};
    // one staged K-step's fragments + MFMAs into ``a``
    auto mma = [&](const bf16_t* As, f32x16_t (&a)[TN][TM]) {
      const bf16_t* Bs = As + BM * ldk;
#pragma unroll
      for (int s = 0; s < KBK / 16; ++s) {
        bf16x8_t wf[TN], xf[TM];
#pragma unroll
        for (int i = 0; i < TN; ++i)
          wf[i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(&Bs[soff(wn0 + i * 32 + fr, s * 2 + fh)]));
#pragma unroll
        for (int j = 0; j < TM; ++j)
          xf[j] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(&As[soff(wm0 + j * 32 + fr, s * 2 + fh)]));
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j)
            a[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i], xf[j], a[i][j], 0, 0, 0);
      }
    };
    // the tile's epilogue (csrc/gemm_epi.h) with its output tile in LDS at Cb;
    // row-side operands of the first prefetch group are issued before the
    // accumulators go to LDS
    auto epilogue = [&](bf16_t* Cb) {
      epi.begin(p, tm);
      bf16_t* Cs = Cb;
      acc_to_lds<TN, TM>(acc, Cs, LDC, wm0, wn0, lane);
      __syncthreads();
      epi.rows(p, Cs, tm);
      __syncthreads();  // Cs is restaged by a later K-step
    };
    for (int kt = 0; kt < nk; ++kt) {
      const bool more_k = kt + 1 < nk;
      const bool more = more_k || tm + GM < tiles_m;
      if (more_k) {
        gload(kt + 1);
      } else if (more) {
        setup_rows(tm + GM);
        gload(0);
      }
      const bf16_t* As = lds + cur * kBuf;
      mma(As, acc);
      if (more_k || (more && !SPLIT_C)) swrite(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
    // D[n][m] -> LDS [m][n] (buffer cur^1 is free: its last reader was the final
    // K-step, which ended with a barrier; buffer cur may already hold the next
    // tile's first K-step)
    epilogue(SPLIT_C ? lds : lds + (cur ^ 1) * kBuf);
    if constexpr (SPLIT_C) {  // stage the next tile's first K-step now that the epilogue is done
      if (tm + GM < tiles_m) swrite(0);
      cur = 0;
      __syncthreads();
    }
  }

  epi.finish(p, reinterpret_cast<float*>(lds), b, gm < tiles_m);
}

// ------------------------------------------------------------------ wgrad
// dW[N, K] = sum_m G[m, n] * pro(A)[m, k], A row-gathered for strided convs.
// Tile TN_ (N) x TK_ (K) (each 64 or 128) x 64 (M-step); each block reduces
// one contiguous M-range and adds its tile into the fp32 dW32 with atomics.  Both operands
// arrive with the reduction index (m) strided, so staging transposes them: a
// thread loads an 8 (m) x 8 (channel) bf16 block as eight 16-B row chunks,
// transposes it in registers (v_perm_b32 half-word selects) and writes eight
// 16-B channel rows of m-contiguous data -- the K-contiguous fragment layout
// the MFMA operands want.
constexpr int WMK = 64;   // M per step
constexpr int LDW = WMK + 8;

__device__ __forceinline__ void transpose8x8(const uint4 (&in)[8], uint4 (&out)[8]) {
  // in[r] = 8 bf16 of row r (elements c = 0..7); out[c] = 8 bf16 (rows 0..7) of column c
  uint32_t w[8][4];
#pragma unroll
  for (int r = 0; r < 8; ++r) { w[r][0] = in[r].x; w[r][1] = in[r].y; w[r][2] = in[r].z; w[r][3] = in[r].w; }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    uint32_t o[4];
#pragma unroll
    for (int rp = 0; rp < 4; ++rp) {
      const uint32_t x0 = w[2 * rp][c >> 1], x1 = w[2 * rp + 1][c >> 1];
      // low half of the output dword = element c of row 2rp, high half = element c of row 2rp+1
      o[rp] = (c & 1) ? __builtin_amdgcn_perm(x1, x0, 0x07060302u) : __builtin_amdgcn_perm(x1, x0, 0x05040100u);
    }
    out[c] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// GPRO: G gets the same BN + ReLU prologue as A (coefficients [scale(N) |
// shift(N)] of pro_coef: the Gram matrix relu(B(X))^T relu(B(X)) when G = A = X,
// N = K).  COLSUM: the blocks of output-tile row 0 also write the column sums of
// the staged A' (as the bf16 values the MFMAs see) behind each split's [N][K]
// slab, i.e. slabs of N * K + K floats.
template <int TN_, int TK_, bool PRO, int GATHER, bool GPRO = false, bool COLSUM = false>
__global__ __launch_bounds__(kThreads, 2) void wgrad1x1_kernel(
    const bf16_t* __restrict__ G, const bf16_t* __restrict__ A, const float* __restrict__ pro_coef,
    float* __restrict__ dw32, int M, int N, int K, int Hout, int Wout, int Hin, int Win, int stride,
    int rows_per_split, int tiles_k, int cin) {
  static_assert(!GPRO || (PRO && GATHER == G_DENSE), "the G prologue serves the dense Gram matrix");
  // [2 buffers][G^T tile TN_ x LDW | A^T tile TK_ x LDW]
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * (TN_ + TK_) * LDW];
  constexpr int kBuf = (TN_ + TK_) * LDW;
  constexpr int WTN = TN_ / 2, WTK = TK_ / 2;  // 2 x 2 waves
  constexpr int FN = WTN / 32, FK = WTK / 32;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // XCD-aware order: hardware block b runs on XCD b % 8; give each XCD a
  // contiguous range of logical ids (bijective for any grid size), and make the
  // tiles of one M-split consecutive, so the blocks that stream the same G/A
  // rows share that XCD's L2 instead of re-reading them from MALL/HBM.
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int xq = nblk >> 3, xr = nblk & 7, xcd = bid & 7;
  const int wid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (bid >> 3);
  const int tiles = (N / TN_) * tiles_k;
  const int split = wid / tiles, tile = wid - split * tiles;
  const int tn = tile / tiles_k, tk = tile - tn * tiles_k;
  const int n0 = tn * TN_, k0 = tk * TK_;
  const int mbeg = split * rows_per_split;
  const int mend = min(M, mbeg + rows_per_split);
  // staging units: an 8 (m) x 8 (channel) block each; TN_ units of G, then TK_ of A
  const bool isA = t >= TN_;
  const bool stager = t < TN_ + TK_;
  const int u = isA ? t - TN_ : t;
  const int cpr = (isA ? TK_ : TN_) / 8;
  const int mg = u / cpr;         // 0..7: rows mg*8 .. +7 of the M-step
  const int cc = (u % cpr) * 8;   // channel chunk within the tile
  // 3x3 weight gradient: K = 9 * cin, this tile's K range lies in one tap (TK_ | cin)
  const int tap = GATHER == G_CONV3 ? k0 / cin : 0;
  const int kin0 = k0 - tap * cin;
  const int tr3 = tap / 3, tq3 = tap - 3 * (tap / 3);
  const int col0 = (isA ? (GATHER == G_CONV3 ? kin0 : k0) : n0) + cc;
  const int ld = isA ? (GATHER == G_CONV3 ? cin : K) : N;
  const int kcoef = GATHER == G_CONV3 ? cin : K;
  const bf16_t* base = isA ? A : G;
  float psc[8], psf[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { psc[j] = 1.f; psf[j] = 0.f; }
  if (PRO && isA && stager) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { psc[j] = pro_coef[col0 + j]; psf[j] = pro_coef[kcoef + col0 + j]; }
  }
  if (GPRO && !isA && stager) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { psc[j] = pro_coef[col0 + j]; psf[j] = pro_coef[N + col0 + j]; }
  }
  float csum[8];  // COLSUM: this A-stager's column sums over its staged rows
#pragma unroll
  for (int j = 0; j < 8; ++j) csum[j] = 0.f;
  (void)csum;
  uint4 rr[8];
  uint32_t rok = 0xffu;  // 3x3: rows of the staged set whose tap lies inside the image
  (void)tr3; (void)tq3;
  // Loads are unconditional (tail rows clamp to row mbeg) so that no load sits
  // behind an exec branch; the tail rows are zeroed when staged to LDS.
  auto gload = [&](int m0) {
    if (!stager) return;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int m1 = m0 + mg * 8 + r;
      const int m = m1 < mend ? m1 : mbeg;
      int64_t src = m;
      if (GATHER != G_DENSE && isA) {
        const int hw = Hout * Wout;
        const int nimg = m / hw, rem = m - nimg * hw;
        const int oh = rem / Wout, ow = rem - oh * Wout;
        if (GATHER == G_STRIDED) {
          src = (static_cast<int64_t>(nimg) * Hin + oh * stride) * Win + ow * stride;
        } else {
          const int ih = oh * stride + tr3 - 1, iw = ow * stride + tq3 - 1;
          const bool ok = static_cast<unsigned>(ih) < static_cast<unsigned>(Hin) &&
                          static_cast<unsigned>(iw) < static_cast<unsigned>(Win);
          src = ok ? (static_cast<int64_t>(nimg) * Hin + ih) * Win + iw : 0;
          rok = ok ? (rok | (1u << r)) : (rok & ~(1u << r));
        }
      }
      rr[r] = ld16(base + src * ld + col0);
    }
  };
  auto swrite = [&](int buf, int m0) {
    if (!stager) return;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const bool ok = m0 + mg * 8 + r < mend && ((rok >> r) & 1u);  // tail rows / padding taps stage as zero
      if ((PRO && isA) || (GPRO && !isA)) {
        float f[8];
        unpack8(rr[r], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float o = fmaf(f[j], psc[j], psf[j]);
          f[j] = o > 0.f ? o : 0.f;
        }
        rr[r] = pack8(f);
      }
      if (!ok) rr[r] = make_uint4(0, 0, 0, 0);
      if (COLSUM && isA) {
        float f[8];
        unpack8(rr[r], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) csum[j] += f[j];
      }
    }
    uint4 tr[8];
    transpose8x8(rr, tr);
    bf16_t* S = lds + buf * kBuf + (isA ? TN_ * LDW : 0);
#pragma unroll
    for (int c = 0; c < 8; ++c) *reinterpret_cast<uint4*>(&S[(cc + c) * LDW + mg * 8]) = tr[c];
  };
  const int wn0 = (wave >> 1) * WTN, wk0 = (wave & 1) * WTK;
  const int fr = lane & 31, fh = lane >> 5;
  f32x16_t acc[FN][FK];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  int cur = 0;
  if (mbeg < mend) {
    gload(mbeg);
    swrite(0, mbeg);
  }
  __syncthreads();
  for (int m0 = mbeg; m0 < mend; m0 += WMK) {
    const bool more = m0 + WMK < mend;
    if (more) gload(m0 + WMK);
    const bf16_t* Gs = lds + cur * kBuf;
    const bf16_t* As = Gs + TN_ * LDW;
#pragma unroll
    for (int s = 0; s < WMK / 16; ++s) {
      bf16x8_t gf[FN], af[FK];
#pragma unroll
      for (int i = 0; i < FN; ++i)
        gf[i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(&Gs[(wn0 + i * 32 + fr) * LDW + s * 16 + fh * 8]));
#pragma unroll
      for (int j = 0; j < FK; ++j)
        af[j] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(&As[(wk0 + j * 32 + fr) * LDW + s * 16 + fh * 8]));
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FK; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gf[i], af[j], acc[i][j], 0, 0, 0);
    }
    if (more) swrite(cur ^ 1, m0 + WMK);
    __syncthreads();
    cur ^= 1;
  }
  // D[n][k]: col k = lane&31, rows n = (r&3) + 8(r>>2) + 4h.  Plain fp32 stores
  // of this split's partial tile into its own slab dw32[split][N][K] (each
  // half-wave writes one 128-B row segment per register); wgrad_reduce_kernel
  // sums the slabs in a fixed order.  Plain stores stream at the HBM rate where
  // fp32 atomics into one [N][K] buffer were capped at ~1.3 TB/s of added bytes
  // (MI355X_MICROARCH.md "Global float atomics") -- 16 splits x 4 MiB at the
  // 7x7 stage was half the kernel's time -- and the result is deterministic.
  float* slab = dw32 + static_cast<int64_t>(split) * (static_cast<int64_t>(N) * K + (COLSUM ? K : 0));
  if constexpr (COLSUM) {
    // fold the 8 row groups of each column chunk (the loop's last barrier freed lds)
    float* cs = reinterpret_cast<float*>(lds);  // [8 (mg)][TK_]
    if (stager && isA) {
#pragma unroll
      for (int j = 0; j < 8; ++j) cs[mg * TK_ + cc + j] = csum[j];
    }
    __syncthreads();
    if (tn == 0 && t < TK_) {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) v += cs[g * TK_ + t];
      slab[static_cast<int64_t>(N) * K + k0 + t] = v;
    }
  }
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        const int k = k0 + wk0 + j * 32 + fr;
        slab_store(slab + static_cast<int64_t>(n) * K + k, acc[i][j][r]);
      }
}

// Block (x, y) sums the slabs (y * chunk + j) * stride, j < min(chunk, count -
// y * chunk), over 64 columns, in a fixed order: into bf16 dW (scaled) when
// ``out`` is given, else as fp32 into the block's first slab (an in-place
// partial: only this block touches those columns of that slab).  Block = 16
// float4 columns x 16 split groups folded in LDS.  Many splits over few
// columns (early layers: 256 slabs of a 64x256 weight) go through two passes:
// partial sums over y-chunks of splits, then the chunk partials.
constexpr int kRedCols = 16, kRedGroups = kThreads / kRedCols;
// ``layout`` 1 (the stem, csrc/stem.hip): the slabs are [64][224] in the stem
// kernel's K order (k = r * 32 + s * 4 + c, s < 8, c < 4) and ``out`` is the
// nn.Conv2d weight gradient [64, 3, 7, 7] channels_last ([n][r][s][c] in
// memory): padding columns are dropped.
__global__ __launch_bounds__(kThreads) void wgrad_reduce_kernel(float* __restrict__ dw32, int64_t nk, int count,
                                                                int chunk, int stride, float scale,
                                                                bf16_t* __restrict__ out, int layout) {
  __shared__ float4 part[kRedGroups][kRedCols];
  const int col = threadIdx.x % kRedCols, grp = threadIdx.x / kRedCols;
  const int64_t i4 = (static_cast<int64_t>(blockIdx.x) * kRedCols + col) * 4;
  const int base = blockIdx.y * chunk;
  const int cnt = (count - base) < chunk ? (count - base) : chunk;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < nk) {
#pragma unroll 4
    for (int sp = grp; sp < cnt; sp += kRedGroups) {
      const f32x4_t v = *reinterpret_cast<const f32x4_t*>(dw32 + static_cast<int64_t>(base + sp) * stride * nk + i4);
      a.x += v[0]; a.y += v[1]; a.z += v[2]; a.w += v[3];
    }
  }
  part[grp][col] = a;
  __syncthreads();
  if (grp == 0 && i4 < nk) {
#pragma unroll
    for (int g = 1; g < kRedGroups; ++g) {
      const float4 v = part[g][col];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    if (out && layout == 1) {
      const float v[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = static_cast<int>(i4) + q, n = idx / 224, k = idx - n * 224;
        const int r = k >> 5, sc = (k >> 2) & 7, c = k & 3;
        if (sc < 7 && c < 3) out[n * 147 + (r * 7 + sc) * 3 + c] = f32_to_bf16(v[q] * scale);
      }
    } else if (out) {
      const uint32_t lo = pack_bf16x2(a.x * scale, a.y * scale);
      const uint32_t hi = pack_bf16x2(a.z * scale, a.w * scale);
      *reinterpret_cast<uint2*>(out + i4) = make_uint2(lo, hi);
    } else {
      *reinterpret_cast<float4*>(dw32 + static_cast<int64_t>(base) * stride * nk + i4) =
          make_float4(a.x * scale, a.y * scale, a.z * scale, a.w * scale);
    }
  }
}

template <int BM, int BN, int MINB, int PRO, int GATHER, int EPI, int KBK>
hipError_t launch_gemm(const GemmParams& p, hipStream_t s) {
  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = p.N / BN;
  // persistent blocks: one round of the resident capacity (256 CUs x MINB), nblk % 8 == 0
  // (1 round measured +2.3% per ResNet-50 step over 2; KDL_TUNE gemm_rounds overrides)
  static const int rounds = tune_int("gemm_rounds", 1);
  const int target = 256 * MINB * rounds;
  int GM = (target + tiles_n - 1) / tiles_n;
  if (GM > tiles_m) GM = tiles_m;
  while ((GM * tiles_n) % 8) ++GM;
  hipLaunchKernelGGL((gemm1x1_kernel<BM, BN, MINB, PRO, GATHER, EPI, KBK>), dim3(GM * tiles_n), dim3(kThreads), 0, s, p,
                     GM, tiles_m, tiles_n);
  return hipGetLastError();
}

// forward convs (prologue / row gather) only ever use the PLAIN and STATS
// epilogues; the dgrad epilogues run without either (3x3 dgrad: MASKX); the
// backward-apply prologue feeds only the dense dgrad epilogues
template <int BM, int BN, int MINB, int PRO, int GATHER, int KBK>
hipError_t dispatch_epi(const GemmParams& p, int epi, hipStream_t s) {
  if constexpr (PRO == PRO_RES || PRO == PRO_RES2) {  // the next block's conv1 (forward, bn1 statistics)
    if (epi == EPI_STATS) return launch_gemm<BM, BN, MINB, PRO, GATHER, EPI_STATS, KBK>(p, s);
    return hipErrorInvalidValue;
  } else if constexpr (PRO == PRO_BWD) {
    switch (epi) {
      case EPI_PLAIN: return launch_gemm<BM, BN, MINB, PRO, GATHER, EPI_PLAIN, KBK>(p, s);
      case EPI_MASKX: return launch_gemm<BM, BN, MINB, PRO, GATHER, EPI_MASKX, KBK>(p, s);
      case EPI_RESBITS: return launch_gemm<BM, BN, MINB, PRO, GATHER, EPI_RESBITS, KBK>(p, s);
      case EPI_RES: return launch_gemm<BM, BN, MINB, PRO, GATHER, EPI_RES, KBK>(p, s);
    }
    return hipErrorInvalidValue;
  } else {
    switch (epi) {
      case EPI_PLAIN: return launch_gemm<BM, BN, MINB, PRO, GATHER, EPI_PLAIN, KBK>(p, s);
      case EPI_STATS: return launch_gemm<BM, BN, MINB, PRO, GATHER, EPI_STATS, KBK>(p, s);
    }
    if constexpr (PRO == PRO_NONE && GATHER == G_DENSE) {
      switch (epi) {
        case EPI_MASKX: return launch_gemm<BM, BN, MINB, PRO, GATHER, EPI_MASKX, KBK>(p, s);
        case EPI_RESBITS: return launch_gemm<BM, BN, MINB, PRO, GATHER, EPI_RESBITS, KBK>(p, s);
        case EPI_RES: return launch_gemm<BM, BN, MINB, PRO, GATHER, EPI_RES, KBK>(p, s);
      }
    }
    if constexpr (PRO == PRO_NONE && GATHER == G_CONV3) {
      if (epi == EPI_MASKX) return launch_gemm<BM, BN, MINB, PRO, GATHER, EPI_MASKX, KBK>(p, s);
    }
    return hipErrorInvalidValue;
  }
}

template <int BM, int BN, int MINB, int KBK = BK>
hipError_t dispatch_pg(const GemmParams& p, int epi, int pro, int gather, hipStream_t s) {
  if (pro == PRO_BWD || pro == PRO_RES || pro == PRO_RES2) {
    if constexpr (BM == 128 && MINB == 2 && KBK == BK) {  // the two configs conv1x1_gemm routes them to
      if (gather != G_DENSE) return hipErrorInvalidValue;
      if (pro == PRO_BWD) return dispatch_epi<BM, BN, MINB, PRO_BWD, G_DENSE, KBK>(p, epi, s);
      if (pro == PRO_RES) return dispatch_epi<BM, BN, MINB, PRO_RES, G_DENSE, KBK>(p, epi, s);
      if constexpr (BN == 64)  // (128 x 128 spills with the fourth coefficient row)
        if (pro == PRO_RES2) return dispatch_epi<BM, BN, MINB, PRO_RES2, G_DENSE, KBK>(p, epi, s);
    }
    return hipErrorInvalidValue;
  }
  if (gather == G_CONV3)
    return pro ? dispatch_epi<BM, BN, MINB, PRO_FWD, G_CONV3, KBK>(p, epi, s) : dispatch_epi<BM, BN, MINB, PRO_NONE, G_CONV3, KBK>(p, epi, s);
  if (pro) return gather ? dispatch_epi<BM, BN, MINB, PRO_FWD, G_STRIDED, KBK>(p, epi, s) : dispatch_epi<BM, BN, MINB, PRO_FWD, G_DENSE, KBK>(p, epi, s);
  return gather ? dispatch_epi<BM, BN, MINB, PRO_NONE, G_STRIDED, KBK>(p, epi, s) : dispatch_epi<BM, BN, MINB, PRO_NONE, G_DENSE, KBK>(p, epi, s);
}

// Tile configs: 0 = 128x128 (2 blocks/CU), 1 = 128x64, 2 = 64x128, 3 = 64x64 (4 blocks/CU),
// 5 = 128x128 with 32-deep K-steps (40 KiB of LDS, 3 blocks/CU).
int pick_config(int M, int N, int K, int epi) {
  static const int forced = tune_int("gemm_cfg", -1);
  if (forced >= 0 && forced <= 5) {
    if ((forced == 0 || forced == 2 || forced == 5) && N % 128) return 3;
    if (forced == 4) return N % 128 ? 1 : 0;
    return forced;
  }
  // Short-K statistics GEMMs (the forward 1x1 convs of stages 1-2) gain from the
  // third resident block of the 32-deep-K config (-8..14 %); dgrad epilogues do
  // not (RESBITS spills at 168 VGPRs) and long K is neutral.
  if (N % 128 == 0 && epi == EPI_STATS && K <= 256) return 5;
  return N % 128 == 0 ? 0 : 1;
}

}  // namespace

namespace {
// KDL_TUNE gemm_core: 0 = register-staged loop only, 1 = LDS-DMA loop wherever it
// applies, -1 (default) = by shape (long K / 3x3 without prologue -> DMA)
int g_core = tune_int("gemm_core", -1);
}  // namespace

int gemm_core_mode() { return g_core; }
void set_gemm_core_mode(int m) { g_core = m; }

hipError_t conv1x1_gemm(const Conv1x1Args& a, hipStream_t s) {
  if (a.K % BK || a.N % 64 || a.M <= 0) return hipErrorInvalidValue;
  GemmParams p{};
  p.A = static_cast<const bf16_t*>(a.A);
  p.B = static_cast<const bf16_t*>(a.B);
  p.C = static_cast<bf16_t*>(a.C);
  p.M = a.M; p.N = a.N; p.K = a.K;
  p.Hout = a.Hout; p.Wout = a.Wout; p.Hin = a.Hin; p.Win = a.Win; p.stride = a.stride;
  p.pro_coef = a.pro_coef;
  p.shift = a.shift; p.acc = a.acc;
  p.ex = static_cast<const bf16_t*>(a.ex); p.emean = a.emean; p.ecoef = a.ecoef;
  p.eres = static_cast<const bf16_t*>(a.eres); p.res_stride = a.res_stride > 0 ? a.res_stride : 1;
  p.res_H = a.res_H; p.res_W = a.res_W;
  p.ebits = a.ebits; p.ex2 = static_cast<const bf16_t*>(a.ex2); p.emean2 = a.emean2; p.acc2 = a.acc2;
  p.fin_ws = a.fin_ws; p.fin_ws2 = a.fin_ws2; p.fin_M = a.fin_M;
  p.bx = static_cast<const bf16_t*>(a.bx); p.bcoef = a.bcoef; p.bcoef2 = a.bcoef2;
  p.aout = static_cast<bf16_t*>(a.aout);
  p.obits = a.obits;
  const bool bpro = a.bx != nullptr;
  if (bpro && !a.bres && (!a.bcoef || a.pro_coef || a.stride > 1 || a.ksize == 3 || a.epi == EPI_STATS))
    return hipErrorInvalidValue;
  if (bpro && a.bres && (!a.bcoef || a.pro_coef || a.stride > 1 || a.ksize == 3 || a.epi != EPI_STATS ||
                         !a.aout || !a.obits || a.K > bwd_kmax(64)))
    return hipErrorInvalidValue;
  if (a.epi != EPI_PLAIN && a.epi != EPI_STATS && a.epi != EPI_MASKX && a.epi != EPI_RESBITS && a.epi != EPI_RES)
    return hipErrorInvalidValue;
  const int pro = bpro ? (a.bres == 2 ? PRO_RES2 : a.bres ? PRO_RES : PRO_BWD)
                : a.pro_coef != nullptr ? PRO_FWD : PRO_NONE;
  int gather = a.stride > 1 ? G_STRIDED : G_DENSE;
  p.Cin = a.K;
  if (a.ksize == 3) {
    // 3x3, pad 1: K = 9 * Cin, B = weight [N][3][3][Cin] (OHWI = channels_last OIHW)
    if (a.Cin <= 0 || a.Cin % BK || a.K != 9 * a.Cin || a.stride < 1 ||
        a.Hout != (a.Hin - 1) / a.stride + 1 || a.Wout != (a.Win - 1) / a.stride + 1 ||
        a.M % (a.Hout * a.Wout))
      return hipErrorInvalidValue;
    gather = G_CONV3;
    p.Cin = a.Cin;
  } else if (a.ksize != 1 && a.ksize != 0) {
    return hipErrorInvalidValue;
  }
  const int epi = a.epi;
  if (epi == EPI_RES || epi == EPI_RESBITS) {
    if (!p.eres) return hipErrorInvalidValue;
  }
  // long K without an A prologue: the LDS-DMA main loop (csrc/igemm.hip)
  const int core = gemm_core_mode();
  // 56x56 3x3 forward with the BN + ReLU prologue: the halo kernel applies it in LDS
  if (pro == PRO_FWD && gather == G_CONV3 && core != 0 && p.K % 64 == 0) {
    p.a_rows = static_cast<int64_t>(p.M / (a.Hout * a.Wout)) * a.Hin * a.Win;
    const hipError_t h = halo3x3(p, epi, s);
    if (h != hipErrorInvalidValue) return h;
    if (p.aout) return hipErrorInvalidValue;  // the write-through of relu(B(x)) is the halo kernel's only
  }
  const int min_k = gather == G_CONV3 ? 0 : 512;
  // (the backward-apply prologue transforms A in registers: register-staged loop)
  if (!pro && core != 0 && (core == 1 || p.K >= min_k) && p.K % 64 == 0) {
    p.a_rows = gather == G_CONV3 ? static_cast<int64_t>(p.M / (a.Hout * a.Wout)) * a.Hin * a.Win
               : gather == G_STRIDED ? static_cast<int64_t>(p.M / (a.Hout * a.Wout)) * a.Hin * a.Win
                                     : p.M;
    if (gather == G_CONV3) {  // early stages: input halo staged once per tile (csrc/halo3x3.hip)
      const hipError_t h = halo3x3(p, epi, s);
      if (h != hipErrorInvalidValue) return h;
    }
    int cfg = igemm_pick(p.M, p.N, p.K);
    // 3x3 at N = 512 (7x7 stage): 256x128 tiles (1 block/CU) beat 128x128 by 2-3 %
    // (86.5-88.5 vs 89-90.6 us, profiles/r02_halo3x3_vs_igemm.jsonl dma1 vs dma2)
    if (gather == G_CONV3 && p.N == 512 && g_forced_cfg_unset()) cfg = 1;
    const hipError_t e = igemm(p, epi, gather, cfg, s);
    if (e != hipErrorInvalidValue) return e;
  }
  if (pro == PRO_RES2) {  // four coefficient rows; 128 x 64 tiles (128 x 128 spills 12 B)
    if (4 * p.K <= 3 * bwd_kmax(64)) return dispatch_pg<128, 64, 2>(p, epi, pro, gather, s);
    return hipErrorInvalidValue;
  }
  if (pro == PRO_BWD || pro == PRO_RES) {  // coefficient table in LDS: 128-wide tiles to K = 512, 64-wide beyond
    if (p.N % 128 == 0 && p.K <= bwd_kmax(128)) return dispatch_pg<128, 128, 2>(p, epi, pro, gather, s);
    if (p.K <= bwd_kmax(64)) return dispatch_pg<128, 64, 2>(p, epi, pro, gather, s);
    return hipErrorInvalidValue;
  }
  switch (pick_config(p.M, p.N, p.K, epi)) {
    case 0: return dispatch_pg<128, 128, 2>(p, epi, pro, gather, s);
    case 1: return dispatch_pg<128, 64, 2>(p, epi, pro, gather, s);
    case 2: return dispatch_pg<64, 128, 3>(p, epi, pro, gather, s);
    case 5: return dispatch_pg<128, 128, 3, 32>(p, epi, pro, gather, s);
    default: return dispatch_pg<64, 64, 4>(p, epi, pro, gather, s);
  }
}

hipError_t conv3x3_dgrad_s2(const Conv1x1Args& a, hipStream_t s) {
  if (a.Cin <= 0 || a.Cin % 64 || a.N % 64 || a.K != 9 * a.Cin || (a.Hout != 2 * a.Hin && a.Hout != 2 * a.Hin - 1) ||
      (a.Wout != 2 * a.Win && a.Wout != 2 * a.Win - 1) ||
      a.M <= 0 || a.M % (a.Hin * a.Win) || (a.epi != EPI_PLAIN && a.epi != EPI_MASKX) || a.pro_coef)
    return hipErrorInvalidValue;
  GemmParams p{};
  p.A = static_cast<const bf16_t*>(a.A);
  p.B = static_cast<const bf16_t*>(a.B);
  p.C = static_cast<bf16_t*>(a.C);
  p.N = a.N; p.K = a.K; p.Cin = a.Cin;
  p.Hin = a.Hin; p.Win = a.Win; p.Hout = a.Hout; p.Wout = a.Wout; p.stride = 2;
  p.mc = a.M;
  p.M = 4 * a.M;  // the launcher pads each class to whole tiles
  p.a_rows = a.M;
  p.acc = a.acc;
  p.ex = static_cast<const bf16_t*>(a.ex); p.emean = a.emean; p.ecoef = a.ecoef;
  p.fin_ws = a.fin_ws; p.fin_M = a.fin_M;
  int cfg = igemm_pick(4 * a.M, a.N, a.K);
  if (cfg == 4) cfg = 1;  // the three-stage loop has no G_DGRAD2 variant
  return igemm(p, a.epi, G_DGRAD2, cfg, s);
}

// Weight-gradient tile (tn x tk): 256 x 256 on the LDS-DMA core where both
// dimensions allow it (8 waves, 1 block/CU: half the operand bytes per MFMA of
// 128 x 128).  Standalone the 3x3 stage-3/4 gradients drop 108 -> 84 us and
// 137 -> 94 us while the 1x1 ones rise 43 -> 55 us, yet in the two-stream step
// the 1x1 ones gain too (fewer, heavier side-stream blocks): same box, job
// steps off / 3x3 only / 3x3 + 1x1 = 12,640 / 12,738-12,755 / 12,780-12,794
// img/s (profiles/r02_wgrad_big_tiles_ab.txt).  Without that overlap (the CTR
// tower's weight gradients) the 1x1 ones stay on 128 tiles (CTR samples/s equal
// within run-to-run noise either way: 3.19-3.33 M vs 3.12-3.31 M).
// KDL_TUNE wgrad_big: 0 off, 1 3x3 only (default), 2 both -- the ResNet engine selects
// 2 when its weight-gradient stream is on (set_wgrad_big, before its workspaces
// are sized); else 128 or 64 per dimension.
int g_wgrad_big = tune_int("wgrad_big", -1);
// bwd (a BN-backward-apply G prologue, csrc/wgrad_dma.hip BWDG): its gx panels
// double G's LDS share, so N tiles of at most 128 with K tiles up to 256 (8 waves)
void wgrad_tiles(int N, int K, bool conv3, int* tn, int* tk, bool bwd = false) {
  if (bwd) {
    *tn = N % 128 == 0 ? 128 : 64;
    *tk = K % 256 == 0 ? 256 : K % 128 == 0 ? 128 : 64;
    return;
  }
  const int big = g_wgrad_big < 0 ? 1 : g_wgrad_big;
  if ((conv3 ? big >= 1 : big >= 2) && gemm_core_mode() != 0 && N % 256 == 0 && K % 256 == 0) {
    *tn = *tk = 256;
    return;
  }
  *tn = N % 128 == 0 ? 128 : 64;
  *tk = K % 128 == 0 ? 128 : 64;
}

int wgrad_splits(int M, int N, int K, bool conv3, bool bwd = false, bool solo = false) {
  int tn, tk;
  wgrad_tiles(N, K, conv3, &tn, &tk, bwd);
  const int tiles = (N / tn) * (K / tk);
  if (solo) {
    // nothing else on the GPU (the CTR tower): ~3 blocks per CU, at least 400
    // batch rows per split so the slab bytes stay below the GEMM's own
    // (batch 4096: 1024x1728 62 -> 40 us at 3 splits, 512x1024 best at 10,
    // 256x512 at 20 of 40; profiles/r04_ctr_tile_probe.txt)
    int splits = 768 / tiles, cap = M / 400;
    if (splits > cap) splits = cap;
    return splits < 1 ? 1 : splits;
  }
  // ~2 blocks per CU (one round): halves the slab bytes of 4 blocks/CU, measured +1.5% per step.
  // Rounded DOWN so the grid never spills a partial second round onto the CUs
  // (3x3 stage-4: 576 blocks = 1.125 rounds took 1.7x the time of 432).
  // 256 x 256 tiles hold one block per CU: half the blocks per round.
  // With the side stream's gradients overlapping the main stream, FEWER blocks
  // win: they leave CUs to the critical path (job step, same box, 256x256 tiles
  // at half the target: 1024 -> 12,460, 512 -> 12,830, 384 -> 13,047, 320 ->
  // 13,078, 256 -> 12,933, 192 -> 12,715 img/s; profiles/r02_wgrad_blocks_sweep.txt).
  // Re-swept on the round-4 step (kdl head, fewer stray launches): 384 wins,
  // 13,818-13,837 vs 13,666-13,756 at 320; 352 / 416 / 448 in between, 512
  // 13,636-13,674, 640 13,215-13,231 (profiles/r04_wgrad_blocks_resweep.txt).
  int target = tune_int("wgrad_blocks", 384);
  if (tn == 256 || (bwd && !(tn == 64 && tk == 64))) target /= 2;  // one (8-wave) block per CU
  int splits = target / tiles;
  const int max_splits = (M + WMK - 1) / WMK;
  if (splits > max_splits) splits = max_splits;
  return splits < 1 ? 1 : splits;
}

// slab capacity for either G mode (plain / BN-backward prologue)
int conv1x1_wgrad_splits(int M, int N, int K, bool solo) {
  const int a = wgrad_splits(M, N, K, false), b = wgrad_splits(M, N, K, false, true);
  const int c = solo ? wgrad_splits(M, N, K, false, false, true) : 0;
  return a > b ? (a > c ? a : c) : (b > c ? b : c);
}

// the caller's preference (an explicit KDL_TUNE wgrad_big wins)
void set_wgrad_big(int mode) {
  static const bool env = tune_has("wgrad_big");
  if (!env) g_wgrad_big = mode;
}

namespace {
template <int TN_, int TK_>
void launch_wgrad(dim3 grid, hipStream_t s, const bf16_t* g, const bf16_t* x, const float* pro, float* dw32, int M,
                  int N, int K, int Hout, int Wout, int Hin, int Win, int stride, int rps, int tiles_k, int mode,
                  int cin) {
#define WG_LAUNCH(P, G)                                                                                             \
  hipLaunchKernelGGL((wgrad1x1_kernel<TN_, TK_, P, G>), grid, dim3(kThreads), 0, s, g, x, pro, dw32, M, N, K, Hout, \
                     Wout, Hin, Win, stride, rps, tiles_k, cin)
  if (pro) {
    if (mode == G_CONV3) WG_LAUNCH(true, G_CONV3);
    else if (mode == G_STRIDED) WG_LAUNCH(true, G_STRIDED);
    else WG_LAUNCH(true, G_DENSE);
  } else {
    if (mode == G_CONV3) WG_LAUNCH(false, G_CONV3);
    else if (mode == G_STRIDED) WG_LAUNCH(false, G_STRIDED);
    else WG_LAUNCH(false, G_DENSE);
  }
#undef WG_LAUNCH
}
}  // namespace

namespace {
// Fixed-order sum of ``nsplit`` fp32 slabs into bf16 dW: one pass, or two when
// the columns alone would leave the chip idle (chunk partials first).
hipError_t wgrad_reduce(float* dw32, int64_t nk, int nsplit, float scale, bf16_t* dW, hipStream_t s,
                        int layout = 0) {
  // timing-only (KDL_TUNE price_wgrad_reduce=0): skip the slab reduce to price its
  // cost in the two-stream step (weight gradients are then garbage)
  static const bool skip = tune_int("price_wgrad_reduce", 1) == 0;
  if (skip) return hipSuccess;
  const int rgrid = static_cast<int>((nk / 4 + kRedCols - 1) / kRedCols);
  // y-blocks to reach ~KDL_TUNE wgrad_red_blocks (2048) blocks in the first pass
  static const int red_target = tune_int("wgrad_red_blocks", 2048);
  int groups = (red_target + rgrid - 1) / rgrid;
  const int by_work = (nsplit + 31) / 32;             // >= 2 slabs per thread in pass 1
  if (groups > by_work) groups = by_work;
  if (groups <= 1) {
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(rgrid), dim3(kThreads), 0, s, dw32, nk, nsplit, nsplit, 1, scale,
                       dW, layout);
    return hipGetLastError();
  }
  const int chunk = (nsplit + groups - 1) / groups;
  groups = (nsplit + chunk - 1) / chunk;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(rgrid, groups), dim3(kThreads), 0, s, dw32, nk, nsplit, chunk, 1,
                     1.0f, static_cast<bf16_t*>(nullptr), 0);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(rgrid), dim3(kThreads), 0, s, dw32, nk, groups, groups, chunk, scale,
                     dW, layout);
  return hipGetLastError();
}

// ------------------------------------------------------------------ Gram fold of a BN-backward weight gradient
// The weight gradient of a 1x1 conv whose output c = W a feeds a BN with
// backward coefficients (k, c1, c0) -- dc = k g + c1 c + c0 -- is
//   dW = dc^T a = diag(k) (g^T a) + diag(c1) W (a^T a) + c0 (1^T a)
// so dc never has to be materialised: G = g^T a on the weight-gradient kernel,
// Q = a^T a and s = 1^T a (a = relu(B(X)), the conv's prologued input) on the
// Gram kernel below, and this fold, all in fp32 (models/resnet_engine.py
// bn_bwd_fuse 3; the BN-backward apply's write-through of dc -- a 4C-channel
// tensor -- disappears from the data gradient).
// W Q is a small fp32 GEMM (N x K x K): 64 x 64 output tiles, 4 x 4 per thread,
// j in chunks of 16 staged through LDS (a per-output K-long dependent-load loop
// took 40 us at N = 256, K = 64).  N, K multiples of 64.
constexpr int kFoldJ = 16;
__global__ __launch_bounds__(256) void gram_fold_kernel(const float* __restrict__ Gm, const float* __restrict__ QS,
                                                        const bf16_t* __restrict__ W, const float* __restrict__ bcoef,
                                                        int N, int K, bf16_t* __restrict__ out) {
  __shared__ float Ws[kFoldJ][64 + 4];  // [j][n]
  __shared__ __attribute__((aligned(16))) float Qs[kFoldJ][64];  // [j][k]
  const int n0 = blockIdx.y * 64, k0 = blockIdx.x * 64;
  const int t = threadIdx.x, tn = (t >> 4) * 4, tk = (t & 15) * 4;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[i][q] = 0.f;
  const int wr = t >> 2, wc = (t & 3) * 4;   // W: row n0 + wr, j0 + wc .. +3
  const int qr = t >> 4, qc = (t & 15) * 4;  // Q: row j0 + qr, k0 + qc .. +3
  for (int j0 = 0; j0 < K; j0 += kFoldJ) {
    const bf16_t* w = W + static_cast<int64_t>(n0 + wr) * K + j0 + wc;
#pragma unroll
    for (int q = 0; q < 4; ++q) Ws[wc + q][wr] = bf16_to_f32(w[q]);
    *reinterpret_cast<float4*>(&Qs[qr][qc]) =
        *reinterpret_cast<const float4*>(QS + static_cast<int64_t>(j0 + qr) * K + k0 + qc);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kFoldJ; ++j) {
      const float4 b = *reinterpret_cast<const float4*>(&Qs[j][tk]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float a = Ws[j][tn + i];
        acc[i][0] = fmaf(a, b.x, acc[i][0]);
        acc[i][1] = fmaf(a, b.y, acc[i][1]);
        acc[i][2] = fmaf(a, b.z, acc[i][2]);
        acc[i][3] = fmaf(a, b.w, acc[i][3]);
      }
    }
    __syncthreads();
  }
  const float* colsum = QS + static_cast<int64_t>(K) * K;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + tn + i;
    const float kc = bcoef[n], c1 = bcoef[N + n], c0 = bcoef[2 * N + n];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = k0 + tk + q;
      const int64_t idx = static_cast<int64_t>(n) * K + k;
      out[idx] = f32_to_bf16(kc * Gm[idx] + c1 * acc[i][q] + c0 * colsum[k]);
    }
  }
}

// Q = a^T a and s = 1^T a of a dense [M][T] operand (T = K = 64 or 128: one
// output tile, on the diagonal): each staged row feeds BOTH MFMA operands, and
// all 256 threads stage (one 8-row x 8-channel unit each per R-row step, R = 256
// x 64 / T) -- the generic weight-gradient kernel staged the same rows twice
// from half its threads and sat latency-bound at ~0.5 TB/s.  A block's rows are
// its own contiguous range (nothing to share through an XCD's L2).
template <int T>
__global__ __launch_bounds__(kThreads, 2) void gram_kernel(const bf16_t* __restrict__ X,
                                                           const float* __restrict__ pro, float* __restrict__ ws,
                                                           int M, int rows_per_split) {
  constexpr int R = kThreads * 64 / T;  // rows per step
  constexpr int LDR = R + 8;
  constexpr int kBuf = T * LDR;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * kBuf];
  constexpr int WT = T / 2, F = WT / 32;  // 2 x 2 waves
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int split = blockIdx.x;
  const int mbeg = split * rows_per_split;
  const int mend = min(M, mbeg + rows_per_split);
  constexpr int cpr = T / 8;
  const int mg = t / cpr, cc = (t % cpr) * 8;
  float psc[8], psf[8], csum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    psc[j] = pro[cc + j];
    psf[j] = pro[T + cc + j];
    csum[j] = 0.f;
  }
  uint4 rr[8];
  auto gload = [&](int m0) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int m1 = m0 + mg * 8 + r;
      rr[r] = ld16(X + static_cast<int64_t>(m1 < mend ? m1 : mbeg) * T + cc);
    }
  };
  auto swrite = [&](int buf, int m0) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      float f[8];
      unpack8(rr[r], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float o = fmaf(f[j], psc[j], psf[j]);
        f[j] = o > 0.f ? o : 0.f;
      }
      rr[r] = m0 + mg * 8 + r < mend ? pack8(f) : make_uint4(0, 0, 0, 0);
      unpack8(rr[r], f);  // the bf16 values the MFMAs see
#pragma unroll
      for (int j = 0; j < 8; ++j) csum[j] += f[j];
    }
    uint4 tr[8];
    transpose8x8(rr, tr);
    bf16_t* S = lds + buf * kBuf;
#pragma unroll
    for (int c = 0; c < 8; ++c) *reinterpret_cast<uint4*>(&S[(cc + c) * LDR + mg * 8]) = tr[c];
  };
  const int wn0 = (wave >> 1) * WT, wk0 = (wave & 1) * WT;
  const int fr = lane & 31, fh = lane >> 5;
  f32x16_t acc[F][F];
#pragma unroll
  for (int i = 0; i < F; ++i)
#pragma unroll
    for (int j = 0; j < F; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  int cur = 0;
  if (mbeg < mend) {
    gload(mbeg);
    swrite(0, mbeg);
  }
  __syncthreads();
  for (int m0 = mbeg; m0 < mend; m0 += R) {
    const bool more = m0 + R < mend;
    if (more) gload(m0 + R);
    const bf16_t* S = lds + cur * kBuf;
#pragma unroll
    for (int s = 0; s < R / 16; ++s) {
      bf16x8_t gf[F], af[F];
#pragma unroll
      for (int i = 0; i < F; ++i) {
        gf[i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(&S[(wn0 + i * 32 + fr) * LDR + s * 16 + fh * 8]));
        af[i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(&S[(wk0 + i * 32 + fr) * LDR + s * 16 + fh * 8]));
      }
#pragma unroll
      for (int i = 0; i < F; ++i)
#pragma unroll
        for (int j = 0; j < F; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gf[i], af[j], acc[i][j], 0, 0, 0);
    }
    if (more) swrite(cur ^ 1, m0 + R);
    __syncthreads();
    cur ^= 1;
  }
  float* slab = ws + static_cast<int64_t>(split) * (T * T + T);
  // column sums: fold the R/8 row groups through LDS (the loop's last barrier freed it)
  float* cs = reinterpret_cast<float*>(lds);  // [R / 8][T]
#pragma unroll
  for (int j = 0; j < 8; ++j) cs[mg * T + cc + j] = csum[j];
  __syncthreads();
  if (t < T) {
    float v = 0.f;
    for (int g = 0; g < R / 8; ++g) v += cs[g * T + t];
    slab[T * T + t] = v;
  }
#pragma unroll
  for (int i = 0; i < F; ++i)
#pragma unroll
    for (int j = 0; j < F; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = wn0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        const int k = wk0 + j * 32 + fr;
        slab_store(slab + n * T + k, acc[i][j][r]);
      }
}

int gram_tile(int K) { return K % 128 == 0 ? 128 : 64; }
bool gram_dedicated(int K) { return K == 64 || K == 128; }

}  // namespace

int conv1x1_gram_splits(int M, int K) {
  if (gram_dedicated(K)) {
    // ~2 blocks per CU at K = 64; half that at 128, whose 66 KB slabs would
    // otherwise rival the operand's own bytes (KDL_TUNE gram_blocks)
    static const int target = tune_int("gram_blocks", 512);
    const int R = kThreads * 64 / K;
    int splits = K == 64 ? target : target / 2;
    const int max_splits = (M + R - 1) / R;
    if (splits > max_splits) splits = max_splits;
    return splits < 1 ? 1 : splits;
  }
  const int t = gram_tile(K), tiles = (K / t) * (K / t);
  int splits = tune_int("wgrad_blocks", 384) / 2 / tiles;  // half the weight-gradient block target
  const int max_splits = (M + WMK - 1) / WMK;
  if (splits > max_splits) splits = max_splits;
  return splits < 1 ? 1 : splits;
}

hipError_t conv1x1_gram(const void* X, const float* pro, float* ws, int M, int K, hipStream_t s) {
  if (K % 64 || M <= 0 || K > 512 || !pro) return hipErrorInvalidValue;
  const bf16_t* x = static_cast<const bf16_t*>(X);
  if (gram_dedicated(K)) {
    const int R = kThreads * 64 / K;
    const int splits = conv1x1_gram_splits(M, K);
    int rps = (M + splits - 1) / splits;
    rps = (rps + R - 1) / R * R;
    const int nsplit = (M + rps - 1) / rps;
    if (K == 64)
      hipLaunchKernelGGL(gram_kernel<64>, dim3(nsplit), dim3(kThreads), 0, s, x, pro, ws, M, rps);
    else
      hipLaunchKernelGGL(gram_kernel<128>, dim3(nsplit), dim3(kThreads), 0, s, x, pro, ws, M, rps);
    RETURN_IF_HIP_ERR(hipGetLastError());
    return wgrad_reduce(ws, static_cast<int64_t>(K) * K + K, nsplit, 1.f, nullptr, s);
  }
  const int t = gram_tile(K), tiles_k = K / t;
  const int splits = conv1x1_gram_splits(M, K);
  int rps = (M + splits - 1) / splits;
  rps = (rps + WMK - 1) / WMK * WMK;
  const int nsplit = (M + rps - 1) / rps;
  dim3 grid(nsplit * tiles_k * tiles_k);
  if (t == 128)
    hipLaunchKernelGGL((wgrad1x1_kernel<128, 128, true, G_DENSE, true, true>), grid, dim3(kThreads), 0, s, x, x, pro,
                       ws, M, K, K, 0, 0, 0, 0, 1, rps, tiles_k, K);
  else
    hipLaunchKernelGGL((wgrad1x1_kernel<64, 64, true, G_DENSE, true, true>), grid, dim3(kThreads), 0, s, x, x, pro,
                       ws, M, K, K, 0, 0, 0, 0, 1, rps, tiles_k, K);
  RETURN_IF_HIP_ERR(hipGetLastError());
  return wgrad_reduce(ws, static_cast<int64_t>(K) * K + K, nsplit, 1.f, nullptr, s);  // fp32, in slab 0
}

hipError_t gram_fold(const float* Gm, const float* QS, const void* W, const float* bcoef, int N, int K, void* out,
                     hipStream_t s) {
  if (N <= 0 || K <= 0 || N % 64 || K % 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gram_fold_kernel, dim3(K / 64, N / 64), dim3(256), 0, s, Gm, QS,
                     static_cast<const bf16_t*>(W), bcoef, N, K, static_cast<bf16_t*>(out));
  return hipGetLastError();
}

hipError_t wgrad_slab_reduce(float* dw32, int64_t nk, int nsplit, float scale, void* dW, hipStream_t s,
                             int layout) {
  return wgrad_reduce(dw32, nk, nsplit, scale, static_cast<bf16_t*>(dW), s, layout);
}

namespace {
// big: the workspace holds wgrad_splits(M, N, K, true) slabs (3x3 256-tile configs)
hipError_t wgrad_impl(const void* G, const void* A, const float* pro_coef, float* dw32, void* dW, float scale,
                      int M, int N, int K, int Hout, int Wout, int Hin, int Win, int stride, int mode, int cin,
                      hipStream_t s, bool big = false, const void* gx = nullptr, const float* gcoef = nullptr,
                      bool solo = false) {
  if (N % 64 || K % 64 || M <= 0) return hipErrorInvalidValue;
  const bool bwd = gx != nullptr;
  // the G prologue exists on the LDS-DMA kernel only
  if (bwd && (gemm_core_mode() == 0 || !gcoef || mode == G_CONV3 || (pro_coef && mode != G_DENSE)))
    return hipErrorInvalidValue;
  int tn, tk;
  wgrad_tiles(N, K, big, &tn, &tk, bwd);
  const int splits = wgrad_splits(M, N, K, big, bwd, solo && !bwd && !big);
  int rps = (M + splits - 1) / splits;
  rps = (rps + WMK - 1) / WMK * WMK;
  int tiles_k = K / tk;
  const int nsplit = (M + rps - 1) / rps;
  dim3 grid(nsplit * (N / tn) * tiles_k);
  const bf16_t* g = static_cast<const bf16_t*>(G);
  const bf16_t* x = static_cast<const bf16_t*>(A);
  bool done = false;
  if (gemm_core_mode() != 0) {  // LDS-DMA pipeline (csrc/wgrad_dma.hip) unless forced off
    WgParams wp{};
    wp.G = g; wp.A = x; wp.pro = pro_coef; wp.dw32 = dw32;
    wp.gx = static_cast<const bf16_t*>(gx); wp.gcoef = gcoef;
    wp.M = M; wp.N = N; wp.K = K; wp.Hout = Hout; wp.Wout = Wout; wp.Hin = Hin; wp.Win = Win;
    wp.stride = stride; wp.cin = cin; wp.rps = rps; wp.tiles_k = tiles_k; wp.mode = mode;
    wp.a_rows = mode == G_DENSE ? M : static_cast<int64_t>(M / (Hout * Wout)) * Hin * Win;
    if (mode != G_DENSE) {
      wp.mg_hw = static_cast<uint32_t>(((uint64_t(1) << 32) + Hout * Wout - 1) / (Hout * Wout));
      wp.mg_w = static_cast<uint32_t>(((uint64_t(1) << 32) + Wout - 1) / Wout);
    }
    const hipError_t e = wgrad_dma(wp, nsplit, tn, tk, s);
    if (e != hipSuccess && e != hipErrorInvalidValue) return e;
    done = e == hipSuccess;
  }
  if (!done && bwd) return hipErrorInvalidValue;
  if (!done) {
    if (tn > 128 || tk > 128) {  // the register-staged kernel has no 256 tiles: same splits, 128 tiles
      tn = tk = 128;
      tiles_k = K / tk;
      grid = dim3(nsplit * (N / tn) * tiles_k);
    }
    if (tn == 128 && tk == 128) launch_wgrad<128, 128>(grid, s, g, x, pro_coef, dw32, M, N, K, Hout, Wout, Hin, Win, stride, rps, tiles_k, mode, cin);
    else if (tn == 128) launch_wgrad<128, 64>(grid, s, g, x, pro_coef, dw32, M, N, K, Hout, Wout, Hin, Win, stride, rps, tiles_k, mode, cin);
    else if (tk == 128) launch_wgrad<64, 128>(grid, s, g, x, pro_coef, dw32, M, N, K, Hout, Wout, Hin, Win, stride, rps, tiles_k, mode, cin);
    else launch_wgrad<64, 64>(grid, s, g, x, pro_coef, dw32, M, N, K, Hout, Wout, Hin, Win, stride, rps, tiles_k, mode, cin);
    RETURN_IF_HIP_ERR(hipGetLastError());
  }
  return wgrad_reduce(dw32, static_cast<int64_t>(N) * K, nsplit, scale, static_cast<bf16_t*>(dW), s);
}
}  // namespace

hipError_t conv1x1_wgrad(const void* G, const void* A, const float* pro_coef, float* dw32, void* dW, float scale,
                         int M, int N, int K, int Hout, int Wout, int Hin, int Win, int stride, hipStream_t s,
                         const void* gx, const float* gcoef, bool solo) {
  return wgrad_impl(G, A, pro_coef, dw32, dW, scale, M, N, K, Hout, Wout, Hin, Win, stride,
                    stride > 1 ? G_STRIDED : G_DENSE, K, s, false, gx, gcoef, solo);
}

int conv3x3_wgrad_slabs(int Nb, int Hin, int Win, int Cin, int Cout, int stride) {
  const int Ho = (Hin - 1) / stride + 1, Wo = (Win - 1) / stride + 1;
  const int M = Nb * Ho * Wo;
  const int a = conv1x1_wgrad_splits(M, Cout, 9 * Cin), b = wgrad_splits(M, Cout, 9 * Cin, true);
  const int dflt = a > b ? a : b;
  const int halo = halo3x3_wgrad_slabs(Nb, Hin, Win, Cin, Cout, stride);
  return halo > dflt ? halo : dflt;
}

hipError_t conv3x3_wgrad(const void* G, const void* A, const float* pro_coef, float* dw32, int64_t dw32_floats,
                         void* dW, float scale, int Nb, int Hin, int Win, int Cin, int Cout, int stride,
                         hipStream_t s) {
  if (Cin % 64 || Cout % 64 || Nb <= 0 || stride < 1) return hipErrorInvalidValue;
  if (gemm_core_mode() != 0) {  // 56x56 stage: input halo staged once per tile (csrc/halo3x3.hip)
    int nslabs = 0;
    const hipError_t e = halo3x3_wgrad(G, A, pro_coef, dw32, dw32_floats, Nb, Hin, Win, Cin, Cout, stride, &nslabs, s);
    if (e == hipSuccess)
      return wgrad_reduce(dw32, static_cast<int64_t>(Cout) * 9 * Cin, nslabs, scale, static_cast<bf16_t*>(dW), s);
    if (e != hipErrorInvalidValue) return e;
  }
  const int Ho = (Hin - 1) / stride + 1, Wo = (Win - 1) / stride + 1;
  const int M = Nb * Ho * Wo;
  // 256 x 256 tiles only when the caller's workspace holds their slab count
  // (conv3x3_wgrad_slabs); a conv1x1_wgrad_splits-sized one keeps 128 tiles
  const bool big = dw32_floats >= static_cast<int64_t>(wgrad_splits(M, Cout, 9 * Cin, true)) * Cout * 9 * Cin;
  return wgrad_impl(G, A, pro_coef, dw32, dW, scale, M, Cout, 9 * Cin, Ho, Wo, Hin, Win, stride, G_CONV3, Cin, s,
                    big);
}

}  // namespace kdl
