// Fused epilogues of the ResNet conv GEMMs, shared by both GEMM main loops
// (csrc/conv1x1.hip: register-staged, short K; csrc/igemm.hip: LDS-DMA
// staged, long K and 3x3 implicit GEMM).
//
// Both kernels finish an output tile the same way: the fp32 accumulators are
// rounded to bf16 into an LDS tile Cs[BM][BN + 8] (row = output pixel m,
// column = output channel n), then every thread owns one 8-channel column
// chunk and walks the tile's rows with 16-byte vectors, applying
//   PLAIN    store as is
//   STATS    + per-channel shifted sums sum(y - s), sum((y - s)^2) (BN forward
//            statistics of the conv output: no separate stats pass)
//   MASKX    dgrad of a layer that follows a BN+ReLU: g' = g * [x*a + b > 0]
//            (mask recomputed from the BN input x) + the BN backward sums
//            sum(g'), sum(g' (x - mean))
//   RESBITS  g = dgrad + d(identity) (optionally stride-gathered), masked by
//            the previous block's packed ReLU bits, + bn3 (and downsample BN)
//            backward sums
//   RES      g = dgrad + d(identity), no mask (network stem)
//   BIAS / BIAS_RELU  y = [relu](c + bias[n]) (the CTR tower's dense layers,
//            csrc/ctr.hip gemm_bias_act; bias fp32 in ``shift`` or bf16 in
//            ``bias16``; c is the bf16-rounded accumulator)
// and after its last tile folds the per-thread sums in LDS and adds them to
// the BN workspace replica of the block (one atomic per channel per block).
#pragma once

#include "bn_fin.h"
#include "common.h"

namespace kdl {
namespace gemm {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(2))) float f2_t;

constexpr int kRep = 32;  // replica count of the BN workspace (== bn_act.hip kReplicas)

enum { EPI_PLAIN = 0, EPI_STATS = 1, EPI_MASKX = 2, EPI_RESBITS = 3, EPI_RES = 4, EPI_BIAS = 5, EPI_BIAS_RELU = 6 };
// A-row addressing: dense rows | stride-s 1x1 gather | 3x3 implicit GEMM (pad 1, stride s) |
// data gradient of a stride-2 3x3 pad-1 conv as four sub-pixel class GEMMs (csrc/igemm.hip)
// G_STEM (csrc/stem.hip): a tile is 2 output rows x 112 columns of one image
// (column chunk cc of ceil(OW / 112)); GEMM row m = 224 tile + l maps to output
// pixel (2 tr + l / 112, 112 cc + l % 112), masked past OH / OW.  Params: Hout
// = OH, Wout = OW, Hin = tile rows per image (ceil(OH / 2)), Win = column chunks.
enum { G_DENSE = 0, G_STRIDED = 1, G_CONV3 = 2, G_DGRAD2 = 3, G_STEM = 4 };

struct GemmParams {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;
  int M, N, K;
  // A row gather (stride-s 1x1 conv): out row (n, oh, ow) reads in row (n, oh*s, ow*s)
  int Hout, Wout, Hin, Win, stride;
  int Cin;                // GATHER == G_CONV3: channels per tap (K = 9 * Cin, Cin % 64 == 0)
  int64_t a_rows;         // rows of the A tensor (buffer bounds of the LDS-DMA loads)
  const float* pro_coef;  // [2K] (3x3: [2Cin]): scale | shift
  // BN-backward-apply prologue of A (register-staged dense GEMM only):
  //   A' = bf16(k[c] A + c1[c] bx + c0[c])  -- the same fmaf nesting and rounding
  // as the standalone apply pass (csrc/bn_act.hip bn_bwd_apply_kernel), so A'
  // is bit-identical to the tensor that pass would have written.
  const bf16_t* bx;       // that BN's input x [M, K]
  const float* bcoef;     // [3K] k | c1 | c0 (the BN workspace's backward coefficients)
  const float* bcoef2;    // PRO_RES2: the downsample BN's [2K] scale | shift (LDS after bcoef's [2K])
  bf16_t* aout;           // optional write-through of A' [M, K] (the blocks of output tile 0)
  // epilogue operands
  const float* shift;   // STATS: [N]; BIAS: fp32 bias [N] (or null)
  const bf16_t* bias16; // BIAS: bf16 bias [N] (when shift is null; both null: no bias)
  float* acc;           // STATS/MASKX/RESBITS: [kRep][2N]
  const bf16_t* ex;     // MASKX/RESBITS: BN input x [M, N]
  const float* emean;   // [N]
  const float* ecoef;   // MASKX: [2N] forward scale | shift of that BN
  const bf16_t* eres;   // RESBITS/RES: d(identity)
  int res_stride;       // 1: eres is [M, N]; s > 1: eres is [Nb, Hin/s.., N] sampled at (h%s==0, w%s==0)
  int res_H, res_W;     // geometry of the C rows (= input resolution) for the strided residual
  const uint8_t* ebits; // RESBITS: [M, N/8]
  const bf16_t* ex2;    // RESBITS: optional second BN input (downsample BN)
  const float* emean2;
  float* acc2;          // its replicas [kRep][2N]
  int price_drop;       // timing-only builds (KDL_TUNE igemm_price): bit 0 drops A's loads, bit 1 B's
  // G_DGRAD2: A = dy [Nb, Hin, Win, Cin] (Hin x Win = each class's pixel grid),
  // C = dx [Nb, Hout = 2 Hin (or 2 Hin - 1), Wout = 2 Win (or 2 Win - 1), N]; class c = 2 py + px owns the
  // dx pixels (2i + py, 2j + px).  mc = Nb Hin Win rows per class, padded to
  // mc_pad (a multiple of BM, set by the launcher); M = 4 mc_pad.
  int mc, mc_pad;
  // BN finalize folded into this GEMM (csrc/bn_fin.h): the workspace of the BN
  // whose sums the epilogue produces (second one: RESBITS' downsample BN), and
  // that BN's element count; null = the host launches the finalize
  float* fin_ws;
  float* fin_ws2;
  float fin_M;
  uint8_t* obits;      // PRO_RES / PRO_RES2 write-through: packed ReLU mask [M, N/8] (out)
};

// csrc/wgrad_dma.hip: weight gradient on the LDS-DMA pipeline into fp32
// slabs dw32[split][N][K] (rps % 64 == 0; tn, tk in {64, 128}).
struct WgParams {
  const bf16_t* G;        // [M][N] output gradient
  const bf16_t* A;        // layer input rows (gathered per mode)
  const float* pro;       // optional BN+ReLU prologue of A: [2 * lda] scale | shift
  // optional BN-backward-apply prologue of G: G' = k[n] G + c1[n] gx + c0[n]
  // (GemmParams::bx / bcoef semantics, per output channel n)
  const bf16_t* gx;       // [M][N]
  const float* gcoef;     // [3N]
  float* dw32;
  int M, N, K;            // K = 9 * cin for 3x3
  int Hout, Wout, Hin, Win, stride, cin;
  int rps, tiles_k, mode; // rows per split, K tiles, G_DENSE | G_STRIDED | G_CONV3
  int64_t a_rows;         // rows of the A tensor (buffer bounds)
  // n / d == umulhi(n, ceil(2^32 / d)) for n * d < 2^32 (host-checked): the
  // per-row image coordinates without integer division in the main loop
  uint32_t mg_hw, mg_w;   // magic multipliers of Hout * Wout and Wout
};
hipError_t wgrad_dma(const WgParams& p, int nsplit, int tn, int tk, hipStream_t s);

// csrc/igemm.hip: LDS-DMA main loop (no A prologue); cfg from igemm_pick.
// Requires K % 64 == 0 (3x3: Cin % 64 == 0) and 32-bit operand byte offsets.
int igemm_pick(int M, int N, int K);
bool g_forced_cfg_unset();  // no KDL_TUNE igemm_cfg / set_igemm_cfg override in force
hipError_t igemm(const GemmParams& p, int epi, int gather, int cfg, hipStream_t s);
// n zeroed ticket counters for one launch, from a per-device ring (self-resetting:
// every kernel that draws from them leaves them zero); null while a stream capture
// is under way on a device whose ring does not exist yet
// csrc/halo3x3.hip: 3x3 stride-1 conv with an LDS-resident input halo (Cin 64 @ 56x56);
// hipErrorInvalidValue when the geometry is not one it serves
hipError_t halo3x3(const GemmParams& p, int epi, hipStream_t s);
// its weight gradient (optional BN + ReLU prologue on A: pro = [scale | shift])
// into one fp32 [64][576] slab per block (*nslabs)
int halo3x3_wgrad_slabs(int Nb, int Hin, int Win, int Cin, int Cout, int stride);
hipError_t halo3x3_wgrad(const void* G, const void* A, const float* pro, float* dw32, int64_t dw32_floats, int Nb,
                         int Hin, int Win, int Cin, int Cout, int stride, int* nslabs, hipStream_t s);

__device__ __forceinline__ uint4 ld16(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }

__device__ __forceinline__ void unpack8(const uint4 v, float (&o)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// packed-fp32 pairs: v_pk_add_f32 / v_pk_fma_f32 halve the epilogue VALU count
__device__ __forceinline__ void unpack4x2(const uint4 v, f2_t (&o)[4]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f2_t{__uint_as_float(w[i] << 16), __uint_as_float(w[i] & 0xffff0000u)};
}

__device__ __forceinline__ uint32_t pack2(const f2_t v) { return pack_bf16x2(v.x, v.y); }

__device__ __forceinline__ f2_t pfma(const f2_t a, const f2_t b, const f2_t c) {
  return __builtin_elementwise_fma(a, b, c);
}

__device__ __forceinline__ uint4 pack8(const float (&o)[8]) {
  return make_uint4(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]), pack_bf16x2(o[4], o[5]),
                    pack_bf16x2(o[6], o[7]));
}

__device__ __forceinline__ void atomic_add_f32(float* p, float v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// D[n][m] of a 32x32x16 MFMA with the weight fragment as the A operand: lane
// (fr, fh) holds column m = fr, rows n = (r&3) + 8(r>>2) + 4fh -- 4 runs of 4
// consecutive channels, written as 8-byte bf16 pairs into Cs[m][n].
template <int TN, int TM>
__device__ __forceinline__ void acc_to_lds(const f32x16_t (&acc)[TN][TM], bf16_t* Cs, int ldc, int wm0, int wn0,
                                           int lane) {
  const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int m = wm0 + j * 32 + fr;
        const int n = wn0 + i * 32 + 8 * g + 4 * fh;
        const uint32_t lo = pack_bf16x2(acc[i][j][4 * g], acc[i][j][4 * g + 1]);
        const uint32_t hi = pack_bf16x2(acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
        *reinterpret_cast<uint2*>(&Cs[m * ldc + n]) = make_uint2(lo, hi);
      }
}

template <int BM, int BN, int NT, int EPI, int GATHER = G_DENSE>
struct Epilogue {
  static constexpr int LDC = BN + 8;
  static constexpr int CPR = BN / 8;           // 16-B chunks per output row
  static constexpr int RPP = NT / CPR;         // rows per epilogue pass
  static constexpr int NP = BM / RPP;          // rows per thread per tile
  // prefetch group (4 rows where 8 spill: RESBITS, and MASKX beside the 256x256 tile's 128 accumulators)
  static constexpr int PG = (EPI == EPI_RESBITS || (EPI == EPI_MASKX && BM * BN >= 256 * 256))
                                ? (NP > 4 ? 4 : NP) : (NP > 8 ? 8 : NP);
  static constexpr bool LX = EPI == EPI_MASKX || EPI == EPI_RESBITS;  // the BN input x
  static constexpr bool LR = EPI == EPI_RESBITS || EPI == EPI_RES;
  // RESBITS' optional second BN input (downsample branch)
  static constexpr bool X2 = EPI == EPI_RESBITS;
  static constexpr bool REDUCE = EPI == EPI_STATS || EPI == EPI_MASKX || EPI == EPI_RESBITS;
  // LDS scratch of finish(): 3 sums x NT threads x 8 channels
  static constexpr int kScratchBytes = REDUCE ? 3 * NT * 8 * 4 : 0;
  static_assert(NT % CPR == 0 && BM % RPP == 0 && NP % PG == 0, "epilogue geometry");

  int t, ec, er0, ch0, n0;
  f2_t s1[4], s2[4], s3[4];
  uint4 pxv[PG], prv[PG], px2[PG];
  uint32_t pbv[PG];
  bool prok[PG];

  __device__ __forceinline__ void init(int t_, int n0_) {
    t = t_;
    n0 = n0_;
    ec = t % CPR;
    er0 = t / CPR;
    ch0 = n0 + ec * 8;
#pragma unroll
    for (int q = 0; q < 4; ++q) { s1[q] = f2_t{0.f, 0.f}; s2[q] = s1[q]; s3[q] = s1[q]; }
  }

  // output row of GEMM row m (-1: padding row past M / past a class's rows)
  __device__ __forceinline__ int row_of(const GemmParams& p, int m) const {
    if constexpr (GATHER == G_STEM) {
      if (p.Wout == 112 && (p.Hout & 1) == 0) return m < p.M ? m : -1;  // 224-px images: identity
      const int tm = m / 224, l = m - tm * 224;
      const int per = p.Hin * p.Win, img = tm / per, rem = tm - img * per;
      const int tr = rem / p.Win, cc = rem - tr * p.Win;
      const int oh = 2 * tr + (l >= 112 ? 1 : 0), ow = 112 * cc + (l >= 112 ? l - 112 : l);
      if (oh >= p.Hout || ow >= p.Wout) return -1;
      return (img * p.Hout + oh) * p.Wout + ow;
    } else if constexpr (GATHER == G_DGRAD2) {
      const int cls = m / p.mc_pad, r = m - cls * p.mc_pad;
      if (r >= p.mc) return -1;
      const int hw = p.Hin * p.Win;
      const int nimg = r / hw, rem = r - nimg * hw;
      const int i = rem / p.Win, j = rem - i * p.Win;
      const int oh = 2 * i + (cls >> 1), ow = 2 * j + (cls & 1);
      if (oh >= p.Hout || ow >= p.Wout) return -1;  // odd input size: the last sub-pixel row / column
      return (nimg * p.Hout + oh) * p.Wout + ow;
    } else {
      return m < p.M ? m : -1;
    }
  }

  // row-side operands (BN input x, d(identity), mask bits) of rows g0.. of tile tm
  __device__ __forceinline__ void prefetch(const GemmParams& p, int tm, int g0) {
#pragma unroll
    for (int i = 0; i < PG; ++i) {
      const int m = row_of(p, tm * BM + (g0 + i) * RPP + er0);
      const bool ok = m >= 0;
      const int64_t go = static_cast<int64_t>(ok ? m : 0) * p.N + ch0;
      if constexpr (LX) pxv[i] = ok ? ld16(p.ex + go) : make_uint4(0, 0, 0, 0);
      if constexpr (EPI == EPI_RESBITS) {
        pbv[i] = ok ? p.ebits[static_cast<int64_t>(m) * (p.N / 8) + (ch0 >> 3)] : 0u;
        if constexpr (X2) px2[i] = (ok && p.ex2) ? ld16(p.ex2 + go) : make_uint4(0, 0, 0, 0);
      }
      if constexpr (LR) {
        const bf16_t* rp = nullptr;
        if (ok) {
          if (p.res_stride == 1) {
            rp = p.eres + go;
          } else {
            const int hw = p.res_H * p.res_W;
            const int nimg = m / hw, rem = m - nimg * hw;
            const int h = rem / p.res_W, w = rem - h * p.res_W;
            if (h % p.res_stride == 0 && w % p.res_stride == 0) {
              const int Ho = (p.res_H + p.res_stride - 1) / p.res_stride;
              const int Wo = (p.res_W + p.res_stride - 1) / p.res_stride;
              rp = p.eres + ((static_cast<int64_t>(nimg) * Ho + h / p.res_stride) * Wo + w / p.res_stride) * p.N + ch0;
            }
          }
        }
        prok[i] = rp != nullptr;
        prv[i] = rp ? ld16(rp) : make_uint4(0, 0, 0, 0);
      }
    }
  }

  // issue the first prefetch group and this thread's per-channel epilogue
  // coefficients before the accumulators go to LDS, so their latency overlaps
  // the LDS round trip (a coefficient load issued in rows() stalls the whole
  // epilogue on one dependent global load per tile)
  // (reload = false: the caller loaded them once with coefs() and keeps them
  // live across tiles)
  __device__ __forceinline__ void begin(const GemmParams& p, int tm, bool reload = true) {
    if constexpr (LX || LR) prefetch(p, tm, 0);
    if (reload) coefs(p);
  }

  f2_t ea[4], eb[4], em[4], em2[4];  // per-channel coefficients of this thread's 8 channels

  __device__ __forceinline__ void coefs(const GemmParams& p) {
#pragma unroll
    for (int q = 0; q < 4; ++q) { ea[q] = f2_t{0.f, 0.f}; eb[q] = ea[q]; em[q] = ea[q]; em2[q] = ea[q]; }
    auto ld2 = [](const float* src, int c) { return *reinterpret_cast<const f2_t*>(src + c); };
    const int N = p.N;
    if constexpr (EPI == EPI_STATS) {
#pragma unroll
      for (int q = 0; q < 4; ++q) em[q] = ld2(p.shift, ch0 + 2 * q);
    } else if constexpr (EPI == EPI_MASKX) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        em[q] = ld2(p.emean, ch0 + 2 * q);
        ea[q] = ld2(p.ecoef, ch0 + 2 * q);
        eb[q] = ld2(p.ecoef, N + ch0 + 2 * q);
      }
    } else if constexpr (EPI == EPI_RESBITS) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        em[q] = ld2(p.emean, ch0 + 2 * q);
        if (p.ex2) em2[q] = ld2(p.emean2, ch0 + 2 * q);
      }
    } else if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) {
      if (p.shift) {
#pragma unroll
        for (int q = 0; q < 4; ++q) ea[q] = ld2(p.shift, ch0 + 2 * q);
      } else if (p.bias16) {
        f2_t b[4];
        unpack4x2(ld16(p.bias16 + ch0), b);
#pragma unroll
        for (int q = 0; q < 4; ++q) ea[q] = b[q];
      }
    }
  }

  // the tile's rows, from Cs[BM][LDC] (after a barrier that follows acc_to_lds)
  __device__ __forceinline__ void rows(const GemmParams& p, const bf16_t* Cs, int tm) {
    const int N = p.N;
#pragma unroll
    for (int g0 = 0; g0 < NP; g0 += PG) {
      uint4 cxv[PG], crv[PG], cx2[PG];
      uint32_t cbv[PG];
      bool crok[PG];
#pragma unroll
      for (int i = 0; i < PG; ++i) { cxv[i] = pxv[i]; crv[i] = prv[i]; cx2[i] = px2[i]; cbv[i] = pbv[i]; crok[i] = prok[i]; }
      (void)cxv; (void)crv; (void)cx2; (void)cbv; (void)crok;
      if constexpr (LX || LR) {
        if (g0 + PG < NP) prefetch(p, tm, g0 + PG);
      }
#pragma unroll
      for (int i = 0; i < PG; ++i) {
        const int row = (g0 + i) * RPP + er0;
        const int m = row_of(p, tm * BM + row);
        if (m < 0) continue;
        const uint4 raw = *reinterpret_cast<const uint4*>(&Cs[row * LDC + ec * 8]);
        const int64_t go = static_cast<int64_t>(m) * N + ch0;
        uint4 xin = make_uint4(0, 0, 0, 0);  // MASKX / RESBITS: the BN input x of this row chunk
        (void)xin;
        if constexpr (LX) xin = cxv[i];
        uint4 out = raw;  // PLAIN / STATS store the tile as it is
        if constexpr (EPI != EPI_PLAIN) {
          f2_t v[4];
          unpack4x2(raw, v);
          uint32_t o[4];
          if constexpr (EPI == EPI_STATS) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const f2_t d = v[q] - em[q];
              s1[q] += d;
              s2[q] = pfma(d, d, s2[q]);
            }
          } else if constexpr (EPI == EPI_MASKX) {
            f2_t x[4];
            unpack4x2(xin, x);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const f2_t z = pfma(x[q], ea[q], eb[q]);
              const f2_t g = f2_t{z.x > 0.f ? v[q].x : 0.f, z.y > 0.f ? v[q].y : 0.f};
              s1[q] += g;
              s2[q] = pfma(g, x[q] - em[q], s2[q]);
              o[q] = pack2(g);
            }
            out = make_uint4(o[0], o[1], o[2], o[3]);
          } else if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              f2_t y = v[q] + ea[q];
              if constexpr (EPI == EPI_BIAS_RELU) y = f2_t{y.x > 0.f ? y.x : 0.f, y.y > 0.f ? y.y : 0.f};
              o[q] = pack2(y);
            }
            out = make_uint4(o[0], o[1], o[2], o[3]);
          } else if constexpr (LR) {  // RESBITS / RES: add d(identity), rounded to bf16
            if (crok[i]) {
              f2_t r[4];
              unpack4x2(crv[i], r);
#pragma unroll
              for (int q = 0; q < 4; ++q) o[q] = pack2(v[q] + r[q]);
              out = make_uint4(o[0], o[1], o[2], o[3]);
            }
            if constexpr (EPI == EPI_RESBITS) {
              unpack4x2(out, v);
              const uint32_t bits = cbv[i];
              f2_t x[4];
              unpack4x2(xin, x);
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const f2_t g = f2_t{(bits >> (2 * q)) & 1u ? v[q].x : 0.f, (bits >> (2 * q + 1)) & 1u ? v[q].y : 0.f};
                v[q] = g;
                s1[q] += g;
                s2[q] = pfma(g, x[q] - em[q], s2[q]);
                o[q] = pack2(g);
              }
              if (X2 && p.ex2) {
                f2_t x2[4];
                unpack4x2(cx2[i], x2);
#pragma unroll
                for (int q = 0; q < 4; ++q) s3[q] = pfma(v[q], x2[q] - em2[q], s3[q]);
              }
              out = make_uint4(o[0], o[1], o[2], o[3]);
            }
          }
        }
        if (EPI != EPI_STATS || p.C) *reinterpret_cast<uint4*>(p.C + go) = out;
      }
    }
  }

  // after the block's last tile (and a barrier: ``sh`` aliases the tile LDS):
  // fold the RPP row groups of each channel chunk, one atomic per channel per
  // sum into this block's replica
  __device__ __forceinline__ void finish(const GemmParams& p, float* sh, int b, bool active) {
    if constexpr (REDUCE) {
      constexpr int NS = 3;
      const int N = p.N;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sh[(0 * NT + t) * 8 + j] = s1[j >> 1][j & 1];
        sh[(1 * NT + t) * 8 + j] = s2[j >> 1][j & 1];
        if constexpr (EPI == EPI_RESBITS) sh[(2 * NT + t) * 8 + j] = s3[j >> 1][j & 1];
      }
      __syncthreads();
      if (active && er0 == 0) {
#pragma unroll
        for (int si = 0; si < NS; ++si) {
          if (si == 2 && !(EPI == EPI_RESBITS && p.ex2)) break;
          float a[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) a[j] = 0.f;
          for (int rr = 0; rr < RPP; ++rr) {
            const int o = (si * NT + rr * CPR + ec) * 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] += sh[o + j];
          }
          float* dst;
          if (si == 0) dst = p.acc + static_cast<int64_t>(b % kRep) * 2 * N + ch0;
          else if (si == 1) dst = p.acc + static_cast<int64_t>(b % kRep) * 2 * N + N + ch0;
          else dst = p.acc2 + static_cast<int64_t>(b % kRep) * 2 * N + N + ch0;
#pragma unroll
          for (int j = 0; j < 8; ++j) atomic_add_f32(dst + j, a[j]);
          if (si == 0 && EPI == EPI_RESBITS && p.ex2) {
            // the downsample BN sees the same masked gradient: same sum(g')
            float* d2 = p.acc2 + static_cast<int64_t>(b % kRep) * 2 * N + ch0;
#pragma unroll
            for (int j = 0; j < 8; ++j) atomic_add_f32(d2 + j, a[j]);
          }
        }
      }
      if (p.fin_ws) finalize_last(p, sh);
    }
  }

  // the last block of this output-channel tile to get here finalizes the
  // tile's channels (csrc/bn_fin.h); every block of the grid calls finish()
  // Hand-off (cdna_hip_programming.md, in-launch split-K recipe): the replica
  // adds are device-scope atomics (performed at the coherence point, visible
  // across XCDs), so a writer only waits for them (vmcnt) before lane 0 draws
  // its ticket -- no per-thread __threadfence (an L2 write-back per thread:
  // that version ran the ResNet step 27 % slower); the last arriver's lane 0
  // takes one agent-scope acquire and the sums are read with agent-scope loads.
  __device__ __forceinline__ void finalize_last(const GemmParams& p, float* sh) {
    const int N = p.N;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's replica atomics acknowledged
    __syncthreads();                                   // every wave's (and the fold's reads of sh)
    const int tiles_n = N / BN;
    const unsigned arrivals = gridDim.x / tiles_n;
    constexpr bool FWD = EPI == EPI_STATS;
    unsigned* cnt = reinterpret_cast<unsigned*>(p.fin_ws + fin_desc_off(N) + kFinDescFloats) + (FWD ? 0 : 32) +
                    n0 / BN;
    int* flag = reinterpret_cast<int*>(sh);
    if (t == 0) {
      const bool last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == arrivals - 1;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      flag[0] = last;
    }
    __syncthreads();
    if (flag[0]) {
      const BnFinDesc d = *reinterpret_cast<const BnFinDesc*>(p.fin_ws + fin_desc_off(N));
      for (int c = n0 + t; c < n0 + BN; c += NT) {
        if constexpr (FWD) {
          fin_fwd_channel(d, p.fin_ws, c, p.fin_M);
        } else {
          fin_bwd_channel(d, p.fin_ws, c, p.fin_M);
          if (EPI == EPI_RESBITS && p.fin_ws2) {
            const BnFinDesc d2 = *reinterpret_cast<const BnFinDesc*>(p.fin_ws2 + fin_desc_off(N));
            fin_bwd_channel(d2, p.fin_ws2, c, p.fin_M);
          }
        }
      }
      if (t == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
};

}  // namespace gemm
}  // namespace kdl
