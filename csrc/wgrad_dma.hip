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

namespace kdl {
namespace gemm {
namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;

constexpr int MK = 64;                  // rows (m) per stage
constexpr uint32_t kOOB = 0x80000000u;  // voffset past every buffer: the load returns zeros

// device-pass guards: referenced in the host pass these builtins make clang
// drop the kernel's host stub (csrc/igemm.hip dma16)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, lds_void_t* dst, uint32_t voff, uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, voff, soff, 0, 0);
#endif
}

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

  const __amdgpu_buffer_rsrc_t rG = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(p.G), (short)0, static_cast<int>(static_cast<int64_t>(p.M) * p.N * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(p.A), (short)0, static_cast<int>(p.a_rows * lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(BWDG ? p.gx : p.G), (short)0, static_cast<int>(static_cast<int64_t>(p.M) * p.N * 2),
      0x00020000);

  // DMA instruction i of this wave: panel (G panels first, then A), 8-row group
  const int lrow = lane >> 3;
  uint32_t gcol[IPW];  // byte offset of this lane's 16-B chunk within its row
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int g = wave * IPW + i;
    const int panel = g / (MK / 8), r = 8 * (g % (MK / 8)) + lrow;
    const int c = (lane & 7) ^ (((r >> 1) & 1) * 4);
    gcol[i] = panel < PN        ? static_cast<uint32_t>((n0 + 64 * panel + 8 * c) * 2)
              : panel < PN + PK ? static_cast<uint32_t>((acol0 + 64 * (panel - PN) + 8 * c) * 2)
                                : static_cast<uint32_t>((n0 + 64 * (panel - PN - PK) + 8 * c) * 2);
  }

  auto issue = [&](int m0, int stage) {
    char* base = lds + stage * STAGE;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int g = wave * IPW + i;
      const int panel = g / (MK / 8), r = 8 * (g % (MK / 8)) + lrow;
      lds_void_t* dst = (lds_void_t*)(base + g * 1024);
      const int m = m0 + r;
      // rows past M: an explicit out-of-range voffset (the range check covers
      // the VGPR offset; soffset stays 0)
      if (panel < PN) {
        dma16(rG, dst, m < p.M ? static_cast<uint32_t>(m * p.N * 2) + gcol[i] : kOOB, 0);
      } else if (BWDG && panel >= PN + PK) {
        dma16(rX, dst, m < p.M ? static_cast<uint32_t>(m * p.N * 2) + gcol[i] : kOOB, 0);
      } else if constexpr (GATHER == G_DENSE) {
        dma16(rA, dst, m < p.M ? static_cast<uint32_t>(m * p.K * 2) + gcol[i] : kOOB, 0);
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
        dma16(rA, dst, off, 0);
      }
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

  if (mbeg < mend) issue(mbeg, 0);
  int st = 0;
  for (int m0 = mbeg; m0 < mend; m0 += MK) {
    __syncthreads();  // stage st landed everywhere; the other stage is free
    if (m0 + MK < mend) issue(m0 + MK, st ^ 1);
    const char* S = lds + st * STAGE;
    const bool tail = (PRO || BWDG) && m0 + MK > mend;  // rows past the range: zero after the prologue
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8_t gf[TN], af[TK];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const char* b = S + goff[i] + s * 16 * 128;
        gf[i] = frag8(tr_read(b), tr_read(b + 4 * 128));
        if constexpr (BWDG) {
          const char* bx = b + (PN + PK) * PANEL;
          const bf16x8_t xf = frag8(tr_read(bx), tr_read(bx + 4 * 128));
          float f[8], x[8];
          unpack8(__builtin_bit_cast(uint4, gf[i]), f);
          unpack8(__builtin_bit_cast(uint4, xf), x);
          const int mrow = m0 + 16 * s + 8 * (lane >> 5);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float o = fmaf(gk[i], f[e], fmaf(gc1[i], x[e], gc0[i]));  // bn_bwd_apply_kernel's nesting
            f[e] = (!tail || mrow + e < mend) ? o : 0.f;
          }
          gf[i] = __builtin_bit_cast(bf16x8_t, pack8(f));
        }
      }
#pragma unroll
      for (int j = 0; j < TK; ++j) {
        const char* b = S + aoff[j] + s * 16 * 128;
        af[j] = frag8(tr_read(b), tr_read(b + 4 * 128));
        if constexpr (PRO) {
          const uint4 raw = __builtin_bit_cast(uint4, af[j]);
          float f[8];
          unpack8(raw, f);
          const int mrow = m0 + 16 * s + 8 * (lane >> 5);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float o = fmaf(f[e], psc[j], psf[j]);
            f[e] = (o > 0.f && (!tail || mrow + e < mend)) ? o : 0.f;
          }
          af[j] = __builtin_bit_cast(bf16x8_t, pack8(f));
        }
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gf[i], af[j], acc[i][j], 0, 0, 0);
    }
    st ^= 1;
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
        __builtin_nontemporal_store(acc[i][j][r], slab + static_cast<int64_t>(n) * p.K + k);
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
