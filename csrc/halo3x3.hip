// 3x3 stride-1 pad-1 convolution with the input tile staged ONCE per tile as
// a halo in LDS (gfx950), for the operand-stream-bound early ResNet stages.
//
// Why: the LDS-DMA implicit GEMM of csrc/igemm.hip fetches every output row's
// input pixel once per tap, so its A stream is 9x the input, and LDS-DMA into
// LDS runs at ~7-10 TB/s chip-wide (docs/perf_notes.md) -- the N = 64 / 128
// layers sit on that stream, not on the MFMAs.  Here a tile is TH full output
// rows of one image (BM = TH * W = 224 pixels); its (TH + 2) x (W + 2) input
// halo (zero padding = buffer-OOB loads) lands in LDS once and the nine taps
// read shifted 32-pixel fragments from it (the weight gradient of the same
// layers, halo3x3_wgrad_kernel below, stages dy rows and the halo the same way
// and reads both transposed).  The weights of the block's BN
// output channels for all nine taps (9 * Cin * BN bf16 = 72 KiB) stay
// resident in LDS for the block's lifetime (persistent blocks, one N tile per
// block), so per tile the only DMA is the halo:
//
//   Cin = 64  (56x56): BN = 64, TH = 4, halo 348 px x 128 B, double-buffered:
//                      the next tile's halo streams in under this tile's MFMAs.
//                      118.7 -> 80.6 us per layer (stage-1 forward and data
//                      gradient; profiles/r02_halo3x3_vs_igemm.jsonl)
//   Cin = 128 (28x28): the template's single-buffered form (BN = 32, TH = 8,
//                      300 px x 256 B) measured equal to the implicit GEMM
//                      (90.0 vs 90.2 us) and is not dispatched: with one
//                      7-wave block per CU the epilogue is not overlapped and
//                      the halo is fetched once per 32-channel N tile.
//
// LDS image: rows of 128 B (one 64-channel chunk of one pixel; a Cin = 128
// pixel is two consecutive rows), 16-B chunk c of row R at chunk position
// c ^ ((R >> 1) & 7) -- swizzled on the SOURCE address because the DMA writes
// lane-linear (the igemm.hip scheme).  Seven waves, one 32-pixel MFMA row
// block each (v_mfma_f32_32x32x16_bf16, weight fragment as the A operand), and
// the fused epilogues of gemm_epi.h (BN statistics for the forward conv, ReLU
// mask + BN backward sums for the stride-1 data gradient).  The DMA is issued
// from inline asm and retired by counted vmcnt + raw barriers (csrc/igemm.hip
// three-stage path) so the next halo stays in flight across the barriers.
#include <cstdlib>

#include "common.h"
#include "gemm_epi.h"
#include "kdl_api.h"
#include "tune.h"

namespace kdl {
namespace {

using namespace gemm;

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((ext_vector_type(4))) int i32x4_t;

constexpr uint32_t kOOB = 0x80000000u;  // voffset past every buffer: zeros
constexpr int kWaves = 7, kNT = 64 * kWaves, kBM = 32 * kWaves;  // 224-pixel tiles
constexpr int kBRows = 576;            // resident weight rows: 9 taps x Cin/64 chunks x BN

__device__ __forceinline__ i32x4_t rsrc_words(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  i32x4_t r;
  r.x = __builtin_amdgcn_readfirstlane(static_cast<int>(a & 0xffffffffu));
  r.y = __builtin_amdgcn_readfirstlane(static_cast<int>((a >> 32) & 0xffffu));
  r.z = __builtin_amdgcn_readfirstlane(static_cast<int>(bytes));
  r.w = 0x00020000;
  return r;
}

// 16 B per lane LDS-DMA (1 KiB per wave instruction at dst + 16 * lane), from
// inline asm: the compiler sees no LDS write, so it adds no waits of its own.
__device__ __forceinline__ void dma16(i32x4_t r, lds_void_t* dst, uint32_t voff) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dst)));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(m0), "v"(voff), "s"(r)
               : "memory", "m0");
#endif
}

// PRO: the previous layer's BN + ReLU, relu(x * scale + shift) with
// p.pro_coef = [scale | shift] per input channel, applied to the halo in LDS
// once it has landed (each lane transforms the 16-B chunks it DMA'd; padding
// pixels stay zero), so the activation a = relu(B(x)) is never written to HBM
template <int CIN, int BN, int TH, bool DOUBLE, int EPI, bool PRO = false>
__global__ __launch_bounds__(kNT, 1) void halo3x3_kernel(GemmParams p, int H, int W, int tiles_m, int tiles_n) {
  constexpr int RP = CIN / 64;             // 128-B LDS rows per pixel
  constexpr int TN = BN / 32;              // 32-wide MFMA column blocks per wave
  static_assert(9 * RP * BN == kBRows, "weights fill the resident block");
  constexpr int B_BYTES = kBRows * 128;
  using Epi = Epilogue<kBM, BN, kNT, EPI>;
  constexpr int LDC = Epi::LDC;
  // halo rows (per buffer) for the largest geometry this instantiation serves
  constexpr int HW_MAX = TH == 4 ? 58 : 30;                    // W + 2
  constexpr int HROWS = ((TH + 2) * HW_MAX * RP + 7) / 8 * 8;  // whole 1-KiB DMA groups
  constexpr int HALO_BYTES = HROWS * 128;
  constexpr int NBUF = DOUBLE ? 2 : 1;
  static_assert(HALO_BYTES >= kBM * LDC * 2 && HALO_BYTES >= Epi::kScratchBytes, "epilogue fits a halo buffer");
  static_assert(B_BYTES + NBUF * HALO_BYTES <= 160 * 1024, "LDS budget");
  constexpr int HI = HROWS / 8;                                // DMA instructions per halo
  constexpr int HIPW = (HI + kWaves - 1) / kWaves;             // per wave (upper bound)
  constexpr int HIPW_MIN = HI / kWaves;                        // per wave (lower bound: counted waits)
  constexpr int BIPW = (kBRows / 8 + kWaves - 1) / kWaves;
  __shared__ __attribute__((aligned(1024))) char lds[B_BYTES + NBUF * HALO_BYTES];
  char* Bs = lds;
  char* Hs = lds + B_BYTES;

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int fr = lane & 31, fh = lane >> 5;
  const int tile_n = blockIdx.x % tiles_n;
  const int gm0 = blockIdx.x / tiles_n, gstride = gridDim.x / tiles_n;
  const int n0 = tile_n * BN;
  const int WP = W + 2;
  const int nh = (TH + 2) * WP * RP;  // halo rows actually used

  const i32x4_t rA = rsrc_words(p.A, static_cast<uint32_t>(p.a_rows * CIN * 2));
  const i32x4_t rB = rsrc_words(p.B, static_cast<uint32_t>(static_cast<int64_t>(p.N) * 9 * CIN * 2));

  // ---- resident weights: row b = (tap * RP + kc) * BN + n -> W[n0 + n][tap * CIN + kc * 64 ..]
#pragma unroll
  for (int i = 0; i < BIPW; ++i) {
    const int g = wave + i * kWaves;
    if (g < kBRows / 8) {
      const int b = 8 * g + (lane >> 3);
      const int c = (lane & 7) ^ ((b >> 1) & 7);
      const int tk = b / BN, n = b - tk * BN;  // tk = tap * RP + kc
      const int tap = tk / RP, kc = tk - tap * RP;
      const uint32_t off = static_cast<uint32_t>(
          (static_cast<int64_t>(n0 + n) * 9 * CIN + tap * CIN + kc * 64 + 8 * c) * 2);
      dma16(rB, (lds_void_t*)(Bs + g * 1024), off);
    }
  }

  // ---- halo geometry per DMA slot (tile-invariant): LDS row R = hp * RP + kc
  int hrow[HIPW], hcol[HIPW], hsub[HIPW];  // input row/col relative to the tile, chunk offset (bytes)
#pragma unroll
  for (int i = 0; i < HIPW; ++i) {
    const int g = wave + i * kWaves;
    const int R = 8 * g + (lane >> 3);
    const int hp = R / RP, kc = R - hp * RP;
    const int c = (lane & 7) ^ ((R >> 1) & 7);
    const int hr = hp / WP;
    hrow[i] = (g < HI && R < nh) ? hr - 1 : -0x4000;  // -0x4000: never inside an image
    hcol[i] = hp - hr * WP - 1;
    hsub[i] = (kc * 64 + 8 * c) * 2;
  }
  // PRO: this lane's chunk of slot i covers channels hsub[i] / 2 .. + 7; the
  // chunk alternates between two channel groups with the slot parity (R's
  // swizzle term (R >> 1) & 7 = (4 wave + 4 i + (lane >> 4)) & 7), so two
  // coefficient sets are held in registers (no loads inside the DMA pipeline)
  static_assert(!PRO || CIN == 64, "halo prologue: one 128-B row per pixel");
  float psc[PRO ? 2 : 1][8], psf[PRO ? 2 : 1][8];
  (void)psc; (void)psf;
  if constexpr (PRO) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int c0 = 8 * ((lane & 7) ^ ((4 * wave + 4 * e + (lane >> 4)) & 7));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        psc[e][j] = p.pro_coef[c0 + j];
        psf[e][j] = p.pro_coef[CIN + c0 + j];
      }
    }
  }
  auto halo_ok = [&](int tm, int i) {
    const int tpi = H / TH;
    const int img = tm / tpi, r0 = (tm - img * tpi) * TH;
    (void)img;
    const int ih = r0 + hrow[i], iw = hcol[i];
    return static_cast<unsigned>(ih) < static_cast<unsigned>(H) && static_cast<unsigned>(iw) < static_cast<unsigned>(W);
  };
  // relu(x * scale + shift) on this lane's in-image chunks of halo buffer ``b``;
  // with p.aout the tile's own pixels (the halo's interior rows) are written
  // through: every pixel of the image is interior to exactly one tile, so the
  // activation is stored once, as the apply pass would have
  auto transform_halo = [&](int tm, int b) {
    char* base = Hs + b * HALO_BYTES;
    const int tpi = H / TH;
    const int img = tm / tpi, r0 = (tm - img * tpi) * TH;
#pragma unroll
    for (int i = 0; i < HIPW; ++i) {
      const int g = wave + i * kWaves;
      if (g < HI && halo_ok(tm, i)) {
        uint4* q = reinterpret_cast<uint4*>(base + g * 1024 + 16 * lane);
        float f[8];
        unpack8(*q, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float o = fmaf(f[j], psc[i & 1][j], psf[i & 1][j]);
          f[j] = o > 0.f ? o : 0.f;
        }
        const uint4 v = pack8(f);
        *q = v;
        if (p.aout && static_cast<unsigned>(hrow[i]) < static_cast<unsigned>(TH)) {
          const int64_t px = (static_cast<int64_t>(img) * H + r0 + hrow[i]) * W + hcol[i];
          *reinterpret_cast<uint4*>(reinterpret_cast<char*>(p.aout) + px * (CIN * 2) + hsub[i]) = v;
        }
      }
    }
  };
  auto issue_halo = [&](int tm, int buf) {
    const int tpi = H / TH;
    const int img = tm / tpi, r0 = (tm - img * tpi) * TH;
    char* base = Hs + buf * HALO_BYTES;
#pragma unroll
    for (int i = 0; i < HIPW; ++i) {
      const int g = wave + i * kWaves;
      if (g < HI) {
        const int ih = r0 + hrow[i], iw = hcol[i];
        const bool ok = static_cast<unsigned>(ih) < static_cast<unsigned>(H) &&
                        static_cast<unsigned>(iw) < static_cast<unsigned>(W);
        const uint32_t off =
            ok ? static_cast<uint32_t>(((static_cast<int64_t>(img) * H + ih) * W + iw) * (CIN * 2) + hsub[i]) : kOOB;
        dma16(rA, (lds_void_t*)(base + g * 1024), off);
      }
    }
  };

  // ---- fragment geometry: this lane's output pixel m = wave * 32 + fr of the
  // tile -> (i, j); tap (r, s) reads halo pixel (i + r) * WP + j + s
  const int m = wave * 32 + fr;
  const int pi = m / W, pj = m - pi * W;
  const int hbase = pi * WP + pj;

  Epi epi;
  epi.init(t, n0);

  int tm = gm0, next = gm0 + gstride;
  int buf = 0;
  if (tm < tiles_m) issue_halo(tm, 0);
  while (tm < tiles_m) {
    if constexpr (DOUBLE) {
      if (next < tiles_m) {
        issue_halo(next, buf ^ 1);
        // retire everything older than the halo just issued (this tile's halo, the weights)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(HIPW_MIN) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (PRO) {
      // the landed halo -> relu(B(x)) in place; raw barrier (a __syncthreads
      // fence would drain the next halo's DMA, vmcnt(0))
      transform_halo(tm, buf);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }

    const char* Hb = Hs + buf * HALO_BYTES;
    f32x16_t acc[TN][1];
#pragma unroll
    for (int i = 0; i < TN; ++i) acc[i][0] = f32x16_t{};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int hp = hbase + (tap / 3) * WP + (tap % 3);
#pragma unroll
      for (int kc = 0; kc < RP; ++kc) {
        const int R = hp * RP + kc;
        const int xr = (R >> 1) & 7;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bf16x8_t xf = *reinterpret_cast<const bf16x8_t*>(Hb + R * 128 + (((2 * s + fh) ^ xr) * 16));
#pragma unroll
          for (int i = 0; i < TN; ++i) {
            const int b = (tap * RP + kc) * BN + i * 32 + fr;
            const bf16x8_t wf =
                *reinterpret_cast<const bf16x8_t*>(Bs + b * 128 + (((2 * s + fh) ^ ((b >> 1) & 7)) * 16));
            acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, xf, acc[i][0], 0, 0, 0);
          }
        }
      }
    }
    // every wave's fragment reads of this halo are done before it becomes the C tile
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    epi.begin(p, tm);
    bf16_t* Cs = reinterpret_cast<bf16_t*>(Hs + buf * HALO_BYTES);
    acc_to_lds<TN, 1>(acc, Cs, LDC, wave * 32, 0, lane);
    __syncthreads();
    epi.rows(p, Cs, tm);
    __syncthreads();  // the C tile is read out before the buffer takes a halo again
    if constexpr (DOUBLE) {
      buf ^= 1;
    } else {
      if (next < tiles_m) issue_halo(next, 0);
    }
    tm = next;
    next += gstride;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  epi.finish(p, reinterpret_cast<float*>(Hs), blockIdx.x, gm0 < tiles_m);
}

template <int CIN, int BN, int TH, bool DOUBLE>
hipError_t launch(const GemmParams& p, int epi, int H, int W, hipStream_t s) {
  if (p.pro_coef && epi != EPI_STATS) return hipErrorInvalidValue;  // the forward conv's prologue only
  const int tiles_m = p.M / kBM;
  const int tiles_n = p.N / BN;
  int per_n = 256 / tiles_n;  // one resident block per CU, each pinned to one N tile
  if (per_n > tiles_m) per_n = tiles_m;
  if (per_n < 1) per_n = 1;
  const dim3 grid(per_n * tiles_n), block(kNT);
  const GemmParams& q = p;
  switch (epi) {
    case EPI_PLAIN:
      hipLaunchKernelGGL((halo3x3_kernel<CIN, BN, TH, DOUBLE, EPI_PLAIN>), grid, block, 0, s, q, H, W, tiles_m, tiles_n);
      break;
    case EPI_STATS:
      if (p.pro_coef)
        hipLaunchKernelGGL((halo3x3_kernel<CIN, BN, TH, DOUBLE, EPI_STATS, true>), grid, block, 0, s, q, H, W, tiles_m,
                           tiles_n);
      else
        hipLaunchKernelGGL((halo3x3_kernel<CIN, BN, TH, DOUBLE, EPI_STATS>), grid, block, 0, s, q, H, W, tiles_m, tiles_n);
      break;
    case EPI_MASKX:
      hipLaunchKernelGGL((halo3x3_kernel<CIN, BN, TH, DOUBLE, EPI_MASKX>), grid, block, 0, s, q, H, W, tiles_m, tiles_n);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

int g_halo = tune_int("halo", 1);          // 0 keeps every 3x3 on the implicit GEMM
int g_halo_pro = tune_int("halo_pro", 1);  // 0: no BN + ReLU prologue on the halo kernels

// ---------------------------------------------------------------- weight gradient
// dW[co][tap][ci] = sum_p dy[p][co] * a[p + tap][ci] for the 56x56, Cin = Cout =
// 64 layers.  The LDS-DMA wgrad (csrc/wgrad_dma.hip) re-fetches the input once
// per tap (9x the tensor through LDS, 205 us per layer); here a block walks a
// contiguous run of 4-row tiles (one image per block at batch 256), stages each
// tile's dy rows [224][64] and its input halo [6 x 58][64] ONCE, double-buffered,
// and all nine taps read shifted windows of the halo.  The reduction index is
// the pixel, so both operands are read TRANSPOSED (ds_read_b64_tr_b16: 4
// consecutive pixel rows of one channel per lane, two reads = the 8-pixel K run
// of v_mfma_f32_32x32x16_bf16).  An 8-pixel run never crosses an image row (56 =
// 7 x 8), so tap (r, s) of pixel k is halo row k + 2 (k / 56) + 58 r + s and the
// run stays 8 consecutive LDS rows.  Eight waves: (co half, ci half, K parity),
// each holding all nine taps of its 32 x 32 block (144 accumulator registers);
// the two K-parity halves are summed through LDS at the end and every block
// writes one fp32 slab (fixed-order reduce: wgrad_slab_reduce).
// LDS rows are 128 B (64 channels), 16-B chunk c of row R at c ^ (((R >> 1) & 1) * 4):
// any 4 consecutive rows of a transposed read hit distinct banks.
constexpr int kWgWaves = 8, kWgNT = 64 * kWgWaves;
constexpr int kWgDyRows = kBM;                      // 224 tile pixels
constexpr int kWgHRows = 352;                       // 6 x 58 = 348 halo pixels, whole 1-KiB groups
constexpr int kWgStage = (kWgDyRows + kWgHRows) * 128;  // 73,728 B
constexpr int kWgIPW = (kWgDyRows + kWgHRows) / 8 / kWgWaves;
static_assert((kWgDyRows + kWgHRows) % (8 * kWgWaves) == 0, "every wave issues the same DMA count");
static_assert(4 * 9 * 16 * 64 * 4 <= 2 * kWgStage, "K-parity combine fits the stage buffers");

typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;

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

__device__ __forceinline__ int trswz(int R) { return ((R >> 1) & 1) * 4; }

// PRO: A is the BN input x and the operand is relu(x * pro[c] + pro[64 + c]),
// applied to the landed halo in LDS (padding pixels stay zero) -- the forward's
// activation is never materialised
template <bool PRO>
__global__ __launch_bounds__(kWgNT, 1) void halo3x3_wgrad_kernel(const bf16_t* G, const bf16_t* A, float* dw32,
                                                                  int nimg, int tiles, int per, const float* pro) {
  constexpr int H = 56, W = 56, WP = 58, TPI = H / 4;
  __shared__ __attribute__((aligned(1024))) char lds[2 * kWgStage];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int tb = blockIdx.x * per;
  const int te = min(tiles, tb + per);
  const i32x4_t rG = rsrc_words(G, static_cast<uint32_t>(tiles) * kWgDyRows * 128u);
  const i32x4_t rA = rsrc_words(A, static_cast<uint32_t>(nimg) * H * W * 128u);

  // ---- DMA slot i of this wave: stage row R8 < 224 = dy pixel, else halo row R8 - 224
  // (geometry recomputed per issue: registers go to the 144 accumulators)
  auto issue = [&](int tile, int buf) {
    const int img = tile / TPI, r0 = (tile - img * TPI) * 4;
    char* base = lds + buf * kWgStage;
#pragma unroll
    for (int i = 0; i < kWgIPW; ++i) {
      const int g = wave + i * kWgWaves;
      lds_void_t* dst = (lds_void_t*)(base + g * 1024);
      if (8 * g < kWgDyRows) {
        const int R = 8 * g + (lane >> 3);
        const int c = (lane & 7) ^ trswz(R);
        dma16(rG, dst, static_cast<uint32_t>(tile) * (kWgDyRows * 128u) + static_cast<uint32_t>(R * 128 + c * 16));
      } else {
        const int R = 8 * g - kWgDyRows + (lane >> 3);
        const int c = (lane & 7) ^ trswz(R);
        const int hr = R / WP;
        const int ih = r0 + hr - 1, iw = R - hr * WP - 1;
        const bool ok = R < 6 * WP && static_cast<unsigned>(ih) < static_cast<unsigned>(H) &&
                        static_cast<unsigned>(iw) < static_cast<unsigned>(W);
        dma16(rA, dst, ok ? static_cast<uint32_t>(((img * H + ih) * W + iw) * 128 + c * 16) : kOOB);
      }
    }
  };

  // ---- transposed fragment geometry (csrc/wgrad_dma.hip): lane (grp, q, pp)
  // reads pixel rows k0 + q and k0 + q + 4 (k0 = 16 ks + 8 (lane >> 5)) at the
  // 8-B column piece 16 (grp & 1) + 4 pp of its 32-channel fragment
  const int grp = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int cob = wave & 1, cib = (wave >> 1) & 1, kpar = wave >> 2;
  const int cdy = (32 * cob + 16 * (grp & 1) + 4 * pp) >> 3;
  const int cin_ = (32 * cib + 16 * (grp & 1) + 4 * pp) >> 3;
  const int dcol0 = 16 * cdy + 8 * (pp & 1), dcol1 = 16 * (cdy ^ 4) + 8 * (pp & 1);
  const int acol0 = 16 * cin_ + 8 * (pp & 1), acol1 = 16 * (cin_ ^ 4) + 8 * (pp & 1);

  f32x16_t acc[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) acc[i] = f32x16_t{};

  // PRO: a halo slot's chunk is logical chunk (lane & 7) ^ trswz(R) with
  // trswz(R) = ((lane >> 4) & 1) * 4 for every halo row R = 8 g - 224 + (lane >> 3):
  // one channel group per lane, its 8 scales / shifts held in registers
  float psc[PRO ? 8 : 1], psf[PRO ? 8 : 1];
  (void)psc; (void)psf;
  if constexpr (PRO) {
    const int c0 = 8 * ((lane & 7) ^ (((lane >> 4) & 1) * 4));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      psc[j] = pro[c0 + j];
      psf[j] = pro[64 + c0 + j];
    }
  }
  auto transform = [&](int tile, int b) {
    const int img = tile / TPI, r0 = (tile - img * TPI) * 4;
    char* base = lds + b * kWgStage;
#pragma unroll
    for (int i = 0; i < kWgIPW; ++i) {
      const int g = wave + i * kWgWaves;
      if (8 * g >= kWgDyRows) {
        const int R = 8 * g - kWgDyRows + (lane >> 3);
        const int hr = R / WP;
        const int ih = r0 + hr - 1, iw = R - hr * WP - 1;
        const bool ok = R < 6 * WP && static_cast<unsigned>(ih) < static_cast<unsigned>(H) &&
                        static_cast<unsigned>(iw) < static_cast<unsigned>(W);
        if (ok) {
          uint4* q = reinterpret_cast<uint4*>(base + g * 1024 + 16 * lane);
          float f[8];
          unpack8(*q, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float o = fmaf(f[j], psc[j], psf[j]);
            f[j] = o > 0.f ? o : 0.f;
          }
          *q = pack8(f);
        }
      }
    }
  };

  int buf = 0;
  if (tb < te) issue(tb, 0);
  for (int tile = tb; tile < te; ++tile) {
    // every wave is done reading the other buffer (last tile) before it is refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (tile + 1 < te) {
      issue(tile + 1, buf ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kWgIPW) : "memory");  // this tile's DMA retired
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // ... on every wave
    asm volatile("" ::: "memory");
    if constexpr (PRO) {  // landed halo -> relu(B(x)) in place, then published (raw barrier: next DMA in flight)
      transform(tile, buf);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    const char* Dy = lds + buf * kWgStage;
    const char* Hs = Dy + kWgDyRows * 128;
#pragma unroll 1
    for (int j = 0; j < 7; ++j) {
      const int k0 = 16 * (2 * j + kpar) + 8 * (lane >> 5);
      const int Rd = k0 + q;
      const char* pd = Dy + Rd * 128 + (trswz(Rd) ? dcol1 : dcol0);
      const bf16x8_t gf = frag8(tr_read(pd), tr_read(pd + 512));
      const int B = k0 + 2 * (k0 / W) + q;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int R = B + (tap / 3) * WP + (tap % 3);
        const char* pa = Hs + R * 128 + (trswz(R) ? acol1 : acol0);
        const bf16x8_t af = frag8(tr_read(pa), tr_read(pa + 512));
        acc[tap] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gf, af, acc[tap], 0, 0, 0);
      }
    }
    buf ^= 1;
  }

  // ---- K-parity halves summed through LDS, then one fp32 slab per block
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  float* X = reinterpret_cast<float*>(lds);
  const int pw = wave & 3;  // (cob, cib) index shared by the two K-parity partners
  if (kpar) {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int r = 0; r < 16; ++r) X[((pw * 9 + tap) * 16 + r) * 64 + lane] = acc[tap][r];
  }
  __syncthreads();
  if (!kpar) {
    float* slab = dw32 + static_cast<int64_t>(blockIdx.x) * 64 * 576;
    const int fh = lane >> 5, fr = lane & 31;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = acc[tap][r] + X[((pw * 9 + tap) * 16 + r) * 64 + lane];
        const int co = 32 * cob + (r & 3) + 8 * (r >> 2) + 4 * fh;
        slab_store(slab + co * 576 + tap * 64 + 32 * cib + fr, v);
      }
  }
}

// blocks of the halo weight gradient: at most KDL_TUNE halo_wg_blocks (default 256 =
// one per CU); it runs on the side stream beside the main stream's kernels
int wg_blocks(int tiles, int* per) {
  static const int cap = [] {
    const int v = tune_int("halo_wg_blocks", 256);
    return v < 8 ? 8 : v;
  }();
  const int p = (tiles + cap - 1) / cap;
  *per = p;
  return (tiles + p - 1) / p;
}

}  // namespace

void set_halo3x3(int on) { g_halo = on; }

namespace gemm {
// 3x3 / stride 1 / pad 1 on the halo kernel when the geometry is one it
// serves (56x56, Cin 64; the forward may carry the BN + ReLU prologue);
// hipErrorInvalidValue = "not here, use igemm / the register-staged loop".
hipError_t halo3x3(const GemmParams& p, int epi, hipStream_t s) {
  if (!g_halo || p.stride != 1 || (p.pro_coef != nullptr && !g_halo_pro)) return hipErrorInvalidValue;
  const int H = p.Hin, W = p.Win;
  if (p.Hout != H || p.Wout != W || p.M % (H * W) || p.K != 9 * p.Cin) return hipErrorInvalidValue;
  if (static_cast<int64_t>(p.a_rows) * p.Cin * 2 >= (int64_t(1) << 31)) return hipErrorInvalidValue;
  if (p.Cin == 64 && W == 56 && H % 4 == 0 && p.N % 64 == 0) return launch<64, 64, 4, true>(p, epi, H, W, s);
  return hipErrorInvalidValue;
}

// fp32 slabs the halo weight gradient writes (0 = shape not served here)
int halo3x3_wgrad_slabs(int Nb, int Hin, int Win, int Cin, int Cout, int stride) {
  if (!g_halo || stride != 1 || Hin != 56 || Win != 56 || Cin != 64 || Cout != 64 || Nb <= 0) return 0;
  int per;
  return wg_blocks(Nb * 14, &per);
}

// dw32: >= halo3x3_wgrad_slabs(...) x 64 x 576 fp32; hipErrorInvalidValue = "not here";
// pro (optional): [scale | shift] of the BN + ReLU between A and the conv
hipError_t halo3x3_wgrad(const void* G, const void* A, const float* pro, float* dw32, int64_t dw32_floats, int Nb,
                         int Hin, int Win, int Cin, int Cout, int stride, int* nslabs, hipStream_t s) {
  if (pro && !g_halo_pro) return hipErrorInvalidValue;
  const int n = halo3x3_wgrad_slabs(Nb, Hin, Win, Cin, Cout, stride);
  if (n == 0 || dw32_floats < static_cast<int64_t>(n) * 64 * 576) return hipErrorInvalidValue;
  if (static_cast<int64_t>(Nb) * 56 * 56 * 128 >= (int64_t(1) << 32)) return hipErrorInvalidValue;
  const int tiles = Nb * 14;
  int per;
  const int grid = wg_blocks(tiles, &per);
  if (pro)
    hipLaunchKernelGGL(halo3x3_wgrad_kernel<true>, dim3(grid), dim3(kWgNT), 0, s, static_cast<const bf16_t*>(G),
                       static_cast<const bf16_t*>(A), dw32, Nb, tiles, per, pro);
  else
    hipLaunchKernelGGL(halo3x3_wgrad_kernel<false>, dim3(grid), dim3(kWgNT), 0, s, static_cast<const bf16_t*>(G),
                       static_cast<const bf16_t*>(A), dw32, Nb, tiles, per, pro);
  *nslabs = grid;
  return hipGetLastError();
}
}  // namespace gemm

}  // namespace kdl
