// ResNet stem: 7x7 / stride 2 / pad 3 convolution of the 3-channel image
// (224x224 -> 112x112 x 64) on MFMA, with the stem BatchNorm's statistics in
// the epilogue (gfx950).
//
// Why a kernel of its own: with Cin = 3 the conv is K = 147 deep and its
// input is 6 B per pixel, which fits neither the 64-channel LDS-DMA chunks of
// csrc/igemm.hip nor the vendor implicit GEMM well (MIOpen: 363 us + an 88 us
// zero-fill of the output + a separate BN statistics pass over the 411 MB
// output; profiles/r02_resnet50_b256_kernel_summary.txt).  Here a tile is two
// output rows (224 pixels) of one image; the 9 x 230 input pixels it reads are
// staged once into LDS with the channel dimension padded to 4 (8 B per
// pixel), so the K order k = r * 32 + s * 4 + c (s padded to 8, c to 4; the
// padding weights are zero) makes every 8-deep MFMA fragment two horizontally
// adjacent input pixels = one aligned 16-B LDS read.  K = 224 = 14 MFMA
// steps of v_mfma_f32_32x32x16_bf16 (weights as the A operand, as csrc/igemm.hip);
// 147/224 of the MFMA work is useful, and the kernel is bound by the 411 MB
// bf16 output write, not by the MFMAs.
//
// Seven waves own one 32-pixel row block each (both 32-channel halves); the
// weights [64][224] stay resident in LDS; the next tile's input is loaded into
// registers under this tile's MFMAs and written to the halo after them.
// Epilogue: gemm_epi.h STATS (per-channel shifted sums into the BN workspace
// replicas) -- the stem BN needs no statistics pass of its own.
#include "common.h"
#include "gemm_epi.h"
#include "kdl_api.h"

namespace kdl {
namespace {

using namespace gemm;

constexpr int kWaves = 7, kNT = 64 * kWaves, kBM = 32 * kWaves;  // 224-pixel tiles
constexpr int kH = 224, kW = 224, kOH = 112, kOW = 112;
constexpr int kHR = 9;                   // input rows per tile (2 output rows, stride 2, 7 taps)
constexpr int kHC = 232;                 // halo pixels per row: iw = -3 .. 228 (+3 offset)
constexpr int kK = 224;                  // 7 r x 8 s x 4 c
constexpr int kLDB = kK + 8;             // weight row stride (bf16): conflict-free fragment reads
constexpr int kRowDw = kW * 3 / 2;       // dwords per input row (336)
constexpr int kSlots = kHR * kRowDw;     // dwords per tile (3024)
constexpr int kPf = (kSlots + kNT - 1) / kNT;  // per thread (7)

template <int EPI>
__global__ __launch_bounds__(kNT, 2) void stem_fwd_kernel(GemmParams p, int tiles) {
  using Epi = Epilogue<kBM, 64, kNT, EPI>;
  constexpr int LDC = Epi::LDC;
  constexpr int B_BYTES = 64 * kLDB * 2;
  constexpr int H_BYTES = kHR * kHC * 8;
  constexpr int C_BYTES = kBM * LDC * 2;
  static_assert(B_BYTES + H_BYTES + C_BYTES >= Epi::kScratchBytes, "finish() scratch fits");
  __shared__ __attribute__((aligned(16))) char lds[B_BYTES + H_BYTES + C_BYTES];
  bf16_t* Bs = reinterpret_cast<bf16_t*>(lds);
  bf16_t* Hs = reinterpret_cast<bf16_t*>(lds + B_BYTES);
  bf16_t* Cs = reinterpret_cast<bf16_t*>(lds + B_BYTES + H_BYTES);

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int fr = lane & 31, fh = lane >> 5;
  const uint16_t* X = reinterpret_cast<const uint16_t*>(p.A);

  // weights (row n: 224 bf16 = 28 uint4) and a zeroed halo (the column and
  // channel padding is never written again)
  for (int i = t; i < 64 * (kK / 8); i += kNT) {
    const int n = i / (kK / 8), c = i - n * (kK / 8);
    *reinterpret_cast<uint4*>(Bs + n * kLDB + 8 * c) = *reinterpret_cast<const uint4*>(p.B + n * kK + 8 * c);
  }
  for (int i = t; i < H_BYTES / 16; i += kNT) reinterpret_cast<uint4*>(Hs)[i] = make_uint4(0, 0, 0, 0);

  // input dwords of tile tm (rows outside the image read as zero)
  uint32_t pf[kPf];
  auto load = [&](int tm) {
    const int img = tm / (kOH / 2), ih0 = (tm - img * (kOH / 2)) * 4 - 3;
#pragma unroll
    for (int q = 0; q < kPf; ++q) {
      const int j = t + q * kNT;
      const int hr = j / kRowDw, wd = j - hr * kRowDw;
      const int ih = ih0 + hr;
      pf[q] = 0u;
      if (j < kSlots && static_cast<unsigned>(ih) < static_cast<unsigned>(kH))
        pf[q] = *reinterpret_cast<const uint32_t*>(X + (static_cast<int64_t>(img) * kH + ih) * (kW * 3) + 2 * wd);
    }
  };
  auto store = [&]() {
    uint16_t* H16 = reinterpret_cast<uint16_t*>(Hs);
#pragma unroll
    for (int q = 0; q < kPf; ++q) {
      const int j = t + q * kNT;
      if (j < kSlots) {
        const int hr = j / kRowDw, wd = j - hr * kRowDw;
        const int e0 = 2 * wd, e1 = e0 + 1;  // element = 3 * pixel + channel
        const int p0 = e0 / 3, p1 = e1 / 3;
        H16[(hr * kHC + p0 + 3) * 4 + (e0 - 3 * p0)] = static_cast<uint16_t>(pf[q] & 0xffffu);
        H16[(hr * kHC + p1 + 3) * 4 + (e1 - 3 * p1)] = static_cast<uint16_t>(pf[q] >> 16);
      }
    }
  };

  // this lane's output pixel of the tile: m = wave * 32 + fr -> (row ohl, col ow);
  // K-step ks reads halo row 2 ohl + ks / 2, pixels 2 ow + s0, +1 (s0 = 4 (ks & 1) + 2 fh)
  const int m = wave * 32 + fr;
  const int ohl = m / kOW, ow = m - ohl * kOW;
  const char* hbase = reinterpret_cast<const char*>(Hs) + ((2 * ohl) * kHC + 2 * ow + 2 * fh) * 8;
  const char* bbase = reinterpret_cast<const char*>(Bs) + (fr * kLDB + 8 * fh) * 2;

  Epi epi;
  epi.init(t, 0);

  int tm = blockIdx.x;
  if (tm < tiles) {
    load(tm);
    store();
  }
  __syncthreads();
  for (; tm < tiles; tm += gridDim.x) {
    const int next = tm + gridDim.x;
    const int drop = p.price_drop;  // timing-only breakdown (set_stem_drop): 1 MFMA, 2 epilogue, 4 input
    if (next < tiles && !(drop & 4)) load(next);  // lands under the MFMAs
    f32x16_t acc[2][1];
    acc[0][0] = f32x16_t{};
    acc[1][0] = f32x16_t{};
    if (!(drop & 1)) {
#pragma unroll
      for (int ks = 0; ks < kK / 16; ++ks) {
        const bf16x8_t xf = *reinterpret_cast<const bf16x8_t*>(hbase + ((ks >> 1) * kHC + 4 * (ks & 1)) * 8);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const bf16x8_t wf = *reinterpret_cast<const bf16x8_t*>(bbase + (i * 32 * kLDB + ks * 16) * 2);
          acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, xf, acc[i][0], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // every wave is done with this halo
    if (next < tiles && !(drop & 4)) store();
    epi.begin(p, tm);
    acc_to_lds<2, 1>(acc, Cs, LDC, wave * 32, 0, lane);
    __syncthreads();  // C tile and the next halo are complete
    if (!(drop & 2)) epi.rows(p, Cs, tm);
  }
  __syncthreads();
  epi.finish(p, reinterpret_cast<float*>(lds), blockIdx.x, blockIdx.x < tiles);
}

int g_stem_drop = 0;

}  // namespace

void set_stem_drop(int bits) { g_stem_drop = bits; }

hipError_t stem7x7_fwd(const void* x, const void* wp, void* y, int Nb, const float* shift, float* acc,
                       hipStream_t s) {
  if (Nb <= 0) return hipErrorInvalidValue;
  GemmParams p{};
  p.A = static_cast<const bf16_t*>(x);
  p.B = static_cast<const bf16_t*>(wp);
  p.C = static_cast<bf16_t*>(y);
  p.M = Nb * kOH * kOW;
  p.N = 64;
  p.K = kK;
  p.shift = shift;
  p.acc = acc;
  p.price_drop = g_stem_drop;
  const int tiles = Nb * (kOH / 2);
  const int grid = tiles < 512 ? tiles : 512;  // two resident blocks per CU
  if (acc) {
    hipLaunchKernelGGL(stem_fwd_kernel<EPI_STATS>, dim3(grid), dim3(kNT), 0, s, p, tiles);
  } else {
    hipLaunchKernelGGL(stem_fwd_kernel<EPI_PLAIN>, dim3(grid), dim3(kNT), 0, s, p, tiles);
  }
  return hipGetLastError();
}

}  // namespace kdl
