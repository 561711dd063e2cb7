// Fused optimizers over a flat, chunked parameter space (gfx950).
//
// The trainer keeps every parameter of a model inside ONE flat bf16 buffer
// (model weights, viewed by the nn.Module), ONE flat bf16 gradient buffer (the
// all-reduce buckets are slices of it, so no pack/unpack copies exist), an fp32
// master copy and the fp32 optimizer state.  The optimizer is then a single
// launch: one 256-thread block per chunk of <= kChunk elements, the chunk
// table (start, length, hyper-parameter group) built once on the host.
//
// Per element the update streams 20 bytes (bf16 grad + f32 master + f32 state
// in, f32 master + f32 state + bf16 param out) with 16-byte vector accesses,
// so it runs at the HBM roof.  Gradient averaging over DP ranks (1/world) is
// folded in as ``grad_scale`` -- the all-reduce is a plain SUM.
#include "common.h"
#include "kdl_api.h"

namespace kdl {

namespace {

template <typename T> struct Ld8;
template <> struct Ld8<bf16_t> {
  __device__ __forceinline__ static void load(const bf16_t* p, float (&o)[8]) { Vec<bf16_t, 8>::load(p, o); }
  __device__ __forceinline__ static void store(bf16_t* p, const float (&o)[8]) { Vec<bf16_t, 8>::store(p, o); }
};
template <> struct Ld8<float> {
  __device__ __forceinline__ static void load(const float* p, float (&o)[8]) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
  __device__ __forceinline__ static void store(float* p, const float (&o)[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(o[4], o[5], o[6], o[7]);
  }
};

template <typename GT, typename PT>
__global__ __launch_bounds__(256) void sgd_chunk_kernel(const OptChunk* __restrict__ chunks,
                                                        float* __restrict__ master,
                                                        float* __restrict__ mom,
                                                        const GT* __restrict__ grad,
                                                        PT* __restrict__ param, OptHyper h) {
  const OptChunk c = chunks[blockIdx.x];
  const float wd = h.wd[c.group];
  const float lr = h.lr * h.lr_scale[c.group];
  for (int i = threadIdx.x * 8; i < c.len; i += 256 * 8) {
    const int64_t idx = c.start + i;
    float g[8], w[8], b[8];
    Ld8<GT>::load(grad + idx, g);
    Ld8<float>::load(master + idx, w);
    if (!h.first_step) Ld8<float>::load(mom + idx, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float gk = fmaf(g[k], h.grad_scale, wd * w[k]);
      float bk = h.first_step ? gk : fmaf(h.momentum, b[k], (1.f - h.dampening) * gk);
      b[k] = bk;
      const float upd = h.nesterov ? fmaf(h.momentum, bk, gk) : bk;
      w[k] = fmaf(-lr, upd, w[k]);
    }
    Ld8<float>::store(master + idx, w);
    Ld8<float>::store(mom + idx, b);
    Ld8<PT>::store(param + idx, w);
  }
}

template <typename GT, typename PT>
__global__ __launch_bounds__(256) void adam_chunk_kernel(const OptChunk* __restrict__ chunks,
                                                         float* __restrict__ master,
                                                         float* __restrict__ m1,
                                                         float* __restrict__ m2,
                                                         const GT* __restrict__ grad,
                                                         PT* __restrict__ param, OptHyper h) {
  const OptChunk c = chunks[blockIdx.x];
  const float wd = h.wd[c.group];
  const float lr = h.lr * h.lr_scale[c.group];
  const float b1 = h.momentum, b2 = h.dampening;
  const float step = lr / h.bc1;
  const float inv_sqrt_bc2 = rsqrtf(h.bc2);
  for (int i = threadIdx.x * 8; i < c.len; i += 256 * 8) {
    const int64_t idx = c.start + i;
    float g[8], w[8], a[8], v[8];
    Ld8<GT>::load(grad + idx, g);
    Ld8<float>::load(master + idx, w);
    Ld8<float>::load(m1 + idx, a);
    Ld8<float>::load(m2 + idx, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float gk = g[k] * h.grad_scale;
      if (h.adam_w) {
        w[k] *= (1.f - lr * wd);
      } else {
        gk = fmaf(wd, w[k], gk);
      }
      a[k] = fmaf(b1, a[k], (1.f - b1) * gk);
      v[k] = fmaf(b2, v[k], (1.f - b2) * gk * gk);
      const float denom = sqrtf(v[k]) * inv_sqrt_bc2 + h.eps;
      w[k] = fmaf(-step, a[k] / denom, w[k]);
    }
    Ld8<float>::store(master + idx, w);
    Ld8<float>::store(m1 + idx, a);
    Ld8<float>::store(m2 + idx, v);
    Ld8<PT>::store(param + idx, w);
  }
}

// Sum of squares per chunk (for global-norm clipping / LARS trust ratios).
template <typename T>
__global__ __launch_bounds__(256) void sumsq_chunk_kernel(const OptChunk* __restrict__ chunks,
                                                          const T* __restrict__ x, float scale,
                                                          float* __restrict__ out) {
  __shared__ float sh[4];
  const OptChunk c = chunks[blockIdx.x];
  float acc = 0.f;
  for (int i = threadIdx.x * 8; i < c.len; i += 256 * 8) {
    float v[8];
    Ld8<T>::load(x + c.start + i, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float s = v[k] * scale;
      acc = fmaf(s, s, acc);
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// Flat copy with dtype cast (master fp32 <-> bf16 param sync, bucket casts).
template <typename S, typename D>
__global__ __launch_bounds__(256) void cast_copy_kernel(const S* __restrict__ src, D* __restrict__ dst,
                                                        int64_t n8) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += static_cast<int64_t>(gridDim.x) * 256) {
    float v[8];
    Ld8<S>::load(src + i * 8, v);
    Ld8<D>::store(dst + i * 8, v);
  }
}

}  // namespace

// dtype codes: 0 = f32, 1 = bf16
#define OPT_DISPATCH2(gd, pd, ...)                                               \
  do {                                                                          \
    if ((gd) == 1 && (pd) == 1) { using GT = bf16_t; using PT = bf16_t; __VA_ARGS__; } \
    else if ((gd) == 1) { using GT = bf16_t; using PT = float; __VA_ARGS__; }   \
    else if ((pd) == 1) { using GT = float; using PT = bf16_t; __VA_ARGS__; }   \
    else { using GT = float; using PT = float; __VA_ARGS__; }                   \
  } while (0)

hipError_t fused_sgd(const OptChunk* chunks, int nchunks, float* master, float* mom,
                     const void* grad, void* param, int gdtype, int pdtype, const OptHyper& h,
                     hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
  OPT_DISPATCH2(gdtype, pdtype,
                hipLaunchKernelGGL((sgd_chunk_kernel<GT, PT>), dim3(nchunks), dim3(256), 0, s,
                                   chunks, master, mom, static_cast<const GT*>(grad),
                                   static_cast<PT*>(param), h));
  return hipGetLastError();
}

hipError_t fused_adam(const OptChunk* chunks, int nchunks, float* master, float* m1, float* m2,
                      const void* grad, void* param, int gdtype, int pdtype, const OptHyper& h,
                      hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
  OPT_DISPATCH2(gdtype, pdtype,
                hipLaunchKernelGGL((adam_chunk_kernel<GT, PT>), dim3(nchunks), dim3(256), 0, s,
                                   chunks, master, m1, m2, static_cast<const GT*>(grad),
                                   static_cast<PT*>(param), h));
  return hipGetLastError();
}

hipError_t chunk_sumsq(const OptChunk* chunks, int nchunks, const void* x, int dtype, float scale,
                       float* out, hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
  if (dtype == 1)
    hipLaunchKernelGGL((sumsq_chunk_kernel<bf16_t>), dim3(nchunks), dim3(256), 0, s, chunks,
                       static_cast<const bf16_t*>(x), scale, out);
  else
    hipLaunchKernelGGL((sumsq_chunk_kernel<float>), dim3(nchunks), dim3(256), 0, s, chunks,
                       static_cast<const float*>(x), scale, out);
  return hipGetLastError();
}

hipError_t cast_copy(const void* src, int sdtype, void* dst, int ddtype, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t n8 = n / 8;  // callers pass multiples of 8 (flat buffers are padded)
  const int grid = mem_bound_grid(n8, 256);
  OPT_DISPATCH2(sdtype, ddtype,
                hipLaunchKernelGGL((cast_copy_kernel<GT, PT>), dim3(grid), dim3(256), 0, s,
                                   static_cast<const GT*>(src), static_cast<PT*>(dst), n8));
  return hipGetLastError();
}

}  // namespace kdl
