// Multi-tensor gradient pack: N autograd-owned gradient tensors -> one flat
// (bucket) buffer in ONE launch (gfx950).
//
// Why: letting autograd accumulate into pre-existing ``.grad`` views of the
// flat buffer costs one read-add-write elementwise launch per parameter
// (rocprofv3: 177 ``CUDAFunctor_add`` launches, 2.1 ms of a 41 ms ResNet-50
// step -- profiles/).  Instead ``.grad`` starts as None, autograd hands over
// its freshly computed gradient tensors, and this kernel gathers them into
// the flat buffer that the all-reduce buckets and the fused optimizer use:
// ~51 MB of bf16 moved once at HBM rate.
//
// Work decomposition: a static chunk table (tensor index, offset in tensor,
// length, destination offset) built once on the host; per step only the
// per-tensor source pointer table changes (161 x 8 bytes for ResNet-50).  A
// null source pointer writes zeros (parameters that received no gradient).
// 16-byte vector loads/stores whenever source and destination are aligned.
#include "common.h"
#include "kdl_api.h"

namespace kdl {
namespace {

// ARGS: the source pointers travel in the kernel arguments (PackPtrs, up to
// kPackArgPtrs tensors) instead of a device table: no per-step host->device
// upload of the table (pinned ring + copy + event) before the launch.
template <typename T, bool ARGS>
__global__ __launch_bounds__(256) void pack_kernel(const PackChunk* __restrict__ chunks,
                                                   const int64_t* __restrict__ src_ptrs, const PackPtrs args,
                                                   T* __restrict__ dst, float scale) {
  const PackChunk c = chunks[blockIdx.x];
  const T* src = ARGS ? static_cast<const T*>(args.p[c.tensor]) : reinterpret_cast<const T*>(src_ptrs[c.tensor]);
  T* d = dst + c.dst_off;
  constexpr int VEC = 16 / sizeof(T);
  if (src == nullptr) {
    for (int i = threadIdx.x * VEC; i < c.len; i += 256 * VEC) {
      if (i + VEC <= c.len) {
        *reinterpret_cast<uint4*>(d + i) = make_uint4(0, 0, 0, 0);
      } else {
        for (int k = i; k < c.len; ++k) d[k] = T(0);
      }
    }
    return;
  }
  const T* s = src + c.src_off;
  const bool aligned = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0;
  if (aligned && scale == 1.f) {
    for (int i = threadIdx.x * VEC; i < c.len; i += 256 * VEC) {
      if (i + VEC <= c.len) {
        *reinterpret_cast<uint4*>(d + i) = *reinterpret_cast<const uint4*>(s + i);
      } else {
        for (int k = i; k < c.len; ++k) d[k] = s[k];
      }
    }
  } else if (aligned) {
    for (int i = threadIdx.x * VEC; i < c.len; i += 256 * VEC) {
      if (i + VEC <= c.len) {
        float v[VEC];
        VecIO<T, VEC>::load(s + i, v);
#pragma unroll
        for (int k = 0; k < VEC; ++k) v[k] *= scale;
        VecIO<T, VEC>::store(d + i, v);
      } else {
        for (int k = i; k < c.len; ++k) {
          float v[1] = {Vec1<T>::ld(s + k) * scale};
          Vec1<T>::st(d + k, v[0]);
        }
      }
    }
  } else {
    for (int i = threadIdx.x; i < c.len; i += 256) Vec1<T>::st(d + i, Vec1<T>::ld(s + i) * scale);
  }
}

// Batched transpose: dst[c * dst_ld + r] = src[r * src_ld + c] for a static list
// of 64x64 tiles: the 1x1 conv weights W[Cout][Cin] -> W^T[Cin][Cout] and the
// per-tap slices of the 3x3 weights W[Cout][3][3][Cin] -> Wd[Cin][3][3][Cout]
// (taps reversed) that the data-gradient GEMMs read as their B operand.  One
// launch per step replaces one ``.t().contiguous()`` copy kernel per conv.
// One 64 x 64 bf16 tile per block: each thread moves a 16-element run of one
// row in (two 16-B loads) and a 16-element run of one column out (two 16-B
// stores) when the run is in bounds and 16-B aligned, element-wise otherwise.
// (Element-wise everywhere moved the step's 51 MB at ~1 TB/s; the launch runs on
// the side stream under the forward's memory-bound stem kernels.)
__global__ __launch_bounds__(256) void transpose_tiles_kernel(const TransposeTile* __restrict__ tiles) {
  __shared__ bf16_t sh[64][64 + 2];
  const TransposeTile tt = tiles[blockIdx.x];
  const int t = threadIdx.x;
  const int lr = t >> 2, lc = (t & 3) * 16;  // 64 rows x 4 threads x 16 elements
  {
    const int r = tt.r0 + lr;
    const bf16_t* src = tt.src + static_cast<int64_t>(r) * tt.src_ld + tt.c0 + lc;
    if (r < tt.rows && tt.c0 + lc + 16 <= tt.cols && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
      const uint4 a = reinterpret_cast<const uint4*>(src)[0], b = reinterpret_cast<const uint4*>(src)[1];
      const bf16_t* pa = reinterpret_cast<const bf16_t*>(&a);
      const bf16_t* pb = reinterpret_cast<const bf16_t*>(&b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sh[lr][lc + j] = pa[j];
        sh[lr][lc + 8 + j] = pb[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int c = tt.c0 + lc + j;
        sh[lr][lc + j] = (r < tt.rows && c < tt.cols) ? tt.src[static_cast<int64_t>(r) * tt.src_ld + c] : bf16_t(0);
      }
    }
  }
  __syncthreads();
  const int c = tt.c0 + lr;  // destination row = source column
  if (c < tt.cols) {
    bf16_t* dst = tt.dst + static_cast<int64_t>(c) * tt.dst_ld + tt.r0 + lc;
    if (tt.r0 + lc + 16 <= tt.rows && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
      uint4 a, b;
      bf16_t* pa = reinterpret_cast<bf16_t*>(&a);
      bf16_t* pb = reinterpret_cast<bf16_t*>(&b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pa[j] = sh[lc + j][lr];
        pb[j] = sh[lc + 8 + j][lr];
      }
      reinterpret_cast<uint4*>(dst)[0] = a;
      reinterpret_cast<uint4*>(dst)[1] = b;
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int r = tt.r0 + lc + j;
        if (r < tt.rows) tt.dst[static_cast<int64_t>(c) * tt.dst_ld + r] = sh[lc + j][lr];
      }
    }
  }
}

}  // namespace

hipError_t transpose_tiles(const TransposeTile* tiles, int ntiles, hipStream_t s) {
  if (ntiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(transpose_tiles_kernel, dim3(ntiles), dim3(256), 0, s, tiles);
  return hipGetLastError();
}

hipError_t pack_tensors(const PackChunk* chunks, int nchunks, const int64_t* src_ptrs, void* dst,
                        int dtype, float scale, hipStream_t s, const PackPtrs* args) {
  if (nchunks <= 0) return hipSuccess;
  const PackPtrs none{};
  const PackPtrs& a = args ? *args : none;
  if (dtype == 1) {
    if (args)
      hipLaunchKernelGGL((pack_kernel<bf16_t, true>), dim3(nchunks), dim3(256), 0, s, chunks, src_ptrs, a,
                         static_cast<bf16_t*>(dst), scale);
    else
      hipLaunchKernelGGL((pack_kernel<bf16_t, false>), dim3(nchunks), dim3(256), 0, s, chunks, src_ptrs, a,
                         static_cast<bf16_t*>(dst), scale);
  } else {
    if (args)
      hipLaunchKernelGGL((pack_kernel<float, true>), dim3(nchunks), dim3(256), 0, s, chunks, src_ptrs, a,
                         static_cast<float*>(dst), scale);
    else
      hipLaunchKernelGGL((pack_kernel<float, false>), dim3(nchunks), dim3(256), 0, s, chunks, src_ptrs, a,
                         static_cast<float*>(dst), scale);
  }
  return hipGetLastError();
}

}  // namespace kdl
