// Common device helpers for the kubedl_amd CDNA4 (gfx950) kernels.
//
// Everything here is written for wave64 / 16-byte-per-lane vector memory
// access (MI355X guide, Guideline 13: bf16 data is always moved as 8-element
// 16-byte vectors).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define RETURN_IF_HIP_ERR(expr)                                                        \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) return _e;                                              \
  } while (0)

namespace kdl {

constexpr int kWave = 64;

typedef uint16_t bf16_t;  // raw bf16 bits

__device__ __forceinline__ float bf16_to_f32(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

typedef __attribute__((ext_vector_type(2))) float kdl_f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 kdl_bf16x2_t;

// round-to-nearest-even, NaN preserved: gfx950's v_cvt_pk_bf16_f32 (one VALU
// instruction per PAIR, vs ~5 integer ops per value for the bit-trick)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const kdl_f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, kdl_bf16x2_t));
}

__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  return static_cast<bf16_t>(pack_bf16x2(f, 0.f) & 0xffffu);
}

// Load/store VEC elements of type T as fp32.  VEC*sizeof(T) is 16 bytes on
// the fast path (8 x bf16 or 4 x f32), so each lane issues one dwordx4.
template <typename T, int VEC> struct Vec;

template <> struct Vec<bf16_t, 8> {
  __device__ __forceinline__ static void load(const bf16_t* p, float (&o)[8]) {
    uint4 v = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = __uint_as_float(w[i] << 16);
      o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store(bf16_t* p, const float (&o)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pack_bf16x2(o[2 * i], o[2 * i + 1]);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};

template <> struct Vec<float, 4> {
  __device__ __forceinline__ static void load(const float* p, float (&o)[4]) {
    float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  __device__ __forceinline__ static void store(float* p, const float (&o)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  }
};

// scalar fallback (unaligned / odd channel counts)
template <typename T> struct Vec1;
template <> struct Vec1<bf16_t> {
  __device__ __forceinline__ static float ld(const bf16_t* p) { return bf16_to_f32(*p); }
  __device__ __forceinline__ static void st(bf16_t* p, float v) { *p = f32_to_bf16(v); }
};
template <> struct Vec1<float> {
  __device__ __forceinline__ static float ld(const float* p) { return *p; }
  __device__ __forceinline__ static void st(float* p, float v) { *p = v; }
};

template <typename T, int VEC> struct VecIO {
  __device__ __forceinline__ static void load(const T* p, float (&o)[VEC]) {
    if constexpr (VEC == 1) {
      o[0] = Vec1<T>::ld(p);
    } else {
      Vec<T, VEC>::load(p, o);
    }
  }
  __device__ __forceinline__ static void store(T* p, const float (&o)[VEC]) {
    if constexpr (VEC == 1) {
      Vec1<T>::st(p, o[0]);
    } else {
      Vec<T, VEC>::store(p, o);
    }
  }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Grid sizing for memory-bound kernels (guide Guideline 11): enough blocks to
// fill 256 CUs several times over, capped so each thread still loops.
__host__ __forceinline__ int mem_bound_grid(int64_t work_items, int block, int cap = 2048) {
  int64_t g = (work_items + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

// Weight-gradient split slabs (fp32 partial tiles, summed by wgrad_reduce_kernel
// right after): plain cacheable stores, so the reduce finds them in the
// Infinity Cache -- nontemporal ones (streamed past the caches) measured
// 0.3 % slower per ResNet-50 step, both of two interleaved rounds
// (profiles/r06_slab_blocks_sweep.txt).
__device__ __forceinline__ void slab_store(float* p, float v) { *p = v; }

}  // namespace kdl
