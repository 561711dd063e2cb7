// LDS-DMA helpers shared by the LDS-DMA GEMM main loops (csrc/igemm.hip,
// csrc/wgrad_dma.hip): raw buffer-resource words and one 16-byte-per-lane
// `buffer_load_dwordx4 ... lds` (1 KiB per wave at M0 + 16 * lane) issued from
// inline asm.  The asm form matters twice: hipcc does not see an LDS write, so
// it inserts no vmcnt wait of its own before the fragment reads of the stage
// being multiplied (the caller's counted s_waitcnt + barrier are the only
// ordering); and M0 is written in the same statement as the load, so no
// compiler-placed spill or M0 use can land between them.
#pragma once

#include <cstdint>

namespace kdl {
namespace lds_dma {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((ext_vector_type(4))) int i32x4_t;

// voffset past every buffer (num_records < 2^31): the load returns zeros
constexpr uint32_t kOOB = 0x80000000u;

// Raw buffer resource words (what __builtin_amdgcn_make_buffer_rsrc builds):
// 48-bit base, stride 0, num_records bytes, raw-buffer flags.
__device__ __forceinline__ i32x4_t rsrc_words(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  i32x4_t r;
  r.x = __builtin_amdgcn_readfirstlane(static_cast<int>(a & 0xffffffffu));
  r.y = __builtin_amdgcn_readfirstlane(static_cast<int>((a >> 32) & 0xffffu));
  r.z = __builtin_amdgcn_readfirstlane(static_cast<int>(bytes));
  r.w = 0x00020000;
  return r;
}

__device__ __forceinline__ void dma16(i32x4_t r, lds_void_t* dst, uint32_t voff, uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dst)));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :
               : "s"(m0), "v"(voff), "s"(r), "s"(soff)
               : "memory", "m0");
#endif
}

// every wave's LDS-DMA loads landed and its LDS reads retired, then the
// workgroup barrier: the stage just landed is visible to every wave, and the
// stage read in the previous step is free to be overwritten
__device__ __forceinline__ void publish_stage() {
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

}  // namespace lds_dma
}  // namespace kdl
