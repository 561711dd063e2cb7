// HIP streams on dedicated hardware queues, and a queue-concurrency probe.
//
// A stream created with an explicit CU mask always gets a hardware queue of
// its own (HIP shares the process's GPU_MAX_HW_QUEUES queues among ordinary
// streams).  Used by kubedl_amd/ops/streams.py's ``dedicated`` mode; measured
// slower than pool streams for the ResNet step (profiles/
// r02_world1_pg_streams_ab.txt), so not the default.  The spin kernel is the
// probe of scripts/probe_queues.py: one wave per launch, so two launches on
// different hardware queues overlap and two on one queue serialise.
#include <vector>

#include "common.h"
#include "kdl_api.h"

namespace kdl {
namespace {

// One wave busy-waits ``ticks`` of the 100 MHz constant clock; bounded by
// construction (every wave exits once the clock passes its deadline).
__global__ void spin_kernel(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(2);
  }
}

}  // namespace

hipError_t make_stream(bool dedicated, int priority, hipStream_t* out) {
  *out = nullptr;
  if (!dedicated) return hipStreamCreateWithPriority(out, hipStreamNonBlocking, priority);
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  int ncu = 0;
  e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  for (int i = 0; i < ncu; ++i) mask[i / 32] |= 1u << (i % 32);
  return hipExtStreamCreateWithCUMask(out, static_cast<uint32_t>(mask.size()), mask.data());
}

hipError_t spin(hipStream_t s, double microseconds) {
  const uint64_t ticks = static_cast<uint64_t>(microseconds * 100.0);  // s_memrealtime: 100 MHz
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, ticks);
  return hipGetLastError();
}

}  // namespace kdl
