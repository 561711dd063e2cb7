// HIP streams on dedicated hardware queues, and a queue-concurrency probe.
//
// A stream created with an explicit CU mask always gets a hardware queue of
// its own (HIP shares the process's GPU_MAX_HW_QUEUES queues among ordinary
// streams).  Used by kubedl_amd/ops/streams.py's ``dedicated`` mode; measured
// slower than pool streams for the ResNet step (profiles/
// r02_world1_pg_streams_ab.txt), so not the default.  ``cus`` < the CU count
// restricts the stream to that many CUs (a partial mask: the engine's
// weight-gradient side stream, EngineOptions.side_cus).  The spin kernel is the
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

hipError_t make_stream(bool dedicated, int priority, hipStream_t* out, int cus) {
  *out = nullptr;
  if (!dedicated && cus <= 0) return hipStreamCreateWithPriority(out, hipStreamNonBlocking, priority);
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  int ncu = 0;
  e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  if (cus <= 0 || cus > ncu) cus = ncu;
  // cus < ncu: a Bresenham-spread subset of the CU ids (every XCD and shader
  // engine keeps a share: consecutive ids are spread over the dies)
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  for (int i = 0; i < ncu; ++i)
    if ((static_cast<int64_t>(i + 1) * cus) / ncu != (static_cast<int64_t>(i) * cus) / ncu) mask[i / 32] |= 1u << (i % 32);
  // (a CU-masked stream takes no priority: it keeps the default)
  return hipExtStreamCreateWithCUMask(out, static_cast<uint32_t>(mask.size()), mask.data());
}

hipError_t spin(hipStream_t s, double microseconds) {
  const uint64_t ticks = static_cast<uint64_t>(microseconds * 100.0);  // s_memrealtime: 100 MHz
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, ticks);
  return hipGetLastError();
}

}  // namespace kdl
