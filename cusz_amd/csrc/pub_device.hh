// cusz_amd/csrc/pub_device.hh -- the last-workgroup publish to host-mapped memory, shared by the
// kernels that end a host-visible stage (pass 1's histogram, the encoders' compress summary).
#pragma once

#include "kernels.hh"

namespace cusz_amd {

// The workgroup that finishes last copies pub.r to the host and raises pub.flag.  The ticket is a
// relaxed atomic taken after the workgroup's barrier (which waits for its memory operations,
// atomics included): the last workgroup reads the words back by agent-scope atomic loads.  (An
// agent-scope release per workgroup would write back the XCD's L2 each time.)  Every thread of
// the workgroup must call it.
__device__ __forceinline__ void publish_last(const HostPub& pub)
{
  if (!pub.flag) return;
  __shared__ uint32_t s_last;
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(pub.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  for (int k = 0; k < pub.r.count; k++)
    for (int i = threadIdx.x; i < pub.r.nwords[k]; i += blockDim.x)
      pub.r.dst[k][i] = __hip_atomic_load(pub.r.src[k] + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(pub.flag, pub.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace cusz_amd
