// cusz_amd/csrc/pub_device.hh -- the last-workgroup publish to host-mapped memory, shared by the
// kernels that end a host-visible stage (pass 1's histogram, the encoders' compress summary).
#pragma once

#include "kernels.hh"

namespace cusz_amd {

// The workgroup that finishes last copies pub.r to the host and raises pub.flag.  Every wave first
// waits for its own outstanding memory operations (s_waitcnt 0: the workgroup barrier alone does
// not wait on vmcnt outside tgsplit mode, so another wave's no-return histogram atomics could
// still be in flight), then the relaxed agent-scope ticket is taken after the barrier; the last
// workgroup reads the words back by agent-scope atomic loads.  (An agent-scope release per
// workgroup would write back the XCD's L2 each time.)  Every thread of the workgroup must call it.
// Two ticket levels (pub.ticket[0..7]: workgroups by blockIdx % 8; [8]: the groups' last ones):
// one word takes at most ~90 returning atomics per µs, so a few thousand workgroups ending
// together on one word would queue for tens of µs.
constexpr uint32_t kPubGroups = 8;
constexpr uint32_t kPubTicketWords = kPubGroups + 1;

// true in every thread of the workgroup that finishes last (ticket: kPubTicketWords words, zeroed
// per call); every thread of every workgroup must call it.  The others' global writes and atomics
// are then complete (read them back by agent-scope atomic loads).
__device__ __forceinline__ bool last_block(uint32_t* ticket)
{
  __shared__ uint32_t s_last;
  __builtin_amdgcn_s_waitcnt(0);  // this wave's stores and atomics have completed
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t n = gridDim.x, g = blockIdx.x % kPubGroups;
    const uint32_t in_group = n / kPubGroups + (g < n % kPubGroups ? 1u : 0u);
    const uint32_t groups = n < kPubGroups ? n : kPubGroups;
    bool last = false;
    if (__hip_atomic_fetch_add(ticket + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_group - 1)
      last = __hip_atomic_fetch_add(ticket + kPubGroups, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == groups - 1;
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}

__device__ __forceinline__ void publish_last(const HostPub& pub)
{
  if (!pub.flag) return;
  if (!last_block(pub.ticket)) return;
  for (int k = 0; k < pub.r.count; k++)
    for (int i = threadIdx.x; i < pub.r.nwords[k]; i += blockDim.x)
      pub.r.dst[k][i] = __hip_atomic_load(pub.r.src[k] + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(pub.flag, pub.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace cusz_amd
