// ipc_sync.hpp -- the node-barrier protocol of the peer-mapped (IPC) form as a device function,
// shared by the stand-alone barrier launch (ipc.hip) and the fused small-message Allreduce
// (fold_kernel.hpp ipc_fused_kernel). It replaces the reference's CPU spin barriers on
// shared-memory flags (src/mpi/ext_mpi_native_exec.c:21-84, OPCODE_NODEBARRIER_ATOMIC_SET/_WAIT
// :513-528).
//
// One lane per workgroup takes part. Every workgroup records its XCC and arrives on this rank's
// per-(slot, phase) counter; the last arriver resets the counter, checks that the launch covered
// every XCD of the census taken at communicator set-up and stores the epoch into every peer's
// flag (system-scope atomic on uncached memory). Every workgroup then waits for every peer's
// flag and acquires at system scope (its XCD's L2 drops lines the peers have since rewritten).
// Phase 0 (before the fold) also releases first: the application's stores into this rank's send
// buffer may sit dirty in any XCD's L2, and the peers read that buffer from memory.
// Every wait is bounded by a wall-clock timeout that sets the error word and lets the kernel end.
#pragma once
#include <hip/hip_runtime.h>

#include "gpu.h"

namespace emac {

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}

struct NodeSync {
  emac_sync *self;
  emac_sync *const *peers;
  int slot, nranks, me;
  unsigned xcc_expect;
  int *err;
  long timeout;
};

// called by lane 0 of every workgroup of the launch
__device__ __forceinline__ void node_barrier_lane(const NodeSync &s, int phase, unsigned long epoch) {
  if (phase == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: L2 write-back
    // hipcc drops the wait behind buffer_wbl2 when nothing else is outstanding
    // (MI355X_MICROARCH.md, compiler hazard): the arrival below must follow the write-back
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  const int slot = s.slot;
  atomicOr(&s.self->xcc[slot][phase][epoch & 1], 1u << xcc_id());
  // (relaxed: the release above has already drained before this add issues)
  const unsigned long arrived =
      __hip_atomic_fetch_add(&s.self->arrive[slot][phase], 1ul, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (arrived == gridDim.x - 1) {  // last workgroup of this rank: every XCD has released
    // the next launch on this slot and phase is stream-ordered behind this one
    __hip_atomic_store(&s.self->arrive[slot][phase], 0ul, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned seen =
        __hip_atomic_load(&s.self->xcc[slot][phase][epoch & 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((seen & s.xcc_expect) != s.xcc_expect) __hip_atomic_fetch_or(s.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&s.self->xcc[slot][phase][(epoch + 1) & 1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int q = 0; q < s.nranks; ++q)
      if (q != s.me)
        __hip_atomic_store(&s.peers[q]->flags[slot][phase][s.me], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // every workgroup waits for every peer itself (one hop less than waiting on the last arriver)
  const long t0 = wall_clock64();
  for (int q = 0; q < s.nranks; ++q) {
    if (q == s.me) continue;
    while (__hip_atomic_load(&s.self->flags[slot][phase][q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      __builtin_amdgcn_s_sleep(4);
      if (wall_clock64() - t0 > s.timeout) {
        __hip_atomic_fetch_or(s.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        q = s.nranks;
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: L2 invalidate
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace emac
