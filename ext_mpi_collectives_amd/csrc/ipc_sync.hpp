// ipc_sync.hpp -- the node-barrier protocol of the peer-mapped (IPC) form as wave-level device
// functions, shared by the stand-alone barrier launch (ipc.hip) and the fused small-message
// Allreduce (fold_kernel.hpp ipc_fused_kernel). It replaces the reference's CPU spin barriers on
// shared-memory flags (src/mpi/ext_mpi_native_exec.c:21-84, OPCODE_NODEBARRIER_ATOMIC_SET/_WAIT
// :513-528).
//
// Placement-free by construction: nothing here depends on which XCD a workgroup lands on.
//  * Flags live in uncached device memory (hipDeviceMallocUncached) and are accessed with
//    system-scope atomics, so no L2 ever holds them.
//  * The data the barrier orders needs no cache maintenance from the barrier's own workgroups:
//    the application's writes to this rank's buffers are written back from every XCD's L2 by
//    the command processor at the end of the producing kernel (the packet boundary before the
//    barrier launch; EXT_MPI_AMD_IPC_RELEASE=1 adds an explicit hipEventReleaseToSystem record,
//    engine.c), the fold between the barriers reads peers with system-coherent sc0 sc1 loads and
//    stores only into this rank's own receive buffer, drained before the phase-1 signal
//    (fold_kernel.hpp kRemote), and the copy-out pulls the other owners' results the same way.
// One wave takes part: lane q signals peer q (stores the epoch into the peer's flag for this rank)
// and waits for peer q's flag, so a barrier over R ranks is R-1 parallel one-way hops.
// Every wait is bounded by a wall-clock timeout. A rank that times out in phase 0 skips its fold
// (nothing stored into a peer that may not have released its receive buffer) and tells every
// peer so (aborted[slot][tag & 1] = tag, before its phase-1 signal); a rank that then completes
// phase 1 of the same Start finds the mark and reports the Start as failed too, because its
// result lacks the chunks the quitter owns. Epochs keep counting on every rank, so the next
// Start on the slot synchronises normally: a timeout costs that one Start, not the communicator.
#pragma once
#include <hip/hip_runtime.h>

#include "gpu.h"

namespace emac {

struct NodeSync {
  emac_sync *self;
  emac_sync *const *peers;
  int slot, nranks, me;
  int *err;  // this slot's error word (pinned host memory)
  long timeout;
  unsigned long tag;  // the Start's phase-1 epoch: names the Start in aborted[]
};

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// lane q < nranks, q != me: store `epoch` into peer q's flag for this rank (self_too: lane me
// also into this rank's own flag for itself -- the fused launch's "every own chunk has landed")
__device__ __forceinline__ void wave_signal(const NodeSync &s, int phase, unsigned long epoch, bool self_too = false) {
  const int q = lane_id();
  if (q < s.nranks && (q != s.me || self_too))
    __hip_atomic_store(&s.peers[q]->flags[s.slot][phase][s.me], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// lane q waits for peer q's flag to reach `epoch` (self_too: lane me for this rank's own flag);
// true (on every lane) iff every one arrived in time
__device__ __forceinline__ bool wave_wait(const NodeSync &s, int phase, unsigned long epoch, bool self_too = false) {
  const int q = lane_id();
  int late = 0;
  if (q < s.nranks && (q != s.me || self_too)) {
    const unsigned long *f = &s.self->flags[s.slot][phase][q];
    const long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > s.timeout) {
        late = 1;
        break;
      }
    }
  }
  return __ballot(late) == 0;
}

__device__ __forceinline__ void wave_report(const NodeSync &s, int e) {
  if (e && lane_id() == 0) __hip_atomic_fetch_or(s.err, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// has a peer given up on this Start? (a mark stored before that peer's phase-1 signal)
__device__ __forceinline__ bool peer_gave_up(const NodeSync &s) {
  return __hip_atomic_load(&s.self->aborted[s.slot][s.tag & 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == s.tag;
}

// Phase 0 (before the fold) for one wave: signal, wait, and decide whether this rank may fold.
// On a timeout the Start is marked abandoned in every peer's block; the marks are acknowledged
// by the peers' memory before the wave goes on (so before this rank's phase-1 signal). A rank
// that arrives after a peer gave up does not fold either.
__device__ __forceinline__ bool wave_phase0(const NodeSync &s, unsigned long epoch, bool signal) {
  if (signal) wave_signal(s, 0, epoch);
  if (!wave_wait(s, 0, epoch)) {
    const int q = lane_id();
    wave_report(s, EMAC_SYNC_ERR_TIMEOUT);
    if (q < s.nranks && q != s.me)
      __hip_atomic_store(&s.peers[q]->aborted[s.slot][s.tag & 1], s.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return false;
  }
  if (peer_gave_up(s)) {
    wave_report(s, EMAC_SYNC_ERR_ABORTED);
    return false;
  }
  return true;
}

// Phase 1 (after every fan-out store of this rank has been acknowledged): signal, wait, and
// report a timeout or a peer that gave up on this Start (its result lacks the quitter's chunks).
__device__ __forceinline__ void wave_phase1(const NodeSync &s, unsigned long epoch) {
  wave_signal(s, 1, epoch);
  const bool in_time = wave_wait(s, 1, epoch);
  wave_report(s, (in_time ? 0 : EMAC_SYNC_ERR_TIMEOUT) | (peer_gave_up(s) ? EMAC_SYNC_ERR_ABORTED : 0));
}

}  // namespace emac
