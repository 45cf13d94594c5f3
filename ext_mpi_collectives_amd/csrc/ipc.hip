// ipc.hip -- peer-mapped execution form (one rank per GPU, buffers shared over xGMI) for gfx950.
//
// The reference's GPU path maps every node peer's device send/recv buffer into each process
// with CUDA IPC (src/gpu/cuda_shmem.c:218-299) and its copy-reduce kernel then loads the
// partners' chunks directly (src/gpu/cuda_core.cu:50-86); ranks synchronise through flags in
// shared memory spun on by the CPU (src/mpi/ext_mpi_native_exec.c:21-84,513-528) around a
// cudaDeviceSynchronize before every barrier. Here the same mapping is made with hipIpc
// (dmabuf) and the node barrier is a small stream-ordered kernel, so a whole Allreduce is three
// launches on the rank's own stream and never returns to the host (one launch for small
// messages: fold_kernel.hpp ipc_fused_kernel):
//
//   node_barrier(in) -> fold of the owner chunks over the peers' mapped send buffers into this
//   rank's library-owned result buffer ("outbox") -> node_barrier(out) -> pull of every owner's
//   result from its outbox into this rank's receive buffer
//
// Peers only ever READ caller memory (the send buffers); nothing of the set-up or of a Start
// writes through a mapping into memory the caller owns (engine.c ipc_exchange).
// Visibility across GPUs: every XCD of a gfx950 has its own L2, and the L2 is neither written
// back nor invalidated for other agents by plain stores/loads. Nothing here relies on where a
// workgroup lands: when a peer sits on another device the application's writes to this rank's
// send buffer are released to system scope by the command processor on every XCD before the
// phase-0 barrier (emac_gpu_event_create_release, recorded by engine.c), the fold and the pull
// are system-coherent by themselves (sc0 sc1 loads, write-through stores drained before the
// next signal), and the flags live in uncached device memory, written and polled with
// system-scope atomics: one 8-byte word per (handle slot, phase, peer), holding the last epoch
// that peer signalled (ipc_sync.hpp). Every wait is bounded by a wall-clock timeout that sets the
// slot's error word in pinned host memory and lets the kernel end; a phase-0 timeout also cancels
// this rank's fold (the go[slot] word of ipc_sync.hpp).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#include "gpu.h"
#include "ipc_sync.hpp"

namespace {

/* EXT_MPI_AMD_DEBUG_HIP=1: report every failing HIP call (and every error cleared after a
   failed probe) on stderr */
inline int ok_at(hipError_t e, const char *what) {
  if (e == hipSuccess) return 0;
  if (getenv("EXT_MPI_AMD_DEBUG_HIP")) fprintf(stderr, "ext_mpi_amd: %s -> %s\n", what, hipGetErrorString(e));
  return EMAC_ERR_DEVICE;
}
#define ok(e) ok_at((e), #e)
inline void clear_error(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess && getenv("EXT_MPI_AMD_DEBUG_HIP"))
    fprintf(stderr, "ext_mpi_amd: %s: cleared %s\n", what, hipGetErrorString(e));
}

// The stand-alone node barrier (ipc_sync.hpp): one wave, lane q talks to peer q. Phase 0 also
// leaves its verdict in go[slot] for the fold launch behind it.
__global__ __launch_bounds__(64) void node_barrier_kernel(emac::NodeSync ns, int phase, unsigned long epoch) {
  if (phase == 0) {
    const bool ok = emac::wave_phase0(ns, epoch, true);
    if (threadIdx.x == 0) __hip_atomic_store(&ns.self->go[ns.slot], ok ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    emac::wave_phase1(ns, epoch);
  }
}

// The split barrier of the pipelined node join: the signal on the stream that produced the data,
// the wait on the stream that consumes it (ipc_sync.hpp; phase 0's wait leaves go[slot]).
__global__ __launch_bounds__(64) void node_signal_kernel(emac::NodeSync ns, int phase, unsigned long epoch) {
  emac::wave_signal(ns, phase, epoch);
}

__global__ __launch_bounds__(64) void node_wait_kernel(emac::NodeSync ns, int phase, unsigned long epoch) {
  if (phase == 0) {
    const bool ok = emac::wave_phase0(ns, epoch, false);
    if (threadIdx.x == 0) __hip_atomic_store(&ns.self->go[ns.slot], ok ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    const bool in_time = emac::wave_wait(ns, 1, epoch);
    emac::wave_report(ns, (in_time ? 0 : EMAC_SYNC_ERR_TIMEOUT) | (emac::peer_gave_up(ns) ? EMAC_SYNC_ERR_ABORTED : 0));
  }
}

// Byte probes of the IPC set-up (engine.c ipc_exchange): one lane per byte. Stores are
// published with a system-scope release (L2 write-back of this XCD); loads follow a system-scope
// acquire (L2 invalidate), so both see memory as the other processes left it.
struct ProbeSet {
  unsigned char *p[EMAC_PROBE_MAX];
  unsigned char v[EMAC_PROBE_MAX];
  int n;
};

__global__ __launch_bounds__(64) void poke_kernel(ProbeSet a) {
  const int i = threadIdx.x;
  if (i < a.n) *reinterpret_cast<volatile unsigned char *>(a.p[i]) = a.v[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // and drop the lines: a valid copy of a peer's line left in this XCD's L2 would be returned
  // to later loads after the peer has restored the byte (measured: 8 processes on one GPU)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ __launch_bounds__(64) void peek_kernel(ProbeSet a, unsigned char *out) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const int i = threadIdx.x;
  if (i < a.n) out[i] = *reinterpret_cast<volatile const unsigned char *>(a.p[i]);
}

// Read-only samples of the IPC set-up (engine.c ipc_exchange): workgroup j reads
// EMAC_SAMPLE_BYTES bytes of buffer j -- EMAC_SAMPLE_SPOTS spots of 8 bytes spread evenly over
// its `len` bytes (all of it when shorter) -- after a system-scope acquire, so an importer and
// the exporter read the same memory whatever either process's L2s held before. Nothing is written
// to the sampled memory.
struct SampleSet {
  const unsigned char *p[EMAC_PROBE_MAX];
  long len[EMAC_PROBE_MAX];
};

__global__ __launch_bounds__(EMAC_SAMPLE_BYTES) void sample_kernel(SampleSet a, unsigned char *out) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const int j = blockIdx.x, i = threadIdx.x;
  const long len = a.len[j];
  long at;
  if (len <= EMAC_SAMPLE_BYTES)
    at = i < len ? i : -1;
  else
    at = (len - 8) * (long)(i >> 3) / (EMAC_SAMPLE_SPOTS - 1) + (i & 7);
  out[j * EMAC_SAMPLE_BYTES + i] = at >= 0 ? *reinterpret_cast<volatile const unsigned char *>(a.p[j] + at) : 0;
}

}  // namespace

extern "C" {

int emac_gpu_poke(void *const *ptrs, const unsigned char *vals, int n, void *stream) {
  ProbeSet a;
  if (n < 0 || n > EMAC_PROBE_MAX) return EMAC_ERR_ARG;
  if (!n) return 0;
  memset(&a, 0, sizeof(a));
  for (int i = 0; i < n; ++i) {
    a.p[i] = static_cast<unsigned char *>(ptrs[i]);
    a.v[i] = vals[i];
  }
  a.n = n;
  hipLaunchKernelGGL(poke_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), a);
  int rc = ok(hipGetLastError());
  return rc ? rc : ok(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
}

int emac_gpu_peek(const void *const *ptrs, unsigned char *vals, int n, void *stream) {
  ProbeSet a;
  unsigned char *d = nullptr;
  if (n < 0 || n > EMAC_PROBE_MAX) return EMAC_ERR_ARG;
  if (!n) return 0;
  memset(&a, 0, sizeof(a));
  for (int i = 0; i < n; ++i) a.p[i] = static_cast<unsigned char *>(const_cast<void *>(ptrs[i]));
  a.n = n;
  if (hipMalloc(&d, EMAC_PROBE_MAX) != hipSuccess) return EMAC_ERR_MALLOC;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(peek_kernel, dim3(1), dim3(64), 0, s, a, d);
  int rc = ok(hipGetLastError());
  if (!rc) rc = ok(hipMemcpyAsync(vals, d, (size_t)n, hipMemcpyDeviceToHost, s));
  if (!rc) rc = ok(hipStreamSynchronize(s));
  (void)hipFree(d);
  return rc;
}

int emac_gpu_sample(const void *const *ptrs, const long *lens, int n, unsigned char *out, void *stream) {
  /* the samples land in pinned, device-mapped host memory kept per device: a set-up makes several
     of these calls, and a hipMalloc / hipFree pair per call would synchronise the device each time */
  static unsigned char *pinned[64];
  SampleSet a;
  int dev = 0;
  if (n < 0 || n > EMAC_PROBE_MAX) return EMAC_ERR_ARG;
  if (!n) return 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return EMAC_ERR_DEVICE;
  if (!pinned[dev] && hipHostMalloc((void **)&pinned[dev], (size_t)EMAC_SAMPLE_BYTES * EMAC_PROBE_MAX,
                                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    pinned[dev] = nullptr;
    return EMAC_ERR_MALLOC;
  }
  memset(&a, 0, sizeof(a));
  for (int i = 0; i < n; ++i) {
    a.p[i] = static_cast<const unsigned char *>(ptrs[i]);
    a.len[i] = lens[i];
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(sample_kernel, dim3((unsigned)n), dim3(EMAC_SAMPLE_BYTES), 0, s, a, pinned[dev]);
  int rc = ok(hipGetLastError());
  if (!rc) rc = ok(hipStreamSynchronize(s));
  if (!rc) memcpy(out, pinned[dev], (size_t)n * EMAC_SAMPLE_BYTES);
  return rc;
}

int emac_gpu_device_uuid(unsigned char *uuid) {
  int dev = 0;
  hipUUID u;
  memset(uuid, 0, 16);
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetUuid(&u, dev) != hipSuccess) {
    clear_error("emac_gpu_device_uuid");
    return EMAC_ERR_DEVICE;
  }
  memcpy(uuid, u.bytes, 16);
  // a runtime that reports no UUID (all zero) would make every GPU look alike, and the peer-mapped
  // forms would then keep device-scope stores across GPUs: identify the device by its PCI location
  static const unsigned char zero[16] = {0};
  if (!memcmp(uuid, zero, 16)) {
    int loc[3] = {-1, -1, -1};
    if (hipDeviceGetAttribute(&loc[0], hipDeviceAttributePciDomainID, dev) != hipSuccess ||
        hipDeviceGetAttribute(&loc[1], hipDeviceAttributePciBusId, dev) != hipSuccess ||
        hipDeviceGetAttribute(&loc[2], hipDeviceAttributePciDeviceId, dev) != hipSuccess) {
      // no identity at all: every GPU would look alike (the caller fails the set-up)
      clear_error("emac_gpu_device_uuid: PCI location");
      return EMAC_ERR_DEVICE;
    }
    uuid[0] = 0xff;  // never a real all-zero UUID
    memcpy(uuid + 4, loc, sizeof(loc));
  }
  return 0;
}

int emac_gpu_ipc_export(const void *p, void *handle, long *offset) {
  void *base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, const_cast<void *>(p)) != hipSuccess) {
    clear_error("emac_gpu_ipc_export: hipMemGetAddressRange");
    return EMAC_ERR_ARG;
  }
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, base) != hipSuccess) {
    clear_error("emac_gpu_ipc_export: hipIpcGetMemHandle");
    if (getenv("EXT_MPI_AMD_DEBUG_HIP")) fprintf(stderr, "ext_mpi_amd: export of %p (base %p, %zu bytes) refused\n", p, base, size);
    return EMAC_ERR_TRANSPORT;
  }
  memcpy(handle, &h, sizeof(h));
  *offset = (long)((const char *)p - (const char *)base);
  return 0;
}

int emac_gpu_ipc_open(const void *handle, void **base) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  if (hipIpcOpenMemHandle(base, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
    clear_error("emac_gpu_ipc_open");
    *base = nullptr;
    return EMAC_ERR_TRANSPORT;
  }
  return 0;
}

int emac_gpu_ipc_close(void *base) { return base ? ok(hipIpcCloseMemHandle(base)) : 0; }

unsigned long long emac_gpu_buffer_id(const void *p) {
  unsigned long long id = 0;
  if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
    clear_error("emac_gpu_buffer_id");
    return 0;
  }
  return id;
}

long emac_gpu_alloc_extent(const void *p, void **base) {
  size_t size = 0;
  *base = nullptr;
  if (hipMemGetAddressRange(base, &size, const_cast<void *>(p)) != hipSuccess) {
    clear_error("emac_gpu_alloc_extent");
    return -1;
  }
  return (long)size;
}

/* A device buffer is exported in place when the runtime knows its allocation (hipMemGetAddressRange):
   small hipMallocs are sub-allocated out of a shared chunk and their handle maps that chunk into
   the peers, which is harmless (the kernels touch only the message range) and every mapping is
   validated by the set-up probe anyway (engine.c ipc_exchange). */
int emac_gpu_ipc_exportable(const void *p) {
  void *base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, const_cast<void *>(p)) != hipSuccess) {
    clear_error("emac_gpu_ipc_exportable");
    return 0;
  }
  return size > 0;
}

int emac_gpu_malloc_uncached(void **p, size_t bytes) {
  *p = nullptr;
  bytes = (bytes + EMAC_IPC_GRANULE - 1) / EMAC_IPC_GRANULE * EMAC_IPC_GRANULE; /* exported whole */
  if (hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached) != hipSuccess) {
    clear_error("emac_gpu_malloc_uncached");
    return EMAC_ERR_MALLOC;
  }
  if (hipMemset(*p, 0, bytes) != hipSuccess) return EMAC_ERR_DEVICE;
  return 0;
}

int emac_gpu_host_alloc_mapped(void **p, size_t bytes) {
  *p = nullptr;
  if (hipHostMalloc(p, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    clear_error("emac_gpu_host_alloc_mapped");
    return EMAC_ERR_MALLOC;
  }
  memset(*p, 0, bytes);
  return 0;
}

int emac_gpu_host_free(void *p) { return p ? ok(hipHostFree(p)) : 0; }

int emac_gpu_event_create_release(void **ev) {
  hipEvent_t e;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToSystem) != hipSuccess) return EMAC_ERR_DEVICE;
  *ev = e;
  return 0;
}

long emac_gpu_wallclock_hz(void) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
    return 100000000L;  // gfx9 s_memrealtime runs at 100 MHz
  return (long)khz * 1000L;
}

int emac_gpu_node_barrier(void *self, void *const *d_peers, int slot, int phase, unsigned long epoch, unsigned long tag,
                          int nranks, int me, int *err, long timeout_ticks, void *stream) {
  const emac::NodeSync ns = {static_cast<emac_sync *>(self), reinterpret_cast<emac_sync *const *>(d_peers), slot,
                             nranks, me, err, timeout_ticks, tag};
  hipLaunchKernelGGL(node_barrier_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), ns, phase, epoch);
  return ok(hipGetLastError());
}

int emac_gpu_node_signal(void *const *d_peers, int slot, int phase, unsigned long epoch, int nranks, int me, void *stream) {
  const emac::NodeSync ns = {nullptr, reinterpret_cast<emac_sync *const *>(d_peers), slot, nranks, me, nullptr, 0, 0};
  hipLaunchKernelGGL(node_signal_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), ns, phase, epoch);
  return ok(hipGetLastError());
}

int emac_gpu_node_wait(void *self, void *const *d_peers, int slot, int phase, unsigned long epoch, unsigned long tag,
                       int nranks, int me, int *err, long timeout_ticks, void *stream) {
  const emac::NodeSync ns = {static_cast<emac_sync *>(self), reinterpret_cast<emac_sync *const *>(d_peers), slot,
                             nranks, me, err, timeout_ticks, tag};
  hipLaunchKernelGGL(node_wait_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), ns, phase, epoch);
  return ok(hipGetLastError());
}

}  // extern "C"
