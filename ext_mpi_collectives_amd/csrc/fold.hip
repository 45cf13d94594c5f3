// fold.hip -- CDNA4 (gfx950) kernels of the bucket-reduction hot path + the HIP runtime ABI.
//
// Replaces gpu_copy_reduce_kernel<T> (reference src/gpu/cuda_core.cu:50-86) and its C-ABI
// (cuda_core.cu:7-106, include/gpu/gpu_core.h:11-22).
//
// The reference kernel walks a per-element descriptor chain in global memory (integer / and %
// per element), reloads and re-stores dst once per SREDUCE line, and writes each fan-out copy
// in a separate launch. Here one launch covers every owner chunk ("bucket") of a plan:
//   * each lane owns 16-byte vectors (dwordx4) of a chunk, U vectors per source in flight;
//   * all R leaf sources are loaded once into VGPRs, then folded in registers in the exact
//     order the reference's SMEMCPY + SREDUCE lines apply them (plan.c's fold tree replayed
//     through per-leaf level codes: a left fold per recursive-halving step, nested);
//   * the result is stored once per destination (fused copy-out fan-out), never re-read.
// HBM traffic per bucket is therefore R reads + D writes of the chunk, the algorithmic
// minimum; the element-wise add is VALU work hidden under the loads (no MFMA: there is no
// contraction here). Integer sums are computed in unsigned arithmetic (two's complement wrap,
// bit-identical to the reference's x86 behaviour without signed-overflow UB); float/double
// keep IEEE round-to-nearest with denormals (no fast-math, no FTZ flags at build time).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#include "fold_kernel.hpp"
#include "gpu.h"

extern "C" {
#define EMAC_DECL(n)                                                                                         \
  int emac_fold_launch_##n(int nsrc, int ch, int fan, int unroll, const emac::Launch *L);                   \
  int emac_fold_launch_##n##_mm(int op, int fan, int unroll, const emac::Launch *L);                        \
  int emac_fold_fused_launch_##n(int nsrc, int ch, const emac::Launch *L, const emac::FusedLaunch *F);       \
  int emac_fold_fused_launch_##n##_mm(int op, const emac::Launch *L, const emac::FusedLaunch *F);
EMAC_DECL(f32)
EMAC_DECL(f64)
EMAC_DECL(i32)
EMAC_DECL(i64)
#undef EMAC_DECL
}

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

}  // namespace

extern "C" {

int emac_gpu_pick_unroll(int op, int nsrc, int tree, int fan, long total_vectors) {
  // returns U | ISSUE << 4 (fold_kernel.hpp, instantiation policy). `tree`: a runtime-code tree
  // (compile-time radix chains take the linear schedules). Measured on MI355X, R = 8 float:
  //  * node form (tools/ldsbench.hip, profiles/r01_ldsbench_issue_*): a back-to-back burst of
  //    every load of a tile wins at <= 2 MiB and >= 64 MiB per rank; between them U = 4 with an
  //    s_sleep after every 4 loads is 4-8 % faster (16 MiB: 41.9 vs 45.2-45.4 us); 64 MiB per
  //    rank prefers U = 2 (183 vs 194 us), >= 128 MiB U = 4;
  //  * one destination (the COMM / IPC owner's local fold, tools/localbench.hip,
  //    profiles/r02_localbench_*): U = 1 up to 1 MiB per leaf, U = 2 at 2 MiB, U = 4 from 4 MiB
  //    (8 x 32 MiB -> 1: 48.2 us at U = 4 against 50.2-50.5 at U = 2; U = 8 within 0.5 % of U = 4).
  using emac::sched;
  const int host = fan & EMAC_FAN_HOST;
  fan &= ~EMAC_FAN_HOST;
  if (op != EMAC_SUM && nsrc > 1) return sched(1, fan == 2 ? 1 | emac::kRemote : 1); /* runtime-leaf-count kernels */
  if (fan == 2) {  // peer-mapped (IPC) form: one system-coherent schedule per shape
    if (tree && nsrc > 1) return sched(emac::tree_unroll(nsrc), 1 | emac::kRemote);
    return sched(nsrc > 8 ? 1 : 2, 1 | emac::kRemote);
  }
  if (nsrc == 1) return total_vectors >= 2048L * EMAC_BLOCK * 2 ? sched(2, 1) : sched(1, 1);
  if (tree) {
    // radix-chain trees at U = 2 (5 <= leaves <= 8): the same staggered issue wins in the
    // middle range (16 MiB x 8, '-2 -2 -2': 44.2 vs 47.4 us), bursts at the ends
    if (fan && nsrc > 4 && nsrc <= 8 && total_vectors >= (192L << 10) && total_vectors < (3L << 20)) return sched(2, 5);
    return sched(emac::tree_unroll(nsrc), 1);
  }
  if (nsrc > 8) return sched(1, 1);
  if (fan) {
    // page-locked host buffers (NODE form): every access crosses PCIe, where a CU's own request
    // rate, not HBM, binds -- the smallest tiles spread a message over the most CUs (better up
    // to 16 MiB per rank, equal at 64 MiB: profiles/r01_host_direct_sweep.json)
    if (host) return sched(1, 1);
    if (total_vectors < (192L << 10)) return sched(2, 1);
    if (total_vectors < (3L << 20)) return sched(4, 5);
    if (total_vectors < (6L << 20)) return sched(2, 1);
    return sched(4, 1);
  }
  if (nsrc <= 8 && total_vectors >= (256L << 10)) return sched(4, 1); /* >= 4 MiB per leaf */
  if (nsrc <= 8 && total_vectors >= (128L << 10)) return sched(2, 1);
  return total_vectors >= 2048L * EMAC_BLOCK * 2 ? sched(2, 1) : sched(1, 1);
}

static int fold_dispatch(int dtype, int op, int nsrc, int fan, int unroll, const emac::Launch &L, int ch) {
  switch (dtype) {
  case EMAC_FLOAT:
    return op == EMAC_SUM ? emac_fold_launch_f32(nsrc, ch, fan, unroll, &L) : emac_fold_launch_f32_mm(op, fan, unroll, &L);
  case EMAC_DOUBLE:
    return op == EMAC_SUM ? emac_fold_launch_f64(nsrc, ch, fan, unroll, &L) : emac_fold_launch_f64_mm(op, fan, unroll, &L);
  case EMAC_INT:
    return op == EMAC_SUM ? emac_fold_launch_i32(nsrc, ch, fan, unroll, &L) : emac_fold_launch_i32_mm(op, fan, unroll, &L);
  case EMAC_LONG:
    return op == EMAC_SUM ? emac_fold_launch_i64(nsrc, ch, fan, unroll, &L) : emac_fold_launch_i64_mm(op, fan, unroll, &L);
  }
  return EMAC_ERR_ARG;
}

int emac_gpu_fold(int dtype, int op, int nsrc, int fan, int unroll, const emac_codes *codes,
                  const emac_bucket *d_buckets, int nb, long ntiles, long tiles_per_bucket, int all_full,
                  const emac_edge *d_edges, int nedges, void *stream) {
  const int ch = emac_tree_kind(codes, op); /* fan: 0 one destination, 1 node fan-out */
  const emac::Launch L = {codes, d_buckets, nb, ntiles, tiles_per_bucket, all_full, d_edges, nedges,
                          static_cast<hipStream_t>(stream), nullptr, nsrc};
  if (op < EMAC_SUM || op > EMAC_MAX) return EMAC_ERR_UNSUPPORTED;
  if (fan != 0 && fan != 1) return EMAC_ERR_ARG; /* peer-mapped launches: emac_gpu_fold_remote */
  if (nb <= 0 || (ntiles <= 0 && nedges <= 0)) return 0;
  if (codes->nlev > emac::kMaxLevels) return EMAC_ERR_UNSUPPORTED;
  return fold_dispatch(dtype, op, nsrc, fan, unroll, L, ch);
}

int emac_gpu_fold_supported(int dtype, int op, int nsrc, int fan, int tree, int unroll, int uniform) {
  static const emac_codes none = {{0}, {0}, 1, 0};
  emac::Launch L = {&none, nullptr, 1, 1, uniform ? 1 : 0, 1, nullptr, 0, nullptr, nullptr, nsrc};
  L.dry = true;
  if (op < EMAC_SUM || op > EMAC_MAX || (fan != 0 && fan != 1)) return 0;
  return fold_dispatch(dtype, op, nsrc, fan, unroll, L, tree) == 0;
}

int emac_copy_fan_launch(int tsize, int width, int unroll, const emac::Launch *L);

int emac_gpu_copy_fan(int tsize, int width, int unroll, const emac_bucket *d_buckets, int nb, long ntiles,
                      long tiles_per_bucket, int all_full, const emac_edge *d_edges, int nedges, void *stream) {
  static const emac_codes copy = {{1}, {1}, 1, 1}; /* one leaf */
  const emac::Launch L = {&copy, d_buckets, nb, ntiles, tiles_per_bucket, all_full, d_edges, nedges,
                          static_cast<hipStream_t>(stream), nullptr, 1};
  if (width < 1 || width >= EMAC_MAX_RANKS) return EMAC_ERR_ARG;
  if (nb <= 0 || (ntiles <= 0 && nedges <= 0)) return 0;
  return emac_copy_fan_launch(tsize, width, unroll, &L);
}

int emac_copy_fan_remote_launch(int tsize, int width, int unroll, const emac::Launch *L);

int emac_gpu_copy_fan_remote(int tsize, int width, int unroll, const emac_bucket *d_buckets, int nb, long ntiles,
                             long tiles_per_bucket, int all_full, const emac_edge *d_edges, int nedges, const unsigned *go,
                             void *stream) {
  static const emac_codes copy = {{1}, {1}, 1, 1}; /* one leaf */
  const emac::Launch L = {&copy, d_buckets, nb, ntiles, tiles_per_bucket, all_full, d_edges, nedges,
                          static_cast<hipStream_t>(stream), go, 1};
  if (width < 1 || width > EMAC_MAX_RANKS || !go) return EMAC_ERR_ARG;
  if (nb <= 0 || (ntiles <= 0 && nedges <= 0)) return 0;
  return emac_copy_fan_remote_launch(tsize, width, unroll, &L);
}

int emac_gpu_fold_remote(int dtype, int op, int nsrc, int unroll, const emac_codes *codes, const emac_bucket *d_buckets,
                         int nb, long ntiles, long tiles_per_bucket, int all_full, const emac_edge *d_edges, int nedges,
                         const unsigned *go, void *stream) {
  const int ch = emac_tree_kind(codes, op);
  const emac::Launch L = {codes, d_buckets, nb, ntiles, tiles_per_bucket, all_full, d_edges, nedges,
                          static_cast<hipStream_t>(stream), go, nsrc};
  if (op < EMAC_SUM || op > EMAC_MAX) return EMAC_ERR_UNSUPPORTED;
  if (!go) return EMAC_ERR_ARG;
  if (nb <= 0 || (ntiles <= 0 && nedges <= 0)) return 0;
  if (codes->nlev > emac::kMaxLevels) return EMAC_ERR_UNSUPPORTED;
  return fold_dispatch(dtype, op, nsrc, 2, unroll, L, ch);
}

int emac_gpu_fold_fused(int dtype, int op, int nsrc, int unroll, const emac_codes *codes, const emac_bucket *d_buckets, int nb,
                        long ntiles, long tiles_per_bucket, int all_full, const emac_edge *d_edges, int nedges,
                        const emac_bucket *d_pull, int pnb, long pntiles, long ptiles_per_bucket, int pall_full,
                        const emac_edge *d_pedges, int pnedges, void *self_sync, void *const *d_peers, int slot,
                        int nranks, int me, int *err, long timeout_ticks, unsigned long epoch0, unsigned long epoch1,
                        void *stream) {
  const int ch = emac_tree_kind(codes, op);
  const emac::Launch L = {codes, d_buckets, nb, ntiles, tiles_per_bucket, all_full, d_edges, nedges,
                          static_cast<hipStream_t>(stream), nullptr, nsrc};
  long work = ntiles + nedges;
  if (pntiles + pnedges > work) work = pntiles + pnedges;
  emac::FusedLaunch F;
  F.pull = {d_pull, pnb, pntiles, ptiles_per_bucket, pall_full, d_pedges, pnedges};
  F.ns = {static_cast<emac_sync *>(self_sync), reinterpret_cast<emac_sync *const *>(d_peers), slot, nranks, me,
          err, timeout_ticks, epoch1};
  F.epoch0 = epoch0;
  F.epoch1 = epoch1;
  /* at most EMAC_FUSED_MAX_WG workgroups: all resident while others wait, few CUs held from the
     rank's other streams while a peer is late */
  F.grid = (int)(work < 1 ? 1 : work > EMAC_FUSED_MAX_WG ? EMAC_FUSED_MAX_WG : work);
  if (codes->nlev > emac::kMaxLevels || nsrc < 2) return EMAC_ERR_UNSUPPORTED;
  if (op < EMAC_SUM || op > EMAC_MAX) return EMAC_ERR_UNSUPPORTED;
  if (nb > 0 && unroll != emac_gpu_pick_unroll(op, nsrc, ch == 1, 2, 0)) return EMAC_ERR_UNSUPPORTED; /* layout's tiles */
  if (pnb > 0 && emac_gpu_pick_unroll(EMAC_SUM, 1, 0, 2, 0) != emac::sched(2, 1 | emac::kRemote)) return EMAC_ERR_UNSUPPORTED;
  if (nb <= 0 && pnb <= 0) {
    F.grid = 1; /* nothing to fold or pull here: the barriers only */
    return emac_fold_fused_launch_f32(nsrc, 0, &L, &F);
  }
  switch (dtype) {
  case EMAC_FLOAT:
    return op == EMAC_SUM ? emac_fold_fused_launch_f32(nsrc, ch, &L, &F) : emac_fold_fused_launch_f32_mm(op, &L, &F);
  case EMAC_DOUBLE:
    return op == EMAC_SUM ? emac_fold_fused_launch_f64(nsrc, ch, &L, &F) : emac_fold_fused_launch_f64_mm(op, &L, &F);
  case EMAC_INT:
    return op == EMAC_SUM ? emac_fold_fused_launch_i32(nsrc, ch, &L, &F) : emac_fold_fused_launch_i32_mm(op, &L, &F);
  case EMAC_LONG:
    return op == EMAC_SUM ? emac_fold_fused_launch_i64(nsrc, ch, &L, &F) : emac_fold_fused_launch_i64_mm(op, &L, &F);
  }
  return EMAC_ERR_ARG;
}

int emac_gpu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
int emac_gpu_get_device(int *dev) { return ok(hipGetDevice(dev)); }
int emac_gpu_set_device(int dev) { return ok(hipSetDevice(dev)); }
int emac_gpu_malloc(void **p, size_t bytes) {
  *p = nullptr;
  if (!bytes) return 0;
  return hipMalloc(p, bytes) == hipSuccess ? 0 : EMAC_ERR_MALLOC;
}
int emac_gpu_free(void *p) { return p ? ok(hipFree(p)) : 0; }
int emac_gpu_memcpy(void *dst, const void *src, size_t bytes) {
  return bytes ? ok(hipMemcpy(dst, src, bytes, hipMemcpyDefault)) : 0;
}
int emac_gpu_memcpy_async(void *dst, const void *src, size_t bytes, void *stream) {
  return bytes ? ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, static_cast<hipStream_t>(stream))) : 0;
}
int emac_gpu_memset_async(void *dst, int v, size_t bytes, void *stream) {
  return bytes ? ok(hipMemsetAsync(dst, v, bytes, static_cast<hipStream_t>(stream))) : 0;
}
int emac_gpu_is_device_pointer(const void *p) {
  hipPointerAttribute_t a;
  if (!p) return 0;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    clear_error("emac_gpu_is_device_pointer");  // unregistered host memory: clear the sticky error
    return 0;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}
int emac_gpu_pinned_view(const void *p, void **dev) {
  hipPointerAttribute_t a;
  if (!p) return EMAC_ERR_ARG;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    clear_error("emac_gpu_pinned_view");  // pageable host memory
    return EMAC_ERR_ARG;
  }
  if (a.type != hipMemoryTypeHost || !a.devicePointer) return EMAC_ERR_ARG;
  *dev = a.devicePointer;  // the device address of p itself (offset into the pinned range kept)
  return 0;
}
int emac_gpu_host_register(void *p, size_t bytes) {
  if (!bytes) return 0;
  if (hipHostRegister(p, bytes, hipHostRegisterDefault) != hipSuccess) {
    clear_error("emac_gpu_host_register");
    return EMAC_ERR_DEVICE;
  }
  return 0;
}
int emac_gpu_host_unregister(void *p) {
  if (hipHostUnregister(p) != hipSuccess) {
    clear_error("emac_gpu_host_unregister");
    return EMAC_ERR_DEVICE;
  }
  return 0;
}
int emac_gpu_stream_create(void **stream) {
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return EMAC_ERR_DEVICE;
  *stream = s;
  return 0;
}
int emac_gpu_stream_destroy(void *stream) { return ok(hipStreamDestroy(static_cast<hipStream_t>(stream))); }
int emac_gpu_stream_sync(void *stream) { return ok(hipStreamSynchronize(static_cast<hipStream_t>(stream))); }
int emac_gpu_stream_query(void *stream) {
  hipError_t e = hipStreamQuery(static_cast<hipStream_t>(stream));
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) {
    clear_error("emac_gpu_stream_query");
    return 0;
  }
  return EMAC_ERR_DEVICE;
}
int emac_gpu_device_sync(void) { return ok(hipDeviceSynchronize()); }
int emac_gpu_event_create(void **ev) {
  hipEvent_t e;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return EMAC_ERR_DEVICE;
  *ev = e;
  return 0;
}
int emac_gpu_event_create_timed(void **ev) {
  hipEvent_t e;
  /* timing only (the tuner's samples): no system-scope fence on record -- the default event's
     cache writeback and invalidate would sit between the launches it brackets and change how
     they run (the deferred-store schedules most) */
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return EMAC_ERR_DEVICE;
  *ev = e;
  return 0;
}
int emac_gpu_event_elapsed_us(void *a, void *b, float *us) {
  float ms = 0.f;
  int rc = ok(hipEventSynchronize(static_cast<hipEvent_t>(b)));
  if (!rc) rc = ok(hipEventElapsedTime(&ms, static_cast<hipEvent_t>(a), static_cast<hipEvent_t>(b)));
  *us = ms * 1000.f;
  return rc;
}
int emac_gpu_event_destroy(void *ev) { return ev ? ok(hipEventDestroy(static_cast<hipEvent_t>(ev))) : 0; }
int emac_gpu_event_record(void *ev, void *stream) {
  return ok(hipEventRecord(static_cast<hipEvent_t>(ev), static_cast<hipStream_t>(stream)));
}
int emac_gpu_stream_wait(void *stream, void *ev) {
  return ok(hipStreamWaitEvent(static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(ev), 0));
}
int emac_gpu_capture_begin(void *stream) {
  return ok(hipStreamBeginCapture(static_cast<hipStream_t>(stream), hipStreamCaptureModeThreadLocal));
}
int emac_gpu_capture_end(void *stream, void **exec) {
  hipGraph_t g = nullptr;
  hipGraphExec_t x = nullptr;
  *exec = nullptr;
  int rc = ok(hipStreamEndCapture(static_cast<hipStream_t>(stream), &g));
  if (!rc && g) rc = ok(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  if (g) (void)hipGraphDestroy(g);
  if (rc || !x) {
    clear_error("emac_gpu_capture_end");
    return rc ? rc : EMAC_ERR_DEVICE;
  }
  *exec = x;
  return 0;
}
int emac_gpu_graph_launch(void *exec, void *stream) {
  return ok(hipGraphLaunch(static_cast<hipGraphExec_t>(exec), static_cast<hipStream_t>(stream)));
}
int emac_gpu_graph_destroy(void *exec) { return exec ? ok(hipGraphExecDestroy(static_cast<hipGraphExec_t>(exec))) : 0; }

}  // extern "C"

// ---- exported device C ABI (include/ext_mpi_amd_gpu.h; reference include/gpu/gpu_core.h) ----
extern "C" {

int ext_mpi_amd_gpu_malloc(void **p, size_t bytes) { return emac_gpu_malloc(p, bytes); }
int ext_mpi_amd_gpu_free(void *p) { return emac_gpu_free(p); }
// hipMemcpyDefault: the direction follows the pointers (unified addressing), so the MPI layer's
// staging through device scratch also takes device-resident caller buffers
int ext_mpi_amd_gpu_memcpy_hd(void *dst, const void *src, size_t bytes) {
  return bytes ? ok(hipMemcpy(dst, src, bytes, hipMemcpyDefault)) : 0;
}
int ext_mpi_amd_gpu_memcpy_dh(void *dst, const void *src, size_t bytes) {
  return bytes ? ok(hipMemcpy(dst, src, bytes, hipMemcpyDefault)) : 0;
}
int ext_mpi_amd_gpu_memcpy_async(void *dst, const void *src, size_t bytes, void *hip_stream) {
  return emac_gpu_memcpy_async(dst, src, bytes, hip_stream);
}
int ext_mpi_amd_gpu_after_default_stream(void *hip_stream) {
  hipEvent_t e;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return EMAC_ERR_DEVICE;
  int rc = ok(hipEventRecord(e, nullptr));
  if (!rc) rc = ok(hipStreamWaitEvent(static_cast<hipStream_t>(hip_stream), e, 0));
  (void)hipEventDestroy(e);  // released once the wait has been satisfied
  return rc;
}
int ext_mpi_amd_gpu_is_device_pointer(const void *p) { return emac_gpu_is_device_pointer(p); }
int ext_mpi_amd_gpu_synchronize(void) { return emac_gpu_device_sync(); }
int ext_mpi_amd_gpu_device_count(void) { return emac_gpu_device_count(); }
int ext_mpi_amd_gpu_device_of(const void *p) {
  hipPointerAttribute_t a;
  if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
    clear_error("ext_mpi_amd_gpu_device_of");
    return -1;
  }
  return (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) ? a.device : -1;
}

// One owner chunk as a one-bucket launch (stream-ordered; the descriptor is staged through a
// small device scratch owned by the call and released after the launch completes).
int ext_mpi_amd_gpu_copy_reduce(int dtype, int op, int nsrc, const void *const *srcs, int ndst, void *const *dsts,
                                long count, void *hip_stream) {
  emac_bucket b;
  emac_codes codes;
  emac_bucket *d = nullptr;
  int tsize = emac_type_size(dtype), rc, i;
  if (tsize < 0 || nsrc < 1 || nsrc > EMAC_MAX_RANKS || ndst < 1 || ndst > EMAC_MAX_RANKS || count < 0)
    return EMAC_ERR_ARG;
  if (!count) return 0;
  memset(&b, 0, sizeof(b));
  memset(&codes, 0, sizeof(codes));
  codes.nlev = 1;
  codes.nleaf = nsrc;
  codes.first[0] = 1;
  codes.close[nsrc - 1] = 1;
  for (i = 0; i < nsrc; i++) b.src[i] = srcs[i];
  for (i = 0; i < ndst; i++) b.dst[i] = dsts[i];
  b.ndst = ndst;
  emac_split_alignment(&b, nsrc, count, tsize);
  emac_edge *edges = nullptr, *d_edges = nullptr;
  int nedges = 0, unroll = 1, all_full = 0;
  long ntiles = 0, tpb = 0;
  const int fan = ndst > 1;
  if (ndst > 1 && ndst != nsrc) return EMAC_ERR_UNSUPPORTED; /* fan-out width is 1 or nsrc */
  if ((rc = emac_layout(&b, 1, op, nsrc, 0, fan, &edges, &nedges, &ntiles, &tpb, &all_full, &unroll))) return rc;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  if (hipMallocAsync((void **)&d, sizeof(b) + sizeof(emac_edge) * (nedges + 1), s) != hipSuccess) {
    free(edges);
    return EMAC_ERR_MALLOC;
  }
  d_edges = reinterpret_cast<emac_edge *>(d + 1);
  rc = ok(hipMemcpyAsync(d, &b, sizeof(b), hipMemcpyHostToDevice, s));
  if (!rc && nedges) rc = ok(hipMemcpyAsync(d_edges, edges, sizeof(emac_edge) * nedges, hipMemcpyHostToDevice, s));
  if (!rc) rc = emac_gpu_fold(dtype, op, nsrc, fan, unroll, &codes, d, 1, ntiles, tpb, all_full, d_edges, nedges, hip_stream);
  (void)hipFreeAsync(d, s);
  if (!rc) rc = ok(hipStreamSynchronize(s));  // the host descriptor lives on this stack frame
  free(edges);
  return rc;
}

}  // extern "C"
