/*
 * gpu.h -- internal C ABI between the host C engine and the HIP code (fold.hip).
 *
 * Replaces the reference's device C-ABI include/gpu/gpu_core.h:11-22 (ext_mpi_gpu_malloc,
 * _free, _memcpy_hd/_dh, _is_device_pointer, _synchronize, _copy_reduce). Differences that
 * matter on MI355X: sizes are size_t (the reference's int caps buffers at 2 GiB, far below
 * 288 GB of HBM3E), every operation is stream-ordered instead of device-synchronous, and
 * the fold takes per-chunk bucket descriptors instead of a per-element descriptor walk.
 */
#ifndef EMAC_GPU_H_
#define EMAC_GPU_H_

#include <stddef.h>
#include "plan.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One owner chunk of a launch: `nsrc` leaves (plan leaf order) folded element-wise and the
   result stored to `ndst` destinations. Element e of the chunk is at src[t] + e (elements). */
typedef struct {
  const void *src[EMAC_MAX_RANKS]; /* leaf pointers at element `head` (the first full vector) */
  long nvec;   /* 16-byte vectors from there (0 if the bucket is misaligned) */
  long tile0;  /* first tile index of this bucket inside the vector launch */
  void *dst[EMAC_MAX_RANKS];       /* destination pointers at element `head` */
  long count;  /* elements */
  long head;   /* leading elements before the first 16-byte aligned vector (edge path) */
  long tail;   /* trailing elements after the vectors (edge path) */
  int ndst;
  int scalar;  /* 1: pointers disagree on 16-byte alignment -> every element on the edge path */
} emac_bucket;

/* Element-granular work kept out of the streaming kernel: the unaligned head and tail of a
   bucket (mode 0), or a range of a misaligned bucket (mode 1). One workgroup per item. */
typedef struct {
  int bucket;
  int mode;
  long start, count;
} emac_edge;
#define EMAC_EDGE_RANGE 65536

#define EMAC_BLOCK 256
/* deferred-store launches over buckets of unequal tile counts: at most this many buckets, whose
   first groups the kernel keeps in LDS (layout.c emac_layout_as; tiles_per_bucket -1 marks them) */
#define EMAC_GROUP_MAP_MAX 64

int emac_gpu_device_count(void);
int emac_gpu_get_device(int *dev);
int emac_gpu_set_device(int dev);
int emac_gpu_malloc(void **p, size_t bytes);
int emac_gpu_free(void *p);
int emac_gpu_memcpy(void *dst, const void *src, size_t bytes); /* synchronous, any direction */
int emac_gpu_memcpy_async(void *dst, const void *src, size_t bytes, void *stream);
int emac_gpu_memset_async(void *dst, int v, size_t bytes, void *stream);
int emac_gpu_is_device_pointer(const void *p);
int emac_gpu_pinned_view(const void *p, void **dev); /* page-locked host memory: its device address */
int emac_gpu_host_register(void *p, size_t bytes);
int emac_gpu_host_unregister(void *p);
int emac_gpu_stream_create(void **stream);
int emac_gpu_stream_destroy(void *stream);
int emac_gpu_stream_sync(void *stream);
int emac_gpu_stream_query(void *stream); /* 1 idle, 0 busy, <0 error */
int emac_gpu_device_sync(void);
int emac_gpu_event_create(void **ev); /* timing disabled */
int emac_gpu_event_create_timed(void **ev);
int emac_gpu_event_elapsed_us(void *a, void *b, float *us); /* waits for b */
int emac_gpu_event_destroy(void *ev);
int emac_gpu_event_record(void *ev, void *stream);
int emac_gpu_stream_wait(void *stream, void *ev); /* stream waits for ev */
/* stream capture into an instantiated graph (thread-local capture mode) */
int emac_gpu_capture_begin(void *stream);
int emac_gpu_capture_end(void *stream, void **exec); /* ends the capture; exec NULL on failure */
int emac_gpu_graph_launch(void *exec, void *stream);
int emac_gpu_graph_destroy(void *exec);

/* ---- peer-mapped (IPC) form, ipc.hip ----
   Per-communicator synchronisation block, in uncached device memory and mapped by every peer:
   flags[slot][phase][q] = last epoch rank q signalled to this rank for that handle slot and
   barrier phase (0: before the fold, 1: after it); arrive = workgroups of this rank's running
   fused launch that finished their fold (the last one signals phase 1); aborted[slot][t & 1] = t
   when some peer gave up on the Start tagged t (a phase-0 timeout: it skipped its fold, so this
   rank's result is incomplete); go[slot] = this rank's phase-0 verdict for the fold launch that
   follows it on the stream (0: a peer did not arrive, store nothing). ipc_sync.hpp. */
#define EMAC_SYNC_SLOTS 1024
#define EMAC_IPC_HANDLE_BYTES 64
typedef struct {
  unsigned long flags[EMAC_SYNC_SLOTS][2][EMAC_MAX_RANKS];
  unsigned long arrive[EMAC_SYNC_SLOTS];
  unsigned long aborted[EMAC_SYNC_SLOTS][2];
  unsigned int go[EMAC_SYNC_SLOTS];
  unsigned char probe[EMAC_MAX_RANKS][8]; /* set-up only: byte [q][0] flipped by peer q through its mapping */
} emac_sync;
/* barrier error bits (the per-slot pinned host word) */
#define EMAC_SYNC_ERR_TIMEOUT 1 /* a peer did not arrive within the timeout */
#define EMAC_SYNC_ERR_ABORTED 2 /* a peer gave up on this Start */

int emac_gpu_ipc_export(const void *p, void *handle, long *offset); /* handle of p's allocation + offset */
int emac_gpu_ipc_open(const void *handle, void **base);
int emac_gpu_ipc_close(void *base);
long emac_gpu_alloc_extent(const void *p, void **base); /* bytes of the allocation holding p, or -1 */
unsigned long long emac_gpu_buffer_id(const void *p);   /* unique id of the allocation, 0 if unknown */
#define EMAC_IPC_GRANULE (2ul << 20) /* library-owned exported allocations: 2 MiB multiples */
int emac_gpu_ipc_exportable(const void *p); /* p lies in a device allocation the runtime can export */
int emac_gpu_malloc_uncached(void **p, size_t bytes); /* zeroed, rounded up to EMAC_IPC_GRANULE */
/* byte probes (IPC set-up): store vals[i] at ptrs[i] / load ptrs[i] into vals[i], system-coherent,
   complete on return */
#define EMAC_PROBE_MAX (2 * EMAC_MAX_RANKS)
int emac_gpu_poke(void *const *ptrs, const unsigned char *vals, int n, void *stream);
int emac_gpu_peek(const void *const *ptrs, unsigned char *vals, int n, void *stream);
/* read-only samples (IPC set-up): EMAC_SAMPLE_BYTES bytes of each of n buffers of lens[i] bytes
   into out[i * EMAC_SAMPLE_BYTES ...] -- EMAC_SAMPLE_SPOTS spots of 8 bytes spread over the buffer
   (the whole buffer, zero-padded, when shorter) -- system-coherent, complete on return */
#define EMAC_SAMPLE_SPOTS 8
#define EMAC_SAMPLE_BYTES (8 * EMAC_SAMPLE_SPOTS)
int emac_gpu_sample(const void *const *ptrs, const long *lens, int n, unsigned char *out, void *stream);
int emac_gpu_device_uuid(unsigned char *uuid); /* 16 bytes identifying the current device */
int emac_gpu_host_alloc_mapped(void **p, size_t bytes); /* pinned, device-visible, zeroed */
int emac_gpu_host_free(void *p);
long emac_gpu_wallclock_hz(void);
/* system-scope release of everything enqueued on `stream` so far, by the command processor on
   every XCD's L2 (an event recorded with hipEventReleaseToSystem): the peers' loads of this
   rank's buffers after the next barrier see it wherever its writers ran */
int emac_gpu_event_create_release(void **ev);
/* node barrier `phase` of the Start tagged `tag` (its phase-1 epoch) on `stream`: one wave */
int emac_gpu_node_barrier(void *self, void *const *d_peers, int slot, int phase, unsigned long epoch, unsigned long tag,
                          int nranks, int me, int *err, long timeout_ticks, void *stream);
/* The peer-mapped node join pipelined by parts in one launch per Start (join_fused.hip): per part
   the copy-in, share-fold and pull segments (stage * EMAC_JOIN_PARTS_MAX + part), each part's
   synchronisation slot and this Start's epochs for it; `ctl` a zeroed emac_join_ctl in device
   memory (the kernel leaves it zeroed). mode: 1 the copy-ins, 2 the node legs (barriers, share
   folds, pulls), 3 both; | 4 when every node runs on this GPU (device-scope write-through of the
   partial instead of system scope). segs NULL: whether the shape has a kernel (0) or not. */
#define EMAC_JOIN_PARTS_MAX 8
typedef struct {
  unsigned tk[3][EMAC_JOIN_PARTS_MAX];   /* per segment (stage, part): the next unclaimed item */
  unsigned done[3][EMAC_JOIN_PARTS_MAX]; /* ... items finished */
  unsigned sig[3][EMAC_JOIN_PARTS_MAX];  /* ... its completion signalled */
  unsigned failed0[EMAC_JOIN_PARTS_MAX], failed1[EMAC_JOIN_PARTS_MAX]; /* a part's barrier failed */
  unsigned out;                                                        /* workgroups done */
} emac_join_ctl;
typedef struct {
  const emac_bucket *d_buckets;
  int nb;
  long ntiles, tiles_per_bucket;
  int all_full;
  const emac_edge *d_edges;
  int nedges;
} emac_join_seg;
int emac_gpu_join_fused(int dtype, int nsrc, const emac_codes *codes, const emac_codes *xcodes, int nparts, int mode,
                        const emac_join_seg *segs, const int *slots, const unsigned long *e0, const unsigned long *e1,
                        void *self_sync, void *const *d_peers, int nranks, int me, int *err, long timeout_ticks, void *ctl,
                        int grid, void *stream);
int emac_gpu_join_grid(void); /* workgroups of the fused join's launch (one per CU) */

/* the two halves of a node barrier (the pipelined node join, engine_join.c), one wave each: signal
   phase `phase` with `epoch` to every peer; wait for every peer's signal (phase 0: and leave the
   verdict in go[slot] for the fold launch behind it, marking the Start abandoned in the peers'
   blocks on a timeout; phase 1: report a timeout or a peer that gave up, as the whole barrier) */
int emac_gpu_node_signal(void *const *d_peers, int slot, int phase, unsigned long epoch, int nranks, int me, void *stream);
int emac_gpu_node_wait(void *self, void *const *d_peers, int slot, int phase, unsigned long epoch, unsigned long tag,
                       int nranks, int me, int *err, long timeout_ticks, void *stream);
/* the whole peer-mapped Allreduce (barrier, fold, barrier, pull) in one launch, small messages.
   The grid is kept small (as many workgroups as tiles, at most 64): every workgroup spins while a
   peer is late, and a wide grid would hold that many CUs from the rank's other streams. */
#define EMAC_FUSED_MAX_WG 64
int emac_gpu_fold_fused(int dtype, int op, int nsrc, int unroll, const emac_codes *codes, const emac_bucket *d_buckets, int nb,
                        long ntiles, long tiles_per_bucket, int all_full, const emac_edge *d_edges, int nedges,
                        const emac_bucket *d_pull, int pnb, long pntiles, long ptiles_per_bucket, int pall_full,
                        const emac_edge *d_pedges, int pnedges, void *self_sync, void *const *d_peers, int slot,
                        int nranks, int me, int *err, long timeout_ticks, unsigned long epoch0, unsigned long epoch1,
                        void *stream);

/* Launch schedule: unroll U (16-byte vectors per lane per leaf; a tile covers EMAC_BLOCK * U
   vectors) in the low 4 bits, load-issue schedule above (fold_kernel.hpp). fan: the fan-out
   width equals nsrc (node / IPC form) instead of 1. */
#define EMAC_FAN_HOST 4 /* or-ed into pick_unroll's fan: node fan-out over page-locked host memory */
int emac_gpu_pick_unroll(int op, int nsrc, int tree, int fan, long total_vectors);

/* Launch the fold over nb device-resident buckets (ntiles tiles in total) on `stream`.
   tiles_per_bucket > 0 declares that every bucket spans exactly that many tiles. */
int emac_gpu_fold(int dtype, int op, int nsrc, int fan, int unroll, const emac_codes *codes,
                  const emac_bucket *d_buckets, int nb, long ntiles, long tiles_per_bucket, int all_full,
                  const emac_edge *d_edges, int nedges, void *stream);
/* 1 when emac_gpu_fold has a kernel for this shape and schedule (tree: emac_tree_kind; uniform:
   every bucket the same tile count, which the deferred-store schedules need), else 0 */
int emac_gpu_fold_supported(int dtype, int op, int nsrc, int fan, int tree, int unroll, int uniform);
/* the same for a peer-mapped launch (fan 2): `go` is the device word the phase-0 barrier before
   it wrote (emac_sync.go[slot]); a workgroup that reads 0 stores nothing */
int emac_gpu_fold_remote(int dtype, int op, int nsrc, int unroll, const emac_codes *codes, const emac_bucket *d_buckets,
                         int nb, long ntiles, long tiles_per_bucket, int all_full, const emac_edge *d_edges, int nedges,
                         const unsigned *go, void *stream);

/* Copy fan-out (fold_copy.hip): every bucket's one leaf stored into its `width` destinations
   (1 .. EMAC_MAX_RANKS - 1), bits moved unchanged; tsize = element bytes (4 or 8). */
int emac_gpu_copy_fan(int tsize, int width, int unroll, const emac_bucket *d_buckets, int nb, long ntiles,
                      long tiles_per_bucket, int all_full, const emac_edge *d_edges, int nedges, void *stream);
/* the peer-mapped pull with fan-out: one leaf in a peer's memory (system-coherent loads), `width`
   destinations (<= EMAC_MAX_RANKS); `go`: the phase-0 verdict word */
int emac_gpu_copy_fan_remote(int tsize, int width, int unroll, const emac_bucket *d_buckets, int nb, long ntiles,
                             long tiles_per_bucket, int all_full, const emac_edge *d_edges, int nedges, const unsigned *go,
                             void *stream);

/* Fold-tree kind of a plan's codes (fold_kernel.hpp template parameter CH): 0 linear (one
   radix), a packed compile-time radix chain (5 bits per level, level 0 lowest) when the kernels
   instantiate it -- EMAC_CHAINS: -2 -2, -2 -2 -2, -4 -2, -2 -4, -2 -2 -2 -2, -4 -4 -- else 1
   (replayed from the runtime level codes). SUM only; MIN / MAX always take the runtime codes. */
#define EMAC_CH(r0, r1, r2, r3) ((r0) | (r1) << 5 | (r2) << 10 | (r3) << 15)
#define EMAC_CHAINS                                                                             \
  { EMAC_CH(2, 2, 0, 0), EMAC_CH(2, 2, 2, 0), EMAC_CH(4, 2, 0, 0), EMAC_CH(2, 4, 0, 0), EMAC_CH(2, 2, 2, 2), \
    EMAC_CH(4, 4, 0, 0) }
int emac_tree_kind(const emac_codes *codes, int op);

/* layout.c: alignment split of a bucket whose pointers sit at its first element, and the
   launch layout (tiles, uniform tiles per bucket, unroll, edge items; caller frees edges). */
void emac_split_alignment(emac_bucket *b, int nsrc, long len, int tsize);
/* tree: 1 for a runtime-code tree (emac_tree_kind == 1), which has its own launch schedules */
int emac_layout(emac_bucket *b, int nb, int op, int nsrc, int tree, int fan, emac_edge **edges, int *nedges,
                long *ntiles, long *tiles_per_bucket, int *all_full, int *unroll);
/* the same with the launch schedule given (forced = U | ISSUE << 4; 0: emac_gpu_pick_unroll) */
int emac_layout_as(emac_bucket *b, int nb, int op, int nsrc, int tree, int fan, int forced, emac_edge **edges,
                   int *nedges, long *ntiles, long *tiles_per_bucket, int *all_full, int *unroll);

#ifdef __cplusplus
}
#endif
#endif
