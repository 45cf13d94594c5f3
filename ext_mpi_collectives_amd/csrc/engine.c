/*
 * engine.c -- persistent-Allreduce handles of the MI355X bucket-reduction path (host C).
 *
 * Mirrors the reference's handle life cycle (src/mpi/ext_mpi_native.c: init :657-1113 with
 * init_epilogue :389-655, Start :215-230, Test/Wait :232-267, Done :269-387) without its
 * text-IR pipeline: at init the planner (plan.c) fixes every owner chunk's fold tree, the
 * device-side bucket descriptors are written once (the analogue of byte_code.c:987-992's
 * descriptor H2D copy), buffers are mapped once; Start only enqueues work on the handle's
 * stream; Wait synchronises that stream.
 *
 * Two execution forms:
 *  NODE: all R node ranks' buffers live in this process (one device). One fold launch per
 *        Start performs copy-in (reduce-scatter) AND copy-out (allgather fan-out): every
 *        bucket reads its R leaves once and stores the result into all R receive buffers.
 *  COMM: one rank per GPU. The reduce-scatter leg moves each rank's slice of every owner
 *        chunk to the owner with grouped RCCL send/recv (one all-to-all round over the
 *        fully connected xGMI links instead of log R recursive-halving rounds, each of
 *        which would be bound by ONE 153 GB/s link); the owner folds the R slices in the
 *        reference's order (bit-exact); the allgather leg pushes the owned chunk to every
 *        peer, again as one grouped round. RCCL's own reductions are never used: their
 *        summation order differs from the reference's.
 * Host (non-device) buffers are supported in both forms by staging through device mirrors
 * (H2D before, D2H after, on the same stream); the buffers are page-locked once at init,
 * as the reference maps its XPMEM peers once (src/mpi/ext_mpi_xpmem.c:68-133).
 */
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "ext_mpi_amd.h"
#include "gpu.h"
#include "plan.h"

#define MAX_HANDLES 4096
#define MAX_COMMS 64

enum { KIND_NODE = 1, KIND_COMM = 2, KIND_IPC = 3 };

/* one peer allocation mapped into this process (hipIpcOpenMemHandle), shared by every handle and
   communicator that references the same allocation (the exporter's handle bytes, allocation id
   and size) and closed when the last of them is done, as the reference closes its cudaIpc
   mappings in EXT_MPI_Done (src/gpu/cuda_shmem.c:301-314). The table is process-wide: the
   runtime sub-allocates small device allocations out of shared chunks, so two communicators'
   synchronisation blocks (or two handles' buffers) of one peer can share a chunk, and opening
   the same chunk twice in one process is refused (measured: the second communicator's set-up
   failed with 8 processes on one MI355X). */
typedef struct {
  unsigned long long buf_id;
  long extent;
  unsigned char handle[EMAC_IPC_HANDLE_BYTES];
  void *base;
  int refs;
} ipc_map;

/* device mirrors of host buffers in the IPC form: exported to the peers, so they are never
   freed while a peer may still map them -- they return to this per-communicator pool at handle
   done and are released only by the (collective) communicator free. Freeing an exported
   allocation before every importer has closed it is undefined behaviour in HIP and was
   measured to corrupt the exporter's later allocations (8 ranks on one GPU). */
typedef struct {
  void *p;
  size_t bytes;
  int busy;
} ipc_mirror;

/* The arena of a peer-mapped communicator: per rank a few large device segments, each exported and
   mapped by every peer once, when it is added, and validated then (a nonce in its head); handles
   carve their outboxes and send-buffer mirrors out of them (first fit, free list per segment). */
#define EMAC_ARENA_SEGS 32
#define EMAC_ARENA_HEAD 256            /* the nonce */
#define EMAC_ARENA_ALIGN 256
#define EMAC_ARENA_MIN (64L << 20)     /* first segment */
typedef struct {
  long off, len;
} arena_free;
typedef struct {
  void *base;
  long bytes;
  arena_free *fr; /* free blocks, ascending offsets, coalesced */
  int nfr, capfr;
} arena_seg;

typedef struct {
  int used;
  int rank, size, device;
  int nodes; /* COMM form: ranks [n * size / nodes, (n + 1) * size / nodes) form node n (0: one node) */
  emac_node_sched ns; /* ... and their inter-node schedule (ext_mpi_amd_comm_set_node_ports) */
  ncclComm_t nccl;
  int loop_group; /* >= 0: in-process loopback communicator (testing transport), no RCCL */
  /* peer-mapped transport (ext_mpi_amd_comm_init_ipc) */
  int ipc;
  ext_mpi_amd_allgather_fn ag;
  void *ag_ctx;
  void *sync;                      /* this rank's emac_sync block (uncached device memory) */
  void *stale_sync[8];             /* blocks of failed set-up rounds (freed with the communicator) */
  int nstale_sync;
  void *peer_sync[EMAC_MAX_RANKS]; /* every rank's block as mapped here (own at [rank]) */
  void *peer_sync_base[EMAC_MAX_RANKS]; /* the mappings (shared table, ipc_map_peer) */
  void **d_peer_sync;              /* the same table in device memory */
  int *err;                        /* pinned host words the barrier kernels report into, one per slot */
  long timeout_ticks;
  unsigned char slot_used[EMAC_SYNC_SLOTS];
  unsigned long slot_epoch[EMAC_SYNC_SLOTS][2]; /* a slot's epochs continue across its handles */
  ipc_mirror *mirrors;
  int nmirrors;
  int cross_device; /* some peer runs on another device: release to system scope before phase 0 */
  /* the arena (library memory the peers read: outboxes, send-buffer mirrors), ipc_allreduce_init */
  arena_seg seg[EMAC_ARENA_SEGS]; /* this rank's segments */
  int nseg;
  void *peer_seg[EMAC_MAX_RANKS][EMAC_ARENA_SEGS]; /* every rank's segment k as reachable here */
  int peer_nseg[EMAC_MAX_RANKS];
  void *bad_seg[EMAC_ARENA_SEGS]; /* own segments some peer could not validate */
  int nbad;
} emac_comm;

/* Loopback groups: every rank of the communicator lives in this process; the i-th handle a
   rank creates on it matches the i-th handle of every other rank (collective call order). */
#define MAX_LOOP_GROUPS 8
#define MAX_LOOP_HANDLES 256
typedef struct {
  int used, size;
  int nh[EMAC_MAX_RANKS];
  int handle[EMAC_MAX_RANKS][MAX_LOOP_HANDLES];
} loop_group;
static loop_group loops[MAX_LOOP_GROUPS];

/* one fold launch over a set of device-resident buckets (a handle's main launch, or one part of
   a pipelined host-staged NODE handle) */
typedef struct {
  emac_bucket *d_buckets;
  int nb;
  long ntiles, tiles_per_bucket;
  int all_full;
  emac_edge *d_edges;
  int nedges;
  int unroll;
} emac_launch;

/* Launch-schedule tuning of a handle's fold (NODE form, and the COMM form's local fold): the
   first Start runs the static pick (emac_gpu_pick_unroll) and warms the buffers, the next
   EMAC_TUNE_ROUNDS x candidates Starts run the candidates round-robin, each between timing events,
   and the Start after them keeps the candidate with the shortest of its samples for the handle's
   lifetime. Every schedule folds in the same order -- the bits do not depend on the choice.
   Measured on MI355X leases (tools/schedbench.hip, tools/nodevar.hip, profiles/r03_schedbench_*,
   profiles/r03_nodevar/): the fastest schedule of a shape moves between leases by more than the
   spread within one (16 MiB x 8 node fold: U 2 48.1 us, U 4 51.8, U 4 staggered 54.1 on one
   lease; U 2 47.1, U 4 46.2 on another), so no fixed threshold table picks it everywhere; one
   sample per candidate (round 3's first tuner) kept U 2 on a lease where U 4 was 2 % faster, hence
   the rounds. A sample runs one candidate on EMAC_TUNE_SPAN Starts in a row: the first, right
   after another schedule's launch, untimed, the others timed as one window with no event between
   them, on events without the system-scope fence (hipEventDisableSystemFence): a single launch
   between two fenced events ranked the schedules against their back-to-back rate (the leaf-major
   deferred schedule 46-47 us alone, 43.9-44.4 us per Start in the bench's steady state, where the
   tile-major one it lost to ran 45.5-46.4 us; profiles/r03_tune/force_ab.txt). Where the caller
   interleaves several handles the window also holds their launches; every candidate sees the same
   pattern. EXT_MPI_AMD_AUTOTUNE=0
   keeps the static pick; EXT_MPI_AMD_FOLD_SCHEDULE=<U | issue << 4> makes one schedule the only
   candidate (A/B runs). */
#define EMAC_TUNE_MAX 6
#define EMAC_TUNE_ROUNDS 3
#define EMAC_TUNE_SPAN 3 /* Starts per sample: one untimed, then the timed window */
#define EMAC_TUNE_MIN_BYTES (16L << 20) /* algorithmic bytes per launch: smaller launches keep the static pick */
typedef struct {
  int n;      /* candidates (0: no tuning) */
  int chosen; /* index of the kept candidate, -1 while measuring */
  int starts;
  emac_launch L[EMAC_TUNE_MAX];
  void *ev[EMAC_TUNE_MAX * EMAC_TUNE_ROUNDS][2]; /* sample i: candidate i % n, round i / n */
  float us[EMAC_TUNE_MAX];                       /* shortest sample per candidate */
} emac_tune;

/* NODE form with host buffers: the message is staged in EMAC_PIPE_PARTS element ranges so that
   the H2D copies of part p+1, the fold of part p and the D2H copies of part p-1 overlap
   (three streams, events between them) */
#define EMAC_PIPE_PARTS 8
#define EMAC_PIPE_MIN_BYTES (4L << 20) /* per rank */
typedef struct {
  int nparts;
  long off[EMAC_PIPE_PARTS + 1]; /* element ranges */
  emac_launch part[EMAC_PIPE_PARTS];
  void *s_in, *s_out;
  void *ev_start, *ev_in[EMAC_PIPE_PARTS], *ev_fold[EMAC_PIPE_PARTS], *ev_done;
} emac_pipe;

typedef struct {
  int kind;
  emac_plan plan;
  int device;
  void *stream;
  emac_bucket *d_buckets;
  int nb;
  long ntiles;
  long tiles_per_bucket; /* > 0 when every bucket has the same tile count */
  int all_full;          /* every bucket is a whole number of tiles */
  int fan;               /* fan-out width == nsrc (node form) */
  emac_edge *d_edges;    /* element-granular work items (device) */
  int nedges;
  int unroll;
  int nsrc;
  size_t bytes; /* message bytes per rank */
  int nbuf;     /* ranks with buffers in this process */
  void *user_send[EMAC_MAX_RANKS], *user_recv[EMAC_MAX_RANKS];
  void *dsend[EMAC_MAX_RANKS], *drecv[EMAC_MAX_RANKS];
  unsigned char send_mirror[EMAC_MAX_RANKS], recv_mirror[EMAC_MAX_RANKS];
  unsigned char send_reg[EMAC_MAX_RANKS], recv_reg[EMAC_MAX_RANKS];
  int host_direct; /* NODE form: some buffer is page-locked host memory the fold reads / writes */
  /* COMM form */
  int comm;
  int me, me_pos;
  void *staging;
  emac_p2p *ops; /* reduce-scatter and allgather point-to-point program (plan.c) */
  int nops;
  int started;
  int loop_index; /* position in the loopback group's per-rank handle list */
  int own_stream; /* 0 once the caller supplied the stream (ext_mpi_amd_set_stream) */
  /* IPC form */
  int slot;                /* synchronisation slot on the communicator */
  int slot_held;
  unsigned long epoch[2];  /* barriers run per phase (before / after the fold) */
  void *mapped[2 * EMAC_MAX_RANKS];
  int nmapped;
  int fused; /* whole Allreduce in one launch (emac_gpu_fold_fused) */
  void *ev_release; /* system-scope release recorded before every phase-0 barrier */
  emac_launch pull; /* every owner's result copied from its outbox into this rank's receive buffer */
  void *outbox;     /* this rank's owner chunks' results (pool memory, exported to the peers) */
  size_t outbox_bytes;
  int done_collective; /* some rank exported caller memory: Done agrees with every peer */
  unsigned char send_arena; /* dsend[0] is an arena block of `bytes` (a send mirror, or in place the one buffer) */
  unsigned char send_local; /* dsend[0] is a plain device mirror (a communicator of one rank) */
  int nodes;            /* COMM form over several nodes: the node legs run (emac_comm_program_nodes) */
  emac_node_sched ns;   /* ... under this inter-node schedule */
  emac_launch xfold[2 * EMAC_MAX_NODE_STEPS]; /* ... and, per exchange step, the fold of the lines' partials */
  void *graph[EXT_MPI_AMD_LEG_ALL + 1]; /* COMM form: captured legs, per subset of EXT_MPI_AMD_LEG_* */
  unsigned char graph_failed[EXT_MPI_AMD_LEG_ALL + 1];
  emac_pipe *pipe; /* pipelined host staging (NODE form), or NULL */
  emac_tune tune;  /* launch-schedule tuning of the fold */
  /* NODE form over several nodes (ext_mpi_amd_node_comm_allreduce_init): every rank of this node
     in this process, the communicator's members being the nodes */
  int hier;
  long stage_stride;    /* staging bytes of each node rank's node legs */
  emac_launch fanout;   /* the copy-out: every owner chunk into the node's other receive buffers */
  /* ... over peer-mapped nodes (node_ipc_init): this node's partials (arena, read by the peers) */
  void *part;
  size_t part_bytes;
  emac_codes xcodes; /* ... and its share fold's tree (a left fold, or pairs for the halving flow) */
} emac_handle;

static emac_handle *handles[MAX_HANDLES];
static emac_comm comms[MAX_COMMS];

static int new_handle_slot(void) {
  int i;
  for (i = 0; i < MAX_HANDLES; i++)
    if (!handles[i]) return i;
  return -1;
}

static void ipc_unmap(void *base);
static void mirror_free(emac_handle *h, void *p);
static void arena_release(emac_comm *cm, void *p, long bytes);

static void pipe_free(emac_pipe *pp) {
  int p;
  if (!pp) return;
  if (pp->s_in) emac_gpu_stream_sync(pp->s_in);
  if (pp->s_out) emac_gpu_stream_sync(pp->s_out);
  for (p = 0; p < pp->nparts; p++) {
    emac_gpu_free(pp->part[p].d_buckets);
    emac_gpu_free(pp->part[p].d_edges);
    emac_gpu_event_destroy(pp->ev_in[p]);
    emac_gpu_event_destroy(pp->ev_fold[p]);
  }
  emac_gpu_event_destroy(pp->ev_start);
  emac_gpu_event_destroy(pp->ev_done);
  if (pp->s_in) emac_gpu_stream_destroy(pp->s_in);
  if (pp->s_out) emac_gpu_stream_destroy(pp->s_out);
  free(pp);
}

static void release(emac_handle *h) {
  int r;
  if (!h) return;
  if (h->stream) {
    emac_gpu_stream_sync(h->stream);
    if (h->own_stream) emac_gpu_stream_destroy(h->stream);
  }
  pipe_free(h->pipe);
  emac_gpu_free(h->d_buckets);
  emac_gpu_free(h->d_edges);
  emac_gpu_free(h->pull.d_buckets);
  emac_gpu_free(h->pull.d_edges);
  for (r = 0; r < h->tune.n; r++) {
    if (h->tune.L[r].d_buckets != h->d_buckets) emac_gpu_free(h->tune.L[r].d_buckets);
    if (h->tune.L[r].d_edges != h->d_edges) emac_gpu_free(h->tune.L[r].d_edges);
  }
  for (r = 0; r < EMAC_TUNE_MAX * EMAC_TUNE_ROUNDS; r++) {
    emac_gpu_event_destroy(h->tune.ev[r][0]);
    emac_gpu_event_destroy(h->tune.ev[r][1]);
  }
  for (r = 0; r < 2 * EMAC_MAX_NODE_STEPS; r++) {
    emac_gpu_free(h->xfold[r].d_buckets);
    emac_gpu_free(h->xfold[r].d_edges);
  }
  emac_gpu_free(h->fanout.d_buckets);
  emac_gpu_free(h->fanout.d_edges);
  emac_gpu_free(h->staging);
  for (r = 0; r < h->nbuf; r++) {
    const int same = h->dsend[r] == h->drecv[r];
    const int own = r == 0 && (h->send_arena || h->send_local); /* send side allocated by the IPC set-up */
    if (r == 0 && h->send_arena)
      arena_release(&comms[h->comm], h->dsend[0], (long)h->bytes);
    else if (r == 0 && h->send_local)
      emac_gpu_free(h->dsend[0]);
    else if (h->send_mirror[r])
      mirror_free(h, h->dsend[r]);
    if (h->recv_mirror[r] && h->drecv[r] && !(same && (h->send_mirror[r] || own))) mirror_free(h, h->drecv[r]);
    if (h->send_reg[r]) emac_gpu_host_unregister(h->user_send[r]);
    if (h->recv_reg[r]) emac_gpu_host_unregister(h->user_recv[r]);
  }
  for (r = 0; r < h->nmapped; r++) ipc_unmap(h->mapped[r]);
  if (h->outbox) arena_release(&comms[h->comm], h->outbox, (long)h->outbox_bytes);
  if (h->part) arena_release(&comms[h->comm], h->part, (long)h->part_bytes);
  emac_gpu_event_destroy(h->ev_release);
  for (r = 0; r <= EXT_MPI_AMD_LEG_ALL; r++) emac_gpu_graph_destroy(h->graph[r]);
  if (h->kind == KIND_IPC && h->slot_held) {
    emac_comm *cm = &comms[h->comm];
    cm->slot_used[h->slot] = 0;
    cm->slot_epoch[h->slot][0] = h->epoch[0];
    cm->slot_epoch[h->slot][1] = h->epoch[1];
  }
  free(h->ops);
  emac_plan_free(&h->plan);
  free(h);
}

/* device mirrors the peers never touch (every receive-side mirror; IPC send mirrors come from
   the communicator's arena, ipc_allreduce_init) */
static int mirror_alloc(emac_handle *h, void **p) { return emac_gpu_malloc(p, h->bytes); }

static void mirror_free(emac_handle *h, void *p) { emac_gpu_free(p); }

/* A buffer the handle can use in place: device memory, and in the IPC form, for a buffer the
   peers read (the send buffer; in place, the one buffer), also exportable
   (emac_gpu_ipc_exportable). The receive buffer of the IPC form is never exported: peers never
   touch it. Anything else gets a device mirror. */
static int in_place_ok(const emac_handle *h, const void *p, int peers_read) {
  if (!emac_gpu_is_device_pointer(p)) return 0;
  return h->kind != KIND_IPC || !peers_read || comms[h->comm].size == 1 || emac_gpu_ipc_exportable(p);
}

/* Page-locking a caller's host buffer is opt-in (EXT_MPI_AMD_HOST_REGISTER=1; never in the IPC
   form). Registered user pages, unregistered at handle release and then freed and reused by the
   application, were twice followed by an asynchronous illegal-address error in a later, unrelated
   launch or copy of the same process (8 IPC processes on one MI355X; the single-process GPU suite
   after the host-buffer tests), and both went away without registration. Unregistered buffers
   are staged by the runtime; buffers the caller already pinned (hipHostMalloc, torch
   pin_memory) are copied at full rate either way. */
static int host_register(const emac_handle *h, const void *p) {
  const char *e = getenv("EXT_MPI_AMD_HOST_REGISTER");
  if (!e || atoi(e) <= 0 || h->kind == KIND_IPC || emac_gpu_is_device_pointer(p)) return 0;
  return emac_gpu_host_register((void *)p, h->bytes) == 0;
}

/* NODE form: host memory the caller already page-locked (hipHostMalloc, torch pin_memory) is
   read and written by the fold kernel itself over PCIe (EXT_MPI_AMD_HOST_DIRECT=0 turns this
   off). One launch replaces R host-to-device copies, the fold and R device-to-host copies, and
   the leaf reads overlap the fan-out writes on the link's two directions. */
static int host_direct(const emac_handle *h, const void *p, void **dev) {
  const char *e = getenv("EXT_MPI_AMD_HOST_DIRECT");
  if (h->kind != KIND_NODE || (e && atoi(e) <= 0)) return 0;
  return emac_gpu_pinned_view(p, dev) == 0;
}

/* Device view of rank r's buffers: usable user device pointers are used in place, page-locked
   host memory in the NODE form through its device address; other buffers get a device mirror
   (in place stays in place), staged in and out on the handle's stream. */
static int map_buffers(emac_handle *h, int r, const void *send, void *recv) {
  int rc;
  void *dv;
  h->user_send[r] = (void *)send;
  h->user_recv[r] = recv;
  if (in_place_ok(h, recv, send == recv)) {
    h->drecv[r] = recv;
  } else if (host_direct(h, recv, &dv)) {
    h->drecv[r] = dv;
    h->host_direct = 1;
  } else {
    /* IPC form, in place: the one buffer is read by the peers -- its mirror comes from the arena
       (ipc_allreduce_init; NULL until then) */
    if (!(h->kind == KIND_IPC && send == recv) && (rc = mirror_alloc(h, &h->drecv[r]))) return rc;
    h->recv_mirror[r] = 1;
    h->recv_reg[r] = host_register(h, recv);
  }
  if (send == recv) {
    h->dsend[r] = h->drecv[r];
  } else if (in_place_ok(h, send, 1)) {
    h->dsend[r] = (void *)send;
  } else if (host_direct(h, send, &dv)) {
    h->dsend[r] = dv;
    h->host_direct = 1;
  } else {
    /* IPC form: from the arena (ipc_allreduce_init; NULL until then) */
    if (h->kind != KIND_IPC && (rc = mirror_alloc(h, &h->dsend[r]))) return rc;
    h->send_mirror[r] = 1;
    h->send_reg[r] = host_register(h, send);
  }
  return 0;
}

/* pointers of a bucket are first set at the start of the whole buffers, then moved to the
   chunk's first element */
static void place_bucket(emac_bucket *b, int nsrc, long off, long len, int tsize) {
  int i;
  for (i = 0; i < nsrc; i++) b->src[i] = (const char *)b->src[i] + off * tsize;
  for (i = 0; i < b->ndst; i++) b->dst[i] = (char *)b->dst[i] + off * tsize;
  emac_split_alignment(b, nsrc, len, tsize);
}

static int upload_launch_as(const emac_handle *h, emac_launch *L, emac_bucket *b, int nb, int nsrc, int tree) {
  emac_edge *edges = NULL;
  int rc;
  if ((rc = emac_layout(b, nb, h->plan.op, nsrc, tree, h->fan, &edges, &L->nedges, &L->ntiles, &L->tiles_per_bucket,
                        &L->all_full, &L->unroll)))
    return rc;
  L->nb = nb;
  if (nb && (rc = emac_gpu_malloc((void **)&L->d_buckets, sizeof(emac_bucket) * (size_t)nb)) == 0)
    rc = emac_gpu_memcpy(L->d_buckets, b, sizeof(emac_bucket) * (size_t)nb);
  if (!rc && L->nedges && (rc = emac_gpu_malloc((void **)&L->d_edges, sizeof(emac_edge) * (size_t)L->nedges)) == 0)
    rc = emac_gpu_memcpy(L->d_edges, edges, sizeof(emac_edge) * (size_t)L->nedges);
  free(edges);
  return rc;
}

static int upload_launch(const emac_handle *h, emac_launch *L, emac_bucket *b, int nb) {
  return upload_launch_as(h, L, b, nb, h->nsrc, emac_tree_kind(&h->plan.codes, h->plan.op) == 1);
}

/* the candidates of emac_tune for a fold of nsrc leaves, fan-out `fan` (0 / 1), vec 16-byte vectors
   per leaf over all buckets, or 0 */
static int tune_candidates(const emac_handle *h, long vec, int *sched) {
  const char *e = getenv("EXT_MPI_AMD_AUTOTUNE");
  const char *g = getenv("EXT_MPI_AMD_GRAPH"); /* captured Starts replay one schedule */
  int n = 0;
  if ((e && atoi(e) <= 0) || (h->kind == KIND_COMM && g && atoi(g) > 0) || h->plan.op != EMAC_SUM || h->nsrc < 2 ||
      h->nsrc > 8 || h->host_direct ||
      emac_tree_kind(&h->plan.codes, h->plan.op) == 1 || (h->fan != 0 && h->fan != 1))
    return 0;
  /* fold_kernel.hpp instantiation policy: (U 2, burst), (U 4, burst), for the node fan-out (U 4,
     s_sleep 2 every 4 loads); deferred stores (kDeferShift) when every bucket has the same tile
     count: (U 2, 4 tiles) and (U 4, 4 tiles) for one destination, (U 2, 4 tiles) and, for the
     fan-out, its leaf-major form (kLeafMajor) over the linear fold or (U 4, 2 tiles) over fold
     trees. A launch of fewer than 256 groups of (U 2, 4 tiles) -- under 8 MiB per leaf -- leaves
     CUs idle under the deferred schedules; there (U 1, burst), twice the per-tile loop's
     workgroups, is offered too. (U 2, 8 tiles), compiled, is no longer offered: never kept. */
  const int small = vec < 256L * 4 * 2 * EMAC_BLOCK;
  const char *f = getenv("EXT_MPI_AMD_FOLD_SCHEDULE"); /* A/B runs: one schedule word, U | issue << 4 */
  if (f && atoi(f) > 0) {
    sched[0] = atoi(f);
    return 1;
  }
  sched[n++] = 2 | 1 << 4;
  sched[n++] = 4 | 1 << 4;
  if (h->fan) sched[n++] = 4 | 5 << 4;
  if (small) sched[n++] = 1 | 1 << 4;
  if (h->tiles_per_bucket > 0) {
    sched[n++] = 2 | (1 | 2 << 11) << 4;
    if (!h->fan)
      sched[n++] = 4 | (1 | 2 << 11) << 4;
    else if (emac_tree_kind(&h->plan.codes, h->plan.op) == 0)
      sched[n++] = 2 | (1 | 2 << 11 | 1 << 13) << 4; /* leaf-major groups: the linear fold's order only */
    else
      sched[n++] = 4 | (1 | 1 << 11) << 4;
  }
  return n;
}

static int upload_buckets(emac_handle *h, emac_bucket *b, int nb) {
  emac_edge *edges = NULL;
  int rc, sched[EMAC_TUNE_MAX], nc, k, i;
  long vec = 0;
  /* (fan | EMAC_FAN_HOST: the schedule for buffers across PCIe, emac_gpu_pick_unroll) */
  if ((rc = emac_layout(b, nb, h->plan.op, h->nsrc, emac_tree_kind(&h->plan.codes, h->plan.op) == 1,
                        h->fan | (h->host_direct ? EMAC_FAN_HOST : 0),
                        &edges, &h->nedges, &h->ntiles, &h->tiles_per_bucket, &h->all_full, &h->unroll)))
    return rc;
  h->nb = nb;
  if (nb && (rc = emac_gpu_malloc((void **)&h->d_buckets, sizeof(emac_bucket) * (size_t)nb)) == 0)
    rc = emac_gpu_memcpy(h->d_buckets, b, sizeof(emac_bucket) * (size_t)nb);
  if (!rc && h->nedges && (rc = emac_gpu_malloc((void **)&h->d_edges, sizeof(emac_edge) * (size_t)h->nedges)) == 0)
    rc = emac_gpu_memcpy(h->d_edges, edges, sizeof(emac_edge) * (size_t)h->nedges);
  free(edges);
  for (i = 0; i < nb; i++) vec += b[i].nvec;
  nc = rc ? 0 : tune_candidates(h, vec, sched);
  if (!nc || vec * 16 * (h->nsrc + (h->fan ? h->nsrc : 1)) < EMAC_TUNE_MIN_BYTES) return rc;
  {
    emac_bucket *tb = (emac_bucket *)malloc(sizeof(emac_bucket) * (size_t)nb);
    if (!tb) return EMAC_ERR_MALLOC;
    h->tune.chosen = -1;
    for (k = 0; k < nc && !rc; k++) {
      emac_launch *L = &h->tune.L[k];
      memcpy(tb, b, sizeof(emac_bucket) * (size_t)nb);
      h->tune.n = k + 1; /* freed by release() from here on */
      if (sched[k] == h->unroll) { /* the static pick: its upload is reused */
        L->d_buckets = h->d_buckets;
        L->nb = nb;
        L->ntiles = h->ntiles;
        L->tiles_per_bucket = h->tiles_per_bucket;
        L->all_full = h->all_full;
        L->d_edges = h->d_edges;
        L->nedges = h->nedges;
        L->unroll = h->unroll;
      } else {
        rc = emac_layout_as(tb, nb, h->plan.op, h->nsrc, 0, h->fan, sched[k], &edges, &L->nedges, &L->ntiles,
                            &L->tiles_per_bucket, &L->all_full, &L->unroll);
        if (!rc) {
          L->nb = nb;
          if ((rc = emac_gpu_malloc((void **)&L->d_buckets, sizeof(emac_bucket) * (size_t)nb)) == 0)
            rc = emac_gpu_memcpy(L->d_buckets, tb, sizeof(emac_bucket) * (size_t)nb);
          if (!rc && L->nedges && (rc = emac_gpu_malloc((void **)&L->d_edges, sizeof(emac_edge) * (size_t)L->nedges)) == 0)
            rc = emac_gpu_memcpy(L->d_edges, edges, sizeof(emac_edge) * (size_t)L->nedges);
          free(edges);
        }
      }
    }
    for (i = 0; i < nc * EMAC_TUNE_ROUNDS && !rc; i++) {
      rc = emac_gpu_event_create_timed(&h->tune.ev[i][0]);
      if (!rc) rc = emac_gpu_event_create_timed(&h->tune.ev[i][1]);
    }
    free(tb);
  }
  return rc;
}

/* The handle's fold launch (fan 0 / 1), with the schedule tuning of emac_tune. */
static int fold_launch(emac_handle *h) {
  emac_tune *t = &h->tune;
  int rc, k;
  if (t->n && t->chosen < 0) {
    const int s = t->starts++, nsamples = t->n * EMAC_TUNE_ROUNDS;
    if (s >= 1 && s <= EMAC_TUNE_SPAN * nsamples) {
      /* sample p: candidate p % n on EMAC_TUNE_SPAN Starts in a row, the first untimed (it follows
         another schedule's launch), the others timed as one window */
      const int p = (s - 1) / EMAC_TUNE_SPAN, pos = (s - 1) % EMAC_TUNE_SPAN;
      const emac_launch *L = &t->L[p % t->n];
      if (pos == 1 && (rc = emac_gpu_event_record(t->ev[p][0], h->stream))) return rc;
      if ((rc = emac_gpu_fold(h->plan.dtype, h->plan.op, h->nsrc, h->fan, L->unroll, &h->plan.codes, L->d_buckets, L->nb,
                              L->ntiles, L->tiles_per_bucket, L->all_full, L->d_edges, L->nedges, h->stream)))
        return rc;
      return pos == EMAC_TUNE_SPAN - 1 ? emac_gpu_event_record(t->ev[p][1], h->stream) : 0;
    }
    if (s == EMAC_TUNE_SPAN * nsamples + 1) { /* keep the fastest: it becomes the handle's launch */
      int best = 0, i;
      for (k = 0; k < t->n; k++) t->us[k] = 1e30f;
      for (i = 0; i < nsamples; i++) {
        float us;
        if ((rc = emac_gpu_event_elapsed_us(t->ev[i][0], t->ev[i][1], &us))) return rc;
        us /= EMAC_TUNE_SPAN - 1;
        if (us < t->us[i % t->n]) t->us[i % t->n] = us;
      }
      for (k = 1; k < t->n; k++)
        if (t->us[k] < t->us[best]) best = k;
      void *old_b = h->d_buckets, *old_e = h->d_edges; /* the static pick's upload */
      if (t->L[best].d_buckets != h->d_buckets) {
        h->d_buckets = t->L[best].d_buckets;
        h->d_edges = t->L[best].d_edges;
        h->nb = t->L[best].nb;
        h->ntiles = t->L[best].ntiles;
        h->tiles_per_bucket = t->L[best].tiles_per_bucket;
        h->all_full = t->L[best].all_full;
        h->nedges = t->L[best].nedges;
        h->unroll = t->L[best].unroll;
      }
      for (k = 0; k < t->n; k++) /* every upload but the kept one; the static pick's may be a candidate's */
        if (k != best && t->L[k].d_buckets != old_b) {
          emac_gpu_free(t->L[k].d_buckets);
          emac_gpu_free(t->L[k].d_edges);
        }
      if (old_b != h->d_buckets) {
        emac_gpu_free(old_b);
        emac_gpu_free(old_e);
      }
      for (k = 0; k < t->n; k++) { /* release() frees the kept launch once, as the handle's */
        t->L[k].d_buckets = h->d_buckets;
        t->L[k].d_edges = h->d_edges;
      }
      t->chosen = best;
      if (getenv("EXT_MPI_AMD_DEBUG_TUNE")) {
        char line[256];
        int at = 0;
        for (k = 0; k < t->n && at < (int)sizeof(line) - 32; k++)
          at += snprintf(line + at, sizeof(line) - (size_t)at, " U%d/%d %.1f", t->L[k].unroll & 15, t->L[k].unroll >> 4,
                         t->us[k]);
        fprintf(stderr, "ext_mpi_amd: fold schedule kept: U %d issue %d (%.1f us; %d candidates:%s)\n", h->unroll & 15,
                h->unroll >> 4, t->us[best], t->n, line);
      }
    }
  }
  return emac_gpu_fold(h->plan.dtype, h->plan.op, h->nsrc, h->fan, h->unroll, &h->plan.codes, h->d_buckets, h->nb, h->ntiles,
                       h->tiles_per_bucket, h->all_full, h->d_edges, h->nedges, h->stream);
}

int ext_mpi_amd_handle_schedule(int handle, int *unroll, int *issue, int *tuned) {
  const emac_handle *h = (handle >= 0 && handle < MAX_HANDLES) ? handles[handle] : NULL;
  if (!h) return EMAC_ERR_ARG;
  if (unroll) *unroll = h->unroll & 15;
  if (issue) *issue = h->unroll >> 4;
  if (tuned) *tuned = h->tune.n ? (h->tune.chosen >= 0 ? 1 : 0) : -1;
  return 0;
}

int ext_mpi_amd_handle_candidates(int handle, int *n, int *sched, int max) {
  const emac_handle *h = (handle >= 0 && handle < MAX_HANDLES) ? handles[handle] : NULL;
  int k;
  if (!h || !n || (max > 0 && !sched)) return EMAC_ERR_ARG;
  *n = h->tune.n;
  for (k = 0; k < h->tune.n && k < max; k++) sched[k] = h->tune.L[k].unroll;
  return 0;
}

/* EXT_MPI_NUM_SOCKETS_PER_NODE as the reference keeps it: one process-wide parameter read at
   init (ext_mpi.c:43-187), applied to every plan built afterwards */
static int g_num_sockets = 1;

int ext_mpi_amd_set_num_sockets(int sockets) {
  const int prev = g_num_sockets;
  if (sockets < 1 || sockets > EMAC_MAX_RANKS) return EMAC_ERR_ARG;
  g_num_sockets = sockets;
  return prev;
}

static int parse_cfg(const char *copyin, int nranks, emac_copyin *cfg) {
  int rc = 0;
  /* one rank: the generator returns before reading the factors (reduce_copyin.c:975) */
  if (!copyin || !*copyin || nranks == 1)
    emac_default_copyin(nranks, cfg);
  else
    rc = emac_parse_copyin(copyin, cfg);
  cfg->sockets = g_num_sockets;
  return rc;
}

static int finish_init(emac_handle *h, int *handle) {
  int slot = new_handle_slot();
  h->own_stream = 1;
  if (slot < 0) return EMAC_ERR_MALLOC;
  handles[slot] = h;
  *handle = slot;
  return 0;
}

/* The NODE form's buckets restricted to message elements [lo, hi): every owner chunk (piece pc,
   position c) clipped to the range; leaves in the plan's fold order, fan-out into every rank's
   receive buffer. Returns the number written to b (capacity npieces * nranks). */
static int node_buckets(const emac_handle *h, long lo, long hi, emac_bucket *b) {
  const int R = h->plan.nranks;
  int pc, c, t, r, nb = 0;
  for (pc = 0; pc < h->plan.npieces; pc++) {
    for (c = 0; c < R; c++) {
      const long off = h->plan.chunk_off[(size_t)pc * R + c], len = h->plan.chunk_len[(size_t)pc * R + c];
      const long a = off > lo ? off : lo, e = off + len < hi ? off + len : hi;
      emac_bucket *bk = &b[nb];
      if (len <= 0 || a >= e) continue;
      memset(bk, 0, sizeof(*bk));
      for (t = 0; t < R; t++) bk->src[t] = h->dsend[h->plan.leaf_rank[c][t]];
      for (r = 0; r < R; r++) bk->dst[r] = h->drecv[r];
      bk->ndst = R;
      place_bucket(bk, R, a, e - a, h->plan.tsize);
      nb++;
    }
  }
  return nb;
}

/* Pipelined staging of a NODE handle whose buffers are mirrored host memory: the message in
   EMAC_PIPE_PARTS element ranges, each its own fold launch between its copies (ext_mpi_amd_start). */
static int node_pipe_init(emac_handle *h) {
  emac_pipe *pp;
  emac_bucket *pb;
  const long count = (long)(h->bytes / (size_t)h->plan.tsize);
  long step;
  int r, p, any = 0, rc = 0;
  for (r = 0; r < h->nbuf; r++) any |= h->send_mirror[r] | h->recv_mirror[r];
  /* opt-in (EXT_MPI_AMD_PIPELINE=1): +12-25 % in a process with few streams, but down to -8 % in
     one that has made many (hardware-queue sharing) */
  if (!any || (long)h->bytes < EMAC_PIPE_MIN_BYTES || !getenv("EXT_MPI_AMD_PIPELINE") ||
      atoi(getenv("EXT_MPI_AMD_PIPELINE")) <= 0)
    return 0;
  pp = (emac_pipe *)calloc(1, sizeof(emac_pipe));
  pb = (emac_bucket *)calloc((size_t)h->plan.npieces * (size_t)h->plan.nranks, sizeof(emac_bucket));
  if (!pp || !pb) {
    free(pp);
    free(pb);
    return EMAC_ERR_MALLOC;
  }
  h->pipe = pp;
  {
    const char *np = getenv("EXT_MPI_AMD_PIPE_PARTS");
    pp->nparts = np ? atoi(np) : EMAC_PIPE_PARTS;
    if (pp->nparts < 1 || pp->nparts > EMAC_PIPE_PARTS) pp->nparts = EMAC_PIPE_PARTS;
  }
  step = ((count + pp->nparts - 1) / pp->nparts + 4095) / 4096 * 4096; /* 16-byte aligned ranges, any type */
  for (p = 0; p < pp->nparts; p++) pp->off[p] = (long)p * step < count ? (long)p * step : count;
  pp->off[pp->nparts] = count;
  for (p = 0; p < pp->nparts && !rc; p++) {
    const int n = node_buckets(h, pp->off[p], pp->off[p + 1], pb);
    rc = upload_launch(h, &pp->part[p], pb, n);
    if (!rc) rc = emac_gpu_event_create(&pp->ev_in[p]);
    if (!rc) rc = emac_gpu_event_create(&pp->ev_fold[p]);
  }
  free(pb);
  if (!rc) rc = emac_gpu_event_create(&pp->ev_start);
  if (!rc) rc = emac_gpu_event_create(&pp->ev_done);
  /* The copy streams get an explicit (least) priority: streams of the default priority share the
     process's few hardware queues round-robin, and a copy stream that landed on the fold
     stream's queue serialised the pipeline (8 x 16 MiB pinned: 20-22 GB/s reduced against 25-26
     unpipelined, depending on how many streams the process had made before); on a priority's own
     queues it ran at 29-31 GB/s whatever came before (profiles/r01_host_pipeline_priority.json). */
  if (!rc) rc = emac_gpu_stream_create_priority(&pp->s_in, 0);
  if (!rc) rc = emac_gpu_stream_create_priority(&pp->s_out, 0);
  return rc;
}

int ext_mpi_amd_node_allreduce_init(int nranks, const void *const *sendbufs, void *const *recvbufs, long count,
                                    int dtype, int op, const char *copyin, int *handle) {
  emac_handle *h;
  emac_copyin cfg;
  emac_bucket *b = NULL;
  int rc, r, nb = 0;
  if (!handle || !sendbufs || !recvbufs || nranks < 1 || nranks > EMAC_MAX_RANKS || count < 0)
    return EMAC_ERR_ARG;
  *handle = -1;
  if ((rc = parse_cfg(copyin, nranks, &cfg))) return rc;
  if (emac_gpu_device_count() <= 0) return EMAC_ERR_DEVICE;
  h = (emac_handle *)calloc(1, sizeof(emac_handle));
  if (!h) return EMAC_ERR_MALLOC;
  h->kind = KIND_NODE;
  if ((rc = emac_plan_build(&h->plan, nranks, count, dtype, op, &cfg))) goto fail;
  emac_gpu_get_device(&h->device);
  h->bytes = (size_t)count * (size_t)h->plan.tsize;
  h->nbuf = nranks;
  h->nsrc = nranks;
  h->fan = nranks > 1;
  for (r = 0; r < nranks; r++)
    if ((rc = map_buffers(h, r, sendbufs[r], recvbufs[r]))) goto fail;
  b = (emac_bucket *)calloc((size_t)h->plan.npieces * nranks, sizeof(emac_bucket));
  if (!b) {
    rc = EMAC_ERR_MALLOC;
    goto fail;
  }
  nb = node_buckets(h, 0, count, b);
  if ((rc = upload_buckets(h, b, nb))) goto fail;
  if ((rc = node_pipe_init(h))) goto fail;
  free(b);
  b = NULL;
  if ((rc = emac_gpu_stream_create(&h->stream))) goto fail;
  if ((rc = finish_init(h, handle))) goto fail;
  return 0;
fail:
  free(b);
  release(h);
  return rc;
}

/* One owner chunk as a persistent handle: the persistent form of the device C-ABI's
   ext_mpi_amd_gpu_copy_reduce (the reference launches one such descriptor per GPU stream,
   byte_code.c:936-992). Leaves are folded in the given order, left to right. */
int ext_mpi_amd_fold_init(int nsrc, const void *const *srcs, int ndst, void *const *dsts, long count, int dtype,
                          int op, int *handle) {
  emac_handle *h;
  emac_bucket b;
  emac_copyin cfg;
  int rc, i;
  if (!handle || !srcs || nsrc < 1 || nsrc > EMAC_MAX_RANKS || ndst < 1 || count < 0) return EMAC_ERR_ARG;
  if (ndst > 1 && ndst != nsrc) return EMAC_ERR_UNSUPPORTED; /* fan-out width is 1 or nsrc */
  *handle = -1;
  if (emac_gpu_device_count() <= 0) return EMAC_ERR_DEVICE;
  for (i = 0; i < nsrc; i++)
    if (!emac_gpu_is_device_pointer(srcs[i])) return EMAC_ERR_ARG;
  for (i = 0; i < ndst; i++)
    if (!emac_gpu_is_device_pointer(dsts[i])) return EMAC_ERR_ARG;
  h = (emac_handle *)calloc(1, sizeof(emac_handle));
  if (!h) return EMAC_ERR_MALLOC;
  h->kind = KIND_NODE;
  /* a linear plan over nsrc leaves supplies the codes (one level, leaves in given order) */
  emac_default_copyin(nsrc, &cfg);
  if ((rc = emac_plan_build(&h->plan, nsrc, count, dtype, op, nsrc > 1 ? &cfg : NULL))) goto fail;
  emac_gpu_get_device(&h->device);
  h->nsrc = nsrc;
  h->fan = ndst > 1;
  memset(&b, 0, sizeof(b));
  for (i = 0; i < nsrc; i++) b.src[i] = srcs[i];
  for (i = 0; i < ndst; i++) b.dst[i] = dsts[i];
  b.ndst = ndst;
  place_bucket(&b, nsrc, 0, count, h->plan.tsize);
  if ((rc = upload_buckets(h, &b, count > 0 ? 1 : 0))) goto fail;
  if ((rc = emac_gpu_stream_create(&h->stream))) goto fail;
  if ((rc = finish_init(h, handle))) goto fail;
  return 0;
fail:
  release(h);
  return rc;
}

/* ------------------------------ COMM form (RCCL) ------------------------------ */

int ext_mpi_amd_get_unique_id(void *id) {
  ncclUniqueId u;
  if (!id) return EMAC_ERR_ARG;
  if (ncclGetUniqueId(&u) != ncclSuccess) return EMAC_ERR_TRANSPORT;
  memcpy(id, &u, sizeof(u));
  return 0;
}

int ext_mpi_amd_comm_init(int rank, int size, const void *id, int device, int *comm) {
  ncclUniqueId u;
  int i;
  if (!id || !comm || size < 1 || size > EMAC_MAX_RANKS || rank < 0 || rank >= size) return EMAC_ERR_ARG;
  if (emac_gpu_device_count() <= 0) return EMAC_ERR_DEVICE;
  for (i = 0; i < MAX_COMMS && comms[i].used; i++);
  if (i == MAX_COMMS) return EMAC_ERR_MALLOC;
  if (device >= 0 && emac_gpu_set_device(device)) return EMAC_ERR_DEVICE;
  emac_gpu_get_device(&comms[i].device);
  memcpy(&u, id, sizeof(u));
  if (ncclCommInitRank(&comms[i].nccl, size, u, rank) != ncclSuccess) return EMAC_ERR_TRANSPORT;
  comms[i].used = 1;
  comms[i].rank = rank;
  comms[i].size = size;
  comms[i].loop_group = -1;
  *comm = i;
  return 0;
}

/* Testing transport: `size` communicators, one per rank, all in this process on the current
   device. Their point-to-point ops are matched in order (as RCCL matches ops between a pair
   inside a group) and executed as device copies when the RECEIVING rank runs the leg, so the
   caller must run each leg on every rank before the next one (ext_mpi_amd_start_legs). */
int ext_mpi_amd_comm_init_loopback(int size, int *comm_of_rank) {
  int g, r, i;
  if (!comm_of_rank || size < 1 || size > EMAC_MAX_RANKS) return EMAC_ERR_ARG;
  if (emac_gpu_device_count() <= 0) return EMAC_ERR_DEVICE;
  for (g = 0; g < MAX_LOOP_GROUPS && loops[g].used; g++);
  if (g == MAX_LOOP_GROUPS) return EMAC_ERR_MALLOC;
  memset(&loops[g], 0, sizeof(loops[g]));
  loops[g].used = 1;
  loops[g].size = size;
  for (r = 0; r < size; r++) {
    for (i = 0; i < MAX_COMMS && comms[i].used; i++);
    if (i == MAX_COMMS) return EMAC_ERR_MALLOC;
    memset(&comms[i], 0, sizeof(comms[i]));
    comms[i].used = 1;
    comms[i].rank = r;
    comms[i].size = size;
    comms[i].loop_group = g;
    emac_gpu_get_device(&comms[i].device);
    comm_of_rank[r] = i;
  }
  return 0;
}

/* ------------------------- peer-mapped form (IPC over xGMI), the reference's GPU path -------
 * cuda_shmem.c:218-299 maps every node peer's device send/recv buffer with cudaIpc and
 * cuda_core.cu:50-86 then loads the partners' chunks directly; ext_mpi_native_exec.c:21-84
 * synchronises the ranks with flags in shared memory. Here: hipIpc (dmabuf) mappings, exchanged
 * through the caller's allgather (the MPI layer passes PMPI_Allgather, as the reference does),
 * and stream-ordered barrier kernels over a per-communicator block of uncached device flags
 * (ipc.hip). Start = system-scope release -> barrier -> fold of this rank's owner chunks over the
 * peers' send buffers into its own receive buffer -> barrier -> pull of every other owner's
 * result from that owner's receive buffer (one launch for small messages). */

static int ipc_agree(emac_comm *cm, int ok_local) {
  int all[EMAC_MAX_RANKS], r;
  if (cm->ag(cm->ag_ctx, &ok_local, all, (long)sizeof(int))) return EMAC_ERR_TRANSPORT;
  for (r = 0; r < cm->size; r++)
    if (!all[r]) return EMAC_ERR_TRANSPORT;
  return 0;
}

static ipc_map *g_maps;
static int g_nmaps;

static void *ipc_map_peer(const unsigned char *handle, unsigned long long buf_id, long extent) {
  int i;
  void *base;
  for (i = 0; i < g_nmaps; i++) {
    ipc_map *m = &g_maps[i];
    if (m->base && m->extent == extent && m->buf_id == buf_id && !memcmp(m->handle, handle, EMAC_IPC_HANDLE_BYTES)) {
      m->refs++;
      return m->base;
    }
  }
  if (emac_gpu_ipc_open(handle, &base)) return NULL;
  for (i = 0; i < g_nmaps && g_maps[i].base; i++);
  if (i == g_nmaps) {
    ipc_map *m = (ipc_map *)realloc(g_maps, sizeof(ipc_map) * (size_t)(g_nmaps + 1));
    if (!m) {
      emac_gpu_ipc_close(base);
      return NULL;
    }
    g_maps = m;
    g_nmaps++;
  }
  g_maps[i].buf_id = buf_id;
  g_maps[i].extent = extent;
  memcpy(g_maps[i].handle, handle, EMAC_IPC_HANDLE_BYTES);
  g_maps[i].base = base;
  g_maps[i].refs = 1;
  return base;
}

static void ipc_unmap(void *base) {
  int i;
  for (i = 0; i < g_nmaps; i++)
    if (g_maps[i].refs > 0 && g_maps[i].base == base) {
      if (--g_maps[i].refs == 0) {
        emac_gpu_ipc_close(base);
        g_maps[i].base = NULL;
      }
      return;
    }
}

static int ipc_mirror_get(emac_comm *cm, void **p, size_t bytes) {
  int i, best = -1, rc;
  for (i = 0; i < cm->nmirrors; i++)
    if (!cm->mirrors[i].busy && cm->mirrors[i].bytes >= bytes &&
        (best < 0 || cm->mirrors[i].bytes < cm->mirrors[best].bytes))
      best = i;
  if (best < 0) {
    ipc_mirror *m = (ipc_mirror *)realloc(cm->mirrors, sizeof(ipc_mirror) * (size_t)(cm->nmirrors + 1));
    if (!m) return EMAC_ERR_MALLOC;
    cm->mirrors = m;
    best = cm->nmirrors;
    bytes = (bytes + EMAC_IPC_GRANULE - 1) / EMAC_IPC_GRANULE * EMAC_IPC_GRANULE; /* never sub-allocated */
    if ((rc = emac_gpu_malloc(&m[best].p, bytes))) return rc;
    m[best].bytes = bytes;
    cm->nmirrors++;
  }
  cm->mirrors[best].busy = 1;
  *p = cm->mirrors[best].p;
  return 0;
}

static void ipc_mirror_put(emac_comm *cm, void *p) {
  int i;
  for (i = 0; i < cm->nmirrors; i++)
    if (cm->mirrors[i].p == p && cm->mirrors[i].busy == 1) cm->mirrors[i].busy = 0; /* poisoned ones stay out */
}

static int ipc_pool_owns(const emac_comm *cm, const void *p) {
  int i;
  for (i = 0; i < cm->nmirrors; i++)
    if ((const char *)p >= (const char *)cm->mirrors[i].p && (const char *)p < (const char *)cm->mirrors[i].p + cm->mirrors[i].bytes)
      return 1;
  return 0;
}

int ext_mpi_amd_comm_malloc(int comm, void **p, unsigned long bytes) {
  if (!p || comm < 0 || comm >= MAX_COMMS || !comms[comm].used) return EMAC_ERR_ARG;
  *p = NULL;
  if (!bytes) return 0;
  if (emac_gpu_set_device(comms[comm].device)) return EMAC_ERR_DEVICE;
  return comms[comm].ipc ? ipc_mirror_get(&comms[comm], p, bytes) : emac_gpu_malloc(p, bytes);
}

int ext_mpi_amd_comm_mfree(int comm, void *p) {
  if (comm < 0 || comm >= MAX_COMMS || !comms[comm].used) return EMAC_ERR_ARG;
  if (!p) return 0;
  if (comms[comm].ipc) {
    ipc_mirror_put(&comms[comm], p);
    return 0;
  }
  return emac_gpu_free(p);
}

static int ipc_agree(emac_comm *cm, int ok_local);
static char *leg_base(const emac_handle *h, int buf);
static int node_radix(const emac_node_sched *ns, int st);

/* Collective: every rank first closes its mappings of the others' memory, then all agree, and
   only then is this rank's exported memory (synchronisation block, mirror pool) freed. */
static void ipc_comm_release(emac_comm *cm) {
  int r, k;
  for (r = 0; r < cm->size; r++) {
    if (r != cm->rank && cm->peer_sync_base[r]) ipc_unmap(cm->peer_sync_base[r]);
    for (k = 0; r != cm->rank && k < cm->peer_nseg[r]; k++) ipc_unmap(cm->peer_seg[r][k]);
  }
  if (cm->ag && cm->size > 1) ipc_agree(cm, 1);
  for (k = 0; k < cm->nseg; k++) {
    emac_gpu_free(cm->seg[k].base);
    free(cm->seg[k].fr);
  }
  for (k = 0; k < cm->nbad; k++) emac_gpu_free(cm->bad_seg[k]);
  for (r = 0; r < cm->nmirrors; r++) emac_gpu_free(cm->mirrors[r].p);
  free(cm->mirrors);
  emac_gpu_free(cm->d_peer_sync);
  emac_gpu_free(cm->sync);
  for (r = 0; r < cm->nstale_sync; r++) emac_gpu_free(cm->stale_sync[r]);
  emac_gpu_host_free(cm->err);
  memset(cm, 0, sizeof(*cm));
}

typedef struct {
  unsigned char handle[EMAC_IPC_HANDLE_BYTES];
  long offset;
  long extent; /* bytes of the exported allocation: the importer's mapping must match */
  unsigned long long buf_id; /* the exporter's allocation id (0: unknown) */
  int status;
  int refused;   /* [0]: the runtime refused to export one of this rank's buffers */
  int caller;    /* [0]: the exported send buffer is caller memory (not a library mirror) */
  int seg;       /* >= 0: an arena block, in the exporter's segment `seg` at `offset` (nothing exported) */
  long lack;     /* [0]: arena bytes this rank could not place: every rank grows the arena first */
  long len;      /* bytes the peers access (the sample spans them) */
  unsigned char sample[EMAC_SAMPLE_BYTES]; /* the exporter's own read of the buffer (ipc_exchange) */
  unsigned char uuid[16];                  /* communicator set-up: the exporter's device */
  unsigned char free_slots[EMAC_SYNC_SLOTS / 8]; /* handle set-up: slots this rank can use */
} ipc_export;

/* The synchronisation blocks: every rank exports its block, maps every peer's and validates the
   mappings with a write probe (as the buffers, ipc_exchange): each rank flips probe[me][0] in
   every peer's block through its mapping and checks that its own block shows every peer's flip.
   The runtime places small allocations side by side in shared chunks, and a second
   communicator's block mapped by a process that already maps the first one's was measured to
   miss (8 processes on one MI355X: one rank never saw a peer's flags), and the runtime may refuse
   to export a fresh block (an allocation placed where a freed one a peer still maps lay; measured
   on a third communicator of 3 processes after 1200 handle lifetimes). A failed round keeps the
   blocks it allocated (peers may map them; freed with the communicator) and retries with a fresh,
   larger allocation. Collective: every rank runs every round whatever failed locally (`rc`). */
#define EMAC_SYNC_ATTEMPTS 8
static int ipc_sync_exchange(emac_comm *cm, int rc, ipc_export *all) {
  ipc_export mine;
  const int R = cm->size;
  int attempt, r;
  for (attempt = 0; attempt < EMAC_SYNC_ATTEMPTS; attempt++) {
    void *pk[EMAC_PROBE_MAX];
    unsigned char vals[EMAC_PROBE_MAX], seen[EMAC_PROBE_MAX];
    int n = 0, good = 1, agreed;
    memset(&mine, 0, sizeof(mine));
    if (!rc && cm->sync) { /* the previous round's block stays allocated until the communicator goes */
      cm->stale_sync[cm->nstale_sync++] = cm->sync;
      cm->sync = NULL;
    }
    if (!rc) rc = emac_gpu_malloc_uncached(&cm->sync, sizeof(emac_sync) << attempt);
    if (!rc) {
      const int er = emac_gpu_ipc_export(cm->sync, mine.handle, &mine.offset);
      if (er == EMAC_ERR_TRANSPORT) {
        mine.refused = 1; /* no peer maps it: this rank misses every flip and the round repeats */
        if (getenv("EXT_MPI_AMD_DEBUG_IPC"))
          fprintf(stderr, "ipc rank %d: export of my synchronisation block refused (attempt %d)\n", cm->rank, attempt);
      } else {
        rc = er;
      }
    }
    if (!rc && !mine.refused) {
      void *b0;
      mine.extent = emac_gpu_alloc_extent(cm->sync, &b0);
      mine.buf_id = emac_gpu_buffer_id(b0);
    }
    mine.status = rc == 0;
    if (!rc) emac_gpu_device_uuid(mine.uuid);
    if (cm->ag(cm->ag_ctx, &mine, all, (long)sizeof(ipc_export))) return EMAC_ERR_TRANSPORT;
    for (r = 0; r < R; r++)
      if (!all[r].status) rc = rc ? rc : EMAC_ERR_TRANSPORT;
    cm->cross_device = 0;
    for (r = 0; !rc && r < R; r++)
      if (memcmp(all[r].uuid, mine.uuid, 16)) cm->cross_device = 1;
    for (r = 0; !rc && r < R; r++) {
      if (r == cm->rank) {
        cm->peer_sync[r] = cm->sync;
        continue;
      }
      cm->peer_sync_base[r] = all[r].refused ? NULL : ipc_map_peer(all[r].handle, all[r].buf_id, all[r].extent);
      if (!cm->peer_sync_base[r]) {
        /* not fatal: the exporter misses this rank's flip below and the round is repeated with
           fresh blocks (measured: an open refused for a second communicator's block, 4 processes) */
        cm->peer_sync[r] = NULL;
        if (getenv("EXT_MPI_AMD_DEBUG_IPC"))
          fprintf(stderr, "ipc rank %d: cannot map peer %d's synchronisation block (attempt %d)\n", cm->rank, r,
                  attempt);
        continue;
      }
      cm->peer_sync[r] = (char *)cm->peer_sync_base[r] + all[r].offset;
      pk[n] = &((emac_sync *)cm->peer_sync[r])->probe[cm->rank][0];
      vals[n++] = (unsigned char)(0x5A ^ (cm->rank + 1));
    }
    if (!rc && R > 1) rc = emac_gpu_poke(pk, vals, n, NULL);
    agreed = ipc_agree(cm, rc == 0); /* every flip has landed */
    if (!rc) rc = agreed;
    if (rc) return rc;
    for (n = 0, r = 0; r < R; r++)
      if (r != cm->rank) pk[n++] = &((emac_sync *)cm->sync)->probe[r][0];
    if ((rc = emac_gpu_peek((const void *const *)pk, seen, n, NULL))) good = 0; /* still in the verdict below */
    for (n = 0, r = 0; r < R; r++)
      if (r != cm->rank) {
        if (!rc && seen[n] != (unsigned char)(0x5A ^ (r + 1))) {
          good = 0;
          if (getenv("EXT_MPI_AMD_DEBUG_IPC"))
            fprintf(stderr, "ipc rank %d: peer %d does not reach my synchronisation block (attempt %d)\n", cm->rank, r,
                    attempt);
        }
        n++;
      }
    memset(vals, 0, sizeof(vals));
    if (!rc) rc = emac_gpu_poke(pk, vals, n, NULL);
    {
      int v[2] = {good, rc == 0}, allv[2 * EMAC_MAX_RANKS], ok = 1, fine = 1;
      if (cm->ag(cm->ag_ctx, v, allv, (long)sizeof(v))) return EMAC_ERR_TRANSPORT;
      for (r = 0; r < R; r++) {
        ok &= allv[2 * r];
        fine &= allv[2 * r + 1];
      }
      if (!fine) return rc ? rc : EMAC_ERR_TRANSPORT;
      if (ok) return 0;
    }
    for (r = 0; r < R; r++)
      if (r != cm->rank && cm->peer_sync_base[r]) {
        ipc_unmap(cm->peer_sync_base[r]);
        cm->peer_sync_base[r] = NULL;
      }
  }
  fprintf(stderr, "ext_mpi_amd: rank %d: synchronisation blocks still unreachable after %d set-up rounds\n", cm->rank,
          EMAC_SYNC_ATTEMPTS);
  return EMAC_ERR_TRANSPORT;
}

int ext_mpi_amd_comm_init_ipc(int rank, int size, ext_mpi_amd_allgather_fn allgather, void *ctx, int device,
                              int *comm) {
  emac_comm *cm;
  ipc_export all[EMAC_MAX_RANKS];
  const char *tmo;
  int i, rc;
  if (!comm || !allgather || size < 1 || size > EMAC_MAX_RANKS || rank < 0 || rank >= size) return EMAC_ERR_ARG;
  *comm = -1;
  for (i = 0; i < MAX_COMMS && comms[i].used; i++);
  if (i == MAX_COMMS) return EMAC_ERR_MALLOC;
  cm = &comms[i];
  memset(cm, 0, sizeof(*cm));
  cm->rank = rank;
  cm->size = size;
  cm->loop_group = -1;
  cm->ipc = 1;
  cm->ag = allgather;
  cm->ag_ctx = ctx;
  /* every rank takes part in every allgather below, whatever failed locally, so that all ranks
     reach the same verdict */
  rc = emac_gpu_device_count() > 0 ? 0 : EMAC_ERR_DEVICE;
  if (!rc && device >= 0) rc = emac_gpu_set_device(device);
  if (!rc) rc = emac_gpu_get_device(&cm->device);
  if (!rc) rc = emac_gpu_host_alloc_mapped((void **)&cm->err, sizeof(int) * EMAC_SYNC_SLOTS);
  rc = ipc_sync_exchange(cm, rc, all);
  if (!rc && (rc = emac_gpu_malloc((void **)&cm->d_peer_sync, sizeof(void *) * (size_t)size)) == 0)
    rc = emac_gpu_memcpy(cm->d_peer_sync, cm->peer_sync, sizeof(void *) * (size_t)size);
  {
    const int agreed = ipc_agree(cm, rc == 0); /* every rank mapped every block */
    if (!rc) rc = agreed;
  }
  if (rc) {
    ipc_comm_release(cm);
    return rc;
  }
  /* a rank that never arrives is reported after this many seconds (default 30) */
  tmo = getenv("EXT_MPI_AMD_BARRIER_TIMEOUT");
  cm->timeout_ticks = (long)((tmo ? atof(tmo) : 30.0) * (double)emac_gpu_wallclock_hz());
  cm->used = 1;
  *comm = i;
  return 0;
}

/* Mapping the peers' buffers (the reference: cuda_shmem.c:218-299 opens every peer's cudaIpc
   handle once at init; EXT_MPI_Done closes them after a node barrier, ext_mpi_native.c:269-387 with
   cuda_shmem.c:190-216,301-314). What can go wrong, and what rules it out here:
   * The runtime's IPC handle of an allocation is a function of the exporter's address and size:
     an allocation freed while a peer still maps it and re-allocated at the same address exports
     the same handle, and importing it resolves to the OLD memory. The rule of the reference rules
     it out for caller memory: a peer-mapped handle's Done is collective (ext_mpi_amd_done: every
     rank closes its mappings, then the ranks agree), so no caller allocation is freed under a
     mapping as long as the caller keeps its buffers until Done.
   * Library memory the peers read -- outboxes, mirrors of send buffers -- lives in the
     communicator's ARENA: a few large segments per rank, each exported and mapped ONCE (when it is
     added) and validated then with a random nonce the owner wrote into its head, so a mapping of
     any other memory cannot pass. Handles carve blocks out of the segments; nothing library-owned
     is exported, imported or closed per handle, and segments are freed only by the collective
     communicator free.
   * Peers never WRITE caller memory, at set-up or later: the send buffer is only read (the fold's
     leaves), each rank's results go to its own outbox, and every rank pulls the results into its
     own receive buffer, which is never exported. A stale mapping could therefore only feed wrong
     leaves, never overwrite anything.
   * Every mapping of a caller's send buffer is still validated, read-only: the exporter samples
     its buffer (emac_gpu_sample: 8 spots of 8 bytes) and publishes the sample with its handle;
     every importer samples the same spots through its mapping. A mismatch, a mapping the runtime
     refuses or one shorter than the exporter's allocation re-places that send buffer in an arena
     mirror (staged in on the handle's stream) and the exchange repeats.
     EXT_MPI_AMD_IPC_FORCE_MIRROR=1 re-places every rank's send buffer in the first round, so the
     mirror path runs deterministically (tests/test_gpu_peer_mapped.py).
   The set-up reads the caller's send buffer: the device is synchronised first, so a kernel still
   filling it cannot make the exporter's and the importers' samples differ. */
#define EMAC_IPC_ATTEMPTS 8

/* ---- the arena ---- */

static int arena_alloc(emac_comm *cm, long bytes, void **p) {
  int k, i;
  bytes = (bytes + EMAC_ARENA_ALIGN - 1) / EMAC_ARENA_ALIGN * EMAC_ARENA_ALIGN;
  if (bytes <= 0) bytes = EMAC_ARENA_ALIGN;
  for (k = 0; k < cm->nseg; k++) {
    arena_seg *s = &cm->seg[k];
    for (i = 0; i < s->nfr; i++)
      if (s->fr[i].len >= bytes) {
        *p = (char *)s->base + s->fr[i].off;
        s->fr[i].off += bytes;
        s->fr[i].len -= bytes;
        if (!s->fr[i].len) {
          memmove(&s->fr[i], &s->fr[i + 1], sizeof(arena_free) * (size_t)(s->nfr - i - 1));
          s->nfr--;
        }
        return 0;
      }
  }
  return EMAC_ERR_MALLOC;
}

static int arena_owns(const emac_comm *cm, const void *p, int *seg) {
  int k;
  for (k = 0; k < cm->nseg; k++)
    if ((const char *)p >= (const char *)cm->seg[k].base && (const char *)p < (const char *)cm->seg[k].base + cm->seg[k].bytes) {
      if (seg) *seg = k;
      return 1;
    }
  return 0;
}

static void arena_release(emac_comm *cm, void *p, long bytes) {
  arena_seg *s;
  long off;
  int k, i;
  if (!p || !cm->used || !arena_owns(cm, p, &k)) return;
  bytes = (bytes + EMAC_ARENA_ALIGN - 1) / EMAC_ARENA_ALIGN * EMAC_ARENA_ALIGN;
  if (bytes <= 0) bytes = EMAC_ARENA_ALIGN;
  s = &cm->seg[k];
  off = (long)((char *)p - (char *)s->base);
  for (i = 0; i < s->nfr && s->fr[i].off < off; i++);
  if (s->nfr == s->capfr) {
    arena_free *f = (arena_free *)realloc(s->fr, sizeof(arena_free) * (size_t)(2 * s->capfr + 8));
    if (!f) return; /* the block stays allocated */
    s->fr = f;
    s->capfr = 2 * s->capfr + 8;
  }
  memmove(&s->fr[i + 1], &s->fr[i], sizeof(arena_free) * (size_t)(s->nfr - i));
  s->fr[i].off = off;
  s->fr[i].len = bytes;
  s->nfr++;
  if (i + 1 < s->nfr && s->fr[i].off + s->fr[i].len == s->fr[i + 1].off) { /* merge with the next */
    s->fr[i].len += s->fr[i + 1].len;
    memmove(&s->fr[i + 1], &s->fr[i + 2], sizeof(arena_free) * (size_t)(s->nfr - i - 2));
    s->nfr--;
  }
  if (i > 0 && s->fr[i - 1].off + s->fr[i - 1].len == s->fr[i].off) { /* and the previous */
    s->fr[i - 1].len += s->fr[i].len;
    memmove(&s->fr[i], &s->fr[i + 1], sizeof(arena_free) * (size_t)(s->nfr - i - 1));
    s->nfr--;
  }
}

typedef struct {
  int status, grow;
  unsigned char handle[EMAC_IPC_HANDLE_BYTES];
  long offset, extent;
  unsigned long long buf_id;
  unsigned char nonce[EMAC_SAMPLE_BYTES];
} arena_export;

static unsigned long long g_nonce_state;

/* Collective: ranks that lack `need` bytes (0: none) add a segment of at least that size (and at
   least their arena's size so far, EMAC_ARENA_MIN at first); every rank maps every new segment
   and checks the nonce in its head through the mapping. A segment some rank cannot map or
   validate is set aside (freed with the communicator) and its owner tries a fresh one. */
static int arena_grow(emac_comm *cm, int rc, long need) {
  const int R = cm->size;
  int attempt, r;
  for (attempt = 0; attempt < EMAC_IPC_ATTEMPTS; attempt++) {
    arena_export mine, all[EMAC_MAX_RANKS];
    void *nb = NULL, *mapped[EMAC_MAX_RANKS];
    unsigned bad = 0, allbad[EMAC_MAX_RANKS], badall = 0;
    long sz = 0;
    int any = 0;
    memset(&mine, 0, sizeof(mine));
    if (!rc && need > 0) {
      long have = 0;
      int i;
      for (i = 0; i < cm->nseg; i++) have += cm->seg[i].bytes;
      sz = need + EMAC_ARENA_HEAD;
      if (sz < have) sz = have;
      if (sz < EMAC_ARENA_MIN) sz = EMAC_ARENA_MIN;
      sz = (long)((sz + (long)EMAC_IPC_GRANULE - 1) / (long)EMAC_IPC_GRANULE * (long)EMAC_IPC_GRANULE);
      if (cm->nseg == EMAC_ARENA_SEGS || cm->nbad == EMAC_ARENA_SEGS) rc = EMAC_ERR_MALLOC;
      if (!rc) rc = emac_gpu_malloc(&nb, (size_t)sz);
      if (!rc) {
        void *b0;
        unsigned long long x = g_nonce_state ^ ((unsigned long long)(size_t)nb * 0x9E3779B97F4A7C15ull) ^
                               ((unsigned long long)cm->rank << 40) ^ (unsigned long long)attempt;
        for (i = 0; i < EMAC_SAMPLE_BYTES; i++) { /* xorshift64* */
          x ^= x >> 12;
          x ^= x << 25;
          x ^= x >> 27;
          mine.nonce[i] = (unsigned char)((x * 0x2545F4914F6CDD1Dull) >> 56);
        }
        g_nonce_state = x + 0x9E3779B97F4A7C15ull;
        /* the nonce is the head's first EMAC_SAMPLE_BYTES bytes: sampled whole (len = that size) */
        rc = emac_gpu_memcpy(nb, mine.nonce, EMAC_SAMPLE_BYTES);
        if (!rc) rc = emac_gpu_device_sync();
        if (!rc) rc = emac_gpu_ipc_export(nb, mine.handle, &mine.offset);
        mine.extent = emac_gpu_alloc_extent(nb, &b0);
        mine.buf_id = emac_gpu_buffer_id(b0);
        if (rc == EMAC_ERR_TRANSPORT) { /* export refused: set aside, try another */
          rc = 0;
          bad = 1u << cm->rank;
        }
      }
      mine.grow = 1;
    }
    mine.status = rc == 0;
    if (cm->ag(cm->ag_ctx, &mine, all, (long)sizeof(mine))) return EMAC_ERR_TRANSPORT;
    for (r = 0; r < R; r++) {
      if (!all[r].status) rc = rc ? rc : EMAC_ERR_TRANSPORT;
      any |= all[r].grow;
    }
    if (rc) {
      if (nb) emac_gpu_free(nb); /* nobody maps it: every rank stops here */
      return rc;
    }
    if (!any) return 0;
    {
      const void *pk[EMAC_MAX_RANKS];
      long pl[EMAC_MAX_RANKS];
      int who[EMAC_MAX_RANKS], n = 0;
      unsigned char seen[EMAC_MAX_RANKS * EMAC_SAMPLE_BYTES];
      for (r = 0; r < R; r++) {
        void *ext_base;
        mapped[r] = NULL;
        if (!all[r].grow || r == cm->rank) continue;
        if (!(mapped[r] = ipc_map_peer(all[r].handle, all[r].buf_id, all[r].extent)) || all[r].offset != 0 ||
            emac_gpu_alloc_extent(mapped[r], &ext_base) != all[r].extent) {
          bad |= 1u << r;
          continue;
        }
        pk[n] = mapped[r];
        pl[n] = EMAC_SAMPLE_BYTES;
        who[n++] = r;
      }
      if (n && (rc = emac_gpu_sample(pk, pl, n, seen, NULL))) return rc;
      for (r = 0; r < n; r++)
        if (memcmp(seen + r * EMAC_SAMPLE_BYTES, all[who[r]].nonce, EMAC_SAMPLE_BYTES)) bad |= 1u << who[r];
    }
    if (cm->ag(cm->ag_ctx, &bad, allbad, (long)sizeof(unsigned))) return EMAC_ERR_TRANSPORT;
    for (r = 0; r < R; r++) badall |= allbad[r];
    for (r = 0; r < R; r++) {
      if (!all[r].grow) continue;
      if ((badall >> r) & 1) {
        if (r == cm->rank) {
          cm->bad_seg[cm->nbad++] = nb; /* a peer may map it: freed with the communicator */
        } else if (mapped[r]) {
          ipc_unmap(mapped[r]);
        }
        if (getenv("EXT_MPI_AMD_DEBUG_IPC"))
          fprintf(stderr, "ipc rank %d: rank %d's new arena segment failed validation (attempt %d)\n", cm->rank, r,
                  attempt);
        continue;
      }
      if (r == cm->rank) {
        arena_seg *s = &cm->seg[cm->nseg];
        memset(s, 0, sizeof(*s));
        s->base = nb;
        s->bytes = sz;
        s->fr = (arena_free *)malloc(sizeof(arena_free) * 8);
        s->capfr = 8;
        if (s->fr) {
          s->fr[0].off = EMAC_ARENA_HEAD;
          s->fr[0].len = sz - EMAC_ARENA_HEAD;
          s->nfr = 1;
        }
        cm->peer_seg[r][cm->nseg++] = nb;
        cm->peer_nseg[r] = cm->nseg;
        need = 0;
      } else {
        cm->peer_seg[r][cm->peer_nseg[r]++] = mapped[r];
      }
    }
    if (!badall) return 0;
  }
  fprintf(stderr, "ext_mpi_amd: rank %d: arena segments still unreachable after %d set-up rounds\n", cm->rank,
          EMAC_IPC_ATTEMPTS);
  return EMAC_ERR_TRANSPORT;
}

/* Byte offset of every piece of position `pos`'s owner chunk inside that rank's outbox: pieces
   back to back, each at the 16-byte phase its elements have in the message (so the fold's leaves,
   the outbox and the receive buffer agree on vector alignment). Returns the outbox bytes. */
static long outbox_layout(const emac_plan *p, int pos, long *at) {
  const int R = p->nranks;
  long cur = 0;
  int pc;
  for (pc = 0; pc < p->npieces; pc++) {
    const long off = p->chunk_off[(size_t)pc * R + pos], len = p->chunk_len[(size_t)pc * R + pos];
    const long a = ((cur + 15) & ~15L) + ((off * p->tsize) & 15);
    if (at) at[pc] = a;
    if (len > 0) cur = a + len * p->tsize;
  }
  return cur;
}

enum { IPC_SEND = 0, IPC_OUTBOX = 1, IPC_NBUF = 2 };

/* One exchange of the IPC set-up (collective whatever failed locally before: `rc`). Every rank
   publishes its send buffer (an exported caller allocation with a sample of it, or an arena block)
   and its outbox (an arena block). On return peer[t][r] holds rank r's buffer t as reachable here,
   all[] the exports, and *miss a bit per rank whose send buffer this rank could not map or validate. */
static int ipc_exchange(emac_handle *h, emac_comm *cm, int rc, long lack, ipc_export *all,
                        void *(*peer)[EMAC_MAX_RANKS], unsigned *miss, int *grow) {
  ipc_export mine[IPC_NBUF];
  const int R = cm->size;
  void *own[IPC_NBUF] = {h->dsend[0], h->outbox};
  const long len[IPC_NBUF] = {(long)h->bytes, (long)h->outbox_bytes};
  int r, t, k;
  memset(mine, 0, sizeof(mine));
  *miss = 0;
  *grow = 0;
  mine[0].lack = lack;
  for (t = 0; t < IPC_NBUF && !rc && !lack; t++) {
    mine[t].len = len[t];
    if (arena_owns(cm, own[t], &k)) {
      mine[t].seg = k;
      mine[t].offset = (long)((char *)own[t] - (char *)cm->seg[k].base);
    } else if (t == IPC_SEND) {
      void *b0;
      const int er = emac_gpu_ipc_export(own[t], mine[t].handle, &mine[t].offset);
      mine[t].seg = -1;
      if (er == EMAC_ERR_TRANSPORT)
        mine[0].refused = 1; /* refused by the runtime: this rank's send buffer is re-placed */
      else
        rc = er;
      mine[t].extent = emac_gpu_alloc_extent(own[t], &b0);
      mine[t].buf_id = emac_gpu_buffer_id(b0);
      if (!rc) rc = emac_gpu_sample((const void *const *)&own[t], &len[t], 1, mine[t].sample, h->stream);
    } else {
      rc = EMAC_ERR_ARG; /* an outbox outside the arena */
    }
  }
  for (r = 0; r < EMAC_SYNC_SLOTS; r++)
    if (!cm->slot_used[r]) mine[0].free_slots[r >> 3] |= (unsigned char)(1u << (r & 7));
  mine[0].status = rc == 0;
  mine[0].caller = mine[0].seg < 0 && !ipc_pool_owns(cm, h->dsend[0]);
  if (cm->ag(cm->ag_ctx, mine, all, (long)sizeof(mine))) return EMAC_ERR_TRANSPORT;
  for (r = 0; r < R; r++) {
    if (!all[IPC_NBUF * r].status && !rc) rc = EMAC_ERR_TRANSPORT;
    if (all[IPC_NBUF * r].lack > 0) *grow = 1;
  }
  if (rc || *grow) return rc; /* (every rank reaches the same verdict) */
  {
    const void *pk[EMAC_MAX_RANKS];
    long pl[EMAC_MAX_RANKS];
    int who[EMAC_MAX_RANKS], n = 0;
    unsigned char seen[EMAC_MAX_RANKS * EMAC_SAMPLE_BYTES];
    for (r = 0; r < R; r++)
      for (t = 0; t < IPC_NBUF; t++) {
        const ipc_export *e = &all[IPC_NBUF * r + t];
        void *base, *ext_base;
        long extent;
        peer[t][r] = NULL;
        if (r == cm->rank) {
          peer[t][r] = own[t];
          continue;
        }
        if (e->seg >= 0) { /* an arena block: the segment was validated when it was added */
          if (e->seg < cm->peer_nseg[r]) peer[t][r] = (char *)cm->peer_seg[r][e->seg] + e->offset;
          if (!peer[t][r]) *miss |= 1u << r;
          continue;
        }
        *miss |= 1u << r; /* until validated below */
        if (all[IPC_NBUF * r].refused || !(base = ipc_map_peer(e->handle, e->buf_id, e->extent))) continue;
        h->mapped[h->nmapped++] = base;
        /* a mapping the runtime can describe must hold the peer's whole allocation (one it cannot
           describe is taken at the exporter's word; the sample still checks it) */
        extent = emac_gpu_alloc_extent(base, &ext_base);
        if (extent < 0) {
          extent = e->extent;
          ext_base = base;
        }
        if (ext_base != base || extent != e->extent || e->offset < 0 || e->offset + e->len > extent) continue;
        peer[t][r] = (char *)base + e->offset;
        pk[n] = peer[t][r];
        pl[n] = e->len;
        who[n++] = r;
      }
    if ((rc = emac_gpu_sample(pk, pl, n, seen, h->stream))) return rc;
    for (t = 0; t < n; t++) {
      if (!memcmp(seen + t * EMAC_SAMPLE_BYTES, all[IPC_NBUF * who[t]].sample, EMAC_SAMPLE_BYTES))
        *miss &= ~(1u << who[t]);
      else
        peer[IPC_SEND][who[t]] = NULL;
    }
    if (getenv("EXT_MPI_AMD_DEBUG_IPC"))
      for (r = 0; r < R; r++)
        if ((*miss >> r) & 1) fprintf(stderr, "ipc rank %d: cannot map or validate peer %d's send buffer\n", cm->rank, r);
  }
  return 0;
}

/* Collective: every rank runs the same exchanges whatever failed locally before (`rc`), so that
   a local failure cannot unmatch the sequence. */
static int ipc_allreduce_init(emac_handle *h, emac_comm *cm, const void *sendbuf, void *recvbuf, int rc) {
  ipc_export all[IPC_NBUF * EMAC_MAX_RANKS];
  void *peer[IPC_NBUF][EMAC_MAX_RANKS];
  long *at = NULL;
  emac_bucket *b = NULL;
  int R = cm->size, r, t, pc, nb = 0, c, slot, attempt;
  const char *fe = getenv("EXT_MPI_AMD_IPC_FORCE_MIRROR");
  const int force = fe && atoi(fe) > 0;
  if (!rc && h->bytes) rc = map_buffers(h, 0, sendbuf, recvbuf);
  if (R == 1 || !h->bytes) { /* nothing to map: this rank folds alone (no peers), or nothing at all */
    if (!rc && h->bytes && !h->dsend[0]) { /* a send mirror map_buffers left to the arena */
      if (!(rc = emac_gpu_malloc(&h->dsend[0], h->bytes))) h->send_local = 1;
      if (h->recv_mirror[0] && !h->drecv[0]) h->drecv[0] = h->dsend[0];
    }
    attempt = 0;
    {
      ipc_export mine;
      memset(&mine, 0, sizeof(mine));
      for (r = 0; r < EMAC_SYNC_SLOTS; r++)
        if (!cm->slot_used[r]) mine.free_slots[r >> 3] |= (unsigned char)(1u << (r & 7));
      mine.status = rc == 0;
      for (r = 0; r < R; r++) all[IPC_NBUF * r] = mine;
      if (R > 1) { /* empty message: agree on the slot only */
        ipc_export g[EMAC_MAX_RANKS];
        if (cm->ag(cm->ag_ctx, &mine, g, (long)sizeof(mine))) return EMAC_ERR_TRANSPORT;
        for (r = 0; r < R; r++) {
          all[IPC_NBUF * r] = g[r];
          if (!g[r].status) rc = rc ? rc : EMAC_ERR_TRANSPORT;
        }
      }
      if (rc) return rc;
    }
  } else {
    /* the samples read the send buffer: work the application still has in flight on it must have
       landed (the reference synchronises the device before every barrier, ext_mpi_native_exec.c:556-558) */
    if (!rc) rc = emac_gpu_device_sync();
    if (!rc) {
      h->outbox_bytes = (size_t)outbox_layout(&h->plan, h->me_pos, NULL);
      if (h->outbox_bytes < 16) h->outbox_bytes = 16;
    }
    for (attempt = 0;; attempt++) {
      unsigned miss, allmiss[EMAC_MAX_RANKS], stale = 0;
      int again = 0, grow = 0;
      /* the outbox, and a send mirror left to the arena (host or non-exportable memory, or a send
         buffer re-placed below); a rank that lacks room says so in the exchange, every rank then
         grows the arena (one collective round) and exchanges again */
      long lack = 0;
      if (!rc && !h->outbox && arena_alloc(cm, (long)h->outbox_bytes, &h->outbox))
        lack += (long)(h->outbox_bytes + EMAC_ARENA_ALIGN - 1) / EMAC_ARENA_ALIGN * EMAC_ARENA_ALIGN;
      if (!rc && !h->dsend[0]) {
        void *p = NULL;
        if (arena_alloc(cm, (long)h->bytes, &p)) {
          lack += (long)(h->bytes + EMAC_ARENA_ALIGN - 1) / EMAC_ARENA_ALIGN * EMAC_ARENA_ALIGN;
        } else {
          h->dsend[0] = p;
          h->send_arena = 1;
          if (h->recv_mirror[0] && !h->drecv[0]) h->drecv[0] = p; /* in place */
        }
      }
      rc = ipc_exchange(h, cm, rc, lack, all, peer, &miss, &grow);
      if (!rc && grow) {
        if (attempt == EMAC_IPC_ATTEMPTS - 1) return EMAC_ERR_MALLOC; /* the same on every rank */
        rc = arena_grow(cm, 0, lack);
        continue;
      }
      if (!rc && force && attempt == 0 && !h->send_arena) miss |= 1u << cm->rank; /* re-place mine */
      if (rc) miss = ~0u; /* a failed rank: the verdict below stops every rank */
      if (cm->ag(cm->ag_ctx, &miss, allmiss, (long)sizeof(miss))) return EMAC_ERR_TRANSPORT;
      for (r = 0; r < R; r++) {
        if (allmiss[r] == ~0u) return rc ? rc : EMAC_ERR_TRANSPORT;
        again |= allmiss[r] != 0;
        stale |= (allmiss[r] >> cm->rank) & 1u;
      }
      if (!again) break;
      if (getenv("EXT_MPI_AMD_DEBUG_IPC"))
        fprintf(stderr, "ipc rank %d: attempt %d: re-placing%s\n", cm->rank, attempt, stale ? " send" : "");
      if (attempt == EMAC_IPC_ATTEMPTS - 1 || (stale && h->send_arena)) {
        fprintf(stderr, "ext_mpi_amd: rank %d: peer mappings still unreachable after %d set-up rounds\n", cm->rank,
                attempt + 1);
        return EMAC_ERR_TRANSPORT;
      }
      for (r = 0; r < h->nmapped; r++) ipc_unmap(h->mapped[r]);
      h->nmapped = 0;
      if (stale) {
        /* this rank's send buffer into an arena mirror (placed at the top of the next round),
           staged in on the handle's stream; in place, the one buffer, staged in and out */
        if (h->dsend[0] == h->drecv[0]) {
          h->recv_mirror[0] = 1;
          h->drecv[0] = NULL;
        } else {
          h->send_mirror[0] = 1;
        }
        h->dsend[0] = NULL;
      }
    }
  }
  /* Done is collective iff some rank's exported send buffer is caller memory (the same verdict on
     every rank): library memory is never freed under a mapping anyway (ext_mpi_amd_done) */
  for (r = 0; R > 1 && h->bytes && r < R; r++) h->done_collective |= all[IPC_NBUF * r].caller;
  /* the synchronisation slot: the lowest one free on every rank (ranks may have released
     their handles in different orders) */
  for (slot = 0; slot < EMAC_SYNC_SLOTS; slot++) {
    for (r = 0; r < R && (all[IPC_NBUF * r].free_slots[slot >> 3] >> (slot & 7)) & 1; r++);
    if (r == R) break;
  }
  if (slot == EMAC_SYNC_SLOTS) return EMAC_ERR_MALLOC; /* same verdict on every rank */
  h->slot = slot;
  cm->slot_used[slot] = 1;
  h->slot_held = 1;
  cm->err[slot] = 0; /* a failure of the slot's previous handle that nobody waited for */
  {
    /* A system-scope release (command processor, every XCD's L2) before each phase-0 barrier,
       by default when some peer sits on another device: its loads of this rank's send buffer go
       over xGMI to HBM and see nothing an L2 still holds. Ranks sharing one device read through
       the same L2s and the packet boundary after the producer kernel suffices, so the release
       (5 us per Start with 2 processes, 9 us with 4: profiles/r02_ipc_latency_release.json) is
       off there. EXT_MPI_AMD_IPC_RELEASE=1 / 0 forces it on / off. */
    const char *e = getenv("EXT_MPI_AMD_IPC_RELEASE");
    const int rel = e ? atoi(e) > 0 : cm->cross_device;
    if (R > 1 && rel && (rc = emac_gpu_event_create_release(&h->ev_release))) return rc;
  }
  h->epoch[0] = cm->slot_epoch[slot][0];
  h->epoch[1] = cm->slot_epoch[slot][1];
  if (!h->bytes) return 0;
  /* this rank's owner chunks (reduce_copyin): leaves from the peers' send buffers in the plan's
     fold order, the result into this rank's outbox (its receive buffer when alone). Then
     (reduce_copyout) every owner's result is PULLED from that owner's outbox into this rank's
     receive buffer, this rank's own last: each rank writes only memory it owns. */
  c = h->me_pos;
  b = (emac_bucket *)calloc((size_t)h->plan.npieces * (size_t)(R + 1), sizeof(emac_bucket));
  at = (long *)calloc((size_t)h->plan.npieces, sizeof(long));
  if (!b || !at) {
    free(b);
    free(at);
    return EMAC_ERR_MALLOC;
  }
  if (R > 1) outbox_layout(&h->plan, c, at);
  for (pc = 0; pc < h->plan.npieces; pc++) {
    long off = h->plan.chunk_off[(size_t)pc * R + c], len = h->plan.chunk_len[(size_t)pc * R + c];
    emac_bucket *bk = &b[nb];
    if (len <= 0) continue;
    for (t = 0; t < R; t++) bk->src[t] = R > 1 ? peer[IPC_SEND][h->plan.leaf_rank[c][t]] : h->dsend[0];
    /* place_bucket moves every pointer by the chunk's message offset */
    bk->dst[0] = R > 1 ? (char *)h->outbox + at[pc] - off * h->plan.tsize : (char *)h->drecv[0];
    bk->ndst = 1;
    place_bucket(bk, R, off, len, h->plan.tsize);
    nb++;
  }
  h->nsrc = R;
  h->fan = R > 1 ? 2 : 0; /* peer-mapped: system-coherent launch */
  if (R > 1) {
    /* the pull, owners in the order after this rank (next owner first), so that at any moment
       the ranks' loads head for different GPUs' links; this rank's own chunk (local) last */
    emac_bucket *pb = b + nb;
    int np = 0, k;
    for (k = 1; k <= R; k++) {
      const int q = (cm->rank + k) % R, cq = h->plan.rank_pos[q];
      outbox_layout(&h->plan, cq, at);
      for (pc = 0; pc < h->plan.npieces; pc++) {
        long off = h->plan.chunk_off[(size_t)pc * R + cq], len = h->plan.chunk_len[(size_t)pc * R + cq];
        if (len <= 0) continue;
        pb[np].src[0] = (char *)peer[IPC_OUTBOX][q] + at[pc] - off * h->plan.tsize;
        pb[np].dst[0] = h->drecv[0];
        pb[np].ndst = 1;
        place_bucket(&pb[np], 1, off, len, h->plan.tsize);
        np++;
      }
    }
    if ((rc = upload_launch_as(h, &h->pull, pb, np, 1, 0))) { /* a copy: the schedule of nsrc 1 for every op */
      free(b);
      free(at);
      return rc;
    }
  }
  free(at);
  {
    /* small messages: barrier, fold, barrier and pull in one launch (EXT_MPI_AMD_IPC_FUSED_MAX
       bytes per rank, default 1 MiB; 0 disables) */
    const char *fm = getenv("EXT_MPI_AMD_IPC_FUSED_MAX");
    const long fused_max = fm ? atol(fm) : (1L << 20);
    h->fused = R > 1 && (long)h->bytes <= fused_max;
  }
  if (getenv("EXT_MPI_AMD_DEBUG_IPC") && (attempt > 0 || atoi(getenv("EXT_MPI_AMD_DEBUG_IPC")) >= 2))
    fprintf(stderr, "ipc rank %d: own send %p recv %p outbox %p bytes %zu, %d buckets, slot %d, %d attempt(s)\n",
            cm->rank, h->dsend[0], h->drecv[0], h->outbox, h->bytes, nb, slot, attempt + 1);
  rc = upload_buckets(h, b, nb);
  free(b);
  return rc;
}

int ext_mpi_amd_comm_free(int comm) {
  if (comm < 0 || comm >= MAX_COMMS || !comms[comm].used) return EMAC_ERR_ARG;
  if (comms[comm].ipc) {
    ipc_comm_release(&comms[comm]);
    return 0;
  }
  if (comms[comm].loop_group >= 0) {
    loop_group *g = &loops[comms[comm].loop_group];
    g->nh[comms[comm].rank] = -1; /* this rank left */
    for (int r = 0; r < g->size; r++)
      if (g->nh[r] >= 0) goto keep;
    g->used = 0;
  keep:;
  } else {
    ncclCommDestroy(comms[comm].nccl);
  }
  comms[comm].used = 0;
  return 0;
}

int ext_mpi_amd_allreduce_init(const void *sendbuf, void *recvbuf, long count, int dtype, int op, int comm,
                               const char *copyin, int *handle) {
  emac_handle *h;
  emac_comm *cm;
  emac_copyin cfg;
  emac_bucket *b = NULL;
  int rc, t, R, nb = 0;
  long stage_total = 0;
  if (!handle || comm < 0 || comm >= MAX_COMMS || !comms[comm].used || count < 0) return EMAC_ERR_ARG;
  *handle = -1;
  cm = &comms[comm];
  R = cm->size / (cm->nodes > 1 && !cm->ipc ? cm->nodes : 1); /* ranks of one node */
  if ((rc = parse_cfg(copyin, R, &cfg))) return rc;
  if (emac_gpu_set_device(cm->device)) return EMAC_ERR_DEVICE;
  h = (emac_handle *)calloc(1, sizeof(emac_handle));
  if (!h) return EMAC_ERR_MALLOC;
  h->kind = cm->ipc ? KIND_IPC : KIND_COMM;
  h->comm = comm;
  h->device = cm->device;
  rc = emac_plan_build(&h->plan, R, count, dtype, op, &cfg);
  if (!rc) {
    h->me = cm->rank;
    h->me_pos = h->plan.rank_pos[h->me % R];
    h->bytes = (size_t)count * (size_t)h->plan.tsize;
    h->nodes = cm->size / R;
    h->ns = cm->ns;
    if (h->nodes > 1 && h->ns.nodes != h->nodes) rc = EMAC_ERR_ARG;
  }
  h->nbuf = 1;
  h->nsrc = R;
  if (cm->ipc) {
    if (!rc) rc = emac_gpu_stream_create(&h->stream);
    if ((rc = ipc_allreduce_init(h, cm, sendbuf, recvbuf, rc))) goto fail;
    if ((rc = finish_init(h, handle))) goto fail;
    return 0;
  }
  if (rc) goto fail;
  if ((rc = map_buffers(h, 0, sendbuf, recvbuf))) goto fail;
  {
    emac_fold *folds = NULL;
    int nf = 0, f;
    emac_bucket *xb = NULL;
    int nxb[2 * EMAC_MAX_NODE_STEPS] = {0}, st;
    const int nsteps = h->nodes > 1 ? h->ns.nsteps + h->ns.nred : 0; /* exchange steps with a fold */
    if ((rc = emac_comm_program_nodes(&h->plan, h->nodes > 1 ? &h->ns : NULL, h->me / R, h->me % R,
                                      (long)((unsigned long)h->dsend[0] & 15ul), &h->ops, &h->nops, &folds, &nf,
                                      &stage_total)))
      goto fail;
    b = (emac_bucket *)calloc((size_t)nf + 1, sizeof(emac_bucket));
    xb = (emac_bucket *)calloc(2 * EMAC_MAX_NODE_STEPS * ((size_t)nf + 1), sizeof(emac_bucket));
    if (!b || !xb || (rc = emac_gpu_malloc(&h->staging, (size_t)(stage_total > 0 ? stage_total : 16)))) {
      free(folds);
      free(xb);
      rc = rc ? rc : EMAC_ERR_MALLOC;
      goto fail;
    }
    for (f = 0; f < nf; f++) {
      const int node_pair = (folds[f].leg & ((1 << EMAC_LEG_STEP_SHIFT) - 1)) == EMAC_LEG_NODES_FOLD;
      const int step = folds[f].leg >> EMAC_LEG_STEP_SHIFT;
      emac_bucket *bk = node_pair ? &xb[(size_t)step * ((size_t)nf + 1) + (size_t)nxb[step]++] : &b[nb++];
      long off = folds[f].offset / h->plan.tsize;
      for (t = 0; t < folds[f].nleaf; t++) {
        /* leaf pointers are shifted back by the result's offset: split_alignment adds it */
        bk->src[t] = leg_base(h, folds[f].buf[t]) + folds[f].loff[t] - folds[f].offset;
      }
      bk->dst[0] = h->drecv[0];
      bk->ndst = 1;
      place_bucket(bk, folds[f].nleaf, off, folds[f].count, h->plan.tsize);
    }
    free(folds);
    for (st = 0; st < nsteps; st++)
      if (nxb[st] &&
          (rc = upload_launch_as(h, &h->xfold[st], xb + (size_t)st * ((size_t)nf + 1), nxb[st], node_radix(&h->ns, st),
                                 0))) {
        free(xb);
        goto fail;
      }
    free(xb);
  }
  if ((rc = upload_buckets(h, b, nb))) goto fail;
  free(b);
  b = NULL;
  if ((rc = emac_gpu_stream_create(&h->stream))) goto fail;
  if (cm->loop_group >= 0) {
    loop_group *g = &loops[cm->loop_group];
    if (g->nh[h->me] < 0 || g->nh[h->me] >= MAX_LOOP_HANDLES) {
      rc = EMAC_ERR_MALLOC;
      goto fail;
    }
    h->loop_index = g->nh[h->me];
  }
  if ((rc = finish_init(h, handle))) goto fail;
  if (cm->loop_group >= 0) loops[cm->loop_group].handle[h->me][loops[cm->loop_group].nh[h->me]++] = *handle;
  return 0;
fail:
  free(b);
  release(h);
  return rc;
}

/* radix of exchange step st: the reduce-scatter steps, then the allgather steps that reduce */
static int node_radix(const emac_node_sched *ns, int st) {
  return st < ns->nsteps ? ns->radix[st] : ns->red_radix[st - ns->nsteps];
}

/* base of buffer `buf` of node rank `l` in this process (0 but in the NODE form over several nodes) */
static char *leg_base_of(const emac_handle *h, int buf, int l) {
  return buf == EMAC_BUF_SEND ? (char *)h->dsend[l]
       : buf == EMAC_BUF_RECV ? (char *)h->drecv[l]
                              : (char *)h->staging + (long)l * h->stage_stride;
}

static char *leg_base(const emac_handle *h, int buf) { return leg_base_of(h, buf, 0); }

/* ------------------------- NODE form over several nodes ------------------------- */

/* The node's copy-out (its allgather): every owner chunk, from its owner's receive buffer, stored
   into the R - 1 other receive buffers (one emac_gpu_copy_fan launch). `b`: scratch of npieces * R
   buckets. */
static int build_node_fanout(emac_handle *h, emac_bucket *b) {
  const int R = h->plan.nranks;
  emac_edge *edges = NULL;
  emac_launch *F = &h->fanout;
  int nfb = 0, pc, c, r, rc;
  if (R < 2) return 0;
  for (pc = 0; pc < h->plan.npieces; pc++)
    for (c = 0; c < R; c++) {
      const long off = h->plan.chunk_off[(size_t)pc * R + c], len = h->plan.chunk_len[(size_t)pc * R + c];
      const int owner = h->plan.pos_rank[c];
      emac_bucket *bk = &b[nfb];
      if (len <= 0) continue;
      memset(bk, 0, sizeof(*bk));
      bk->src[0] = h->drecv[owner];
      for (r = 0; r < R; r++)
        if (r != owner) bk->dst[bk->ndst++] = h->drecv[r];
      place_bucket(bk, 1, off, len, h->plan.tsize);
      nfb++;
    }
  if ((rc = emac_layout(b, nfb, EMAC_SUM, 1, 0, 0, &edges, &F->nedges, &F->ntiles, &F->tiles_per_bucket, &F->all_full,
                        &F->unroll)))
    return rc;
  F->nb = nfb;
  if (nfb && (rc = emac_gpu_malloc((void **)&F->d_buckets, sizeof(emac_bucket) * (size_t)nfb)) == 0)
    rc = emac_gpu_memcpy(F->d_buckets, b, sizeof(emac_bucket) * (size_t)nfb);
  if (!rc && F->nedges && (rc = emac_gpu_malloc((void **)&F->d_edges, sizeof(emac_edge) * (size_t)F->nedges)) == 0)
    rc = emac_gpu_memcpy(F->d_edges, edges, sizeof(emac_edge) * (size_t)F->nedges);
  free(edges);
  return rc;
}

/* a launch of `nsrc`-leaf buckets under the schedule of fan-out form `fan` (2: peer-mapped) */
static int upload_launch_fan(const emac_handle *h, emac_launch *L, emac_bucket *b, int nb, int nsrc, int fan) {
  emac_edge *edges = NULL;
  int rc;
  if ((rc = emac_layout(b, nb, nsrc > 1 ? h->plan.op : EMAC_SUM, nsrc, 0, fan, &edges, &L->nedges, &L->ntiles,
                        &L->tiles_per_bucket, &L->all_full, &L->unroll)))
    return rc;
  L->nb = nb;
  if (nb && (rc = emac_gpu_malloc((void **)&L->d_buckets, sizeof(emac_bucket) * (size_t)nb)) == 0)
    rc = emac_gpu_memcpy(L->d_buckets, b, sizeof(emac_bucket) * (size_t)nb);
  if (!rc && L->nedges && (rc = emac_gpu_malloc((void **)&L->d_edges, sizeof(emac_edge) * (size_t)L->nedges)) == 0)
    rc = emac_gpu_memcpy(L->d_edges, edges, sizeof(emac_edge) * (size_t)L->nedges);
  free(edges);
  return rc;
}

/* The fold tree of a share of the peer-mapped node join over n partials: a left fold (levels 1),
   or `levels` levels of pairs (the halving flow) -- the shape of a '6;1 -2 ... 2 ...' plan */
static int node_fold_codes(int n, int levels, int dtype, emac_codes *c) {
  emac_copyin cfg;
  emac_plan p;
  char cp[96];
  int at, k, rc;
  memset(c, 0, sizeof(*c));
  if (levels <= 1) {
    c->first[0] = 1;
    c->close[n - 1] = 1;
    c->nlev = 1;
    c->nleaf = n;
    return 0;
  }
  at = snprintf(cp, sizeof(cp), "6;1");
  for (k = 0; k < levels; k++) at += snprintf(cp + at, sizeof(cp) - (size_t)at, " -2");
  for (k = 0; k < levels; k++) at += snprintf(cp + at, sizeof(cp) - (size_t)at, " 2");
  if ((rc = emac_parse_copyin(cp, &cfg))) return rc;
  cfg.sockets = 1;
  if ((rc = emac_plan_build(&p, n, (long)n * 16, dtype, EMAC_SUM, &cfg))) return rc;
  *c = p.codes;
  emac_plan_free(&p);
  return 0;
}

/* The NODE form over peer-mapped nodes: node_comm_allreduce_init on an ext_mpi_amd_comm_init_ipc
   communicator -- one process per GPU, each member a node of R ranks whose buffers all live on
   its GPU. The inter-node schedule must be one reduce-scatter step over every node (EXT_MPI_NUM_PORTS
   'N(-(N-1) (N-1))', the default for a node count that is not a power of two) -- every element's
   value is then ONE fold of the N node partials in its line's order, whoever computes it -- or,
   for SUM, one port per step over 2^k nodes (the default there) -- every value a balanced tree of
   pairs over the task bits (plan.c emac_node_single, emac_node_shares): so the inter-node legs
   become peer loads instead of point-to-point lines. A Start runs
    1. the node's copy-in: every owner chunk folded over the node's send buffers, in the plan's leaf
       order, into this node's partial block (arena memory the peers map; fold_launch, tuned);
    2. barrier(in); the fold of this node's share of every node rank's chunk: the N nodes' partials
       read in place (system-coherent loads over xGMI), in the line's order, into this node's outbox
       (arena); barrier(out) -- the IPC form's protocol (ipc_sync.hpp, epochs, timeout recovery);
    3. the pull fused with the copy-out: every node's share (this node's own too) read once from
       its outbox and stored into all R receive buffers (emac_gpu_copy_fan_remote), the nodes
       after this one first.
   No caller memory is exported -- the peers read only the two arena blocks -- so the handle's Done
   is local. Collective over the communicator (the exchanges run whatever failed locally). */
static int node_ipc_init(emac_handle *h, emac_comm *cm, int rc) {
  typedef struct {
    long lack;
    int status;
    int seg[2];
    long offset[2];
    unsigned char free_slots[EMAC_SYNC_SLOTS / 8];
  } nx_export;
  nx_export mine, all[EMAC_MAX_RANKS];
  void *peer_part[EMAC_MAX_RANKS], *peer_out[EMAC_MAX_RANKS];
  emac_share *sh[EMAC_MAX_RANKS] = {0};
  int nsh[EMAC_MAX_RANKS] = {0};
  emac_bucket *b = NULL;
  const int N = cm->size, R = h->plan.nranks;
  const long ts = h->plan.tsize;
  int attempt, r, k, me, i, slot, nb, pc;
  h->part_bytes = h->outbox_bytes = h->bytes > 16 ? h->bytes : 16;
  for (attempt = 0;; attempt++) {
    long lack = 0;
    int grow = 0;
    if (!rc && !h->part && arena_alloc(cm, (long)h->part_bytes, &h->part))
      lack += (long)(h->part_bytes + EMAC_ARENA_ALIGN - 1) / EMAC_ARENA_ALIGN * EMAC_ARENA_ALIGN;
    if (!rc && !h->outbox && arena_alloc(cm, (long)h->outbox_bytes, &h->outbox))
      lack += (long)(h->outbox_bytes + EMAC_ARENA_ALIGN - 1) / EMAC_ARENA_ALIGN * EMAC_ARENA_ALIGN;
    memset(&mine, 0, sizeof(mine));
    for (k = 0; !rc && !lack && k < 2; k++) {
      void *p = k ? h->outbox : h->part;
      int sg;
      if (!arena_owns(cm, p, &sg)) {
        rc = EMAC_ERR_ARG;
      } else {
        mine.seg[k] = sg;
        mine.offset[k] = (long)((char *)p - (char *)cm->seg[sg].base);
      }
    }
    mine.lack = rc ? 0 : lack;
    mine.status = rc == 0;
    for (r = 0; r < EMAC_SYNC_SLOTS; r++)
      if (!cm->slot_used[r]) mine.free_slots[r >> 3] |= (unsigned char)(1u << (r & 7));
    if (cm->ag(cm->ag_ctx, &mine, all, (long)sizeof(mine))) return EMAC_ERR_TRANSPORT;
    for (r = 0; r < N; r++) {
      if (!all[r].status && !rc) rc = EMAC_ERR_TRANSPORT;
      if (all[r].lack > 0) grow = 1;
    }
    if (rc) return rc; /* the same verdict on every rank */
    if (!grow) break;
    if (attempt == EMAC_IPC_ATTEMPTS - 1) return EMAC_ERR_MALLOC;
    if ((rc = arena_grow(cm, 0, lack))) return rc;
  }
  for (r = 0; r < N; r++) {
    if (r == cm->rank) {
      peer_part[r] = h->part;
      peer_out[r] = h->outbox;
      continue;
    }
    peer_part[r] = all[r].seg[0] < cm->peer_nseg[r] ? (char *)cm->peer_seg[r][all[r].seg[0]] + all[r].offset[0] : NULL;
    peer_out[r] = all[r].seg[1] < cm->peer_nseg[r] ? (char *)cm->peer_seg[r][all[r].seg[1]] + all[r].offset[1] : NULL;
    if (!peer_part[r] || !peer_out[r]) rc = EMAC_ERR_TRANSPORT;
  }
  if ((rc = ipc_agree(cm, rc == 0))) return rc;
  for (slot = 0; slot < EMAC_SYNC_SLOTS; slot++) { /* the lowest slot free on every rank */
    for (r = 0; r < N && (all[r].free_slots[slot >> 3] >> (slot & 7)) & 1; r++);
    if (r == N) break;
  }
  if (slot == EMAC_SYNC_SLOTS) return EMAC_ERR_MALLOC; /* the same verdict on every rank */
  h->slot = slot;
  cm->slot_used[slot] = 1;
  h->slot_held = 1;
  cm->err[slot] = 0;
  {
    const char *e = getenv("EXT_MPI_AMD_IPC_RELEASE"); /* as ipc_allreduce_init */
    const int rel = e ? atoi(e) > 0 : cm->cross_device;
    if (N > 1 && rel && (rc = emac_gpu_event_create_release(&h->ev_release))) return rc;
  }
  h->epoch[0] = cm->slot_epoch[slot][0];
  h->epoch[1] = cm->slot_epoch[slot][1];
  /* the parts of every node rank's chunk (plan.c emac_node_shares; one node: the chunk itself) */
  for (me = 0; me < R && !rc; me++) {
    if (N > 1) {
      rc = emac_node_shares(&h->plan, &h->ns, me, &sh[me], &nsh[me]);
    } else if (!(sh[me] = (emac_share *)calloc((size_t)h->plan.npieces + 1, sizeof(emac_share)))) {
      rc = EMAC_ERR_MALLOC;
    } else {
      for (pc = 0; pc < h->plan.npieces; pc++) {
        emac_share *x = &sh[me][nsh[me]++];
        x->off = h->plan.chunk_off[(size_t)pc * R + h->plan.rank_pos[me]];
        x->len = h->plan.chunk_len[(size_t)pc * R + h->plan.rank_pos[me]];
        x->node = 0;
        x->nleaf = 1;
      }
    }
  }
  for (me = 0, k = 0; me < R; me++) k += nsh[me];
  if (!rc) /* the halving flow folds log2 N levels of pairs, one step over every node a left fold */
    rc = node_fold_codes(N, N > 1 && emac_node_single(&h->ns) == 2 ? h->ns.nsteps : 1, h->plan.dtype, &h->xcodes);
  if (!rc && !(b = (emac_bucket *)calloc((size_t)(k + h->plan.npieces * R) + 1, sizeof(emac_bucket)))) rc = EMAC_ERR_MALLOC;
  /* 1. the copy-in: every owner chunk into this node's partial block (at its message offset) */
  for (nb = 0, pc = 0; !rc && pc < h->plan.npieces; pc++)
    for (i = 0; i < R; i++) {
      const long off = h->plan.chunk_off[(size_t)pc * R + i], len = h->plan.chunk_len[(size_t)pc * R + i];
      emac_bucket *bk = &b[nb];
      int t;
      if (len <= 0) continue;
      memset(bk, 0, sizeof(*bk));
      for (t = 0; t < R; t++) bk->src[t] = h->dsend[h->plan.leaf_rank[i][t]];
      bk->dst[0] = h->part;
      bk->ndst = 1;
      place_bucket(bk, R, off, len, ts);
      nb++;
    }
  h->nsrc = R;
  h->fan = 0;
  if (!rc) rc = upload_buckets(h, b, nb);
  /* 2. this node's shares: the N partials in place, in the line's order, into the outbox */
  for (nb = 0, me = 0; !rc && me < R; me++)
    for (i = 0; i < nsh[me]; i++) {
      const emac_share *x = &sh[me][i];
      emac_bucket *bk = &b[nb];
      int l;
      if (x->node != cm->rank || x->len <= 0) continue;
      memset(bk, 0, sizeof(*bk));
      for (l = 0; l < x->nleaf; l++) bk->src[l] = peer_part[x->leaf_node[l]]; /* in h->xcodes' order */
      bk->dst[0] = h->outbox;
      bk->ndst = 1;
      place_bucket(bk, x->nleaf, x->off, x->len, ts);
      nb++;
    }
  if (!rc) rc = upload_launch_fan(h, &h->xfold[0], b, nb, N, 2);
  /* 3. the pull, fused with the copy-out: every share read once from its node's outbox and stored
     into all R receive buffers, the nodes after this one first (their loads head for different
     GPUs' links), this node's own last */
  for (nb = 0, k = 1; !rc && k <= N; k++) {
    const int q = (cm->rank + k) % N;
    for (me = 0; me < R; me++)
      for (i = 0; i < nsh[me]; i++) {
        const emac_share *x = &sh[me][i];
        emac_bucket *bk = &b[nb];
        int d;
        if (x->node != q || x->len <= 0) continue;
        memset(bk, 0, sizeof(*bk));
        bk->src[0] = peer_out[q];
        for (d = 0; d < R; d++) bk->dst[d] = h->drecv[d];
        bk->ndst = R;
        place_bucket(bk, 1, x->off, x->len, ts);
        nb++;
      }
  }
  if (!rc) rc = upload_launch_fan(h, &h->pull, b, nb, 1, 2);
  for (me = 0; me < R; me++) free(sh[me]);
  free(b);
  return rc;
}

/* Every rank of this node in this process (the NODE form: all their buffers on this GPU), the
   nodes joined by `comm`, whose members are the nodes (RCCL, or loopback for testing), under the
   communicator's inter-node schedule (ext_mpi_amd_comm_set_node_ports with nodes == its size;
   otherwise emac_node_sched_build's default). A Start runs
    1. the node's copy-in: every owner chunk folded over the node's send buffers, in the plan's
       leaf order, into its owner's receive buffer -- the COMM form's reduce-scatter leg and fold
       without moving a byte, the leaves read where they lie (one launch, fold_launch);
    2. the node legs of every node rank me (emac_comm_program_nodes of global rank
       node * R + me; its column peers are rank me of the other nodes, i.e. the other members),
       one RCCL group per leg for all node ranks, ordered by node rank within each peer so that
       the k-th send of a pair matches its k-th receive, and each exchange step's fold for all
       node ranks in one launch;
    3. the copy-out: every owner chunk stored into the node's other receive buffers (the node
       allgather, emac_gpu_copy_fan).
   The bits are the COMM form's over nodes * R ranks, one per process -- the reference's
   multi-node composition (ext_mpi_native.c:879-1000: reduce_copyin over the node, the
   EXT_MPI_NUM_PORTS schedule between nodes, reduce_copyout). */
int ext_mpi_amd_node_comm_allreduce_init(int nranks, const void *const *sendbufs, void *const *recvbufs, long count,
                                         int dtype, int op, int comm, const char *copyin, int *handle) {
  emac_handle *h;
  emac_comm *cm;
  emac_copyin cfg;
  emac_bucket *b = NULL, *xb = NULL;
  emac_p2p *prog_ops[EMAC_MAX_RANKS] = {0};
  emac_fold *prog_folds[EMAC_MAX_RANKS] = {0};
  int prog_nops[EMAC_MAX_RANKS] = {0}, prog_nf[EMAC_MAX_RANKS] = {0};
  int nxb[2 * EMAC_MAX_NODE_STEPS] = {0};
  const int R = nranks;
  int rc, r, me, i, t, pc, c, nb = 0, nsteps, nf_all = 0, no_all = 0;
  long stage_max = 0;
  if (!handle || !sendbufs || !recvbufs || R < 1 || R > EMAC_MAX_RANKS || count < 0 || comm < 0 ||
      comm >= MAX_COMMS || !comms[comm].used)
    return EMAC_ERR_ARG;
  *handle = -1;
  cm = &comms[comm];
  if (cm->nodes > 1 && cm->nodes != cm->size) return EMAC_ERR_ARG; /* the members are the nodes */
  if ((rc = parse_cfg(copyin, R, &cfg))) return rc;
  if (emac_gpu_set_device(cm->device)) return EMAC_ERR_DEVICE;
  h = (emac_handle *)calloc(1, sizeof(emac_handle));
  if (!h) return EMAC_ERR_MALLOC;
  h->kind = KIND_COMM;
  h->hier = 1;
  h->comm = comm;
  h->device = cm->device;
  if ((rc = emac_plan_build(&h->plan, R, count, dtype, op, &cfg))) goto fail;
  h->me = cm->rank; /* this node */
  h->bytes = (size_t)count * (size_t)h->plan.tsize;
  h->nodes = cm->size;
  if (h->nodes > 1 && cm->nodes == cm->size)
    h->ns = cm->ns; /* ext_mpi_amd_comm_set_node_ports */
  else if (h->nodes > 1 && (rc = emac_node_sched_build(&h->ns, h->nodes, NULL)))
    goto fail;
  h->nbuf = R;
  h->nsrc = R;
  h->fan = 0;
  if (cm->ipc) { /* peer-mapped nodes: collective from here on, whatever fails locally */
    const int single = h->nodes > 1 ? emac_node_single(&h->ns) : 1;
    if (!single || (single == 2 && op != EMAC_SUM)) rc = EMAC_ERR_UNSUPPORTED; /* (the same on every rank) */
    for (r = 0; r < R && !rc; r++) rc = map_buffers(h, r, sendbufs[r], recvbufs[r]); /* local: device mirrors */
    h->kind = KIND_IPC;
    if ((rc = node_ipc_init(h, cm, rc))) goto fail;
    if ((rc = emac_gpu_stream_create(&h->stream))) goto fail;
    if ((rc = finish_init(h, handle))) goto fail;
    return 0;
  }
  for (r = 0; r < R; r++)
    if ((rc = map_buffers(h, r, sendbufs[r], recvbufs[r]))) goto fail;
  /* 1. the copy-in: owner chunk (piece pc, position c) into its owner's receive buffer */
  b = (emac_bucket *)calloc((size_t)h->plan.npieces * R + 1, sizeof(emac_bucket));
  if (!b) {
    rc = EMAC_ERR_MALLOC;
    goto fail;
  }
  for (pc = 0; pc < h->plan.npieces; pc++)
    for (c = 0; c < R; c++) {
      const long off = h->plan.chunk_off[(size_t)pc * R + c], len = h->plan.chunk_len[(size_t)pc * R + c];
      emac_bucket *bk = &b[nb];
      if (len <= 0) continue;
      memset(bk, 0, sizeof(*bk));
      for (t = 0; t < R; t++) bk->src[t] = h->dsend[h->plan.leaf_rank[c][t]];
      bk->dst[0] = h->drecv[h->plan.pos_rank[c]];
      bk->ndst = 1;
      place_bucket(bk, R, off, len, h->plan.tsize);
      nb++;
    }
  if ((rc = upload_buckets(h, b, nb))) goto fail;
  /* 3. the copy-out: owner chunk into the R - 1 other receive buffers */
  if ((rc = build_node_fanout(h, b))) goto fail;
  /* 2. the node legs of every node rank: their programs, the peers turned into members */
  nsteps = h->nodes > 1 ? h->ns.nsteps + h->ns.nred : 0;
  for (me = 0; me < R && h->nodes > 1; me++) {
    long st = 0;
    if ((rc = emac_comm_program_nodes(&h->plan, &h->ns, h->me, me, (long)((unsigned long)h->dsend[me] & 15ul),
                                      &prog_ops[me], &prog_nops[me], &prog_folds[me], &prog_nf[me], &st)))
      goto fail;
    if (st > stage_max) stage_max = st;
    no_all += prog_nops[me];
    nf_all += prog_nf[me];
  }
  h->stage_stride = (stage_max + 255) / 256 * 256;
  if ((rc = emac_gpu_malloc(&h->staging, (size_t)(h->stage_stride > 0 ? h->stage_stride * R : 16)))) goto fail;
  h->ops = (emac_p2p *)malloc(sizeof(emac_p2p) * (size_t)(no_all + 1));
  xb = (emac_bucket *)calloc(2 * EMAC_MAX_NODE_STEPS * ((size_t)nf_all + 1), sizeof(emac_bucket));
  if (!h->ops || !xb) {
    rc = EMAC_ERR_MALLOC;
    goto fail;
  }
  /* legs in program order, node ranks in ascending order inside each (the pairs' matching order) */
  for (me = 0; me < R; me++)
    for (i = 0; i < prog_nops[me]; i++) {
      emac_p2p o = prog_ops[me][i];
      const int base = o.leg & ((1 << EMAC_LEG_STEP_SHIFT) - 1);
      if (base != EMAC_LEG_NODES_RS && base != EMAC_LEG_NODES_AG) continue; /* the node's own legs: steps 1, 3 */
      if (o.peer % R != me) {
        rc = EMAC_ERR_UNSUPPORTED; /* not a program of this shape */
        goto fail;
      }
      o.peer /= R;
      o.local = me;
      h->ops[h->nops++] = o;
    }
  for (me = 0; me < R; me++)
    for (i = 0; i < prog_nf[me]; i++) {
      const emac_fold *f = &prog_folds[me][i];
      int step;
      emac_bucket *bk;
      if ((f->leg & ((1 << EMAC_LEG_STEP_SHIFT) - 1)) != EMAC_LEG_NODES_FOLD) continue; /* step 1 folds the node */
      step = f->leg >> EMAC_LEG_STEP_SHIFT;
      if (step < 0 || step >= nsteps) {
        rc = EMAC_ERR_UNSUPPORTED; /* not a program of this shape */
        goto fail;
      }
      bk = &xb[(size_t)step * ((size_t)nf_all + 1) + (size_t)nxb[step]++];
      for (t = 0; t < f->nleaf; t++) bk->src[t] = leg_base_of(h, f->buf[t], me) + f->loff[t] - f->offset;
      bk->dst[0] = h->drecv[me];
      bk->ndst = 1;
      place_bucket(bk, f->nleaf, f->offset / h->plan.tsize, f->count, h->plan.tsize);
    }
  for (i = 0; i < nsteps; i++)
    if (nxb[i] &&
        (rc = upload_launch_as(h, &h->xfold[i], xb + (size_t)i * ((size_t)nf_all + 1), nxb[i], node_radix(&h->ns, i), 0)))
      goto fail;
  if ((rc = emac_gpu_stream_create(&h->stream))) goto fail;
  if (cm->loop_group >= 0) {
    loop_group *g = &loops[cm->loop_group];
    if (g->nh[h->me] < 0 || g->nh[h->me] >= MAX_LOOP_HANDLES) {
      rc = EMAC_ERR_MALLOC;
      goto fail;
    }
    h->loop_index = g->nh[h->me];
  }
  if ((rc = finish_init(h, handle))) goto fail;
  if (cm->loop_group >= 0) loops[cm->loop_group].handle[h->me][loops[cm->loop_group].nh[h->me]++] = *handle;
  rc = 0;
  goto out;
fail:
  release(h);
out:
  for (me = 0; me < R; me++) {
    free(prog_ops[me]);
    free(prog_folds[me]);
  }
  free(b);
  free(xb);
  return rc;
}

static emac_handle *get(int handle);

/* Loopback transport: every receive of this leg copies the matching send of the peer (the
   k-th send of q to me in this leg matches my k-th receive from q). */
static int run_leg_loopback(emac_handle *h, int leg) {
  loop_group *g = &loops[comms[h->comm].loop_group];
  int seen[EMAC_MAX_RANKS][EMAC_MAX_RANKS], i, j, rc;
  memset(seen, 0, sizeof(seen));
  for (i = 0; i < h->nops; i++) {
    const emac_p2p *o = &h->ops[i];
    emac_handle *hq;
    int q = o->peer, k, found = 0;
    if (o->leg != leg || o->is_send) continue;
    k = seen[q][o->local]++; /* per (peer, node rank): the NODE form over nodes orders them so */
    if (h->loop_index >= g->nh[q]) return EMAC_ERR_TRANSPORT; /* peer has no matching handle */
    hq = get(g->handle[q][h->loop_index]);
    if (!hq) return EMAC_ERR_TRANSPORT;
    for (j = 0; j < hq->nops; j++) {
      const emac_p2p *so = &hq->ops[j];
      if (so->leg == leg && so->is_send && so->peer == h->me && so->local == o->local && k-- == 0) {
        if (so->bytes != o->bytes) return EMAC_ERR_TRANSPORT;
        if ((rc = emac_gpu_memcpy_async(leg_base_of(h, o->buf, o->local) + o->offset,
                                        leg_base_of(hq, so->buf, so->local) + so->offset, (size_t)o->bytes, h->stream)))
          return rc;
        found = 1;
        break;
      }
    }
    if (!found) return EMAC_ERR_TRANSPORT;
  }
  return 0;
}

/* Walk the point-to-point program of one leg as ONE RCCL group (all peers at once). */
static int run_leg(emac_handle *h, int leg) {
  emac_comm *cm = &comms[h->comm];
  hipStream_t s = (hipStream_t)h->stream;
  int i, bad = 0;
  if (cm->loop_group >= 0) return run_leg_loopback(h, leg);
  if (ncclGroupStart() != ncclSuccess) return EMAC_ERR_TRANSPORT;
  for (i = 0; i < h->nops && !bad; i++) {
    const emac_p2p *o = &h->ops[i];
    char *base;
    if (o->leg != leg) continue;
    base = leg_base_of(h, o->buf, o->local);
    if (o->is_send)
      bad = ncclSend(base + o->offset, (size_t)o->bytes, ncclInt8, o->peer, cm->nccl, s) != ncclSuccess;
    else
      bad = ncclRecv(base + o->offset, (size_t)o->bytes, ncclInt8, o->peer, cm->nccl, s) != ncclSuccess;
  }
  if (ncclGroupEnd() != ncclSuccess) bad = 1;
  return bad ? EMAC_ERR_TRANSPORT : 0;
}

static int stage_in(emac_handle *h) {
  int r, rc;
  for (r = 0; r < h->nbuf; r++) {
    void *src = h->send_mirror[r] ? h->user_send[r] : (h->recv_mirror[r] && h->dsend[r] == h->drecv[r] ? h->user_recv[r] : NULL);
    if (src && (rc = emac_gpu_memcpy_async(h->dsend[r], src, h->bytes, h->stream))) return rc;
  }
  return 0;
}

static int stage_out(emac_handle *h) {
  int r, rc;
  for (r = 0; r < h->nbuf; r++)
    if (h->recv_mirror[r] && (rc = emac_gpu_memcpy_async(h->user_recv[r], h->drecv[r], h->bytes, h->stream)))
      return rc;
  return 0;
}

static emac_handle *get(int handle) {
  if (handle < 0 || handle >= MAX_HANDLES) return NULL;
  return handles[handle];
}

static unsigned *ipc_go(const emac_handle *h) {
  return (unsigned *)((char *)comms[h->comm].sync + offsetof(emac_sync, go)) + h->slot;
}

/* IPC form: node barrier `phase` (0 before the fold: every rank's send buffer is ready and its
   receive buffer free; 1 after it: every fan-out store has landed) on the handle's stream. The
   Start is named by its phase-1 epoch (`tag`, ipc_sync.hpp). Phase 0 is preceded by a
   system-scope release of everything enqueued before it, done by the command processor on every
   XCD: the peers' loads of this rank's buffers do not depend on where its writers ran. */
static int ipc_barrier(emac_handle *h, int phase) {
  emac_comm *cm = &comms[h->comm];
  int rc;
  unsigned long epoch, tag;
  if (phase == 0 && h->ev_release && (rc = emac_gpu_event_record(h->ev_release, h->stream))) return rc;
  epoch = ++h->epoch[phase];
  tag = phase ? epoch : h->epoch[1] + 1;
  return emac_gpu_node_barrier(cm->sync, (void *const *)cm->d_peer_sync, h->slot, phase, epoch, tag, cm->size, cm->rank,
                               cm->err + h->slot, cm->timeout_ticks, h->stream);
}

/* barrier errors are reported through the slot's pinned word (ipc_sync.hpp), read and cleared
   when the Start is waited for: the next Start on the handle synchronises normally */
static int ipc_status(const emac_handle *h) {
  volatile int *w;
  int e;
  if (h->kind != KIND_IPC || !h->slot_held) return 0;
  w = (volatile int *)comms[h->comm].err + h->slot;
  e = *w;
  if (!e) return 0;
  *w = 0;
  fprintf(stderr, "ext_mpi_amd: rank %d: node barrier failed:%s%s\n", comms[h->comm].rank,
          (e & EMAC_SYNC_ERR_TIMEOUT) ? " a peer did not arrive within EXT_MPI_AMD_BARRIER_TIMEOUT" : "",
          (e & EMAC_SYNC_ERR_ABORTED) ? " a peer gave up on this Allreduce" : "");
  return EMAC_ERR_TRANSPORT;
}

/* A pipelined NODE Start: H2D of every part on s_in, the part's fold on the handle's stream
   after its copies, its D2H on s_out after its fold; the handle's stream then waits for the
   last D2H, so Wait / Test and the next Start see the whole Allreduce. */
static int pipe_start(emac_handle *h) {
  emac_pipe *pp = h->pipe;
  const size_t ts = (size_t)h->plan.tsize;
  int p, r, rc;
  /* the caller's earlier work on the handle's stream (and the previous Start) comes first */
  if ((rc = emac_gpu_event_record(pp->ev_start, h->stream)) || (rc = emac_gpu_stream_wait(pp->s_in, pp->ev_start)))
    return rc;
  for (p = 0; p < pp->nparts; p++) {
    const size_t o = (size_t)pp->off[p] * ts, n = (size_t)(pp->off[p + 1] - pp->off[p]) * ts;
    for (r = 0; r < h->nbuf && n; r++) {
      const void *src = h->send_mirror[r] ? h->user_send[r]
                                          : (h->recv_mirror[r] && h->dsend[r] == h->drecv[r] ? h->user_recv[r] : NULL);
      if (src && (rc = emac_gpu_memcpy_async((char *)h->dsend[r] + o, (const char *)src + o, n, pp->s_in))) return rc;
    }
    if ((rc = emac_gpu_event_record(pp->ev_in[p], pp->s_in))) return rc;
  }
  for (p = 0; p < pp->nparts; p++) {
    const emac_launch *L = &pp->part[p];
    if ((rc = emac_gpu_stream_wait(h->stream, pp->ev_in[p]))) return rc;
    if ((rc = emac_gpu_fold(h->plan.dtype, h->plan.op, h->nsrc, h->fan, L->unroll, &h->plan.codes, L->d_buckets, L->nb,
                            L->ntiles, L->tiles_per_bucket, L->all_full, L->d_edges, L->nedges, h->stream)))
      return rc;
    if ((rc = emac_gpu_event_record(pp->ev_fold[p], h->stream))) return rc;
  }
  for (p = 0; p < pp->nparts; p++) {
    const size_t o = (size_t)pp->off[p] * ts, n = (size_t)(pp->off[p + 1] - pp->off[p]) * ts;
    if ((rc = emac_gpu_stream_wait(pp->s_out, pp->ev_fold[p]))) return rc;
    for (r = 0; r < h->nbuf && n; r++)
      if (h->recv_mirror[r] &&
          (rc = emac_gpu_memcpy_async((char *)h->user_recv[r] + o, (const char *)h->drecv[r] + o, n, pp->s_out)))
        return rc;
  }
  if ((rc = emac_gpu_event_record(pp->ev_done, pp->s_out)) || (rc = emac_gpu_stream_wait(h->stream, pp->ev_done)))
    return rc;
  h->started = 1;
  return 0;
}

/* Everything a Start (or a subset of its legs) enqueues on the handle's stream. */
static int enqueue_legs(emac_handle *h, int legs) {
  int rc, multi;
  const int core = EXT_MPI_AMD_LEG_REDUCE_SCATTER | EXT_MPI_AMD_LEG_FOLD | EXT_MPI_AMD_LEG_ALLGATHER;
  multi = h->kind == KIND_COMM && h->plan.nranks > 1 && !h->hier; /* the node's own p2p legs */
  if ((legs & EXT_MPI_AMD_LEG_STAGE_IN) && (rc = stage_in(h))) return rc;
  if (h->kind == KIND_IPC && h->hier) { /* the NODE form over peer-mapped nodes (node_ipc_init) */
    const int nodes = comms[h->comm].size;
    if ((legs & EXT_MPI_AMD_LEG_FOLD) && (rc = fold_launch(h))) return rc; /* the copy-in */
    if (legs & (EXT_MPI_AMD_LEG_NODES_RS | EXT_MPI_AMD_LEG_NODES_FOLD | EXT_MPI_AMD_LEG_NODES_AG)) {
      const emac_launch *X = &h->xfold[0];
      if ((rc = ipc_barrier(h, 0))) return rc;
      if ((X->nb || X->nedges) &&
          (rc = emac_gpu_fold_remote(h->plan.dtype, nodes > 1 ? h->plan.op : EMAC_SUM, nodes, X->unroll, &h->xcodes,
                                     X->d_buckets, X->nb, X->ntiles, X->tiles_per_bucket, X->all_full, X->d_edges,
                                     X->nedges, ipc_go(h), h->stream)))
        return rc;
      if ((rc = ipc_barrier(h, 1))) return rc;
      if ((h->pull.nb || h->pull.nedges) &&
          (rc = emac_gpu_copy_fan_remote(h->plan.tsize, h->plan.nranks, h->pull.unroll, h->pull.d_buckets, h->pull.nb,
                                         h->pull.ntiles, h->pull.tiles_per_bucket, h->pull.all_full, h->pull.d_edges,
                                         h->pull.nedges, ipc_go(h), h->stream)))
        return rc;
    }
    if ((legs & EXT_MPI_AMD_LEG_ALLGATHER) && h->fanout.nb &&
        (rc = emac_gpu_copy_fan(h->plan.tsize, h->plan.nranks - 1, h->fanout.unroll, h->fanout.d_buckets, h->fanout.nb,
                                h->fanout.ntiles, h->fanout.tiles_per_bucket, h->fanout.all_full, h->fanout.d_edges,
                                h->fanout.nedges, h->stream)))
      return rc;
    if ((legs & EXT_MPI_AMD_LEG_STAGE_OUT) && (rc = stage_out(h))) return rc;
    return 0;
  }
  if (h->kind == KIND_IPC && h->fused && (legs & core) == core) {
    emac_comm *cm = &comms[h->comm];
    unsigned long e0, e1;
    if (h->ev_release && (rc = emac_gpu_event_record(h->ev_release, h->stream))) return rc; /* as ipc_barrier(h, 0) */
    e0 = ++h->epoch[0];
    e1 = ++h->epoch[1];
    if ((rc = emac_gpu_fold_fused(h->plan.dtype, h->plan.op, h->nsrc, h->unroll, &h->plan.codes, h->d_buckets, h->nb, h->ntiles,
                                  h->tiles_per_bucket, h->all_full, h->d_edges, h->nedges, h->pull.d_buckets, h->pull.nb,
                                  h->pull.ntiles, h->pull.tiles_per_bucket, h->pull.all_full, h->pull.d_edges,
                                  h->pull.nedges, cm->sync,
                                  (void *const *)cm->d_peer_sync, h->slot, cm->size, cm->rank, cm->err + h->slot,
                                  cm->timeout_ticks, e0, e1, h->stream)))
      return rc;
    if ((legs & EXT_MPI_AMD_LEG_STAGE_OUT) && (rc = stage_out(h))) return rc;
    return 0;
  }
  if ((legs & EXT_MPI_AMD_LEG_REDUCE_SCATTER) && h->kind == KIND_IPC && h->plan.nranks > 1 &&
      (rc = ipc_barrier(h, 0)))
    return rc;
  if ((legs & EXT_MPI_AMD_LEG_REDUCE_SCATTER) && multi && (rc = run_leg(h, EMAC_LEG_RS))) return rc;
  if ((legs & EXT_MPI_AMD_LEG_FOLD) && h->fan == 2 &&
      (rc = emac_gpu_fold_remote(h->plan.dtype, h->plan.op, h->nsrc, h->unroll, &h->plan.codes, h->d_buckets, h->nb,
                                 h->ntiles, h->tiles_per_bucket, h->all_full, h->d_edges, h->nedges, ipc_go(h), h->stream)))
    return rc;
  if ((legs & EXT_MPI_AMD_LEG_FOLD) && h->fan != 2 && (rc = fold_launch(h))) return rc;
  if (h->kind == KIND_COMM && h->nodes > 1) {
    /* several nodes: per step the exchange of the lines with the column peers and the fold of
       the kept lines' partials (a left fold of radix leaves in the order the program lists
       them), then the exchanges back in reverse step order (emac_comm_program_nodes). A step
       selector in the legs' high bits (EXT_MPI_AMD_LEG_STEP) runs that step's legs alone. */
    int st;
    const int nsteps = h->ns.nsteps + h->ns.nred, only = (legs >> EMAC_LEG_STEP_SHIFT) & 31;
    for (st = 0; st < nsteps; st++) {
      const emac_launch *X = &h->xfold[st];
      const int rad = node_radix(&h->ns, st);
      emac_codes lin;
      memset(&lin, 0, sizeof(lin));
      lin.first[0] = 1; /* one level: a left fold */
      lin.close[rad - 1] = 1;
      lin.nlev = 1;
      lin.nleaf = rad;
      if (only && st != only - 1) continue;
      if ((legs & EXT_MPI_AMD_LEG_NODES_RS) && (rc = run_leg(h, EMAC_LEG_NODES_RS | st << EMAC_LEG_STEP_SHIFT)))
        return rc;
      if ((legs & EXT_MPI_AMD_LEG_NODES_FOLD) && X->nb &&
          (rc = emac_gpu_fold(h->plan.dtype, h->plan.op, rad, 0, X->unroll, &lin, X->d_buckets, X->nb,
                              X->ntiles, X->tiles_per_bucket, X->all_full, X->d_edges, X->nedges, h->stream)))
        return rc;
    }
    for (st = 0; st < h->ns.nagp; st++) { /* the copying allgather steps, block growing */
      if (only && st != only - 1) continue;
      if ((legs & EXT_MPI_AMD_LEG_NODES_AG) && (rc = run_leg(h, EMAC_LEG_NODES_AG | st << EMAC_LEG_STEP_SHIFT)))
        return rc;
    }
  }
  if ((legs & EXT_MPI_AMD_LEG_ALLGATHER) && multi && (rc = run_leg(h, EMAC_LEG_AG))) return rc;
  if ((legs & EXT_MPI_AMD_LEG_ALLGATHER) && h->hier && h->fanout.nb &&
      (rc = emac_gpu_copy_fan(h->plan.tsize, h->plan.nranks - 1, h->fanout.unroll, h->fanout.d_buckets, h->fanout.nb,
                              h->fanout.ntiles, h->fanout.tiles_per_bucket, h->fanout.all_full, h->fanout.d_edges,
                              h->fanout.nedges, h->stream)))
    return rc;
  if ((legs & EXT_MPI_AMD_LEG_ALLGATHER) && h->kind == KIND_IPC && h->plan.nranks > 1) {
    static const emac_codes copy = {{1}, {1}, 1, 1}; /* one leaf: a copy */
    if ((rc = ipc_barrier(h, 1))) return rc;
    if ((rc = emac_gpu_fold_remote(h->plan.dtype, EMAC_SUM, 1, h->pull.unroll, &copy, h->pull.d_buckets, h->pull.nb,
                                   h->pull.ntiles, h->pull.tiles_per_bucket, h->pull.all_full, h->pull.d_edges,
                                   h->pull.nedges, ipc_go(h), h->stream)))
      return rc;
  }
  if ((legs & EXT_MPI_AMD_LEG_STAGE_OUT) && (rc = stage_out(h))) return rc;
  return 0;
}

/* COMM form with device buffers, EXT_MPI_AMD_GRAPH=1: the legs of a Start captured once into a
   HIP graph (RCCL's grouped send/recv, the fold and its edge launch) and replayed by one
   hipGraphLaunch, per subset of legs; a capture that fails falls back to eager launches for good
   (graph_failed). Host buffers (pageable staging copies) are never captured. Opt-in: on a 1-rank
   communicator (the fold alone) a Start + Wait took 17.9 us replayed against 12.0 us eager
   (profiles/r02_graph_latency.json, the runtime's replay floor); with the two RCCL legs of N > 1
   ranks the balance is unmeasured here. */
static int graph_ok(const emac_handle *h) {
  const char *e = getenv("EXT_MPI_AMD_GRAPH");
  int r;
  if (h->kind != KIND_COMM || !e || atoi(e) <= 0) return 0;
  for (r = 0; r < h->nbuf; r++)
    if (h->send_mirror[r] || h->recv_mirror[r]) return 0;
  return 1;
}

int ext_mpi_amd_start_legs(int handle, int legs) {
  emac_handle *h = get(handle);
  int rc, key;
  if (!h) return EMAC_ERR_ARG;
  if (emac_gpu_set_device(h->device)) return EMAC_ERR_DEVICE;
  if (h->pipe && (legs & EXT_MPI_AMD_LEG_ALL) == EXT_MPI_AMD_LEG_ALL) return pipe_start(h);
  key = legs & EXT_MPI_AMD_LEG_ALL;
  if (legs >> EMAC_LEG_STEP_SHIFT) { /* one node step alone (loopback lock-step): never captured */
    if ((rc = enqueue_legs(h, legs))) return rc;
    h->started = 1;
    return 0;
  }
  if (graph_ok(h) && !h->graph[key] && !h->graph_failed[key]) {
    if (emac_gpu_capture_begin(h->stream) == 0) {
      const int erc = enqueue_legs(h, legs);
      const int crc = emac_gpu_capture_end(h->stream, &h->graph[key]);
      if (erc || crc) {
        h->graph[key] = NULL;
        h->graph_failed[key] = 1;
      }
    } else {
      h->graph_failed[key] = 1;
    }
  }
  if (h->graph[key]) {
    if ((rc = emac_gpu_graph_launch(h->graph[key], h->stream))) return rc;
  } else if ((rc = enqueue_legs(h, legs))) {
    return rc;
  }
  h->started = 1;
  return 0;
}

int ext_mpi_amd_start(int handle) { return ext_mpi_amd_start_legs(handle, EXT_MPI_AMD_LEG_ALL); }

int ext_mpi_amd_set_stream(int handle, void *stream) {
  emac_handle *h = get(handle);
  if (!h || !stream) return EMAC_ERR_ARG;
  emac_gpu_stream_sync(h->stream);
  if (h->own_stream) emac_gpu_stream_destroy(h->stream);
  h->stream = stream;
  h->own_stream = 0;
  return 0;
}

int ext_mpi_amd_test(int handle) {
  emac_handle *h = get(handle);
  int rc;
  if (!h) return EMAC_ERR_ARG;
  if (!h->started) return 1;
  rc = emac_gpu_stream_query(h->stream);
  if (rc == 1) {
    h->started = 0;
    if (ipc_status(h)) return EMAC_ERR_TRANSPORT;
  }
  return rc;
}

int ext_mpi_amd_wait(int handle) {
  emac_handle *h = get(handle);
  int rc;
  if (!h) return EMAC_ERR_ARG;
  rc = emac_gpu_stream_sync(h->stream);
  h->started = 0;
  return rc ? rc : ipc_status(h);
}

/* Done of a peer-mapped handle over caller memory is collective over the communicator, as the
   reference's (EXT_MPI_Done_native -> ext_mpi_gpu_destroy_shared_memory's node barrier,
   cuda_shmem.c:190-216, then cudaIpcCloseMemHandle, :301-314): every rank closes its mappings of
   the peers' buffers, then the ranks agree, so when Done returns no peer maps this rank's buffers
   any more and the caller may free them (ipc_exchange). A handle whose exported buffers are all
   library memory (mirrors, the MPI layer's scratch) is released locally: that memory returns to
   the communicator's pool and is only freed by the collective communicator free. */
int ext_mpi_amd_done(int handle) {
  emac_handle *h = get(handle);
  int comm, collective;
  if (!h) return EMAC_ERR_ARG;
  handles[handle] = NULL;
  comm = h->comm;
  collective = h->kind == KIND_IPC && h->done_collective && comms[comm].used && comms[comm].size > 1;
  release(h);
  return collective ? ipc_agree(&comms[comm], 1) : 0;
}

void *ext_mpi_amd_stream(int handle) {
  emac_handle *h = get(handle);
  return h ? h->stream : NULL;
}

int ext_mpi_amd_plan_describe(int nranks, long count, int dtype, const char *copyin, int pos, long *piece_off,
                              long *piece_len, int max_pieces, int *owner_rank, int *leaf_ranks,
                              unsigned char *first, unsigned char *close, int *nlev) {
  emac_plan p;
  emac_copyin cfg;
  int rc, pc, t, n;
  if (nranks < 1 || nranks > EMAC_MAX_RANKS || pos < 0 || pos >= nranks) return EMAC_ERR_ARG;
  if ((rc = parse_cfg(copyin, nranks, &cfg))) return rc;
  if ((rc = emac_plan_build(&p, nranks, count, dtype, EMAC_SUM, &cfg))) return rc;
  n = p.npieces < max_pieces ? p.npieces : max_pieces;
  for (pc = 0; pc < n; pc++) {
    piece_off[pc] = p.chunk_off[(size_t)pc * nranks + pos];
    piece_len[pc] = p.chunk_len[(size_t)pc * nranks + pos];
  }
  *owner_rank = p.pos_rank[pos];
  for (t = 0; t < p.codes.nleaf; t++) {
    leaf_ranks[t] = p.leaf_rank[pos][t];
    first[t] = p.codes.first[t];
    close[t] = p.codes.close[t];
  }
  *nlev = p.codes.nlev;
  rc = p.npieces;
  emac_plan_free(&p);
  return rc;
}

int ext_mpi_amd_comm_program(int nranks, int rank, long count, int dtype, const char *copyin, long send_phase,
                             ext_mpi_amd_p2p *ops, int max_ops, int *nops, ext_mpi_amd_fold *folds, int max_folds,
                             int *nfolds, long *staging_bytes) {
  return ext_mpi_amd_comm_program_nodes(1, nranks, rank, count, dtype, copyin, send_phase, ops, max_ops, nops, folds,
                                        max_folds, nfolds, staging_bytes);
}

int ext_mpi_amd_comm_set_node_ports(int comm, int nodes, const int *ports) {
  emac_node_sched ns;
  int rc;
  if (comm < 0 || comm >= MAX_COMMS || !comms[comm].used) return EMAC_ERR_ARG;
  if (nodes < 1 || comms[comm].size % nodes) return EMAC_ERR_ARG;
  /* a peer-mapped communicator's members are nodes only as a whole (node_comm_allreduce_init) */
  if (nodes > EMAC_MAX_NODES || (nodes > 1 && comms[comm].ipc && nodes != comms[comm].size)) return EMAC_ERR_UNSUPPORTED;
  if ((rc = emac_node_sched_build(&ns, nodes, ports))) return rc;
  comms[comm].nodes = nodes;
  comms[comm].ns = ns;
  return 0;
}

int ext_mpi_amd_comm_set_nodes(int comm, int nodes) {
  if (nodes > 1 && (nodes & (nodes - 1))) return EMAC_ERR_ARG; /* one port per step: a power of two */
  return ext_mpi_amd_comm_set_node_ports(comm, nodes, NULL);
}

int ext_mpi_amd_node_shares(int nodes, const int *ports, int ranks_per_node, long count, int dtype, const char *copyin,
                            int me, long *off, long *len, int *node, int *leaf_nodes, int max_shares, int *nshares,
                            int *levels) {
  emac_node_sched ns;
  emac_plan p;
  emac_copyin cfg;
  emac_share *sh = NULL;
  int rc, i, l, n = 0;
  if (!nshares || ranks_per_node < 1 || ranks_per_node > EMAC_MAX_RANKS || nodes < 2 || nodes > EMAC_MAX_NODES ||
      me < 0 || me >= ranks_per_node || count < 0)
    return EMAC_ERR_ARG;
  if ((rc = emac_node_sched_build(&ns, nodes, ports))) return rc;
  if ((rc = parse_cfg(copyin, ranks_per_node, &cfg))) return rc;
  if ((rc = emac_plan_build(&p, ranks_per_node, count, dtype, EMAC_SUM, &cfg))) return rc;
  rc = emac_node_shares(&p, &ns, me, &sh, &n);
  for (i = 0; !rc && i < n && i < max_shares; i++) {
    off[i] = sh[i].off;
    len[i] = sh[i].len;
    node[i] = sh[i].node;
    for (l = 0; l < nodes; l++) leaf_nodes[(size_t)i * (size_t)nodes + l] = sh[i].leaf_node[l];
  }
  if (!rc) *nshares = n;
  if (!rc && levels) *levels = emac_node_single(&ns) == 2 ? ns.nsteps : 1;
  if (!rc && n > max_shares) rc = EMAC_ERR_ARG;
  free(sh);
  emac_plan_free(&p);
  return rc;
}

int ext_mpi_amd_comm_program_nodes(int nodes, int ranks_per_node, int rank, long count, int dtype, const char *copyin,
                                   long send_phase, ext_mpi_amd_p2p *ops, int max_ops, int *nops,
                                   ext_mpi_amd_fold *folds, int max_folds, int *nfolds, long *staging_bytes) {
  if (nodes > 1 && (nodes & (nodes - 1))) return EMAC_ERR_ARG; /* one port per step: a power of two */
  return ext_mpi_amd_comm_program_node_ports(nodes, NULL, ranks_per_node, rank, count, dtype, copyin, send_phase, ops,
                                             max_ops, nops, folds, max_folds, nfolds, staging_bytes);
}

int ext_mpi_amd_comm_program_node_ports(int nodes, const int *ports, int ranks_per_node, int rank, long count,
                                        int dtype, const char *copyin, long send_phase, ext_mpi_amd_p2p *ops,
                                        int max_ops, int *nops, ext_mpi_amd_fold *folds, int max_folds, int *nfolds,
                                        long *staging_bytes) {
  emac_node_sched ns;
  emac_plan p;
  emac_copyin cfg;
  emac_p2p *o = NULL;
  emac_fold *f = NULL;
  const int R = ranks_per_node;
  int rc, i, t, no = 0, nf = 0;
  if (R < 1 || R > EMAC_MAX_RANKS || nodes < 1 || nodes > EMAC_MAX_NODES || rank < 0 || rank >= nodes * R)
    return EMAC_ERR_ARG;
  if ((rc = emac_node_sched_build(&ns, nodes, ports))) return rc;
  if ((rc = parse_cfg(copyin, R, &cfg))) return rc;
  if ((rc = emac_plan_build(&p, R, count, dtype, EMAC_SUM, &cfg))) return rc;
  if ((rc = emac_comm_program_nodes(&p, nodes > 1 ? &ns : NULL, rank / R, rank % R, send_phase, &o, &no, &f, &nf,
                                    staging_bytes)))
    goto out;
  if (no > max_ops || nf > max_folds) {
    rc = EMAC_ERR_ARG;
    goto out;
  }
  for (i = 0; i < no; i++) {
    ops[i].leg = o[i].leg;
    ops[i].peer = o[i].peer;
    ops[i].is_send = o[i].is_send;
    ops[i].buf = o[i].buf;
    ops[i].offset = o[i].offset;
    ops[i].bytes = o[i].bytes;
  }
  for (i = 0; i < nf; i++) {
    memset(&folds[i], 0, sizeof(folds[i]));
    folds[i].piece = f[i].piece;
    folds[i].offset = f[i].offset;
    folds[i].count = f[i].count;
    folds[i].nleaf = f[i].nleaf;
    folds[i].leg = f[i].leg;
    for (t = 0; t < f[i].nleaf; t++) {
      folds[i].buf[t] = f[i].buf[t];
      folds[i].leaf_offset[t] = f[i].loff[t];
    }
  }
  *nops = no;
  *nfolds = nf;
out:
  free(o);
  free(f);
  emac_plan_free(&p);
  return rc;
}

const char *ext_mpi_amd_version(void) { return "ext_mpi_collectives_amd 0.1 (gfx950)"; }

/* ---- layout self-check (host only, no device): the NODE form's buckets and launch layout for
   buffers at the given 16-byte phases, with every access the kernels would make replayed on the
   host (fold_kernel tiles, fold_edge_kernel items; fold_kernel.hpp). Returns the number of
   accesses outside a buffer's [0, count) elements or destination elements not written exactly
   once per launch; -1 on a set-up error. Test infrastructure for the planner/layout pair. */
typedef struct {
  long count;
  int tsize;
  long bad;
  unsigned char *hits; /* per destination rank and element: writes seen */
} chk_state;

static long chk_elem(const void *base, const void *p, int tsize) {
  return (long)(((const char *)p - (const char *)base) / tsize);
}

static void chk_access(chk_state *st, long e, int r, int write) {
  if (e < 0 || e >= st->count) {
    if (st->bad++ < 3) fprintf(stderr, "layout check: %s of element %ld (count %ld) rank %d\n", write ? "store" : "load", e, st->count, r);
    return;
  }
  if (write) st->hits[(size_t)r * (size_t)st->count + (size_t)e]++;
}

int ext_mpi_amd_check_node_layout(int nranks, long count, int dtype, int op, const char *copyin, const int *phase,
                                  int fan) {
  emac_handle hh, *h = &hh;
  emac_copyin cfg;
  emac_bucket *b = NULL;
  emac_edge *edges = NULL;
  emac_launch L;
  chk_state st;
  int rc, r, nb, i, t, d;
  const long base_stride = 1L << 40;
  if (nranks < 1 || nranks > EMAC_MAX_RANKS || count < 0) return -1;
  memset(h, 0, sizeof(*h));
  memset(&L, 0, sizeof(L));
  if (parse_cfg(copyin, nranks, &cfg) || emac_plan_build(&h->plan, nranks, count, dtype, op, &cfg)) return -1;
  h->kind = KIND_NODE;
  h->bytes = (size_t)count * (size_t)h->plan.tsize;
  h->nbuf = h->nsrc = nranks;
  h->fan = fan ? nranks > 1 : 0;
  for (r = 0; r < nranks; r++) { /* fake, disjoint buffers at the requested 16-byte phases */
    h->dsend[r] = (void *)(base_stride * (2 * r + 1) + (phase ? phase[2 * r] : 0));
    h->drecv[r] = (void *)(base_stride * (2 * r + 2) + (phase ? phase[2 * r + 1] : 0));
  }
  b = (emac_bucket *)calloc((size_t)h->plan.npieces * nranks + 1, sizeof(emac_bucket));
  st.count = count;
  st.tsize = h->plan.tsize;
  st.bad = 0;
  st.hits = (unsigned char *)calloc((size_t)nranks * (size_t)(count + 1), 1);
  if (!b || !st.hits) {
    rc = -1;
    goto out;
  }
  nb = node_buckets(h, 0, count, b);
  if (!h->fan)
    for (i = 0; i < nb; i++) b[i].ndst = 1; /* COMM-like fan-out 1: only the first destination */
  if ((rc = emac_layout(b, nb, op, h->nsrc, emac_tree_kind(&h->plan.codes, op) == 1, h->fan, &edges, &L.nedges, &L.ntiles,
                        &L.tiles_per_bucket, &L.all_full, &L.unroll))) {
    rc = -1;
    goto out;
  }
  {
    const long EPV = 16 / h->plan.tsize, TILE = (long)EMAC_BLOCK * (L.unroll & 15);
    long tile;
    /* fold_kernel: each tile's vectors of its bucket */
    for (tile = 0; tile < L.ntiles; tile++) {
      int bi;
      long tt, v, v0, v1;
      if (L.tiles_per_bucket > 0) {
        bi = (int)(tile / L.tiles_per_bucket);
        tt = tile - (long)bi * L.tiles_per_bucket;
      } else {
        int lo = 0, hi = nb - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (b[mid].tile0 <= tile)
            lo = mid;
          else
            hi = mid - 1;
        }
        bi = lo;
        tt = tile - b[lo].tile0;
      }
      if (bi < 0 || bi >= nb) {
        st.bad++;
        continue;
      }
      v0 = tt * TILE;
      v1 = (L.all_full || (tt + 1) * TILE <= b[bi].nvec) ? v0 + TILE : b[bi].nvec;
      for (v = v0; v < v1; v++)
        for (i = 0; i < (int)EPV; i++) {
          for (t = 0; t < h->nsrc; t++) {
            /* which rank's send buffer leaf t points into (the fake bases are 2^40 apart) */
            const long bi_rank = ((long)((const char *)b[bi].src[t] - (const char *)0) / base_stride - 1) / 2;
            chk_access(&st, chk_elem(h->dsend[bi_rank], b[bi].src[t], st.tsize) + v * EPV + i, (int)bi_rank, 0);
          }
          for (d = 0; d < b[bi].ndst; d++) {
            const long dr = ((long)((const char *)b[bi].dst[d] - (const char *)0) / base_stride - 2) / 2;
            chk_access(&st, chk_elem(h->drecv[dr], b[bi].dst[d], st.tsize) + v * EPV + i, (int)dr, 1);
          }
        }
    }
    /* fold_edge_kernel items */
    for (i = 0; i < L.nedges; i++) {
      const emac_edge it = edges[i];
      const emac_bucket *bk = &b[it.bucket];
      long k, e, n = it.mode == 1 ? it.count : bk->head + bk->tail;
      for (k = 0; k < n; k++) {
        if (it.mode == 1)
          e = it.start + k;
        else
          e = k < bk->head ? k : bk->head + bk->nvec * EPV + (k - bk->head);
        e -= bk->head; /* pointers sit at element head */
        for (t = 0; t < h->nsrc; t++) {
          const long sr = ((long)((const char *)bk->src[t] - (const char *)0) / base_stride - 1) / 2;
          chk_access(&st, chk_elem(h->dsend[sr], bk->src[t], st.tsize) + e, (int)sr, 0);
        }
        for (d = 0; d < bk->ndst; d++) {
          const long dr = ((long)((const char *)bk->dst[d] - (const char *)0) / base_stride - 2) / 2;
          chk_access(&st, chk_elem(h->drecv[dr], bk->dst[d], st.tsize) + e, (int)dr, 1);
        }
      }
    }
  }
  /* every destination element written exactly once (fan-out N) / the first destination (fan 1) */
  for (r = 0; r < (h->fan ? nranks : 1); r++) {
    long e;
    for (e = 0; e < count; e++)
      if (st.hits[(size_t)r * (size_t)count + (size_t)e] != (h->fan || r == 0 ? 1 : 0)) {
        if (st.bad++ < 3)
          fprintf(stderr, "layout check: rank %d element %ld written %d times\n", r, e,
                  st.hits[(size_t)r * (size_t)count + (size_t)e]);
      }
  }
  rc = st.bad > 0x7fffffff ? 0x7fffffff : (int)st.bad;
out:
  free(edges);
  free(b);
  free(st.hits);
  emac_plan_free(&h->plan);
  return rc;
}
