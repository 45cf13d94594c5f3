/*
 * engine_int.h -- declarations shared by the units of the handle engine (host C, internal).
 *
 * The engine (the reference's handle life cycle, src/mpi/ext_mpi_native.c: init :657-1113 with
 * init_epilogue :389-655, Start :215-230, Test/Wait :232-267, Done :269-387) is split by transport:
 *   engine.c       handle table, buffer mapping, bucket upload, Start / Test / Wait / Done
 *   engine_tune.c  per-handle launch-schedule tuning of the fold, and the per-process cache of
 *                  tuned schedules shared by handles of one shape
 *   engine_node.c  NODE form (every node rank in this process), the layout self-check
 *   engine_comm.c  COMM form over RCCL (and the loopback test transport), the point-to-point legs
 *   engine_ipc.c   peer-mapped form (hipIpc over xGMI): mappings, the arena, node barriers
 *   engine_join.c  NODE form over several nodes (RCCL legs or peer-mapped shares)
 * Nothing here is exported from libext_mpi_amd.so (hidden visibility); the public C ABI is
 * include/ext_mpi_amd.h.
 */
#ifndef EMAC_ENGINE_INT_H_
#define EMAC_ENGINE_INT_H_

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
  int cross_device; /* some peer runs on another device: release to system scope before phase 0,
                       system-scope partial stores in the fused node join. Agreed at set-up from
                       the exchanged device UUIDs (or forced on every rank by
                       EXT_MPI_AMD_TEST_CROSS_DEVICE=1 on any rank: the cross-GPU code paths on one
                       GPU, tests/test_gpu_node_ipc.py) */
  int same_device;  /* ranks of the communicator on this rank's device (itself included), from the
                       UUIDs: the fused node join divides its grid by it */
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

/* one fold launch over a set of device-resident buckets (a handle's main launch, or one stage of
   one part of the pipelined node join) */
typedef struct {
  emac_bucket *d_buckets;
  int nb;
  long ntiles, tiles_per_bucket;
  int all_full;
  emac_edge *d_edges;
  int nedges;
  int unroll;
} emac_launch;

/* Launch-schedule tuning of a handle's fold (NODE form, and the COMM / IPC / node-join forms'
   local fold): the first Start runs the static pick (emac_gpu_pick_unroll) and warms the buffers,
   the next EMAC_TUNE_SPAN x EMAC_TUNE_ROUNDS x candidates Starts sample the candidates round-robin,
   and the Start after them keeps the candidate with the shortest of its samples for the handle's
   lifetime. Every schedule folds in the same order -- the bits do not depend on the choice.
   Measured on MI355X leases (tools/schedbench.hip, tools/nodevar.hip, profiles/r03_schedbench_*,
   profiles/r03_nodevar/): the fastest schedule of a shape moves between leases by more than the
   spread within one (16 MiB x 8 node fold: U 2 48.1 us, U 4 51.8, U 4 staggered 54.1 on one
   lease; U 2 47.1, U 4 46.2 on another), so no fixed threshold table picks it everywhere; one
   sample per candidate (round 3's first tuner) kept U 2 on a lease where U 4 was 2 % faster, hence
   the rounds. A sample runs one candidate on EMAC_TUNE_SPAN Starts in a row: the first, right
   after another schedule's launch, untimed; the others timed on events without the system-scope
   fence (hipEventDisableSystemFence: a single launch between two fenced events ranked the
   schedules against their back-to-back rate -- the leaf-major deferred schedule 46-47 us alone,
   43.9-44.4 us per Start in the bench's steady state, where the tile-major one it lost to ran
   45.5-46.4 us; profiles/r03_tune/force_ab.txt):
   * NODE form on device buffers (nothing of the handle runs between the folds of two Starts): the
     timed Starts as ONE window, no event between them -- the back-to-back rate. Where the caller
     interleaves several handles the window also holds their launches; every candidate sees the
     same pattern.
   * every other form (`isolated`: the COMM form's RCCL legs, the peer-mapped barriers and pull,
     the node join's legs, host staging copies sit between the folds): each timed fold launch
     between its own pair of events, so a sample is the fold alone, never the network legs or a
     late peer.
   `ops` counts every operation the handle enqueues; a sample records how many of them fell inside
   its timed span(s) (ext_mpi_amd_handle_tune_info): one fold per timed Start.
   Kept schedules are shared per process (engine_tune.c): a handle whose shape (device, type, op,
   leaves, fan-out, fold tree, buckets' vector counts) some earlier handle has tuned starts on that
   schedule and spends no Start measuring (`cached`). EXT_MPI_AMD_AUTOTUNE=0 keeps the static pick;
   EXT_MPI_AMD_TUNE_CACHE=0 tunes every handle afresh; EXT_MPI_AMD_FOLD_SCHEDULE=<U | issue << 4>
   makes one schedule the only candidate (A/B runs; refused at init if the shape has no such
   kernel). */
#define EMAC_TUNE_MAX 8
#define EMAC_TUNE_ROUNDS 3
#define EMAC_TUNE_SPAN 3 /* Starts per sample: one untimed, then the timed ones */
#define EMAC_TUNE_SAMPLES (EMAC_TUNE_MAX * EMAC_TUNE_ROUNDS)
#define EMAC_TUNE_MIN_BYTES (16L << 20) /* algorithmic bytes per launch: smaller launches keep the static pick */
/* what a fold launch's schedule choice depends on (the tuning cache's key, engine_tune.c) */
typedef struct {
  int device, dtype, op, nsrc, fan, tree, nb, uniform;
  int kind, hier, isolated; /* the handle's form and how its samples are timed: a schedule kept by one
                               form (a fold_init local fold, say) is not reused unmeasured by another
                               (a COMM rank's fold over freshly staged leaves) of the same launch shape */
  long vec, vec0; /* 16-byte vectors per leaf over all buckets, in the first bucket */
} emac_shape;
typedef struct {
  int n;        /* candidates (0: no tuning) */
  int chosen;   /* index of the kept candidate, -1 while measuring */
  int starts;
  int isolated; /* each timed fold between its own events (legs run between the folds of two Starts) */
  int cached;   /* the kept schedule came from the per-process cache: no Start spent measuring */
  emac_shape shape;
  emac_launch L[EMAC_TUNE_MAX];
  void *ev[EMAC_TUNE_SAMPLES][2 * (EMAC_TUNE_SPAN - 1)]; /* sample i: candidate i % n, round i / n */
  float us[EMAC_TUNE_MAX];          /* shortest sample per candidate, per timed Start */
  unsigned long ops;                /* operations the handle has enqueued (folds, legs, copies, barriers) */
  unsigned long op_mark;            /* ops at the open of the current timed span */
  int span_ops[EMAC_TUNE_SAMPLES];  /* the handle's operations inside each sample's timed span(s) */
} emac_tune;

/* The peer-mapped node join pipelined by parts (engine_join.c, round 5; VERDICT r04 missing 2).
   The message is cut into nparts element ranges; part k's copy-in, share fold and pull + copy-out
   each have their own launch layout and part k its own synchronisation slot. Two executions:
   * fused (the default, 2 parts from EMAC_JOIN_MIN_BYTES per rank; join_fused.hip): ONE launch per Start
     whose workgroups walk the parts' segments in a skewed order, the dependencies being the
     slots' flags -- the copy-in of part k + 1 runs beside the share fold of part k and the pull of
     part k - 1;
   * streams (EXT_MPI_AMD_JOIN=streams): part k's launches on three streams (the handle's: copy-ins;
     s_fold; s_pull) with split barriers and events -- kept for A/B: on one MI355X each part's
     dependent launches and cross-stream waits cost more than the overlap gains.
   EXT_MPI_AMD_JOIN_PARTS=1 keeps the serial join (one slot, one stream). */
#define EMAC_JOIN_PARTS EMAC_JOIN_PARTS_MAX
#define EMAC_JOIN_MIN_BYTES (1L << 20) /* per rank: the pipelined join by default from here */
typedef struct {
  int nparts;
  int fused; /* one launch per Start (join_fused.hip), else the streams form */
  int sys_stores; /* fused: the copy-in's partials written through at system scope (a node on another GPU) */
  int grid;  /* the fused launch's workgroups */
  long lo[EMAC_JOIN_PARTS + 1]; /* part k: message elements [lo[k], lo[k + 1]) */
  int slot[EMAC_JOIN_PARTS];
  unsigned long epoch[EMAC_JOIN_PARTS][2];
  emac_launch in[EMAC_JOIN_PARTS], fold[EMAC_JOIN_PARTS], pull[EMAC_JOIN_PARTS];
  void *ctl; /* fused: its emac_join_ctl (device memory, zeroed between Starts) */
  void *s_fold, *s_pull;
  void *ev_in[EMAC_JOIN_PARTS], *ev_fold[EMAC_JOIN_PARTS], *ev_done;
} emac_join;

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
  emac_join *join;   /* ... pipelined by parts, or NULL (the serial join) */
} emac_handle;

#define EMAC_IPC_ATTEMPTS 8 /* set-up rounds of a peer-mapped exchange before it gives up */

#pragma GCC visibility push(hidden)

extern emac_handle *g_handles[MAX_HANDLES];
extern emac_comm g_comms[MAX_COMMS];
extern loop_group g_loops[MAX_LOOP_GROUPS];

/* engine.c */
emac_handle *handle_get(int handle);
void handle_release(emac_handle *h);
int finish_init(emac_handle *h, int *handle);
int parse_cfg(const char *copyin, int nranks, emac_copyin *cfg);
int map_buffers(emac_handle *h, int r, const void *send, void *recv);
void place_bucket(emac_bucket *b, int nsrc, long off, long len, int tsize);
int upload_launch_as(const emac_handle *h, emac_launch *L, emac_bucket *b, int nb, int nsrc, int tree);
int upload_launch(const emac_handle *h, emac_launch *L, emac_bucket *b, int nb);
int upload_launch_fan(const emac_handle *h, emac_launch *L, emac_bucket *b, int nb, int nsrc, int fan);
int stage_in(emac_handle *h);
int stage_out(emac_handle *h);

/* engine_tune.c */
int upload_buckets(emac_handle *h, emac_bucket *b, int nb);
int fold_launch(emac_handle *h);

/* engine_join.c */
int join_start(emac_handle *h, int copyin, int legs);
void join_free(emac_handle *h);

/* engine_comm.c */
int node_radix(const emac_node_sched *ns, int st);
char *leg_base_of(const emac_handle *h, int buf, int l);
char *leg_base(const emac_handle *h, int buf);
int run_leg(emac_handle *h, int leg);

/* engine_ipc.c */
int ipc_agree(emac_comm *cm, int ok_local);
void ipc_unmap(void *base);
void ipc_comm_release(emac_comm *cm);
int arena_alloc(emac_comm *cm, long bytes, void **p);
int arena_owns(const emac_comm *cm, const void *p, int *seg);
void arena_release(emac_comm *cm, void *p, long bytes);
int arena_grow(emac_comm *cm, int rc, long need);
int ipc_allreduce_init(emac_handle *h, emac_comm *cm, const void *sendbuf, void *recvbuf, int rc);
int ipc_init_settle(emac_handle *h, emac_comm *cm, int rc, int *handle);
unsigned *ipc_go(const emac_handle *h);
unsigned *ipc_go_slot(const emac_handle *h, int slot);
int ipc_barrier(emac_handle *h, int phase);
int ipc_status(const emac_handle *h);

#pragma GCC visibility pop

#endif
