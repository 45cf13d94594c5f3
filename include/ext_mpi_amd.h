/*
 * ext_mpi_amd.h -- MPI-free C ABI of the MI355X bucket-reduction path
 * (libext_mpi_amd.so, ext_mpi_collectives_amd/).
 *
 * Plain C: pointers, sizes and int handles only. Every entry point mirrors a reference entry
 * point (paths relative to the eth-cscs/ext_mpi_collectives checkout):
 *
 *   ext_mpi_amd_allreduce_init   <- EXT_MPI_Allreduce_init      include/mpi/ext_mpi.h:75-77,
 *                                   src/mpi/ext_mpi.c:974-979 -> ext_mpi_allreduce_init_general
 *                                   :626-729 (one rank per GPU; legs over RCCL on xGMI)
 *   ext_mpi_amd_node_allreduce_init <- the same persistent Allreduce with every node rank's
 *                                   buffers mapped into one process: the reference maps peers
 *                                   with XPMEM (src/mpi/ext_mpi_xpmem.c:68-133) or CUDA IPC
 *                                   (src/gpu/cuda_shmem.c:218-299) and executes copy-in
 *                                   method 6 on them; here all ranks live in one GPU's HBM
 *   ext_mpi_amd_start            <- EXT_MPI_Start  ext_mpi.h:86, ext_mpi.c:1011-1017
 *   ext_mpi_amd_test             <- EXT_MPI_Test   ext_mpi.h:87, ext_mpi.c:1019-1025
 *   ext_mpi_amd_wait             <- EXT_MPI_Wait   ext_mpi.h:88, ext_mpi.c:1027-1033
 *   ext_mpi_amd_done             <- EXT_MPI_Done   ext_mpi.h:89, ext_mpi.c:1035-1041
 *   ext_mpi_amd_get_unique_id /
 *   ext_mpi_amd_comm_init / _free <- the node communicator set-up of EXT_MPI_Init_native
 *                                   (src/mpi/ext_mpi_native.c:1895-1911), which the MPI layer
 *                                   (libext_mpi_collectives.so) bootstraps with PMPI_Bcast
 *   ext_mpi_amd_plan_describe    <- the text IR the reference's pipe-stage tests print
 *                                   (tests/test_*.c): the fold schedule, for inspection/tests
 *
 * Return codes: 0 success; EXT_MPI_AMD_ERROR_MALLOC (-1) and EXT_MPI_AMD_ERROR_SHMEM (-2) as
 * ERROR_MALLOC / ERROR_SHMEM in include/core/constants.h:67-69; the others are new. Unlike
 * the reference (which exit()s on GPU errors, src/gpu/cuda_core.cu:14-48), errors are
 * returned, never fatal.
 *
 * Configuration: `copyin` is an EXT_MPI_COPYIN string ("6;1 -8 8", "6;1 -2 -2 -2 2 2 2",
 * "6;-64 -8 8"; method 5 cyclic, 6 recursive, 7 tree, 8 / 9 / 10 as their staged aliases);
 * NULL means "6;1 -R R" (the reference requires the variable, README "Installation").
 * Threading: MPI_THREAD_SERIALIZED, like the reference.
 */
#ifndef EXT_MPI_AMD_H_
#define EXT_MPI_AMD_H_

#ifdef __cplusplus
extern "C" {
#endif

/* element types (reference opcode order: OPCODE_REDUCE_SUM_DOUBLE, _LONG_INT, _FLOAT, _INT) */
#define EXT_MPI_AMD_DOUBLE 0
#define EXT_MPI_AMD_LONG 1
#define EXT_MPI_AMD_FLOAT 2
#define EXT_MPI_AMD_INT 3
/* element operations: SUM is the hot path; MIN / MAX follow the reference's CPU reduction
   (src/mpi/ext_mpi_native_exec.c:240-318: the accumulator takes the incoming element iff it
   compares less / greater), which its GPU kernel (src/gpu/cuda_core.cu:88-106) does not cover */
#define EXT_MPI_AMD_SUM 0
#define EXT_MPI_AMD_MIN 1
#define EXT_MPI_AMD_MAX 2

#define EXT_MPI_AMD_SUCCESS 0
#define EXT_MPI_AMD_ERROR_MALLOC (-1)
#define EXT_MPI_AMD_ERROR_SHMEM (-2)
#define EXT_MPI_AMD_ERROR_ARG (-3)
#define EXT_MPI_AMD_ERROR_UNSUPPORTED (-4)
#define EXT_MPI_AMD_ERROR_DEVICE (-5)
#define EXT_MPI_AMD_ERROR_TRANSPORT (-6)

#define EXT_MPI_AMD_UNIQUE_ID_BYTES 128
#define EXT_MPI_AMD_MAX_RANKS 16
#define EXT_MPI_AMD_MAX_NODES 64 /* nodes of one communicator's inter-node schedule */

/* ---- persistent Allreduce, every node rank's buffers in this process (one device) ---- */
int ext_mpi_amd_node_allreduce_init(int nranks, const void *const *sendbufs, void *const *recvbufs, long count,
                                    int dtype, int op, const char *copyin, int *handle);

/* ---- one owner chunk as a persistent handle (device pointers): dsts[d] = fold of srcs in the
 * given order, ((srcs[0] + srcs[1]) + srcs[2]) + ... ; ndst is 1 or nsrc. The persistent form of
 * the reference's per-stream copy/reduce descriptor (src/core/byte_code.c:936-992,
 * src/gpu/cuda_core.cu:88-106). */
int ext_mpi_amd_fold_init(int nsrc, const void *const *srcs, int ndst, void *const *dsts, long count, int dtype,
                          int op, int *handle);

/* ---- node communicator: one rank per GPU, reduce-scatter / allgather legs over RCCL ---- */
int ext_mpi_amd_get_unique_id(void *id /* EXT_MPI_AMD_UNIQUE_ID_BYTES */);
int ext_mpi_amd_comm_init(int rank, int size, const void *id, int device, int *comm);
int ext_mpi_amd_comm_free(int comm);
/* Testing transport: `size` communicators (one per rank) living in this process on the current
 * device; point-to-point ops become device copies executed by the receiving rank. Run each leg
 * on every rank before the next one (ext_mpi_amd_start_legs). Not for production. */
int ext_mpi_amd_comm_init_loopback(int size, int *comm_of_rank);
/* Peer-mapped communicator: one rank per GPU, every rank's device send buffer mapped into every
 * other rank with hipIpc (the reference's src/gpu/cuda_shmem.c:218-299 cudaIpc mapping), the
 * owner's fold reading the peers' chunks over xGMI into a library-owned result buffer that every
 * rank then pulls from into its own receive buffer (peers never write caller memory), node
 * barriers as stream-ordered kernels. `allgather` is called collectively (same order on every
 * rank) at communicator and handle set-up and at a handle's ext_mpi_amd_done: it must gather
 * `bytes` bytes from every rank into `recv` in rank order (as PMPI_Allgather(send, bytes,
 * MPI_BYTE, recv, bytes, MPI_BYTE, comm)) and return 0; it must stay callable while the
 * communicator lives. */
typedef int (*ext_mpi_amd_allgather_fn)(void *ctx, const void *send, void *recv, long bytes);
int ext_mpi_amd_comm_init_ipc(int rank, int size, ext_mpi_amd_allgather_fn allgather, void *ctx, int device,
                              int *comm);
int ext_mpi_amd_allreduce_init(const void *sendbuf, void *recvbuf, long count, int dtype, int op, int comm,
                               const char *copyin, int *handle);
/* Device memory owned by communicator `comm`, for buffers the caller itself hands to
 * ext_mpi_amd_allreduce_init (the MPI layer's self-test and blocking scratch). On a peer-mapped
 * communicator it comes from the pool of exported allocations that only the collective
 * ext_mpi_amd_comm_free returns to the runtime: a buffer released here while a slower peer still
 * maps it is never freed under that peer (freeing an exported allocation before every importer
 * has closed it corrupts later allocations). Elsewhere plain device memory. */
int ext_mpi_amd_comm_malloc(int comm, void **p, unsigned long bytes);
int ext_mpi_amd_comm_mfree(int comm, void *p);

/* ---- execution (stream-ordered on the handle's own HIP stream) ---- */
int ext_mpi_amd_start(int handle);
int ext_mpi_amd_test(int handle); /* 1 complete, 0 in flight, <0 error */
int ext_mpi_amd_wait(int handle);
/* Release a handle. On a peer-mapped communicator of more than one rank whose handle maps some
 * rank's caller-owned device send buffer this is collective, like the reference's EXT_MPI_Done (a
 * node barrier, src/gpu/cuda_shmem.c:190-216): every rank must call it, in the same order as its
 * other collective Done calls on that communicator, and once it returns no peer maps this rank's
 * buffers -- they may be freed. Handles over library memory only (host buffers, staged through
 * device mirrors) are released locally. */
int ext_mpi_amd_done(int handle);
void *ext_mpi_amd_stream(int handle); /* hipStream_t the handle runs on */
/* The fold's launch schedule (U 16-byte vectors per lane per leaf, load-issue schedule) and
 * whether it was tuned on this handle's first Starts (1 kept, 0 still measuring, -1 not tuned:
 * EXT_MPI_AMD_AUTOTUNE=0 or a shape with one schedule). Introspection for benchmarks. */
int ext_mpi_amd_handle_schedule(int handle, int *unroll, int *issue, int *tuned);
/* The schedules the tuner measures on this handle's first Starts: *n of them (0: untuned), the
 * first min(*n, max) written to sched as U | issue << 4. Introspection for tests. */
int ext_mpi_amd_handle_candidates(int handle, int *n, int *sched, int max);
/* The tuner's state of a handle (introspection for tests and benchmarks). A sample is one
 * candidate on three Starts in a row: the first untimed, the other timed_starts_per_sample timed --
 * as one window in the NODE form on device buffers, each fold launch between its own events in
 * every form that runs other operations between two folds (`isolated`: RCCL legs, barriers, pulls,
 * staging copies). ops_in_sample[i] counts the operations the handle enqueued inside sample i's
 * timed span(s): one fold per timed Start when the samples time the fold alone. `cached`: the
 * schedule came from an earlier handle of the same shape (nothing measured on this one). */
#define EXT_MPI_AMD_TUNE_MAX 8
typedef struct {
  int candidates;              /* 0: not tuned */
  int chosen;                  /* kept candidate, -1 while measuring */
  int cached;
  int isolated;
  int starts;                  /* Starts counted by the tuner */
  int timed_starts_per_sample;
  int samples;                 /* candidates x rounds (0 when cached) */
  int schedule[EXT_MPI_AMD_TUNE_MAX]; /* U | issue << 4 per candidate */
  float us[EXT_MPI_AMD_TUNE_MAX];     /* shortest sample per candidate, per timed Start (once kept) */
  int ops_in_sample[EXT_MPI_AMD_TUNE_MAX * 3];
} ext_mpi_amd_tune_info;
int ext_mpi_amd_handle_tune_info(int handle, ext_mpi_amd_tune_info *info);
/* Forget every kept schedule of this process (the next handle of each shape tunes afresh); returns
 * the number of entries dropped. EXT_MPI_AMD_TUNE_CACHE=0 bypasses the cache altogether. */
int ext_mpi_amd_tune_cache_clear(void);
/* Run later Starts on a caller-owned hipStream_t (e.g. to serialise several handles). */
int ext_mpi_amd_set_stream(int handle, void *hip_stream);
/* Start a subset of the legs (benchmarking / profiling): the reference interleaves them in one
   byte-code stream (src/mpi/ext_mpi_native_exec.c:345-587); here they are separable. */
#define EXT_MPI_AMD_LEG_STAGE_IN 1       /* H2D of host send buffers */
#define EXT_MPI_AMD_LEG_REDUCE_SCATTER 2 /* COMM form: slice exchange (reduce_copyin transport) */
#define EXT_MPI_AMD_LEG_FOLD 4           /* the bucket fold kernel (+ node fan-out) */
#define EXT_MPI_AMD_LEG_ALLGATHER 8      /* COMM form: owned chunk to every peer (reduce_copyout) */
#define EXT_MPI_AMD_LEG_STAGE_OUT 16     /* D2H of host receive buffers */
#define EXT_MPI_AMD_LEG_STAGE 17         /* both staging copies */
/* COMM form over several nodes (ext_mpi_amd_comm_set_node_ports), between the fold and the allgather: */
#define EXT_MPI_AMD_LEG_NODES_RS 32      /* per exchange step: lines traded with the other nodes' column peers */
#define EXT_MPI_AMD_LEG_NODES_FOLD 64    /* per exchange step: the lines' partials folded */
#define EXT_MPI_AMD_LEG_NODES_AG 128     /* per copying allgather step: finished lines sent on */
#define EXT_MPI_AMD_LEG_ALL 255
/* legs | EXT_MPI_AMD_LEG_STEP(s): the node legs of step s alone (a testing transport driving the
   steps in lock-step; s counts the exchange steps -- reduce-scatter steps, then allgather steps
   that reduce -- for NODES_RS / NODES_FOLD, and the copying allgather steps for NODES_AG);
   without it every step runs, in order */
#define EXT_MPI_AMD_LEG_STEP(s) (((s) + 1) << 8)
int ext_mpi_amd_start_legs(int handle, int legs);

/* ---- introspection (no GPU needed) ----
 * Fold schedule of owner position `pos` of an nranks-rank plan: element range of each piece
 * and the node ranks of the leaves in fold order; level codes per leaf. Returns the number of
 * pieces written (<= max_pieces) or an error code. leaf_ranks needs nranks ints; first/close
 * need nranks bytes each. owner_rank receives the node rank owning position `pos`. */
int ext_mpi_amd_plan_describe(int nranks, long count, int dtype, const char *copyin, int pos, long *piece_off,
                              long *piece_len, int max_pieces, int *owner_rank, int *leaf_ranks,
                              unsigned char *first, unsigned char *close, int *nlev);

/* Program of node rank `rank` in the COMM form (what Start executes, as data): point-to-point
 * ops of the reduce-scatter leg (leg == EXT_MPI_AMD_LEG_REDUCE_SCATTER) and the allgather leg
 * (EXT_MPI_AMD_LEG_ALLGATHER), and the owner's folds (leaf buffers/offsets in fold order,
 * codes as in ext_mpi_amd_plan_describe). Buffers: 0 send, 1 recv, 2 staging. Offsets in
 * bytes. send_phase = send buffer address mod 16 (staging slots share it). */
typedef struct {
  int leg, peer, is_send, buf;
  long offset, bytes;
} ext_mpi_amd_p2p;
typedef struct {
  int piece;
  long offset; /* bytes: the result in recv */
  long count;  /* elements */
  int buf[EXT_MPI_AMD_MAX_RANKS];
  long leaf_offset[EXT_MPI_AMD_MAX_RANKS];
  int nleaf; /* leaves used: nranks (the node's fold) or a node step's radix */
  int leg;   /* EXT_MPI_AMD_LEG_FOLD, or EXT_MPI_AMD_LEG_NODES_FOLD | step << 8 */
} ext_mpi_amd_fold;
int ext_mpi_amd_comm_program(int nranks, int rank, long count, int dtype, const char *copyin, long send_phase,
                             ext_mpi_amd_p2p *ops, int max_ops, int *nops, ext_mpi_amd_fold *folds, int max_folds,
                             int *nfolds, long *staging_bytes);
/* The same for `nodes` (1..EXT_MPI_AMD_MAX_NODES) nodes of ranks_per_node ranks under the inter-node ports `ports`
   (as ext_mpi_amd_comm_set_node_ports); `rank` is global (node-major); node legs and folds carry
   their step in leg >> 8. _nodes: the one-port schedule of a power of two. */
int ext_mpi_amd_comm_program_node_ports(int nodes, const int *ports, int ranks_per_node, int rank, long count,
                                        int dtype, const char *copyin, long send_phase, ext_mpi_amd_p2p *ops,
                                        int max_ops, int *nops, ext_mpi_amd_fold *folds, int max_folds, int *nfolds,
                                        long *staging_bytes);
int ext_mpi_amd_comm_program_nodes(int nodes, int ranks_per_node, int rank, long count, int dtype, const char *copyin,
                                   long send_phase, ext_mpi_amd_p2p *ops, int max_ops, int *nops,
                                   ext_mpi_amd_fold *folds, int max_folds, int *nfolds, long *staging_bytes);

/* ---- several nodes (§8f row 3, the inter-node ports schedule) ----
 * The reference runs an Allreduce over several nodes as: the node's copy-in (the same
 * reduce_copies_* emission as one node, into shared memory), the inter-node algorithm of
 * src/core/allreduce_recursive.c:222-453 over the node partials (EXT_MPI_NUM_PORTS), the node's
 * copy-out (src/mpi/ext_mpi_native.c:879-1000). On an RCCL (or loopback) communicator whose ranks
 * [n * size/nodes, (n + 1) * size/nodes) form node n, nodes <= EXT_MPI_AMD_MAX_NODES, set before
 * ext_mpi_amd_allreduce_init; copyin then describes ONE node (its ranks_per_node positions).
 * `ports` is the reference's num_ports list, 0-terminated: the reduce-scatter ports (negative,
 * radix |p| + 1 each), then the allgather ports (positive) whose radices multiply to `nodes` --
 * e.g. {-1, -1, 1, 1, 0} for 4 nodes, one port per step; {-2, 2, 0} for 3 nodes; with fewer
 * reduce-scatter steps ({3, 0}, {-1, 1, 1, 0}) the first allgather steps reduce inside the groups
 * left, each node in its own order (allreduce_recursive.c:348-403); NULL: one port per step for
 * a power of two, else one step of radix `nodes`. _set_nodes: the one-port schedule of a power of
 * two. Peer-mapped communicators are single-node (EXT_MPI_AMD_ERROR_UNSUPPORTED), as are lists
 * ending in a reduce-scatter port. */
int ext_mpi_amd_comm_set_node_ports(int comm, int nodes, const int *ports);
int ext_mpi_amd_comm_set_nodes(int comm, int nodes);

/* The same multi-node Allreduce with every rank of THIS node in this process (the NODE form's
 * buffers: nranks send / receive buffers on this process's device) and `comm` (RCCL or loopback)
 * having one member per node: member n is node n. The inter-node schedule is the one
 * ext_mpi_amd_comm_set_node_ports(comm, size, ports) set, else the default for `size` nodes.
 * A Start folds the node's copy-in over the send buffers where they lie (no intra-node transfer),
 * runs every node rank's node legs (rank me of each node is a column peer of rank me of the
 * others) as one RCCL group per leg, and stores each owner chunk into the node's other receive
 * buffers. Bits identical to ext_mpi_amd_allreduce_init on size * nranks ranks of one process each
 * (ext_mpi_native.c:879-1000).
 * On a peer-mapped communicator (ext_mpi_amd_comm_init_ipc; collective over it) the node legs are
 * peer loads instead: the copy-in goes into a partial block of the communicator's arena, then
 * barrier, each node folds its share of every node rank's chunk over the N partials read in place
 * (in the reference's line order), barrier, every share is pulled into the chunk owners' receive
 * buffers, and the copy-out follows. Only one reduce-scatter step over every node
 * (ext_mpi_amd_comm_set_node_ports(comm, size, {-(size-1), size-1, 0}), the default when size is
 * not a power of two) and, for SUM, one port per step over 2^k nodes (the default there) are
 * taken there; other lists return EXT_MPI_AMD_ERROR_UNSUPPORTED on every member. No caller memory is exported: Done is local. */
int ext_mpi_amd_node_comm_allreduce_init(int nranks, const void *const *sendbufs, void *const *recvbufs, long count,
                                         int dtype, int op, int comm, const char *copyin, int *handle);

/* The shares the peer-mapped node join folds (introspection for tests, no GPU): for node rank `me`
 * of `ranks_per_node`, under the inter-node list `ports` (0-terminated, NULL: the default) over
 * `nodes` nodes, each part of me's chunk as (off[i], len[i]) elements of the message, the node that
 * folds it (node[i]) and the nodes whose partials it folds, in order (leaf_nodes[i * nodes ..]).
 * Only one reduce-scatter step over every node (every part a left fold: *levels = 1) or one port
 * per step over 2^k nodes (every part k levels of pairs of consecutive leaves: *levels = k); else
 * EXT_MPI_AMD_ERROR_UNSUPPORTED. *nshares receives the count (ERROR_ARG if above max_shares). */
int ext_mpi_amd_node_shares(int nodes, const int *ports, int ranks_per_node, long count, int dtype, const char *copyin,
                            int me, long *off, long *len, int *node, int *leaf_nodes, int max_shares, int *nshares,
                            int *levels);

/* EXT_MPI_NUM_SOCKETS_PER_NODE (src/mpi/ext_mpi.c:43-187, a process-wide parameter): sockets per
 * node for every handle / plan made afterwards. It moves the tree method's (7 / 10) last-step
 * roots (reduce_copyin.c:860-864) and nothing else in the arithmetic. Returns the previous value,
 * or EXT_MPI_AMD_ERROR_ARG. A node size it does not divide is rejected at init. */
int ext_mpi_amd_set_num_sockets(int sockets);

/* The NODE form over peer-mapped nodes: the parts its join is pipelined by (1: the serial join;
 * EXT_MPI_AMD_JOIN_PARTS, engine_join.c), 0 for any other handle, or EXT_MPI_AMD_ERROR_ARG. */
int ext_mpi_amd_handle_join_parts(int handle);

/* A peer-mapped handle's cross-GPU settings (diagnostics for tests; no reference counterpart), as
 * EXT_MPI_AMD_IPC_* bits: the communicator's agreed verdict that some rank runs on another device
 * (device UUIDs exchanged at ext_mpi_amd_comm_init_ipc, or EXT_MPI_AMD_TEST_CROSS_DEVICE=1 on any
 * rank), a system-scope release recorded before every phase-0 barrier, and the fused node join's
 * partial stores at system or device scope. 0 for other handles, EXT_MPI_AMD_ERROR_ARG for none. */
#define EXT_MPI_AMD_IPC_CROSS_DEVICE 1
#define EXT_MPI_AMD_IPC_RELEASE_EVENT 2
#define EXT_MPI_AMD_IPC_SYS_STORES 4
#define EXT_MPI_AMD_IPC_DEV_STORES 8
int ext_mpi_amd_handle_ipc_flags(int handle);

const char *ext_mpi_amd_version(void);
/* "sha <commit>[+dirty] src <hash>": the commit and the hash of the product sources (csrc/,
 * include/) this binary was built from (ext_mpi_collectives_amd/_stamp.py). No reference
 * counterpart: it lets a test run state which build it exercised. */
const char *ext_mpi_amd_build_info(void);

#ifdef __cplusplus
}
#endif
#endif
