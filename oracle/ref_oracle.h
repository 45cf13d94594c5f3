/*
 * ref_oracle.h -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * CPU restatement of ext_mpi_collectives' single-node copy-in schedules -- methods 5
 * ("cyclic"), 6 ("recursive") and 7 ("tree"), 8 / 9 / 10 being the same on a staging copy --
 * and of its element-wise MPI_SUM / MIN / MAX loops. Only tests/, the smoke()
 * hook and bench.py's cpu_baseline leg may load this library.
 *
 * Reference files restated (paths relative to the reference checkout):
 *   src/mpi/ext_mpi_native_exec.c:207-318    reduction(), SUM/MIN/MAX      -> ref_reduction.c
 *   src/core/reduce_copyin.c:396-427         ext_mpi_sizes_displs          -> ref_schedule.c
 *   src/core/reduce_copyin.c:375-394         ext_mpi_rank_order            -> ref_schedule.c
 *   src/core/reduce_copyin.c:482-486         get_rank_cyclic               -> ref_schedule.c
 *   src/core/reduce_copyin.c:531-634         reduce_copies_cyclic          -> ref_schedule.c
 *   src/core/reduce_copyin.c:844-968         reduce_copies_tree            -> ref_schedule.c
 *   src/core/reduce_copyin.c:674-842         reduce_copies_recursive       -> ref_schedule.c
 *   src/core/reduce_copyin.c:970-1084        reduce_copies_one_socket      -> ref_schedule.c
 *   src/core/reduce_copyin.c:1418-1681       allreduce_copyin / _copyout   -> ref_schedule.c
 *   src/mpi/ext_mpi_xpmem.c:114-130          rank-relative buffer rotation -> ref_emulate.c, ref_schedule.c
 *   src/gpu/cuda_shmem.c:280-296             (the same rotation, device)   -> ref_schedule.c
 *   src/mpi/ext_mpi_native_exec.c:21-84      node barriers (as phases)     -> ref_emulate.c
 *   src/mpi/debug_persistent.c:426-497       known-answer input pattern    -> ref_emulate.c
 *   src/mpi/ext_mpi_native.c:879-1000,
 *   src/core/allreduce_recursive.c:222-453   several nodes (ports)         -> ref_emulate.c
 *
 * Parity pinning: the reference's own known-answer test pattern (debug_persistent.c) and the
 * method-6 schedules captured from the reference generators, both
 * committed under tests/golden/. The reference itself may not be executed here.
 * Methods 5 / 7 / 8 / 10 and num_sockets > 1 have no captured schedule: they are pinned by the
 * known-answer pattern (integer sums) and by an independent algebraic statement of each fold
 * order in tests/test_oracle.py -- "restatement-pinned", see DESIGN.md section 2.
 */
#ifndef REF_ORACLE_H_
#define REF_ORACLE_H_

#ifdef __cplusplus
extern "C" {
#endif

/* element types, in the order of the reference's OPCODE_REDUCE_SUM_* cases */
enum { REF_DOUBLE = 0, REF_LONG = 1, REF_FLOAT = 2, REF_INT = 3, REF_CHAR = 4 };

/* schedule line kinds: SMEMCPY, SREDUCE, and a SET_NODE_BARRIER phase marker */
enum { REF_OP_COPY = 0, REF_OP_SUM = 1, REF_OP_PHASE = 2 };
/* buffer classes of the IR (RECVBUF / SENDBUF, rank-relative index) */
enum { REF_BUF_RECV = 0, REF_BUF_SEND = 1 };

typedef struct {
  int op;
  int dbuf, drel; /* destination: buffer class, rank-relative index */
  long doff;      /* byte offset */
  int sbuf, srel;
  long soff;
  long bytes;
} ref_op;

int ref_type_size(int dtype);

/* ext_mpi_native_exec.c:207-234: p1[i] += p2[i] for i < n elements */
void ref_reduction(int dtype, void *p1, const void *p2, long n);

/* element operations (get_reduction_op, include/mpi/ext_mpi_native.h:77-140) */
enum { REF_RED_SUM = 0, REF_RED_MIN = 1, REF_RED_MAX = 2 };
/* ext_mpi_native_exec.c:207-318: SUM as above; MIN / MAX: p1[i] takes p2[i] iff p2[i] < / > p1[i] */
void ref_reduction_op(int op, int dtype, void *p1, const void *p2, long n);

/* reduce_copyin.c:396-427. sizes/displs in bytes; displs has R+1 entries. */
void ref_sizes_displs(int R, long bytes, int tsize, long size_l, long *sizes, long *displs);

/* reduce_copyin.c:375-394 (in place on ranks[size]) */
void ref_rank_order(int size, int nfactors, const int *factors, int *ranks);

/* Parse "method;f0 f1 ..." (ports_groups.c:18-35). Returns number of factors, -1 on error. */
int ref_parse_copyin(const char *s, int *method, int *factors, int max_factors);

/*
 * Per-rank program of the copy-in (stage=1) or copy-out (stage=2) leg, single node,
 * one socket. node_rank is the caller's rank in the node communicator. Returns the
 * number of ops written to out (or -1 if cap is exceeded / unsupported factors).
 */
int ref_schedule(int R, int node_rank, long bytes, int dtype, const int *factors, int nfactors,
                 int in_place, int stage, ref_op *out, int cap);
/* the same for copy-in method 5..10 and EXT_MPI_NUM_SOCKETS_PER_NODE = num_sockets */
int ref_schedule_m(int R, int node_rank, long bytes, int dtype, int method, int num_sockets, const int *factors,
                   int nfactors, int in_place, int stage, ref_op *out, int cap);
/* get_rank_cyclic (reduce_copyin.c:482-486) and the buffer table that decodes it
   (ext_mpi_xpmem.c:114-130): the node rank found at table index `index` of node rank `me` */
int ref_get_rank_cyclic(int num_sockets, int R, const int *ranks, int me_pos, int other_pos);
int ref_decode_peer(int num_sockets, int R, int me, int index);

/*
 * Single-process emulation of an R-rank Allreduce: executes every rank's copy-in then
 * copy-out program phase by phase (a phase ends at a SET_NODE_BARRIER; all ranks pass
 * it before any rank continues), resolving rank-relative buffer indices as in
 * ext_mpi_xpmem.c:114-130. sendbufs/recvbufs are arrays of R host pointers; with
 * in_place != 0 the data is taken from recvbufs. Returns 0 on success.
 */
int ref_emulate(int R, long count, int dtype, const char *copyin, int in_place,
                void *const *sendbufs, void *const *recvbufs);
/* the same with element operation `op` (REF_RED_*) on every SREDUCE line */
int ref_emulate_op(int R, long count, int dtype, int op, const char *copyin, int in_place,
                   void *const *sendbufs, void *const *recvbufs);
/* ... and with num_sockets sockets per node (changes the tree method's roots) */
int ref_emulate_op_s(int R, long count, int dtype, int op, const char *copyin, int in_place, int num_sockets,
                     void *const *sendbufs, void *const *recvbufs);

#define REF_MAX_NODES 64 /* nodes of the inter-node emulation (the product: EMAC_MAX_NODES) */
/* nodes (<= REF_MAX_NODES) nodes of R ranks under the inter-node ports list `ports` (0-terminated, the
   reference's EXT_MPI_NUM_PORTS: reduce-scatter ports, negative, then allgather ports;
   src/mpi/ext_mpi_native.c:879-1000 with src/core/allreduce_recursive.c:222-453, raw_code.c and
   rank_permutation.c): each node's copy-in, allreduce_core over the node partials task by task,
   the copy-out. nodes * R buffers, node-major. ref_emulate_nodes: one port per step, 2^k nodes. */
int ref_emulate_node_ports(int nodes, const int *ports, int R, long count, int dtype, int red, const char *copyin,
                           int in_place, int num_sockets, void *const *sendbufs, void *const *recvbufs);
int ref_emulate_nodes(int nodes, int R, long count, int dtype, int red, const char *copyin, int in_place,
                      int num_sockets, void *const *sendbufs, void *const *recvbufs);

/* Known-answer input pattern of debug_persistent.c:491-497 (CPU: add=73, GPU: add=0). */
void ref_kat_fill(void *buf, long count, int tsize, int world_rank, long add);

/*
 * Threaded CPU baseline: R pthreads, each running its own rank's copy-in+copy-out program
 * over shared host buffers with spin barriers at phase markers (the reference's CPU
 * executor shape: one pass per SREDUCE line). Runs `iters` allreduces and returns the
 * elapsed wall seconds (or a negative value on error).
 */
double ref_cpu_allreduce_threads(int R, long count, int dtype, const char *copyin,
                                 void *const *sendbufs, void *const *recvbufs, long iters);
/* The same over nsets rotated buffer sets (set k = buffers [k * R, (k + 1) * R); iteration i
   uses set i % nsets), so the working set can exceed the host's caches. */
double ref_cpu_allreduce_threads_sets(int R, long count, int dtype, const char *copyin, int nsets,
                                      void *const *sendbufs, void *const *recvbufs, long iters);

#ifdef __cplusplus
}
#endif
#endif
