/*
 * plan.h -- schedule planner of the MI355X bucket-reduction path (host C, no HIP).
 *
 * The reference compiles EXT_MPI_COPYIN into a text IR of SMEMCPY/SREDUCE lines
 * (src/core/reduce_copyin.c:674-842), assembles it into bytecode (src/core/byte_code.c) and
 * interprets it line by line. This planner computes the same arithmetic directly:
 *
 *   - the chunk partition of the message (reduce_copyin.c:396-427), nested through the "1"
 *     sub-splits of the factor list (reduce_copies_one_socket, reduce_copyin.c:970-1084),
 *   - the permuted rank order of radix chains (reduce_copyin.c:375-394),
 *   - for every owner chunk, the exact fold tree its elements are summed in: the left fold
 *     of each reduce-scatter step nested step over step, flattened to a leaf order plus
 *     per-leaf level codes that a register-resident kernel replays without any intermediate
 *     buffer. The three copy-in generators differ only in which partials a step folds and
 *     where the result lands, never in the tree's shape:
 *       method 6 recursive (reduce_copyin.c:687-744): own partial first, then the radix
 *         group's partners by ascending substep, positions from ext_mpi_rank_order;
 *       method 5 cyclic (:531-634): own partial, then positions p - gb, p - 2 gb, ...
 *         (mod R), identity rank order; the chunk completes at its own position;
 *       method 7 tree (:844-968): the partial at root gb * socket + p mod gb first, then
 *         positions gb * q + p mod gb for q != socket ascending; socket is p / (R / radix) at
 *         the last step when the node has several sockets, else 0.
 *     Who folds a chunk (here: its owner position, one pass) is free; the order is not.
 *
 * Because every leaf is read exactly once and the tree is evaluated in registers, a whole
 * multi-step reduce-scatter (and the allgather fan-out) becomes ONE pass over HBM while the
 * per-element operation order, and therefore every float/double bit, stays the reference's.
 */
#ifndef EMAC_PLAN_H_
#define EMAC_PLAN_H_

#ifdef __cplusplus
extern "C" {
#endif

#define EMAC_MAX_RANKS 16  /* ranks of one node fold (sources and fan-out destinations) */
#define EMAC_MAX_LEVELS 8  /* radices in one leg */
#define EMAC_MAX_SPLITS 4  /* nested "1 <members>" sub-split levels of one copy-in string */
#define EMAC_MAX_PIECES 65536

/* element types: same codes as include/ext_mpi_amd.h */
enum { EMAC_DOUBLE = 0, EMAC_LONG = 1, EMAC_FLOAT = 2, EMAC_INT = 3 };
enum { EMAC_SUM = 0, EMAC_MIN = 1, EMAC_MAX = 2 };

/* error codes (the first two follow include/core/constants.h:67-69 of the reference) */
enum {
  EMAC_OK = 0,
  EMAC_ERR_MALLOC = -1,
  EMAC_ERR_SHMEM = -2,
  EMAC_ERR_ARG = -3,
  EMAC_ERR_UNSUPPORTED = -4,
  EMAC_ERR_DEVICE = -5,
  EMAC_ERR_TRANSPORT = -6
};

/* One level of "split radices... [1 <members> <next level>]". Level 0 spans the node. A level
   followed by a sub-split runs over `sub` members strided by g = size/sub (the positions that
   share p mod g); the next level spans the contiguous block of g positions holding p, on the
   chunk this level assigned to p (reduce_copyin.c:976-981, :1011-1020). */
typedef struct {
  int split;                    /* k>0 equal pieces, -k fixed k-element fractions */
  int nrs, rs[EMAC_MAX_LEVELS]; /* reduce-scatter radices, in application order */
  int nag, ag[EMAC_MAX_LEVELS]; /* allgather radices (0 of them = direct push) */
  int sub;                      /* members per group when a sub-split follows, else 0 */
} emac_level;

typedef struct {
  int method;  /* 5 cyclic, 6 recursive, 7 tree; 8 / 9 / 10 are their shm-staged aliases */
  int sockets; /* EXT_MPI_NUM_SOCKETS_PER_NODE (0 or 1: one); moves the tree method's last roots */
  int nlv;
  emac_level lv[EMAC_MAX_SPLITS];
} emac_copyin;

/* the generator family of a method: 5, 6 or 7 (reduce_copyin.c:1525-1526 map 8-10 to 5-7) */
int emac_method_base(int method);

int emac_parse_copyin(const char *s, emac_copyin *out);
void emac_default_copyin(int nranks, emac_copyin *out); /* "6;1 -R R" */
int emac_validate_copyin(const emac_copyin *c, int nranks);
int emac_type_size(int dtype);

/* per-leaf replay codes of a fold tree (shared by every chunk of a plan) */
typedef struct {
  unsigned char first[EMAC_MAX_RANKS]; /* bit l: leaf t opens a fresh level-l accumulator */
  unsigned char close[EMAC_MAX_RANKS]; /* levels completed right after leaf t */
  /* levels are the reduce-scatter radices of every split level, level 0's first */
  int nlev;
  int nleaf;
} emac_codes;

typedef struct {
  int nranks;
  int dtype, tsize, op;
  long count;                             /* elements */
  emac_copyin cfg;
  int pos_rank[EMAC_MAX_RANKS];           /* position -> node rank */
  int rank_pos[EMAC_MAX_RANKS];           /* node rank -> position */
  int npieces;
  long *chunk_off;                        /* [piece * nranks + position], elements */
  long *chunk_len;
  int leaf_rank[EMAC_MAX_RANKS][EMAC_MAX_RANKS]; /* [owner position][leaf t] = node rank */
  emac_codes codes;
} emac_plan;

/* ---- COMM form (one rank per GPU): the point-to-point legs and the owner's fold, as data ----
 * Built once per handle; the RCCL executor (engine.c) only walks it. Exported through
 * ext_mpi_amd_comm_program so the same program can be executed by a host transport in tests. */
enum { EMAC_BUF_SEND = 0, EMAC_BUF_RECV = 1, EMAC_BUF_STAGE = 2 };
/* legs, as the EXT_MPI_AMD_LEG_* bits of include/ext_mpi_amd.h: the node's reduce-scatter, its
   fold, [two nodes: the node-pair exchange of the owned chunk's halves, their fold, the exchange
   back,] the node's allgather */
enum {
  EMAC_LEG_RS = 2,
  EMAC_LEG_FOLD = 4,
  EMAC_LEG_AG = 8,
  EMAC_LEG_NODES_RS = 32,
  EMAC_LEG_NODES_FOLD = 64,
  EMAC_LEG_NODES_AG = 128
};
#define EMAC_MAX_NODES 64
#define EMAC_MAX_NODE_STEPS 6 /* inter-node reduce-scatter steps (one port per step over 64 nodes) */
#define EMAC_LEG_STEP_SHIFT 8 /* node legs and folds carry their step: leg | step << 8 */

/* The inter-node schedule of several nodes (src/core/allreduce_recursive.c:222-453, the
   EXT_MPI_NUM_PORTS list): reduce-scatter steps of radix |port| + 1 over the tasks, the tasks
   being the nodes in the order ext_mpi_rank_order gives them over the allgather radices
   (ext_mpi_native.c:879-912, rank_permutation.c:89-228). */
typedef struct {
  int nodes;
  int nsteps;                         /* reduce-scatter steps between the nodes */
  int radix[EMAC_MAX_NODE_STEPS];     /* their radices, first step first */
  int gm;                             /* tasks per group holding the same lines after them */
  int nred;                           /* allgather steps that still reduce, inside a gm group */
  int red_radix[EMAC_MAX_NODE_STEPS]; /* their radices */
  int nagp;                           /* allgather steps that copy */
  int agp_radix[EMAC_MAX_NODE_STEPS]; /* their radices */
  int task_node[EMAC_MAX_NODES];      /* task -> node */
  int node_task[EMAC_MAX_NODES];      /* node -> task */
} emac_node_sched;
/* `ports`: the reference's list (0-terminated: every reduce-scatter port, negative, then every
   allgather port, positive; the allgather radices multiply to `nodes`, the reduce-scatter ones to
   a divisor of it -- the first allgather steps then reduce inside the groups the reduce-scatter
   leaves, e.g. "4(3)", "4(-1 1 1)"), or NULL for the default: one port per step ("-1 ... 1 ...")
   when `nodes` is a power of two, else one step of radix `nodes`. 0 or EMAC_ERR_ARG /
   EMAC_ERR_UNSUPPORTED. */
int emac_node_sched_build(emac_node_sched *s, int nodes, const int *ports);

typedef struct {
  int leg;     /* EMAC_LEG_RS or EMAC_LEG_AG */
  int peer;    /* node rank */
  int is_send;
  int buf;     /* EMAC_BUF_* */
  long offset; /* bytes */
  long bytes;
  int local;   /* the NODE form over several nodes: the node rank whose buffers the op uses (else 0) */
} emac_p2p;

typedef struct {
  int piece;
  long offset;                   /* byte offset of the result in the receive buffer */
  long count;                    /* elements */
  int buf[EMAC_MAX_RANKS];       /* per leaf (plan leaf order): EMAC_BUF_SEND, _RECV or _STAGE */
  long loff[EMAC_MAX_RANKS];     /* per leaf: byte offset of the first element */
  int nleaf;                     /* the node's R, or a node step's radix */
  int leg;                       /* EMAC_LEG_FOLD or EMAC_LEG_NODES_FOLD | step << 8 */
} emac_fold;

/* Program of node rank `me`: ops (reduce-scatter ops first, then allgather ops), one fold per
   non-empty piece, and the staging bytes. Peer slots in staging start at `send_phase` mod 16
   so they share the 16-byte phase of the send buffer. Caller frees *ops and *folds. */
int emac_comm_program(const emac_plan *p, int me, long send_phase, emac_p2p **ops, int *nops, emac_fold **folds,
                      int *nfolds, long *staging_bytes);
/* The same for rank `me` of node `node` under the inter-node schedule `ns` (NULL: one node), nodes
   of p->nranks ranks each (global rank = node * p->nranks + me, the peers in *ops are global
   ranks), as ext_mpi_native.c:879-1000 composes it: after the node's reduce-scatter and fold
   each owner chunk holds the node's partial of its elements; the message is cut into one line per
   node (ext_mpi_native.c:768-786), laid out in task order; at step st every task keeps the lines
   of its sub-group, sends each other sub-group's lines to the task of the same column there and
   receives its own lines' partials from those (NODES_RS | st << 8, only the part inside this
   rank's chunk: the same rank of each node carries it), folds them in the order raw_code.c:
   270-340 replays allreduce_core's reducefrom lists (NODES_FOLD | st << 8), and after the last
   step the finished lines go back in the reverse step order (NODES_AG | st << 8); the node's
   allgather then distributes the chunk. */
int emac_comm_program_nodes(const emac_plan *p, const emac_node_sched *ns, int node, int me, long send_phase,
                            emac_p2p **ops, int *nops, emac_fold **folds, int *nfolds, long *staging_bytes);

/* The NODE form over peer-mapped nodes (engine.c node_ipc_init) runs the inter-node schedule as
   shares instead of point-to-point lines: one reduce-scatter step over every node (program_nodes'
   "single" flow: every element's value is ONE fold of the N node partials, in the order its line's
   task gives, whoever computes it); or one port per step over 2^k nodes (program_nodes' halving
   flow: every value a balanced tree of pairwise sums over the task bits, high bit first -- the same
   whoever computes each pair, for SUM, where a + b == b + a). emac_node_single: 1 for one step over
   every node, 2 for the halving flow, else 0. */
int emac_node_single(const emac_node_sched *ns);
typedef struct {
  long off, len;                  /* elements of the message */
  int node;                       /* the node that folds this part (every node copies it back) */
  int nleaf;                      /* nodes whose partials it folds, in fold order */
  int nlev;                       /* 1: a left fold of the leaves; k: k levels of pairs (halving) */
  int leaf_node[EMAC_MAX_NODES];
} emac_share;
/* The parts of node rank `me`'s chunk (every piece): node task_node[u] folds the u-th N-th of the
   piece's chunk -- for one step over every node cut at the line boundaries, each part with its
   line's leaf order (task t's line: t - 1, t, t + 1, ..., t + N - 2 mod N, the last-step rule of
   raw_code.c); for the halving flow with the tasks in bit-reversed order, folded as k levels of
   pairs. *out is malloc'd. 0 or an EMAC_ERR_* code. */
int emac_node_shares(const emac_plan *p, const emac_node_sched *ns, int me, emac_share **out, int *nout);

/* Build the plan of an nranks-rank Allreduce of `count` elements. 0 or an EMAC_ERR_* code. */
int emac_plan_build(emac_plan *p, int nranks, long count, int dtype, int op, const emac_copyin *cfg);
void emac_plan_free(emac_plan *p);

#ifdef __cplusplus
}
#endif
#endif
