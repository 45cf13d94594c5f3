/*
 * ref_emulate.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Single-process emulator of an R-rank, single-node ext_mpi Allreduce (copy-in methods 5-10):
 * every rank's copy-in and copy-out program (ref_schedule.c) is executed against host
 * buffers, phase by phase. A phase ends at a SET_NODE_BARRIER line; the reference orders
 * each step after its partners' previous step with pairwise spin flags
 * (ext_mpi_native_exec.c:21-84, :513-528), which a global lock-step reproduces for a
 * race-free schedule. Rank-relative buffer indices resolve as ext_mpi_xpmem.c:114-130:
 * index j of rank r is the buffer of node rank (r + j) mod R.
 */
#include <stdlib.h>
#include <string.h>
#include "ref_oracle.h"

#define MAX_FACTORS 64

typedef struct {
  ref_op *ops;
  int n;
  int pc;
} rank_prog;

static int build_programs(int R, long count, int dtype, const char *copyin, int in_place, int num_sockets,
                          rank_prog *progs) {
  int method, factors[MAX_FACTORS], nf, r, cap;
  long bytes = count * (long)ref_type_size(dtype);
  nf = ref_parse_copyin(copyin, &method, factors, MAX_FACTORS);
  if (nf < 1) return -1;
  cap = 8 * R * (R + 8) * (factors[0] > 0 ? factors[0] : 1) + 256;
  if (method < 5 || method > 10) return -1; /* 8 / 9 / 10 = 5 / 6 / 7 on shm staging */
  for (r = 0; r < R; r++) {
    int n1, n2;
    progs[r].ops = (ref_op *)malloc(sizeof(ref_op) * (size_t)cap * 2);
    progs[r].pc = 0;
    n1 = ref_schedule_m(R, r, bytes, dtype, method, num_sockets, factors, nf, in_place, 1, progs[r].ops, cap);
    if (n1 < 0) return -1;
    progs[r].ops[n1].op = REF_OP_PHASE; /* copy-in and copy-out are separate stages */
    n2 = ref_schedule_m(R, r, bytes, dtype, method, num_sockets, factors, nf, in_place, 2, progs[r].ops + n1 + 1, cap);
    if (n2 < 0) return -1;
    progs[r].n = n1 + 1 + n2;
  }
  return 0;
}

static void exec_op(int R, int r, const ref_op *o, int dtype, int red, void *const *send, void *const *recv) {
  char *dst = (char *)(o->dbuf == REF_BUF_RECV ? recv : send)[(r + o->drel) % R] + o->doff;
  const char *src = (const char *)(o->sbuf == REF_BUF_RECV ? recv : send)[(r + o->srel) % R] + o->soff;
  if (o->op == REF_OP_COPY) {
    if (dst != src) memmove(dst, src, (size_t)o->bytes);
  } else if (o->op == REF_OP_SUM) {
    ref_reduction_op(red, dtype, dst, src, o->bytes / ref_type_size(dtype));
  }
}

int ref_emulate(int R, long count, int dtype, const char *copyin, int in_place,
                void *const *sendbufs, void *const *recvbufs) {
  return ref_emulate_op(R, count, dtype, REF_RED_SUM, copyin, in_place, sendbufs, recvbufs);
}

int ref_emulate_op(int R, long count, int dtype, int red, const char *copyin, int in_place,
                   void *const *sendbufs, void *const *recvbufs) {
  return ref_emulate_op_s(R, count, dtype, red, copyin, in_place, 1, sendbufs, recvbufs);
}

int ref_emulate_op_s(int R, long count, int dtype, int red, const char *copyin, int in_place, int num_sockets,
                     void *const *sendbufs, void *const *recvbufs) {
  rank_prog *progs;
  void *const *send = in_place ? recvbufs : sendbufs;
  int r, active, rc = 0;
  if (R < 1 || count < 0 || ref_type_size(dtype) <= 0) return -1;
  if (R == 1) { /* a one-rank allreduce is a copy */
    if (!in_place) memcpy(recvbufs[0], sendbufs[0], (size_t)(count * ref_type_size(dtype)));
    return 0;
  }
  progs = (rank_prog *)calloc((size_t)R, sizeof(rank_prog));
  if (build_programs(R, count, dtype, copyin, in_place, num_sockets, progs)) {
    rc = -1;
    goto done;
  }
  do {
    active = 0;
    for (r = 0; r < R; r++) {
      rank_prog *p = &progs[r];
      while (p->pc < p->n && p->ops[p->pc].op != REF_OP_PHASE) exec_op(R, r, &p->ops[p->pc++], dtype, red, send, recvbufs);
      if (p->pc < p->n) p->pc++; /* step over the phase marker */
      if (p->pc < p->n) active = 1;
    }
  } while (active);
done:
  for (r = 0; r < R; r++) free(progs[r].ops);
  free(progs);
  return rc;
}

/* Several nodes, one port per step (EXT_MPI_NUM_PORTS "-1 1", "-1 -1 1 1", ...). ext_mpi_native.c:879-1000 composes: the node's
   copy-in -- reduce_copies_one_socket with in_out = 1 and one_node = 0 (reduce_copyin.c:1497-1500):
   the same reduce-scatter emission as one node, into shared memory -- then the inter-node
   algorithm of allreduce_recursive.c:222-453 over the node partials: with one port a single
   radix-2 step, each line reduced from the two nodes' partials of it (:248-347, reducefrom of the
   own line and the line received from the partner node), the lines exchanged back (:406-437), then
   the node's copy-out. Every element thus ends as ONE two-operand reduction of the two node
   partials; a two-operand SUM is commutative, so which partial is the accumulator changes no bit
   (MIN / MAX with NaNs or signed zeros would depend on it: node 0's partial is taken first here,
   parity for those inputs is unpinned). Ranks [0, R) are node 0, [R, 2R) node 1. */
int ref_emulate_nodes(int nodes, int R, long count, int dtype, int red, const char *copyin, int in_place,
                      int num_sockets, void *const *sendbufs, void *const *recvbufs) {
  int n, r, b, rc;
  const size_t bytes = (size_t)count * (size_t)ref_type_size(dtype);
  if (nodes < 1 || nodes > 16 || (nodes & (nodes - 1)) || R < 1 || ref_type_size(dtype) <= 0) return -1;
  for (n = 0; n < nodes; n++)
    if ((rc = ref_emulate_op_s(R, count, dtype, red, copyin, in_place, num_sockets, sendbufs + n * R, recvbufs + n * R)))
      return rc;
  /* 2^k nodes: k radix-2 steps. allreduce_core pairs task t with t ^ 2^(k-1-s) at step s
     (:261-284, highest bit first), and ext_mpi_native.c:879-912 runs it on tasks permuted by
     ext_mpi_rank_order over the factors (2, ..., 2) -- a bit reversal, task t = node bitrev(t)
     (rank_permutation.c:133-139, :176-200) -- so in node order step s pairs n with n ^ 2^s: the
     partials combine as a balanced pairwise tree, lowest node bit first, each combination one
     two-operand reduction (node n's partial first here; commutative for SUM) */
  for (b = 1; b < nodes; b <<= 1)
    for (n = 0; n < nodes; n += 2 * b) ref_reduction_op(red, dtype, recvbufs[n * R], recvbufs[(n + b) * R], count);
  for (r = 1; r < nodes * R; r++) memcpy(recvbufs[r], recvbufs[0], bytes);
  return 0;
}

/* debug_persistent.c:491-497 (host pattern, add = 73) and :426-432 (device pattern, add = 0) */
void ref_kat_fill(void *buf, long count, int tsize, int world_rank, long add) {
  long i, words = (count * tsize) / (long)sizeof(long int);
  for (i = 0; i < words; i++) ((long int *)buf)[i] = world_rank * count + i + add;
  if ((count * tsize) % (long)sizeof(long int)) ((int *)buf)[count - 1] = (int)(world_rank * count + count - 1);
}

/* exported for the threaded baseline */
int ref_build_programs_(int R, long count, int dtype, const char *copyin, int in_place, void *progs_out) {
  return build_programs(R, count, dtype, copyin, in_place, 1, (rank_prog *)progs_out);
}
