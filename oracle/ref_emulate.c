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

/* rank_perm_heuristic, rank_permutation.c:12-87 (qsort over equal values taken as stable, as
   glibc's merge-sort qsort leaves them) */
static void ref_perm_heuristic(int num_nodes, const long *counts, int *rank_perm) {
  long value[REF_MAX_NODES], v2[REF_MAX_NODES], aval[REF_MAX_NODES];
  int key[REF_MAX_NODES], color[REF_MAX_NODES], k2[REF_MAX_NODES], c2[REF_MAX_NODES], akey[REF_MAX_NODES], num_colors = num_nodes, i, j, k;
  for (i = 0; i < num_nodes; i++) {
    value[i] = counts[i];
    key[i] = color[i] = i;
  }
  while (num_colors > 1) {
    for (i = 0; i < num_colors; i++) {
      aval[i] = 0;
      akey[i] = i;
    }
    for (i = 0; i < num_nodes; i++) aval[color[i]] += value[i];
    if (num_colors % 2) aval[0] = 0;
    for (i = 0; i < num_colors; i++) /* a stable (bubble) sort by value */
      for (j = num_colors - 1; j > i; j--)
        if (aval[j - 1] > aval[j]) {
          long tv = aval[j - 1];
          int tk = akey[j - 1];
          aval[j - 1] = aval[j];
          akey[j - 1] = akey[j];
          aval[j] = tv;
          akey[j] = tk;
        }
    k = 0;
    if (!(num_colors % 2)) {
      for (i = 0; i < num_colors; i++)
        for (j = 0; j < num_nodes; j++) {
          const int want = (i % 2) ? akey[num_colors - 1 - i / 2] : akey[i / 2];
          if (want == color[j]) {
            v2[k] = value[j];
            k2[k] = key[j];
            c2[k++] = i / 2;
          }
        }
    } else {
      for (j = 0; j < num_nodes; j++)
        if (color[j] == 0) {
          v2[k] = value[j];
          k2[k] = key[j];
          c2[k++] = 0;
        }
      for (i = 0; i < num_colors - 1; i++)
        for (j = 0; j < num_nodes; j++) {
          const int want = (i % 2) ? akey[num_colors - 1 - i / 2] : akey[i / 2 + 1];
          if (want == color[j]) {
            v2[k] = value[j];
            k2[k] = key[j];
            c2[k++] = i / 2 + 1;
          }
        }
    }
    for (i = 0; i < num_nodes; i++) {
      value[i] = v2[i];
      key[i] = k2[i];
      color[i] = c2[i];
    }
    num_colors = (num_colors + 1) / 2;
  }
  for (i = 0; i < num_nodes; i++) rank_perm[i] = key[i];
}

/* Several nodes (EXT_MPI_NUM_PORTS "N(-p0 -p1 ... q0 q1 ...)"). ext_mpi_native.c:879-1000 composes:
   the node's copy-in -- reduce_copies_one_socket with in_out = 1 and one_node = 0
   (reduce_copyin.c:1497-1500): the same reduce-scatter emission as one node, into shared memory --
   then the inter-node algorithm of allreduce_recursive.c:222-453 (allreduce_core) over the node
   partials, then the node's copy-out. Restated here as the reference runs it, task by task:
   * the message is cut into one line per node (ext_mpi_native.c:768-786: count / N elements, the
     remainder to the low nodes), the algorithm runs on tasks, node n being task t with
     perm[t] = n (rank_permutation.c:133-139; lines mapped back with perm, :176-200).
     ext_mpi_native.c:879-897 writes ext_mpi_rank_order's permutation as RANK_PERM, but the
     forward pass tests its own still-NULL local rank_perm (rank_permutation.c:90,106) and always
     replaces it: the identity when every line has the same size, else rank_perm_heuristic over
     the line sizes (:111-122) -- the lines being, for a list without reduce-scatter ports
     (allreduce_short, ext_mpi_native.c:667,768-788), the whole message in line 0.
     raw_code.c:238-356 lays the lines out in task order (line k at the sizes of lines 0..k-1);
   * reduce-scatter step s (ports[s] < 0, radix p + 1 = |ports[s]| + 1) splits each group of G
     tasks into p + 1 sub-groups of Gn = G / (p + 1); every task keeps the lines of its sub-group,
     receiving from its column peers i = 0..p-1, (t + Gn (i + 1)) mod G in the group (:248-316),
     their partial of them, and reduces them in the order raw_code.c:270-340 replays the
     reducefrom lists: the first step (not the last) r_0 (received into line 2lb) += own,
     += r_1 .. r_{p-1}; a middle step own (2lb) += r_0 .. r_{p-1}; the last step r_{p-1}
     (received into lb) += own, += r_0 .. r_{p-2};
   * the allgather steps (:347-437) copy the finished lines back: every rank ends with line k as
     task k computed it.
   Only lists whose reduce-scatter part covers every node are restated (the allgather steps then
   copy); one ending in a reduce-scatter port, or reducing inside the allgather steps, is refused.
   Ranks [n R, (n + 1) R) are node n. */
int ref_emulate_node_ports(int nodes, const int *ports, int R, long count, int dtype, int red, const char *copyin,
                           int in_place, int num_sockets, void *const *sendbufs, void *const *recvbufs) {
  const int ts = ref_type_size(dtype);
  int rad[8], ag[8] = {0}, nrs = 0, nag = 0, task_node[REF_MAX_NODES], node_task[REF_MAX_NODES], n, r, t, k, s, i, j, G, g, gm, rc = 0, prod_rs = 1,
      prod_ag = 1;
  long lo[REF_MAX_NODES + 1];
  char **cur = NULL, **nxt = NULL;
  const size_t bytes = (size_t)count * (size_t)ts;
  if (nodes < 1 || nodes > REF_MAX_NODES || R < 1 || ts <= 0) return -1;
  for (n = 0; n < nodes; n++)
    if ((rc = ref_emulate_op_s(R, count, dtype, red, copyin, in_place, num_sockets, sendbufs + n * R, recvbufs + n * R)))
      return rc;
  if (nodes == 1) return 0;
  for (i = 0; ports[i] < 0; i++) {
    if (nrs == 8) return -1;
    rad[nrs++] = 1 - ports[i];
    prod_rs *= 1 - ports[i];
  }
  for (; ports[i] > 0; i++) {
    if (nag == 8) return -1;
    ag[nag++] = ports[i] + 1;
    prod_ag *= ports[i] + 1;
  }
  /* the reduce-scatter radices leave groups of gm = nodes / prod_rs tasks holding the same lines;
     the allgather steps while their block is smaller than gm reduce inside it (:347-403), the rest
     copy (:404-437) */
  if (ports[i] || !nag || prod_ag != nodes || nodes % prod_rs) return -1;
  gm = nodes / prod_rs;
  for (j = 0, g = 1; g < gm; g *= ag[j], j++);
  if (g != gm) return -1; /* an allgather step straddling gm: not restated */
  {
    long sz[REF_MAX_NODES];
    int equal = 1;
    for (t = 0; t < nodes; t++) {
      sz[t] = nrs ? count / nodes + (t < count % nodes) : (t ? 0 : count);
      equal &= sz[t] == sz[0];
    }
    for (t = 0; t < nodes; t++) task_node[t] = t;
    if (!equal) ref_perm_heuristic(nodes, sz, task_node);
  }
  for (t = 0; t < nodes; t++) node_task[task_node[t]] = t;
  lo[0] = 0;
  for (k = 0; k < nodes; k++) {
    const int m = task_node[k];
    lo[k + 1] = lo[k] + count / nodes + (m < count % nodes);
  }
  cur = (char **)calloc((size_t)nodes, sizeof(char *));
  nxt = (char **)calloc((size_t)nodes, sizeof(char *));
  if (!cur || !nxt) {
    rc = -1;
    goto out;
  }
  for (t = 0; t < nodes; t++) {
    cur[t] = (char *)malloc(bytes ? bytes : 1);
    nxt[t] = (char *)malloc(bytes ? bytes : 1);
    if (!cur[t] || !nxt[t]) {
      rc = -1;
      goto out;
    }
    memcpy(cur[t], recvbufs[task_node[t] * R], bytes); /* task t's node partial */
  }
  for (G = nodes, s = 0; s < nrs; G /= rad[s], s++) {
    const int p = rad[s] - 1, Gn = G / rad[s], last = s == nrs - 1;
    for (t = 0; t < nodes; t++) {
      int peer[REF_MAX_NODES];
      const long a = lo[t / Gn * Gn], b = lo[t / Gn * Gn + Gn];
      char *acc = nxt[t] + a * ts;
      const long len = b - a;
      for (i = 0; i < p; i++) peer[i] = (t + Gn * (i + 1)) % G + t / G * G;
      if (len <= 0) continue;
      if (last) {
        memcpy(acc, cur[peer[p - 1]] + a * ts, (size_t)(len * ts));
        ref_reduction_op(red, dtype, acc, cur[t] + a * ts, len);
        for (i = 0; i < p - 1; i++) ref_reduction_op(red, dtype, acc, cur[peer[i]] + a * ts, len);
      } else if (s == 0) {
        memcpy(acc, cur[peer[0]] + a * ts, (size_t)(len * ts));
        ref_reduction_op(red, dtype, acc, cur[t] + a * ts, len);
        for (i = 1; i < p; i++) ref_reduction_op(red, dtype, acc, cur[peer[i]] + a * ts, len);
      } else {
        memcpy(acc, cur[t] + a * ts, (size_t)(len * ts));
        for (i = 0; i < p; i++) ref_reduction_op(red, dtype, acc, cur[peer[i]] + a * ts, len);
      }
    }
    for (t = 0; t < nodes; t++) { /* the kept lines move on; the rest is dead */
      char *x = cur[t];
      cur[t] = nxt[t];
      nxt[t] = x;
    }
  }
  /* the allgather steps. While the block is smaller than gm (:347-403), every task sends all lines
     of its gm group to the tasks (t + g (i + 1)) mod gnext of its block and reduces what comes
     back, in its own order -- the first step of the whole algorithm (no reduce-scatter step
     before) r_0 (into lb) += own, += r_1 ..; any later one own (lb) += r_0 .. -- so the tasks of a
     block may end with differently associated sums. Then (:404-437) every task receives the lines
     of the other g-blocks of its gnext-block from the task at its own position in that g-block. */
  for (j = 0, g = 1; g < gm; g *= ag[j], j++) {
    const int q = ag[j] - 1, gnext = g * ag[j], first = nrs == 0 && j == 0;
    for (t = 0; t < nodes; t++) {
      int peer[REF_MAX_NODES];
      const long a = lo[t / gm * gm], b = lo[t / gm * gm + gm], len = b - a;
      char *acc = nxt[t] + a * ts;
      for (i = 0; i < q; i++) peer[i] = (t + g * (i + 1)) % gnext + t / gnext * gnext;
      if (len <= 0) continue;
      if (first) {
        memcpy(acc, cur[peer[0]] + a * ts, (size_t)(len * ts));
        ref_reduction_op(red, dtype, acc, cur[t] + a * ts, len);
        for (i = 1; i < q; i++) ref_reduction_op(red, dtype, acc, cur[peer[i]] + a * ts, len);
      } else {
        memcpy(acc, cur[t] + a * ts, (size_t)(len * ts));
        for (i = 0; i < q; i++) ref_reduction_op(red, dtype, acc, cur[peer[i]] + a * ts, len);
      }
    }
    for (t = 0; t < nodes; t++) {
      char *x = cur[t];
      cur[t] = nxt[t];
      nxt[t] = x;
    }
  }
  for (; j < nag; g *= ag[j], j++) {
    const int gnext = g * ag[j];
    for (t = 0; t < nodes; t++) {
      memcpy(nxt[t], cur[t], bytes);
      for (k = t / gnext * gnext; k < t / gnext * gnext + gnext; k += g) {
        const int src = k / g * g + t % g; /* the task at t's position in that g-block */
        const long a = lo[k], b = lo[k + g];
        if (k / g != t / g && b > a) memcpy(nxt[t] + a * ts, cur[src] + a * ts, (size_t)((b - a) * ts));
      }
    }
    for (t = 0; t < nodes; t++) {
      char *x = cur[t];
      cur[t] = nxt[t];
      nxt[t] = x;
    }
  }
  for (r = 0; r < nodes * R; r++) memcpy(recvbufs[r], cur[node_task[r / R]], bytes);
out:
  for (t = 0; t < nodes && cur && nxt; t++) {
    free(cur[t]);
    free(nxt[t]);
  }
  free(cur);
  free(nxt);
  return rc;
}

/* one port per step over 2^k nodes ("-1 ... -1 1 ... 1") */
int ref_emulate_nodes(int nodes, int R, long count, int dtype, int red, const char *copyin, int in_place,
                      int num_sockets, void *const *sendbufs, void *const *recvbufs) {
  int ports[2 * 8 + 1], k = 0, i;
  if (nodes < 1 || nodes > REF_MAX_NODES || (nodes & (nodes - 1))) return -1;
  while ((1 << k) < nodes) k++;
  for (i = 0; i < k; i++) {
    ports[i] = -1;
    ports[k + i] = 1;
  }
  ports[2 * k] = 0;
  return ref_emulate_node_ports(nodes, ports, R, count, dtype, red, copyin, in_place, num_sockets, sendbufs, recvbufs);
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
