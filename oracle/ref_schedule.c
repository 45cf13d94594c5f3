/*
 * ref_schedule.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Restatement of the method-6 ("recursive") single-node schedule generator of
 * src/core/reduce_copyin.c. Only the SMEMCPY / SREDUCE lines and the SET_NODE_BARRIER
 * markers are emitted; WAIT_NODE_BARRIER and memory-fence lines carry no data semantics
 * once phases are executed in lock-step (ref_emulate.c). Scope: one node, including the "1"
 * sub-split of the factor list (reduce_copies_one_socket's multi-level form, :970-1084).
 *
 * Sockets: with EXT_MPI_NUM_SOCKETS_PER_NODE > 1 the generator runs over the same node-wide
 * positions (ext_mpi_native.c:700-724); num_sockets only changes get_rank_cyclic's encoding of
 * a partner (:482-486), which the buffer table decodes back to the same node rank, and the
 * barrier/fence lines. The SMEMCPY / SREDUCE arithmetic restated here is therefore the same.
 *
 * Positions vs node ranks: the generator works on positions p in a permuted rank order
 * (ranks[p] is the node rank at position p, ext_mpi_rank_order); buffer indices in the
 * emitted lines are node-rank differences (get_rank_cyclic), i.e. rank-relative.
 */
#include <stdlib.h>
#include <string.h>
#include "ref_oracle.h"

/* reduce_copyin.c:396-427 */
void ref_sizes_displs(int R, long bytes, int tsize, long size_l, long *sizes, long *displs) {
  long nelem = bytes / tsize;
  int i;
  if (!size_l) {
    long base = nelem / R, extra = nelem % R;
    for (i = 0; i < R; i++) {
      long len = base + (i < extra ? 1 : 0);
      long first = (i < extra) ? base * i + i : base * i + extra;
      sizes[i] = len * tsize;
      displs[i] = first * tsize;
    }
  } else {
    long fixed = size_l * tsize;
    if (fixed > bytes) fixed = bytes;
    for (i = 0; i < R; i++) {
      displs[i] = i ? displs[i - 1] + sizes[i - 1] : 0;
      /* every rank but the last takes `fixed` bytes while they last; the last takes the rest */
      sizes[i] = (displs[i] + fixed <= bytes && i < R - 1) ? fixed : bytes - displs[i];
    }
  }
  displs[R] = displs[R - 1] + sizes[R - 1];
}

/* reduce_copyin.c:375-394. Note the deepest call (one factor left) leaves its block unchanged. */
void ref_rank_order(int size, int nfactors, const int *factors, int *ranks) {
  int f, blk, i, j;
  int *tmp, *sub;
  if (!nfactors) return;
  f = abs(factors[0]);
  blk = size / f;
  if (nfactors == 1) return;
  tmp = (int *)malloc(sizeof(int) * size);
  sub = (int *)malloc(sizeof(int) * blk);
  for (i = 0; i < blk; i++)
    for (j = 0; j < f; j++) tmp[i + j * blk] = ranks[i * f + j];
  for (j = 0; j < f; j++) {
    for (i = 0; i < blk; i++) sub[i] = tmp[i + j * blk];
    ref_rank_order(blk, nfactors - 1, factors + 1, sub);
    for (i = 0; i < blk; i++) ranks[i + j * blk] = sub[i];
  }
  free(sub);
  free(tmp);
}

/* ports_groups.c:18-35 */
int ref_parse_copyin(const char *s, int *method, int *factors, int max_factors) {
  const char *c = s;
  char *end;
  int n = 0;
  long v = strtol(c, &end, 10);
  if (end == c) return -1;
  *method = (int)v;
  c = end;
  while (*c == ' ' || *c == ';') c++;
  while (*c) {
    v = strtol(c, &end, 10);
    if (end == c) return -1;
    if (n >= max_factors) return -1;
    factors[n++] = (int)v;
    c = end;
    while (*c == ' ') c++;
  }
  return n;
}

/* get_rank_cyclic at num_sockets == 1 (reduce_copyin.c:482-486) */
static int rel_index(int R, const int *ranks, int me_pos, int other_pos) {
  return (R + ranks[other_pos] - ranks[me_pos]) % R;
}

typedef struct {
  ref_op *ops;
  int n, cap, overflow;
} prog_t;

static void emit(prog_t *p, int op, int dbuf, int drel, long doff, int sbuf, int srel, long soff,
                 long bytes) {
  if (p->n >= p->cap) {
    p->overflow = 1;
    return;
  }
  p->ops[p->n].op = op;
  p->ops[p->n].dbuf = dbuf;
  p->ops[p->n].drel = drel;
  p->ops[p->n].doff = doff;
  p->ops[p->n].sbuf = sbuf;
  p->ops[p->n].srel = srel;
  p->ops[p->n].soff = soff;
  p->ops[p->n].bytes = bytes;
  p->n++;
}

static void phase(prog_t *p) { emit(p, REF_OP_PHASE, 0, 0, 0, 0, 0, 0, 0); }

/*
 * reduce_copies_recursive, reduce_copyin.c:674-842.
 * stage 1 emits the reduce-scatter part (:687-744), stage 2 the allgather part
 * (:745-838). f[0..nf) are the radices after factors[0]: negative = reduce-scatter,
 * positive = allgather. pos is this rank's position.
 */
static void recursive_legs(prog_t *p, int NR, int R, int nf, const int *f, long bytes, int tsize, int pos,
                           const int *ranks, long size_l, long off0, int stage, int first_call) {
  /* NR: ranks of the node (buffer-index modulus); R: members of this level (socket_size) */
  long sizes[R], displs[R + 1];
  int nrs, s, q, i, base, gb, copied = 0;
  int *ag_base = (int *)calloc(nf > 0 ? nf : 1, sizeof(int));
  ref_sizes_displs(R, bytes, tsize, size_l, sizes, displs);
  for (nrs = 0; nrs < nf && f[nrs] < 0; nrs++);

  /* ---- reduce-scatter: recursive halving by radix |f[s]| (:687-744) ---- */
  gb = 1;
  for (s = 0; s < nrs; s++) gb *= -f[s];
  base = 0; /* rstart: first position of this rank's block at step s */
  for (s = 0; s < nrs; s++) {
    int fs = -f[s], qme;
    gb /= fs;
    if (stage == 1) phase(p);
    qme = (pos - base) / gb;
    for (q = 0; q < fs; q++) {
      long off, len;
      int partner;
      if (q == qme) continue;
      off = displs[(pos / gb) * gb] + off0;
      len = 0;
      for (i = 0; i < gb; i++) len += sizes[(pos / gb) * gb + i];
      partner = base + gb * q + pos % gb;
      if (len > 0 && stage == 1) {
        if (first_call && s == 0) {
          if (!copied) { /* own contribution, once (:721-725) */
            emit(p, REF_OP_COPY, REF_BUF_RECV, 0, off, REF_BUF_SEND, 0, off, len);
            copied = 1;
          }
          emit(p, REF_OP_SUM, REF_BUF_RECV, 0, off, REF_BUF_SEND, rel_index(NR, ranks, pos, partner),
               off, len);
        } else {
          emit(p, REF_OP_SUM, REF_BUF_RECV, 0, off, REF_BUF_RECV, rel_index(NR, ranks, pos, partner),
               off, len);
        }
      }
    }
    base += qme * gb;
  }

  if (stage != 2) {
    free(ag_base);
    return;
  }
  /* ---- allgather (:745-838) ---- */
  if (nrs < nf) {
    /* recursive doubling over the positive radices. The block bases are computed
       walking the radices from the last one down (:757-773). */
    int prod = 1;
    for (s = 0; s < nrs; s++) prod *= -f[s];
    gb = prod;
    base = 0;
    for (s = nf - 1; s >= 0 && f[s] > 0; s--) {
      gb /= f[s];
      ag_base[s] = base;
      base += ((pos - base) / gb) * gb;
    }
    for (s = nrs, gb = 1; s < nf; gb *= f[s], s++) {
      if (gb > 1) phase(p); /* wait_allgather_recursive between doubling steps (:776-782) */
      for (q = 0; q < f[s]; q++) {
        long off, len;
        int target;
        if (q == (pos - ag_base[s]) / gb) continue;
        off = displs[(pos / gb) * gb] + off0;
        len = 0;
        for (i = 0; i < gb; i++) len += sizes[(pos / gb) * gb + i];
        target = ag_base[s] + gb * q + pos % gb;
        if (len > 0)
          emit(p, REF_OP_COPY, REF_BUF_RECV, rel_index(NR, ranks, pos, target), off, REF_BUF_RECV, 0,
               off, len);
      }
    }
    phase(p); /* final wait_allgather_recursive (:798-803) */
  } else {
    /* no allgather radices: push the owned chunk to every other rank (:805-811) */
    for (i = 1; i < R; i++) {
      long off = displs[pos] + off0, len = sizes[pos];
      if (len > 0)
        emit(p, REF_OP_COPY, REF_BUF_RECV, rel_index(NR, ranks, pos, (pos + i) % R), off, REF_BUF_RECV,
             0, off, len);
    }
    phase(p);
  }
  free(ag_base);
}

/* reduce_copies_one_socket (reduce_copyin.c:970-1084). A "1" at index nloc of the factor list
   opens a sub-split: factors[nloc+1] = sloc members per group. This level then runs over the
   sloc positions strided by g = size / sloc that share pos % g (:976-981), and the level named
   by the factors after nloc+1 runs over the contiguous block of g positions holding pos, on the
   chunk this level assigned to pos (:1011-1020 / :1058-1067); the copy-out nests the other way
   round (:1020-1031). */
static int one_socket(prog_t *p, int NR, int size, int nfactors, const int *factors, long add, long bytes, int tsize,
                      int pos, const int *ranks, int first_call, int stage) {
  int nloc, sloc, g, i, rank_loc = -1, rank_loci = -1;
  int ranks_loc[size > 0 ? size : 1], ranks_loci[size > 0 ? size : 1];
  long sizes[size + 1], displs[size + 2];
  if (size <= 1) return 0;
  if (nfactors < 2) return -1;
  for (nloc = 1; nloc < nfactors && factors[nloc] != 1; nloc++);
  if (nloc != nfactors) {
    if (nloc + 2 >= nfactors) return -1;
    sloc = factors[nloc + 1];
    if (sloc < 1 || size % sloc) return -1;
    /* :1066-1067 reuse the piece loop's variable: an equal split into >1 pieces above a
       sub-split does not terminate in the reference's generator */
    if (factors[0] > 1) return -1;
  } else {
    sloc = size;
  }
  g = size / sloc;
  for (i = 0; i < sloc; i++) ranks_loc[i] = ranks[i * g + pos % g];
  for (i = 0; i < sloc; i++)
    if (ranks_loc[i] == ranks[pos]) rank_loc = i;
  for (i = 0; i < g; i++) ranks_loci[i] = ranks[i + pos / g * g];
  for (i = 0; i < g; i++)
    if (ranks_loci[i] == ranks[pos]) rank_loci = i;
  if (factors[0] < 0) {
    /* fixed fraction of -factors[0] elements per member (:994-1033) */
    if (stage == 1)
      recursive_legs(p, NR, sloc, nloc - 1, factors + 1, bytes, tsize, rank_loc, ranks_loc, -factors[0], add, 1,
                     first_call);
    if (nloc != nfactors) {
      ref_sizes_displs(sloc, bytes, tsize, -factors[0], sizes, displs);
      if (one_socket(p, NR, g, nfactors - nloc - 2, factors + nloc + 2, add + displs[rank_loc], sizes[rank_loc], tsize,
                     rank_loci, ranks_loci, 0, stage))
        return -1;
    }
    if (stage == 2)
      recursive_legs(p, NR, sloc, nloc - 1, factors + 1, bytes, tsize, rank_loc, ranks_loc, -factors[0], add, 2, 0);
  } else {
    /* factors[0] equal pieces, each with its own schedule (:1035-1081) */
    long nelem = bytes / tsize;
    for (i = 0; i < factors[0]; i++) {
      long len = nelem / factors[0], first;
      if (i >= nelem % factors[0]) {
        first = len * i + nelem % factors[0];
      } else {
        first = len * i + i;
        len++;
      }
      if (len > 0 || size != NR) {
        if (stage == 1)
          recursive_legs(p, NR, sloc, nloc - 1, factors + 1, len * tsize, tsize, rank_loc, ranks_loc, 0,
                         add + first * tsize, 1, first_call);
        if (nloc != nfactors) {
          ref_sizes_displs(sloc, len * tsize, tsize, 0, sizes, displs);
          if (one_socket(p, NR, g, nfactors - nloc - 2, factors + nloc + 2, add + first * tsize + displs[rank_loc],
                         sizes[rank_loc], tsize, rank_loci, ranks_loci, 0, stage))
            return -1;
        }
        if (stage == 2)
          recursive_legs(p, NR, sloc, nloc - 1, factors + 1, len * tsize, tsize, rank_loc, ranks_loc, 0,
                         add + first * tsize, 2, 0);
      }
    }
  }
  return 0;
}

/* Every level's radix chain must cover its members exactly (the reference silently produces a
   partial reduction otherwise). Returns 0 if the factor list is a valid method-6 list. */
static int check_level(int size, const int *factors, int nfactors) {
  int prod_rs = 1, prod_ag = 1, i, nrs = 0, nag = 0, nloc, sloc;
  if (nfactors < 2 || factors[0] == 0) return -1;
  for (nloc = 1; nloc < nfactors && factors[nloc] != 1; nloc++);
  sloc = size;
  if (nloc != nfactors) {
    if (nloc + 2 >= nfactors) return -1;
    sloc = factors[nloc + 1];
    if (sloc < 2 || size % sloc || size / sloc < 2 || factors[0] > 1) return -1;
    if (check_level(size / sloc, factors + nloc + 2, nfactors - nloc - 2)) return -1;
  }
  for (i = 1; i < nloc; i++) {
    if (factors[i] < 0) {
      if (nag) return -1; /* radices must be all reduce-scatter first, then allgather */
      prod_rs *= -factors[i];
      nrs++;
    } else if (factors[i] > 1) {
      prod_ag *= factors[i];
      nag++;
    } else {
      return -1;
    }
  }
  if (!nrs || prod_rs != sloc) return -1;
  if (nag && prod_ag != sloc) return -1;
  return 0;
}

/* ext_mpi_generate_allreduce_copyin (:1418-1542) / _copyout (:1544-1681), methods 6 and 9 */
int ref_schedule(int R, int node_rank, long bytes, int dtype, const int *factors, int nfactors,
                 int in_place, int stage, ref_op *out, int cap) {
  prog_t prog;
  int ranks[R], pos = -1, i, nrs, tsize = ref_type_size(dtype);
  if (tsize <= 0 || check_level(R, factors, nfactors)) return -1;
  prog.ops = out;
  prog.n = 0;
  prog.cap = cap;
  prog.overflow = 0;
  for (i = 0; i < R; i++) ranks[i] = i;
  for (nrs = 1; nrs < nfactors && factors[nrs] < 0; nrs++);
  ref_rank_order(R, nrs - 1, factors + 1, ranks); /* :1495-1504 */
  for (i = 0; i < R; i++)
    if (ranks[i] == node_rank) pos = i;
  if (pos < 0) return -1;
  if (one_socket(&prog, R, R, nfactors, factors, 0, bytes, tsize, pos, ranks, !in_place, stage) < 0) return -1;
  if (prog.overflow) return -1;
  return prog.n;
}
