/*
 * ref_schedule.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Restatement of the single-node schedule generators of src/core/reduce_copyin.c: copy-in
 * methods 5 ("cyclic", reduce_copies_cyclic :531-634), 6 ("recursive",
 * reduce_copies_recursive :674-842) and 7 ("tree", reduce_copies_tree :844-968); 8 / 9 / 10 are
 * the same generators on a shared-memory staging copy of the send buffer (:1508-1528), so their
 * arithmetic is that of 5 / 6 / 7. Only the SMEMCPY / SREDUCE lines and the SET_NODE_BARRIER
 * markers are emitted; WAIT_NODE_BARRIER and memory-fence lines carry no data semantics
 * once phases are executed in lock-step (ref_emulate.c). Scope: one node, including the "1"
 * sub-split of the factor list (reduce_copies_one_socket's multi-level form, :970-1084).
 *
 * Sockets: with EXT_MPI_NUM_SOCKETS_PER_NODE > 1 the generator runs over the same node-wide
 * positions (ext_mpi_native.c:700-724). get_rank_cyclic (:482-486) then encodes a partner
 * socket-relatively, and the buffer table rotates per socket (ext_mpi_xpmem.c:114-130,
 * cuda_shmem.c:280-296): ref_get_rank_cyclic / ref_decode_peer restate both, and
 * tests/test_oracle.py checks that decoding an encoded partner gives back its node rank for
 * every node size, socket count and rank pair -- so the lines below address peers with the
 * one-socket encoding. Sockets do change the arithmetic of the tree method: its last
 * reduce-scatter step accumulates into the position of the rank's socket (:860-864).
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

/* get_rank_cyclic (reduce_copyin.c:482-486): the buffer-table index under which position
   `me_pos` finds the buffer of position `other_pos` */
int ref_get_rank_cyclic(int num_sockets, int R, const int *ranks, int me_pos, int other_pos) {
  const int ssize = R / num_sockets;
  return (R + ranks[other_pos] / ssize * ssize - ranks[me_pos] / ssize * ssize) % R +
         (ssize + ranks[other_pos] % ssize - ranks[me_pos] % ssize) % ssize;
}

/* The buffer table of node rank `me` (ext_mpi_xpmem.c:114-130, cuda_shmem.c:280-296): entry i
   starts as node rank i's buffer, is rotated left by me's socket base, then every socket block
   is rotated left by me's rank within its socket, and entry 0 is the own buffer. Returns the
   node rank whose buffer sits at `index`. */
int ref_decode_peer(int num_sockets, int R, int me, int index) {
  int table[R], tmp[R], i, j, k;
  const int ssize = R / num_sockets;
  for (i = 0; i < R; i++) table[i] = i;
  for (j = 0; j < me / ssize * ssize; j++) {
    const int a = table[0];
    for (i = 0; i < R - 1; i++) table[i] = table[i + 1];
    table[R - 1] = a;
  }
  for (k = 0; k < num_sockets; k++)
    for (j = 0; j < me % ssize; j++) {
      const int a = table[ssize * k];
      for (i = ssize * k; i < ssize * (k + 1) - 1; i++) table[i] = table[i + 1];
      table[ssize * (k + 1) - 1] = a;
    }
  table[0] = me;
  (void)tmp;
  return table[index];
}

/* the one-socket encoding: decoding it with one socket gives the same node rank as decoding
   get_rank_cyclic's encoding with any socket count (tests/test_oracle.py) */
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

/*
 * reduce_copies_cyclic, reduce_copyin.c:531-634 (copy-in methods 5 / 8). Identity rank order.
 * Reduce-scatter step s (radix |f[s]|, gb = product of the later radices): position pos adds
 * into its chunks pos .. pos + gb - 1 the same chunks of the partners pos - gb * q (q = 1 ..
 * |f[s]| - 1), taken from their send buffers while the chunk still holds the raw data
 * (`used` <= 1, :569-572), else from their receive buffers (the partial sums of step s - 1).
 * Allgather: doubling pushes of the held chunks to pos - gb * q (:582-603), or the owned chunk
 * pushed to every other position (:604-611).
 */
static void cyclic_legs(prog_t *p, int NR, int R, int nf, const int *f, long bytes, int tsize, int pos,
                        const int *ranks, long size_l, long off0, int stage, int first_call) {
  long sizes[R], displs[R + 1];
  int used[R], first_used[R], nrs, s, q, i, gb;
  ref_sizes_displs(R, bytes, tsize, size_l, sizes, displs);
  for (i = 0; i < R; i++) used[i] = first_used[i] = 0;
  for (nrs = 0; nrs < nf && f[nrs] < 0; nrs++);
  for (s = 0, gb = 1; s < nrs; s++) gb *= -f[s];
  for (s = 0; s < nrs; s++) {
    const int fs = -f[s];
    gb /= fs;
    if (stage == 1) phase(p);
    for (i = 0; i + gb < R && i < gb; i++) { /* :544-556 */
      const int c = (2 * R + pos + i) % R;
      if (first_call && !used[i + gb]) {
        if (!first_used[i]) {
          if (sizes[c] > 0 && stage == 1)
            emit(p, REF_OP_COPY, REF_BUF_RECV, 0, displs[c] + off0, REF_BUF_SEND, 0, displs[c] + off0, sizes[c]);
          first_used[i] = 1;
        }
        used[i] = used[i + gb] = 1;
      }
    }
    for (q = 1; q < fs; q++) { /* :557-580 */
      const int partner = ((R - gb * q) % R + pos) % R;
      for (i = 0; i + gb * q < R && i < gb; i++) {
        const int c = (2 * R + pos + i) % R;
        if (sizes[c] > 0 && stage == 1)
          emit(p, REF_OP_SUM, REF_BUF_RECV, 0, displs[c] + off0,
               (first_call && used[i + gb * q] <= 1) ? REF_BUF_SEND : REF_BUF_RECV, rel_index(NR, ranks, pos, partner),
               displs[c] + off0, sizes[c]);
        used[i] = used[i + gb * q] = 2;
      }
    }
  }
  if (stage != 2) return;
  if (nrs < nf) { /* :582-603 */
    for (s = nrs, gb = 1; s < nf; gb *= f[s], s++) {
      for (q = 1; q < f[s]; q++) {
        const int partner = ((R - gb * q) % R + pos) % R;
        for (i = 0; i + gb * q < R && i < gb; i++) {
          const int c = (2 * R + pos + i) % R;
          if (sizes[c] > 0)
            emit(p, REF_OP_COPY, REF_BUF_RECV, rel_index(NR, ranks, pos, partner), displs[c] + off0, REF_BUF_RECV, 0,
                 displs[c] + off0, sizes[c]);
        }
      }
      phase(p);
    }
  } else { /* :604-631 */
    for (i = 1; i < R; i++)
      if (sizes[pos] > 0)
        emit(p, REF_OP_COPY, REF_BUF_RECV, rel_index(NR, ranks, pos, (pos + i) % R), displs[pos] + off0, REF_BUF_RECV,
             0, displs[pos] + off0, sizes[pos]);
    phase(p);
  }
}

/*
 * reduce_copies_tree, reduce_copyin.c:844-968 (copy-in methods 7 / 10), one node: the staging
 * buffer is the receive buffer (reduce_copies_one_socket :972-974). Reduce-scatter step s (gb as
 * above): position pos accumulates its block pos / gb (gb chunks) into the buffer of position
 * root = gb * socket + pos % gb, adding the block of positions gb * q + pos % gb (q != socket,
 * ascending), from send buffers at step 0 (the root's own block copied first), else from the
 * receive buffers. socket = pos / (R / |f[s]|) at the step with gb == 1 when the node has
 * several sockets (:860-864), else 0. Allgather (positive radices, :898-961): block pos / gb
 * copied from the root's buffer to the positions gb * q + pos % gb; without allgather radices
 * the reference stops (:962-964).
 */
static int tree_legs(prog_t *p, int NR, int R, int nf, const int *f, long bytes, int tsize, int pos, const int *ranks,
                     long size_l, long off0, int stage, int first_call, int num_sockets) {
  long sizes[R], displs[R + 1];
  int nrs, s, q, i, gb, flag_first = 1;
  ref_sizes_displs(R, bytes, tsize, size_l, sizes, displs);
  for (nrs = 0; nrs < nf && f[nrs] < 0; nrs++);
  if (nrs == nf) return -1; /* "reduce_copies_tree not implemented" */
  for (s = 0, gb = 1; s < nrs; s++) gb *= -f[s];
  for (s = 0; s < nrs; s++) {
    const int fs = -f[s];
    int socket, root;
    long off, len = 0;
    gb /= fs;
    socket = (num_sockets > 1 && gb == 1) ? pos / (R / fs) : 0;
    root = (gb * socket + pos % gb) % R;
    if (stage == 1) phase(p);
    off = displs[(pos / gb) * gb] + off0;
    for (i = 0; i < gb; i++) len += sizes[(pos / gb) * gb + i];
    for (q = 0; q < fs; q++) {
      const int src = (gb * q + pos % gb) % R;
      if (q == socket) continue;
      if (len <= 0 || stage != 1) continue;
      if (first_call && s == 0) {
        if (flag_first) {
          emit(p, REF_OP_COPY, REF_BUF_RECV, rel_index(NR, ranks, pos, root), off, REF_BUF_SEND,
               rel_index(NR, ranks, pos, root), off, len);
          flag_first = 0;
        }
        emit(p, REF_OP_SUM, REF_BUF_RECV, rel_index(NR, ranks, pos, root), off, REF_BUF_SEND,
             rel_index(NR, ranks, pos, src), off, len);
      } else {
        emit(p, REF_OP_SUM, REF_BUF_RECV, rel_index(NR, ranks, pos, root), off, REF_BUF_RECV,
             rel_index(NR, ranks, pos, src), off, len);
      }
    }
  }
  if (stage != 2) return 0;
  for (s = nrs, gb = 1; s < nf; gb *= f[s], s++) {
    const int socket = (num_sockets > 1 && gb == 1) ? pos / (R / f[s]) : 0;
    const int root = (gb * socket + pos % gb) % R;
    long off = displs[(pos / gb) * gb] + off0, len = 0;
    if (gb > 1) phase(p); /* wait_allgather_recursive (:929-935) */
    for (i = 0; i < gb; i++) len += sizes[(pos / gb) * gb + i];
    for (q = 0; q < f[s]; q++) {
      const int dst = (gb * q + pos % gb) % R;
      if (q == socket || len <= 0) continue;
      emit(p, REF_OP_COPY, REF_BUF_RECV, rel_index(NR, ranks, pos, dst), off, REF_BUF_RECV,
           rel_index(NR, ranks, pos, root), off, len);
    }
  }
  phase(p); /* :956-961 */
  return 0;
}

/* one leg of method m (5 cyclic, 6 recursive, 7 tree) */
static int method_legs(int method, prog_t *p, int NR, int R, int nf, const int *f, long bytes, int tsize, int pos,
                       const int *ranks, long size_l, long off0, int stage, int first_call, int num_sockets) {
  if (method == 5) {
    cyclic_legs(p, NR, R, nf, f, bytes, tsize, pos, ranks, size_l, off0, stage, first_call);
    return 0;
  }
  if (method == 7) return tree_legs(p, NR, R, nf, f, bytes, tsize, pos, ranks, size_l, off0, stage, first_call, num_sockets);
  recursive_legs(p, NR, R, nf, f, bytes, tsize, pos, ranks, size_l, off0, stage, first_call);
  return 0;
}

/* reduce_copies_one_socket (reduce_copyin.c:970-1084). A "1" at index nloc of the factor list
   opens a sub-split: factors[nloc+1] = sloc members per group. This level then runs over the
   sloc positions strided by g = size / sloc that share pos % g (:976-981), and the level named
   by the factors after nloc+1 runs over the contiguous block of g positions holding pos, on the
   chunk this level assigned to pos (:1011-1020 / :1058-1067); the copy-out nests the other way
   round (:1020-1031). */
static int one_socket(prog_t *p, int method, int num_sockets, int NR, int size, int nfactors, const int *factors, long add,
                      long bytes, int tsize, int pos, const int *ranks, int first_call, int stage) {
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
    if (stage == 1 && method_legs(method, p, NR, sloc, nloc - 1, factors + 1, bytes, tsize, rank_loc, ranks_loc,
                                  -factors[0], add, 1, first_call, num_sockets))
      return -1;
    if (nloc != nfactors) {
      ref_sizes_displs(sloc, bytes, tsize, -factors[0], sizes, displs);
      if (one_socket(p, method, num_sockets, NR, g, nfactors - nloc - 2, factors + nloc + 2, add + displs[rank_loc],
                     sizes[rank_loc], tsize, rank_loci, ranks_loci, 0, stage))
        return -1;
    }
    if (stage == 2 && method_legs(method, p, NR, sloc, nloc - 1, factors + 1, bytes, tsize, rank_loc, ranks_loc,
                                  -factors[0], add, 2, 0, num_sockets))
      return -1;
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
        if (stage == 1 && method_legs(method, p, NR, sloc, nloc - 1, factors + 1, len * tsize, tsize, rank_loc,
                                      ranks_loc, 0, add + first * tsize, 1, first_call, num_sockets))
          return -1;
        if (nloc != nfactors) {
          ref_sizes_displs(sloc, len * tsize, tsize, 0, sizes, displs);
          if (one_socket(p, method, num_sockets, NR, g, nfactors - nloc - 2, factors + nloc + 2,
                         add + first * tsize + displs[rank_loc], sizes[rank_loc], tsize, rank_loci, ranks_loci, 0, stage))
            return -1;
        }
        if (stage == 2 && method_legs(method, p, NR, sloc, nloc - 1, factors + 1, len * tsize, tsize, rank_loc,
                                      ranks_loc, 0, add + first * tsize, 2, 0, num_sockets))
          return -1;
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

/* ext_mpi_generate_allreduce_copyin (:1418-1542) / _copyout (:1544-1681): methods 5 / 8 with the
   identity rank order, 6 / 9 and 7 / 10 with ext_mpi_rank_order (:1487-1528) */
int ref_schedule_m(int R, int node_rank, long bytes, int dtype, int method, int num_sockets, const int *factors,
                   int nfactors, int in_place, int stage, ref_op *out, int cap) {
  prog_t prog;
  int ranks[R], pos = -1, i, nrs, tsize = ref_type_size(dtype);
  if (method >= 8 && method <= 10) method -= 3; /* the same generator on the staging copy (:1525-1526) */
  if (method < 5 || method > 7 || num_sockets < 1 || R % num_sockets) return -1;
  if (tsize <= 0 || check_level(R, factors, nfactors)) return -1;
  prog.ops = out;
  prog.n = 0;
  prog.cap = cap;
  prog.overflow = 0;
  for (i = 0; i < R; i++) ranks[i] = i;
  if (method >= 6) {
    for (nrs = 1; nrs < nfactors && factors[nrs] < 0; nrs++);
    ref_rank_order(R, nrs - 1, factors + 1, ranks); /* :1495-1504 */
  }
  for (i = 0; i < R; i++)
    if (ranks[i] == node_rank) pos = i;
  if (pos < 0) return -1;
  if (one_socket(&prog, method, num_sockets, R, R, nfactors, factors, 0, bytes, tsize, pos, ranks, !in_place, stage) < 0)
    return -1;
  if (prog.overflow) return -1;
  return prog.n;
}

int ref_schedule(int R, int node_rank, long bytes, int dtype, const int *factors, int nfactors, int in_place, int stage,
                 ref_op *out, int cap) {
  return ref_schedule_m(R, node_rank, bytes, dtype, 6, 1, factors, nfactors, in_place, stage, out, cap);
}
