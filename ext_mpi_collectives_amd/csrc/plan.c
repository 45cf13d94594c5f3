/*
 * plan.c -- EXT_MPI_COPYIN parsing, chunk partition and fold-tree construction.
 * See plan.h for the design; reference citations are to /root/reference (read-only).
 */
#include <stdlib.h>
#include <string.h>
#include "plan.h"

int emac_type_size(int dtype) {
  switch (dtype) {
  case EMAC_DOUBLE: return 8;
  case EMAC_LONG: return 8;
  case EMAC_FLOAT: return 4;
  case EMAC_INT: return 4;
  }
  return -1;
}

/* Grammar "method;f0 f1 f2 ..." of EXT_MPI_COPYIN / MPI_Info "ext_mpi_copyin"
   (src/core/ports_groups.c:18-35): f0 = split, then negative reduce-scatter radices, then
   positive allgather radices; a "1" (never a radix) opens a sub-split "1 <members> <level>"
   whose level has the same grammar (reduce_copyin.c:974-981). */
int emac_parse_copyin(const char *s, emac_copyin *out) {
  long v[4 * (2 + 2 * EMAC_MAX_LEVELS)];
  int n = 0, i, L = 0;
  const char *c = s;
  char *end;
  emac_level *lv;
  if (!s) return EMAC_ERR_ARG;
  memset(out, 0, sizeof(*out));
  while (*c == ' ') c++;
  while (*c) {
    if (n >= (int)(sizeof(v) / sizeof(v[0]))) return EMAC_ERR_UNSUPPORTED;
    v[n] = strtol(c, &end, 10);
    if (end == c) return EMAC_ERR_ARG;
    n++;
    c = end;
    if (n == 1) {
      while (*c == ' ') c++;
      if (*c != ';') return EMAC_ERR_ARG;
      c++;
    }
    while (*c == ' ' || *c == ',') c++;
  }
  if (n < 3) return EMAC_ERR_ARG; /* method, split and at least one radix */
  out->method = (int)v[0];
  i = 1;
  for (;;) {
    if (L >= EMAC_MAX_SPLITS) return EMAC_ERR_UNSUPPORTED;
    lv = &out->lv[L++];
    if (i >= n) return EMAC_ERR_ARG;
    lv->split = (int)v[i++];
    for (; i < n && v[i] != 1; i++) {
      if (v[i] < 0) {
        if (lv->nag) return EMAC_ERR_ARG; /* reduce-scatter radices come first */
        if (lv->nrs >= EMAC_MAX_LEVELS) return EMAC_ERR_UNSUPPORTED;
        lv->rs[lv->nrs++] = (int)-v[i];
      } else {
        if (lv->nag >= EMAC_MAX_LEVELS) return EMAC_ERR_UNSUPPORTED;
        lv->ag[lv->nag++] = (int)v[i];
      }
    }
    if (i == n) break;
    /* "1 <members>": the next level follows */
    if (i + 2 >= n) return EMAC_ERR_ARG;
    lv->sub = (int)v[i + 1];
    if (lv->sub < 1) return EMAC_ERR_ARG;
    i += 2;
  }
  out->nlv = L;
  return EMAC_OK;
}

void emac_default_copyin(int nranks, emac_copyin *out) {
  memset(out, 0, sizeof(*out));
  out->method = 6;
  out->nlv = 1;
  out->lv[0].split = 1;
  out->lv[0].nrs = 1;
  out->lv[0].rs[0] = nranks;
  out->lv[0].nag = 1;
  out->lv[0].ag[0] = nranks;
}

int emac_method_base(int method) { return method >= 8 && method <= 10 ? method - 3 : method; }

int emac_validate_copyin(const emac_copyin *c, int nranks) {
  int i, L, size = nranks, nlev = 0, base = emac_method_base(c->method);
  if (base < 5 || base > 7) return EMAC_ERR_UNSUPPORTED;
  if (c->nlv < 1) return EMAC_ERR_ARG;
  if (c->sockets < 0 || (c->sockets > 1 && nranks % c->sockets)) return EMAC_ERR_ARG;
  /* the cyclic and tree generators index their partners over the whole node: a sub-split
     level would mix rank-relative and level-relative positions (reduce_copyin.c:540-560,
     :866-880); only the recursive generator is defined on one */
  if (base != 6 && c->nlv > 1) return EMAC_ERR_UNSUPPORTED;
  /* reduce_copyin.c:962-964: the tree without allgather radices is not implemented */
  if (base == 7 && c->lv[0].nag == 0) return EMAC_ERR_UNSUPPORTED;
  for (L = 0; L < c->nlv; L++) {
    const emac_level *v = &c->lv[L];
    int prs = 1, pag = 1, members = size;
    if (v->split == 0 || v->nrs < 1) return EMAC_ERR_ARG;
    if (v->split > EMAC_MAX_PIECES) return EMAC_ERR_UNSUPPORTED;
    if (L < c->nlv - 1) {
      /* a sub-split needs members dividing the level, and the next level at least 2 wide */
      if (v->sub < 2 || size % v->sub || size / v->sub < 2) return EMAC_ERR_ARG;
      /* reduce_copyin.c:1035-1067 reuse the piece loop's variable inside a sub-split: more
         than one equal piece above a sub-split never terminates in the reference */
      if (v->split > 1) return EMAC_ERR_UNSUPPORTED;
      members = v->sub;
    } else if (v->sub) {
      return EMAC_ERR_ARG;
    }
    for (i = 0; i < v->nrs; i++) {
      if (v->rs[i] < 2) return EMAC_ERR_ARG;
      prs *= v->rs[i];
    }
    for (i = 0; i < v->nag; i++) {
      if (v->ag[i] < 2) return EMAC_ERR_ARG;
      pag *= v->ag[i];
    }
    /* every radix chain must cover its level exactly: the reference silently produces a
       partial reduction otherwise; here it is rejected */
    if (prs != members) return EMAC_ERR_ARG;
    if (v->nag && pag != members) return EMAC_ERR_ARG;
    nlev += v->nrs;
    size /= members;
  }
  if (nlev > EMAC_MAX_LEVELS) return EMAC_ERR_UNSUPPORTED;
  return EMAC_OK;
}

/* Chunk partition in elements (reduce_copyin.c:396-427): equal split with the remainder
   on the low positions, or fixed `frac`-element fractions with the rest on the last. */
static void partition(int R, long nelem, long frac, long *off, long *len) {
  int i;
  if (!frac) {
    long base = nelem / R, extra = nelem % R;
    for (i = 0; i < R; i++) {
      len[i] = base + (i < extra);
      off[i] = base * i + (i < extra ? i : extra);
    }
    return;
  }
  if (frac > nelem) frac = nelem;
  for (i = 0; i < R; i++) {
    off[i] = i ? off[i - 1] + len[i - 1] : 0;
    len[i] = (i < R - 1 && off[i] + frac <= nelem) ? frac : nelem - off[i];
  }
}

/* Position order of a radix chain (reduce_copyin.c:375-394): the positions of each radix
   group are spread by the group's stride so that recursive halving pairs far ranks first.
   The innermost radix keeps its block as is. */
static void position_order(int size, int nf, const int *f, int *ranks) {
  int stride, i, j, sub[EMAC_MAX_RANKS], tmp[EMAC_MAX_RANKS];
  if (nf < 2) return;
  stride = size / f[0];
  for (i = 0; i < stride; i++)
    for (j = 0; j < f[0]; j++) tmp[i + j * stride] = ranks[i * f[0] + j];
  for (j = 0; j < f[0]; j++) {
    memcpy(sub, tmp + j * stride, sizeof(int) * stride);
    position_order(stride, nf - 1, f + 1, sub);
    memcpy(ranks + j * stride, sub, sizeof(int) * stride);
  }
}

/* Block of level L holding absolute position P: its first position and width, P's offset in it,
   and the stride g of the level's member groups (g = 1 without a sub-split). */
static void level_block(const emac_copyin *c, int R, int L, int P, int *base, int *size, int *p, int *g) {
  int l, b = 0, sz = R, gg;
  for (l = 0;; l++) {
    gg = c->lv[l].sub ? sz / c->lv[l].sub : 1;
    if (l == L) break;
    b += ((P - b) / gg) * gg;
    sz = gg;
  }
  *base = b;
  *size = sz;
  *p = P - b;
  *g = gg;
}

/* Leaves, in evaluation order, of the value absolute position P holds for its chunk after
   reduce-scatter step s of level L. Step s combines rs[s] partials of step s-1: P's own first,
   then the partners of its radix group in ascending group index (reduce_copyin.c:687-744).
   Below step 0 of a level L > 0 the partial is level L-1's complete value of that position. */
static void tree_leaves(const emac_plan *pl, int L, int s, int P, int *out, int *k) {
  const emac_level *v = &pl->cfg.lv[L];
  int base, size, p, g, m, o, gb = 1, i, q, mbase, qme;
  if (s < 0) {
    if (L == 0)
      out[(*k)++] = pl->pos_rank[P];
    else
      tree_leaves(pl, L - 1, pl->cfg.lv[L - 1].nrs - 1, P, out, k);
    return;
  }
  level_block(&pl->cfg, pl->nranks, L, P, &base, &size, &p, &g);
  m = p / g; /* member index within the strided group (rank_loc) */
  o = p % g;
  for (i = s + 1; i < v->nrs; i++) gb *= v->rs[i];
  mbase = (m / (gb * v->rs[s])) * (gb * v->rs[s]);
  qme = (m - mbase) / gb;
  tree_leaves(pl, L, s - 1, P, out, k);
  for (q = 0; q < v->rs[s]; q++)
    if (q != qme) tree_leaves(pl, L, s - 1, base + (mbase + gb * q + m % gb) * g + o, out, k);
}

/* Method 5 (reduce_copyin.c:531-634): after step s position p holds, for its chunks, the left fold
   of its own step s-1 partial and those of p - gb_s * q (q = 1 .. rs[s]-1, mod R); positions are
   node ranks (identity order). */
static void cyclic_leaves(const emac_plan *pl, int s, int p, int *out, int *k) {
  const emac_level *v = &pl->cfg.lv[0];
  const int R = pl->nranks;
  int gb = 1, i, q;
  if (s < 0) {
    out[(*k)++] = pl->pos_rank[p];
    return;
  }
  for (i = s + 1; i < v->nrs; i++) gb *= v->rs[i];
  for (q = 0; q < v->rs[s]; q++) cyclic_leaves(pl, s - 1, ((p - gb * q) % R + R) % R, out, k);
}

/* Method 7 (reduce_copyin.c:844-968): step s folds into position rho = gb_s * socket + r the
   step s-1 partials of rho, then of gb_s * q + r (q != socket ascending), r = rho mod gb_s;
   socket = p / (R / rs[s]) for the writer p = (j / gb_s) * gb_s + r of chunk j at the step with
   gb_s == 1 on a multi-socket node (:860-864), else 0. */
static int tree_socket(const emac_plan *pl, int s, int gb, int p) {
  const emac_level *v = &pl->cfg.lv[0];
  return pl->cfg.sockets > 1 && gb == 1 ? p / (pl->nranks / v->rs[s]) : 0;
}

static void tree7_leaves(const emac_plan *pl, int s, int rho, int j, int *out, int *k) {
  const emac_level *v = &pl->cfg.lv[0];
  int gb = 1, i, q, r, sock;
  if (s < 0) {
    out[(*k)++] = pl->pos_rank[rho];
    return;
  }
  for (i = s + 1; i < v->nrs; i++) gb *= v->rs[i];
  r = rho % gb;
  sock = tree_socket(pl, s, gb, (j / gb) * gb + r);
  tree7_leaves(pl, s - 1, rho, j, out, k);
  for (q = 0; q < v->rs[s]; q++)
    if (q != sock) tree7_leaves(pl, s - 1, gb * q + r, j, out, k);
}

/* Replay codes of the composite tree: its levels are the reduce-scatter radices of level 0,
   then of level 1, ... (level 0's are the fastest-varying digits of the leaf index). */
static void build_codes(const emac_copyin *c, emac_codes *codes) {
  int t, l, L, rad[EMAC_MAX_LEVELS];
  memset(codes, 0, sizeof(*codes));
  for (L = 0; L < c->nlv; L++)
    for (l = 0; l < c->lv[L].nrs; l++) rad[codes->nlev++] = c->lv[L].rs[l];
  codes->nleaf = 1;
  for (l = 0; l < codes->nlev; l++) codes->nleaf *= rad[l];
  for (t = 0; t < codes->nleaf; t++) {
    int rem = t, closing = 1;
    for (l = 0; l < codes->nlev; l++) {
      int d = rem % rad[l];
      rem /= rad[l];
      if (d == 0) codes->first[t] |= (unsigned char)(1u << l);
      if (closing && d == rad[l] - 1)
        codes->close[t]++;
      else
        closing = 0;
    }
  }
}

static int level_pieces(const emac_level *v) { return v->split > 0 ? v->split : 1; }

/* Final chunks of relative position p in the level-L block of width `size`, inside the region
   [off, off+len) this block works on, appended in piece order (reduce_copyin.c:994-1081). */
static void level_chunks(const emac_copyin *c, int L, int size, int p, long off, long len, long *coff, long *clen,
                         int *k) {
  const emac_level *v = &c->lv[L];
  int members = v->sub ? v->sub : size, g = size / members, pc;
  long o[EMAC_MAX_RANKS], l[EMAC_MAX_RANKS], frac = v->split < 0 ? -(long)v->split : 0;
  for (pc = 0; pc < level_pieces(v); pc++) {
    long plen = len, poff = off;
    if (v->split > 0) { /* piece pc of an equal split (:1035-1044) */
      long base = len / v->split, extra = len % v->split;
      plen = base + (pc < extra);
      poff = off + base * pc + (pc < extra ? pc : extra);
    }
    partition(members, plen, frac, o, l);
    if (v->sub) {
      level_chunks(c, L + 1, g, p % g, poff + o[p / g], l[p / g], coff, clen, k);
    } else {
      coff[*k] = poff + o[p];
      clen[*k] = l[p];
      (*k)++;
    }
  }
}

int emac_plan_build(emac_plan *p, int nranks, long count, int dtype, int op, const emac_copyin *cfg) {
  int i, pc, k, L;
  long *coff, *clen;
  memset(p, 0, sizeof(*p));
  if (nranks < 1 || nranks > EMAC_MAX_RANKS || count < 0) return EMAC_ERR_ARG;
  if (emac_type_size(dtype) < 0 || op < EMAC_SUM || op > EMAC_MAX) return EMAC_ERR_ARG;
  p->nranks = nranks;
  p->dtype = dtype;
  p->tsize = emac_type_size(dtype);
  p->op = op;
  p->count = count;
  if (cfg) {
    p->cfg = *cfg;
  } else {
    emac_default_copyin(nranks, &p->cfg);
  }
  if (nranks == 1) { /* one rank: the allreduce is a copy; one leaf, one level */
    memset(&p->cfg.lv, 0, sizeof(p->cfg.lv));
    p->cfg.nlv = 1;
    p->cfg.lv[0].split = 1;
    p->cfg.lv[0].nrs = 1;
    p->cfg.lv[0].rs[0] = 1;
  } else {
    int rc = emac_validate_copyin(&p->cfg, nranks);
    if (rc) return rc;
  }
  /* rank order from the leading reduce-scatter radices (ext_mpi_native.c:715-724); the cyclic
     generator keeps the identity order (reduce_copyin.c:1487-1504) */
  for (i = 0; i < nranks; i++) p->pos_rank[i] = i;
  if (emac_method_base(p->cfg.method) != 5) position_order(nranks, p->cfg.lv[0].nrs, p->cfg.lv[0].rs, p->pos_rank);
  for (i = 0; i < nranks; i++) p->rank_pos[p->pos_rank[i]] = i;

  p->npieces = 1;
  for (L = 0; L < p->cfg.nlv; L++) p->npieces *= level_pieces(&p->cfg.lv[L]);
  p->chunk_off = (long *)malloc(sizeof(long) * (size_t)p->npieces * nranks);
  p->chunk_len = (long *)malloc(sizeof(long) * (size_t)p->npieces * nranks);
  coff = (long *)malloc(sizeof(long) * (size_t)p->npieces);
  clen = (long *)malloc(sizeof(long) * (size_t)p->npieces);
  if (!p->chunk_off || !p->chunk_len || !coff || !clen) {
    free(coff);
    free(clen);
    emac_plan_free(p);
    return EMAC_ERR_MALLOC;
  }
  for (i = 0; i < nranks; i++) {
    k = 0;
    level_chunks(&p->cfg, 0, nranks, i, 0, count, coff, clen, &k);
    for (pc = 0; pc < p->npieces; pc++) {
      p->chunk_off[(size_t)pc * nranks + i] = coff[pc];
      p->chunk_len[(size_t)pc * nranks + i] = clen[pc];
    }
  }
  free(coff);
  free(clen);
  for (i = 0; i < nranks; i++) {
    k = 0;
    const int last = p->cfg.lv[p->cfg.nlv - 1].nrs - 1;
    if (nranks == 1)
      p->leaf_rank[0][k++] = 0;
    else if (emac_method_base(p->cfg.method) == 5)
      cyclic_leaves(p, last, i, p->leaf_rank[i], &k);
    else if (emac_method_base(p->cfg.method) == 7)
      tree7_leaves(p, last, tree_socket(p, last, 1, i), i, p->leaf_rank[i], &k);
    else
      tree_leaves(p, p->cfg.nlv - 1, last, i, p->leaf_rank[i], &k);
  }
  build_codes(&p->cfg, &p->codes);
  return EMAC_OK;
}

void emac_plan_free(emac_plan *p) {
  free(p->chunk_off);
  free(p->chunk_len);
  p->chunk_off = p->chunk_len = NULL;
}

/* Reduce-scatter leg: one all-to-all round -- the slice of every owner chunk goes straight to
   its owner (the multi-step recursive halving of reduce_copyin.c:687-744 moves the same bytes
   in log R rounds, each bound by a single xGMI link). Allgather leg: the owned, folded chunk to
   every peer (reduce_copyin.c:745-838 as one round). Staging holds the R-1 received slices of
   each owned chunk, one 16-byte aligned slot per peer. */
int emac_comm_program(const emac_plan *p, int me, long send_phase, emac_p2p **ops_out, int *nops_out,
                      emac_fold **folds_out, int *nfolds_out, long *staging_bytes) {
  return emac_comm_program_nodes(p, NULL, 0, me, send_phase, ops_out, nops_out, folds_out, nfolds_out, staging_bytes);
}

int emac_node_sched_build(emac_node_sched *s, int nodes, const int *ports) {
  int def[2 * EMAC_MAX_NODE_STEPS + 1], ag[2 * EMAC_MAX_NODE_STEPS] = {0}, nag = 0, i, j, g, prod_rs = 1, prod_ag = 1;
  if (!s || nodes < 1 || nodes > EMAC_MAX_NODES) return EMAC_ERR_ARG;
  memset(s, 0, sizeof(*s));
  s->nodes = nodes;
  for (i = 0; i < nodes; i++) s->task_node[i] = s->node_task[i] = i;
  if (nodes == 1) return EMAC_OK; /* one node: no inter-node step, whatever the ports say */
  if (!ports) {
    int k = 0;
    while ((1 << k) < nodes) k++;
    if ((1 << k) == nodes && k <= EMAC_MAX_NODE_STEPS) { /* one port per step */
      for (i = 0; i < k; i++) {
        def[i] = -1;
        def[k + i] = 1;
      }
      def[2 * k] = 0;
    } else if (nodes <= EMAC_MAX_RANKS) { /* one step of radix `nodes` */
      def[0] = -(nodes - 1);
      def[1] = nodes - 1;
      def[2] = 0;
    } else { /* more nodes than one fold takes leaves: a step per prime factor, largest first */
      int f[2 * EMAC_MAX_NODE_STEPS], nf = 0, m = nodes, d;
      for (d = EMAC_MAX_RANKS; d >= 2; d--)
        while (m % d == 0 && d > 1) {
          int q, prime = 1;
          for (q = 2; q * q <= d; q++)
            if (d % q == 0) prime = 0;
          if (!prime) break;
          if (nf == EMAC_MAX_NODE_STEPS) return EMAC_ERR_UNSUPPORTED;
          f[nf++] = d;
          m /= d;
        }
      if (m != 1) return EMAC_ERR_UNSUPPORTED; /* a prime factor above EMAC_MAX_RANKS */
      for (i = 0; i < nf; i++) {
        def[i] = -(f[i] - 1);
        def[nf + i] = f[nf - 1 - i] - 1;
      }
      def[2 * nf] = 0;
    }
    ports = def;
  }
  /* allreduce_core (allreduce_recursive.c:222-453): the reduce-scatter ports first (negative),
     then the allgather ports (positive); a list ending in a negative port is reduce_scatter_core,
     not this path. The reduce-scatter steps leave groups of gm = nodes / prod_rs tasks holding
     the same lines; the allgather steps whose block is still smaller than gm reduce inside it
     (:348-403), the others copy (:404-437). */
  for (i = 0; ports[i] < 0; i++) {
    /* a step folds radix partials in one launch of at most EMAC_MAX_RANKS leaves */
    if (s->nsteps == EMAC_MAX_NODE_STEPS || 1 - ports[i] > EMAC_MAX_RANKS) return EMAC_ERR_UNSUPPORTED;
    s->radix[s->nsteps++] = 1 - ports[i];
    prod_rs *= 1 - ports[i];
  }
  for (; ports[i] > 0; i++) {
    if (nag == 2 * EMAC_MAX_NODE_STEPS) return EMAC_ERR_UNSUPPORTED;
    ag[nag++] = ports[i] + 1;
    prod_ag *= ports[i] + 1;
  }
  if (ports[i] != 0 || !nag) return EMAC_ERR_UNSUPPORTED;
  if (prod_ag != nodes || nodes % prod_rs) return EMAC_ERR_ARG;
  s->gm = nodes / prod_rs;
  for (j = 0, g = 1; g < s->gm; g *= ag[j], j++) {
    if (s->nred == EMAC_MAX_NODE_STEPS || ag[j] > EMAC_MAX_RANKS) return EMAC_ERR_UNSUPPORTED;
    s->red_radix[s->nred++] = ag[j];
  }
  if (g != s->gm) return EMAC_ERR_UNSUPPORTED; /* an allgather step across the group boundary */
  for (; j < nag; j++) {
    if (s->nagp == EMAC_MAX_NODE_STEPS) return EMAC_ERR_UNSUPPORTED;
    s->agp_radix[s->nagp++] = ag[j];
  }
  /* the task order depends on the message size: node_task_order, per program */
  return EMAC_OK;
}

/* rank_perm_heuristic (rank_permutation.c:12-87): pairs groups ("colors") of nodes by their
   summed line sizes, smallest with largest, halving the colors each round; the nodes end in the
   order perm[task]. The qsort there compares sizes only; ties keep their order here, as glibc's
   merge-sort qsort leaves them (an introsort qsort may not: parity with such a C library is
   unpinned where sizes tie). */
static void node_heuristic(int n, const long *sizes, int *perm) {
  long value[EMAC_MAX_NODES], cval[EMAC_MAX_NODES];
  int key[EMAC_MAX_NODES], color[EMAC_MAX_NODES], k2[EMAC_MAX_NODES], c2[EMAC_MAX_NODES], ckey[EMAC_MAX_NODES];
  long v2[EMAC_MAX_NODES];
  int ncol = n, i, j, k;
  for (i = 0; i < n; i++) {
    value[i] = sizes[i];
    key[i] = color[i] = i;
  }
  while (ncol > 1) {
    for (i = 0; i < ncol; i++) {
      cval[i] = 0;
      ckey[i] = i;
    }
    for (i = 0; i < n; i++) cval[color[i]] += value[i];
    if (ncol % 2) cval[0] = 0;
    for (i = 1; i < ncol; i++) { /* stable insertion sort by value */
      const long v = cval[i];
      const int kk = ckey[i];
      for (j = i - 1; j >= 0 && cval[j] > v; j--) {
        cval[j + 1] = cval[j];
        ckey[j + 1] = ckey[j];
      }
      cval[j + 1] = v;
      ckey[j + 1] = kk;
    }
    k = 0;
    if (!(ncol % 2)) {
      for (i = 0; i < ncol; i++)
        for (j = 0; j < n; j++)
          if (ckey[i % 2 ? ncol - 1 - i / 2 : i / 2] == color[j]) {
            v2[k] = value[j];
            k2[k] = key[j];
            c2[k++] = i / 2;
          }
    } else {
      for (j = 0; j < n; j++)
        if (color[j] == 0) {
          v2[k] = value[j];
          k2[k] = key[j];
          c2[k++] = 0;
        }
      for (i = 0; i < ncol - 1; i++)
        for (j = 0; j < n; j++)
          if (ckey[i % 2 ? ncol - 1 - i / 2 : i / 2 + 1] == color[j]) {
            v2[k] = value[j];
            k2[k] = key[j];
            c2[k++] = i / 2 + 1;
          }
    }
    for (i = 0; i < n; i++) {
      value[i] = v2[i];
      key[i] = k2[i];
      color[i] = c2[i];
    }
    ncol = (ncol + 1) / 2;
  }
  for (i = 0; i < n; i++) perm[i] = key[i];
}

/* The task order the reference's generators run with, as they run: ext_mpi_native.c:879-897
   writes ext_mpi_rank_order's permutation as PARAMETER RANK_PERM, but
   ext_mpi_generate_rank_permutation_forward tests its own still-NULL local rank_perm
   (rank_permutation.c:90,106) and so always replaces it -- with the identity when every line has
   the same size, else with rank_perm_heuristic over the line sizes (:111-122); the backward pass
   maps with that one (:170-200). The line sizes are count / N elements, the remainder to the low
   nodes (ext_mpi_native.c:768-786), or, for a list without reduce-scatter ports (allreduce_short,
   :667), the whole message in line 0. */
static void node_task_order(emac_node_sched *ns, long count) {
  long sz[EMAC_MAX_NODES];
  int i, equal = 1;
  const int N = ns->nodes;
  for (i = 0; i < N; i++) {
    sz[i] = ns->nsteps ? count / N + (i < count % N) : (i ? 0 : count);
    equal &= sz[i] == sz[0];
  }
  if (equal)
    for (i = 0; i < N; i++) ns->task_node[i] = i;
  else
    node_heuristic(N, sz, ns->task_node);
  for (i = 0; i < N; i++) ns->node_task[ns->task_node[i]] = i;
}

/* the element range [*lo, *hi) of the lines (tasks) [a, b) in the message of `count` elements:
   one line per node (ext_mpi_native.c:768-786: count / nodes, the remainder to the low nodes),
   laid out in task order (raw_code.c:238-356 addresses line n at the sizes of lines 0..n-1,
   mmsizes of each line's node after rank_permutation_backward) */
static void task_lines(const emac_node_sched *ns, long count, int a, int b, long *lo, long *hi) {
  const int N = ns->nodes;
  long off = 0;
  int k;
  *lo = 0;
  for (k = 0; k < b; k++) {
    const int n = ns->task_node[k];
    const long sz = count / N + (n < count % N);
    if (k == a) *lo = off;
    off += sz;
  }
  *hi = off;
  if (a >= b) *lo = off;
}

/* intersection of [a, b) and [c, d) as (offset, length) */
static void clip(long a, long b, long c, long d, long *off, long *len) {
  const long lo = a > c ? a : c, hi = b < d ? b : d;
  *off = lo;
  *len = hi > lo ? hi - lo : 0;
}

static int program_nodes(const emac_plan *p, const emac_node_sched *ns, int node, int me, long send_phase, long count,
                         emac_p2p **ops_out, int *nops_out, emac_fold **folds_out, int *nfolds_out,
                         long *staging_bytes);

int emac_comm_program_nodes(const emac_plan *p, const emac_node_sched *ns, int node, int me, long send_phase,
                            emac_p2p **ops_out, int *nops_out, emac_fold **folds_out, int *nfolds_out,
                            long *staging_bytes) {
  emac_node_sched nsl;
  long count = 0;
  int pc, q;
  for (pc = 0; pc < p->npieces; pc++) /* the message's elements: the pieces' chunks tile it */
    for (q = 0; q < p->nranks; q++) count += p->chunk_len[(size_t)pc * p->nranks + q];
  if (ns) { /* this message's task order */
    nsl = *ns;
    node_task_order(&nsl, count);
    ns = &nsl;
  }
  return program_nodes(p, ns, node, me, send_phase, count, ops_out, nops_out, folds_out, nfolds_out, staging_bytes);
}

int emac_node_single(const emac_node_sched *ns) {
  int st, halving = ns->nsteps > 0 && ns->nred == 0 && ns->nagp == ns->nsteps; /* program_nodes' condition */
  for (st = 0; st < ns->nsteps; st++) halving &= ns->radix[st] == 2;
  for (st = 0; st < ns->nagp; st++) halving &= ns->agp_radix[st] == 2;
  if (halving) return 2;
  if (ns->nsteps == 1 && ns->nred == 0 && ns->radix[0] == ns->nodes) return 1;
  return 0;
}

int emac_node_shares(const emac_plan *p, const emac_node_sched *ns0, int me, emac_share **out, int *nout) {
  emac_node_sched ns = *ns0;
  const int R = p->nranks, N = ns.nodes, pos = p->rank_pos[me];
  long count = 0;
  const int flow = emac_node_single(&ns), K = ns.nsteps;
  int pc, q, u, t, i, n = 0;
  emac_share *sh;
  *out = NULL;
  *nout = 0;
  if (!flow || me < 0 || me >= R) return EMAC_ERR_UNSUPPORTED;
  for (pc = 0; pc < p->npieces; pc++)
    for (q = 0; q < R; q++) count += p->chunk_len[(size_t)pc * R + q];
  node_task_order(&ns, count);
  sh = (emac_share *)calloc((size_t)p->npieces * (size_t)N * (size_t)N + 1, sizeof(emac_share));
  if (!sh) return EMAC_ERR_MALLOC;
  for (pc = 0; pc < p->npieces; pc++) {
    const long off = p->chunk_off[(size_t)pc * R + pos], len = p->chunk_len[(size_t)pc * R + pos];
    for (u = 0; u < N; u++) { /* task u's share (program_nodes: mo, ml), line by line */
      const long mo = off + len * u / N, ml = off + len * (u + 1) / N - mo;
      if (flow == 2 && ml > 0) { /* halving: one tree for the whole share, leaves by bit-reversed task */
        emac_share *s = &sh[n++];
        s->off = mo;
        s->len = ml;
        s->node = ns.task_node[u];
        s->nleaf = N;
        s->nlev = K;
        for (i = 0; i < N; i++) {
          int b, r = 0;
          for (b = 0; b < K; b++) r |= ((i >> b) & 1) << (K - 1 - b);
          s->leaf_node[i] = ns.task_node[r];
        }
        continue;
      }
      for (t = 0; t < N && ml > 0; t++) {
        long a, b, so, sl;
        emac_share *s;
        task_lines(&ns, count, t, t + 1, &a, &b);
        clip(a, b, mo, mo + ml, &so, &sl);
        if (sl <= 0) continue;
        s = &sh[n++];
        s->off = so;
        s->len = sl;
        s->node = ns.task_node[u];
        s->nleaf = N;
        s->nlev = 1;
        s->leaf_node[0] = ns.task_node[(t + N - 1) % N];
        s->leaf_node[1] = ns.task_node[t];
        for (i = 0; i < N - 2; i++) s->leaf_node[2 + i] = ns.task_node[(t + i + 1) % N];
      }
    }
  }
  *out = sh;
  *nout = n;
  return 0;
}

static int program_nodes(const emac_plan *p, const emac_node_sched *ns, int node, int me, long send_phase, long count,
                         emac_p2p **ops_out, int *nops_out, emac_fold **folds_out, int *nfolds_out,
                         long *staging_bytes) {
  const int K = ns ? ns->nsteps : 0, nodes = ns ? ns->nodes : 1, task = ns ? ns->node_task[node] : 0;
  const int KR = ns ? ns->nred : 0, KA = ns ? ns->nagp : 0, gm = ns ? ns->gm : 1;
  int R = p->nranks, me_pos, pc, q, t, nops = 0, nf = 0, leg, g0, st, i, nx = 0, G, Gn, j, g;
  long ts = p->tsize, total = 0;
  long *slot0, *stride, *xslot;
  emac_p2p *ops;
  emac_fold *folds;
  int halving = K > 0 && KR == 0, single;
  if (nodes < 1 || nodes > EMAC_MAX_NODES || node < 0 || node >= nodes || me < 0 || me >= R) return EMAC_ERR_ARG;
  for (st = 0; st < K; st++) {
    nx += ns->radix[st] - 1;
    halving &= ns->radix[st] == 2;
  }
  for (j = 0; j < KR; j++) nx += ns->red_radix[j] - 1;
  for (j = 0; j < KA; j++) {
    nx += ns->agp_radix[j] - 1; /* (bounds the copy ops below) */
    halving &= ns->agp_radix[j] == 2;
  }
  halving &= KA == K; /* the halves come back in K radix-2 copying steps */
  single = !halving && K == 1 && KR == 0; /* one reduce-scatter step over every node */
  me_pos = p->rank_pos[me];
  g0 = node * R; /* global rank of this node's first rank */
  slot0 = (long *)malloc(sizeof(long) * (size_t)p->npieces);
  stride = (long *)malloc(sizeof(long) * (size_t)p->npieces);
  xslot = (long *)malloc(sizeof(long) * (size_t)p->npieces * (size_t)(nx > 0 ? nx : 1));
  ops = (emac_p2p *)malloc(sizeof(emac_p2p) * (size_t)(4 * p->npieces * R + 4 * nx * p->npieces + 1));
  folds = (emac_fold *)calloc((size_t)((1 + K + KR + nodes) * p->npieces) + 1, sizeof(emac_fold));
  if (!slot0 || !stride || !xslot || !ops || !folds) {
    free(slot0);
    free(stride);
    free(xslot);
    free(ops);
    free(folds);
    return EMAC_ERR_MALLOC;
  }
  for (pc = 0; pc < p->npieces; pc++) {
    long off = p->chunk_off[(size_t)pc * R + me_pos], len = p->chunk_len[(size_t)pc * R + me_pos];
    long phase = (send_phase + off * ts) & 15;
    stride[pc] = ((len * ts + 15) / 16) * 16 + 16;
    slot0[pc] = total + phase;
    total += (long)(R - 1) * stride[pc];
  }
  /* node steps: one slot per piece, step and column peer for that peer's partial of the lines this
     task keeps (inside this rank's chunk), at the 16-byte phase those lines have in the receive
     buffer (send_phase stands for it) */
  for (pc = 0; pc < p->npieces; pc++) {
    const long off = p->chunk_off[(size_t)pc * R + me_pos], len = p->chunk_len[(size_t)pc * R + me_pos];
    int x = 0;
    long hlo = off, hn = len;
    for (G = nodes, st = 0; st < K; G /= ns->radix[st], st++) {
      long a, b, ko, kl;
      Gn = G / ns->radix[st];
      task_lines(ns, count, task / Gn * Gn, task / Gn * Gn + Gn, &a, &b);
      clip(a, b, off, off + len, &ko, &kl);
      if (halving) { /* the half of the current range this node keeps (see below) */
        const int bit = (task >> (K - 1 - st)) & 1;
        const long h0 = (hn + 1) / 2;
        if (bit) hlo += h0;
        hn = bit ? hn - h0 : h0;
        ko = hlo;
        kl = hn;
      }
      if (single) { /* this task's share of the chunk (see below) */
        ko = off + len * task / nodes;
        kl = off + len * (task + 1) / nodes - ko;
      }
      for (i = 0; i < ns->radix[st] - 1; i++) {
        total = (total + 15) / 16 * 16;
        xslot[(size_t)pc * nx + x++] = total + ((send_phase + ko * ts) & 15);
        total += ((kl * ts + 15) / 16) * 16 + 16;
      }
    }
    for (j = 0; j < KR; j++) { /* the allgather steps that reduce: every line of the gm group */
      long a, b, ko, kl;
      task_lines(ns, count, task / gm * gm, task / gm * gm + gm, &a, &b);
      clip(a, b, off, off + len, &ko, &kl);
      for (i = 0; i < ns->red_radix[j] - 1; i++) {
        total = (total + 15) / 16 * 16;
        xslot[(size_t)pc * nx + x++] = total + ((send_phase + ko * ts) & 15);
        total += ((kl * ts + 15) / 16) * 16 + 16;
      }
    }
  }
#define SLOT(pc, q) (slot0[pc] + (long)(((q) - me - 1 + R) % R) * stride[pc])
  for (leg = 0; leg < 2; leg++) {
    for (pc = 0; pc < p->npieces; pc++) {
      long myoff = p->chunk_off[(size_t)pc * R + me_pos] * ts, mylen = p->chunk_len[(size_t)pc * R + me_pos] * ts;
      for (q = 0; q < R; q++) {
        long qoff, qlen;
        if (q == me) continue;
        qoff = p->chunk_off[(size_t)pc * R + p->rank_pos[q]] * ts;
        qlen = p->chunk_len[(size_t)pc * R + p->rank_pos[q]] * ts;
        if (leg == 0) {
          if (qlen > 0) ops[nops++] = (emac_p2p){EMAC_LEG_RS, g0 + q, 1, EMAC_BUF_SEND, qoff, qlen, 0};
          if (mylen > 0) ops[nops++] = (emac_p2p){EMAC_LEG_RS, g0 + q, 0, EMAC_BUF_STAGE, SLOT(pc, q), mylen, 0};
        } else {
          if (mylen > 0) ops[nops++] = (emac_p2p){EMAC_LEG_AG, g0 + q, 1, EMAC_BUF_RECV, myoff, mylen, 0};
          if (qlen > 0) ops[nops++] = (emac_p2p){EMAC_LEG_AG, g0 + q, 0, EMAC_BUF_RECV, qoff, qlen, 0};
        }
      }
    }
  }
  for (pc = 0; pc < p->npieces; pc++) {
    long off = p->chunk_off[(size_t)pc * R + me_pos], len = p->chunk_len[(size_t)pc * R + me_pos];
    emac_fold *f = &folds[nf];
    if (len <= 0) continue;
    f->piece = pc;
    f->offset = off * ts;
    f->count = len;
    f->nleaf = R;
    f->leg = EMAC_LEG_FOLD;
    for (t = 0; t < R; t++) {
      q = p->leaf_rank[me_pos][t];
      f->buf[t] = q == me ? EMAC_BUF_SEND : EMAC_BUF_STAGE;
      f->loff[t] = q == me ? off * ts : SLOT(pc, q);
    }
    nf++;
  }
#undef SLOT
  /* the inter-node steps (allreduce_recursive.c:248-347). Step st splits each task group of G
     tasks into radix sub-groups of Gn; task `task` keeps the lines of its sub-group and trades
     with its column peers (task + Gn * (i + 1)) % G in its group, i = 0 .. radix - 2 (:261-316),
     which are nodes task_node[] (same rank `me` there). The kept lines' fold follows the
     accumulator order raw_code.c:270-340 gives allreduce_core's lines (r_i = column peer i's
     partial, own = this node's):
       a middle step:            own, r_0, ..., r_{p-1}   (reducefrom line+3lb.. into 2lb, :283-293)
       the first (not last):     r_0, own, r_1, ...       (r_0 received into 2lb, then the own line)
       the last:                 r_{p-1}, own, r_0, ..., r_{p-2}  (r_{p-1} received into lb, :318-343)
     -- for SUM only the association matters (a + b == b + a). */
  /* One port per step over 2^k nodes: every value is a balanced pairwise tree (a + b == b + a at
     each step), the same whichever task of a pair computes it, so the lines need not be followed:
     step st pairs task t with t ^ 2^(K-1-st) (allreduce_core, :261-284), the owned range halves
     at every step (the task with that bit clear keeps the lower half) and every rank of a node
     carries an equal share. */
  for (st = 0; halving && st < K; st++)
    for (pc = 0; pc < p->npieces; pc++) {
      long lo = p->chunk_off[(size_t)pc * R + me_pos], n = p->chunk_len[(size_t)pc * R + me_pos];
      long hoff[2], hlen[2];
      const int tb = K - 1 - st, partner = ns->task_node[task ^ (1 << tb)] * R + me, bit = (task >> tb) & 1,
                lg = st << EMAC_LEG_STEP_SHIFT;
      const int la = (K - 1 - st) << EMAC_LEG_STEP_SHIFT; /* its allgather step: the reverse order */
      int s2;
      for (s2 = 0; s2 < st; s2++) { /* this step's range */
        const long h0 = (n + 1) / 2, b2 = (task >> (K - 1 - s2)) & 1;
        if (b2) lo += h0;
        n = b2 ? n - h0 : h0;
      }
      hoff[0] = lo;
      hlen[0] = (n + 1) / 2;
      hoff[1] = lo + hlen[0];
      hlen[1] = n - hlen[0];
      if (hlen[1 - bit] > 0)
        ops[nops++] = (emac_p2p){EMAC_LEG_NODES_RS | lg, partner, 1, EMAC_BUF_RECV, hoff[1 - bit] * ts, hlen[1 - bit] * ts, 0};
      if (hlen[bit] > 0) {
        emac_fold *f = &folds[nf++];
        /* raw_code.c's accumulator: the partner's partial first at the first and the last step,
           the own one in between */
        const int own = st > 0 && st < K - 1 ? 0 : 1;
        ops[nops++] = (emac_p2p){EMAC_LEG_NODES_RS | lg, partner, 0, EMAC_BUF_STAGE, xslot[(size_t)pc * nx + st],
                                 hlen[bit] * ts, 0};
        f->piece = pc;
        f->offset = hoff[bit] * ts;
        f->count = hlen[bit];
        f->nleaf = 2;
        f->leg = EMAC_LEG_NODES_FOLD | lg;
        f->buf[own] = EMAC_BUF_RECV;
        f->loff[own] = hoff[bit] * ts;
        f->buf[1 - own] = EMAC_BUF_STAGE;
        f->loff[1 - own] = xslot[(size_t)pc * nx + st];
        ops[nops++] = (emac_p2p){EMAC_LEG_NODES_AG | la, partner, 1, EMAC_BUF_RECV, hoff[bit] * ts, hlen[bit] * ts, 0};
      }
      if (hlen[1 - bit] > 0)
        ops[nops++] = (emac_p2p){EMAC_LEG_NODES_AG | la, partner, 0, EMAC_BUF_RECV, hoff[1 - bit] * ts, hlen[1 - bit] * ts, 0};
    }
  /* One reduce-scatter step over every node (N(-(N-1) ...)): every element's value is ONE fold
     of the N node partials, in the order its line's task gives (r_{N-2}, own, r_0, ..., r_{N-3}
     with r_i = task (l + i + 1) mod N, the last-step rule below), whichever node computes it. So
     the work is shared out evenly instead: task t folds the t-th N-th of every rank's chunk, cut
     at the line boundaries inside it, each piece with its line's leaf order; the finished shares
     go to every node in the first copying allgather leg. Every rank sends and receives
     (N-1)/N of its chunk each way. */
  for (pc = 0; single && pc < p->npieces; pc++) {
    const long off = p->chunk_off[(size_t)pc * R + me_pos], len = p->chunk_len[(size_t)pc * R + me_pos];
    const long mo = off + len * task / nodes, ml = off + len * (task + 1) / nodes - mo;
    int u, x;
    for (u = 0, x = 0; u < nodes; u++) { /* the other tasks' shares to them, their partials of mine */
      const long uo = off + len * u / nodes, ul = off + len * (u + 1) / nodes - uo;
      const int gp = ns->task_node[u] * R + me;
      if (u == task) continue;
      if (ul > 0) ops[nops++] = (emac_p2p){EMAC_LEG_NODES_RS, gp, 1, EMAC_BUF_RECV, uo * ts, ul * ts, 0};
      if (ml > 0) ops[nops++] = (emac_p2p){EMAC_LEG_NODES_RS, gp, 0, EMAC_BUF_STAGE, xslot[(size_t)pc * nx + x], ml * ts, 0};
      x++;
    }
    for (t = 0; t < nodes && ml > 0; t++) { /* my share, line by line */
      long a, b, so, sl;
      int order[EMAC_MAX_NODES], n = 0, l;
      emac_fold *f;
      task_lines(ns, count, t, t + 1, &a, &b);
      clip(a, b, mo, mo + ml, &so, &sl);
      if (sl <= 0) continue;
      order[n++] = (t + nodes - 1) % nodes;
      order[n++] = t;
      for (i = 0; i < nodes - 2; i++) order[n++] = (t + i + 1) % nodes;
      f = &folds[nf++];
      f->piece = pc;
      f->offset = so * ts;
      f->count = sl;
      f->nleaf = nodes;
      f->leg = EMAC_LEG_NODES_FOLD;
      for (l = 0; l < nodes; l++) {
        const int u2 = order[l]; /* the task whose partial this leaf is */
        f->buf[l] = u2 == task ? EMAC_BUF_RECV : EMAC_BUF_STAGE;
        f->loff[l] = u2 == task ? so * ts : xslot[(size_t)pc * nx + (u2 < task ? u2 : u2 - 1)] + (so - mo) * ts;
      }
    }
    for (u = 0; u < nodes; u++) { /* the finished shares, to and from every node */
      const long uo = off + len * u / nodes, ul = off + len * (u + 1) / nodes - uo;
      const int gp = ns->task_node[u] * R + me;
      if (u == task) continue;
      if (ml > 0) ops[nops++] = (emac_p2p){EMAC_LEG_NODES_AG, gp, 1, EMAC_BUF_RECV, mo * ts, ml * ts, 0};
      if (ul > 0) ops[nops++] = (emac_p2p){EMAC_LEG_NODES_AG, gp, 0, EMAC_BUF_RECV, uo * ts, ul * ts, 0};
    }
  }
  /* otherwise the lines are followed as the reference lays them out */
  for (G = nodes, st = 0; !halving && !single && st < K; G /= ns->radix[st], st++) {
    const int rad = ns->radix[st], lg = st << EMAC_LEG_STEP_SHIFT, last = st == K - 1;
    int xs = 0, s2;
    Gn = G / rad;
    for (s2 = 0; s2 < st; s2++) xs += ns->radix[s2] - 1; /* this step's first staging slot */
    for (pc = 0; pc < p->npieces; pc++) {
      const long off = p->chunk_off[(size_t)pc * R + me_pos], len = p->chunk_len[(size_t)pc * R + me_pos];
      long a, b, ko, kl;
      int peer_task[EMAC_MAX_NODES];
      task_lines(ns, count, task / Gn * Gn, task / Gn * Gn + Gn, &a, &b);
      clip(a, b, off, off + len, &ko, &kl);
      for (i = 0; i < rad - 1; i++) peer_task[i] = (task + Gn * (i + 1)) % G + task / G * G;
      for (i = 0; i < rad - 1; i++) { /* the peer's sub-group's lines to it, its partial of mine from it */
        const int gp = ns->task_node[peer_task[i]] * R + me;
        long po, pl;
        task_lines(ns, count, peer_task[i] / Gn * Gn, peer_task[i] / Gn * Gn + Gn, &a, &b);
        clip(a, b, off, off + len, &po, &pl);
        if (pl > 0) ops[nops++] = (emac_p2p){EMAC_LEG_NODES_RS | lg, gp, 1, EMAC_BUF_RECV, po * ts, pl * ts, 0};
        if (kl > 0)
          ops[nops++] = (emac_p2p){EMAC_LEG_NODES_RS | lg, gp, 0, EMAC_BUF_STAGE, xslot[(size_t)pc * nx + xs + i], kl * ts, 0};
      }
      if (kl > 0) {
        emac_fold *f = &folds[nf++];
        int order[EMAC_MAX_NODES], n = 0;
        /* leaf order: -1 = own, i = column peer i */
        if (last) {
          order[n++] = rad - 2;
          order[n++] = -1;
          for (i = 0; i < rad - 2; i++) order[n++] = i;
        } else if (st == 0) {
          order[n++] = 0;
          order[n++] = -1;
          for (i = 1; i < rad - 1; i++) order[n++] = i;
        } else {
          order[n++] = -1;
          for (i = 0; i < rad - 1; i++) order[n++] = i;
        }
        f->piece = pc;
        f->offset = ko * ts;
        f->count = kl;
        f->nleaf = rad;
        f->leg = EMAC_LEG_NODES_FOLD | lg;
        for (t = 0; t < rad; t++) {
          f->buf[t] = order[t] < 0 ? EMAC_BUF_RECV : EMAC_BUF_STAGE;
          f->loff[t] = order[t] < 0 ? ko * ts : xslot[(size_t)pc * nx + xs + order[t]];
        }
      }
    }
  }
  /* the allgather steps that still reduce (allreduce_recursive.c:348-403): while the block g of
     an allgather radix is smaller than gm, every task sends all lines of its gm group to the
     tasks (t + g (i + 1)) mod gnext of its block and folds what comes back, in its own order --
     the first step of all (no reduce-scatter step before): r_0, own, r_1, ...; any later one:
     own, r_0, ... -- so the tasks of a block may keep differently associated sums */
  for (j = 0, g = 1; !halving && j < KR; g *= ns->red_radix[j], j++) {
    const int rad = ns->red_radix[j], gnext = g * rad, xst = K + j, lg = xst << EMAC_LEG_STEP_SHIFT;
    int xs = 0, s2, peer_task[EMAC_MAX_NODES];
    for (s2 = 0; s2 < K; s2++) xs += ns->radix[s2] - 1;
    for (s2 = 0; s2 < j; s2++) xs += ns->red_radix[s2] - 1;
    for (i = 0; i < rad - 1; i++) peer_task[i] = (task + g * (i + 1)) % gnext + task / gnext * gnext;
    for (pc = 0; pc < p->npieces; pc++) {
      const long off = p->chunk_off[(size_t)pc * R + me_pos], len = p->chunk_len[(size_t)pc * R + me_pos];
      long a, b, ho, hl;
      task_lines(ns, count, task / gm * gm, task / gm * gm + gm, &a, &b);
      clip(a, b, off, off + len, &ho, &hl);
      if (hl <= 0) continue;
      for (i = 0; i < rad - 1; i++) {
        const int gp = ns->task_node[peer_task[i]] * R + me;
        ops[nops++] = (emac_p2p){EMAC_LEG_NODES_RS | lg, gp, 1, EMAC_BUF_RECV, ho * ts, hl * ts, 0};
        ops[nops++] = (emac_p2p){EMAC_LEG_NODES_RS | lg, gp, 0, EMAC_BUF_STAGE, xslot[(size_t)pc * nx + xs + i], hl * ts, 0};
      }
      {
        emac_fold *f = &folds[nf++];
        int order[EMAC_MAX_NODES], n = 0;
        if (K == 0 && j == 0) {
          order[n++] = 0;
          order[n++] = -1;
          for (i = 1; i < rad - 1; i++) order[n++] = i;
        } else {
          order[n++] = -1;
          for (i = 0; i < rad - 1; i++) order[n++] = i;
        }
        f->piece = pc;
        f->offset = ho * ts;
        f->count = hl;
        f->nleaf = rad;
        f->leg = EMAC_LEG_NODES_FOLD | lg;
        for (t = 0; t < rad; t++) {
          f->buf[t] = order[t] < 0 ? EMAC_BUF_RECV : EMAC_BUF_STAGE;
          f->loff[t] = order[t] < 0 ? ho * ts : xslot[(size_t)pc * nx + xs + order[t]];
        }
      }
    }
  }
  /* the allgather steps that copy (:404-437), block g from gm up: every task sends the lines of
     its g-block to the tasks (t + g (i + 1)) mod gnext of its block and receives from each of
     them the lines of its g-block -- the task at its own position there (NODES_AG | step << 8,
     run in this order) */
  for (j = 0, g = gm; !halving && !single && j < KA; g *= ns->agp_radix[j], j++) {
    const int rad = ns->agp_radix[j], gnext = g * rad, lg = j << EMAC_LEG_STEP_SHIFT;
    for (pc = 0; pc < p->npieces; pc++) {
      const long off = p->chunk_off[(size_t)pc * R + me_pos], len = p->chunk_len[(size_t)pc * R + me_pos];
      long a, b, mo, ml;
      task_lines(ns, count, task / g * g, task / g * g + g, &a, &b);
      clip(a, b, off, off + len, &mo, &ml);
      for (i = 0; i < rad - 1; i++) {
        const int pt = (task + g * (i + 1)) % gnext + task / gnext * gnext, gp = ns->task_node[pt] * R + me;
        long po, pl;
        task_lines(ns, count, pt / g * g, pt / g * g + g, &a, &b);
        clip(a, b, off, off + len, &po, &pl);
        if (ml > 0) ops[nops++] = (emac_p2p){EMAC_LEG_NODES_AG | lg, gp, 1, EMAC_BUF_RECV, mo * ts, ml * ts, 0};
        if (pl > 0) ops[nops++] = (emac_p2p){EMAC_LEG_NODES_AG | lg, gp, 0, EMAC_BUF_RECV, po * ts, pl * ts, 0};
      }
    }
  }
  free(slot0);
  free(stride);
  free(xslot);
  *ops_out = ops;
  *nops_out = nops;
  *folds_out = folds;
  *nfolds_out = nf;
  *staging_bytes = total;
  return EMAC_OK;
}
