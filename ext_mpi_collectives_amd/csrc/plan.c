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
   (src/core/ports_groups.c:18-35): f0 = split, then negative reduce-scatter radices,
   then positive allgather radices. */
int emac_parse_copyin(const char *s, emac_copyin *out) {
  long v[2 + 2 * EMAC_MAX_LEVELS];
  int n = 0, i;
  const char *c = s;
  char *end;
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
  out->split = (int)v[1];
  for (i = 2; i < n; i++) {
    if (v[i] < 0) {
      if (out->nag) return EMAC_ERR_ARG; /* reduce-scatter radices come first */
      if (out->nrs >= EMAC_MAX_LEVELS) return EMAC_ERR_UNSUPPORTED;
      out->rs[out->nrs++] = (int)-v[i];
    } else {
      if (out->nag >= EMAC_MAX_LEVELS) return EMAC_ERR_UNSUPPORTED;
      out->ag[out->nag++] = (int)v[i];
    }
  }
  return EMAC_OK;
}

void emac_default_copyin(int nranks, emac_copyin *out) {
  memset(out, 0, sizeof(*out));
  out->method = 6;
  out->split = 1;
  out->nrs = 1;
  out->rs[0] = nranks;
  out->nag = 1;
  out->ag[0] = nranks;
}

int emac_validate_copyin(const emac_copyin *c, int nranks) {
  int i, prs = 1, pag = 1;
  if (c->method != 6 && c->method != 9) return EMAC_ERR_UNSUPPORTED;
  if (c->split == 0 || c->nrs < 1) return EMAC_ERR_ARG;
  if (c->split > EMAC_MAX_PIECES) return EMAC_ERR_UNSUPPORTED;
  for (i = 0; i < c->nrs; i++) {
    if (c->rs[i] < 2) return EMAC_ERR_ARG;
    prs *= c->rs[i];
  }
  for (i = 0; i < c->nag; i++) {
    if (c->ag[i] < 2) return EMAC_ERR_UNSUPPORTED; /* a "1" opens a multi-socket sub-split */
    pag *= c->ag[i];
  }
  /* every radix chain must cover the node exactly: the reference silently produces a partial
     reduction otherwise; here it is rejected */
  if (prs != nranks) return EMAC_ERR_ARG;
  if (c->nag && pag != nranks) return EMAC_ERR_ARG;
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

/* Leaves, in evaluation order, of the value position p holds for its chunk after
   reduce-scatter step s. Step s combines f[s] partials of step s-1: p's own first, then
   the partners of p's radix group in ascending group index. */
static void tree_leaves(const emac_plan *pl, int s, int p, int *out, int *k) {
  int gb = 1, i, q, base, qme;
  if (s < 0) {
    out[(*k)++] = pl->pos_rank[p];
    return;
  }
  for (i = s + 1; i < pl->cfg.nrs; i++) gb *= pl->cfg.rs[i];
  base = (p / (gb * pl->cfg.rs[s])) * (gb * pl->cfg.rs[s]);
  qme = (p - base) / gb;
  tree_leaves(pl, s - 1, p, out, k);
  for (q = 0; q < pl->cfg.rs[s]; q++)
    if (q != qme) tree_leaves(pl, s - 1, base + gb * q + p % gb, out, k);
}

static void build_codes(const emac_copyin *c, emac_codes *codes) {
  int t, l;
  memset(codes, 0, sizeof(*codes));
  codes->nlev = c->nrs;
  codes->nleaf = 1;
  for (l = 0; l < c->nrs; l++) codes->nleaf *= c->rs[l];
  for (t = 0; t < codes->nleaf; t++) {
    int rem = t, closing = 1;
    for (l = 0; l < c->nrs; l++) {
      int d = rem % c->rs[l];
      rem /= c->rs[l];
      if (d == 0) codes->first[t] |= (unsigned char)(1u << l);
      if (closing && d == c->rs[l] - 1)
        codes->close[t]++;
      else
        closing = 0;
    }
  }
}

int emac_plan_build(emac_plan *p, int nranks, long count, int dtype, int op, const emac_copyin *cfg) {
  int i, pc, k;
  long frac = 0;
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
    p->cfg.nrs = 1;
    p->cfg.rs[0] = 1;
    p->cfg.nag = 0;
    p->cfg.split = 1;
  } else {
    int rc = emac_validate_copyin(&p->cfg, nranks);
    if (rc) return rc;
  }
  for (i = 0; i < nranks; i++) p->pos_rank[i] = i;
  position_order(nranks, p->cfg.nrs, p->cfg.rs, p->pos_rank);
  for (i = 0; i < nranks; i++) p->rank_pos[p->pos_rank[i]] = i;

  if (p->cfg.split > 0) {
    p->npieces = p->cfg.split;
  } else {
    p->npieces = 1;
    frac = -(long)p->cfg.split;
  }
  p->chunk_off = (long *)malloc(sizeof(long) * (size_t)p->npieces * nranks);
  p->chunk_len = (long *)malloc(sizeof(long) * (size_t)p->npieces * nranks);
  if (!p->chunk_off || !p->chunk_len) {
    emac_plan_free(p);
    return EMAC_ERR_MALLOC;
  }
  for (pc = 0; pc < p->npieces; pc++) {
    /* piece pc of an equal split (reduce_copyin.c:1035-1044), then its own partition */
    long plen = count, poff = 0;
    if (p->cfg.split > 0) {
      long base = count / p->cfg.split, extra = count % p->cfg.split;
      plen = base + (pc < extra);
      poff = base * pc + (pc < extra ? pc : extra);
    }
    partition(nranks, plen, frac, p->chunk_off + (size_t)pc * nranks, p->chunk_len + (size_t)pc * nranks);
    for (i = 0; i < nranks; i++) p->chunk_off[(size_t)pc * nranks + i] += poff;
  }
  for (i = 0; i < nranks; i++) {
    k = 0;
    if (nranks == 1)
      p->leaf_rank[0][k++] = 0;
    else
      tree_leaves(p, p->cfg.nrs - 1, i, p->leaf_rank[i], &k);
  }
  if (nranks == 1) {
    memset(&p->codes, 0, sizeof(p->codes));
    p->codes.nlev = 1;
    p->codes.nleaf = 1;
    p->codes.first[0] = 1;
    p->codes.close[0] = 1;
  } else {
    build_codes(&p->cfg, &p->codes);
  }
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
  int R = p->nranks, me_pos = p->rank_pos[me], pc, q, t, nops = 0, nf = 0, leg;
  long ts = p->tsize, total = 0;
  long *slot0 = (long *)malloc(sizeof(long) * (size_t)p->npieces);
  long *stride = (long *)malloc(sizeof(long) * (size_t)p->npieces);
  emac_p2p *ops = (emac_p2p *)malloc(sizeof(emac_p2p) * (size_t)(4 * p->npieces * R + 1));
  emac_fold *folds = (emac_fold *)calloc((size_t)p->npieces + 1, sizeof(emac_fold));
  if (!slot0 || !stride || !ops || !folds) {
    free(slot0);
    free(stride);
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
          if (qlen > 0) ops[nops++] = (emac_p2p){EMAC_LEG_RS, q, 1, EMAC_BUF_SEND, qoff, qlen};
          if (mylen > 0) ops[nops++] = (emac_p2p){EMAC_LEG_RS, q, 0, EMAC_BUF_STAGE, SLOT(pc, q), mylen};
        } else {
          if (mylen > 0) ops[nops++] = (emac_p2p){EMAC_LEG_AG, q, 1, EMAC_BUF_RECV, myoff, mylen};
          if (qlen > 0) ops[nops++] = (emac_p2p){EMAC_LEG_AG, q, 0, EMAC_BUF_RECV, qoff, qlen};
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
    for (t = 0; t < R; t++) {
      q = p->leaf_rank[me_pos][t];
      f->buf[t] = q == me ? EMAC_BUF_SEND : EMAC_BUF_STAGE;
      f->loff[t] = q == me ? off * ts : SLOT(pc, q);
    }
    nf++;
  }
#undef SLOT
  free(slot0);
  free(stride);
  *ops_out = ops;
  *nops_out = nops;
  *folds_out = folds;
  *nfolds_out = nf;
  *staging_bytes = total;
  return EMAC_OK;
}
