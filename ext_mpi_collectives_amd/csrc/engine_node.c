/*
 * engine_node.c -- the NODE form: every node rank's buffers in this process on one device, one
 * fold launch per Start (copy-in and copy-out fused); the host-side layout self-check of the planner / layout pair (engine_int.h).
 */
#include "engine_int.h"

/* The NODE form's buckets restricted to message elements [lo, hi): every owner chunk (piece pc,
   position c) clipped to the range; leaves in the plan's fold order, fan-out into every rank's
   receive buffer. Returns the number written to b (capacity npieces * nranks). */
static int node_buckets(const emac_handle *h, long lo, long hi, emac_bucket *b) {
  const int R = h->plan.nranks;
  int pc, c, t, r, nb = 0;
  for (pc = 0; pc < h->plan.npieces; pc++) {
    for (c = 0; c < R; c++) {
      const long off = h->plan.chunk_off[(size_t)pc * R + c], len = h->plan.chunk_len[(size_t)pc * R + c];
      const long a = off > lo ? off : lo, e = off + len < hi ? off + len : hi;
      emac_bucket *bk = &b[nb];
      if (len <= 0 || a >= e) continue;
      memset(bk, 0, sizeof(*bk));
      for (t = 0; t < R; t++) bk->src[t] = h->dsend[h->plan.leaf_rank[c][t]];
      for (r = 0; r < R; r++) bk->dst[r] = h->drecv[r];
      bk->ndst = R;
      place_bucket(bk, R, a, e - a, h->plan.tsize);
      nb++;
    }
  }
  return nb;
}

int ext_mpi_amd_node_allreduce_init(int nranks, const void *const *sendbufs, void *const *recvbufs, long count,
                                    int dtype, int op, const char *copyin, int *handle) {
  emac_handle *h;
  emac_copyin cfg;
  emac_bucket *b = NULL;
  int rc, r, nb = 0;
  if (!handle || !sendbufs || !recvbufs || nranks < 1 || nranks > EMAC_MAX_RANKS || count < 0)
    return EMAC_ERR_ARG;
  *handle = -1;
  if ((rc = parse_cfg(copyin, nranks, &cfg))) return rc;
  if (emac_gpu_device_count() <= 0) return EMAC_ERR_DEVICE;
  h = (emac_handle *)calloc(1, sizeof(emac_handle));
  if (!h) return EMAC_ERR_MALLOC;
  h->kind = KIND_NODE;
  if ((rc = emac_plan_build(&h->plan, nranks, count, dtype, op, &cfg))) goto fail;
  emac_gpu_get_device(&h->device);
  h->bytes = (size_t)count * (size_t)h->plan.tsize;
  h->nbuf = nranks;
  h->nsrc = nranks;
  h->fan = nranks > 1;
  for (r = 0; r < nranks; r++)
    if ((rc = map_buffers(h, r, sendbufs[r], recvbufs[r]))) goto fail;
  b = (emac_bucket *)calloc((size_t)h->plan.npieces * nranks, sizeof(emac_bucket));
  if (!b) {
    rc = EMAC_ERR_MALLOC;
    goto fail;
  }
  nb = node_buckets(h, 0, count, b);
  if ((rc = upload_buckets(h, b, nb))) goto fail;
  free(b);
  b = NULL;
  if ((rc = emac_gpu_stream_create(&h->stream))) goto fail;
  if ((rc = finish_init(h, handle))) goto fail;
  return 0;
fail:
  free(b);
  handle_release(h);
  return rc;
}

/* One owner chunk as a persistent handle: the persistent form of the device C-ABI's
   ext_mpi_amd_gpu_copy_reduce (the reference launches one such descriptor per GPU stream,
   byte_code.c:936-992). Leaves are folded in the given order, left to right. */
int ext_mpi_amd_fold_init(int nsrc, const void *const *srcs, int ndst, void *const *dsts, long count, int dtype,
                          int op, int *handle) {
  emac_handle *h;
  emac_bucket b;
  emac_copyin cfg;
  int rc, i;
  if (!handle || !srcs || nsrc < 1 || nsrc > EMAC_MAX_RANKS || ndst < 1 || count < 0) return EMAC_ERR_ARG;
  if (ndst > 1 && ndst != nsrc) return EMAC_ERR_UNSUPPORTED; /* fan-out width is 1 or nsrc */
  *handle = -1;
  if (emac_gpu_device_count() <= 0) return EMAC_ERR_DEVICE;
  for (i = 0; i < nsrc; i++)
    if (!emac_gpu_is_device_pointer(srcs[i])) return EMAC_ERR_ARG;
  for (i = 0; i < ndst; i++)
    if (!emac_gpu_is_device_pointer(dsts[i])) return EMAC_ERR_ARG;
  h = (emac_handle *)calloc(1, sizeof(emac_handle));
  if (!h) return EMAC_ERR_MALLOC;
  h->kind = KIND_NODE;
  /* a linear plan over nsrc leaves supplies the codes (one level, leaves in given order) */
  emac_default_copyin(nsrc, &cfg);
  if ((rc = emac_plan_build(&h->plan, nsrc, count, dtype, op, nsrc > 1 ? &cfg : NULL))) goto fail;
  emac_gpu_get_device(&h->device);
  h->nsrc = nsrc;
  h->fan = ndst > 1;
  memset(&b, 0, sizeof(b));
  for (i = 0; i < nsrc; i++) b.src[i] = srcs[i];
  for (i = 0; i < ndst; i++) b.dst[i] = dsts[i];
  b.ndst = ndst;
  place_bucket(&b, nsrc, 0, count, h->plan.tsize);
  if ((rc = upload_buckets(h, &b, count > 0 ? 1 : 0))) goto fail;
  if ((rc = emac_gpu_stream_create(&h->stream))) goto fail;
  if ((rc = finish_init(h, handle))) goto fail;
  return 0;
fail:
  handle_release(h);
  return rc;
}

/* ---- layout self-check (host only, no device): the NODE form's buckets and launch layout for
   buffers at the given 16-byte phases, with every access the kernels would make replayed on the
   host (fold_kernel tiles, fold_edge_kernel items; fold_kernel.hpp). Returns the number of
   accesses outside a buffer's [0, count) elements or destination elements not written exactly
   once per launch; -1 on a set-up error. Test infrastructure for the planner/layout pair. */
typedef struct {
  long count;
  int tsize;
  long bad;
  unsigned char *hits; /* per destination rank and element: writes seen */
} chk_state;

static long chk_elem(const void *base, const void *p, int tsize) {
  return (long)(((const char *)p - (const char *)base) / tsize);
}

static void chk_access(chk_state *st, long e, int r, int write) {
  if (e < 0 || e >= st->count) {
    if (st->bad++ < 3) fprintf(stderr, "layout check: %s of element %ld (count %ld) rank %d\n", write ? "store" : "load", e, st->count, r);
    return;
  }
  if (write) st->hits[(size_t)r * (size_t)st->count + (size_t)e]++;
}

int ext_mpi_amd_check_node_layout(int nranks, long count, int dtype, int op, const char *copyin, const int *phase,
                                  int fan) {
  emac_handle hh, *h = &hh;
  emac_copyin cfg;
  emac_bucket *b = NULL;
  emac_edge *edges = NULL;
  emac_launch L;
  chk_state st;
  int rc, r, nb, i, t, d;
  const long base_stride = 1L << 40;
  if (nranks < 1 || nranks > EMAC_MAX_RANKS || count < 0) return -1;
  memset(h, 0, sizeof(*h));
  memset(&L, 0, sizeof(L));
  if (parse_cfg(copyin, nranks, &cfg) || emac_plan_build(&h->plan, nranks, count, dtype, op, &cfg)) return -1;
  h->kind = KIND_NODE;
  h->bytes = (size_t)count * (size_t)h->plan.tsize;
  h->nbuf = h->nsrc = nranks;
  h->fan = fan ? nranks > 1 : 0;
  for (r = 0; r < nranks; r++) { /* fake, disjoint buffers at the requested 16-byte phases */
    h->dsend[r] = (void *)(base_stride * (2 * r + 1) + (phase ? phase[2 * r] : 0));
    h->drecv[r] = (void *)(base_stride * (2 * r + 2) + (phase ? phase[2 * r + 1] : 0));
  }
  b = (emac_bucket *)calloc((size_t)h->plan.npieces * nranks + 1, sizeof(emac_bucket));
  st.count = count;
  st.tsize = h->plan.tsize;
  st.bad = 0;
  st.hits = (unsigned char *)calloc((size_t)nranks * (size_t)(count + 1), 1);
  if (!b || !st.hits) {
    rc = -1;
    goto out;
  }
  nb = node_buckets(h, 0, count, b);
  if (!h->fan)
    for (i = 0; i < nb; i++) b[i].ndst = 1; /* COMM-like fan-out 1: only the first destination */
  if ((rc = emac_layout(b, nb, op, h->nsrc, emac_tree_kind(&h->plan.codes, op) == 1, h->fan, &edges, &L.nedges, &L.ntiles,
                        &L.tiles_per_bucket, &L.all_full, &L.unroll))) {
    rc = -1;
    goto out;
  }
  {
    const long EPV = 16 / h->plan.tsize, TILE = (long)EMAC_BLOCK * (L.unroll & 15);
    long tile;
    /* fold_kernel: each tile's vectors of its bucket */
    for (tile = 0; tile < L.ntiles; tile++) {
      int bi;
      long tt, v, v0, v1;
      if (L.tiles_per_bucket > 0) {
        bi = (int)(tile / L.tiles_per_bucket);
        tt = tile - (long)bi * L.tiles_per_bucket;
      } else {
        int lo = 0, hi = nb - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (b[mid].tile0 <= tile)
            lo = mid;
          else
            hi = mid - 1;
        }
        bi = lo;
        tt = tile - b[lo].tile0;
      }
      if (bi < 0 || bi >= nb) {
        st.bad++;
        continue;
      }
      v0 = tt * TILE;
      v1 = (L.all_full || (tt + 1) * TILE <= b[bi].nvec) ? v0 + TILE : b[bi].nvec;
      for (v = v0; v < v1; v++)
        for (i = 0; i < (int)EPV; i++) {
          for (t = 0; t < h->nsrc; t++) {
            /* which rank's send buffer leaf t points into (the fake bases are 2^40 apart) */
            const long bi_rank = ((long)((const char *)b[bi].src[t] - (const char *)0) / base_stride - 1) / 2;
            chk_access(&st, chk_elem(h->dsend[bi_rank], b[bi].src[t], st.tsize) + v * EPV + i, (int)bi_rank, 0);
          }
          for (d = 0; d < b[bi].ndst; d++) {
            const long dr = ((long)((const char *)b[bi].dst[d] - (const char *)0) / base_stride - 2) / 2;
            chk_access(&st, chk_elem(h->drecv[dr], b[bi].dst[d], st.tsize) + v * EPV + i, (int)dr, 1);
          }
        }
    }
    /* fold_edge_kernel items */
    for (i = 0; i < L.nedges; i++) {
      const emac_edge it = edges[i];
      const emac_bucket *bk = &b[it.bucket];
      long k, e, n = it.mode == 1 ? it.count : bk->head + bk->tail;
      for (k = 0; k < n; k++) {
        if (it.mode == 1)
          e = it.start + k;
        else
          e = k < bk->head ? k : bk->head + bk->nvec * EPV + (k - bk->head);
        e -= bk->head; /* pointers sit at element head */
        for (t = 0; t < h->nsrc; t++) {
          const long sr = ((long)((const char *)bk->src[t] - (const char *)0) / base_stride - 1) / 2;
          chk_access(&st, chk_elem(h->dsend[sr], bk->src[t], st.tsize) + e, (int)sr, 0);
        }
        for (d = 0; d < bk->ndst; d++) {
          const long dr = ((long)((const char *)bk->dst[d] - (const char *)0) / base_stride - 2) / 2;
          chk_access(&st, chk_elem(h->drecv[dr], bk->dst[d], st.tsize) + e, (int)dr, 1);
        }
      }
    }
  }
  /* every destination element written exactly once (fan-out N) / the first destination (fan 1) */
  for (r = 0; r < (h->fan ? nranks : 1); r++) {
    long e;
    for (e = 0; e < count; e++)
      if (st.hits[(size_t)r * (size_t)count + (size_t)e] != (h->fan || r == 0 ? 1 : 0)) {
        if (st.bad++ < 3)
          fprintf(stderr, "layout check: rank %d element %ld written %d times\n", r, e,
                  st.hits[(size_t)r * (size_t)count + (size_t)e]);
      }
  }
  rc = st.bad > 0x7fffffff ? 0x7fffffff : (int)st.bad;
out:
  free(edges);
  free(b);
  free(st.hits);
  emac_plan_free(&h->plan);
  return rc;
}
