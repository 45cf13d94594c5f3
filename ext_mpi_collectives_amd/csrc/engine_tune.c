/*
 * engine_tune.c -- launch-schedule tuning of a handle's fold (engine_int.h).
 */
#include "engine_int.h"

/* the candidates of emac_tune for a fold of nsrc leaves, fan-out `fan` (0 / 1), vec 16-byte vectors
   per leaf over all buckets, or 0 */
static int tune_candidates(const emac_handle *h, long vec, int *sched) {
  const char *e = getenv("EXT_MPI_AMD_AUTOTUNE");
  const char *g = getenv("EXT_MPI_AMD_GRAPH"); /* captured Starts replay one schedule */
  int n = 0;
  if ((e && atoi(e) <= 0) || (h->kind == KIND_COMM && g && atoi(g) > 0) || h->plan.op != EMAC_SUM || h->nsrc < 2 ||
      h->nsrc > 8 || h->host_direct ||
      emac_tree_kind(&h->plan.codes, h->plan.op) == 1 || (h->fan != 0 && h->fan != 1))
    return 0;
  /* fold_kernel.hpp instantiation policy: (U 2, burst), (U 4, burst), for the node fan-out (U 4,
     s_sleep 2 every 4 loads); deferred stores (kDeferShift) when every bucket has the same tile
     count: (U 2, 4 tiles) and (U 4, 4 tiles) for one destination, (U 2, 4 tiles) and, for the
     fan-out, its leaf-major form (kLeafMajor) over the linear fold or (U 4, 2 tiles) over fold
     trees. A launch of fewer than 256 groups of (U 2, 4 tiles) -- under 8 MiB per leaf -- leaves
     CUs idle under the deferred schedules; there (U 1, burst), twice the per-tile loop's
     workgroups, is offered too. (U 2, 8 tiles), compiled, is no longer offered: never kept. */
  const int small = vec < 256L * 4 * 2 * EMAC_BLOCK;
  const char *f = getenv("EXT_MPI_AMD_FOLD_SCHEDULE"); /* A/B runs: one schedule word, U | issue << 4 */
  if (f && atoi(f) > 0) {
    sched[0] = atoi(f);
    return 1;
  }
  sched[n++] = 2 | 1 << 4;
  sched[n++] = 4 | 1 << 4;
  if (h->fan) sched[n++] = 4 | 5 << 4;
  if (small) sched[n++] = 1 | 1 << 4;
  if (h->tiles_per_bucket > 0) {
    sched[n++] = 2 | (1 | 2 << 11) << 4;
    if (!h->fan)
      sched[n++] = 4 | (1 | 2 << 11) << 4;
    else if (emac_tree_kind(&h->plan.codes, h->plan.op) == 0)
      sched[n++] = 2 | (1 | 2 << 11 | 1 << 13) << 4; /* leaf-major groups: the linear fold's order only */
    else
      sched[n++] = 4 | (1 | 1 << 11) << 4;
  }
  return n;
}

int upload_buckets(emac_handle *h, emac_bucket *b, int nb) {
  emac_edge *edges = NULL;
  int rc, sched[EMAC_TUNE_MAX], nc, k, i;
  long vec = 0;
  /* (fan | EMAC_FAN_HOST: the schedule for buffers across PCIe, emac_gpu_pick_unroll) */
  if ((rc = emac_layout(b, nb, h->plan.op, h->nsrc, emac_tree_kind(&h->plan.codes, h->plan.op) == 1,
                        h->fan | (h->host_direct ? EMAC_FAN_HOST : 0),
                        &edges, &h->nedges, &h->ntiles, &h->tiles_per_bucket, &h->all_full, &h->unroll)))
    return rc;
  h->nb = nb;
  if (nb && (rc = emac_gpu_malloc((void **)&h->d_buckets, sizeof(emac_bucket) * (size_t)nb)) == 0)
    rc = emac_gpu_memcpy(h->d_buckets, b, sizeof(emac_bucket) * (size_t)nb);
  if (!rc && h->nedges && (rc = emac_gpu_malloc((void **)&h->d_edges, sizeof(emac_edge) * (size_t)h->nedges)) == 0)
    rc = emac_gpu_memcpy(h->d_edges, edges, sizeof(emac_edge) * (size_t)h->nedges);
  free(edges);
  for (i = 0; i < nb; i++) vec += b[i].nvec;
  nc = rc ? 0 : tune_candidates(h, vec, sched);
  if (!nc || vec * 16 * (h->nsrc + (h->fan ? h->nsrc : 1)) < EMAC_TUNE_MIN_BYTES) return rc;
  {
    emac_bucket *tb = (emac_bucket *)malloc(sizeof(emac_bucket) * (size_t)nb);
    if (!tb) return EMAC_ERR_MALLOC;
    h->tune.chosen = -1;
    for (k = 0; k < nc && !rc; k++) {
      emac_launch *L = &h->tune.L[k];
      memcpy(tb, b, sizeof(emac_bucket) * (size_t)nb);
      h->tune.n = k + 1; /* freed by handle_release() from here on */
      if (sched[k] == h->unroll) { /* the static pick: its upload is reused */
        L->d_buckets = h->d_buckets;
        L->nb = nb;
        L->ntiles = h->ntiles;
        L->tiles_per_bucket = h->tiles_per_bucket;
        L->all_full = h->all_full;
        L->d_edges = h->d_edges;
        L->nedges = h->nedges;
        L->unroll = h->unroll;
      } else {
        rc = emac_layout_as(tb, nb, h->plan.op, h->nsrc, 0, h->fan, sched[k], &edges, &L->nedges, &L->ntiles,
                            &L->tiles_per_bucket, &L->all_full, &L->unroll);
        if (!rc) {
          L->nb = nb;
          if ((rc = emac_gpu_malloc((void **)&L->d_buckets, sizeof(emac_bucket) * (size_t)nb)) == 0)
            rc = emac_gpu_memcpy(L->d_buckets, tb, sizeof(emac_bucket) * (size_t)nb);
          if (!rc && L->nedges && (rc = emac_gpu_malloc((void **)&L->d_edges, sizeof(emac_edge) * (size_t)L->nedges)) == 0)
            rc = emac_gpu_memcpy(L->d_edges, edges, sizeof(emac_edge) * (size_t)L->nedges);
          free(edges);
        }
      }
    }
    for (i = 0; i < nc * EMAC_TUNE_ROUNDS && !rc; i++) {
      rc = emac_gpu_event_create_timed(&h->tune.ev[i][0]);
      if (!rc) rc = emac_gpu_event_create_timed(&h->tune.ev[i][1]);
    }
    free(tb);
  }
  return rc;
}

/* The handle's fold launch (fan 0 / 1), with the schedule tuning of emac_tune. */
int fold_launch(emac_handle *h) {
  emac_tune *t = &h->tune;
  int rc, k;
  if (t->n && t->chosen < 0) {
    const int s = t->starts++, nsamples = t->n * EMAC_TUNE_ROUNDS;
    if (s >= 1 && s <= EMAC_TUNE_SPAN * nsamples) {
      /* sample p: candidate p % n on EMAC_TUNE_SPAN Starts in a row, the first untimed (it follows
         another schedule's launch), the others timed as one window */
      const int p = (s - 1) / EMAC_TUNE_SPAN, pos = (s - 1) % EMAC_TUNE_SPAN;
      const emac_launch *L = &t->L[p % t->n];
      if (pos == 1 && (rc = emac_gpu_event_record(t->ev[p][0], h->stream))) return rc;
      if ((rc = emac_gpu_fold(h->plan.dtype, h->plan.op, h->nsrc, h->fan, L->unroll, &h->plan.codes, L->d_buckets, L->nb,
                              L->ntiles, L->tiles_per_bucket, L->all_full, L->d_edges, L->nedges, h->stream)))
        return rc;
      return pos == EMAC_TUNE_SPAN - 1 ? emac_gpu_event_record(t->ev[p][1], h->stream) : 0;
    }
    if (s == EMAC_TUNE_SPAN * nsamples + 1) { /* keep the fastest: it becomes the handle's launch */
      int best = 0, i;
      for (k = 0; k < t->n; k++) t->us[k] = 1e30f;
      for (i = 0; i < nsamples; i++) {
        float us;
        if ((rc = emac_gpu_event_elapsed_us(t->ev[i][0], t->ev[i][1], &us))) return rc;
        us /= EMAC_TUNE_SPAN - 1;
        if (us < t->us[i % t->n]) t->us[i % t->n] = us;
      }
      for (k = 1; k < t->n; k++)
        if (t->us[k] < t->us[best]) best = k;
      void *old_b = h->d_buckets, *old_e = h->d_edges; /* the static pick's upload */
      if (t->L[best].d_buckets != h->d_buckets) {
        h->d_buckets = t->L[best].d_buckets;
        h->d_edges = t->L[best].d_edges;
        h->nb = t->L[best].nb;
        h->ntiles = t->L[best].ntiles;
        h->tiles_per_bucket = t->L[best].tiles_per_bucket;
        h->all_full = t->L[best].all_full;
        h->nedges = t->L[best].nedges;
        h->unroll = t->L[best].unroll;
      }
      for (k = 0; k < t->n; k++) /* every upload but the kept one; the static pick's may be a candidate's */
        if (k != best && t->L[k].d_buckets != old_b) {
          emac_gpu_free(t->L[k].d_buckets);
          emac_gpu_free(t->L[k].d_edges);
        }
      if (old_b != h->d_buckets) {
        emac_gpu_free(old_b);
        emac_gpu_free(old_e);
      }
      for (k = 0; k < t->n; k++) { /* handle_release() frees the kept launch once, as the handle's */
        t->L[k].d_buckets = h->d_buckets;
        t->L[k].d_edges = h->d_edges;
      }
      t->chosen = best;
      if (getenv("EXT_MPI_AMD_DEBUG_TUNE")) {
        char line[256];
        int at = 0;
        for (k = 0; k < t->n && at < (int)sizeof(line) - 32; k++)
          at += snprintf(line + at, sizeof(line) - (size_t)at, " U%d/%d %.1f", t->L[k].unroll & 15, t->L[k].unroll >> 4,
                         t->us[k]);
        fprintf(stderr, "ext_mpi_amd: fold schedule kept: U %d issue %d (%.1f us; %d candidates:%s)\n", h->unroll & 15,
                h->unroll >> 4, t->us[best], t->n, line);
      }
    }
  }
  return emac_gpu_fold(h->plan.dtype, h->plan.op, h->nsrc, h->fan, h->unroll, &h->plan.codes, h->d_buckets, h->nb, h->ntiles,
                       h->tiles_per_bucket, h->all_full, h->d_edges, h->nedges, h->stream);
}

int ext_mpi_amd_handle_schedule(int handle, int *unroll, int *issue, int *tuned) {
  const emac_handle *h = (handle >= 0 && handle < MAX_HANDLES) ? g_handles[handle] : NULL;
  if (!h) return EMAC_ERR_ARG;
  if (unroll) *unroll = h->unroll & 15;
  if (issue) *issue = h->unroll >> 4;
  if (tuned) *tuned = h->tune.n ? (h->tune.chosen >= 0 ? 1 : 0) : -1;
  return 0;
}

int ext_mpi_amd_handle_candidates(int handle, int *n, int *sched, int max) {
  const emac_handle *h = (handle >= 0 && handle < MAX_HANDLES) ? g_handles[handle] : NULL;
  int k;
  if (!h || !n || (max > 0 && !sched)) return EMAC_ERR_ARG;
  *n = h->tune.n;
  for (k = 0; k < h->tune.n && k < max; k++) sched[k] = h->tune.L[k].unroll;
  return 0;
}
