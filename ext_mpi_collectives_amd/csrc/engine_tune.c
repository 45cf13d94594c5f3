/*
 * engine_tune.c -- launch-schedule tuning of a handle's fold, and the per-process cache of the
 * schedules it kept (engine_int.h, emac_tune).
 */
#include "engine_int.h"

/* ---- the per-process cache of kept schedules ----
   A shape is what the fold launch depends on: the device, element type, operation, leaf count,
   fan-out form, fold tree, and the buckets' vector counts (their number, the total, the first
   bucket's and whether all are equal -- the tile layout follows from these). Handles of one shape
   run the same kernels over the same tiles, so the first handle's kept schedule serves every later
   one of the same form: the blocking front end's cached handles (one per buffer set,
   mpi_interface.c), an application's re-created persistent requests. (The bench creates all its
   rotated buffer sets before their first Start, so each of those tunes on its own; bench.py reports
   every set's kept schedule.) The key also holds the handle's form (kind, hier) and whether its
   samples were isolated: the same launch shape measured 4-20 % apart between a fold_init handle and
   a COMM rank's fold of freshly staged leaves, so neither reuses the other's schedule. Entries are
   replaced oldest first. */
_Static_assert(EXT_MPI_AMD_TUNE_MAX == EMAC_TUNE_MAX && EXT_MPI_AMD_TUNE_MAX * 3 == EMAC_TUNE_SAMPLES,
               "ext_mpi_amd_tune_info mirrors emac_tune");
#define EMAC_TUNE_CACHE 64
typedef struct {
  int used;
  emac_shape k;
  int sched;
} tune_entry;
static tune_entry g_tcache[EMAC_TUNE_CACHE];
static int g_tcache_next;

static int cache_enabled(void) {
  const char *c = getenv("EXT_MPI_AMD_TUNE_CACHE");
  const char *f = getenv("EXT_MPI_AMD_FOLD_SCHEDULE"); /* A/B runs neither read nor feed it */
  return !(c && atoi(c) <= 0) && !(f && atoi(f) > 0);
}

static void shape_key(const emac_handle *h, const emac_bucket *b, int nb, emac_shape *k) {
  int i;
  memset(k, 0, sizeof(*k));
  k->device = h->device;
  k->dtype = h->plan.dtype;
  k->op = h->plan.op;
  k->nsrc = h->nsrc;
  k->fan = h->fan;
  k->tree = emac_tree_kind(&h->plan.codes, h->plan.op);
  k->kind = h->kind;
  k->hier = h->hier;
  k->isolated = h->tune.isolated;
  k->nb = nb;
  k->vec0 = nb ? b[0].nvec : 0;
  k->uniform = 1;
  for (i = 0; i < nb; i++) {
    k->vec += b[i].nvec;
    if (b[i].nvec != k->vec0) k->uniform = 0;
  }
}

static int same_shape(const emac_shape *a, const emac_shape *k) {
  return a->device == k->device && a->dtype == k->dtype && a->op == k->op && a->nsrc == k->nsrc && a->fan == k->fan &&
         a->tree == k->tree && a->kind == k->kind && a->hier == k->hier &&
         a->isolated == k->isolated && a->nb == k->nb && a->uniform == k->uniform && a->vec == k->vec && a->vec0 == k->vec0;
}

static tune_entry *cache_find(const emac_shape *k) {
  int i;
  for (i = 0; i < EMAC_TUNE_CACHE; i++)
    if (g_tcache[i].used && same_shape(&g_tcache[i].k, k)) return &g_tcache[i];
  return NULL;
}

static void cache_store(const emac_shape *k, int sched) {
  tune_entry *e = cache_find(k);
  if (!e) {
    e = &g_tcache[g_tcache_next];
    g_tcache_next = (g_tcache_next + 1) % EMAC_TUNE_CACHE;
  }
  e->k = *k;
  e->used = 1;
  e->sched = sched;
}

int ext_mpi_amd_tune_cache_clear(void) {
  int i, n = 0;
  for (i = 0; i < EMAC_TUNE_CACHE; i++) n += g_tcache[i].used;
  memset(g_tcache, 0, sizeof(g_tcache));
  g_tcache_next = 0;
  return n;
}

/* the candidates of emac_tune for a fold of nsrc leaves, fan-out `fan` (0 / 1), vec 16-byte vectors
   per leaf over all buckets: their number, 0 (no tuning), or EMAC_ERR_UNSUPPORTED for a forced
   schedule the shape has no kernel for */
static int tune_candidates(const emac_handle *h, long vec, int *sched) {
  const char *e = getenv("EXT_MPI_AMD_AUTOTUNE");
  const char *g = getenv("EXT_MPI_AMD_GRAPH"); /* captured Starts replay one schedule */
  const int tree = emac_tree_kind(&h->plan.codes, h->plan.op);
  int n = 0;
  if ((e && atoi(e) <= 0) || (h->kind == KIND_COMM && g && atoi(g) > 0) || h->plan.op != EMAC_SUM || h->nsrc < 2 ||
      h->nsrc > 8 || h->host_direct || tree == 1 || (h->fan != 0 && h->fan != 1))
    return 0;
  /* fold_kernel.hpp instantiation policy: (U 2, burst), (U 4, burst), for the node fan-out (U 4,
     s_sleep 2 every 4 loads); deferred stores (kDeferShift) when every bucket has the same tile
     count: (U 2, 4 tiles) and (U 4, 4 tiles) for one destination; for the fan-out (U 2, 4 tiles),
     (U 4, 2 tiles) and the leaf-major form (kLeafMajor) of (U 2, 4 tiles), over a compile-time chain
     also with the opening leaves copied (kLmOpenCopy).
     (U 4, 2 tiles) had the fewest DRAM credit stalls and the shortest busy time at 256 MiB per rank
     (profiles/r03_pmc_defer/stalls_per_request.txt: write-credit stalls 0.17 per request against
     0.71-0.86 for the per-tile schedules) and is offered again for the linear fold (round 3 had
     replaced it by the leaf-major groups there). A launch of fewer than 256 groups of (U 2, 4
     tiles) -- under 8 MiB per leaf -- leaves CUs idle under the deferred schedules; there (U 1,
     burst), twice the per-tile loop's workgroups, is offered too. (U 2, 8 tiles), compiled, is no
     longer offered: never kept. Two tiles per workgroup at U 2 or U 1 ("half grid", round 4) were
     measured 13.7 us on configs[2]'s launch against 11.3 for U 4 (profiles/r04/pmc256/time_int4.json)
     and are not built. */
  const int small = vec < 256L * 4 * 2 * EMAC_BLOCK;
  const char *f = getenv("EXT_MPI_AMD_FOLD_SCHEDULE"); /* A/B runs: one schedule word, U | issue << 4 */
  if (f && atoi(f) > 0) {
    int ns, fn, known = 0;
    sched[0] = atoi(f);
    if (emac_gpu_fold_supported(h->plan.dtype, h->plan.op, h->nsrc, h->fan, tree, sched[0], h->tiles_per_bucket > 0))
      return 1;
    /* a word some other tuned shape has a kernel for (a fan-out-only schedule met by a local fold, a
       width-specific one by another leaf count): this handle keeps its static pick; a word no shape
       has a kernel for is a mistake, refused at init */
    static const int chains[] = EMAC_CHAINS;
    int c;
    for (ns = 2; ns <= 8 && !known; ns++)
      for (fn = 0; fn <= 1 && !known; fn++)
        for (c = -1; c < (int)(sizeof(chains) / sizeof(chains[0])) && !known; c++) /* the linear fold, then the chains */
          known = emac_gpu_fold_supported(h->plan.dtype, EMAC_SUM, ns, fn, c < 0 ? 0 : chains[c], sched[0], 1);
    if (!known) return EMAC_ERR_UNSUPPORTED;
    if (getenv("EXT_MPI_AMD_DEBUG_TUNE"))
      fprintf(stderr, "ext_mpi_amd: EXT_MPI_AMD_FOLD_SCHEDULE %d has no kernel for this handle (%d leaves, fan %d): "
                      "static pick kept\n", sched[0], h->nsrc, h->fan);
    return 0;
  }
  /* one destination, 4 or 8 leaves, from 8 MiB per leaf (the local fold of SURVEY 8(d), the serial
     node join's copy-in): forced one at a time on the local fold, 8 x 32 MiB -> 1, two leases, six
     passes (profiles/r06/localab/), (U 2, burst) ran 49.8-50.6 us and (U 4, 4 tiles) 48.2-49.4
     against 47.3-48.1 for the other candidates, yet the tuner had kept (U 4, 4 tiles) on two of
     four handles of one lease; they are not offered there, (U 4, 2 tiles) is (47.6-47.9 us) */
  const int big1 = !h->fan && !small && (h->nsrc == 4 || h->nsrc == 8);
  if (!big1) sched[n++] = 2 | 1 << 4;
  sched[n++] = 4 | 1 << 4;
  /* the node fan-outs of 4 and 8 ranks: (U 4, staggered) with buffer loads (fold_kernel.hpp
     kBufLoad), and from 32 MiB per leaf (U 4, burst) with buffer loads and device-scope streaming
     stores (kDevStore; below 32 MiB no gain was measured); other widths (U 4, staggered) as is */
  if (h->fan && (h->nsrc == 4 || h->nsrc == 8)) {
    sched[n++] = 4 | (5 | 1 << 15) << 4;
    if (vec * 16 >= (32L << 20)) sched[n++] = 4 | (1 | 1 << 14 | 1 << 15) << 4;
  } else if (h->fan) {
    sched[n++] = 4 | 5 << 4;
  } else if (h->nsrc == 4 || h->nsrc == 8) {  /* one destination: (U 4, staggered) with buffer loads */
    sched[n++] = 4 | (5 | 1 << 15) << 4;
  }
  if (small) sched[n++] = 1 | 1 << 4;
  /* unequal buckets (the -k fractions), at most EMAC_GROUP_MAP_MAX: the fan-out's leaf-major groups
     through the layout's bucket map (layout.c; the other deferred schedules need equal buckets) */
  if (h->tiles_per_bucket <= 0 && h->fan && h->nb > 0 && h->nb <= EMAC_GROUP_MAP_MAX) {
    sched[n++] = 2 | (1 | 2 << 11 | 1 << 13) << 4;
    if (tree > 1) sched[n++] = 2 | (1 | 2 << 11 | 1 << 13 | 1 << 16) << 4;
  }
  if (h->tiles_per_bucket > 0) {
    sched[n++] = 2 | (1 | 2 << 11) << 4;
    if (!h->fan) {
      sched[n++] = big1 ? 4 | (1 | 1 << 11) << 4 : 4 | (1 | 2 << 11) << 4;
    } else {
      sched[n++] = 4 | (1 | 1 << 11) << 4;
      /* leaf-major groups (kLeafMajor): the linear fold and the compile-time chains; a chain also in the
         form that copies each level-0 group's opening leaf into its accumulator (kLmOpenCopy): which of
         the two is faster depends on the chain (fold_kernel.hpp) */
      sched[n++] = 2 | (1 | 2 << 11 | 1 << 13) << 4;
      if (tree > 1) sched[n++] = 2 | (1 | 2 << 11 | 1 << 13 | 1 << 16) << 4;
    }
  }
  return n;
}

/* the forms whose Starts enqueue other operations between two folds (everything but the NODE form
   on device buffers): their samples time each fold alone */
static int tune_isolated(const emac_handle *h) {
  int r;
  if (h->kind != KIND_NODE || h->hier) return 1;
  for (r = 0; r < h->nbuf; r++)
    if (h->send_mirror[r] || h->recv_mirror[r]) return 1;
  return 0;
}

/* a launch of the buckets b under schedule `sched` (the buckets' tile fields are rewritten) */
static int upload_as(const emac_handle *h, emac_launch *L, emac_bucket *b, int nb, int sched) {
  emac_edge *edges = NULL;
  int rc = emac_layout_as(b, nb, h->plan.op, h->nsrc, 0, h->fan, sched, &edges, &L->nedges, &L->ntiles,
                          &L->tiles_per_bucket, &L->all_full, &L->unroll);
  if (!rc) {
    L->nb = nb;
    if ((rc = emac_gpu_malloc((void **)&L->d_buckets, sizeof(emac_bucket) * (size_t)nb)) == 0)
      rc = emac_gpu_memcpy(L->d_buckets, b, sizeof(emac_bucket) * (size_t)nb);
    if (!rc && L->nedges && (rc = emac_gpu_malloc((void **)&L->d_edges, sizeof(emac_edge) * (size_t)L->nedges)) == 0)
      rc = emac_gpu_memcpy(L->d_edges, edges, sizeof(emac_edge) * (size_t)L->nedges);
    free(edges);
  }
  return rc;
}

/* the handle's launch becomes L (its previous upload freed unless L is it) */
static void adopt(emac_handle *h, const emac_launch *L) {
  if (L->d_buckets == h->d_buckets) return;
  emac_gpu_free(h->d_buckets);
  emac_gpu_free(h->d_edges);
  h->d_buckets = L->d_buckets;
  h->d_edges = L->d_edges;
  h->nb = L->nb;
  h->ntiles = L->ntiles;
  h->tiles_per_bucket = L->tiles_per_bucket;
  h->all_full = L->all_full;
  h->nedges = L->nedges;
  h->unroll = L->unroll;
}

int upload_buckets(emac_handle *h, emac_bucket *b, int nb) {
  emac_edge *edges = NULL;
  emac_tune *t = &h->tune;
  const tune_entry *hit;
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
  /* the size gate first: a handle too small to tune never looks at a forced schedule word */
  if (rc || vec * 16 * (h->nsrc + (h->fan ? h->nsrc : 1)) < EMAC_TUNE_MIN_BYTES) return rc;
  nc = tune_candidates(h, vec, sched);
  if (nc <= 0) return nc;
  t->isolated = tune_isolated(h);
  shape_key(h, b, nb, &t->shape);
  if (cache_enabled() && (hit = cache_find(&t->shape)) != NULL) {
    /* a shape some handle has tuned: its kept schedule from Start 1, nothing measured */
    emac_launch *L = &t->L[0];
    if (hit->sched == h->unroll) {
      *L = (emac_launch){h->d_buckets, h->nb, h->ntiles, h->tiles_per_bucket, h->all_full, h->d_edges, h->nedges,
                         h->unroll};
    } else {
      emac_bucket *tb = (emac_bucket *)malloc(sizeof(emac_bucket) * (size_t)nb);
      if (!tb) return EMAC_ERR_MALLOC;
      memcpy(tb, b, sizeof(emac_bucket) * (size_t)nb);
      rc = upload_as(h, L, tb, nb, hit->sched);
      free(tb);
      if (rc) {
        emac_gpu_free(L->d_buckets);
        emac_gpu_free(L->d_edges);
        memset(L, 0, sizeof(*L));
        return rc;
      }
      adopt(h, L);
    }
    t->n = 1;
    t->chosen = 0;
    t->cached = 1;
    return 0;
  }
  {
    emac_bucket *tb = (emac_bucket *)malloc(sizeof(emac_bucket) * (size_t)nb);
    if (!tb) return EMAC_ERR_MALLOC;
    t->chosen = -1;
    for (k = 0; k < nc && !rc; k++) {
      emac_launch *L = &t->L[k];
      memcpy(tb, b, sizeof(emac_bucket) * (size_t)nb);
      t->n = k + 1; /* freed by handle_release() from here on */
      if (sched[k] == h->unroll) /* the static pick: its upload is reused */
        *L = (emac_launch){h->d_buckets, h->nb, h->ntiles, h->tiles_per_bucket, h->all_full, h->d_edges, h->nedges,
                           h->unroll};
      else
        rc = upload_as(h, L, tb, nb, sched[k]);
    }
    for (i = 0; i < nc * EMAC_TUNE_ROUNDS && !rc; i++)
      for (k = 0; k < 2 * (EMAC_TUNE_SPAN - 1) && !rc; k++)
        if (t->isolated || k == 0 || k == 2 * (EMAC_TUNE_SPAN - 1) - 1) rc = emac_gpu_event_create_timed(&t->ev[i][k]);
    free(tb);
  }
  return rc;
}

/* the kept candidate: the shortest of every candidate's samples */
static int tune_keep(emac_handle *h) {
  emac_tune *t = &h->tune;
  const int nsamples = t->n * EMAC_TUNE_ROUNDS, last = 2 * (EMAC_TUNE_SPAN - 1) - 1;
  int best = 0, i, k, rc;
  for (k = 0; k < t->n; k++) t->us[k] = 1e30f;
  for (i = 0; i < nsamples; i++) {
    float us = 0.f, part;
    if (t->isolated) {
      for (k = 0; k < EMAC_TUNE_SPAN - 1; k++) {
        if ((rc = emac_gpu_event_elapsed_us(t->ev[i][2 * k], t->ev[i][2 * k + 1], &part))) return rc;
        us += part;
      }
    } else if ((rc = emac_gpu_event_elapsed_us(t->ev[i][0], t->ev[i][last], &us))) {
      return rc;
    }
    us /= EMAC_TUNE_SPAN - 1;
    if (us < t->us[i % t->n]) t->us[i % t->n] = us;
  }
  for (k = 1; k < t->n; k++)
    if (t->us[k] < t->us[best]) best = k;
  {
    void *old_b = h->d_buckets; /* the static pick's upload */
    adopt(h, &t->L[best]);
    for (k = 0; k < t->n; k++) /* every upload but the kept one; the static pick's was freed by adopt */
      if (k != best && t->L[k].d_buckets != old_b) {
        emac_gpu_free(t->L[k].d_buckets);
        emac_gpu_free(t->L[k].d_edges);
      }
    for (k = 0; k < t->n; k++) { /* handle_release() frees the kept launch once, as the handle's */
      t->L[k].d_buckets = h->d_buckets;
      t->L[k].d_edges = h->d_edges;
    }
  }
  t->chosen = best;
  if (cache_enabled()) cache_store(&t->shape, h->unroll);
  if (getenv("EXT_MPI_AMD_DEBUG_TUNE")) {
    char line[320];
    int at = 0;
    for (k = 0; k < t->n && at < (int)sizeof(line) - 32; k++)
      at += snprintf(line + at, sizeof(line) - (size_t)at, " U%d/%d %.1f", t->L[k].unroll & 15, t->L[k].unroll >> 4,
                     t->us[k]);
    fprintf(stderr, "ext_mpi_amd: fold schedule kept: U %d issue %d (%.1f us; %d candidates%s:%s)\n", h->unroll & 15,
            h->unroll >> 4, t->us[best], t->n, t->isolated ? ", isolated samples" : "", line);
  }
  return 0;
}

/* The handle's fold launch (fan 0 / 1), with the schedule tuning of emac_tune. */
int fold_launch(emac_handle *h) {
  emac_tune *t = &h->tune;
  int rc;
  t->ops++;
  if (t->n && t->chosen < 0) {
    const int s = t->starts++, nsamples = t->n * EMAC_TUNE_ROUNDS;
    if (s >= 1 && s <= EMAC_TUNE_SPAN * nsamples) {
      /* sample p: candidate p % n on EMAC_TUNE_SPAN Starts in a row, the first untimed (it follows
         another schedule's launch); the others timed as one window, or each alone (isolated) */
      const int p = (s - 1) / EMAC_TUNE_SPAN, pos = (s - 1) % EMAC_TUNE_SPAN;
      const emac_launch *L = &t->L[p % t->n];
      const int open = pos >= 1 && (t->isolated || pos == 1), close = pos >= 1 && (t->isolated || pos == EMAC_TUNE_SPAN - 1);
      const int e0 = pos < 1 ? 0 : t->isolated ? 2 * (pos - 1) : 0;
      const int e1 = pos < 1 ? 0 : t->isolated ? 2 * (pos - 1) + 1 : 2 * (EMAC_TUNE_SPAN - 1) - 1;
      if (open) {
        if ((rc = emac_gpu_event_record(t->ev[p][e0], h->stream))) return rc;
        t->op_mark = t->ops - 1; /* this fold included */
      }
      if ((rc = emac_gpu_fold(h->plan.dtype, h->plan.op, h->nsrc, h->fan, L->unroll, &h->plan.codes, L->d_buckets, L->nb,
                              L->ntiles, L->tiles_per_bucket, L->all_full, L->d_edges, L->nedges, h->stream)))
        return rc;
      if (close) {
        t->span_ops[p] += (int)(t->ops - t->op_mark);
        return emac_gpu_event_record(t->ev[p][e1], h->stream);
      }
      return 0;
    }
    if (s == EMAC_TUNE_SPAN * nsamples + 1 && (rc = tune_keep(h))) /* the kept one becomes the handle's launch */
      return rc;
  }
  return emac_gpu_fold(h->plan.dtype, h->plan.op, h->nsrc, h->fan, h->unroll, &h->plan.codes, h->d_buckets, h->nb, h->ntiles,
                       h->tiles_per_bucket, h->all_full, h->d_edges, h->nedges, h->stream);
}

int ext_mpi_amd_handle_schedule(int handle, int *unroll, int *issue, int *tuned) {
  const emac_handle *h = handle_get(handle);
  if (!h) return EMAC_ERR_ARG;
  if (unroll) *unroll = h->unroll & 15;
  if (issue) *issue = h->unroll >> 4;
  if (tuned) *tuned = h->tune.n ? (h->tune.chosen >= 0 ? 1 : 0) : -1;
  return 0;
}

int ext_mpi_amd_handle_candidates(int handle, int *n, int *sched, int max) {
  const emac_handle *h = handle_get(handle);
  int k;
  if (!h || !n || (max > 0 && !sched)) return EMAC_ERR_ARG;
  *n = h->tune.n;
  for (k = 0; k < h->tune.n && k < max; k++) sched[k] = h->tune.L[k].unroll;
  return 0;
}

int ext_mpi_amd_handle_tune_info(int handle, ext_mpi_amd_tune_info *info) {
  const emac_handle *h = handle_get(handle);
  const emac_tune *t;
  int k;
  if (!h || !info) return EMAC_ERR_ARG;
  t = &h->tune;
  memset(info, 0, sizeof(*info));
  info->candidates = t->n;
  info->chosen = t->n ? t->chosen : -1;
  info->cached = t->cached;
  info->isolated = t->isolated;
  info->starts = t->starts;
  info->timed_starts_per_sample = EMAC_TUNE_SPAN - 1;
  info->samples = t->cached ? 0 : t->n * EMAC_TUNE_ROUNDS;
  for (k = 0; k < t->n && k < EXT_MPI_AMD_TUNE_MAX; k++) {
    info->schedule[k] = t->L[k].unroll;
    info->us[k] = t->chosen >= 0 && !t->cached ? t->us[k] : 0.f;
  }
  for (k = 0; k < info->samples && k < EXT_MPI_AMD_TUNE_MAX * 3; k++) info->ops_in_sample[k] = t->span_ops[k];
  return 0;
}
