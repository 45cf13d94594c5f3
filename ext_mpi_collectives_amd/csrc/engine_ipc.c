/*
 * engine_ipc.c -- the peer-mapped form (hipIpc over xGMI, the reference's cudaIpc design):
 * mappings of the peers' buffers, the communicator's arena, the set-up exchanges and the node
 * barriers (engine_int.h).
 */
#include "engine_int.h"

/* ------------------------- peer-mapped form (IPC over xGMI), the reference's GPU path -------
 * cuda_shmem.c:218-299 maps every node peer's device send/recv buffer with cudaIpc and
 * cuda_core.cu:50-86 then loads the partners' chunks directly; ext_mpi_native_exec.c:21-84
 * synchronises the ranks with flags in shared memory. Here: hipIpc (dmabuf) mappings, exchanged
 * through the caller's allgather (the MPI layer passes PMPI_Allgather, as the reference does),
 * and stream-ordered barrier kernels over a per-communicator block of uncached device flags
 * (ipc.hip). Start = system-scope release -> barrier -> fold of this rank's owner chunks over the
 * peers' send buffers into its own receive buffer -> barrier -> pull of every other owner's
 * result from that owner's receive buffer (one launch for small messages). */

int ipc_agree(emac_comm *cm, int ok_local) {
  int all[EMAC_MAX_RANKS], r;
  if (cm->ag(cm->ag_ctx, &ok_local, all, (long)sizeof(int))) return EMAC_ERR_TRANSPORT;
  for (r = 0; r < cm->size; r++)
    if (!all[r]) return EMAC_ERR_TRANSPORT;
  return 0;
}

static ipc_map *g_maps;
static int g_nmaps;

static void *ipc_map_peer(const unsigned char *handle, unsigned long long buf_id, long extent) {
  int i;
  void *base;
  for (i = 0; i < g_nmaps; i++) {
    ipc_map *m = &g_maps[i];
    if (m->base && m->extent == extent && m->buf_id == buf_id && !memcmp(m->handle, handle, EMAC_IPC_HANDLE_BYTES)) {
      m->refs++;
      return m->base;
    }
  }
  if (emac_gpu_ipc_open(handle, &base)) return NULL;
  for (i = 0; i < g_nmaps && g_maps[i].base; i++);
  if (i == g_nmaps) {
    ipc_map *m = (ipc_map *)realloc(g_maps, sizeof(ipc_map) * (size_t)(g_nmaps + 1));
    if (!m) {
      emac_gpu_ipc_close(base);
      return NULL;
    }
    g_maps = m;
    g_nmaps++;
  }
  g_maps[i].buf_id = buf_id;
  g_maps[i].extent = extent;
  memcpy(g_maps[i].handle, handle, EMAC_IPC_HANDLE_BYTES);
  g_maps[i].base = base;
  g_maps[i].refs = 1;
  return base;
}

void ipc_unmap(void *base) {
  int i;
  for (i = 0; i < g_nmaps; i++)
    if (g_maps[i].refs > 0 && g_maps[i].base == base) {
      if (--g_maps[i].refs == 0) {
        emac_gpu_ipc_close(base);
        g_maps[i].base = NULL;
      }
      return;
    }
}

static int ipc_mirror_get(emac_comm *cm, void **p, size_t bytes) {
  int i, best = -1, rc;
  for (i = 0; i < cm->nmirrors; i++)
    if (!cm->mirrors[i].busy && cm->mirrors[i].bytes >= bytes &&
        (best < 0 || cm->mirrors[i].bytes < cm->mirrors[best].bytes))
      best = i;
  if (best < 0) {
    ipc_mirror *m = (ipc_mirror *)realloc(cm->mirrors, sizeof(ipc_mirror) * (size_t)(cm->nmirrors + 1));
    if (!m) return EMAC_ERR_MALLOC;
    cm->mirrors = m;
    best = cm->nmirrors;
    bytes = (bytes + EMAC_IPC_GRANULE - 1) / EMAC_IPC_GRANULE * EMAC_IPC_GRANULE; /* never sub-allocated */
    if ((rc = emac_gpu_malloc(&m[best].p, bytes))) return rc;
    m[best].bytes = bytes;
    cm->nmirrors++;
  }
  cm->mirrors[best].busy = 1;
  *p = cm->mirrors[best].p;
  return 0;
}

static void ipc_mirror_put(emac_comm *cm, void *p) {
  int i;
  for (i = 0; i < cm->nmirrors; i++)
    if (cm->mirrors[i].p == p && cm->mirrors[i].busy == 1) cm->mirrors[i].busy = 0; /* poisoned ones stay out */
}

static int ipc_pool_owns(const emac_comm *cm, const void *p) {
  int i;
  for (i = 0; i < cm->nmirrors; i++)
    if ((const char *)p >= (const char *)cm->mirrors[i].p && (const char *)p < (const char *)cm->mirrors[i].p + cm->mirrors[i].bytes)
      return 1;
  return 0;
}

int ext_mpi_amd_comm_malloc(int comm, void **p, unsigned long bytes) {
  if (!p || comm < 0 || comm >= MAX_COMMS || !g_comms[comm].used) return EMAC_ERR_ARG;
  *p = NULL;
  if (!bytes) return 0;
  if (emac_gpu_set_device(g_comms[comm].device)) return EMAC_ERR_DEVICE;
  return g_comms[comm].ipc ? ipc_mirror_get(&g_comms[comm], p, bytes) : emac_gpu_malloc(p, bytes);
}

int ext_mpi_amd_comm_mfree(int comm, void *p) {
  if (comm < 0 || comm >= MAX_COMMS || !g_comms[comm].used) return EMAC_ERR_ARG;
  if (!p) return 0;
  if (g_comms[comm].ipc) {
    ipc_mirror_put(&g_comms[comm], p);
    return 0;
  }
  return emac_gpu_free(p);
}


/* Collective: every rank first closes its mappings of the others' memory, then all agree, and
   only then is this rank's exported memory (synchronisation block, mirror pool) freed. */
void ipc_comm_release(emac_comm *cm) {
  int r, k;
  for (r = 0; r < cm->size; r++) {
    if (r != cm->rank && cm->peer_sync_base[r]) ipc_unmap(cm->peer_sync_base[r]);
    for (k = 0; r != cm->rank && k < cm->peer_nseg[r]; k++) ipc_unmap(cm->peer_seg[r][k]);
  }
  if (cm->ag && cm->size > 1) ipc_agree(cm, 1);
  for (k = 0; k < cm->nseg; k++) {
    emac_gpu_free(cm->seg[k].base);
    free(cm->seg[k].fr);
  }
  for (k = 0; k < cm->nbad; k++) emac_gpu_free(cm->bad_seg[k]);
  for (r = 0; r < cm->nmirrors; r++) emac_gpu_free(cm->mirrors[r].p);
  free(cm->mirrors);
  emac_gpu_free(cm->d_peer_sync);
  emac_gpu_free(cm->sync);
  for (r = 0; r < cm->nstale_sync; r++) emac_gpu_free(cm->stale_sync[r]);
  emac_gpu_host_free(cm->err);
  memset(cm, 0, sizeof(*cm));
}

typedef struct {
  unsigned char handle[EMAC_IPC_HANDLE_BYTES];
  long offset;
  long extent; /* bytes of the exported allocation: the importer's mapping must match */
  unsigned long long buf_id; /* the exporter's allocation id (0: unknown) */
  int status;
  int refused;   /* [0]: the runtime refused to export one of this rank's buffers */
  int caller;    /* [0]: the exported send buffer is caller memory (not a library mirror) */
  int seg;       /* >= 0: an arena block, in the exporter's segment `seg` at `offset` (nothing exported) */
  long lack;     /* [0]: arena bytes this rank could not place: every rank grows the arena first */
  long len;      /* bytes the peers access (the sample spans them) */
  unsigned char sample[EMAC_SAMPLE_BYTES]; /* the exporter's own read of the buffer (ipc_exchange) */
  unsigned char uuid[16];                  /* communicator set-up: the exporter's device */
  int force_cross; /* communicator set-up: EXT_MPI_AMD_TEST_CROSS_DEVICE=1 on the exporter */
  unsigned char free_slots[EMAC_SYNC_SLOTS / 8]; /* handle set-up: slots this rank can use */
} ipc_export;

/* The synchronisation blocks: every rank exports its block, maps every peer's and validates the
   mappings with a write probe (as the buffers, ipc_exchange): each rank flips probe[me][0] in
   every peer's block through its mapping and checks that its own block shows every peer's flip.
   The runtime places small allocations side by side in shared chunks, and a second
   communicator's block mapped by a process that already maps the first one's was measured to
   miss (8 processes on one MI355X: one rank never saw a peer's flags), and the runtime may refuse
   to export a fresh block (an allocation placed where a freed one a peer still maps lay; measured
   on a third communicator of 3 processes after 1200 handle lifetimes). A failed round keeps the
   blocks it allocated (peers may map them; freed with the communicator) and retries with a fresh,
   larger allocation. Collective: every rank runs every round whatever failed locally (`rc`). */
#define EMAC_SYNC_ATTEMPTS 8
static int ipc_sync_exchange(emac_comm *cm, int rc, ipc_export *all) {
  ipc_export mine;
  const int R = cm->size;
  int attempt, r;
  for (attempt = 0; attempt < EMAC_SYNC_ATTEMPTS; attempt++) {
    void *pk[EMAC_PROBE_MAX];
    unsigned char vals[EMAC_PROBE_MAX], seen[EMAC_PROBE_MAX];
    int n = 0, good = 1, agreed;
    memset(&mine, 0, sizeof(mine));
    if (!rc && cm->sync) { /* the previous round's block stays allocated until the communicator goes */
      cm->stale_sync[cm->nstale_sync++] = cm->sync;
      cm->sync = NULL;
    }
    if (!rc) rc = emac_gpu_malloc_uncached(&cm->sync, sizeof(emac_sync) << attempt);
    if (!rc) {
      const int er = emac_gpu_ipc_export(cm->sync, mine.handle, &mine.offset);
      if (er == EMAC_ERR_TRANSPORT) {
        mine.refused = 1; /* no peer maps it: this rank misses every flip and the round repeats */
        if (getenv("EXT_MPI_AMD_DEBUG_IPC"))
          fprintf(stderr, "ipc rank %d: export of my synchronisation block refused (attempt %d)\n", cm->rank, attempt);
      } else {
        rc = er;
      }
    }
    if (!rc && !mine.refused) {
      void *b0;
      mine.extent = emac_gpu_alloc_extent(cm->sync, &b0);
      mine.buf_id = emac_gpu_buffer_id(b0);
    }
    /* a device this rank cannot identify fails the set-up on every rank: taken for the same device
       as a peer on another GPU, it would keep device-scope stores between GPUs */
    if (!rc) rc = emac_gpu_device_uuid(mine.uuid);
    {
      const char *fc = getenv("EXT_MPI_AMD_TEST_CROSS_DEVICE");
      mine.force_cross = fc && atoi(fc) > 0;
    }
    mine.status = rc == 0;
    if (cm->ag(cm->ag_ctx, &mine, all, (long)sizeof(ipc_export))) return EMAC_ERR_TRANSPORT;
    for (r = 0; r < R; r++)
      if (!all[r].status) rc = rc ? rc : EMAC_ERR_TRANSPORT;
    /* the same verdict on every rank: every rank sees every UUID and every test flag. A forced
       verdict runs the cross-GPU code (system-scope release, system-scope partial stores of the
       fused node join) with every rank on one GPU; same_device still counts the ranks really
       sharing this device, so the fused join's grid stays divided among them */
    cm->cross_device = 0;
    cm->same_device = 0;
    for (r = 0; !rc && r < R; r++) {
      if (memcmp(all[r].uuid, mine.uuid, 16))
        cm->cross_device = 1;
      else
        cm->same_device++;
      if (all[r].force_cross) cm->cross_device = 1;
    }
    for (r = 0; !rc && r < R; r++) {
      if (r == cm->rank) {
        cm->peer_sync[r] = cm->sync;
        continue;
      }
      cm->peer_sync_base[r] = all[r].refused ? NULL : ipc_map_peer(all[r].handle, all[r].buf_id, all[r].extent);
      if (!cm->peer_sync_base[r]) {
        /* not fatal: the exporter misses this rank's flip below and the round is repeated with
           fresh blocks (measured: an open refused for a second communicator's block, 4 processes) */
        cm->peer_sync[r] = NULL;
        if (getenv("EXT_MPI_AMD_DEBUG_IPC"))
          fprintf(stderr, "ipc rank %d: cannot map peer %d's synchronisation block (attempt %d)\n", cm->rank, r,
                  attempt);
        continue;
      }
      cm->peer_sync[r] = (char *)cm->peer_sync_base[r] + all[r].offset;
      pk[n] = &((emac_sync *)cm->peer_sync[r])->probe[cm->rank][0];
      vals[n++] = (unsigned char)(0x5A ^ (cm->rank + 1));
    }
    if (!rc && R > 1) rc = emac_gpu_poke(pk, vals, n, NULL);
    agreed = ipc_agree(cm, rc == 0); /* every flip has landed */
    if (!rc) rc = agreed;
    if (rc) return rc;
    for (n = 0, r = 0; r < R; r++)
      if (r != cm->rank) pk[n++] = &((emac_sync *)cm->sync)->probe[r][0];
    if ((rc = emac_gpu_peek((const void *const *)pk, seen, n, NULL))) good = 0; /* still in the verdict below */
    for (n = 0, r = 0; r < R; r++)
      if (r != cm->rank) {
        if (!rc && seen[n] != (unsigned char)(0x5A ^ (r + 1))) {
          good = 0;
          if (getenv("EXT_MPI_AMD_DEBUG_IPC"))
            fprintf(stderr, "ipc rank %d: peer %d does not reach my synchronisation block (attempt %d)\n", cm->rank, r,
                    attempt);
        }
        n++;
      }
    memset(vals, 0, sizeof(vals));
    if (!rc) rc = emac_gpu_poke(pk, vals, n, NULL);
    {
      int v[2] = {good, rc == 0}, allv[2 * EMAC_MAX_RANKS], ok = 1, fine = 1;
      if (cm->ag(cm->ag_ctx, v, allv, (long)sizeof(v))) return EMAC_ERR_TRANSPORT;
      for (r = 0; r < R; r++) {
        ok &= allv[2 * r];
        fine &= allv[2 * r + 1];
      }
      if (!fine) return rc ? rc : EMAC_ERR_TRANSPORT;
      if (ok) return 0;
    }
    for (r = 0; r < R; r++)
      if (r != cm->rank && cm->peer_sync_base[r]) {
        ipc_unmap(cm->peer_sync_base[r]);
        cm->peer_sync_base[r] = NULL;
      }
  }
  fprintf(stderr, "ext_mpi_amd: rank %d: synchronisation blocks still unreachable after %d set-up rounds\n", cm->rank,
          EMAC_SYNC_ATTEMPTS);
  return EMAC_ERR_TRANSPORT;
}

int ext_mpi_amd_comm_init_ipc(int rank, int size, ext_mpi_amd_allgather_fn allgather, void *ctx, int device,
                              int *comm) {
  emac_comm *cm;
  ipc_export all[EMAC_MAX_RANKS];
  const char *tmo;
  int i, rc;
  if (!comm || !allgather || size < 1 || size > EMAC_MAX_RANKS || rank < 0 || rank >= size) return EMAC_ERR_ARG;
  *comm = -1;
  for (i = 0; i < MAX_COMMS && g_comms[i].used; i++);
  if (i == MAX_COMMS) return EMAC_ERR_MALLOC;
  cm = &g_comms[i];
  memset(cm, 0, sizeof(*cm));
  cm->rank = rank;
  cm->size = size;
  cm->loop_group = -1;
  cm->ipc = 1;
  cm->ag = allgather;
  cm->ag_ctx = ctx;
  /* every rank takes part in every allgather below, whatever failed locally, so that all ranks
     reach the same verdict */
  rc = emac_gpu_device_count() > 0 ? 0 : EMAC_ERR_DEVICE;
  if (!rc && device >= 0) rc = emac_gpu_set_device(device);
  if (!rc) rc = emac_gpu_get_device(&cm->device);
  if (!rc) rc = emac_gpu_host_alloc_mapped((void **)&cm->err, sizeof(int) * EMAC_SYNC_SLOTS);
  rc = ipc_sync_exchange(cm, rc, all);
  if (!rc && (rc = emac_gpu_malloc((void **)&cm->d_peer_sync, sizeof(void *) * (size_t)size)) == 0)
    rc = emac_gpu_memcpy(cm->d_peer_sync, cm->peer_sync, sizeof(void *) * (size_t)size);
  {
    const int agreed = ipc_agree(cm, rc == 0); /* every rank mapped every block */
    if (!rc) rc = agreed;
  }
  if (rc) {
    ipc_comm_release(cm);
    return rc;
  }
  /* a rank that never arrives is reported after this many seconds (default 30) */
  tmo = getenv("EXT_MPI_AMD_BARRIER_TIMEOUT");
  cm->timeout_ticks = (long)((tmo ? atof(tmo) : 30.0) * (double)emac_gpu_wallclock_hz());
  cm->used = 1;
  *comm = i;
  return 0;
}

/* Mapping the peers' buffers (the reference: cuda_shmem.c:218-299 opens every peer's cudaIpc
   handle once at init; EXT_MPI_Done closes them after a node barrier, ext_mpi_native.c:269-387 with
   cuda_shmem.c:190-216,301-314). What can go wrong, and what rules it out here:
   * The runtime's IPC handle of an allocation is a function of the exporter's address and size:
     an allocation freed while a peer still maps it and re-allocated at the same address exports
     the same handle, and importing it resolves to the OLD memory. The rule of the reference rules
     it out for caller memory: a peer-mapped handle's Done is collective (ext_mpi_amd_done: every
     rank closes its mappings, then the ranks agree), so no caller allocation is freed under a
     mapping as long as the caller keeps its buffers until Done.
   * Library memory the peers read -- outboxes, mirrors of send buffers -- lives in the
     communicator's ARENA: a few large segments per rank, each exported and mapped ONCE (when it is
     added) and validated then with a random nonce the owner wrote into its head, so a mapping of
     any other memory cannot pass. Handles carve blocks out of the segments; nothing library-owned
     is exported, imported or closed per handle, and segments are freed only by the collective
     communicator free.
   * Peers never WRITE caller memory, at set-up or later: the send buffer is only read (the fold's
     leaves), each rank's results go to its own outbox, and every rank pulls the results into its
     own receive buffer, which is never exported. A stale mapping could therefore only feed wrong
     leaves, never overwrite anything.
   * Every mapping of a caller's send buffer is still validated, read-only: the exporter samples
     its buffer (emac_gpu_sample: 8 spots of 8 bytes) and publishes the sample with its handle;
     every importer samples the same spots through its mapping. A mismatch, a mapping the runtime
     refuses or one shorter than the exporter's allocation re-places that send buffer in an arena
     mirror (staged in on the handle's stream) and the exchange repeats.
     EXT_MPI_AMD_IPC_FORCE_MIRROR=1 re-places every rank's send buffer in the first round, so the
     mirror path runs deterministically (tests/test_gpu_peer_mapped.py).
   The set-up reads the caller's send buffer: the device is synchronised first, so a kernel still
   filling it cannot make the exporter's and the importers' samples differ. */

/* ---- the arena ---- */

int arena_alloc(emac_comm *cm, long bytes, void **p) {
  int k, i;
  bytes = (bytes + EMAC_ARENA_ALIGN - 1) / EMAC_ARENA_ALIGN * EMAC_ARENA_ALIGN;
  if (bytes <= 0) bytes = EMAC_ARENA_ALIGN;
  for (k = 0; k < cm->nseg; k++) {
    arena_seg *s = &cm->seg[k];
    for (i = 0; i < s->nfr; i++)
      if (s->fr[i].len >= bytes) {
        *p = (char *)s->base + s->fr[i].off;
        s->fr[i].off += bytes;
        s->fr[i].len -= bytes;
        if (!s->fr[i].len) {
          memmove(&s->fr[i], &s->fr[i + 1], sizeof(arena_free) * (size_t)(s->nfr - i - 1));
          s->nfr--;
        }
        return 0;
      }
  }
  return EMAC_ERR_MALLOC;
}

int arena_owns(const emac_comm *cm, const void *p, int *seg) {
  int k;
  for (k = 0; k < cm->nseg; k++)
    if ((const char *)p >= (const char *)cm->seg[k].base && (const char *)p < (const char *)cm->seg[k].base + cm->seg[k].bytes) {
      if (seg) *seg = k;
      return 1;
    }
  return 0;
}

void arena_release(emac_comm *cm, void *p, long bytes) {
  arena_seg *s;
  long off;
  int k, i;
  if (!p || !cm->used || !arena_owns(cm, p, &k)) return;
  bytes = (bytes + EMAC_ARENA_ALIGN - 1) / EMAC_ARENA_ALIGN * EMAC_ARENA_ALIGN;
  if (bytes <= 0) bytes = EMAC_ARENA_ALIGN;
  s = &cm->seg[k];
  off = (long)((char *)p - (char *)s->base);
  for (i = 0; i < s->nfr && s->fr[i].off < off; i++);
  if (s->nfr == s->capfr) {
    arena_free *f = (arena_free *)realloc(s->fr, sizeof(arena_free) * (size_t)(2 * s->capfr + 8));
    if (!f) return; /* the block stays allocated */
    s->fr = f;
    s->capfr = 2 * s->capfr + 8;
  }
  memmove(&s->fr[i + 1], &s->fr[i], sizeof(arena_free) * (size_t)(s->nfr - i));
  s->fr[i].off = off;
  s->fr[i].len = bytes;
  s->nfr++;
  if (i + 1 < s->nfr && s->fr[i].off + s->fr[i].len == s->fr[i + 1].off) { /* merge with the next */
    s->fr[i].len += s->fr[i + 1].len;
    memmove(&s->fr[i + 1], &s->fr[i + 2], sizeof(arena_free) * (size_t)(s->nfr - i - 2));
    s->nfr--;
  }
  if (i > 0 && s->fr[i - 1].off + s->fr[i - 1].len == s->fr[i].off) { /* and the previous */
    s->fr[i - 1].len += s->fr[i].len;
    memmove(&s->fr[i], &s->fr[i + 1], sizeof(arena_free) * (size_t)(s->nfr - i - 1));
    s->nfr--;
  }
}

typedef struct {
  int status, grow;
  unsigned char handle[EMAC_IPC_HANDLE_BYTES];
  long offset, extent;
  unsigned long long buf_id;
  unsigned char nonce[EMAC_SAMPLE_BYTES];
} arena_export;

static unsigned long long g_nonce_state;
#define EMAC_ARENA_FAILED 0x80000000u /* arena_grow's verdict word: this rank failed locally */

/* Collective: ranks that lack `need` bytes (0: none) add a segment of at least that size (and at
   least their arena's size so far, EMAC_ARENA_MIN at first); every rank maps every new segment
   and checks the nonce in its head through the mapping. A segment some rank cannot map or
   validate is set aside (freed with the communicator) and its owner tries a fresh one. */
int arena_grow(emac_comm *cm, int rc, long need) {
  const int R = cm->size;
  int attempt, r;
  for (attempt = 0; attempt < EMAC_IPC_ATTEMPTS; attempt++) {
    arena_export mine, all[EMAC_MAX_RANKS];
    void *nb = NULL, *mapped[EMAC_MAX_RANKS];
    unsigned bad = 0, allbad[EMAC_MAX_RANKS], badall = 0;
    long sz = 0;
    int any = 0;
    memset(&mine, 0, sizeof(mine));
    if (!rc && need > 0) {
      long have = 0;
      int i;
      for (i = 0; i < cm->nseg; i++) have += cm->seg[i].bytes;
      sz = need + EMAC_ARENA_HEAD;
      if (sz < have) sz = have;
      if (sz < EMAC_ARENA_MIN) sz = EMAC_ARENA_MIN;
      sz = (long)((sz + (long)EMAC_IPC_GRANULE - 1) / (long)EMAC_IPC_GRANULE * (long)EMAC_IPC_GRANULE);
      if (cm->nseg == EMAC_ARENA_SEGS || cm->nbad == EMAC_ARENA_SEGS) rc = EMAC_ERR_MALLOC;
      if (!rc) rc = emac_gpu_malloc(&nb, (size_t)sz);
      if (!rc) {
        void *b0;
        unsigned long long x = g_nonce_state ^ ((unsigned long long)(size_t)nb * 0x9E3779B97F4A7C15ull) ^
                               ((unsigned long long)cm->rank << 40) ^ (unsigned long long)attempt;
        for (i = 0; i < EMAC_SAMPLE_BYTES; i++) { /* xorshift64* */
          x ^= x >> 12;
          x ^= x << 25;
          x ^= x >> 27;
          mine.nonce[i] = (unsigned char)((x * 0x2545F4914F6CDD1Dull) >> 56);
        }
        g_nonce_state = x + 0x9E3779B97F4A7C15ull;
        /* the nonce is the head's first EMAC_SAMPLE_BYTES bytes: sampled whole (len = that size) */
        rc = emac_gpu_memcpy(nb, mine.nonce, EMAC_SAMPLE_BYTES);
        if (!rc) rc = emac_gpu_device_sync();
        if (!rc) rc = emac_gpu_ipc_export(nb, mine.handle, &mine.offset);
        mine.extent = emac_gpu_alloc_extent(nb, &b0);
        mine.buf_id = emac_gpu_buffer_id(b0);
        if (rc == EMAC_ERR_TRANSPORT) { /* export refused: set aside, try another */
          rc = 0;
          bad = 1u << cm->rank;
        }
      }
      mine.grow = 1;
    }
    mine.status = rc == 0;
    if (cm->ag(cm->ag_ctx, &mine, all, (long)sizeof(mine))) return EMAC_ERR_TRANSPORT;
    for (r = 0; r < R; r++) {
      if (!all[r].status) rc = rc ? rc : EMAC_ERR_TRANSPORT;
      any |= all[r].grow;
    }
    if (rc) {
      if (nb) emac_gpu_free(nb); /* nobody maps it: every rank stops here */
      return rc;
    }
    if (!any) return 0;
    {
      const void *pk[EMAC_MAX_RANKS];
      long pl[EMAC_MAX_RANKS];
      int who[EMAC_MAX_RANKS], n = 0;
      unsigned char seen[EMAC_MAX_RANKS * EMAC_SAMPLE_BYTES];
      for (r = 0; r < R; r++) {
        void *ext_base;
        mapped[r] = NULL;
        if (!all[r].grow || r == cm->rank) continue;
        if (!(mapped[r] = ipc_map_peer(all[r].handle, all[r].buf_id, all[r].extent)) || all[r].offset != 0 ||
            emac_gpu_alloc_extent(mapped[r], &ext_base) != all[r].extent) {
          bad |= 1u << r;
          continue;
        }
        pk[n] = mapped[r];
        pl[n] = EMAC_SAMPLE_BYTES;
        who[n++] = r;
      }
      /* a local failure still takes part in the verdict below (every peer is in that allgather);
         EXT_MPI_AMD_TEST_FAIL_ARENA_SAMPLE=1 fails the sample here (tests/ipc_worker.py "arenafault") */
      if (n) {
        const char *f = getenv("EXT_MPI_AMD_TEST_FAIL_ARENA_SAMPLE");
        rc = f && atoi(f) > 0 ? EMAC_ERR_DEVICE : emac_gpu_sample(pk, pl, n, seen, NULL);
        if (rc) bad |= EMAC_ARENA_FAILED;
      }
      for (r = 0; !rc && r < n; r++)
        if (memcmp(seen + r * EMAC_SAMPLE_BYTES, all[who[r]].nonce, EMAC_SAMPLE_BYTES)) bad |= 1u << who[r];
    }
    if (cm->ag(cm->ag_ctx, &bad, allbad, (long)sizeof(unsigned))) return EMAC_ERR_TRANSPORT;
    for (r = 0; r < R; r++) badall |= allbad[r];
    if (badall & EMAC_ARENA_FAILED) {
      /* some rank could not validate this round: every rank drops the round's new segments (its own
         kept aside, a peer may map it; freed with the communicator) and reports the failure */
      for (r = 0; r < R; r++) {
        if (!all[r].grow) continue;
        if (r == cm->rank)
          cm->bad_seg[cm->nbad++] = nb;
        else if (mapped[r])
          ipc_unmap(mapped[r]);
      }
      return rc ? rc : EMAC_ERR_TRANSPORT;
    }
    for (r = 0; r < R; r++) {
      if (!all[r].grow) continue;
      if ((badall >> r) & 1) {
        if (r == cm->rank) {
          cm->bad_seg[cm->nbad++] = nb; /* a peer may map it: freed with the communicator */
        } else if (mapped[r]) {
          ipc_unmap(mapped[r]);
        }
        if (getenv("EXT_MPI_AMD_DEBUG_IPC"))
          fprintf(stderr, "ipc rank %d: rank %d's new arena segment failed validation (attempt %d)\n", cm->rank, r,
                  attempt);
        continue;
      }
      if (r == cm->rank) {
        arena_seg *s = &cm->seg[cm->nseg];
        memset(s, 0, sizeof(*s));
        s->base = nb;
        s->bytes = sz;
        s->fr = (arena_free *)malloc(sizeof(arena_free) * 8);
        s->capfr = 8;
        if (s->fr) {
          s->fr[0].off = EMAC_ARENA_HEAD;
          s->fr[0].len = sz - EMAC_ARENA_HEAD;
          s->nfr = 1;
        }
        cm->peer_seg[r][cm->nseg++] = nb;
        cm->peer_nseg[r] = cm->nseg;
        need = 0;
      } else {
        cm->peer_seg[r][cm->peer_nseg[r]++] = mapped[r];
      }
    }
    if (!badall) return 0;
  }
  fprintf(stderr, "ext_mpi_amd: rank %d: arena segments still unreachable after %d set-up rounds\n", cm->rank,
          EMAC_IPC_ATTEMPTS);
  return EMAC_ERR_TRANSPORT;
}

/* Byte offset of every piece of position `pos`'s owner chunk inside that rank's outbox: pieces
   back to back, each at the 16-byte phase its elements have in the message (so the fold's leaves,
   the outbox and the receive buffer agree on vector alignment). Returns the outbox bytes. */
static long outbox_layout(const emac_plan *p, int pos, long *at) {
  const int R = p->nranks;
  long cur = 0;
  int pc;
  for (pc = 0; pc < p->npieces; pc++) {
    const long off = p->chunk_off[(size_t)pc * R + pos], len = p->chunk_len[(size_t)pc * R + pos];
    const long a = ((cur + 15) & ~15L) + ((off * p->tsize) & 15);
    if (at) at[pc] = a;
    if (len > 0) cur = a + len * p->tsize;
  }
  return cur;
}

enum { IPC_SEND = 0, IPC_OUTBOX = 1, IPC_NBUF = 2 };

/* One exchange of the IPC set-up (collective whatever failed locally before: `rc`). Every rank
   publishes its send buffer (an exported caller allocation with a sample of it, or an arena block)
   and its outbox (an arena block). On return peer[t][r] holds rank r's buffer t as reachable here,
   all[] the exports, and *miss a bit per rank whose send buffer this rank could not map or validate. */
static int ipc_exchange(emac_handle *h, emac_comm *cm, int rc, long lack, ipc_export *all,
                        void *(*peer)[EMAC_MAX_RANKS], unsigned *miss, int *grow) {
  ipc_export mine[IPC_NBUF];
  const int R = cm->size;
  void *own[IPC_NBUF] = {h->dsend[0], h->outbox};
  const long len[IPC_NBUF] = {(long)h->bytes, (long)h->outbox_bytes};
  int r, t, k;
  memset(mine, 0, sizeof(mine));
  *miss = 0;
  *grow = 0;
  mine[0].lack = lack;
  for (t = 0; t < IPC_NBUF && !rc && !lack; t++) {
    mine[t].len = len[t];
    if (arena_owns(cm, own[t], &k)) {
      mine[t].seg = k;
      mine[t].offset = (long)((char *)own[t] - (char *)cm->seg[k].base);
    } else if (t == IPC_SEND) {
      void *b0;
      const int er = emac_gpu_ipc_export(own[t], mine[t].handle, &mine[t].offset);
      mine[t].seg = -1;
      if (er == EMAC_ERR_TRANSPORT)
        mine[0].refused = 1; /* refused by the runtime: this rank's send buffer is re-placed */
      else
        rc = er;
      mine[t].extent = emac_gpu_alloc_extent(own[t], &b0);
      mine[t].buf_id = emac_gpu_buffer_id(b0);
      if (!rc) rc = emac_gpu_sample((const void *const *)&own[t], &len[t], 1, mine[t].sample, h->stream);
    } else {
      rc = EMAC_ERR_ARG; /* an outbox outside the arena */
    }
  }
  for (r = 0; r < EMAC_SYNC_SLOTS; r++)
    if (!cm->slot_used[r]) mine[0].free_slots[r >> 3] |= (unsigned char)(1u << (r & 7));
  mine[0].status = rc == 0;
  mine[0].caller = mine[0].seg < 0 && !ipc_pool_owns(cm, h->dsend[0]);
  if (cm->ag(cm->ag_ctx, mine, all, (long)sizeof(mine))) return EMAC_ERR_TRANSPORT;
  for (r = 0; r < R; r++) {
    if (!all[IPC_NBUF * r].status && !rc) rc = EMAC_ERR_TRANSPORT;
    if (all[IPC_NBUF * r].lack > 0) *grow = 1;
  }
  if (rc || *grow) return rc; /* (every rank reaches the same verdict) */
  {
    const void *pk[EMAC_MAX_RANKS];
    long pl[EMAC_MAX_RANKS];
    int who[EMAC_MAX_RANKS], n = 0;
    unsigned char seen[EMAC_MAX_RANKS * EMAC_SAMPLE_BYTES];
    for (r = 0; r < R; r++)
      for (t = 0; t < IPC_NBUF; t++) {
        const ipc_export *e = &all[IPC_NBUF * r + t];
        void *base, *ext_base;
        long extent;
        peer[t][r] = NULL;
        if (r == cm->rank) {
          peer[t][r] = own[t];
          continue;
        }
        if (e->seg >= 0) { /* an arena block: the segment was validated when it was added */
          if (e->seg < cm->peer_nseg[r]) peer[t][r] = (char *)cm->peer_seg[r][e->seg] + e->offset;
          if (!peer[t][r]) *miss |= 1u << r;
          continue;
        }
        *miss |= 1u << r; /* until validated below */
        if (all[IPC_NBUF * r].refused || !(base = ipc_map_peer(e->handle, e->buf_id, e->extent))) continue;
        h->mapped[h->nmapped++] = base;
        /* a mapping the runtime can describe must hold the peer's whole allocation (one it cannot
           describe is taken at the exporter's word; the sample still checks it) */
        extent = emac_gpu_alloc_extent(base, &ext_base);
        if (extent < 0) {
          extent = e->extent;
          ext_base = base;
        }
        if (ext_base != base || extent != e->extent || e->offset < 0 || e->offset + e->len > extent) continue;
        peer[t][r] = (char *)base + e->offset;
        pk[n] = peer[t][r];
        pl[n] = e->len;
        who[n++] = r;
      }
    if ((rc = emac_gpu_sample(pk, pl, n, seen, h->stream))) return rc;
    for (t = 0; t < n; t++) {
      if (!memcmp(seen + t * EMAC_SAMPLE_BYTES, all[IPC_NBUF * who[t]].sample, EMAC_SAMPLE_BYTES))
        *miss &= ~(1u << who[t]);
      else
        peer[IPC_SEND][who[t]] = NULL;
    }
    if (getenv("EXT_MPI_AMD_DEBUG_IPC"))
      for (r = 0; r < R; r++)
        if ((*miss >> r) & 1) fprintf(stderr, "ipc rank %d: cannot map or validate peer %d's send buffer\n", cm->rank, r);
  }
  return 0;
}

/* Collective: every rank runs the same exchanges whatever failed locally before (`rc`), so that
   a local failure cannot unmatch the sequence. */
int ipc_allreduce_init(emac_handle *h, emac_comm *cm, const void *sendbuf, void *recvbuf, int rc) {
  ipc_export all[IPC_NBUF * EMAC_MAX_RANKS];
  void *peer[IPC_NBUF][EMAC_MAX_RANKS];
  long *at = NULL;
  emac_bucket *b = NULL;
  int R = cm->size, r, t, pc, nb = 0, c, slot, attempt;
  const char *fe = getenv("EXT_MPI_AMD_IPC_FORCE_MIRROR");
  const int force = fe && atoi(fe) > 0;
  if (!rc && h->bytes) rc = map_buffers(h, 0, sendbuf, recvbuf);
  if (R == 1 || !h->bytes) { /* nothing to map: this rank folds alone (no peers), or nothing at all */
    if (!rc && h->bytes && !h->dsend[0]) { /* a send mirror map_buffers left to the arena */
      if (!(rc = emac_gpu_malloc(&h->dsend[0], h->bytes))) h->send_local = 1;
      if (h->recv_mirror[0] && !h->drecv[0]) h->drecv[0] = h->dsend[0];
    }
    attempt = 0;
    {
      ipc_export mine;
      memset(&mine, 0, sizeof(mine));
      for (r = 0; r < EMAC_SYNC_SLOTS; r++)
        if (!cm->slot_used[r]) mine.free_slots[r >> 3] |= (unsigned char)(1u << (r & 7));
      mine.status = rc == 0;
      for (r = 0; r < R; r++) all[IPC_NBUF * r] = mine;
      if (R > 1) { /* empty message: agree on the slot only */
        ipc_export g[EMAC_MAX_RANKS];
        if (cm->ag(cm->ag_ctx, &mine, g, (long)sizeof(mine))) return EMAC_ERR_TRANSPORT;
        for (r = 0; r < R; r++) {
          all[IPC_NBUF * r] = g[r];
          if (!g[r].status) rc = rc ? rc : EMAC_ERR_TRANSPORT;
        }
      }
      if (rc) return rc;
    }
  } else {
    /* the samples read the send buffer: work the application still has in flight on it must have
       landed (the reference synchronises the device before every barrier, ext_mpi_native_exec.c:556-558) */
    if (!rc) rc = emac_gpu_device_sync();
    if (!rc) {
      h->outbox_bytes = (size_t)outbox_layout(&h->plan, h->me_pos, NULL);
      if (h->outbox_bytes < 16) h->outbox_bytes = 16;
    }
    for (attempt = 0;; attempt++) {
      unsigned miss, allmiss[EMAC_MAX_RANKS], stale = 0;
      int again = 0, grow = 0;
      /* the outbox, and a send mirror left to the arena (host or non-exportable memory, or a send
         buffer re-placed below); a rank that lacks room says so in the exchange, every rank then
         grows the arena (one collective round) and exchanges again */
      long lack = 0;
      if (!rc && !h->outbox && arena_alloc(cm, (long)h->outbox_bytes, &h->outbox))
        lack += (long)(h->outbox_bytes + EMAC_ARENA_ALIGN - 1) / EMAC_ARENA_ALIGN * EMAC_ARENA_ALIGN;
      if (!rc && !h->dsend[0]) {
        void *p = NULL;
        if (arena_alloc(cm, (long)h->bytes, &p)) {
          lack += (long)(h->bytes + EMAC_ARENA_ALIGN - 1) / EMAC_ARENA_ALIGN * EMAC_ARENA_ALIGN;
        } else {
          h->dsend[0] = p;
          h->send_arena = 1;
          if (h->recv_mirror[0] && !h->drecv[0]) h->drecv[0] = p; /* in place */
        }
      }
      rc = ipc_exchange(h, cm, rc, lack, all, peer, &miss, &grow);
      if (!rc && grow) {
        if (attempt == EMAC_IPC_ATTEMPTS - 1) return EMAC_ERR_MALLOC; /* the same on every rank */
        rc = arena_grow(cm, 0, lack);
        continue;
      }
      if (!rc && force && attempt == 0 && !h->send_arena) miss |= 1u << cm->rank; /* re-place mine */
      if (rc) miss = ~0u; /* a failed rank: the verdict below stops every rank */
      if (cm->ag(cm->ag_ctx, &miss, allmiss, (long)sizeof(miss))) return EMAC_ERR_TRANSPORT;
      for (r = 0; r < R; r++) {
        if (allmiss[r] == ~0u) return rc ? rc : EMAC_ERR_TRANSPORT;
        again |= allmiss[r] != 0;
        stale |= (allmiss[r] >> cm->rank) & 1u;
      }
      if (!again) break;
      if (getenv("EXT_MPI_AMD_DEBUG_IPC"))
        fprintf(stderr, "ipc rank %d: attempt %d: re-placing%s\n", cm->rank, attempt, stale ? " send" : "");
      if (attempt == EMAC_IPC_ATTEMPTS - 1 || (stale && h->send_arena)) {
        fprintf(stderr, "ext_mpi_amd: rank %d: peer mappings still unreachable after %d set-up rounds\n", cm->rank,
                attempt + 1);
        return EMAC_ERR_TRANSPORT;
      }
      for (r = 0; r < h->nmapped; r++) ipc_unmap(h->mapped[r]);
      h->nmapped = 0;
      if (stale) {
        /* this rank's send buffer into an arena mirror (placed at the top of the next round),
           staged in on the handle's stream; in place, the one buffer, staged in and out */
        if (h->dsend[0] == h->drecv[0]) {
          h->recv_mirror[0] = 1;
          h->drecv[0] = NULL;
        } else {
          h->send_mirror[0] = 1;
        }
        h->dsend[0] = NULL;
      }
    }
  }
  /* Done is collective iff some rank's exported send buffer is caller memory (the same verdict on
     every rank): library memory is never freed under a mapping anyway (ext_mpi_amd_done) */
  for (r = 0; R > 1 && h->bytes && r < R; r++) h->done_collective |= all[IPC_NBUF * r].caller;
  /* the synchronisation slot: the lowest one free on every rank (ranks may have released
     their handles in different orders) */
  for (slot = 0; slot < EMAC_SYNC_SLOTS; slot++) {
    for (r = 0; r < R && (all[IPC_NBUF * r].free_slots[slot >> 3] >> (slot & 7)) & 1; r++);
    if (r == R) break;
  }
  if (slot == EMAC_SYNC_SLOTS) return EMAC_ERR_MALLOC; /* same verdict on every rank */
  h->slot = slot;
  cm->slot_used[slot] = 1;
  h->slot_held = 1;
  cm->err[slot] = 0; /* a failure of the slot's previous handle that nobody waited for */
  {
    /* A system-scope release (command processor, every XCD's L2) before each phase-0 barrier,
       by default when some peer sits on another device: its loads of this rank's send buffer go
       over xGMI to HBM and see nothing an L2 still holds. Ranks sharing one device read through
       the same L2s and the packet boundary after the producer kernel suffices, so the release
       (5 us per Start with 2 processes, 9 us with 4: profiles/r02_ipc_latency_release.json) is
       off there. EXT_MPI_AMD_IPC_RELEASE=1 / 0 forces it on / off. */
    const char *e = getenv("EXT_MPI_AMD_IPC_RELEASE");
    const int rel = e ? atoi(e) > 0 : cm->cross_device;
    if (R > 1 && rel && (rc = emac_gpu_event_create_release(&h->ev_release))) return rc;
  }
  h->epoch[0] = cm->slot_epoch[slot][0];
  h->epoch[1] = cm->slot_epoch[slot][1];
  if (!h->bytes) return 0;
  /* this rank's owner chunks (reduce_copyin): leaves from the peers' send buffers in the plan's
     fold order, the result into this rank's outbox (its receive buffer when alone). Then
     (reduce_copyout) every owner's result is PULLED from that owner's outbox into this rank's
     receive buffer, this rank's own last: each rank writes only memory it owns. */
  c = h->me_pos;
  b = (emac_bucket *)calloc((size_t)h->plan.npieces * (size_t)(R + 1), sizeof(emac_bucket));
  at = (long *)calloc((size_t)h->plan.npieces, sizeof(long));
  if (!b || !at) {
    free(b);
    free(at);
    return EMAC_ERR_MALLOC;
  }
  if (R > 1) outbox_layout(&h->plan, c, at);
  for (pc = 0; pc < h->plan.npieces; pc++) {
    long off = h->plan.chunk_off[(size_t)pc * R + c], len = h->plan.chunk_len[(size_t)pc * R + c];
    emac_bucket *bk = &b[nb];
    if (len <= 0) continue;
    for (t = 0; t < R; t++) bk->src[t] = R > 1 ? peer[IPC_SEND][h->plan.leaf_rank[c][t]] : h->dsend[0];
    /* place_bucket moves every pointer by the chunk's message offset */
    bk->dst[0] = R > 1 ? (char *)h->outbox + at[pc] - off * h->plan.tsize : (char *)h->drecv[0];
    bk->ndst = 1;
    place_bucket(bk, R, off, len, h->plan.tsize);
    nb++;
  }
  h->nsrc = R;
  h->fan = R > 1 ? 2 : 0; /* peer-mapped: system-coherent launch */
  if (R > 1) {
    /* the pull, owners in the order after this rank (next owner first), so that at any moment
       the ranks' loads head for different GPUs' links; this rank's own chunk (local) last */
    emac_bucket *pb = b + nb;
    int np = 0, k;
    for (k = 1; k <= R; k++) {
      const int q = (cm->rank + k) % R, cq = h->plan.rank_pos[q];
      outbox_layout(&h->plan, cq, at);
      for (pc = 0; pc < h->plan.npieces; pc++) {
        long off = h->plan.chunk_off[(size_t)pc * R + cq], len = h->plan.chunk_len[(size_t)pc * R + cq];
        if (len <= 0) continue;
        pb[np].src[0] = (char *)peer[IPC_OUTBOX][q] + at[pc] - off * h->plan.tsize;
        pb[np].dst[0] = h->drecv[0];
        pb[np].ndst = 1;
        place_bucket(&pb[np], 1, off, len, h->plan.tsize);
        np++;
      }
    }
    if ((rc = upload_launch_as(h, &h->pull, pb, np, 1, 0))) { /* a copy: the schedule of nsrc 1 for every op */
      free(b);
      free(at);
      return rc;
    }
  }
  free(at);
  {
    /* small messages: barrier, fold, barrier and pull in one launch (EXT_MPI_AMD_IPC_FUSED_MAX
       bytes per rank, default 1 MiB; 0 disables) */
    const char *fm = getenv("EXT_MPI_AMD_IPC_FUSED_MAX");
    const long fused_max = fm ? atol(fm) : (1L << 20);
    h->fused = R > 1 && (long)h->bytes <= fused_max;
  }
  if (getenv("EXT_MPI_AMD_DEBUG_IPC") && (attempt > 0 || atoi(getenv("EXT_MPI_AMD_DEBUG_IPC")) >= 2))
    fprintf(stderr, "ipc rank %d: own send %p recv %p outbox %p bytes %zu, %d buckets, slot %d, %d attempt(s)\n",
            cm->rank, h->dsend[0], h->drecv[0], h->outbox, h->bytes, nb, slot, attempt + 1);
  rc = upload_buckets(h, b, nb);
  free(b);
  return rc;
}

unsigned *ipc_go(const emac_handle *h) { return ipc_go_slot(h, h->slot); }
unsigned *ipc_go_slot(const emac_handle *h, int slot) {
  return (unsigned *)((char *)g_comms[h->comm].sync + offsetof(emac_sync, go)) + slot;
}

/* The end of a peer-mapped handle's set-up (after ipc_allreduce_init / node_ipc_init, whose
   exchanges every rank runs whatever failed locally): every rank learns whether every other one
   succeeded. A local failure after the last exchange -- an upload, the release event, the handle
   table -- would otherwise leave this rank's peers holding mappings of its send buffer and a
   handle they would Start alone. On failure every rank releases its half-made handle (closing its
   mappings) and, when some rank's exported send buffer is caller memory, the ranks agree once more
   -- ext_mpi_amd_done's rule -- so that no peer maps a caller buffer when the init returns. Takes
   ownership of h. */
int ipc_init_settle(emac_handle *h, emac_comm *cm, int rc, int *handle) {
  int agreed = 0, collective;
  if (!rc) rc = finish_init(h, handle);
  if (cm->size > 1) agreed = ipc_agree(cm, rc == 0);
  if (!rc && !agreed) return 0;
  if (!rc) { /* this rank succeeded, a peer did not */
    g_handles[*handle] = NULL;
    *handle = -1;
    rc = agreed;
  }
  collective = h->done_collective && cm->size > 1;
  handle_release(h);
  if (collective) ipc_agree(cm, 1);
  return rc;
}

/* IPC form: node barrier `phase` (0 before the fold: every rank's send buffer is ready and its
   receive buffer free; 1 after it: every fan-out store has landed) on the handle's stream. The
   Start is named by its phase-1 epoch (`tag`, ipc_sync.hpp). Phase 0 is preceded by a
   system-scope release of everything enqueued before it, done by the command processor on every
   XCD: the peers' loads of this rank's buffers do not depend on where its writers ran. */
int ipc_barrier(emac_handle *h, int phase) {
  emac_comm *cm = &g_comms[h->comm];
  int rc;
  unsigned long epoch, tag;
  h->tune.ops++;
  if (phase == 0 && h->ev_release && (rc = emac_gpu_event_record(h->ev_release, h->stream))) return rc;
  epoch = ++h->epoch[phase];
  tag = phase ? epoch : h->epoch[1] + 1;
  return emac_gpu_node_barrier(cm->sync, (void *const *)cm->d_peer_sync, h->slot, phase, epoch, tag, cm->size, cm->rank,
                               cm->err + h->slot, cm->timeout_ticks, h->stream);
}

/* barrier errors are reported through the slot's pinned word (ipc_sync.hpp), read and cleared
   when the Start is waited for: the next Start on the handle synchronises normally */
int ipc_status(const emac_handle *h) {
  volatile int *w;
  int e, k;
  if (h->kind != KIND_IPC || !h->slot_held) return 0;
  w = (volatile int *)g_comms[h->comm].err + h->slot;
  e = *w;
  *w = 0;
  for (k = 1; h->join && k < h->join->nparts; k++) { /* every part's slot (its first is h->slot) */
    w = (volatile int *)g_comms[h->comm].err + h->join->slot[k];
    e |= *w;
    *w = 0;
  }
  if (!e) return 0;
  fprintf(stderr, "ext_mpi_amd: rank %d: node barrier failed:%s%s\n", g_comms[h->comm].rank,
          (e & EMAC_SYNC_ERR_TIMEOUT) ? " a peer did not arrive within EXT_MPI_AMD_BARRIER_TIMEOUT" : "",
          (e & EMAC_SYNC_ERR_ABORTED) ? " a peer gave up on this Allreduce" : "");
  return EMAC_ERR_TRANSPORT;
}

int ext_mpi_amd_handle_ipc_flags(int handle) {
  const emac_handle *h = handle_get(handle);
  int f = 0;
  if (!h) return EMAC_ERR_ARG;
  if (h->kind != KIND_IPC) return 0;
  if (g_comms[h->comm].cross_device) f |= EXT_MPI_AMD_IPC_CROSS_DEVICE;
  if (h->ev_release) f |= EXT_MPI_AMD_IPC_RELEASE_EVENT;
  if (h->join && h->join->fused) f |= h->join->sys_stores ? EXT_MPI_AMD_IPC_SYS_STORES : EXT_MPI_AMD_IPC_DEV_STORES;
  return f;
}
