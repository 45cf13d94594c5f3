/*
 * engine_join.c -- the NODE form over several nodes: every rank of this node in this process,
 * the nodes joined by a communicator whose members are the nodes -- RCCL (or loopback) legs of
 * the inter-node ports schedule, or peer-mapped shares (engine_int.h).
 */
#include "engine_int.h"

/* ------------------------- NODE form over several nodes ------------------------- */

/* The node's copy-out (its allgather): every owner chunk, from its owner's receive buffer, stored
   into the R - 1 other receive buffers (one emac_gpu_copy_fan launch). `b`: scratch of npieces * R
   buckets. */
static int build_node_fanout(emac_handle *h, emac_bucket *b) {
  const int R = h->plan.nranks;
  emac_edge *edges = NULL;
  emac_launch *F = &h->fanout;
  int nfb = 0, pc, c, r, rc;
  if (R < 2) return 0;
  for (pc = 0; pc < h->plan.npieces; pc++)
    for (c = 0; c < R; c++) {
      const long off = h->plan.chunk_off[(size_t)pc * R + c], len = h->plan.chunk_len[(size_t)pc * R + c];
      const int owner = h->plan.pos_rank[c];
      emac_bucket *bk = &b[nfb];
      if (len <= 0) continue;
      memset(bk, 0, sizeof(*bk));
      bk->src[0] = h->drecv[owner];
      for (r = 0; r < R; r++)
        if (r != owner) bk->dst[bk->ndst++] = h->drecv[r];
      place_bucket(bk, 1, off, len, h->plan.tsize);
      nfb++;
    }
  if ((rc = emac_layout(b, nfb, EMAC_SUM, 1, 0, 0, &edges, &F->nedges, &F->ntiles, &F->tiles_per_bucket, &F->all_full,
                        &F->unroll)))
    return rc;
  F->nb = nfb;
  if (nfb && (rc = emac_gpu_malloc((void **)&F->d_buckets, sizeof(emac_bucket) * (size_t)nfb)) == 0)
    rc = emac_gpu_memcpy(F->d_buckets, b, sizeof(emac_bucket) * (size_t)nfb);
  if (!rc && F->nedges && (rc = emac_gpu_malloc((void **)&F->d_edges, sizeof(emac_edge) * (size_t)F->nedges)) == 0)
    rc = emac_gpu_memcpy(F->d_edges, edges, sizeof(emac_edge) * (size_t)F->nedges);
  free(edges);
  return rc;
}


/* The fold tree of a share of the peer-mapped node join over n partials: a left fold (levels 1),
   or `levels` levels of pairs (the halving flow) -- the shape of a '6;1 -2 ... 2 ...' plan */
static int node_fold_codes(int n, int levels, int dtype, emac_codes *c) {
  emac_copyin cfg;
  emac_plan p;
  char cp[96];
  int at, k, rc;
  memset(c, 0, sizeof(*c));
  if (levels <= 1) {
    c->first[0] = 1;
    c->close[n - 1] = 1;
    c->nlev = 1;
    c->nleaf = n;
    return 0;
  }
  at = snprintf(cp, sizeof(cp), "6;1");
  for (k = 0; k < levels; k++) at += snprintf(cp + at, sizeof(cp) - (size_t)at, " -2");
  for (k = 0; k < levels; k++) at += snprintf(cp + at, sizeof(cp) - (size_t)at, " 2");
  if ((rc = emac_parse_copyin(cp, &cfg))) return rc;
  cfg.sockets = 1;
  if ((rc = emac_plan_build(&p, n, (long)n * 16, dtype, EMAC_SUM, &cfg))) return rc;
  *c = p.codes;
  emac_plan_free(&p);
  return 0;
}

/* A bucket of the peer-mapped join before placement: pointers at message element 0, elements
   [off, off + len) of the message */
typedef struct {
  emac_bucket b;
  int nsrc;
  long off, len;
} jproto;

/* the prototypes' elements inside [lo, hi), placed into b (pointers at their first element,
   alignment split): the number of buckets */
static int place_part(emac_bucket *b, const jproto *p, int n, long lo, long hi, long ts) {
  int i, nb = 0;
  for (i = 0; i < n; i++) {
    const long a = p[i].off > lo ? p[i].off : lo, e = p[i].off + p[i].len < hi ? p[i].off + p[i].len : hi;
    if (e <= a) continue;
    b[nb] = p[i].b;
    place_bucket(&b[nb], p[i].nsrc, a, e - a, (int)ts);
    nb++;
  }
  return nb;
}

/* The join's settings from this rank's environment; node_ipc_init takes rank 0's for every rank (the
   ranks must run the same slot and epoch protocol, whatever their environments say):
   EXT_MPI_AMD_JOIN_PARTS (0: unset), EXT_MPI_AMD_JOIN=streams, EXT_MPI_AMD_JOIN_SYSSTORE=1 (A/B:
   system-scope partial stores in the fused join with every node on one GPU too) */
typedef struct {
  int parts, streams, sys_stores;
} join_env;

static join_env join_env_local(void) {
  const char *p = getenv("EXT_MPI_AMD_JOIN_PARTS"), *j = getenv("EXT_MPI_AMD_JOIN"), *y = getenv("EXT_MPI_AMD_JOIN_SYSSTORE");
  join_env e;
  e.parts = p && *p ? atoi(p) : 0;
  if (p && *p && e.parts < 1) e.parts = 1;
  e.streams = j && !strcmp(j, "streams");
  e.sys_stores = y && atoi(y) > 0;
  return e;
}

/* the parts of the pipelined join: the agreed EXT_MPI_AMD_JOIN_PARTS (1: the serial join), else 2
   over several nodes from EMAC_JOIN_MIN_BYTES per rank. With nodes sharing one MI355X (16 MiB per
   rank, 8 ranks per node) the fused join with 2 parts took 150.7 against 187.6 us per Start at 2
   nodes and 274.8 against 389.6 at 4; 4 parts were no faster (profiles/r05/join/) */
static int join_parts(const emac_handle *h, int nodes, int env_parts) {
  int n = nodes > 1 && (long)h->bytes >= EMAC_JOIN_MIN_BYTES ? 2 : 1;
  if (env_parts > 0) n = env_parts;
  return n < 1 ? 1 : n > EMAC_JOIN_PARTS ? EMAC_JOIN_PARTS : n;
}

/* a launch of nb buckets of nsrc leaves with the tiles of schedule `unroll` (the fused join's
   segments: the kernel's own U per stage) */
static int upload_forced(emac_launch *L, emac_bucket *b, int nb, int nsrc, int unroll) {
  emac_edge *edges = NULL;
  int rc;
  memset(L, 0, sizeof(*L));
  if ((rc = emac_layout_as(b, nb, EMAC_SUM, nsrc, 0, 0, unroll, &edges, &L->nedges, &L->ntiles, &L->tiles_per_bucket,
                           &L->all_full, &L->unroll)))
    return rc;
  L->nb = nb;
  if (nb && (rc = emac_gpu_malloc((void **)&L->d_buckets, sizeof(emac_bucket) * (size_t)nb)) == 0)
    rc = emac_gpu_memcpy(L->d_buckets, b, sizeof(emac_bucket) * (size_t)nb);
  if (!rc && L->nedges && (rc = emac_gpu_malloc((void **)&L->d_edges, sizeof(emac_edge) * (size_t)L->nedges)) == 0)
    rc = emac_gpu_memcpy(L->d_edges, edges, sizeof(emac_edge) * (size_t)L->nedges);
  free(edges);
  return rc;
}

/* first element of part k of n over count elements: equal parts cut at 1024-element multiples (the
   cuts keep every bucket's 16-byte phase), the last part to the end */
static long join_cut(long count, int n, int k) {
  long c;
  if (k >= n) return count;
  c = count / n * k / 1024 * 1024;
  return c < count ? c : count;
}

/* The NODE form over peer-mapped nodes: node_comm_allreduce_init on an ext_mpi_amd_comm_init_ipc
   communicator -- one process per GPU, each member a node of R ranks whose buffers all live on
   its GPU. The inter-node schedule must be one reduce-scatter step over every node (EXT_MPI_NUM_PORTS
   'N(-(N-1) (N-1))', the default for a node count that is not a power of two) -- every element's
   value is then ONE fold of the N node partials in its line's order, whoever computes it -- or,
   for SUM, one port per step over 2^k nodes (the default there) -- every value a balanced tree of
   pairs over the task bits (plan.c emac_node_single, emac_node_shares): so the inter-node legs
   become peer loads instead of point-to-point lines. A Start runs
    1. the node's copy-in: every owner chunk folded over the node's send buffers, in the plan's leaf
       order, into this node's partial block (arena memory the peers map; fold_launch, tuned);
    2. barrier(in); the fold of this node's share of every node rank's chunk: the N nodes' partials
       read in place (system-coherent loads over xGMI), in the line's order, into this node's outbox
       (arena); barrier(out) -- the IPC form's protocol (ipc_sync.hpp, epochs, timeout recovery);
    3. the pull fused with the copy-out: every node's share (this node's own too) read once from
       its outbox and stored into all R receive buffers (emac_gpu_copy_fan_remote), the nodes
       after this one first.
   No caller memory is exported -- the peers read only the two arena blocks -- so the handle's Done
   is local. Collective over the communicator (the exchanges run whatever failed locally). */
static int node_ipc_init(emac_handle *h, emac_comm *cm, int rc) {
  typedef struct {
    long lack;
    int status;
    int seg[2];
    long offset[2];
    join_env env; /* rank 0's is every rank's */
    unsigned char free_slots[EMAC_SYNC_SLOTS / 8];
  } nx_export;
  nx_export mine, all[EMAC_MAX_RANKS];
  void *peer_part[EMAC_MAX_RANKS], *peer_out[EMAC_MAX_RANKS];
  emac_share *sh[EMAC_MAX_RANKS] = {0};
  int nsh[EMAC_MAX_RANKS] = {0};
  emac_bucket *b = NULL;
  jproto *pin = NULL, *psh = NULL, *ppl = NULL;
  const int N = cm->size, R = h->plan.nranks;
  const long ts = h->plan.tsize;
  emac_join *J = NULL;
  join_env env;
  int attempt, r, k, me, i, slot, pc, nparts, pslot[EMAC_JOIN_PARTS], nin = 0, nshr = 0, npl = 0;
  h->part_bytes = h->outbox_bytes = h->bytes > 16 ? h->bytes : 16;
  /* the pipelined join's state, before the exchange: a failure here is in its verdict */
  if (!rc && !(J = (emac_join *)calloc(1, sizeof(emac_join)))) rc = EMAC_ERR_MALLOC;
  for (attempt = 0;; attempt++) {
    long lack = 0;
    int grow = 0;
    if (!rc && !h->part && arena_alloc(cm, (long)h->part_bytes, &h->part))
      lack += (long)(h->part_bytes + EMAC_ARENA_ALIGN - 1) / EMAC_ARENA_ALIGN * EMAC_ARENA_ALIGN;
    if (!rc && !h->outbox && arena_alloc(cm, (long)h->outbox_bytes, &h->outbox))
      lack += (long)(h->outbox_bytes + EMAC_ARENA_ALIGN - 1) / EMAC_ARENA_ALIGN * EMAC_ARENA_ALIGN;
    memset(&mine, 0, sizeof(mine));
    for (k = 0; !rc && !lack && k < 2; k++) {
      void *p = k ? h->outbox : h->part;
      int sg;
      if (!arena_owns(cm, p, &sg)) {
        rc = EMAC_ERR_ARG;
      } else {
        mine.seg[k] = sg;
        mine.offset[k] = (long)((char *)p - (char *)cm->seg[sg].base);
      }
    }
    mine.lack = rc ? 0 : lack;
    mine.env = join_env_local();
    mine.status = rc == 0;
    for (r = 0; r < EMAC_SYNC_SLOTS; r++)
      if (!cm->slot_used[r]) mine.free_slots[r >> 3] |= (unsigned char)(1u << (r & 7));
    if (cm->ag(cm->ag_ctx, &mine, all, (long)sizeof(mine))) rc = EMAC_ERR_TRANSPORT;
    for (r = 0; !rc && r < N; r++) {
      if (!all[r].status) rc = EMAC_ERR_TRANSPORT;
      if (all[r].lack > 0) grow = 1;
    }
    if (!rc && grow && attempt == EMAC_IPC_ATTEMPTS - 1) rc = EMAC_ERR_MALLOC;
    if (!rc && grow) rc = arena_grow(cm, 0, lack);
    if (rc || !grow) break; /* the same verdict on every rank */
  }
  if (rc) {
    free(J);
    return rc;
  }
  env = all[0].env;
  for (r = 0; r < N; r++) {
    if (r == cm->rank) {
      peer_part[r] = h->part;
      peer_out[r] = h->outbox;
      continue;
    }
    peer_part[r] = all[r].seg[0] < cm->peer_nseg[r] ? (char *)cm->peer_seg[r][all[r].seg[0]] + all[r].offset[0] : NULL;
    peer_out[r] = all[r].seg[1] < cm->peer_nseg[r] ? (char *)cm->peer_seg[r][all[r].seg[1]] + all[r].offset[1] : NULL;
    if (!peer_part[r] || !peer_out[r]) rc = EMAC_ERR_TRANSPORT;
  }
  if ((rc = ipc_agree(cm, rc == 0))) {
    free(J);
    return rc;
  }
  /* the pipelined join (emac_join): the same part count on every rank (the message size and rank
     0's environment), one slot per part */
  /* the share fold's tree: the halving flow folds log2 N levels of pairs, one step over every node a
     left fold */
  if ((rc = node_fold_codes(N, N > 1 && emac_node_single(&h->ns) == 2 ? h->ns.nsteps : 1, h->plan.dtype, &h->xcodes))) {
    free(J);
    return rc; /* (a function of the shape alone: the same on every rank) */
  }
  nparts = join_parts(h, N, env.parts);
  /* a shape the fused join has no kernel for (leaf counts other than 1, 2, 4, 8, MIN / MAX,
     irregular fold trees) keeps the serial join -- the same verdict on every rank (same shape) */
  if (nparts > 1 && !env.streams &&
      (h->plan.op != EMAC_SUM || emac_gpu_join_fused(h->plan.dtype, R, &h->plan.codes, &h->xcodes, nparts, 3, NULL, NULL, NULL,
                                                     NULL, NULL, NULL, N, cm->rank, NULL, 0, NULL, 0, NULL)))
    nparts = 1;
  for (k = 0, slot = 0; k < nparts; k++, slot++) { /* the lowest slots free on every rank */
    for (; slot < EMAC_SYNC_SLOTS; slot++) {
      for (r = 0; r < N && (all[r].free_slots[slot >> 3] >> (slot & 7)) & 1; r++);
      if (r == N) break;
    }
    if (slot == EMAC_SYNC_SLOTS) {
      free(J);
      return EMAC_ERR_MALLOC; /* the same verdict on every rank */
    }
    pslot[k] = slot;
  }
  if (nparts > 1) {
    h->join = J;
    h->join->nparts = nparts;
    h->join->fused = !env.streams;
    /* the copy-in's partials go to memory at system scope when some node runs on another GPU
       (every rank has the same cross_device verdict), else at device scope */
    h->join->sys_stores = cm->cross_device || env.sys_stores;
    for (k = 0; k < nparts; k++) {
      h->join->slot[k] = pslot[k];
      cm->slot_used[pslot[k]] = 1;
      cm->err[pslot[k]] = 0;
      h->join->epoch[k][0] = cm->slot_epoch[pslot[k]][0];
      h->join->epoch[k][1] = cm->slot_epoch[pslot[k]][1];
    }
  } else {
    free(J);
  }
  slot = pslot[0];
  h->slot = slot;
  cm->slot_used[slot] = 1;
  h->slot_held = 1;
  cm->err[slot] = 0;
  {
    const char *e = getenv("EXT_MPI_AMD_IPC_RELEASE"); /* as ipc_allreduce_init */
    const int rel = e ? atoi(e) > 0 : cm->cross_device;
    if (N > 1 && rel && (rc = emac_gpu_event_create_release(&h->ev_release))) return rc;
  }
  h->epoch[0] = cm->slot_epoch[slot][0];
  h->epoch[1] = cm->slot_epoch[slot][1];
  /* the parts of every node rank's chunk (plan.c emac_node_shares; one node: the chunk itself) */
  for (me = 0; me < R && !rc; me++) {
    if (N > 1) {
      rc = emac_node_shares(&h->plan, &h->ns, me, &sh[me], &nsh[me]);
    } else if (!(sh[me] = (emac_share *)calloc((size_t)h->plan.npieces + 1, sizeof(emac_share)))) {
      rc = EMAC_ERR_MALLOC;
    } else {
      for (pc = 0; pc < h->plan.npieces; pc++) {
        emac_share *x = &sh[me][nsh[me]++];
        x->off = h->plan.chunk_off[(size_t)pc * R + h->plan.rank_pos[me]];
        x->len = h->plan.chunk_len[(size_t)pc * R + h->plan.rank_pos[me]];
        x->node = 0;
        x->nleaf = 1;
      }
    }
  }
  for (me = 0, k = 0; me < R; me++) k += nsh[me];
  if (!rc && (!(pin = (jproto *)calloc((size_t)h->plan.npieces * R + 1, sizeof(jproto))) ||
              !(psh = (jproto *)calloc((size_t)k + 1, sizeof(jproto))) || !(ppl = (jproto *)calloc((size_t)k + 1, sizeof(jproto))) ||
              !(b = (emac_bucket *)calloc((size_t)(k + h->plan.npieces * R) + 1, sizeof(emac_bucket)))))
    rc = EMAC_ERR_MALLOC;
  /* 1. the copy-in: every owner chunk into this node's partial block (at its message offset) */
  for (pc = 0; !rc && pc < h->plan.npieces; pc++)
    for (i = 0; i < R; i++) {
      const long off = h->plan.chunk_off[(size_t)pc * R + i], len = h->plan.chunk_len[(size_t)pc * R + i];
      jproto *x = &pin[nin];
      int t;
      if (len <= 0) continue;
      for (t = 0; t < R; t++) x->b.src[t] = h->dsend[h->plan.leaf_rank[i][t]];
      x->b.dst[0] = h->part;
      x->b.ndst = 1;
      x->nsrc = R;
      x->off = off;
      x->len = len;
      nin++;
    }
  /* 2. this node's shares: the N partials in place, in the line's order, into the outbox */
  for (me = 0; !rc && me < R; me++)
    for (i = 0; i < nsh[me]; i++) {
      const emac_share *x = &sh[me][i];
      jproto *y = &psh[nshr];
      int l;
      if (x->node != cm->rank || x->len <= 0) continue;
      for (l = 0; l < x->nleaf; l++) y->b.src[l] = peer_part[x->leaf_node[l]]; /* in h->xcodes' order */
      y->b.dst[0] = h->outbox;
      y->b.ndst = 1;
      y->nsrc = x->nleaf;
      y->off = x->off;
      y->len = x->len;
      nshr++;
    }
  /* 3. the pull, fused with the copy-out: every share read once from its node's outbox and stored
     into all R receive buffers, the nodes after this one first (their loads head for different
     GPUs' links), this node's own last */
  for (k = 1; !rc && k <= N; k++) {
    const int q = (cm->rank + k) % N;
    for (me = 0; me < R; me++)
      for (i = 0; i < nsh[me]; i++) {
        const emac_share *x = &sh[me][i];
        jproto *y = &ppl[npl];
        int d;
        if (x->node != q || x->len <= 0) continue;
        y->b.src[0] = peer_out[q];
        for (d = 0; d < R; d++) y->b.dst[d] = h->drecv[d];
        y->b.ndst = R;
        y->nsrc = 1;
        y->off = x->off;
        y->len = x->len;
        npl++;
      }
  }
  h->nsrc = R;
  h->fan = 0;
  if (!h->join) { /* the serial join: one launch per stage over every bucket */
    if (!rc) rc = upload_buckets(h, b, place_part(b, pin, nin, 0, h->plan.count, ts)); /* tuned */
    if (!rc) rc = upload_launch_fan(h, &h->xfold[0], b, place_part(b, psh, nshr, 0, h->plan.count, ts), N, 2);
    if (!rc) rc = upload_launch_fan(h, &h->pull, b, place_part(b, ppl, npl, 0, h->plan.count, ts), 1, 2);
  } else if (h->join->fused) { /* part k: the buckets' elements inside [lo[k], lo[k + 1]), one launch */
    emac_join *J = h->join;
    emac_join_ctl zero;
    memset(&zero, 0, sizeof(zero));
    for (k = 0; k <= J->nparts; k++) J->lo[k] = join_cut(h->plan.count, J->nparts, k);
    for (k = 0; !rc && k < J->nparts; k++) {
      /* the kernel's tiles (join_fused.hip: 1024-lane workgroups): 2 vectors per lane for the copy-in
         and the pull, 1 for the share fold -- in layout units of EMAC_BLOCK lanes, U 8 and 4 */
      if (!rc) rc = upload_forced(&J->in[k], b, place_part(b, pin, nin, J->lo[k], J->lo[k + 1], ts), R, 8 | 1 << 4);
      if (!rc) rc = upload_forced(&J->fold[k], b, place_part(b, psh, nshr, J->lo[k], J->lo[k + 1], ts), N, 4 | 1 << 4);
      if (!rc) rc = upload_forced(&J->pull[k], b, place_part(b, ppl, npl, J->lo[k], J->lo[k + 1], ts), 1, 8 | 1 << 4);
    }
    if (!rc && (rc = emac_gpu_malloc(&J->ctl, sizeof(emac_join_ctl))) == 0) rc = emac_gpu_memcpy(J->ctl, &zero, sizeof(zero));
    if (!rc) {
      /* join_fused.hip: one 1024-lane workgroup per CU; the nodes sharing this GPU (by UUID: the
         1-GPU rehearsal, or a mixed placement) divide it, so every node's workgroups find room
         beside the others' waiting ones */
      const int g = emac_gpu_join_grid() / (cm->same_device > 1 ? cm->same_device : 1);
      J->grid = g < 8 ? 8 : g > 4096 ? 4096 : g;
    }
  } else { /* part k: the buckets' elements inside [lo[k], lo[k + 1]) */
    emac_join *J = h->join;
    for (k = 0; k <= J->nparts; k++) J->lo[k] = join_cut(h->plan.count, J->nparts, k);
    for (k = 0; !rc && k < J->nparts; k++) {
      if (!rc) rc = upload_launch_as(h, &J->in[k], b, place_part(b, pin, nin, J->lo[k], J->lo[k + 1], ts), R,
                                     emac_tree_kind(&h->plan.codes, h->plan.op) == 1);
      if (!rc) rc = upload_launch_fan(h, &J->fold[k], b, place_part(b, psh, nshr, J->lo[k], J->lo[k + 1], ts), N, 2);
      if (!rc) rc = upload_launch_fan(h, &J->pull[k], b, place_part(b, ppl, npl, J->lo[k], J->lo[k + 1], ts), 1, 2);
      if (!rc) rc = emac_gpu_event_create(&J->ev_in[k]);
      if (!rc) rc = emac_gpu_event_create(&J->ev_fold[k]);
    }
    if (!rc) rc = emac_gpu_event_create(&J->ev_done);
    if (!rc) rc = emac_gpu_stream_create(&J->s_fold);
    if (!rc) rc = emac_gpu_stream_create(&J->s_pull);
  }
  free(pin);
  free(psh);
  free(ppl);
  for (me = 0; me < R; me++) free(sh[me]);
  free(b);
  return rc;
}

/* Every rank of this node in this process (the NODE form: all their buffers on this GPU), the
   nodes joined by `comm`, whose members are the nodes (RCCL, or loopback for testing), under the
   communicator's inter-node schedule (ext_mpi_amd_comm_set_node_ports with nodes == its size;
   otherwise emac_node_sched_build's default). A Start runs
    1. the node's copy-in: every owner chunk folded over the node's send buffers, in the plan's
       leaf order, into its owner's receive buffer -- the COMM form's reduce-scatter leg and fold
       without moving a byte, the leaves read where they lie (one launch, fold_launch);
    2. the node legs of every node rank me (emac_comm_program_nodes of global rank
       node * R + me; its column peers are rank me of the other nodes, i.e. the other members),
       one RCCL group per leg for all node ranks, ordered by node rank within each peer so that
       the k-th send of a pair matches its k-th receive, and each exchange step's fold for all
       node ranks in one launch;
    3. the copy-out: every owner chunk stored into the node's other receive buffers (the node
       allgather, emac_gpu_copy_fan).
   The bits are the COMM form's over nodes * R ranks, one per process -- the reference's
   multi-node composition (ext_mpi_native.c:879-1000: reduce_copyin over the node, the
   EXT_MPI_NUM_PORTS schedule between nodes, reduce_copyout). */
int ext_mpi_amd_node_comm_allreduce_init(int nranks, const void *const *sendbufs, void *const *recvbufs, long count,
                                         int dtype, int op, int comm, const char *copyin, int *handle) {
  emac_handle *h;
  emac_comm *cm;
  emac_copyin cfg;
  emac_bucket *b = NULL, *xb = NULL;
  emac_p2p *prog_ops[EMAC_MAX_RANKS] = {0};
  emac_fold *prog_folds[EMAC_MAX_RANKS] = {0};
  int prog_nops[EMAC_MAX_RANKS] = {0}, prog_nf[EMAC_MAX_RANKS] = {0};
  int nxb[2 * EMAC_MAX_NODE_STEPS] = {0};
  const int R = nranks;
  int rc, r, me, i, t, pc, c, nb = 0, nsteps, nf_all = 0, no_all = 0;
  long stage_max = 0;
  if (!handle || !sendbufs || !recvbufs || R < 1 || R > EMAC_MAX_RANKS || count < 0 || comm < 0 ||
      comm >= MAX_COMMS || !g_comms[comm].used)
    return EMAC_ERR_ARG;
  *handle = -1;
  cm = &g_comms[comm];
  if (cm->nodes > 1 && cm->nodes != cm->size) return EMAC_ERR_ARG; /* the members are the nodes */
  if ((rc = parse_cfg(copyin, R, &cfg))) return rc;
  if (emac_gpu_set_device(cm->device)) return EMAC_ERR_DEVICE;
  h = (emac_handle *)calloc(1, sizeof(emac_handle));
  if (!h) return EMAC_ERR_MALLOC;
  h->kind = KIND_COMM;
  h->hier = 1;
  h->comm = comm;
  h->device = cm->device;
  if ((rc = emac_plan_build(&h->plan, R, count, dtype, op, &cfg))) goto fail;
  h->me = cm->rank; /* this node */
  h->bytes = (size_t)count * (size_t)h->plan.tsize;
  h->nodes = cm->size;
  if (h->nodes > 1 && cm->nodes == cm->size)
    h->ns = cm->ns; /* ext_mpi_amd_comm_set_node_ports */
  else if (h->nodes > 1 && (rc = emac_node_sched_build(&h->ns, h->nodes, NULL)))
    goto fail;
  h->nbuf = R;
  h->nsrc = R;
  h->fan = 0;
  if (cm->ipc) { /* peer-mapped nodes: collective from here on, whatever fails locally */
    const int single = h->nodes > 1 ? emac_node_single(&h->ns) : 1;
    if (!single || (single == 2 && op != EMAC_SUM)) rc = EMAC_ERR_UNSUPPORTED; /* (the same on every rank) */
    for (r = 0; r < R && !rc; r++) rc = map_buffers(h, r, sendbufs[r], recvbufs[r]); /* local: device mirrors */
    h->kind = KIND_IPC;
    rc = node_ipc_init(h, cm, rc);
    if (!rc) rc = emac_gpu_stream_create(&h->stream);
    rc = ipc_init_settle(h, cm, rc, handle);
    goto out;
  }
  for (r = 0; r < R; r++)
    if ((rc = map_buffers(h, r, sendbufs[r], recvbufs[r]))) goto fail;
  /* 1. the copy-in: owner chunk (piece pc, position c) into its owner's receive buffer */
  b = (emac_bucket *)calloc((size_t)h->plan.npieces * R + 1, sizeof(emac_bucket));
  if (!b) {
    rc = EMAC_ERR_MALLOC;
    goto fail;
  }
  for (pc = 0; pc < h->plan.npieces; pc++)
    for (c = 0; c < R; c++) {
      const long off = h->plan.chunk_off[(size_t)pc * R + c], len = h->plan.chunk_len[(size_t)pc * R + c];
      emac_bucket *bk = &b[nb];
      if (len <= 0) continue;
      memset(bk, 0, sizeof(*bk));
      for (t = 0; t < R; t++) bk->src[t] = h->dsend[h->plan.leaf_rank[c][t]];
      bk->dst[0] = h->drecv[h->plan.pos_rank[c]];
      bk->ndst = 1;
      place_bucket(bk, R, off, len, h->plan.tsize);
      nb++;
    }
  if ((rc = upload_buckets(h, b, nb))) goto fail;
  /* 3. the copy-out: owner chunk into the R - 1 other receive buffers */
  if ((rc = build_node_fanout(h, b))) goto fail;
  /* 2. the node legs of every node rank: their programs, the peers turned into members */
  nsteps = h->nodes > 1 ? h->ns.nsteps + h->ns.nred : 0;
  for (me = 0; me < R && h->nodes > 1; me++) {
    long st = 0;
    if ((rc = emac_comm_program_nodes(&h->plan, &h->ns, h->me, me, (long)((unsigned long)h->dsend[me] & 15ul),
                                      &prog_ops[me], &prog_nops[me], &prog_folds[me], &prog_nf[me], &st)))
      goto fail;
    if (st > stage_max) stage_max = st;
    no_all += prog_nops[me];
    nf_all += prog_nf[me];
  }
  h->stage_stride = (stage_max + 255) / 256 * 256;
  if ((rc = emac_gpu_malloc(&h->staging, (size_t)(h->stage_stride > 0 ? h->stage_stride * R : 16)))) goto fail;
  h->ops = (emac_p2p *)malloc(sizeof(emac_p2p) * (size_t)(no_all + 1));
  xb = (emac_bucket *)calloc(2 * EMAC_MAX_NODE_STEPS * ((size_t)nf_all + 1), sizeof(emac_bucket));
  if (!h->ops || !xb) {
    rc = EMAC_ERR_MALLOC;
    goto fail;
  }
  /* legs in program order, node ranks in ascending order inside each (the pairs' matching order) */
  for (me = 0; me < R; me++)
    for (i = 0; i < prog_nops[me]; i++) {
      emac_p2p o = prog_ops[me][i];
      const int base = o.leg & ((1 << EMAC_LEG_STEP_SHIFT) - 1);
      if (base != EMAC_LEG_NODES_RS && base != EMAC_LEG_NODES_AG) continue; /* the node's own legs: steps 1, 3 */
      if (o.peer % R != me) {
        rc = EMAC_ERR_UNSUPPORTED; /* not a program of this shape */
        goto fail;
      }
      o.peer /= R;
      o.local = me;
      h->ops[h->nops++] = o;
    }
  for (me = 0; me < R; me++)
    for (i = 0; i < prog_nf[me]; i++) {
      const emac_fold *f = &prog_folds[me][i];
      int step;
      emac_bucket *bk;
      if ((f->leg & ((1 << EMAC_LEG_STEP_SHIFT) - 1)) != EMAC_LEG_NODES_FOLD) continue; /* step 1 folds the node */
      step = f->leg >> EMAC_LEG_STEP_SHIFT;
      if (step < 0 || step >= nsteps) {
        rc = EMAC_ERR_UNSUPPORTED; /* not a program of this shape */
        goto fail;
      }
      bk = &xb[(size_t)step * ((size_t)nf_all + 1) + (size_t)nxb[step]++];
      for (t = 0; t < f->nleaf; t++) bk->src[t] = leg_base_of(h, f->buf[t], me) + f->loff[t] - f->offset;
      bk->dst[0] = h->drecv[me];
      bk->ndst = 1;
      place_bucket(bk, f->nleaf, f->offset / h->plan.tsize, f->count, h->plan.tsize);
    }
  for (i = 0; i < nsteps; i++)
    if (nxb[i] &&
        (rc = upload_launch_as(h, &h->xfold[i], xb + (size_t)i * ((size_t)nf_all + 1), nxb[i], node_radix(&h->ns, i), 0)))
      goto fail;
  if ((rc = emac_gpu_stream_create(&h->stream))) goto fail;
  if (cm->loop_group >= 0) {
    loop_group *g = &g_loops[cm->loop_group];
    if (g->nh[h->me] < 0 || g->nh[h->me] >= MAX_LOOP_HANDLES) {
      rc = EMAC_ERR_MALLOC;
      goto fail;
    }
    h->loop_index = g->nh[h->me];
  }
  if ((rc = finish_init(h, handle))) goto fail;
  if (cm->loop_group >= 0) g_loops[cm->loop_group].handle[h->me][g_loops[cm->loop_group].nh[h->me]++] = *handle;
  rc = 0;
  goto out;
fail:
  handle_release(h);
out:
  for (me = 0; me < R; me++) {
    free(prog_ops[me]);
    free(prog_folds[me]);
  }
  free(b);
  free(xb);
  return rc;
}

int ext_mpi_amd_node_shares(int nodes, const int *ports, int ranks_per_node, long count, int dtype, const char *copyin,
                            int me, long *off, long *len, int *node, int *leaf_nodes, int max_shares, int *nshares,
                            int *levels) {
  emac_node_sched ns;
  emac_plan p;
  emac_copyin cfg;
  emac_share *sh = NULL;
  int rc, i, l, n = 0;
  if (!nshares || ranks_per_node < 1 || ranks_per_node > EMAC_MAX_RANKS || nodes < 2 || nodes > EMAC_MAX_NODES ||
      me < 0 || me >= ranks_per_node || count < 0)
    return EMAC_ERR_ARG;
  if ((rc = emac_node_sched_build(&ns, nodes, ports))) return rc;
  if ((rc = parse_cfg(copyin, ranks_per_node, &cfg))) return rc;
  if ((rc = emac_plan_build(&p, ranks_per_node, count, dtype, EMAC_SUM, &cfg))) return rc;
  rc = emac_node_shares(&p, &ns, me, &sh, &n);
  for (i = 0; !rc && i < n && i < max_shares; i++) {
    off[i] = sh[i].off;
    len[i] = sh[i].len;
    node[i] = sh[i].node;
    for (l = 0; l < nodes; l++) leaf_nodes[(size_t)i * (size_t)nodes + l] = sh[i].leaf_node[l];
  }
  if (!rc) *nshares = n;
  if (!rc && levels) *levels = emac_node_single(&ns) == 2 ? ns.nsteps : 1;
  if (!rc && n > max_shares) rc = EMAC_ERR_ARG;
  free(sh);
  emac_plan_free(&p);
  return rc;
}

/* A Start of the pipelined peer-mapped join (emac_join): per part k,
     copy-in stream (the handle's):  copy-in k -> [release] -> signal phase 0 of slot k -> event in[k]
     fold stream:   wait in[k] -> wait phase 0 of slot k (go) -> share fold k -> signal phase 1 -> event fold[k]
     pull stream:   wait fold[k] -> wait phase 1 of slot k -> pull + copy-out k (go)
   and the handle's stream waits for the pull stream's last launch, so Test / Wait / the next Start
   see the whole Allreduce. The local order between the stages of part k is the events'; the peers'
   is the slot's flags, as in the serial join (ipc_sync.hpp), with the same timeout and abandon
   rules per part: a part that times out costs the Start (every part's slot reports to Wait), and
   the next Start synchronises normally on every slot. `copyin` / `legs`: the copy-ins, the node
   legs (barriers, share folds, pulls), or both (ext_mpi_amd_start_legs times each alone; the legs
   alone read the partials the last copy-ins left). The next Start's copy-in of part k follows
   this Start's last pull on the handle's stream, so no node overwrites its partial while a peer's
   share fold of this Start may still read it (that peer signalled phase 1 of every part first). */
int join_start(emac_handle *h, int copyin, int legs) {
  emac_comm *cm = &g_comms[h->comm];
  emac_join *J = h->join;
  const int N = cm->size;
  int k, rc;
  if (J->fused) {
    emac_join_seg seg[3 * EMAC_JOIN_PARTS_MAX];
    unsigned long e0[EMAC_JOIN_PARTS_MAX], e1[EMAC_JOIN_PARTS_MAX];
    memset(seg, 0, sizeof(seg));
    for (k = 0; k < J->nparts; k++) {
      const emac_launch *st[3] = {&J->in[k], &J->fold[k], &J->pull[k]};
      int i;
      for (i = 0; i < 3; i++)
        seg[i * EMAC_JOIN_PARTS_MAX + k] = (emac_join_seg){st[i]->d_buckets, st[i]->nb, st[i]->ntiles, st[i]->tiles_per_bucket,
                                                           st[i]->all_full, st[i]->d_edges, st[i]->nedges};
      if (legs) { /* the epochs advance with the node legs only (the copy-ins alone signal nothing) */
        e0[k] = ++J->epoch[k][0];
        e1[k] = ++J->epoch[k][1];
      } else {
        e0[k] = J->epoch[k][0];
        e1[k] = J->epoch[k][1];
      }
    }
    h->tune.ops++;
    const int dev_scope = !J->sys_stores;
    return emac_gpu_join_fused(h->plan.dtype, h->nsrc, &h->plan.codes, &h->xcodes, J->nparts,
                               (copyin ? 1 : 0) | (legs ? 2 : 0) | (dev_scope ? 4 : 0),
                               seg, J->slot, e0, e1, cm->sync, (void *const *)cm->d_peer_sync, N, cm->rank,
                               cm->err + J->slot[0], cm->timeout_ticks, J->ctl, J->grid, h->stream);
  }
  for (k = 0; k < J->nparts; k++) {
    const emac_launch *I = &J->in[k], *X = &J->fold[k], *P = &J->pull[k];
    const int slot = J->slot[k];
    unsigned long e0, e1;
    h->tune.ops++;
    if (copyin && (I->nb || I->nedges) &&
        (rc = emac_gpu_fold(h->plan.dtype, h->plan.op, h->nsrc, 0, I->unroll, &h->plan.codes, I->d_buckets, I->nb, I->ntiles,
                            I->tiles_per_bucket, I->all_full, I->d_edges, I->nedges, h->stream)))
      return rc;
    if (!legs) continue; /* the copy-ins alone (ext_mpi_amd_start_legs: a part of the Start timed alone) */
    if (h->ev_release && (rc = emac_gpu_event_record(h->ev_release, h->stream))) return rc; /* as ipc_barrier(h, 0) */
    e0 = ++J->epoch[k][0];
    e1 = ++J->epoch[k][1];
    if ((rc = emac_gpu_node_signal((void *const *)cm->d_peer_sync, slot, 0, e0, N, cm->rank, h->stream)) ||
        (rc = emac_gpu_event_record(J->ev_in[k], h->stream)) || (rc = emac_gpu_stream_wait(J->s_fold, J->ev_in[k])) ||
        (rc = emac_gpu_node_wait(cm->sync, (void *const *)cm->d_peer_sync, slot, 0, e0, e1, N, cm->rank, cm->err + slot,
                                 cm->timeout_ticks, J->s_fold)))
      return rc;
    if ((X->nb || X->nedges) &&
        (rc = emac_gpu_fold_remote(h->plan.dtype, N > 1 ? h->plan.op : EMAC_SUM, N, X->unroll, &h->xcodes, X->d_buckets, X->nb,
                                   X->ntiles, X->tiles_per_bucket, X->all_full, X->d_edges, X->nedges, ipc_go_slot(h, slot),
                                   J->s_fold)))
      return rc;
    if ((rc = emac_gpu_node_signal((void *const *)cm->d_peer_sync, slot, 1, e1, N, cm->rank, J->s_fold)) ||
        (rc = emac_gpu_event_record(J->ev_fold[k], J->s_fold)) || (rc = emac_gpu_stream_wait(J->s_pull, J->ev_fold[k])) ||
        (rc = emac_gpu_node_wait(cm->sync, (void *const *)cm->d_peer_sync, slot, 1, e1, e1, N, cm->rank, cm->err + slot,
                                 cm->timeout_ticks, J->s_pull)))
      return rc;
    if ((P->nb || P->nedges) &&
        (rc = emac_gpu_copy_fan_remote(h->plan.tsize, h->plan.nranks, P->unroll, P->d_buckets, P->nb, P->ntiles,
                                       P->tiles_per_bucket, P->all_full, P->d_edges, P->nedges, ipc_go_slot(h, slot),
                                       J->s_pull)))
      return rc;
  }
  if (!legs) return 0;
  if ((rc = emac_gpu_event_record(J->ev_done, J->s_pull))) return rc;
  return emac_gpu_stream_wait(h->stream, J->ev_done);
}

/* the pipelined join's launches, streams and events; its slots (with their epochs) back to the
   communicator */
void join_free(emac_handle *h) {
  emac_join *J = h->join;
  int k;
  if (!J) return;
  if (J->s_fold) emac_gpu_stream_sync(J->s_fold);
  if (J->s_pull) emac_gpu_stream_sync(J->s_pull);
  for (k = 0; k < J->nparts; k++) {
    emac_gpu_free(J->in[k].d_buckets);
    emac_gpu_free(J->in[k].d_edges);
    emac_gpu_free(J->fold[k].d_buckets);
    emac_gpu_free(J->fold[k].d_edges);
    emac_gpu_free(J->pull[k].d_buckets);
    emac_gpu_free(J->pull[k].d_edges);
    emac_gpu_event_destroy(J->ev_in[k]);
    emac_gpu_event_destroy(J->ev_fold[k]);
    if (h->slot_held) {
      emac_comm *cm = &g_comms[h->comm];
      cm->slot_used[J->slot[k]] = 0;
      cm->slot_epoch[J->slot[k]][0] = J->epoch[k][0];
      cm->slot_epoch[J->slot[k]][1] = J->epoch[k][1];
    }
  }
  emac_gpu_event_destroy(J->ev_done);
  emac_gpu_free(J->ctl);
  if (J->s_fold) emac_gpu_stream_destroy(J->s_fold);
  if (J->s_pull) emac_gpu_stream_destroy(J->s_pull);
  free(J);
  h->join = NULL;
}

int ext_mpi_amd_handle_join_parts(int handle) {
  const emac_handle *h = handle_get(handle);
  if (!h) return EMAC_ERR_ARG;
  if (h->kind != KIND_IPC || !h->hier) return 0;
  return h->join ? h->join->nparts : 1;
}
