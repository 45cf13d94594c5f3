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
    unsigned char free_slots[EMAC_SYNC_SLOTS / 8];
  } nx_export;
  nx_export mine, all[EMAC_MAX_RANKS];
  void *peer_part[EMAC_MAX_RANKS], *peer_out[EMAC_MAX_RANKS];
  emac_share *sh[EMAC_MAX_RANKS] = {0};
  int nsh[EMAC_MAX_RANKS] = {0};
  emac_bucket *b = NULL;
  const int N = cm->size, R = h->plan.nranks;
  const long ts = h->plan.tsize;
  int attempt, r, k, me, i, slot, nb, pc;
  h->part_bytes = h->outbox_bytes = h->bytes > 16 ? h->bytes : 16;
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
    mine.status = rc == 0;
    for (r = 0; r < EMAC_SYNC_SLOTS; r++)
      if (!cm->slot_used[r]) mine.free_slots[r >> 3] |= (unsigned char)(1u << (r & 7));
    if (cm->ag(cm->ag_ctx, &mine, all, (long)sizeof(mine))) return EMAC_ERR_TRANSPORT;
    for (r = 0; r < N; r++) {
      if (!all[r].status && !rc) rc = EMAC_ERR_TRANSPORT;
      if (all[r].lack > 0) grow = 1;
    }
    if (rc) return rc; /* the same verdict on every rank */
    if (!grow) break;
    if (attempt == EMAC_IPC_ATTEMPTS - 1) return EMAC_ERR_MALLOC;
    if ((rc = arena_grow(cm, 0, lack))) return rc;
  }
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
  if ((rc = ipc_agree(cm, rc == 0))) return rc;
  for (slot = 0; slot < EMAC_SYNC_SLOTS; slot++) { /* the lowest slot free on every rank */
    for (r = 0; r < N && (all[r].free_slots[slot >> 3] >> (slot & 7)) & 1; r++);
    if (r == N) break;
  }
  if (slot == EMAC_SYNC_SLOTS) return EMAC_ERR_MALLOC; /* the same verdict on every rank */
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
  if (!rc) /* the halving flow folds log2 N levels of pairs, one step over every node a left fold */
    rc = node_fold_codes(N, N > 1 && emac_node_single(&h->ns) == 2 ? h->ns.nsteps : 1, h->plan.dtype, &h->xcodes);
  if (!rc && !(b = (emac_bucket *)calloc((size_t)(k + h->plan.npieces * R) + 1, sizeof(emac_bucket)))) rc = EMAC_ERR_MALLOC;
  /* 1. the copy-in: every owner chunk into this node's partial block (at its message offset) */
  for (nb = 0, pc = 0; !rc && pc < h->plan.npieces; pc++)
    for (i = 0; i < R; i++) {
      const long off = h->plan.chunk_off[(size_t)pc * R + i], len = h->plan.chunk_len[(size_t)pc * R + i];
      emac_bucket *bk = &b[nb];
      int t;
      if (len <= 0) continue;
      memset(bk, 0, sizeof(*bk));
      for (t = 0; t < R; t++) bk->src[t] = h->dsend[h->plan.leaf_rank[i][t]];
      bk->dst[0] = h->part;
      bk->ndst = 1;
      place_bucket(bk, R, off, len, ts);
      nb++;
    }
  h->nsrc = R;
  h->fan = 0;
  if (!rc) rc = upload_buckets(h, b, nb);
  /* 2. this node's shares: the N partials in place, in the line's order, into the outbox */
  for (nb = 0, me = 0; !rc && me < R; me++)
    for (i = 0; i < nsh[me]; i++) {
      const emac_share *x = &sh[me][i];
      emac_bucket *bk = &b[nb];
      int l;
      if (x->node != cm->rank || x->len <= 0) continue;
      memset(bk, 0, sizeof(*bk));
      for (l = 0; l < x->nleaf; l++) bk->src[l] = peer_part[x->leaf_node[l]]; /* in h->xcodes' order */
      bk->dst[0] = h->outbox;
      bk->ndst = 1;
      place_bucket(bk, x->nleaf, x->off, x->len, ts);
      nb++;
    }
  if (!rc) rc = upload_launch_fan(h, &h->xfold[0], b, nb, N, 2);
  /* 3. the pull, fused with the copy-out: every share read once from its node's outbox and stored
     into all R receive buffers, the nodes after this one first (their loads head for different
     GPUs' links), this node's own last */
  for (nb = 0, k = 1; !rc && k <= N; k++) {
    const int q = (cm->rank + k) % N;
    for (me = 0; me < R; me++)
      for (i = 0; i < nsh[me]; i++) {
        const emac_share *x = &sh[me][i];
        emac_bucket *bk = &b[nb];
        int d;
        if (x->node != q || x->len <= 0) continue;
        memset(bk, 0, sizeof(*bk));
        bk->src[0] = peer_out[q];
        for (d = 0; d < R; d++) bk->dst[d] = h->drecv[d];
        bk->ndst = R;
        place_bucket(bk, 1, x->off, x->len, ts);
        nb++;
      }
  }
  if (!rc) rc = upload_launch_fan(h, &h->pull, b, nb, 1, 2);
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
