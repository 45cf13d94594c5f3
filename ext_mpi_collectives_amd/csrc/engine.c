/*
 * engine.c -- persistent-Allreduce handles of the MI355X bucket-reduction path (host C): the
 * handle table, buffer mapping, bucket upload and Start / Test / Wait / Done of every form.
 *
 * Mirrors the reference's handle life cycle (src/mpi/ext_mpi_native.c: init :657-1113 with
 * init_epilogue :389-655, Start :215-230, Test/Wait :232-267, Done :269-387) without its
 * text-IR pipeline: at init the planner (plan.c) fixes every owner chunk's fold tree, the
 * device-side bucket descriptors are written once (the analogue of byte_code.c:987-992's
 * descriptor H2D copy), buffers are mapped once; Start only enqueues work on the handle's
 * stream; Wait synchronises that stream.
 *
 * Execution forms (one unit each, engine_int.h):
 *  NODE: all R node ranks' buffers live in this process (one device). One fold launch per
 *        Start performs copy-in (reduce-scatter) AND copy-out (allgather fan-out): every
 *        bucket reads its R leaves once and stores the result into all R receive buffers.
 *  COMM: one rank per GPU. The reduce-scatter leg moves each rank's slice of every owner
 *        chunk to the owner with grouped RCCL send/recv (one all-to-all round over the
 *        fully connected xGMI links instead of log R recursive-halving rounds, each of
 *        which would be bound by ONE 153 GB/s link); the owner folds the R slices in the
 *        reference's order (bit-exact); the allgather leg pushes the owned chunk to every
 *        peer, again as one grouped round. RCCL's own reductions are never used: their
 *        summation order differs from the reference's.
 *  IPC:  one rank per GPU, the peers' buffers mapped (the reference's cudaIpc design).
 * Host (non-device) buffers are supported in every form by staging through device mirrors
 * (H2D before, D2H after, on the same stream), or read and written in place by the NODE form's
 * fold when the caller page-locked them.
 */
#include "engine_int.h"

static void mirror_free(emac_handle *h, void *p);

/* a launch or copy the handle enqueues (counted for the tuner's samples, emac_tune.ops) */
#define OP(h, call) ((h)->tune.ops++, (call))

emac_handle *g_handles[MAX_HANDLES];
emac_comm g_comms[MAX_COMMS];

static int new_handle_slot(void) {
  int i;
  for (i = 0; i < MAX_HANDLES; i++)
    if (!g_handles[i]) return i;
  return -1;
}

void handle_release(emac_handle *h) {
  int r;
  if (!h) return;
  if (h->stream) {
    emac_gpu_stream_sync(h->stream);
    if (h->own_stream) emac_gpu_stream_destroy(h->stream);
  }
  emac_gpu_free(h->d_buckets);
  emac_gpu_free(h->d_edges);
  emac_gpu_free(h->pull.d_buckets);
  emac_gpu_free(h->pull.d_edges);
  for (r = 0; r < h->tune.n; r++) {
    if (h->tune.L[r].d_buckets != h->d_buckets) emac_gpu_free(h->tune.L[r].d_buckets);
    if (h->tune.L[r].d_edges != h->d_edges) emac_gpu_free(h->tune.L[r].d_edges);
  }
  for (r = 0; r < EMAC_TUNE_SAMPLES; r++) {
    int e;
    for (e = 0; e < 2 * (EMAC_TUNE_SPAN - 1); e++) emac_gpu_event_destroy(h->tune.ev[r][e]);
  }
  for (r = 0; r < 2 * EMAC_MAX_NODE_STEPS; r++) {
    emac_gpu_free(h->xfold[r].d_buckets);
    emac_gpu_free(h->xfold[r].d_edges);
  }
  emac_gpu_free(h->fanout.d_buckets);
  emac_gpu_free(h->fanout.d_edges);
  emac_gpu_free(h->staging);
  for (r = 0; r < h->nbuf; r++) {
    const int same = h->dsend[r] == h->drecv[r];
    const int own = r == 0 && (h->send_arena || h->send_local); /* send side allocated by the IPC set-up */
    if (r == 0 && h->send_arena)
      arena_release(&g_comms[h->comm], h->dsend[0], (long)h->bytes);
    else if (r == 0 && h->send_local)
      emac_gpu_free(h->dsend[0]);
    else if (h->send_mirror[r])
      mirror_free(h, h->dsend[r]);
    if (h->recv_mirror[r] && h->drecv[r] && !(same && (h->send_mirror[r] || own))) mirror_free(h, h->drecv[r]);
    if (h->send_reg[r]) emac_gpu_host_unregister(h->user_send[r]);
    if (h->recv_reg[r]) emac_gpu_host_unregister(h->user_recv[r]);
  }
  for (r = 0; r < h->nmapped; r++) ipc_unmap(h->mapped[r]);
  if (h->outbox) arena_release(&g_comms[h->comm], h->outbox, (long)h->outbox_bytes);
  if (h->part) arena_release(&g_comms[h->comm], h->part, (long)h->part_bytes);
  emac_gpu_event_destroy(h->ev_release);
  for (r = 0; r <= EXT_MPI_AMD_LEG_ALL; r++) emac_gpu_graph_destroy(h->graph[r]);
  if (h->join) { /* the pipelined join: every part's slot, the first being h->slot */
    join_free(h);
  } else if (h->kind == KIND_IPC && h->slot_held) {
    emac_comm *cm = &g_comms[h->comm];
    cm->slot_used[h->slot] = 0;
    cm->slot_epoch[h->slot][0] = h->epoch[0];
    cm->slot_epoch[h->slot][1] = h->epoch[1];
  }
  free(h->ops);
  emac_plan_free(&h->plan);
  free(h);
}

/* device mirrors the peers never touch (every receive-side mirror; IPC send mirrors come from
   the communicator's arena, ipc_allreduce_init) */
static int mirror_alloc(emac_handle *h, void **p) { return emac_gpu_malloc(p, h->bytes); }

static void mirror_free(emac_handle *h, void *p) { emac_gpu_free(p); }

/* A buffer the handle can use in place: device memory, and in the IPC form, for a buffer the
   peers read (the send buffer; in place, the one buffer), also exportable
   (emac_gpu_ipc_exportable). The receive buffer of the IPC form is never exported: peers never
   touch it. Anything else gets a device mirror. */
static int in_place_ok(const emac_handle *h, const void *p, int peers_read) {
  if (!emac_gpu_is_device_pointer(p)) return 0;
  return h->kind != KIND_IPC || !peers_read || g_comms[h->comm].size == 1 || emac_gpu_ipc_exportable(p);
}

/* Page-locking a caller's host buffer is opt-in (EXT_MPI_AMD_HOST_REGISTER=1; never in the IPC
   form). Registered user pages, unregistered at handle release and then freed and reused by the
   application, were twice followed by an asynchronous illegal-address error in a later, unrelated
   launch or copy of the same process (8 IPC processes on one MI355X; the single-process GPU suite
   after the host-buffer tests), and both went away without registration. Unregistered buffers
   are staged by the runtime; buffers the caller already pinned (hipHostMalloc, torch
   pin_memory) are copied at full rate either way. */
static int host_register(const emac_handle *h, const void *p) {
  const char *e = getenv("EXT_MPI_AMD_HOST_REGISTER");
  if (!e || atoi(e) <= 0 || h->kind == KIND_IPC || emac_gpu_is_device_pointer(p)) return 0;
  return emac_gpu_host_register((void *)p, h->bytes) == 0;
}

/* NODE form: host memory the caller already page-locked (hipHostMalloc, torch pin_memory) is
   read and written by the fold kernel itself over PCIe (EXT_MPI_AMD_HOST_DIRECT=0 turns this
   off). One launch replaces R host-to-device copies, the fold and R device-to-host copies, and
   the leaf reads overlap the fan-out writes on the link's two directions. */
static int host_direct(const emac_handle *h, const void *p, void **dev) {
  const char *e = getenv("EXT_MPI_AMD_HOST_DIRECT");
  if (h->kind != KIND_NODE || (e && atoi(e) <= 0)) return 0;
  return emac_gpu_pinned_view(p, dev) == 0;
}

/* Device view of rank r's buffers: usable user device pointers are used in place, page-locked
   host memory in the NODE form through its device address; other buffers get a device mirror
   (in place stays in place), staged in and out on the handle's stream. */
int map_buffers(emac_handle *h, int r, const void *send, void *recv) {
  int rc;
  void *dv;
  h->user_send[r] = (void *)send;
  h->user_recv[r] = recv;
  if (in_place_ok(h, recv, send == recv)) {
    h->drecv[r] = recv;
  } else if (host_direct(h, recv, &dv)) {
    h->drecv[r] = dv;
    h->host_direct = 1;
  } else {
    /* IPC form, in place: the one buffer is read by the peers -- its mirror comes from the arena
       (ipc_allreduce_init; NULL until then) */
    if (!(h->kind == KIND_IPC && send == recv) && (rc = mirror_alloc(h, &h->drecv[r]))) return rc;
    h->recv_mirror[r] = 1;
    h->recv_reg[r] = host_register(h, recv);
  }
  if (send == recv) {
    h->dsend[r] = h->drecv[r];
  } else if (in_place_ok(h, send, 1)) {
    h->dsend[r] = (void *)send;
  } else if (host_direct(h, send, &dv)) {
    h->dsend[r] = dv;
    h->host_direct = 1;
  } else {
    /* IPC form: from the arena (ipc_allreduce_init; NULL until then) */
    if (h->kind != KIND_IPC && (rc = mirror_alloc(h, &h->dsend[r]))) return rc;
    h->send_mirror[r] = 1;
    h->send_reg[r] = host_register(h, send);
  }
  return 0;
}

/* pointers of a bucket are first set at the start of the whole buffers, then moved to the
   chunk's first element */
void place_bucket(emac_bucket *b, int nsrc, long off, long len, int tsize) {
  int i;
  for (i = 0; i < nsrc; i++) b->src[i] = (const char *)b->src[i] + off * tsize;
  for (i = 0; i < b->ndst; i++) b->dst[i] = (char *)b->dst[i] + off * tsize;
  emac_split_alignment(b, nsrc, len, tsize);
}

int upload_launch_as(const emac_handle *h, emac_launch *L, emac_bucket *b, int nb, int nsrc, int tree) {
  emac_edge *edges = NULL;
  int rc;
  if ((rc = emac_layout(b, nb, h->plan.op, nsrc, tree, h->fan, &edges, &L->nedges, &L->ntiles, &L->tiles_per_bucket,
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

int upload_launch(const emac_handle *h, emac_launch *L, emac_bucket *b, int nb) {
  return upload_launch_as(h, L, b, nb, h->nsrc, emac_tree_kind(&h->plan.codes, h->plan.op) == 1);
}

/* a launch of `nsrc`-leaf buckets under the schedule of fan-out form `fan` (2: peer-mapped) */
int upload_launch_fan(const emac_handle *h, emac_launch *L, emac_bucket *b, int nb, int nsrc, int fan) {
  emac_edge *edges = NULL;
  int rc;
  if ((rc = emac_layout(b, nb, nsrc > 1 ? h->plan.op : EMAC_SUM, nsrc, 0, fan, &edges, &L->nedges, &L->ntiles,
                        &L->tiles_per_bucket, &L->all_full, &L->unroll)))
    return rc;
  L->nb = nb;
  if (nb && (rc = emac_gpu_malloc((void **)&L->d_buckets, sizeof(emac_bucket) * (size_t)nb)) == 0)
    rc = emac_gpu_memcpy(L->d_buckets, b, sizeof(emac_bucket) * (size_t)nb);
  if (!rc && L->nedges && (rc = emac_gpu_malloc((void **)&L->d_edges, sizeof(emac_edge) * (size_t)L->nedges)) == 0)
    rc = emac_gpu_memcpy(L->d_edges, edges, sizeof(emac_edge) * (size_t)L->nedges);
  free(edges);
  return rc;
}
/* EXT_MPI_NUM_SOCKETS_PER_NODE as the reference keeps it: one process-wide parameter read at
   init (ext_mpi.c:43-187), applied to every plan built afterwards */
static int g_num_sockets = 1;

int ext_mpi_amd_set_num_sockets(int sockets) {
  const int prev = g_num_sockets;
  if (sockets < 1 || sockets > EMAC_MAX_RANKS) return EMAC_ERR_ARG;
  g_num_sockets = sockets;
  return prev;
}

int parse_cfg(const char *copyin, int nranks, emac_copyin *cfg) {
  int rc = 0;
  /* one rank: the generator returns before reading the factors (reduce_copyin.c:975) */
  if (!copyin || !*copyin || nranks == 1)
    emac_default_copyin(nranks, cfg);
  else
    rc = emac_parse_copyin(copyin, cfg);
  cfg->sockets = g_num_sockets;
  return rc;
}

int finish_init(emac_handle *h, int *handle) {
  int slot = new_handle_slot();
  h->own_stream = 1;
  if (slot < 0) return EMAC_ERR_MALLOC;
  g_handles[slot] = h;
  *handle = slot;
  return 0;
}

int stage_in(emac_handle *h) {
  int r, rc;
  for (r = 0; r < h->nbuf; r++) {
    void *src = h->send_mirror[r] ? h->user_send[r] : (h->recv_mirror[r] && h->dsend[r] == h->drecv[r] ? h->user_recv[r] : NULL);
    if (src && (rc = OP(h, emac_gpu_memcpy_async(h->dsend[r], src, h->bytes, h->stream)))) return rc;
  }
  return 0;
}

int stage_out(emac_handle *h) {
  int r, rc;
  for (r = 0; r < h->nbuf; r++)
    if (h->recv_mirror[r] && (rc = OP(h, emac_gpu_memcpy_async(h->user_recv[r], h->drecv[r], h->bytes, h->stream))))
      return rc;
  return 0;
}

emac_handle *handle_get(int handle) {
  if (handle < 0 || handle >= MAX_HANDLES) return NULL;
  return g_handles[handle];
}

/* Everything a Start (or a subset of its legs) enqueues on the handle's stream. */
static int enqueue_legs(emac_handle *h, int legs) {
  int rc, multi;
  const int core = EXT_MPI_AMD_LEG_REDUCE_SCATTER | EXT_MPI_AMD_LEG_FOLD | EXT_MPI_AMD_LEG_ALLGATHER;
  multi = h->kind == KIND_COMM && h->plan.nranks > 1 && !h->hier; /* the node's own p2p legs */
  if ((legs & EXT_MPI_AMD_LEG_STAGE_IN) && (rc = stage_in(h))) return rc;
  if (h->kind == KIND_IPC && h->hier) { /* the NODE form over peer-mapped nodes (node_ipc_init) */
    const int nodes = g_comms[h->comm].size;
    if (h->join) { /* pipelined by parts: the copy-in, and the node legs fused with the copy-out */
      const int nl = EXT_MPI_AMD_LEG_NODES_RS | EXT_MPI_AMD_LEG_NODES_FOLD | EXT_MPI_AMD_LEG_NODES_AG;
      if ((legs & nl) != nl && (legs & nl) != 0) return EMAC_ERR_UNSUPPORTED; /* the legs of a part go together */
      if ((legs & (EXT_MPI_AMD_LEG_FOLD | nl)) && (rc = join_start(h, (legs & EXT_MPI_AMD_LEG_FOLD) != 0, (legs & nl) != 0)))
        return rc;
      if ((legs & EXT_MPI_AMD_LEG_STAGE_OUT) && (rc = stage_out(h))) return rc;
      return 0;
    }
    if ((legs & EXT_MPI_AMD_LEG_FOLD) && (rc = fold_launch(h))) return rc; /* the copy-in */
    if (legs & (EXT_MPI_AMD_LEG_NODES_RS | EXT_MPI_AMD_LEG_NODES_FOLD | EXT_MPI_AMD_LEG_NODES_AG)) {
      const emac_launch *X = &h->xfold[0];
      if ((rc = ipc_barrier(h, 0))) return rc;
      if ((X->nb || X->nedges) &&
          (rc = OP(h, emac_gpu_fold_remote(h->plan.dtype, nodes > 1 ? h->plan.op : EMAC_SUM, nodes, X->unroll, &h->xcodes,
                                     X->d_buckets, X->nb, X->ntiles, X->tiles_per_bucket, X->all_full, X->d_edges,
                                     X->nedges, ipc_go(h), h->stream))))
        return rc;
      if ((rc = ipc_barrier(h, 1))) return rc;
      if ((h->pull.nb || h->pull.nedges) &&
          (rc = OP(h, emac_gpu_copy_fan_remote(h->plan.tsize, h->plan.nranks, h->pull.unroll, h->pull.d_buckets, h->pull.nb,
                                         h->pull.ntiles, h->pull.tiles_per_bucket, h->pull.all_full, h->pull.d_edges,
                                         h->pull.nedges, ipc_go(h), h->stream))))
        return rc;
    }
    if ((legs & EXT_MPI_AMD_LEG_ALLGATHER) && h->fanout.nb &&
        (rc = OP(h, emac_gpu_copy_fan(h->plan.tsize, h->plan.nranks - 1, h->fanout.unroll, h->fanout.d_buckets, h->fanout.nb,
                                h->fanout.ntiles, h->fanout.tiles_per_bucket, h->fanout.all_full, h->fanout.d_edges,
                                h->fanout.nedges, h->stream))))
      return rc;
    if ((legs & EXT_MPI_AMD_LEG_STAGE_OUT) && (rc = stage_out(h))) return rc;
    return 0;
  }
  if (h->kind == KIND_IPC && h->fused && (legs & core) == core) {
    emac_comm *cm = &g_comms[h->comm];
    unsigned long e0, e1;
    if (h->ev_release && (rc = emac_gpu_event_record(h->ev_release, h->stream))) return rc; /* as ipc_barrier(h, 0) */
    e0 = ++h->epoch[0];
    e1 = ++h->epoch[1];
    if ((rc = OP(h, emac_gpu_fold_fused(h->plan.dtype, h->plan.op, h->nsrc, h->unroll, &h->plan.codes, h->d_buckets, h->nb, h->ntiles,
                                  h->tiles_per_bucket, h->all_full, h->d_edges, h->nedges, h->pull.d_buckets, h->pull.nb,
                                  h->pull.ntiles, h->pull.tiles_per_bucket, h->pull.all_full, h->pull.d_edges,
                                  h->pull.nedges, cm->sync,
                                  (void *const *)cm->d_peer_sync, h->slot, cm->size, cm->rank, cm->err + h->slot,
                                  cm->timeout_ticks, e0, e1, h->stream))))
      return rc;
    if ((legs & EXT_MPI_AMD_LEG_STAGE_OUT) && (rc = stage_out(h))) return rc;
    return 0;
  }
  if ((legs & EXT_MPI_AMD_LEG_REDUCE_SCATTER) && h->kind == KIND_IPC && h->plan.nranks > 1 &&
      (rc = ipc_barrier(h, 0)))
    return rc;
  if ((legs & EXT_MPI_AMD_LEG_REDUCE_SCATTER) && multi && (rc = run_leg(h, EMAC_LEG_RS))) return rc;
  if ((legs & EXT_MPI_AMD_LEG_FOLD) && h->fan == 2 &&
      (rc = OP(h, emac_gpu_fold_remote(h->plan.dtype, h->plan.op, h->nsrc, h->unroll, &h->plan.codes, h->d_buckets, h->nb,
                                 h->ntiles, h->tiles_per_bucket, h->all_full, h->d_edges, h->nedges, ipc_go(h), h->stream))))
    return rc;
  if ((legs & EXT_MPI_AMD_LEG_FOLD) && h->fan != 2 && (rc = fold_launch(h))) return rc;
  if (h->kind == KIND_COMM && h->nodes > 1) {
    /* several nodes: per step the exchange of the lines with the column peers and the fold of
       the kept lines' partials (a left fold of radix leaves in the order the program lists
       them), then the exchanges back in reverse step order (emac_comm_program_nodes). A step
       selector in the legs' high bits (EXT_MPI_AMD_LEG_STEP) runs that step's legs alone. */
    int st;
    const int nsteps = h->ns.nsteps + h->ns.nred, only = (legs >> EMAC_LEG_STEP_SHIFT) & 31;
    for (st = 0; st < nsteps; st++) {
      const emac_launch *X = &h->xfold[st];
      const int rad = node_radix(&h->ns, st);
      emac_codes lin;
      memset(&lin, 0, sizeof(lin));
      lin.first[0] = 1; /* one level: a left fold */
      lin.close[rad - 1] = 1;
      lin.nlev = 1;
      lin.nleaf = rad;
      if (only && st != only - 1) continue;
      if ((legs & EXT_MPI_AMD_LEG_NODES_RS) && (rc = run_leg(h, EMAC_LEG_NODES_RS | st << EMAC_LEG_STEP_SHIFT)))
        return rc;
      if ((legs & EXT_MPI_AMD_LEG_NODES_FOLD) && X->nb &&
          (rc = OP(h, emac_gpu_fold(h->plan.dtype, h->plan.op, rad, 0, X->unroll, &lin, X->d_buckets, X->nb,
                              X->ntiles, X->tiles_per_bucket, X->all_full, X->d_edges, X->nedges, h->stream))))
        return rc;
    }
    for (st = 0; st < h->ns.nagp; st++) { /* the copying allgather steps, block growing */
      if (only && st != only - 1) continue;
      if ((legs & EXT_MPI_AMD_LEG_NODES_AG) && (rc = run_leg(h, EMAC_LEG_NODES_AG | st << EMAC_LEG_STEP_SHIFT)))
        return rc;
    }
  }
  if ((legs & EXT_MPI_AMD_LEG_ALLGATHER) && multi && (rc = run_leg(h, EMAC_LEG_AG))) return rc;
  if ((legs & EXT_MPI_AMD_LEG_ALLGATHER) && h->hier && h->fanout.nb &&
      (rc = OP(h, emac_gpu_copy_fan(h->plan.tsize, h->plan.nranks - 1, h->fanout.unroll, h->fanout.d_buckets, h->fanout.nb,
                              h->fanout.ntiles, h->fanout.tiles_per_bucket, h->fanout.all_full, h->fanout.d_edges,
                              h->fanout.nedges, h->stream))))
    return rc;
  if ((legs & EXT_MPI_AMD_LEG_ALLGATHER) && h->kind == KIND_IPC && h->plan.nranks > 1) {
    static const emac_codes copy = {{1}, {1}, 1, 1}; /* one leaf: a copy */
    if ((rc = ipc_barrier(h, 1))) return rc;
    if ((rc = OP(h, emac_gpu_fold_remote(h->plan.dtype, EMAC_SUM, 1, h->pull.unroll, &copy, h->pull.d_buckets, h->pull.nb,
                                   h->pull.ntiles, h->pull.tiles_per_bucket, h->pull.all_full, h->pull.d_edges,
                                   h->pull.nedges, ipc_go(h), h->stream))))
      return rc;
  }
  if ((legs & EXT_MPI_AMD_LEG_STAGE_OUT) && (rc = stage_out(h))) return rc;
  return 0;
}

/* COMM form with device buffers, EXT_MPI_AMD_GRAPH=1: the legs of a Start captured once into a
   HIP graph (RCCL's grouped send/recv, the fold and its edge launch) and replayed by one
   hipGraphLaunch, per subset of legs; a capture that fails falls back to eager launches for good
   (graph_failed). Host buffers (pageable staging copies) are never captured. Opt-in: on a 1-rank
   communicator (the fold alone) a Start + Wait took 17.9 us replayed against 12.0 us eager
   (profiles/r02_graph_latency.json, the runtime's replay floor); with the two RCCL legs of N > 1
   ranks the balance is unmeasured here. */
static int graph_ok(const emac_handle *h) {
  const char *e = getenv("EXT_MPI_AMD_GRAPH");
  int r;
  if (h->kind != KIND_COMM || !e || atoi(e) <= 0) return 0;
  for (r = 0; r < h->nbuf; r++)
    if (h->send_mirror[r] || h->recv_mirror[r]) return 0;
  return 1;
}

int ext_mpi_amd_start_legs(int handle, int legs) {
  emac_handle *h = handle_get(handle);
  int rc, key;
  if (!h) return EMAC_ERR_ARG;
  if (emac_gpu_set_device(h->device)) return EMAC_ERR_DEVICE;
  key = legs & EXT_MPI_AMD_LEG_ALL;
  if (legs >> EMAC_LEG_STEP_SHIFT) { /* one node step alone (loopback lock-step): never captured */
    if ((rc = enqueue_legs(h, legs))) return rc;
    h->started = 1;
    return 0;
  }
  if (graph_ok(h) && !h->graph[key] && !h->graph_failed[key]) {
    if (emac_gpu_capture_begin(h->stream) == 0) {
      const int erc = enqueue_legs(h, legs);
      const int crc = emac_gpu_capture_end(h->stream, &h->graph[key]);
      if (erc || crc) {
        h->graph[key] = NULL;
        h->graph_failed[key] = 1;
      }
    } else {
      h->graph_failed[key] = 1;
    }
  }
  if (h->graph[key]) {
    if ((rc = emac_gpu_graph_launch(h->graph[key], h->stream))) return rc;
  } else if ((rc = enqueue_legs(h, legs))) {
    return rc;
  }
  h->started = 1;
  return 0;
}

int ext_mpi_amd_start(int handle) { return ext_mpi_amd_start_legs(handle, EXT_MPI_AMD_LEG_ALL); }

int ext_mpi_amd_set_stream(int handle, void *stream) {
  emac_handle *h = handle_get(handle);
  if (!h || !stream) return EMAC_ERR_ARG;
  emac_gpu_stream_sync(h->stream);
  if (h->own_stream) emac_gpu_stream_destroy(h->stream);
  h->stream = stream;
  h->own_stream = 0;
  return 0;
}

int ext_mpi_amd_test(int handle) {
  emac_handle *h = handle_get(handle);
  int rc;
  if (!h) return EMAC_ERR_ARG;
  if (!h->started) return 1;
  rc = emac_gpu_stream_query(h->stream);
  if (rc == 1) {
    h->started = 0;
    if (ipc_status(h)) return EMAC_ERR_TRANSPORT;
  }
  return rc;
}

int ext_mpi_amd_wait(int handle) {
  emac_handle *h = handle_get(handle);
  int rc;
  if (!h) return EMAC_ERR_ARG;
  rc = emac_gpu_stream_sync(h->stream);
  h->started = 0;
  return rc ? rc : ipc_status(h);
}

/* Done of a peer-mapped handle over caller memory is collective over the communicator, as the
   reference's (EXT_MPI_Done_native -> ext_mpi_gpu_destroy_shared_memory's node barrier,
   cuda_shmem.c:190-216, then cudaIpcCloseMemHandle, :301-314): every rank closes its mappings of
   the peers' buffers, then the ranks agree, so when Done returns no peer maps this rank's buffers
   any more and the caller may free them (ipc_exchange). A handle whose exported buffers are all
   library memory (mirrors, the MPI layer's scratch) is released locally: that memory returns to
   the communicator's pool and is only freed by the collective communicator free. */
int ext_mpi_amd_done(int handle) {
  emac_handle *h = handle_get(handle);
  int comm, collective;
  if (!h) return EMAC_ERR_ARG;
  g_handles[handle] = NULL;
  comm = h->comm;
  collective = h->kind == KIND_IPC && h->done_collective && g_comms[comm].used && g_comms[comm].size > 1;
  handle_release(h);
  return collective ? ipc_agree(&g_comms[comm], 1) : 0;
}

void *ext_mpi_amd_stream(int handle) {
  emac_handle *h = handle_get(handle);
  return h ? h->stream : NULL;
}

int ext_mpi_amd_plan_describe(int nranks, long count, int dtype, const char *copyin, int pos, long *piece_off,
                              long *piece_len, int max_pieces, int *owner_rank, int *leaf_ranks,
                              unsigned char *first, unsigned char *close, int *nlev) {
  emac_plan p;
  emac_copyin cfg;
  int rc, pc, t, n;
  if (nranks < 1 || nranks > EMAC_MAX_RANKS || pos < 0 || pos >= nranks) return EMAC_ERR_ARG;
  if ((rc = parse_cfg(copyin, nranks, &cfg))) return rc;
  if ((rc = emac_plan_build(&p, nranks, count, dtype, EMAC_SUM, &cfg))) return rc;
  n = p.npieces < max_pieces ? p.npieces : max_pieces;
  for (pc = 0; pc < n; pc++) {
    piece_off[pc] = p.chunk_off[(size_t)pc * nranks + pos];
    piece_len[pc] = p.chunk_len[(size_t)pc * nranks + pos];
  }
  *owner_rank = p.pos_rank[pos];
  for (t = 0; t < p.codes.nleaf; t++) {
    leaf_ranks[t] = p.leaf_rank[pos][t];
    first[t] = p.codes.first[t];
    close[t] = p.codes.close[t];
  }
  *nlev = p.codes.nlev;
  rc = p.npieces;
  emac_plan_free(&p);
  return rc;
}

const char *ext_mpi_amd_version(void) { return "ext_mpi_collectives_amd 0.1 (gfx950)"; }

/* "sha <HEAD>[+dirty] src <hash>": the commit and the product sources this binary was built from
   (build/stamp.c, written by _stamp.py on every make) */
extern const char emac_build_stamp[];
const char *ext_mpi_amd_build_info(void) { return emac_build_stamp; }
