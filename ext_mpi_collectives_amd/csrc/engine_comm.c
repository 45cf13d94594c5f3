/*
 * engine_comm.c -- the COMM form: one rank per GPU, the reduce-scatter and allgather legs as
 * grouped RCCL point-to-point rounds over xGMI (or the in-process loopback transport for tests),
 * the owner's fold in the reference's order; the program builders exported for host transports
 * (engine_int.h).
 */
#include "engine_int.h"

loop_group g_loops[MAX_LOOP_GROUPS];

/* ------------------------------ COMM form (RCCL) ------------------------------ */

int ext_mpi_amd_get_unique_id(void *id) {
  ncclUniqueId u;
  if (!id) return EMAC_ERR_ARG;
  if (ncclGetUniqueId(&u) != ncclSuccess) return EMAC_ERR_TRANSPORT;
  memcpy(id, &u, sizeof(u));
  return 0;
}

int ext_mpi_amd_comm_init(int rank, int size, const void *id, int device, int *comm) {
  ncclUniqueId u;
  int i;
  if (!id || !comm || size < 1 || size > EMAC_MAX_RANKS || rank < 0 || rank >= size) return EMAC_ERR_ARG;
  if (emac_gpu_device_count() <= 0) return EMAC_ERR_DEVICE;
  for (i = 0; i < MAX_COMMS && g_comms[i].used; i++);
  if (i == MAX_COMMS) return EMAC_ERR_MALLOC;
  if (device >= 0 && emac_gpu_set_device(device)) return EMAC_ERR_DEVICE;
  emac_gpu_get_device(&g_comms[i].device);
  memcpy(&u, id, sizeof(u));
  if (ncclCommInitRank(&g_comms[i].nccl, size, u, rank) != ncclSuccess) return EMAC_ERR_TRANSPORT;
  g_comms[i].used = 1;
  g_comms[i].rank = rank;
  g_comms[i].size = size;
  g_comms[i].loop_group = -1;
  *comm = i;
  return 0;
}

/* Testing transport: `size` communicators, one per rank, all in this process on the current
   device. Their point-to-point ops are matched in order (as RCCL matches ops between a pair
   inside a group) and executed as device copies when the RECEIVING rank runs the leg, so the
   caller must run each leg on every rank before the next one (ext_mpi_amd_start_legs). */
int ext_mpi_amd_comm_init_loopback(int size, int *comm_of_rank) {
  int g, r, i;
  if (!comm_of_rank || size < 1 || size > EMAC_MAX_RANKS) return EMAC_ERR_ARG;
  if (emac_gpu_device_count() <= 0) return EMAC_ERR_DEVICE;
  for (g = 0; g < MAX_LOOP_GROUPS && g_loops[g].used; g++);
  if (g == MAX_LOOP_GROUPS) return EMAC_ERR_MALLOC;
  memset(&g_loops[g], 0, sizeof(g_loops[g]));
  g_loops[g].used = 1;
  g_loops[g].size = size;
  for (r = 0; r < size; r++) {
    for (i = 0; i < MAX_COMMS && g_comms[i].used; i++);
    if (i == MAX_COMMS) return EMAC_ERR_MALLOC;
    memset(&g_comms[i], 0, sizeof(g_comms[i]));
    g_comms[i].used = 1;
    g_comms[i].rank = r;
    g_comms[i].size = size;
    g_comms[i].loop_group = g;
    emac_gpu_get_device(&g_comms[i].device);
    comm_of_rank[r] = i;
  }
  return 0;
}

int ext_mpi_amd_comm_free(int comm) {
  if (comm < 0 || comm >= MAX_COMMS || !g_comms[comm].used) return EMAC_ERR_ARG;
  if (g_comms[comm].ipc) {
    ipc_comm_release(&g_comms[comm]);
    return 0;
  }
  if (g_comms[comm].loop_group >= 0) {
    loop_group *g = &g_loops[g_comms[comm].loop_group];
    g->nh[g_comms[comm].rank] = -1; /* this rank left */
    for (int r = 0; r < g->size; r++)
      if (g->nh[r] >= 0) goto keep;
    g->used = 0;
  keep:;
  } else {
    ncclCommDestroy(g_comms[comm].nccl);
  }
  g_comms[comm].used = 0;
  return 0;
}

int ext_mpi_amd_allreduce_init(const void *sendbuf, void *recvbuf, long count, int dtype, int op, int comm,
                               const char *copyin, int *handle) {
  emac_handle *h;
  emac_comm *cm;
  emac_copyin cfg;
  emac_bucket *b = NULL;
  int rc, t, R, nb = 0;
  long stage_total = 0;
  if (!handle || comm < 0 || comm >= MAX_COMMS || !g_comms[comm].used || count < 0) return EMAC_ERR_ARG;
  *handle = -1;
  cm = &g_comms[comm];
  R = cm->size / (cm->nodes > 1 && !cm->ipc ? cm->nodes : 1); /* ranks of one node */
  if ((rc = parse_cfg(copyin, R, &cfg))) return rc;
  if (emac_gpu_set_device(cm->device)) return EMAC_ERR_DEVICE;
  h = (emac_handle *)calloc(1, sizeof(emac_handle));
  if (!h) return EMAC_ERR_MALLOC;
  h->kind = cm->ipc ? KIND_IPC : KIND_COMM;
  h->comm = comm;
  h->device = cm->device;
  rc = emac_plan_build(&h->plan, R, count, dtype, op, &cfg);
  if (!rc) {
    h->me = cm->rank;
    h->me_pos = h->plan.rank_pos[h->me % R];
    h->bytes = (size_t)count * (size_t)h->plan.tsize;
    h->nodes = cm->size / R;
    h->ns = cm->ns;
    if (h->nodes > 1 && h->ns.nodes != h->nodes) rc = EMAC_ERR_ARG;
  }
  h->nbuf = 1;
  h->nsrc = R;
  if (cm->ipc) {
    if (!rc) rc = emac_gpu_stream_create(&h->stream);
    return ipc_init_settle(h, cm, ipc_allreduce_init(h, cm, sendbuf, recvbuf, rc), handle);
  }
  if (rc) goto fail;
  if ((rc = map_buffers(h, 0, sendbuf, recvbuf))) goto fail;
  {
    emac_fold *folds = NULL;
    int nf = 0, f;
    emac_bucket *xb = NULL;
    int nxb[2 * EMAC_MAX_NODE_STEPS] = {0}, st;
    const int nsteps = h->nodes > 1 ? h->ns.nsteps + h->ns.nred : 0; /* exchange steps with a fold */
    if ((rc = emac_comm_program_nodes(&h->plan, h->nodes > 1 ? &h->ns : NULL, h->me / R, h->me % R,
                                      (long)((unsigned long)h->dsend[0] & 15ul), &h->ops, &h->nops, &folds, &nf,
                                      &stage_total)))
      goto fail;
    b = (emac_bucket *)calloc((size_t)nf + 1, sizeof(emac_bucket));
    xb = (emac_bucket *)calloc(2 * EMAC_MAX_NODE_STEPS * ((size_t)nf + 1), sizeof(emac_bucket));
    if (!b || !xb || (rc = emac_gpu_malloc(&h->staging, (size_t)(stage_total > 0 ? stage_total : 16)))) {
      free(folds);
      free(xb);
      rc = rc ? rc : EMAC_ERR_MALLOC;
      goto fail;
    }
    for (f = 0; f < nf; f++) {
      const int node_pair = (folds[f].leg & ((1 << EMAC_LEG_STEP_SHIFT) - 1)) == EMAC_LEG_NODES_FOLD;
      const int step = folds[f].leg >> EMAC_LEG_STEP_SHIFT;
      emac_bucket *bk = node_pair ? &xb[(size_t)step * ((size_t)nf + 1) + (size_t)nxb[step]++] : &b[nb++];
      long off = folds[f].offset / h->plan.tsize;
      for (t = 0; t < folds[f].nleaf; t++) {
        /* leaf pointers are shifted back by the result's offset: split_alignment adds it */
        bk->src[t] = leg_base(h, folds[f].buf[t]) + folds[f].loff[t] - folds[f].offset;
      }
      bk->dst[0] = h->drecv[0];
      bk->ndst = 1;
      place_bucket(bk, folds[f].nleaf, off, folds[f].count, h->plan.tsize);
    }
    free(folds);
    for (st = 0; st < nsteps; st++)
      if (nxb[st] &&
          (rc = upload_launch_as(h, &h->xfold[st], xb + (size_t)st * ((size_t)nf + 1), nxb[st], node_radix(&h->ns, st),
                                 0))) {
        free(xb);
        goto fail;
      }
    free(xb);
  }
  if ((rc = upload_buckets(h, b, nb))) goto fail;
  free(b);
  b = NULL;
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
  return 0;
fail:
  free(b);
  handle_release(h);
  return rc;
}

/* radix of exchange step st: the reduce-scatter steps, then the allgather steps that reduce */
int node_radix(const emac_node_sched *ns, int st) {
  return st < ns->nsteps ? ns->radix[st] : ns->red_radix[st - ns->nsteps];
}

/* base of buffer `buf` of node rank `l` in this process (0 but in the NODE form over several nodes) */
char *leg_base_of(const emac_handle *h, int buf, int l) {
  return buf == EMAC_BUF_SEND ? (char *)h->dsend[l]
       : buf == EMAC_BUF_RECV ? (char *)h->drecv[l]
                              : (char *)h->staging + (long)l * h->stage_stride;
}

char *leg_base(const emac_handle *h, int buf) { return leg_base_of(h, buf, 0); }

/* Loopback transport: every receive of this leg copies the matching send of the peer (the
   k-th send of q to me in this leg matches my k-th receive from q). */
static int run_leg_loopback(emac_handle *h, int leg) {
  loop_group *g = &g_loops[g_comms[h->comm].loop_group];
  int seen[EMAC_MAX_RANKS][EMAC_MAX_RANKS], i, j, rc;
  memset(seen, 0, sizeof(seen));
  for (i = 0; i < h->nops; i++) {
    const emac_p2p *o = &h->ops[i];
    emac_handle *hq;
    int q = o->peer, k, found = 0;
    if (o->leg != leg || o->is_send) continue;
    k = seen[q][o->local]++; /* per (peer, node rank): the NODE form over nodes orders them so */
    if (h->loop_index >= g->nh[q]) return EMAC_ERR_TRANSPORT; /* peer has no matching handle */
    hq = handle_get(g->handle[q][h->loop_index]);
    if (!hq) return EMAC_ERR_TRANSPORT;
    for (j = 0; j < hq->nops; j++) {
      const emac_p2p *so = &hq->ops[j];
      if (so->leg == leg && so->is_send && so->peer == h->me && so->local == o->local && k-- == 0) {
        if (so->bytes != o->bytes) return EMAC_ERR_TRANSPORT;
        if ((rc = emac_gpu_memcpy_async(leg_base_of(h, o->buf, o->local) + o->offset,
                                        leg_base_of(hq, so->buf, so->local) + so->offset, (size_t)o->bytes, h->stream)))
          return rc;
        found = 1;
        break;
      }
    }
    if (!found) return EMAC_ERR_TRANSPORT;
  }
  return 0;
}

/* Walk the point-to-point program of one leg as ONE RCCL group (all peers at once). */
int run_leg(emac_handle *h, int leg) {
  emac_comm *cm = &g_comms[h->comm];
  hipStream_t s = (hipStream_t)h->stream;
  int i, bad = 0;
  h->tune.ops++;
  if (cm->loop_group >= 0) return run_leg_loopback(h, leg);
  if (ncclGroupStart() != ncclSuccess) return EMAC_ERR_TRANSPORT;
  for (i = 0; i < h->nops && !bad; i++) {
    const emac_p2p *o = &h->ops[i];
    char *base;
    if (o->leg != leg) continue;
    base = leg_base_of(h, o->buf, o->local);
    if (o->is_send)
      bad = ncclSend(base + o->offset, (size_t)o->bytes, ncclInt8, o->peer, cm->nccl, s) != ncclSuccess;
    else
      bad = ncclRecv(base + o->offset, (size_t)o->bytes, ncclInt8, o->peer, cm->nccl, s) != ncclSuccess;
  }
  if (ncclGroupEnd() != ncclSuccess) bad = 1;
  return bad ? EMAC_ERR_TRANSPORT : 0;
}

int ext_mpi_amd_comm_program(int nranks, int rank, long count, int dtype, const char *copyin, long send_phase,
                             ext_mpi_amd_p2p *ops, int max_ops, int *nops, ext_mpi_amd_fold *folds, int max_folds,
                             int *nfolds, long *staging_bytes) {
  return ext_mpi_amd_comm_program_nodes(1, nranks, rank, count, dtype, copyin, send_phase, ops, max_ops, nops, folds,
                                        max_folds, nfolds, staging_bytes);
}

int ext_mpi_amd_comm_set_node_ports(int comm, int nodes, const int *ports) {
  emac_node_sched ns;
  int rc;
  if (comm < 0 || comm >= MAX_COMMS || !g_comms[comm].used) return EMAC_ERR_ARG;
  if (nodes < 1 || g_comms[comm].size % nodes) return EMAC_ERR_ARG;
  /* a peer-mapped communicator's members are nodes only as a whole (node_comm_allreduce_init) */
  if (nodes > EMAC_MAX_NODES || (nodes > 1 && g_comms[comm].ipc && nodes != g_comms[comm].size)) return EMAC_ERR_UNSUPPORTED;
  if ((rc = emac_node_sched_build(&ns, nodes, ports))) return rc;
  g_comms[comm].nodes = nodes;
  g_comms[comm].ns = ns;
  return 0;
}

int ext_mpi_amd_comm_set_nodes(int comm, int nodes) {
  if (nodes > 1 && (nodes & (nodes - 1))) return EMAC_ERR_ARG; /* one port per step: a power of two */
  return ext_mpi_amd_comm_set_node_ports(comm, nodes, NULL);
}

int ext_mpi_amd_comm_program_nodes(int nodes, int ranks_per_node, int rank, long count, int dtype, const char *copyin,
                                   long send_phase, ext_mpi_amd_p2p *ops, int max_ops, int *nops,
                                   ext_mpi_amd_fold *folds, int max_folds, int *nfolds, long *staging_bytes) {
  if (nodes > 1 && (nodes & (nodes - 1))) return EMAC_ERR_ARG; /* one port per step: a power of two */
  return ext_mpi_amd_comm_program_node_ports(nodes, NULL, ranks_per_node, rank, count, dtype, copyin, send_phase, ops,
                                             max_ops, nops, folds, max_folds, nfolds, staging_bytes);
}

int ext_mpi_amd_comm_program_node_ports(int nodes, const int *ports, int ranks_per_node, int rank, long count,
                                        int dtype, const char *copyin, long send_phase, ext_mpi_amd_p2p *ops,
                                        int max_ops, int *nops, ext_mpi_amd_fold *folds, int max_folds, int *nfolds,
                                        long *staging_bytes) {
  emac_node_sched ns;
  emac_plan p;
  emac_copyin cfg;
  emac_p2p *o = NULL;
  emac_fold *f = NULL;
  const int R = ranks_per_node;
  int rc, i, t, no = 0, nf = 0;
  if (R < 1 || R > EMAC_MAX_RANKS || nodes < 1 || nodes > EMAC_MAX_NODES || rank < 0 || rank >= nodes * R)
    return EMAC_ERR_ARG;
  if ((rc = emac_node_sched_build(&ns, nodes, ports))) return rc;
  if ((rc = parse_cfg(copyin, R, &cfg))) return rc;
  if ((rc = emac_plan_build(&p, R, count, dtype, EMAC_SUM, &cfg))) return rc;
  if ((rc = emac_comm_program_nodes(&p, nodes > 1 ? &ns : NULL, rank / R, rank % R, send_phase, &o, &no, &f, &nf,
                                    staging_bytes)))
    goto out;
  if (no > max_ops || nf > max_folds) {
    rc = EMAC_ERR_ARG;
    goto out;
  }
  for (i = 0; i < no; i++) {
    ops[i].leg = o[i].leg;
    ops[i].peer = o[i].peer;
    ops[i].is_send = o[i].is_send;
    ops[i].buf = o[i].buf;
    ops[i].offset = o[i].offset;
    ops[i].bytes = o[i].bytes;
  }
  for (i = 0; i < nf; i++) {
    memset(&folds[i], 0, sizeof(folds[i]));
    folds[i].piece = f[i].piece;
    folds[i].offset = f[i].offset;
    folds[i].count = f[i].count;
    folds[i].nleaf = f[i].nleaf;
    folds[i].leg = f[i].leg;
    for (t = 0; t < f[i].nleaf; t++) {
      folds[i].buf[t] = f[i].buf[t];
      folds[i].leaf_offset[t] = f[i].loff[t];
    }
  }
  *nops = no;
  *nfolds = nf;
out:
  free(o);
  free(f);
  emac_plan_free(&p);
  return rc;
}
