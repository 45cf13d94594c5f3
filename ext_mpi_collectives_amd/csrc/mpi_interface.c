/*
 * mpi_interface.c -- libext_mpi_collectives.so: the reference's PMPI drop-in surface for the
 * persistent Allreduce, on top of the MPI-free engine (libext_mpi_amd.so).
 *
 * Reference surface restated (src/mpi/ext_mpi_interface.c):
 *   MPI_Init / MPI_Init_thread / MPI_Finalize    :71-183  (thread level capped at SERIALIZED)
 *   MPI_Allreduce_init                           :185-192 (inert placeholder request from
 *                                                          Recv_init + request->handle map)
 *   MPI_Start(all), MPI_Wait(all|any|some),
 *   MPI_Test(all|any|some), MPI_Request_free     :248-426 (requests not owned -> PMPI_*)
 * and the native API EXT_MPI_Init / _Allreduce_init / _Start / _Test / _Wait / _Done /
 * _Finalize (src/mpi/ext_mpi.c:974-1061, include/mpi/ext_mpi.h:69-89).
 *
 * Configuration as the reference reads it (ext_mpi.c:43-187; rank 0 reads the environment and
 * broadcasts): EXT_MPI_COPYIN, EXT_MPI_VERBOSE, EXT_MPI_DEBUG (default 1: the known-answer
 * self-test of debug_persistent.c:393-568 runs inside every Allreduce_init),
 * EXT_MPI_NUM_TASKS_PER_SOCKET (ranks per socket: with the sockets, the node size -- a physical
 * node may hold several logical ones), EXT_MPI_NUM_PORTS (the reference's "nodes(ports)" grammar,
 * ports_groups.c:55-110: the reduce-scatter ports, then the allgather ports, of allreduce_core),
 * EXT_MPI_NUM_SOCKETS_PER_NODE (any divisor of the node size: sockets change the reference's
 * partner encoding and barrier scope, and the tree method's last-step roots -- the one place
 * they reach the fold arithmetic, ext_mpi_amd_set_num_sockets). MPI_Info
 * key "ext_mpi_copyin" overrides nothing the environment sets (num_ports_factors.c:25-36:
 * env > info > default).
 *
 * Blocking front end (EXT_MPI_BLOCKING; ext_mpi_interface.c:507-535, ext_mpi_native_blocking.c:
 * 189-290, 662-741): MPI_Allreduce on MPI_COMM_WORLD and on communicators made by
 * MPI_Comm_dup/create/create_group/split/split_type (:640-729) runs the same persistent engine
 * through a per-communicator cache of handles keyed on (buffers, count, type, parameter row).
 * The copy-in factors come from the reference's parameter file
 * ext_mpi_allreduce_blocking_<nodes>_<cores>.txt (/dev/shm first, then the working directory):
 * one row per message-size threshold, host rows then device rows (README "blocking"); a row's
 * ports column sets the inter-node schedule of the handles made for it, and a row naming another
 * node count or a schedule this path does not take goes to PMPI_Allreduce.
 *
 * Transport (EXT_MPI_AMD_TRANSPORT): "ipc" (default) maps every rank's device buffers into every
 * other rank with hipIpc, as the reference maps them with cudaIpc (src/gpu/cuda_shmem.c:218-299),
 * bootstrapped with PMPI_Allgather; "rccl" runs the legs as RCCL point-to-point rounds,
 * bootstrapped with PMPI_Bcast of the unique id. One engine communicator per MPI communicator,
 * cached as an MPI attribute and destroyed with it. The communicator lies within one node, or
 * spans up to EXT_MPI_AMD_MAX_NODES (64) nodes of equal size in node-major rank order: then the legs run over RCCL with
 * the reference's inter-node schedule (EXT_MPI_NUM_PORTS; unset: one port per step for a power of
 * two, else one step; ext_mpi_amd_comm_set_node_ports); other inter-node shapes return
 * EXT_MPI_AMD_ERROR_UNSUPPORTED (the blocking front end hands them to PMPI).
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ext_mpi.h"
#include "ext_mpi_amd.h"
#include "ext_mpi_amd_gpu.h"
#include "ext_mpi_interface.h"

/* ------------------------------------------------------------------ configuration */

static char cfg_copyin[1024];
static int cfg_has_copyin = 0;
static int cfg_verbose = 0;
static int cfg_debug = 1;
static int cfg_num_sockets = -1;
static int cfg_tasks_per_socket = -1; /* EXT_MPI_NUM_TASKS_PER_SOCKET: ranks of a (logical) socket */
static int cfg_ports_nodes = 0;      /* EXT_MPI_NUM_PORTS: its nodes (0 unset, -1 not this path) */
#define EMAC_PORTS_MAX 17 /* a 0-terminated ports list: 64 nodes at one port per step take 12 */
static int cfg_ports[EMAC_PORTS_MAX]; /* ... its 0-terminated port list (parse_ports) */
static int cfg_blocking = 0;
static int cfg_rccl = 0; /* EXT_MPI_AMD_TRANSPORT=rccl: legs over RCCL instead of hipIpc mappings */
/* Accepted as the reference reads them (ext_mpi.c:58-66, 88-116), with nothing to switch here:
   EXT_MPI_ALTERNATING -- the reference keeps two byte-code copies and swaps them per Start
   (ext_mpi_native.c:215-230, 554-617) so a Start's flags cannot meet the previous one's; here
   every Start is stream-ordered behind the previous and the barrier epochs count per slot;
   EXT_MPI_FAST -- executes the schedule as generated C source (source_code.c) with the same
   arithmetic; there is no interpreter to replace. EXT_MPI_NOT_RECURSIVE selects the
   non-recursive inter-node generator (allreduce.c), out of scope: communicators of several nodes
   are refused under it (the blocking front end hands them to PMPI), one node is unaffected. */
static int cfg_alternating = -1, cfg_fast = 0, cfg_not_recursive = 0;
static int initialised = 0;
static int comm_keyval = MPI_KEYVAL_INVALID;
static int blocking_keyval = MPI_KEYVAL_INVALID;

static int env_int(const char *name, int *out) {
  const char *c = getenv(name);
  int v;
  if (c && sscanf(c, "%d", &v) == 1) {
    *out = v;
    return 1;
  }
  return 0;
}

/* EXT_MPI_NUM_PORTS and the ports column of a blocking parameter row, in the grammar of
   ext_mpi_scan_ports_groups (ports_groups.c:55-110; README: "4(-1 -1 1 1)", "1(-1)"):
   "G(p0 p1 ...)" with G the nodes of the group and p the ports of each inter-node step
   (negative: reduce-scatter, positive: allgather; radix |p| + 1). ' ', ',' and '_' separate.
   Taken here: one group, "1(...)" (one node, no inter-node step) or allreduce_core's list
   (allreduce_recursive.c:222-453): the reduce-scatter ports, then the allgather ports whose
   radices multiply to G -- "4(-1 -1 1 1)", "3(-2 2)", "6(-1 -2 2 1)", and with fewer
   reduce-scatter steps the first allgather steps reduce: "4(3)", "4(-1 1 1)". A bare port list
   (which the reference's scanner runs past the end of) is read as the ports of one group of that
   many nodes. Returns the group's nodes and the 0-terminated list in ports[] (EMAC_PORTS_MAX
   entries at most), 0 for an empty string, or -1 when the string names anything else: several
   groups, a list ending in a reduce-scatter port (reduce_scatter_core), radices that do not fit G. */
static int parse_ports(const char *s, int *ports) {
  int groups = 0, bare = 0, nodes = 0, n = 0, in_group = 0, ok = 1, i, prs = 1, pag = 1, seen_ag = 0;
  const char *p = s;
  ports[0] = 0;
  while (p && *p) {
    char *end;
    long v;
    if (*p == ' ' || *p == ',' || *p == '_') {
      p++;
      continue;
    }
    if (*p == ')') {
      if (!in_group) ok = 0;
      in_group = 0;
      p++;
      continue;
    }
    v = strtol(p, &end, 10);
    if (end == p) return -1;
    p = end;
    while (*p == ' ' || *p == '_') p++;
    if (*p == '(') { /* the group's node count */
      if (in_group || ++groups > 1 || v < 1) ok = 0;
      nodes = (int)v;
      in_group = 1;
      p++;
      continue;
    }
    if (!in_group) bare = 1;
    if (n == EMAC_PORTS_MAX - 1 || v == 0 || v < -(EXT_MPI_AMD_MAX_NODES - 1) || v > EXT_MPI_AMD_MAX_NODES - 1) {
      ok = 0;
      continue;
    }
    ports[n++] = (int)v;
    ports[n] = 0;
  }
  if (!n && !groups) return 0;
  if (!ok || in_group || (bare && groups)) return -1;
  if (nodes == 1) return 1; /* one node: its ports name no inter-node step */
  for (i = 0; i < n; i++) {
    if (ports[i] < 0) {
      if (seen_ag) return -1; /* a reduce-scatter step after an allgather step */
      prs *= 1 - ports[i];
    } else {
      seen_ag = 1;
      pag *= 1 + ports[i];
    }
  }
  /* the allgather radices multiply to the nodes, the reduce-scatter ones to a divisor of it
     (the first allgather steps then reduce inside the groups left, emac_node_sched_build) */
  if (!seen_ag || pag > 16 || pag % prs || (nodes && nodes != pag)) return -1;
  return pag;
}

static void read_env(void) {
  int rank, len = 0;
  PMPI_Comm_rank(MPI_COMM_WORLD, &rank);
  if (rank == 0) {
    const char *c = getenv("EXT_MPI_COPYIN");
    cfg_verbose = getenv("EXT_MPI_VERBOSE") != NULL;
    cfg_blocking = getenv("EXT_MPI_BLOCKING") != NULL; /* ext_mpi_interface.c:46-51 */
    env_int("EXT_MPI_DEBUG", &cfg_debug);
    env_int("EXT_MPI_NUM_SOCKETS_PER_NODE", &cfg_num_sockets);
    env_int("EXT_MPI_NUM_TASKS_PER_SOCKET", &cfg_tasks_per_socket);
    cfg_ports_nodes = parse_ports(getenv("EXT_MPI_NUM_PORTS"), cfg_ports); /* ext_mpi.c:124-157 */
    cfg_rccl = getenv("EXT_MPI_AMD_TRANSPORT") && !strcmp(getenv("EXT_MPI_AMD_TRANSPORT"), "rccl");
    if (env_int("EXT_MPI_NOT_RECURSIVE", &cfg_not_recursive))
      printf("# EXT_MPI not recursive = %d\n", cfg_not_recursive); /* ext_mpi.c:58-63 prints it always */
    if (env_int("EXT_MPI_FAST", &cfg_fast) && cfg_verbose) printf("# EXT_MPI fast %d\n", cfg_fast);
    if (getenv("EXT_MPI_ALTERNATING")) {
      const char a = getenv("EXT_MPI_ALTERNATING")[0];
      if (a == '0' || a == '1') cfg_alternating = a - '0';
      if (cfg_verbose && cfg_alternating >= 0) printf(cfg_alternating ? "# EXT_MPI alternating\n" : "# EXT_MPI not alternating\n");
    }
    if (c) {
      strncpy(cfg_copyin, c, sizeof(cfg_copyin) - 1);
      len = (int)strlen(cfg_copyin) + 1;
    }
  }
  PMPI_Bcast(&cfg_verbose, 1, MPI_INT, 0, MPI_COMM_WORLD);
  PMPI_Bcast(&cfg_blocking, 1, MPI_INT, 0, MPI_COMM_WORLD);
  PMPI_Bcast(&cfg_debug, 1, MPI_INT, 0, MPI_COMM_WORLD);
  PMPI_Bcast(&cfg_num_sockets, 1, MPI_INT, 0, MPI_COMM_WORLD);
  PMPI_Bcast(&cfg_tasks_per_socket, 1, MPI_INT, 0, MPI_COMM_WORLD);
  PMPI_Bcast(&cfg_ports_nodes, 1, MPI_INT, 0, MPI_COMM_WORLD);
  PMPI_Bcast(cfg_ports, EMAC_PORTS_MAX, MPI_INT, 0, MPI_COMM_WORLD);
  PMPI_Bcast(&cfg_rccl, 1, MPI_INT, 0, MPI_COMM_WORLD);
  PMPI_Bcast(&cfg_alternating, 1, MPI_INT, 0, MPI_COMM_WORLD);
  PMPI_Bcast(&cfg_fast, 1, MPI_INT, 0, MPI_COMM_WORLD);
  PMPI_Bcast(&cfg_not_recursive, 1, MPI_INT, 0, MPI_COMM_WORLD);
  PMPI_Bcast(&len, 1, MPI_INT, 0, MPI_COMM_WORLD);
  if (len > 0) PMPI_Bcast(cfg_copyin, len, MPI_CHAR, 0, MPI_COMM_WORLD);
  cfg_has_copyin = len > 0;
  if (cfg_num_sockets > 0) ext_mpi_amd_set_num_sockets(cfg_num_sockets);
}

/* ------------------------------------------- request -> handle map (hash_table.c:8-58) */

typedef struct {
  MPI_Request req;
  int handle;
  int used;
} req_slot;

static req_slot *rmap = NULL;
static int rmap_cap = 0, rmap_n = 0;

static unsigned long req_hash(const MPI_Request *r) {
  const unsigned char *p = (const unsigned char *)r;
  unsigned long h = 1469598103934665603ul;
  size_t i;
  for (i = 0; i < sizeof(MPI_Request); i++) h = (h ^ p[i]) * 1099511628211ul;
  return h;
}

static int rmap_find(const MPI_Request *r) {
  unsigned long i;
  int k;
  if (!rmap_cap) return -1;
  for (k = 0, i = req_hash(r) % (unsigned long)rmap_cap; k < rmap_cap; k++, i = (i + 1) % (unsigned long)rmap_cap) {
    if (!rmap[i].used) return -1;
    if (rmap[i].used == 1 && !memcmp(&rmap[i].req, r, sizeof(MPI_Request))) return (int)i;
  }
  return -1;
}

static int rmap_insert(const MPI_Request *r, int handle);

static void rmap_grow(void) {
  req_slot *old = rmap;
  int i, oldcap = rmap_cap;
  rmap_cap = oldcap ? oldcap * 2 : 256;
  rmap = (req_slot *)calloc((size_t)rmap_cap, sizeof(req_slot));
  rmap_n = 0;
  for (i = 0; i < oldcap; i++)
    if (old[i].used == 1) rmap_insert(&old[i].req, old[i].handle);
  free(old);
}

static int rmap_insert(const MPI_Request *r, int handle) {
  unsigned long i;
  if (2 * (rmap_n + 1) > rmap_cap) rmap_grow();
  for (i = req_hash(r) % (unsigned long)rmap_cap; rmap[i].used == 1; i = (i + 1) % (unsigned long)rmap_cap);
  rmap[i].req = *r;
  rmap[i].handle = handle;
  rmap[i].used = 1;
  rmap_n++;
  return 0;
}

static void rmap_delete(int slot) {
  rmap[slot].used = 2; /* tombstone keeps probe chains intact */
  rmap_n--;
}

static int request_handle(const MPI_Request *r) {
  int s = rmap_find(r);
  return s < 0 ? -1 : rmap[s].handle;
}

/* ------------------------------------------ communicator -> node communicator of the engine */

/* Default: the peer-mapped form (every rank's device buffers mapped into every other rank with
   hipIpc, exchanged with PMPI_Allgather as ext_mpi_sendrecvbuf_init_gpu does with cudaIpc,
   cuda_shmem.c:218-299). EXT_MPI_AMD_TRANSPORT=rccl: an RCCL communicator bootstrapped with
   PMPI_Bcast of the unique id. Either is cached as an attribute of the MPI communicator and
   destroyed with it. The communicator must lie within one node. */
typedef struct {
  int ext_comm;
  int nodes;     /* comm_topology: 1, or the nodes of an RCCL communicator over several */
  int nsize;     /* ranks per node */
  MPI_Comm boot; /* private duplicate the IPC bootstrap exchanges run on */
} comm_attr;

static int mpi_allgather_cb(void *ctx, const void *send, void *recv, long bytes) {
  comm_attr *a = (comm_attr *)ctx;
  return PMPI_Allgather((void *)send, (int)bytes, MPI_BYTE, recv, (int)bytes, MPI_BYTE, a->boot) == MPI_SUCCESS ? 0 : -1;
}

static int comm_attr_delete(MPI_Comm comm, int keyval, void *attr, void *extra) {
  comm_attr *a = (comm_attr *)attr;
  (void)comm;
  (void)keyval;
  (void)extra;
  if (a) {
    ext_mpi_amd_comm_free(a->ext_comm);
    if (a->boot != MPI_COMM_NULL) PMPI_Comm_free(&a->boot);
    free(a);
  }
  return MPI_SUCCESS;
}

/* The communicator's node layout (collective): *nodes = 1 (one node) or up to 64 nodes of equal
   size in node-major rank order (the reference's row layout, ext_mpi_native.c:879-960), 0 for
   any other shape; *nsize = ranks per node, *nrank = rank in the node. The reference's node
   is EXT_MPI_NUM_TASKS_PER_SOCKET x sockets consecutive ranks when that is set (ext_mpi.c:195-215,
   :638): a physical node may hold several logical ones. */
static void comm_topology(MPI_Comm comm, int *nodes, int *nsize, int *nrank) {
  int size, rank, v[2];
  MPI_Comm node;
  PMPI_Comm_size(comm, &size);
  PMPI_Comm_rank(comm, &rank);
  PMPI_Comm_split_type(comm, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &node);
  PMPI_Comm_size(node, nsize);
  PMPI_Comm_rank(node, nrank);
  PMPI_Comm_free(&node);
  if (cfg_tasks_per_socket > 0) {
    const int lsize = cfg_tasks_per_socket * (cfg_num_sockets > 0 ? cfg_num_sockets : 1);
    if (lsize <= *nsize && *nsize % lsize == 0) {
      *nsize = lsize;
      *nrank = rank % lsize;
    }
  }
  *nodes = *nsize > 0 && size % *nsize == 0 ? size / *nsize : 0;
  v[0] = *nsize == size;
  v[1] = *nodes >= 2 && *nodes <= EXT_MPI_AMD_MAX_NODES && *nrank == rank % *nsize;
  PMPI_Allreduce(MPI_IN_PLACE, v, 2, MPI_INT, MPI_MIN, comm);
  *nodes = v[0] ? 1 : v[1] ? *nodes : 0;
}

/* EXT_MPI_NUM_PORTS for a communicator of `nodes` nodes: *ports = its list, or NULL for the
   default (one port per step for a power of two, else one step of radix `nodes`); -1 when it
   names a schedule this path does not take or another node count */
static int env_ports(int nodes, const int **ports) {
  *ports = NULL;
  if (nodes <= 1 || cfg_ports_nodes == 0) return 0;
  if (cfg_ports_nodes != nodes) return -1; /* not this path (-1), or a group of another size */
  *ports = cfg_ports;
  return 0;
}

/* The engine communicator of `comm` (collective at its first use): *nodes / *nsize its node layout.
   Over several nodes it starts with the default inter-node schedule; every handle sets its own
   (EXT_MPI_NUM_PORTS or a blocking parameter row, ext_mpi_amd_comm_set_node_ports) before it is
   made, so the first message size cannot decide the communicator's fate. `check_env`: refuse
   (ERROR_UNSUPPORTED, nothing created) when EXT_MPI_NUM_PORTS names a schedule this path does not
   take over these nodes -- the persistent path's verdict; the blocking path checks per call. */
static int node_comm(MPI_Comm comm, const void *devbuf, int check_env, int *ext_comm, int *nodes_out,
                     int *nsize_out) {
  comm_attr *a;
  int flag, size, rank, nsize, nrank, device, ndev, rc, nodes;
  unsigned char id[EXT_MPI_AMD_UNIQUE_ID_BYTES];
  if (comm_keyval == MPI_KEYVAL_INVALID) return EXT_MPI_AMD_ERROR_ARG;
  PMPI_Comm_get_attr(comm, comm_keyval, &a, &flag);
  if (flag && a) {
    *ext_comm = a->ext_comm;
    if (nodes_out) *nodes_out = a->nodes;
    if (nsize_out) *nsize_out = a->nsize;
    return 0;
  }
  PMPI_Comm_size(comm, &size);
  PMPI_Comm_rank(comm, &rank);
  comm_topology(comm, &nodes, &nsize, &nrank);
  if (!nodes) return EXT_MPI_AMD_ERROR_UNSUPPORTED; /* other inter-node shapes: out of scope */
  if (check_env && nodes > 1) {
    const int *hp;
    if (cfg_not_recursive || env_ports(nodes, &hp)) return EXT_MPI_AMD_ERROR_UNSUPPORTED;
  }
  ndev = ext_mpi_amd_gpu_device_count();
  device = ext_mpi_amd_gpu_device_of(devbuf);
  if (device < 0) device = ndev > 0 ? nrank % ndev : -1;
  a = (comm_attr *)calloc(1, sizeof(comm_attr));
  if (!a) return EXT_MPI_AMD_ERROR_MALLOC;
  a->boot = MPI_COMM_NULL;
  a->nodes = nodes;
  a->nsize = nsize;
  if (!cfg_rccl && nodes == 1) { /* peer mappings reach the ranks of one node only */
    PMPI_Comm_dup(comm, &a->boot);
    /* collective even without a device: every rank reaches the same verdict */
    rc = ext_mpi_amd_comm_init_ipc(rank, size, mpi_allgather_cb, a, ndev > 0 ? device : -1, ext_comm);
    if (rc) {
      PMPI_Comm_free(&a->boot);
      free(a);
      return rc;
    }
  } else {
    if (rank == 0 && (rc = ext_mpi_amd_get_unique_id(id))) memset(id, 0, sizeof(id));
    PMPI_Bcast(id, EXT_MPI_AMD_UNIQUE_ID_BYTES, MPI_BYTE, 0, comm);
    rc = ndev > 0 ? ext_mpi_amd_comm_init(rank, size, id, device, ext_comm) : EXT_MPI_AMD_ERROR_DEVICE;
    if (rc == 0 && nodes > 1 && (rc = ext_mpi_amd_comm_set_node_ports(*ext_comm, nodes, NULL)))
      ext_mpi_amd_comm_free(*ext_comm);
    flag = rc == 0;
    PMPI_Allreduce(MPI_IN_PLACE, &flag, 1, MPI_INT, MPI_MIN, comm);
    if (!flag) {
      if (rc == 0) ext_mpi_amd_comm_free(*ext_comm);
      free(a);
      return rc ? rc : EXT_MPI_AMD_ERROR_TRANSPORT;
    }
  }
  a->ext_comm = *ext_comm;
  PMPI_Comm_set_attr(comm, comm_keyval, a);
  if (nodes_out) *nodes_out = nodes;
  if (nsize_out) *nsize_out = nsize;
  return 0;
}

/* ------------------------------------------------ datatype / op (ext_mpi_native.h:77-140) */

static int map_type(MPI_Datatype t) {
  if (t == MPI_FLOAT || t == MPI_REAL || t == MPI_REAL4) return EXT_MPI_AMD_FLOAT;
  if (t == MPI_DOUBLE || t == MPI_DOUBLE_PRECISION || t == MPI_REAL8) return EXT_MPI_AMD_DOUBLE;
  if (t == MPI_INT || t == MPI_INTEGER || t == MPI_INTEGER4) return EXT_MPI_AMD_INT;
  if (t == MPI_LONG || t == MPI_INTEGER8) return EXT_MPI_AMD_LONG;
  return -1;
}

/* get_reduction_op (include/mpi/ext_mpi_native.h:77-140): SUM, MIN and MAX; user ops -> PMPI */
static int map_op(MPI_Op op) {
  if (op == MPI_SUM) return EXT_MPI_AMD_SUM;
  if (op == MPI_MIN) return EXT_MPI_AMD_MIN;
  if (op == MPI_MAX) return EXT_MPI_AMD_MAX;
  return -1;
}

/* ------------------------------------------- known-answer self-test (debug_persistent.c) */

static void kat_fill(void *buf, long count, int tsize, int world_rank, long add) {
  long i, words = (count * tsize) / (long)sizeof(long);
  for (i = 0; i < words; i++) ((long *)buf)[i] = world_rank * count + i + add;
  if ((count * tsize) % (long)sizeof(long)) ((int *)buf)[count - 1] = (int)(world_rank * count + count - 1);
}

/* debug_persistent.c:393-568: the same schedule on an integer view of the same byte size,
   checked word for word against PMPI_Allreduce. Host pattern +73, device pattern +0. */
static int known_answer_test(void *recvbuf, int in_place, int count, int tsize, MPI_Comm comm, int ext_comm,
                             const char *copyin) {
  int world_rank, on_dev = ext_mpi_amd_gpu_is_device_pointer(recvbuf), rc = 0, bad = 0, h = -1;
  int itype = tsize == 8 ? EXT_MPI_AMD_LONG : EXT_MPI_AMD_INT;
  size_t bytes = (size_t)count * (size_t)tsize;
  void *hs = malloc(bytes ? bytes : 1), *hr = malloc(bytes ? bytes : 1), *ref = malloc(bytes ? bytes : 1);
  void *ds = NULL, *dr = NULL;
  long i;
  PMPI_Comm_rank(MPI_COMM_WORLD, &world_rank);
  kat_fill(hs, count, tsize, world_rank, on_dev ? 0 : 73);
  PMPI_Allreduce(hs, ref, count, tsize == 8 ? MPI_LONG : MPI_INT, MPI_SUM, comm);
  if (on_dev) {
    /* communicator-owned: released below while slower peers may still map them */
    if ((rc = ext_mpi_amd_comm_malloc(ext_comm, &dr, bytes))) goto out;
    if (!in_place && (rc = ext_mpi_amd_comm_malloc(ext_comm, &ds, bytes))) goto out;
    if ((rc = ext_mpi_amd_gpu_memcpy_hd(in_place ? dr : ds, hs, bytes))) goto out;
    rc = ext_mpi_amd_allreduce_init(in_place ? dr : ds, dr, count, itype, EXT_MPI_AMD_SUM, ext_comm, copyin, &h);
  } else {
    if (in_place) memcpy(hr, hs, bytes);
    rc = ext_mpi_amd_allreduce_init(in_place ? hr : hs, hr, count, itype, EXT_MPI_AMD_SUM, ext_comm, copyin, &h);
  }
  if (!rc) rc = ext_mpi_amd_start(h);
  if (!rc) rc = ext_mpi_amd_wait(h);
  if (h >= 0) ext_mpi_amd_done(h);
  if (!rc && on_dev) rc = ext_mpi_amd_gpu_memcpy_dh(hr, dr, bytes);
  if (!rc) {
    if (tsize == 8) {
      for (i = 0; i < count; i++) bad |= ((long *)hr)[i] != ((long *)ref)[i];
    } else {
      for (i = 0; i < count; i++) bad |= ((int *)hr)[i] != ((int *)ref)[i];
    }
  }
out:
  ext_mpi_amd_comm_mfree(ext_comm, ds);
  ext_mpi_amd_comm_mfree(ext_comm, dr);
  free(hs);
  free(hr);
  free(ref);
  if (!rc && bad) {
    printf("logical error in EXT_MPI_Allreduce %d\n", world_rank); /* debug_persistent.c:542-545 */
    rc = EXT_MPI_AMD_ERROR_ARG;
  }
  return rc;
}


/* ------------------------------------------- blocking MPI_Allreduce (EXT_MPI_BLOCKING) */

#define BROWS 64
#define BCACHE 16
#define BLOCKING_MAX_BYTES (1024L * 1024L * 100L) /* ext_mpi_interface.c:517 */

typedef struct {
  long msize;  /* message size in bytes from which the row applies */
  int sockets; /* logical sockets per node */
  int nodes;   /* "<nodes>(<ports>)" field, parse_ports: its nodes (-1: not this path) */
  int ports[EMAC_PORTS_MAX]; /* ... its 0-terminated port list */
  char copyin[256];
} brow;

typedef struct {
  const void *send;
  void *recv;
  int count, dtype, op, side, row, handle;
  unsigned long used;
  long serial; /* creation number: equal on every rank for the same collective creation */
} bentry;

/* Per-communicator state of the blocking path (comm_comm_blocking, ext_mpi_native_blocking.c). */
typedef struct {
  int status; /* 0 not yet bound, 1 bound to ext_comm, <0 engine error, 2 not for this path */
  int ext_comm;
  int nodes, nsize; /* comm_topology (nodes 0: a shape this path does not take); nodes < 0: not yet */
  int loaded, nrow[2]; /* [0] host rows, [1] device rows */
  brow row[2][BROWS];
  bentry cache[BCACHE];
  unsigned long clock;
  long serial;
  void *scratch;
  size_t scratch_bytes;
} bcomm;

static void bcomm_drop(bcomm *b, int i) {
  if (b->cache[i].handle >= 0) ext_mpi_amd_done(b->cache[i].handle);
  memset(&b->cache[i], 0, sizeof(bentry));
  b->cache[i].handle = -1;
}

static int bcomm_delete(MPI_Comm comm, int keyval, void *attr, void *extra) {
  bcomm *b = (bcomm *)attr;
  int i;
  (void)comm;
  (void)keyval;
  (void)extra;
  if (b) {
    for (i = 0; i < BCACHE; i++) bcomm_drop(b, i);
    /* the scratch belongs to the engine communicator (freed with it if that went first) */
    if (b->scratch) ext_mpi_amd_comm_mfree(b->ext_comm, b->scratch);
    free(b);
  }
  return MPI_SUCCESS;
}

/* add_comm_to_blocking (ext_mpi_interface.c:640-651); MPI_COMM_WORLD is added whatever its
   size (:57-60). */
static void blocking_register(MPI_Comm comm, int any_size) {
  bcomm *b;
  int size, i;
  if (!cfg_blocking || blocking_keyval == MPI_KEYVAL_INVALID || comm == MPI_COMM_NULL) return;
  PMPI_Comm_size(comm, &size);
  if (size <= 1 && !any_size) return;
  b = (bcomm *)calloc(1, sizeof(bcomm));
  if (!b) return;
  for (i = 0; i < BCACHE; i++) b->cache[i].handle = -1;
  b->nodes = -1;
  PMPI_Comm_set_attr(comm, blocking_keyval, b);
}

/* init_blocking_native (ext_mpi_native_blocking.c:189-290): "<bytes> <sockets> <ports>
   <copyin>" per line, '_' standing for ' '; a non-increasing size starts the device rows. The
   file is ext_mpi_allreduce_blocking_<nodes>_<cores per node>.txt (:225-230). */
static void blocking_load_rows(bcomm *b, MPI_Comm comm) {
  char fname[256], ports[1000], cf[1000];
  long ms, prev = -1;
  int so, rank, side = 0, i;
  FILE *f;
  PMPI_Comm_rank(comm, &rank);
  b->loaded = 1;
  snprintf(fname, sizeof(fname), "/dev/shm/ext_mpi_allreduce_blocking_%d_%d.txt", b->nodes, b->nsize);
  f = fopen(fname, "r");
  if (!f) {
    snprintf(fname, sizeof(fname), "ext_mpi_allreduce_blocking_%d_%d.txt", b->nodes, b->nsize);
    f = fopen(fname, "r");
  }
  if (!f) {
    if (rank == 0 && cfg_verbose) printf("# EXT_MPI blocking: file %s missing, using the persistent copyin\n", fname);
    return;
  }
  while (fscanf(f, "%ld %d %999s %999s", &ms, &so, ports, cf) == 4) {
    brow *r;
    if (ms <= prev) side = 1;
    prev = ms;
    if (b->nrow[side] == BROWS) continue;
    r = &b->row[side][b->nrow[side]++];
    r->msize = ms;
    r->sockets = so;
    r->nodes = parse_ports(ports, r->ports);
    for (i = 0; cf[i]; i++)
      if (cf[i] == '_') cf[i] = ' ';
    snprintf(r->copyin, sizeof(r->copyin), "%.255s", cf);
  }
  fclose(f);
}

/* Row choice of EXT_MPI_Allreduce_native (ext_mpi_native_blocking.c:687-688): the last row whose
   size does not exceed the message, else the first. */
static int blocking_select_row(const bcomm *b, int side, long bytes) {
  int n = b->nrow[side], i = 0;
  if (!n) return -1;
  while (b->row[side][i].msize <= bytes && i + 1 < n) i++;
  if (b->row[side][i].msize > bytes && i > 0) i--;
  return i;
}

/* 0: done, 1: not for this path (caller uses PMPI_Allreduce), <0: engine error. */
static int blocking_allreduce(const void *sendbuf, void *recvbuf, int count, int dtype, int op, int tsize, bcomm *b,
                              MPI_Comm comm) {
  size_t bytes = (size_t)count * (size_t)tsize, need, stride;
  int on_dev, side, row, i, rc, slot = -1, in_place, rank, row_sockets = 0, staged;
  const char *copyin = NULL;
  const void *s;
  void *r;
  bentry *e;
  if (sendbuf == MPI_IN_PLACE) sendbuf = recvbuf; /* ext_mpi_blocking.c:427-429 */
  in_place = sendbuf == recvbuf;
  if (b->nodes < 0) {
    int nrank;
    comm_topology(comm, &b->nodes, &b->nsize, &nrank); /* collective: every rank, first call */
  }
  if (!b->nodes || (b->nodes > 1 && cfg_not_recursive)) return 1; /* an inter-node shape this path does not take */
  if (!b->loaded) blocking_load_rows(b, comm);
  on_dev = ext_mpi_amd_gpu_is_device_pointer(recvbuf) && ext_mpi_amd_gpu_is_device_pointer(sendbuf);
  side = on_dev && b->nrow[1] ? 1 : 0;
  row = blocking_select_row(b, side, (long)bytes);
  if (row >= 0) {
    const brow *w = &b->row[side][row];
    /* the row's inter-node schedule must be one this path takes, over this communicator's nodes */
    if (w->nodes != b->nodes) return 1;
    if (w->sockets < 1 || b->nsize % w->sockets) return 1;
    copyin = w->copyin;
    row_sockets = w->sockets;
  } else if (cfg_has_copyin) {
    copyin = cfg_copyin;
  }
  /* without a row the communicator's own EXT_MPI_NUM_PORTS governs; one naming another node
     count or a list this path does not take goes to PMPI (same verdict on every rank) */
  if (row < 0 && b->nodes > 1) {
    const int *hp;
    if (env_ports(b->nodes, &hp)) return 1;
  }
  if (b->status == 0) {
    rc = node_comm(comm, recvbuf, 0, &b->ext_comm, NULL, NULL);
    b->status = rc == 0 ? 1 : rc == EXT_MPI_AMD_ERROR_UNSUPPORTED ? 2 : rc;
  }
  if (b->status != 1) return b->status == 2 ? 1 : b->status;
  /* Host buffers go through device scratch (no page-locking of caller memory that may be freed
     between calls), and so do device buffers on the peer-mapped transport: a cached handle must
     not keep mappings of caller allocations the application may free and re-allocate between two
     calls (the reference hooks cudaFree for that, cuda_shmem.c); the scratch is library memory,
     so dropping a cached handle is local on every rank (ext_mpi_amd_done). */
  staged = !on_dev || !cfg_rccl;
  if (!staged) {
    s = sendbuf;
    r = recvbuf;
  } else {
    stride = (bytes + 255) & ~(size_t)255;
    need = in_place ? stride : 2 * stride;
    if (need < 256) need = 256;
    if (b->scratch_bytes < need) {
      for (i = 0; i < BCACHE; i++)
        if (b->cache[i].handle >= 0 && b->cache[i].send == b->scratch) bcomm_drop(b, i);
      /* communicator-owned (peers may still map the old scratch): back to its pool, not freed */
      ext_mpi_amd_comm_mfree(b->ext_comm, b->scratch);
      b->scratch = NULL;
      b->scratch_bytes = 0;
      if ((rc = ext_mpi_amd_comm_malloc(b->ext_comm, &b->scratch, need))) return rc;
      b->scratch_bytes = need;
    }
    s = b->scratch;
    r = in_place ? b->scratch : (char *)b->scratch + stride;
    /* synchronous copies in and out: stream-ordered ones on the handle's stream measured slower on
       MI355X (2 and 4 ranks sharing one GPU, 1 KiB - 16 MiB: 83-169 us against 39-141 us per call,
       profiles/r04/blocking_staging.txt): they go to a DMA engine, whose latency the synchronous
       blit-kernel copies do not pay. (Round 4's opt-in for them was removed) */
    if (bytes && (rc = ext_mpi_amd_gpu_memcpy_hd((void *)s, sendbuf, bytes))) return rc;
  }
  for (i = 0; i < BCACHE; i++) {
    e = &b->cache[i];
    if (e->handle >= 0 && e->send == s && e->recv == r && e->count == count && e->dtype == dtype && e->op == op &&
        e->side == side &&
        e->row == row) {
      slot = i;
      break;
    }
  }
  if (!cfg_rccl) {
    /* a peer-mapped handle embeds every rank's buffers: it is reused only if every rank found
       the same one (same creation); otherwise every rank creates a new one, in step */
    long v[2];
    v[0] = slot >= 0 ? b->cache[slot].serial : -1;
    v[1] = slot >= 0 ? -b->cache[slot].serial : 1;
    PMPI_Allreduce(MPI_IN_PLACE, v, 2, MPI_LONG, MPI_MIN, comm);
    if (v[0] < 0 || v[0] != -v[1]) {
      if (slot >= 0) bcomm_drop(b, slot); /* keep keys unique: the new handle replaces it */
      slot = -1;
    }
  }
  if (slot < 0) {
    slot = 0;
    for (i = 0; i < BCACHE; i++) {
      if (b->cache[i].handle < 0) {
        slot = i;
        break;
      }
      if (b->cache[i].used < b->cache[slot].used) slot = i;
    }
    bcomm_drop(b, slot);
    e = &b->cache[slot];
    /* a parameter-file row names its own socket count (ext_mpi_native_blocking.c:189-290) and
       inter-node ports; a handle keeps the schedule it was made with. Both are restored on every
       exit; a row whose ports the engine refuses (e.g. an allgather step crossing the
       reduce-scatter groups) goes to PMPI like any row this path does not take. */
    const int prev_sockets = row_sockets > 0 ? ext_mpi_amd_set_num_sockets(row_sockets) : 0;
    const int *hp = NULL;
    int pmpi = 0;
    if (b->nodes > 1) {
      if (row >= 0)
        hp = b->row[side][row].ports;
      else if (env_ports(b->nodes, &hp))
        pmpi = 1;
      if (!pmpi && ext_mpi_amd_comm_set_node_ports(b->ext_comm, b->nodes, hp)) pmpi = 1;
    }
    rc = pmpi ? 0 : ext_mpi_amd_allreduce_init(s, r, count, dtype, op, b->ext_comm, copyin, &e->handle);
    if (prev_sockets > 0) ext_mpi_amd_set_num_sockets(prev_sockets);
    if (b->nodes > 1) { /* back to the communicator's own (EXT_MPI_NUM_PORTS or the default) */
      if (env_ports(b->nodes, &hp)) hp = NULL;
      ext_mpi_amd_comm_set_node_ports(b->ext_comm, b->nodes, hp);
    }
    if (pmpi || rc) {
      e->handle = -1;
      return pmpi ? 1 : rc;
    }
    e->send = s;
    e->recv = r;
    e->serial = ++b->serial;
    e->count = count;
    e->dtype = dtype;
    e->op = op;
    e->side = side;
    e->row = row;
    if (cfg_verbose) {
      PMPI_Comm_rank(comm, &rank);
      if (rank == 0)
        printf("# EXT_MPI blocking allreduce %zu bytes %s copyin %s\n", bytes, on_dev ? "device" : "host",
               copyin ? copyin : "(default 6;1 -R R)");
    }
  }
  e = &b->cache[slot];
  e->used = ++b->clock;
  if ((rc = ext_mpi_amd_start(e->handle)) || (rc = ext_mpi_amd_wait(e->handle))) return rc;
  if (staged && bytes && (rc = ext_mpi_amd_gpu_memcpy_dh(recvbuf, r, bytes))) return rc;
  return 0;
}

/* ------------------------------------------------------------------- native API */

int EXT_MPI_Init(void) {
  if (initialised) return 0;
  read_env();
  PMPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, comm_attr_delete, &comm_keyval, NULL);
  PMPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, bcomm_delete, &blocking_keyval, NULL);
  initialised = 1;
  if (cfg_blocking) {
    int rank;
    PMPI_Comm_rank(MPI_COMM_WORLD, &rank);
    if (rank == 0 && cfg_verbose) printf("# EXT_MPI blocking\n"); /* ext_mpi_interface.c:52-54 */
    blocking_register(MPI_COMM_WORLD, 1);
  }
  return 0;
}

int EXT_MPI_Initialized(int *flag) {
  *flag = initialised;
  return 0;
}

int EXT_MPI_Finalize(void) {
  if (!initialised) return 0;
  initialised = 0;
  /* MPI_COMM_WORLD's attributes are not deleted by MPI_Finalize: release the blocking cache
     first (its handles use the RCCL communicator), then the RCCL communicator; the other
     communicators' go with MPI_Comm_free. */
  PMPI_Comm_delete_attr(MPI_COMM_WORLD, blocking_keyval);
  PMPI_Comm_delete_attr(MPI_COMM_WORLD, comm_keyval);
  return 0;
}

int EXT_MPI_Allreduce_init(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                           MPI_Comm comm, MPI_Info info, int *handle) {
  int dtype = map_type(datatype), eop = map_op(op), ext_comm, rc, flag = 0, rank, tsize, nodes = 1, nsize = 1;
  const char *copyin = NULL;
  char info_copyin[1024];
  *handle = -1;
  if (!initialised) EXT_MPI_Init();
  if (dtype < 0 || eop < 0 || count < 0) return EXT_MPI_AMD_ERROR_UNSUPPORTED;
  if (sendbuf == MPI_IN_PLACE) sendbuf = recvbuf; /* ext_mpi.c:651-653 */
  if (cfg_has_copyin) {
    copyin = cfg_copyin;
  } else if (info != MPI_INFO_NULL) {
    PMPI_Info_get(info, "ext_mpi_copyin", (int)sizeof(info_copyin) - 1, info_copyin, &flag);
    if (flag) copyin = info_copyin;
  }
  if ((rc = node_comm(comm, recvbuf, 1, &ext_comm, &nodes, &nsize))) return rc;
  /* sockets change the partner encoding and the tree method's last roots (plan.h): they must
     divide the ranks of a node */
  if (cfg_num_sockets > 1 && nsize % cfg_num_sockets) return EXT_MPI_AMD_ERROR_UNSUPPORTED;
  if (nodes > 1) { /* this handle's inter-node schedule: EXT_MPI_NUM_PORTS or the default */
    const int *hp;
    if (cfg_not_recursive) return EXT_MPI_AMD_ERROR_UNSUPPORTED;
    if (env_ports(nodes, &hp)) return EXT_MPI_AMD_ERROR_UNSUPPORTED;
    if ((rc = ext_mpi_amd_comm_set_node_ports(ext_comm, nodes, hp))) return rc;
  }
  PMPI_Type_size(datatype, &tsize);
  if (cfg_debug && (rc = known_answer_test(recvbuf, sendbuf == recvbuf, count, tsize, comm, ext_comm, copyin)))
    return rc;
  rc = ext_mpi_amd_allreduce_init(sendbuf, recvbuf, count, dtype, eop, ext_comm, copyin, handle);
  if (cfg_verbose) {
    PMPI_Comm_rank(comm, &rank);
    if (rank == 0) printf("# EXT_MPI allreduce parameters copyin %s\n", copyin ? copyin : "(default 6;1 -R R)");
  }
  return rc;
}

int EXT_MPI_Start(int handle) { return handle >= 0 ? ext_mpi_amd_start(handle) : -1; }
int EXT_MPI_Test(int handle) { return handle >= 0 ? ext_mpi_amd_test(handle) : -1; }
int EXT_MPI_Wait(int handle) { return handle >= 0 ? ext_mpi_amd_wait(handle) : -1; }
int EXT_MPI_Done(int handle) { return handle >= 0 ? ext_mpi_amd_done(handle) : -1; }

/* ------------------------------------------------------------------- PMPI hooks */

int MPI_Init(int *argc, char ***argv) {
  int ret = PMPI_Init(argc, argv);
  EXT_MPI_Init();
  return ret;
}

int MPI_Init_thread(int *argc, char ***argv, int required, int *provided) {
  int ret = PMPI_Init_thread(argc, argv, required, provided);
  EXT_MPI_Init();
  if (!(*provided == MPI_THREAD_SINGLE || *provided == MPI_THREAD_FUNNELED || *provided == MPI_THREAD_SERIALIZED))
    *provided = MPI_THREAD_SERIALIZED;
  return ret;
}

int MPI_Finalize(void) {
  EXT_MPI_Finalize();
  free(rmap);
  rmap = NULL;
  rmap_cap = rmap_n = 0;
  return PMPI_Finalize();
}

int MPI_Allreduce_init(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                       MPI_Info info, MPI_Request *request) {
  int handle, ret;
  /* an inert persistent request that only names the operation (ext_mpi_interface.c:187) */
  PMPI_Recv_init(NULL, 0, datatype, MPI_PROC_NULL, 0, comm, request);
  ret = EXT_MPI_Allreduce_init(sendbuf, recvbuf, count, datatype, op, comm, info, &handle);
  if (!ret) rmap_insert(request, handle);
  return ret;
}

int MPI_Request_free(MPI_Request *request) {
  int s = rmap_find(request);
  if (s >= 0) {
    EXT_MPI_Done(rmap[s].handle);
    rmap_delete(s);
  }
  return PMPI_Request_free(request);
}

int MPI_Start(MPI_Request *request) {
  int h = request_handle(request);
  if (h >= 0) return EXT_MPI_Start(h) < 0 ? MPI_ERR_OTHER : MPI_SUCCESS;
  return PMPI_Start(request);
}

int MPI_Startall(int count, MPI_Request array_of_requests[]) {
  int i, ret;
  for (i = 0; i < count; i++) {
    ret = MPI_Start(&array_of_requests[i]);
    if (ret != MPI_SUCCESS) return ret;
  }
  return MPI_SUCCESS;
}

int MPI_Wait(MPI_Request *request, MPI_Status *status) {
  int h = request_handle(request);
  if (h >= 0) return EXT_MPI_Wait(h) < 0 ? MPI_ERR_OTHER : MPI_SUCCESS;
  return PMPI_Wait(request, status);
}

int MPI_Test(MPI_Request *request, int *flag, MPI_Status *status) {
  int h = request_handle(request);
  if (h >= 0) {
    int r = EXT_MPI_Test(h);
    if (r < 0) return MPI_ERR_OTHER;
    *flag = r;
    return MPI_SUCCESS;
  }
  return PMPI_Test(request, flag, status);
}

static int owns_any(int count, MPI_Request reqs[]) {
  int i;
  for (i = 0; i < count; i++)
    if (request_handle(&reqs[i]) >= 0) return 1;
  return 0;
}

int MPI_Waitall(int count, MPI_Request array_of_requests[], MPI_Status array_of_statuses[]) {
  int i, ret;
  if (!owns_any(count, array_of_requests)) return PMPI_Waitall(count, array_of_requests, array_of_statuses);
  for (i = 0; i < count; i++) {
    ret = MPI_Wait(&array_of_requests[i],
                   array_of_statuses == MPI_STATUSES_IGNORE ? MPI_STATUS_IGNORE : &array_of_statuses[i]);
    if (ret != MPI_SUCCESS) return ret;
  }
  return MPI_SUCCESS;
}

int MPI_Testall(int count, MPI_Request array_of_requests[], int *flag, MPI_Status array_of_statuses[]) {
  int i, ret, f;
  if (!owns_any(count, array_of_requests)) return PMPI_Testall(count, array_of_requests, flag, array_of_statuses);
  *flag = 1;
  for (i = 0; i < count; i++) {
    ret = MPI_Test(&array_of_requests[i], &f,
                   array_of_statuses == MPI_STATUSES_IGNORE ? MPI_STATUS_IGNORE : &array_of_statuses[i]);
    if (ret != MPI_SUCCESS) return ret;
    if (!f) *flag = 0;
  }
  return MPI_SUCCESS;
}

int MPI_Testany(int count, MPI_Request array_of_requests[], int *indx, int *flag, MPI_Status *status) {
  int i, ret, f;
  if (!owns_any(count, array_of_requests)) return PMPI_Testany(count, array_of_requests, indx, flag, status);
  *flag = 0;
  for (i = 0; i < count; i++) {
    ret = MPI_Test(&array_of_requests[i], &f, status);
    if (ret != MPI_SUCCESS) return ret;
    if (f) {
      *flag = 1;
      *indx = i;
      return MPI_SUCCESS;
    }
  }
  return MPI_SUCCESS;
}

int MPI_Waitany(int count, MPI_Request array_of_requests[], int *indx, MPI_Status *status) {
  int flag = 0, ret;
  if (!owns_any(count, array_of_requests)) return PMPI_Waitany(count, array_of_requests, indx, status);
  while (!flag) {
    ret = MPI_Testany(count, array_of_requests, indx, &flag, status);
    if (ret != MPI_SUCCESS) return ret;
  }
  return MPI_SUCCESS;
}

int MPI_Waitsome(int incount, MPI_Request array_of_requests[], int *outcount, int array_of_indices[],
                 MPI_Status array_of_statuses[]) {
  if (!owns_any(incount, array_of_requests))
    return PMPI_Waitsome(incount, array_of_requests, outcount, array_of_indices, array_of_statuses);
  *outcount = 1;
  return MPI_Waitany(incount, array_of_requests, &array_of_indices[0],
                     array_of_statuses == MPI_STATUSES_IGNORE ? MPI_STATUS_IGNORE : &array_of_statuses[0]);
}

int MPI_Testsome(int incount, MPI_Request array_of_requests[], int *outcount, int array_of_indices[],
                 MPI_Status array_of_statuses[]) {
  int flag = 0, ret;
  if (!owns_any(incount, array_of_requests))
    return PMPI_Testsome(incount, array_of_requests, outcount, array_of_indices, array_of_statuses);
  ret = MPI_Testany(incount, array_of_requests, &array_of_indices[0], &flag,
                    array_of_statuses == MPI_STATUSES_IGNORE ? MPI_STATUS_IGNORE : &array_of_statuses[0]);
  *outcount = flag ? 1 : 0;
  return ret;
}

/* Blocking MPI_Allreduce (ext_mpi_interface.c:507-535): SUM / MIN / MAX over the four types below 100 MB on
   a registered communicator; anything else goes to PMPI_Allreduce. */
int MPI_Allreduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op, MPI_Comm comm) {
  int dtype = map_type(datatype), eop = map_op(op), tsize, flag = 0, rc, rank;
  bcomm *b = NULL;
  if (cfg_blocking && initialised && dtype >= 0 && eop >= 0 && count >= 0) {
    PMPI_Type_size(datatype, &tsize);
    if ((long)count * tsize < BLOCKING_MAX_BYTES) {
      PMPI_Comm_get_attr(comm, blocking_keyval, &b, &flag);
      if (flag && b) {
        rc = blocking_allreduce(sendbuf, recvbuf, count, dtype, eop, tsize, b, comm);
        if (rc == 0) return MPI_SUCCESS;
        if (rc < 0) {
          PMPI_Comm_rank(comm, &rank);
          fprintf(stderr, "EXT_MPI blocking allreduce failed on rank %d: %d\n", rank, rc);
          return MPI_ERR_OTHER;
        }
      }
    }
  }
  return PMPI_Allreduce(sendbuf, recvbuf, count, datatype, op, comm);
}

/* Communicators the blocking path serves (ext_mpi_interface.c:663-721). */
int MPI_Comm_dup(MPI_Comm comm, MPI_Comm *newcomm) {
  int ret = PMPI_Comm_dup(comm, newcomm);
  if (ret == MPI_SUCCESS) blocking_register(*newcomm, 0);
  return ret;
}

int MPI_Comm_create(MPI_Comm comm, MPI_Group group, MPI_Comm *newcomm) {
  int ret = PMPI_Comm_create(comm, group, newcomm);
  if (ret == MPI_SUCCESS) blocking_register(*newcomm, 0);
  return ret;
}

int MPI_Comm_create_group(MPI_Comm comm, MPI_Group group, int tag, MPI_Comm *newcomm) {
  int ret = PMPI_Comm_create_group(comm, group, tag, newcomm);
  if (ret == MPI_SUCCESS) blocking_register(*newcomm, 0);
  return ret;
}

int MPI_Comm_split(MPI_Comm comm, int color, int key, MPI_Comm *newcomm) {
  int ret = PMPI_Comm_split(comm, color, key, newcomm);
  if (ret == MPI_SUCCESS) blocking_register(*newcomm, 0);
  return ret;
}

int MPI_Comm_split_type(MPI_Comm comm, int split_type, int key, MPI_Info info, MPI_Comm *newcomm) {
  int ret = PMPI_Comm_split_type(comm, split_type, key, info, newcomm);
  if (ret == MPI_SUCCESS) blocking_register(*newcomm, 0);
  return ret;
}
