"""MI355X-native bucket-reduction path of ext_mpi_collectives (persistent MPI_SUM Allreduce).

The product is the C library ``libext_mpi_amd.so`` (host C engine + gfx950 HIP kernels, built
from ``csrc/``) and its PMPI layer ``libext_mpi_collectives.so``. This module is a thin ctypes
front-end for tests and benchmarks; it mirrors the reference's native API
(``EXT_MPI_Allreduce_init / EXT_MPI_Start / EXT_MPI_Test / EXT_MPI_Wait / EXT_MPI_Done``,
include/mpi/ext_mpi.h:69-89) with integer handles and plain pointers. Buffers are passed as
raw device/host addresses (e.g. ``tensor.data_ptr()``); nothing here computes on the CPU.

There is no fallback: if the native library is missing, importing :func:`lib` raises.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
# EXT_MPI_AMD_LIB: another build of the same library (A/B runs of build options)
LIB_PATH = os.environ.get("EXT_MPI_AMD_LIB") or os.path.join(HERE, "libext_mpi_amd.so")
MPI_LIB_PATH = os.path.join(HERE, "libext_mpi_collectives.so")

DOUBLE, LONG, FLOAT, INT = 0, 1, 2, 3
SUM, MIN, MAX = 0, 1, 2  # element operations (include/ext_mpi_amd.h EXT_MPI_AMD_SUM / _MIN / _MAX)
UNIQUE_ID_BYTES = 128
MAX_RANKS = 16
TUNE_MAX = 8  # include/ext_mpi_amd.h EXT_MPI_AMD_TUNE_MAX
ERRORS = {-1: "ERROR_MALLOC", -2: "ERROR_SHMEM", -3: "ERROR_ARG", -4: "ERROR_UNSUPPORTED",
          -5: "ERROR_DEVICE", -6: "ERROR_TRANSPORT"}
ERROR_MALLOC, ERROR_SHMEM, ERROR_ARG, ERROR_UNSUPPORTED, ERROR_DEVICE, ERROR_TRANSPORT = -1, -2, -3, -4, -5, -6

_TORCH_DTYPE_CODES = {"torch.float32": FLOAT, "torch.float64": DOUBLE, "torch.int32": INT,
                      "torch.int64": LONG}
_NUMPY_DTYPE_CODES = {"float32": FLOAT, "float64": DOUBLE, "int32": INT, "int64": LONG}


class P2P(ctypes.Structure):
    _fields_ = [("leg", ctypes.c_int), ("peer", ctypes.c_int), ("is_send", ctypes.c_int), ("buf", ctypes.c_int),
                ("offset", ctypes.c_long), ("bytes", ctypes.c_long)]


class FoldDesc(ctypes.Structure):
    _fields_ = [("piece", ctypes.c_int), ("offset", ctypes.c_long), ("count", ctypes.c_long),
                ("buf", ctypes.c_int * MAX_RANKS), ("leaf_offset", ctypes.c_long * MAX_RANKS),
                ("nleaf", ctypes.c_int), ("leg", ctypes.c_int)]


BUF_SEND, BUF_RECV, BUF_STAGE = 0, 1, 2

# int (*)(void *ctx, const void *send, void *recv, long bytes) -- include/ext_mpi_amd.h
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long)
_ipc_callbacks = {}  # comm -> the ctypes callback (must outlive the communicator)


class ExtMpiError(RuntimeError):
    def __init__(self, what, code):
        super().__init__(f"{what} failed: {ERRORS.get(code, code)} ({code})")
        self.code = code


def build(with_mpi=True):
    """Compile the native libraries in-tree (hipcc --offload-arch=gfx950)."""
    targets = ["all"] if with_mpi else [os.path.join("..", "libext_mpi_amd.so")]
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(HERE, "csrc")] + targets, check=True)


_lib = None


def lib():
    """The loaded native library. Raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run ext_mpi_collectives_amd.build() "
                              "(the HIP path has no CPU fallback)")
        # One HIP runtime per process: torch's bundled runtime is needed as "libamdhip64.so", this
        # library's as "libamdhip64.so.7" (the SONAME both carry). With torch loaded first the
        # loader reuses its runtime for this library; the other order loads /opt/rocm's copy and
        # torch then loads a second one (two runtimes corrupted the heap at exit on this image).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        c_int, c_long, c_void_p = ctypes.c_int, ctypes.c_long, ctypes.c_void_p
        P = ctypes.POINTER
        L.ext_mpi_amd_node_allreduce_init.argtypes = [c_int, P(c_void_p), P(c_void_p), c_long, c_int, c_int,
                                                      ctypes.c_char_p, P(c_int)]
        L.ext_mpi_amd_node_comm_allreduce_init.argtypes = [c_int, P(c_void_p), P(c_void_p), c_long, c_int, c_int,
                                                           c_int, ctypes.c_char_p, P(c_int)]
        L.ext_mpi_amd_fold_init.argtypes = [c_int, P(c_void_p), c_int, P(c_void_p), c_long, c_int, c_int, P(c_int)]
        L.ext_mpi_amd_get_unique_id.argtypes = [c_void_p]
        L.ext_mpi_amd_comm_init.argtypes = [c_int, c_int, c_void_p, c_int, P(c_int)]
        L.ext_mpi_amd_comm_free.argtypes = [c_int]
        L.ext_mpi_amd_comm_init_loopback.argtypes = [c_int, P(c_int)]
        L.ext_mpi_amd_comm_init_ipc.argtypes = [c_int, c_int, ALLGATHER_FN, c_void_p, c_int, P(c_int)]
        L.ext_mpi_amd_allreduce_init.argtypes = [c_void_p, c_void_p, c_long, c_int, c_int, c_int,
                                                 ctypes.c_char_p, P(c_int)]
        for name in ("start", "test", "wait", "done"):
            getattr(L, "ext_mpi_amd_" + name).argtypes = [c_int]
            getattr(L, "ext_mpi_amd_" + name).restype = c_int
        L.ext_mpi_amd_set_stream.argtypes = [c_int, c_void_p]
        L.ext_mpi_amd_start_legs.argtypes = [c_int, c_int]
        L.ext_mpi_amd_stream.argtypes = [c_int]
        L.ext_mpi_amd_stream.restype = c_void_p
        L.ext_mpi_amd_handle_schedule.argtypes = [c_int, P(c_int), P(c_int), P(c_int)]
        L.ext_mpi_amd_handle_candidates.argtypes = [c_int, P(c_int), P(c_int), c_int]
        L.ext_mpi_amd_handle_tune_info.argtypes = [c_int, c_void_p]
        L.ext_mpi_amd_tune_cache_clear.argtypes = []
        L.ext_mpi_amd_plan_describe.argtypes = [c_int, c_long, c_int, ctypes.c_char_p, c_int, P(c_long),
                                                P(c_long), c_int, P(c_int), P(c_int), P(ctypes.c_ubyte),
                                                P(ctypes.c_ubyte), P(c_int)]
        L.ext_mpi_amd_comm_program.argtypes = [c_int, c_int, c_long, c_int, ctypes.c_char_p, c_long,
                                               P(P2P), c_int, P(c_int), P(FoldDesc), c_int, P(c_int), P(c_long)]
        L.ext_mpi_amd_comm_program_nodes.argtypes = [c_int, c_int, c_int, c_long, c_int, ctypes.c_char_p, c_long,
                                                     P(P2P), c_int, P(c_int), P(FoldDesc), c_int, P(c_int), P(c_long)]
        L.ext_mpi_amd_comm_program_node_ports.argtypes = [c_int, P(c_int), c_int, c_int, c_long, c_int,
                                                          ctypes.c_char_p, c_long, P(P2P), c_int, P(c_int),
                                                          P(FoldDesc), c_int, P(c_int), P(c_long)]
        L.ext_mpi_amd_comm_set_nodes.argtypes = [c_int, c_int]
        L.ext_mpi_amd_comm_set_node_ports.argtypes = [c_int, c_int, P(c_int)]
        L.ext_mpi_amd_set_num_sockets.argtypes = [c_int]
        L.ext_mpi_amd_set_num_sockets.restype = c_int
        L.ext_mpi_amd_version.restype = ctypes.c_char_p
        L.ext_mpi_amd_build_info.restype = ctypes.c_char_p
        L.ext_mpi_amd_handle_join_parts.argtypes = [c_int]
        L.ext_mpi_amd_handle_ipc_flags.argtypes = [c_int]
        L.ext_mpi_amd_gpu_malloc.argtypes = [P(c_void_p), ctypes.c_size_t]
        L.ext_mpi_amd_gpu_free.argtypes = [c_void_p]
        L.ext_mpi_amd_gpu_memcpy_hd.argtypes = [c_void_p, c_void_p, ctypes.c_size_t]
        L.ext_mpi_amd_gpu_memcpy_dh.argtypes = [c_void_p, c_void_p, ctypes.c_size_t]
        _lib = L
    return _lib


def dtype_code(dt):
    """Map a torch/numpy dtype (or its name) to the library's element type code."""
    key = str(dt)
    if key in _TORCH_DTYPE_CODES:
        return _TORCH_DTYPE_CODES[key]
    if key in _NUMPY_DTYPE_CODES:
        return _NUMPY_DTYPE_CODES[key]
    raise ValueError(f"unsupported element type {dt} (float, double, int, long only)")


def _check(what, rc):
    if rc < 0:
        raise ExtMpiError(what, rc)
    return rc


def _enc(copyin):
    return copyin.encode() if copyin else None


def node_allreduce_init(sendptrs, recvptrs, count, dtype, copyin=None, op=SUM):
    """Persistent Allreduce over len(sendptrs) node ranks whose buffers all live in this
    process (device or host addresses). Returns an integer handle."""
    n = len(sendptrs)
    s = (ctypes.c_void_p * n)(*sendptrs)
    r = (ctypes.c_void_p * n)(*recvptrs)
    h = ctypes.c_int(-1)
    _check("ext_mpi_amd_node_allreduce_init",
           lib().ext_mpi_amd_node_allreduce_init(n, s, r, count, dtype, op, _enc(copyin), ctypes.byref(h)))
    return h.value


def node_comm_allreduce_init(sendptrs, recvptrs, count, dtype, comm, copyin=None, op=SUM):
    """Persistent Allreduce over several nodes with every rank of this node in this process
    (len(sendptrs) node ranks, device buffers on this process's GPU) and `comm` having one member
    per node (RCCL or loopback): the NODE form's copy-in, the inter-node legs of every node rank,
    the node's copy-out. Bits equal allreduce_init over size * len(sendptrs) ranks."""
    n = len(sendptrs)
    s = (ctypes.c_void_p * n)(*sendptrs)
    r = (ctypes.c_void_p * n)(*recvptrs)
    h = ctypes.c_int(-1)
    _check("ext_mpi_amd_node_comm_allreduce_init",
           lib().ext_mpi_amd_node_comm_allreduce_init(n, s, r, count, dtype, op, comm, _enc(copyin), ctypes.byref(h)))
    return h.value


def fold_init(srcptrs, dstptrs, count, dtype, op=SUM):
    """Persistent fold of one chunk: every dst = ((src0 + src1) + src2) + ... (device pointers)."""
    s = (ctypes.c_void_p * len(srcptrs))(*srcptrs)
    d = (ctypes.c_void_p * len(dstptrs))(*dstptrs)
    h = ctypes.c_int(-1)
    _check("ext_mpi_amd_fold_init",
           lib().ext_mpi_amd_fold_init(len(srcptrs), s, len(dstptrs), d, count, dtype, op, ctypes.byref(h)))
    return h.value


def get_unique_id():
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    _check("ext_mpi_amd_get_unique_id", lib().ext_mpi_amd_get_unique_id(buf))
    return buf.raw


def comm_init(rank, size, unique_id, device=-1):
    c = ctypes.c_int(-1)
    buf = ctypes.create_string_buffer(bytes(unique_id), UNIQUE_ID_BYTES)
    _check("ext_mpi_amd_comm_init", lib().ext_mpi_amd_comm_init(rank, size, buf, device, ctypes.byref(c)))
    return c.value


def comm_init_loopback(size):
    """Testing transport: one communicator per rank, all in this process on the current device."""
    comms = (ctypes.c_int * size)()
    _check("ext_mpi_amd_comm_init_loopback", lib().ext_mpi_amd_comm_init_loopback(size, comms))
    return list(comms)


def comm_init_ipc(rank, size, allgather, device=-1):
    """Peer-mapped communicator (hipIpc over xGMI): one rank per GPU, or several processes on one.

    ``allgather(payload: bytes) -> list[bytes]`` must return every rank's payload in rank order
    (a bootstrap exchange, called collectively at communicator and handle set-up only)."""
    def _cb(ctx, send, recv, nbytes):
        try:
            parts = allgather(ctypes.string_at(send, nbytes))
            blob = b"".join(bytes(x) for x in parts)
            if len(parts) != size or len(blob) != nbytes * size:
                return -1
            ctypes.memmove(recv, blob, len(blob))
            return 0
        except Exception:  # noqa: BLE001 -- reported to the C side as a transport failure
            return -1
    cb = ALLGATHER_FN(_cb)
    c = ctypes.c_int(-1)
    _check("ext_mpi_amd_comm_init_ipc", lib().ext_mpi_amd_comm_init_ipc(rank, size, cb, None, device, ctypes.byref(c)))
    _ipc_callbacks[c.value] = cb
    return c.value


def torch_allgather(group=None):
    """Bootstrap exchange for :func:`comm_init_ipc` over an initialised torch.distributed group."""
    import torch.distributed as dist

    def ag(payload):
        out = [None] * dist.get_world_size(group)
        dist.all_gather_object(out, payload, group=group)
        return out
    return ag


def comm_free(comm):
    _check("ext_mpi_amd_comm_free", lib().ext_mpi_amd_comm_free(comm))
    _ipc_callbacks.pop(comm, None)


def allreduce_init(sendptr, recvptr, count, dtype, comm, copyin=None, op=SUM):
    """Persistent Allreduce of this rank's buffer over a communicator (one rank per GPU)."""
    h = ctypes.c_int(-1)
    _check("ext_mpi_amd_allreduce_init",
           lib().ext_mpi_amd_allreduce_init(sendptr, recvptr, count, dtype, op, comm, _enc(copyin), ctypes.byref(h)))
    return h.value


def start(h):
    return _check("ext_mpi_amd_start", lib().ext_mpi_amd_start(h))


def test(h):
    return _check("ext_mpi_amd_test", lib().ext_mpi_amd_test(h))


def wait(h):
    return _check("ext_mpi_amd_wait", lib().ext_mpi_amd_wait(h))


def done(h):
    return _check("ext_mpi_amd_done", lib().ext_mpi_amd_done(h))


LEG_STAGE_IN, LEG_REDUCE_SCATTER, LEG_FOLD, LEG_ALLGATHER, LEG_STAGE_OUT = 1, 2, 4, 8, 16
LEG_NODES_RS, LEG_NODES_FOLD, LEG_NODES_AG = 32, 64, 128  # 2^k nodes (comm_set_nodes), per step
LEG_STAGE, LEG_ALL = 17, 255
LEG_STEP_SHIFT = 8  # node legs / folds carry their step: leg | step << 8


def LEG_STEP(s):
    """start_legs selector: the node legs of step s alone (loopback lock-step)"""
    return (s + 1) << LEG_STEP_SHIFT


def node_shares(nodes, ports, ranks_per_node, count, dtype, copyin, me, max_shares=4096):
    """The parts of node rank `me`'s chunk the peer-mapped node join folds: (levels, list of
    (off, len, folding node, [leaf nodes in fold order])) -- levels 1: a left fold of the leaves,
    k: k levels of pairs of consecutive leaves (ext_mpi_amd_node_shares)."""
    off = (ctypes.c_long * max_shares)()
    ln = (ctypes.c_long * max_shares)()
    nd = (ctypes.c_int * max_shares)()
    lv = (ctypes.c_int * (max_shares * nodes))()
    n, levels = ctypes.c_int(0), ctypes.c_int(1)
    _check("ext_mpi_amd_node_shares", lib().ext_mpi_amd_node_shares(nodes, _ports(ports), ranks_per_node, count, dtype,
                                                                       _enc(copyin), me, off, ln, nd, lv, max_shares,
                                                                       ctypes.byref(n), ctypes.byref(levels)))
    return levels.value, [(off[i], ln[i], nd[i], list(lv[i * nodes:(i + 1) * nodes])) for i in range(n.value)]


def default_node_ports(nodes):
    """The inter-node ports list without EXT_MPI_NUM_PORTS (plan.c emac_node_sched_build): one
    port per step for a power of two, else one step of radix `nodes` up to 16 nodes, else one
    step per prime factor, largest first (the allgather steps in reverse)."""
    k = (nodes - 1).bit_length()
    if 1 << k == nodes:
        return [-1] * k + [1] * k
    if nodes <= MAX_RANKS:
        return [-(nodes - 1), nodes - 1]
    f, m = [], nodes
    for d in range(MAX_RANKS, 1, -1):
        while m % d == 0 and all(d % q for q in range(2, int(d ** 0.5) + 1)):
            f.append(d)
            m //= d
    if m != 1:  # a prime factor above MAX_RANKS: plan.c emac_node_sched_build refuses it (UNSUPPORTED)
        raise ValueError(f"{nodes} nodes: prime factor {m} > {MAX_RANKS} leaves per step")
    return [1 - d for d in f] + [d - 1 for d in reversed(f)]


def node_steps(nodes, ports=None):
    """(exchange steps, copying allgather steps) of the inter-node schedule (plan.h
    emac_node_sched): the reduce-scatter steps and the allgather steps that still reduce inside
    the groups they leave, then the allgather steps that copy. ports None: one port per step
    for a power of two, else one step of radix `nodes`."""
    if nodes <= 1:
        return 0, 0
    if ports is None:
        ports = default_node_ports(nodes)
    rs = [1 - p for p in ports if p < 0]
    ag = [p + 1 for p in ports if p > 0]
    gm = nodes
    for r in rs:
        gm //= r
    g, nred = 1, 0
    while g < gm:
        g *= ag[nred]
        nred += 1
    return len(rs) + nred, len(ag) - nred


def lockstep_legs(nodes=1, ports=None):
    """The legs of one Start in the order a lock-step driver runs them on every rank: stage-in,
    reduce-scatter, fold, per node exchange step the line exchange and its fold, the copying
    allgather steps, allgather, stage-out. `ports`: the inter-node list (see node_steps)."""
    nx, na = node_steps(nodes, ports)
    legs = [LEG_STAGE_IN, LEG_REDUCE_SCATTER, LEG_FOLD]
    for st in range(nx):
        legs += [LEG_NODES_RS | LEG_STEP(st), LEG_NODES_FOLD | LEG_STEP(st)]
    legs += [LEG_NODES_AG | LEG_STEP(j) for j in range(na)]
    return legs + [LEG_ALLGATHER, LEG_STAGE_OUT]


def start_legs(h, legs):
    return _check("ext_mpi_amd_start_legs", lib().ext_mpi_amd_start_legs(h, legs))


def set_stream(h, stream_ptr):
    return _check("ext_mpi_amd_set_stream", lib().ext_mpi_amd_set_stream(h, stream_ptr))


def stream(h):
    """hipStream_t (as int) the handle's work runs on."""
    return lib().ext_mpi_amd_stream(h)


def handle_schedule(h):
    """The fold's launch schedule: dict(unroll, issue, tuned) -- tuned 1 when the handle's first
    Starts measured the candidates and kept the fastest, 0 while measuring, -1 untuned."""
    u, i, t = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _check("ext_mpi_amd_handle_schedule", lib().ext_mpi_amd_handle_schedule(h, ctypes.byref(u), ctypes.byref(i),
                                                                           ctypes.byref(t)))
    return {"unroll": u.value, "issue": i.value, "tuned": t.value}


def handle_candidates(h):
    """The schedules the tuner measures on the handle's first Starts: [(unroll, issue)], [] untuned."""
    n, sched = ctypes.c_int(), (ctypes.c_int * 16)()
    _check("ext_mpi_amd_handle_candidates", lib().ext_mpi_amd_handle_candidates(h, ctypes.byref(n), sched, 16))
    return [(sched[k] & 15, sched[k] >> 4) for k in range(min(n.value, 16))]


class TuneInfo(ctypes.Structure):
    """include/ext_mpi_amd.h ext_mpi_amd_tune_info"""
    _fields_ = [("candidates", ctypes.c_int), ("chosen", ctypes.c_int), ("cached", ctypes.c_int),
                ("isolated", ctypes.c_int), ("starts", ctypes.c_int), ("timed_starts_per_sample", ctypes.c_int),
                ("samples", ctypes.c_int), ("schedule", ctypes.c_int * TUNE_MAX), ("us", ctypes.c_float * TUNE_MAX),
                ("ops_in_sample", ctypes.c_int * (TUNE_MAX * 3))]


def handle_tune_info(h):
    """The tuner's state of a handle: dict(candidates, chosen, cached, isolated, starts,
    timed_starts_per_sample, schedules=[(unroll, issue)], us=[per candidate], ops_in_sample=[...])."""
    t = TuneInfo()
    _check("ext_mpi_amd_handle_tune_info", lib().ext_mpi_amd_handle_tune_info(h, ctypes.byref(t)))
    n = min(t.candidates, TUNE_MAX)
    return {"candidates": t.candidates, "chosen": t.chosen, "cached": t.cached, "isolated": t.isolated,
            "starts": t.starts, "timed_starts_per_sample": t.timed_starts_per_sample, "samples": t.samples,
            "schedules": [(t.schedule[k] & 15, t.schedule[k] >> 4) for k in range(n)],
            "us": [round(t.us[k], 3) for k in range(n)],
            "ops_in_sample": list(t.ops_in_sample[:min(t.samples, TUNE_MAX * 3)])}


def tune_cache_clear():
    """Forget every kept fold schedule of this process; returns the number of entries dropped."""
    return lib().ext_mpi_amd_tune_cache_clear()


def plan_describe(nranks, count, dtype, copyin, pos, max_pieces=4096):
    """Fold schedule of owner position ``pos`` (no GPU needed).

    Returns dict(owner, pieces=[(off, len)], leaves=[node ranks in fold order],
    first=[...], close=[...], nlev)."""
    off = (ctypes.c_long * max_pieces)()
    ln = (ctypes.c_long * max_pieces)()
    owner = ctypes.c_int()
    leaves = (ctypes.c_int * MAX_RANKS)()
    first = (ctypes.c_ubyte * MAX_RANKS)()
    close = (ctypes.c_ubyte * MAX_RANKS)()
    nlev = ctypes.c_int()
    n = _check("ext_mpi_amd_plan_describe",
               lib().ext_mpi_amd_plan_describe(nranks, count, dtype, _enc(copyin), pos, off, ln, max_pieces,
                                                ctypes.byref(owner), leaves, first, close, ctypes.byref(nlev)))
    return {"owner": owner.value, "pieces": [(off[i], ln[i]) for i in range(min(n, max_pieces))],
            "leaves": list(leaves[:nranks]), "first": list(first[:nranks]), "close": list(close[:nranks]),
            "nlev": nlev.value}


def comm_program(nranks, rank, count, dtype, copyin=None, send_phase=0, max_ops=65536, max_folds=4096):
    """What Start executes for node rank ``rank`` in the COMM form (no GPU needed).

    Returns (ops, folds, staging_bytes): ops = [(leg, peer, is_send, buf, offset, bytes)],
    folds = [(offset, count, [(buf, leaf_offset)] in fold order)]."""
    o, f, stage = comm_program_nodes(1, nranks, rank, count, dtype, copyin, send_phase, max_ops, max_folds)
    return o, [(off, n, leaves) for off, n, leaves, _ in f], stage


def _ports(ports):
    """The reference's 0-terminated num_ports list (None: NULL, the default schedule)."""
    return None if ports is None else (ctypes.c_int * (len(ports) + 1))(*ports, 0)


def comm_program_nodes(nodes, ranks_per_node, rank, count, dtype, copyin=None, send_phase=0, max_ops=65536,
                       max_folds=4096, ports=None):
    """comm_program over ``nodes`` nodes under the inter-node ports list ``ports`` (None: one port
    per step, 2^k nodes); ``rank`` is global (node-major). Folds are (offset, count,
    [(buf, leaf_offset)], leg) with leg LEG_FOLD (the node's fold) or LEG_NODES_FOLD | step << 8
    (the kept lines' partials in the reference's accumulator order)."""
    ops = (P2P * max_ops)()
    folds = (FoldDesc * max_folds)()
    nops, nf, stage = ctypes.c_int(), ctypes.c_int(), ctypes.c_long()
    _check("ext_mpi_amd_comm_program_node_ports",
           lib().ext_mpi_amd_comm_program_node_ports(nodes, _ports(ports), ranks_per_node, rank, count, dtype,
                                                     _enc(copyin), send_phase, ops, max_ops, ctypes.byref(nops), folds,
                                                     max_folds, ctypes.byref(nf), ctypes.byref(stage)))
    o = [(x.leg, x.peer, x.is_send, x.buf, x.offset, x.bytes) for x in ops[:nops.value]]
    f = [(x.offset, x.count, [(x.buf[t], x.leaf_offset[t]) for t in range(x.nleaf)], x.leg) for x in folds[:nf.value]]
    return o, f, stage.value


def comm_set_nodes(comm, nodes, ports=None):
    """Declare the ranks of an RCCL / loopback communicator `nodes` nodes of size / nodes
    consecutive ranks each, under the inter-node ports list `ports` (the reference's
    EXT_MPI_NUM_PORTS, e.g. [-2, 2] for 3 nodes; None: one port per step for a power of two,
    else one step of radix `nodes`)."""
    return _check("ext_mpi_amd_comm_set_node_ports", lib().ext_mpi_amd_comm_set_node_ports(comm, nodes, _ports(ports)))


def set_num_sockets(sockets):
    """EXT_MPI_NUM_SOCKETS_PER_NODE for every handle / plan made afterwards; returns the previous
    value. Sockets move the tree method's (7 / 10) last-step roots, nothing else."""
    return _check("ext_mpi_amd_set_num_sockets", lib().ext_mpi_amd_set_num_sockets(sockets))


class num_sockets:
    """``with num_sockets(2): ...`` -- set_num_sockets for the block, restored after."""

    def __init__(self, sockets):
        self.sockets = sockets

    def __enter__(self):
        self.prev = set_num_sockets(self.sockets)
        return self

    def __exit__(self, *exc):
        set_num_sockets(self.prev)
        return False


def version():
    return lib().ext_mpi_amd_version().decode()


def build_info():
    """The loaded library's build stamp: {"sha": commit[+dirty], "src": source hash} (_stamp.py)."""
    from . import _stamp
    return _stamp.parse(lib().ext_mpi_amd_build_info().decode())


def check_build():
    """The loaded library's stamp against the sources beside it. Returns the stamp dict with "tree"
    (this tree's source hash) and "match"; raises if the binary was built from other sources."""
    from . import _stamp
    info = build_info()
    info["tree"] = _stamp.source_hash()
    info["match"] = info.get("src") == info["tree"]
    if not info["match"]:
        raise RuntimeError(f"{LIB_PATH} was built from sources {info.get('src')}, this tree's are {info['tree']}: "
                           "rebuild it (make -C ext_mpi_collectives_amd/csrc)")
    return info


def handle_join_parts(h):
    """The parts a peer-mapped node join is pipelined by (1: serial), 0 for other handles."""
    n = lib().ext_mpi_amd_handle_join_parts(h)
    _check("ext_mpi_amd_handle_join_parts", min(n, 0))
    return n


IPC_CROSS_DEVICE, IPC_RELEASE_EVENT, IPC_SYS_STORES, IPC_DEV_STORES = 1, 2, 4, 8


def handle_ipc_flags(h):
    """A peer-mapped handle's cross-GPU settings (IPC_* bits, include/ext_mpi_amd.h), 0 for others."""
    n = lib().ext_mpi_amd_handle_ipc_flags(h)
    _check("ext_mpi_amd_handle_ipc_flags", min(n, 0))
    return n
