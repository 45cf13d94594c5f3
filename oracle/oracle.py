"""ctypes front-end of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this
module. It loads ``oracle/liboracle.so`` (built by ``oracle/Makefile``), a C restatement of the
reference's copy-in schedules -- method 6 recursive (src/core/reduce_copyin.c:674-842), 5 cyclic
(:531-634), 7 tree (:844-968), 8-10 the same on a staging copy, with :375-427, :482-486,
:970-1084, :1418-1681 around them -- of the buffer-table rotation (src/mpi/ext_mpi_xpmem.c:114-130)
and of its SUM/MIN/MAX loops (src/mpi/ext_mpi_native_exec.c:207-318).
See oracle/ref_oracle.h for the per-function citations.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

# element type codes (ref_oracle.h)
DOUBLE, LONG, FLOAT, INT, CHAR = 0, 1, 2, 3, 4
SUM, MIN, MAX = 0, 1, 2  # element operations (ref_oracle.h REF_RED_*)
NP_DTYPE = {DOUBLE: np.float64, LONG: np.int64, FLOAT: np.float32, INT: np.int32, CHAR: np.int8}
BY_NAME = {"double": DOUBLE, "f64": DOUBLE, "long": LONG, "int64": LONG, "float": FLOAT,
           "f32": FLOAT, "int": INT, "int32": INT}

OP_COPY, OP_SUM, OP_PHASE = 0, 1, 2
BUF_RECV, BUF_SEND = 0, 1


class RefOp(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int), ("dbuf", ctypes.c_int), ("drel", ctypes.c_int),
                ("doff", ctypes.c_long), ("sbuf", ctypes.c_int), ("srel", ctypes.c_int),
                ("soff", ctypes.c_long), ("bytes", ctypes.c_long)]


_lib = None


def build():
    """Compile liboracle.so with the oracle's own Makefile (gcc -O3 -fPIC)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.ref_schedule.restype = ctypes.c_int
        _lib.ref_schedule.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.POINTER(RefOp), ctypes.c_int]
        _lib.ref_emulate.restype = ctypes.c_int
        _lib.ref_emulate.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_char_p,
                                     ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                     ctypes.POINTER(ctypes.c_void_p)]
        _lib.ref_emulate_op.restype = ctypes.c_int
        _lib.ref_emulate_op.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                        ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                        ctypes.POINTER(ctypes.c_void_p)]
        _lib.ref_sizes_displs.restype = None
        _lib.ref_sizes_displs.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_long,
                                          ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_long)]
        _lib.ref_rank_order.restype = None
        _lib.ref_rank_order.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_int)]
        _lib.ref_parse_copyin.restype = ctypes.c_int
        _lib.ref_parse_copyin.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                          ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        _lib.ref_kat_fill.restype = None
        _lib.ref_kat_fill.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_long]
        _lib.ref_reduction.restype = None
        _lib.ref_reduction.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
        _lib.ref_cpu_allreduce_threads.restype = ctypes.c_double
        _lib.ref_cpu_allreduce_threads.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_int,
                                                   ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p),
                                                   ctypes.POINTER(ctypes.c_void_p), ctypes.c_long]
        _lib.ref_emulate_op_s.restype = ctypes.c_int
        _lib.ref_emulate_op_s.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                          ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                          ctypes.POINTER(ctypes.c_void_p)]
        _lib.ref_emulate_nodes.restype = ctypes.c_int
        _lib.ref_emulate_nodes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                           ctypes.POINTER(ctypes.c_void_p)]
        _lib.ref_emulate_node_ports.restype = ctypes.c_int
        _lib.ref_emulate_node_ports.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_long,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p)]
        _lib.ref_get_rank_cyclic.restype = ctypes.c_int
        _lib.ref_get_rank_cyclic.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                             ctypes.c_int]
        _lib.ref_decode_peer.restype = ctypes.c_int
        _lib.ref_decode_peer.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        _lib.ref_cpu_allreduce_threads_sets.restype = ctypes.c_double
        _lib.ref_cpu_allreduce_threads_sets.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_char_p,
                                                        ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                                        ctypes.POINTER(ctypes.c_void_p), ctypes.c_long]
    return _lib


def parse_copyin(s):
    method = ctypes.c_int()
    factors = (ctypes.c_int * 64)()
    n = lib().ref_parse_copyin(s.encode(), ctypes.byref(method), factors, 64)
    if n < 0:
        raise ValueError(f"bad copyin string {s!r}")
    return method.value, list(factors[:n])


def sizes_displs(R, nbytes, tsize, size_l=0):
    sizes = (ctypes.c_long * R)()
    displs = (ctypes.c_long * (R + 1))()
    lib().ref_sizes_displs(R, nbytes, tsize, size_l, sizes, displs)
    return list(sizes), list(displs)


def rank_order(R, factors):
    ranks = (ctypes.c_int * R)(*range(R))
    f = (ctypes.c_int * max(1, len(factors)))(*factors)
    lib().ref_rank_order(R, len(factors), f, ranks)
    return list(ranks)


def schedule(R, node_rank, nbytes, dtype, copyin, in_place=False, stage=1):
    """Program of one rank: list of (op, dbuf, drel, doff, sbuf, srel, soff, bytes)."""
    _, factors = parse_copyin(copyin)
    f = (ctypes.c_int * len(factors))(*factors)
    cap = 16 * R * (R + 8) * max(1, factors[0]) + 256
    out = (RefOp * cap)()
    n = lib().ref_schedule(R, node_rank, nbytes, dtype, f, len(factors), int(in_place), stage, out, cap)
    if n < 0:
        raise ValueError(f"unsupported schedule {copyin!r} for R={R}")
    return [(o.op, o.dbuf, o.drel, o.doff, o.sbuf, o.srel, o.soff, o.bytes) for o in out[:n]]


def _ptrs(arrays):
    return (ctypes.c_void_p * len(arrays))(*[a.ctypes.data for a in arrays])


def allreduce(sends, copyin, in_place=False, op=SUM, num_sockets=1):
    """Reference result of an R-rank Allreduce(op: SUM, MIN or MAX) of the host arrays ``sends``
    (copy-in methods 5-10 of the reference's single-node generators, num_sockets per node).

    Returns the list of R receive arrays (all equal for a correct schedule).
    """
    R = len(sends)
    a0 = np.ascontiguousarray(sends[0])
    code = {np.dtype(np.float64): DOUBLE, np.dtype(np.int64): LONG, np.dtype(np.float32): FLOAT,
            np.dtype(np.int32): INT}[a0.dtype]
    sends = [np.ascontiguousarray(s) for s in sends]
    if in_place:
        recvs = [s.copy() for s in sends]
    else:
        recvs = [np.full_like(s, -1) for s in sends]
    rc = lib().ref_emulate_op_s(R, a0.size, code, op, copyin.encode(), int(in_place), num_sockets, _ptrs(sends),
                                _ptrs(recvs))
    if rc != 0:
        raise ValueError(f"oracle rejected copyin {copyin!r} for R={R}")
    return recvs


def allreduce_nodes(sends, copyin, nodes=2, in_place=False, op=SUM, num_sockets=1, ports=None):
    """Reference result over `nodes` nodes of len(sends) // nodes ranks each (node-major): each
    node's copy-in, allreduce_core over the node partials under `ports` (the EXT_MPI_NUM_PORTS
    list, e.g. [-2, 2] for 3 nodes; None: one port per step, 2^k nodes), the copy-out."""
    W = len(sends)
    a0 = np.ascontiguousarray(sends[0])
    code = {np.dtype(np.float64): DOUBLE, np.dtype(np.int64): LONG, np.dtype(np.float32): FLOAT,
            np.dtype(np.int32): INT}[a0.dtype]
    sends = [np.ascontiguousarray(s) for s in sends]
    recvs = [s.copy() for s in sends] if in_place else [np.full_like(s, -1) for s in sends]
    if ports is None:
        rc = lib().ref_emulate_nodes(nodes, W // nodes, a0.size, code, op, copyin.encode(), int(in_place),
                                     num_sockets, _ptrs(sends), _ptrs(recvs))
    else:
        pl = (ctypes.c_int * (len(ports) + 1))(*ports, 0)
        rc = lib().ref_emulate_node_ports(nodes, pl, W // nodes, a0.size, code, op, copyin.encode(), int(in_place),
                                          num_sockets, _ptrs(sends), _ptrs(recvs))
    if rc != 0:
        raise ValueError(f"oracle rejected copyin {copyin!r} for {nodes} x {W // nodes}")
    return recvs


def kat_fill(count, dtype_code, world_rank, add):
    """Known-answer input of debug_persistent.c:491-497 (add=73) / :426-432 (add=0)."""
    tsize = np.dtype(NP_DTYPE[dtype_code]).itemsize
    buf = np.zeros(count, dtype=NP_DTYPE[dtype_code])
    lib().ref_kat_fill(buf.ctypes.data, count, tsize, world_rank, add)
    return buf


def cpu_allreduce_threads(sends, recvs, copyin, iters):
    """Run the threaded CPU baseline `iters` times; returns elapsed seconds."""
    R = len(sends)
    code = {np.dtype(np.float64): DOUBLE, np.dtype(np.int64): LONG, np.dtype(np.float32): FLOAT,
            np.dtype(np.int32): INT}[sends[0].dtype]
    t = lib().ref_cpu_allreduce_threads(R, sends[0].size, code, copyin.encode(), _ptrs(sends),
                                        _ptrs(recvs), iters)
    if t < 0:
        raise ValueError("cpu baseline failed")
    return t


def cpu_allreduce_threads_sets(sets, copyin, iters):
    """The threaded CPU baseline over rotated buffer sets: `sets` is a list of (sends, recvs)
    pairs of R arrays each; iteration i runs on set i % len(sets). Returns elapsed seconds."""
    R = len(sets[0][0])
    code = {np.dtype(np.float64): DOUBLE, np.dtype(np.int64): LONG, np.dtype(np.float32): FLOAT,
            np.dtype(np.int32): INT}[sets[0][0][0].dtype]
    sends = [a for s, _ in sets for a in s]
    recvs = [a for _, r in sets for a in r]
    t = lib().ref_cpu_allreduce_threads_sets(R, sets[0][0][0].size, code, copyin.encode(), len(sets), _ptrs(sends),
                                             _ptrs(recvs), iters)
    if t < 0:
        raise ValueError("cpu baseline failed")
    return t


def get_rank_cyclic(num_sockets, R, ranks, me_pos, other_pos):
    """reduce_copyin.c:482-486: the buffer-table index of position other_pos seen from me_pos."""
    arr = (ctypes.c_int * R)(*ranks)
    return lib().ref_get_rank_cyclic(num_sockets, R, arr, me_pos, other_pos)


def decode_peer(num_sockets, R, me, index):
    """ext_mpi_xpmem.c:114-130: node rank whose buffer sits at table index `index` of node rank me."""
    return lib().ref_decode_peer(num_sockets, R, me, index)
