"""GPU parity of the HIP path (called through the C ABI) against the CPU oracle.

Bar (BASELINE.json north_star): bit-exact for int / long; float / double must match the
reference CPU path within (R-1)*u*sum|x| -- the implementation keeps the reference's
per-element operation order, so the tests assert 0 ulp (bitwise equality) for every type.
"""
import ctypes

import numpy as np
import pytest

import ext_mpi_collectives_amd as emac
from helpers import NP, xorshift_inputs

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TORCH = {emac.FLOAT: torch.float32, emac.DOUBLE: torch.float64, emac.INT: torch.int32, emac.LONG: torch.int64}
TUNE_STARTS = 1 + 3 * 3 * emac.TUNE_MAX + 1  # enough Starts for any handle's tuning to keep a schedule
TUNE_1 = 1 + 3 * 3 + 1  # ... for a handle with one candidate (a forced schedule word)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    emac.lib()


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def run_node(sends, code, copyin, in_place=False, repeats=1, op=emac.SUM):
    """Node-form Allreduce of host arrays `sends` on device buffers; returns host results."""
    R = len(sends)
    count = sends[0].size
    dsend = [_dev(s) for s in sends]
    drecv = dsend if in_place else [torch.full((count,), -1, dtype=TORCH[code], device="cuda") for _ in range(R)]
    h = emac.node_allreduce_init([t.data_ptr() for t in dsend], [t.data_ptr() for t in drecv], count, code, copyin,
                                 op=op)
    try:
        for _ in range(repeats):
            if in_place:
                for t, s in zip(drecv, sends):
                    t.copy_(torch.from_numpy(s))
            torch.cuda.synchronize()
            emac.start(h)
            emac.wait(h)
    finally:
        emac.done(h)
    return [t.cpu().numpy() for t in drecv]


def assert_bitwise(got, want, what=""):
    for g, w in zip(got, want):
        if not np.array_equal(g.view(np.uint8), w.view(np.uint8)):
            bad = np.nonzero(g.view(np.uint8) != w.view(np.uint8))[0]
            raise AssertionError(f"{what}: {bad.size} differing bytes, first at byte {bad[0]}")


CONFIGS = [
    (2, "6;1 -2 2"), (3, "6;1 -3 3"), (4, "6;1 -4 4"), (4, "6;1 -2 -2 2 2"), (6, "6;1 -2 -3 3 2"),
    (8, "6;1 -8 8"), (8, "6;1 -2 -2 -2 2 2 2"), (8, "6;1 -4 -2 2 4"), (8, "6;-64 -8 8"), (8, "6;3 -8 8"),
    (8, "9;1 -8 8"), (12, "6;1 -3 -4 4 3"), (16, "6;1 -16 16"), (16, "6;1 -2 -2 -2 -2 2 2 2 2"),
    # "1 <members>" sub-splits (two-level trees, reduce_copyin.c:970-1084)
    (8, "6;1 -4 4 1 4 1 -2 2"), (8, "6;-3 -2 -2 2 2 1 4 2 -2 2"), (16, "6;1 -4 4 1 4 1 -2 -2 2 2"),
]
CODES = [emac.FLOAT, emac.DOUBLE, emac.INT, emac.LONG]


@pytest.mark.parametrize("R,copyin", CONFIGS)
@pytest.mark.parametrize("code", CODES)
def test_node_parity_vs_oracle(oracle, R, copyin, code):
    for count in (0, 1, 5, 1031, 65536 + 3):
        sends = xorshift_inputs(R, count, code, seed_base=0x5EED0000 + count)
        want = oracle.allreduce(sends, copyin)
        got = run_node(sends, code, copyin)
        assert_bitwise(got, want, f"R={R} {copyin} code={code} n={count}")


# copy-in methods 5 cyclic / 7 tree (8 / 10 staged aliases) and sockets per node (the tree's roots)
METHOD_CONFIGS = [
    (4, "5;1 -4 4", 1), (6, "5;1 -2 -3 3 2", 1), (8, "5;1 -2 -2 -2 2 2 2", 2), (8, "5;1 -4 -2 2 4", 1),
    (8, "8;3 -8 8", 1), (16, "5;1 -4 -4 4 4", 4),
    (4, "7;1 -4 4", 2), (6, "7;1 -2 -3 3 2", 3), (8, "7;1 -2 -2 -2 2 2 2", 2), (8, "7;1 -2 -4 4 2", 4),
    (8, "7;1 -4 -2 2 4", 1), (8, "10;-64 -8 8", 1), (12, "7;1 -3 -4 4 3", 4), (16, "7;1 -4 -4 4 4", 2),
]


@pytest.mark.parametrize("R,copyin,sockets", METHOD_CONFIGS)
@pytest.mark.parametrize("code", CODES)
def test_node_methods_vs_oracle(oracle, R, copyin, sockets, code):
    for count in (0, 1, 5, 1031, 65536 + 3):
        sends = xorshift_inputs(R, count, code, seed_base=0x5EED7000 + count)
        want = oracle.allreduce(sends, copyin, num_sockets=sockets)
        with emac.num_sockets(sockets):
            got = run_node(sends, code, copyin)
        assert_bitwise(got, want, f"R={R} {copyin} sockets={sockets} code={code} n={count}")


@pytest.mark.parametrize("R,copyin,sockets", [(8, "7;1 -2 -4 4 2", 4), (8, "5;1 -4 -2 2 4", 1),
                                              (6, "7;1 -3 -2 2 3", 2)])
def test_comm_loopback_methods_vs_oracle(oracle, R, copyin, sockets):
    for code in (emac.FLOAT, emac.DOUBLE):
        for count in (1, 1031, 65536 + 5):
            sends = xorshift_inputs(R, count, code, seed_base=0xC0A70000 + count)
            want = oracle.allreduce(sends, copyin, num_sockets=sockets)
            with emac.num_sockets(sockets):
                got = run_comm_loopback(sends, code, copyin, phase=[(r * 3) % 4 for r in range(R)])
            assert_bitwise(got, want, f"comm R={R} {copyin} sockets={sockets} code={code} n={count}")


def test_methods_full_size_random_double(oracle):
    """configs[3]-sized (256 MiB per rank, random doubles) tree with two sockets and cyclic
    methods: bit-exact against the oracle's emulation of the same generator."""
    rng = np.random.default_rng(0x7EE)
    count = 32 << 20
    sends = [rng.standard_normal(count) for _ in range(8)]
    for copyin, sockets in (("7;1 -2 -4 4 2", 2), ("5;1 -8 8", 1)):
        want = oracle.allreduce(sends, copyin, num_sockets=sockets)
        with emac.num_sockets(sockets):
            got = run_node(sends, emac.DOUBLE, copyin)
        assert_bitwise(got, want, f"{copyin} sockets={sockets}")
        del want, got


@pytest.mark.parametrize("code", CODES)
def test_node_in_place(oracle, code):
    sends = xorshift_inputs(8, 100003, code)
    want = oracle.allreduce(sends, "6;1 -8 8", in_place=True)
    assert_bitwise(run_node(sends, code, "6;1 -8 8", in_place=True, repeats=2), want, "in place")


def test_node_known_answer_fixtures():
    import glob
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    for path in sorted(glob.glob(os.path.join(here, "golden", "kat_*.npz"))):
        f = np.load(path)
        R, count, itemsize, _ = (int(x) for x in f["meta"])
        code = emac.INT if itemsize == 4 else emac.LONG
        for copyin in (f"6;1 -{R} {R}", None):
            got = run_node(list(f["inputs"]), code, copyin)
            for g in got:
                assert np.array_equal(g, f["expected"]), path


def test_host_buffers_staged(oracle):
    """The path starts and ends in host memory (XPMEM-mapped buffers in the reference)."""
    R, count = 4, 300007
    sends = xorshift_inputs(R, count, emac.FLOAT)
    recvs = [np.full(count, -1, dtype=np.float32) for _ in range(R)]
    h = emac.node_allreduce_init([s.ctypes.data for s in sends], [r.ctypes.data for r in recvs], count, emac.FLOAT,
                                 "6;1 -4 4")
    try:
        for _ in range(2):
            emac.start(h)
            emac.wait(h)
    finally:
        emac.done(h)
    assert_bitwise(recvs, oracle.allreduce(sends, "6;1 -4 4"), "host staged")


@pytest.mark.parametrize("direct", ["1", "0"])
@pytest.mark.parametrize("code,R,count,copyin,in_place,elem_off", [
    (emac.FLOAT, 4, 300007, "6;1 -4 4", False, 0),
    (emac.FLOAT, 8, 16384, "6;1 -2 -2 -2 2 2 2", True, 0),
    (emac.DOUBLE, 3, 100003, "6;3 -3 3", False, 1),                # views 8 bytes into the pinned block
    (emac.INT, 4, 1 << 20, "6;-64 -4 4", False, 3),                # 12 bytes in: element-granular edges
    (emac.LONG, 8, 5, "6;1 -8 8", True, 0)])
def test_pinned_host_buffers(oracle, monkeypatch, direct, code, R, count, copyin, in_place, elem_off):
    """Page-locked host buffers (torch pin_memory) in the NODE form: read and written by the fold
    kernel over PCIe (default), or staged through device mirrors (EXT_MPI_AMD_HOST_DIRECT=0).
    Views that start inside a pinned block check that the device address keeps the offset."""
    monkeypatch.setenv("EXT_MPI_AMD_HOST_DIRECT", direct)
    sends = xorshift_inputs(R, count, code, seed_base=0x7107 + count)
    blocks_s = [torch.empty(count + elem_off, dtype=TORCH[code]).pin_memory() for _ in range(R)]
    blocks_r = blocks_s if in_place else [torch.empty(count + elem_off, dtype=TORCH[code]).pin_memory()
                                          for _ in range(R)]
    ts = [b[elem_off:] for b in blocks_s]
    tr = [b[elem_off:] for b in blocks_r]
    h = emac.node_allreduce_init([t.data_ptr() for t in ts], [t.data_ptr() for t in tr], count, code, copyin)
    try:
        for _ in range(2):
            for t, s in zip(ts, sends):
                t.copy_(torch.from_numpy(s))
            if not in_place:
                for t in tr:
                    t.fill_(-1)
            emac.start(h)
            emac.wait(h)
            assert_bitwise([t.numpy() for t in tr], oracle.allreduce(sends, copyin, in_place=in_place),
                           f"pinned host direct={direct}")
            if not in_place:  # the send buffers are read only
                assert_bitwise([t.numpy() for t in ts], sends, "pinned send buffers unchanged")
    finally:
        emac.done(h)


@pytest.mark.parametrize("code,R,count,copyin,in_place", [
    (emac.FLOAT, 8, (4 << 20) + 7, "6;1 -8 8", False),
    (emac.DOUBLE, 4, (1 << 20) + 1001, "6;1 -2 -2 2 2", True),
    (emac.INT, 3, 3 << 20, "6;3 -3 3", False),                    # three pieces per chunk
    (emac.LONG, 8, 1 << 20, "6;-64 -8 8", False)])
def test_host_buffers_staged_large(oracle, monkeypatch, code, R, count, copyin, in_place):
    """Host buffers of >= 4 MiB per rank staged through device mirrors (EXT_MPI_AMD_HOST_DIRECT=0:
    H2D, fold, D2H on the handle's stream); repeated Starts restage every time."""
    monkeypatch.setenv("EXT_MPI_AMD_HOST_DIRECT", "0")
    sends = xorshift_inputs(R, count, code, seed_base=0x9191 + count)
    recvs = [s.copy() for s in sends] if in_place else [np.full(count, -1, dtype=s.dtype) for s in sends]
    h = emac.node_allreduce_init([(r if in_place else s).ctypes.data for s, r in zip(sends, recvs)],
                                 [r.ctypes.data for r in recvs], count, code, copyin)
    try:
        for _ in range(3):
            if in_place:
                for r, s in zip(recvs, sends):
                    r[:] = s
            emac.start(h)
            emac.wait(h)
            assert_bitwise(recvs, oracle.allreduce(sends, copyin, in_place=in_place), "host staged")
    finally:
        emac.done(h)


def test_misaligned_buffers_take_element_path(oracle):
    """Buffers whose 16-byte phases differ fall back to the element-granular kernel path."""
    R, count = 4, 50001
    sends = xorshift_inputs(R, count, emac.FLOAT)
    want = oracle.allreduce(sends, "6;1 -4 4")
    base = [torch.zeros(count + 4, dtype=torch.float32, device="cuda") for _ in range(R)]
    outs = [torch.zeros(count + 4, dtype=torch.float32, device="cuda") for _ in range(R)]
    dsend = [b[r % 3: r % 3 + count] for r, b in enumerate(base)]  # element offsets 0,1,2,0
    drecv = [o[1: 1 + count] for o in outs]
    for t, s in zip(dsend, sends):
        t.copy_(torch.from_numpy(s))
    h = emac.node_allreduce_init([t.data_ptr() for t in dsend], [t.data_ptr() for t in drecv], count, emac.FLOAT,
                                 "6;1 -4 4")
    emac.start(h)
    emac.wait(h)
    emac.done(h)
    assert_bitwise([t.cpu().numpy() for t in drecv], want, "misaligned")
    # guard elements around the receive windows are untouched
    for o in outs:
        assert o[0].item() == 0.0 and o[count + 1].item() == 0.0


def test_test_and_wait_semantics():
    R, count = 8, 1 << 20
    sends = [torch.ones(count, device="cuda") * r for r in range(R)]
    recvs = [torch.empty(count, device="cuda") for _ in range(R)]
    h = emac.node_allreduce_init([t.data_ptr() for t in sends], [t.data_ptr() for t in recvs], count, emac.FLOAT)
    assert emac.test(h) == 1  # nothing started
    emac.start(h)
    while emac.test(h) == 0:
        pass
    assert emac.test(h) == 1
    emac.done(h)
    for r in recvs:
        assert torch.all(r == 28.0)


def test_config2_full_size_bitexact(oracle):
    """BASELINE config 2: float MPI_SUM, 16 MiB per rank, 8 ranks, '6;1 -8 8' -- full size."""
    count = (16 << 20) // 4
    sends = xorshift_inputs(8, count, emac.FLOAT)
    assert_bitwise(run_node(sends, emac.FLOAT, "6;1 -8 8"), oracle.allreduce(sends, "6;1 -8 8"), "config 2")


@pytest.mark.parametrize("code", [emac.INT, emac.LONG])
def test_config3_int_long_4mib_bitexact(oracle, code):
    """BASELINE config 3: int + long int MPI_SUM, 4 MiB, bit-exact vs the CPU path."""
    count = (4 << 20) // np.dtype(NP[code]).itemsize
    sends = xorshift_inputs(8, count, code)
    for copyin in ("6;1 -8 8", "6;1 -2 -2 -2 2 2 2"):
        assert_bitwise(run_node(sends, code, copyin), oracle.allreduce(sends, copyin), f"config 3 {copyin}")


def _assert_ranks_bitwise(got, want, what):
    """every rank's result against the oracle's (all equal for a correct schedule)"""
    for r, g in enumerate(got):
        if not np.array_equal(g.view(np.uint8), want[r].view(np.uint8)):
            bad = np.flatnonzero(g.view(np.uint8) != want[r].view(np.uint8))
            raise AssertionError(f"{what}: rank {r}: {bad.size} differing bytes, first at byte {bad[0]}")


@pytest.mark.parametrize("copyin", ["6;1 -8 8", "6;1 -2 -2 -2 2 2 2"])
def test_config4_random_double_256mib_node(oracle, copyin):
    """BASELINE configs[3]'s message (double MPI_SUM, 256 MiB per rank, 8 ranks) with random
    non-integer doubles, so every summation order gives different bits: the node form must
    reproduce the reference's order exactly (0 ulp against the oracle)."""
    count = (256 << 20) // 8
    sends = xorshift_inputs(8, count, emac.DOUBLE, seed_base=0xC4D00000)
    want = oracle.allreduce(sends, copyin)
    got = run_node(sends, emac.DOUBLE, copyin)
    _assert_ranks_bitwise(got, want, f"config 4 node {copyin}")


@pytest.mark.parametrize("copyin", ["6;1 -8 8", "6;1 -2 -2 -2 2 2 2"])
def test_config4_random_double_256mib_comm_loopback(oracle, copyin):
    """The same message through the communicator form (staging slots, reduce-scatter and
    allgather leg programs, the owner's fold; loopback transport on the one GPU)."""
    count = (256 << 20) // 8
    sends = xorshift_inputs(8, count, emac.DOUBLE, seed_base=0xC4D10000)
    want = oracle.allreduce(sends, copyin)
    got = run_comm_loopback(sends, emac.DOUBLE, copyin)
    _assert_ranks_bitwise(got, want, f"config 4 comm {copyin}")


@pytest.mark.parametrize("nbytes", [8, 512 << 20])
def test_config5_float_sweep_endpoints(oracle, nbytes):
    """BASELINE configs[4]'s sweep endpoints (float MPI_SUM, 8 B and 512 MiB per rank, 8 ranks)."""
    count = nbytes // 4
    for copyin in ("6;1 -8 8",) if nbytes > 8 else ("6;1 -8 8", "6;-64 -8 8", "6;1 -2 -2 -2 2 2 2"):
        sends = xorshift_inputs(8, count, emac.FLOAT, seed_base=0xC5E00000 + nbytes)
        want = oracle.allreduce(sends, copyin)
        got = run_node(sends, emac.FLOAT, copyin)
        _assert_ranks_bitwise(got, want, f"config 5 {nbytes} B {copyin}")
        del sends, want, got


def test_comm_single_rank_rccl():
    """COMM form over an RCCL communicator of size 1 (the multi-GPU legs need >1 GPU)."""
    uid = emac.get_unique_id()
    comm = emac.comm_init(0, 1, uid, 0)
    x = torch.randn(12345, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    h = emac.allreduce_init(x.data_ptr(), y.data_ptr(), x.numel(), emac.DOUBLE, comm)
    emac.start(h)
    emac.wait(h)
    emac.done(h)
    emac.comm_free(comm)
    assert torch.equal(x, y)


@pytest.mark.parametrize("code", CODES)
@pytest.mark.parametrize("nsrc,ndst", [(1, 1), (3, 1), (8, 1), (8, 8), (16, 1)])
def test_fold_handle_and_copy_reduce(code, nsrc, ndst):
    """The persistent one-chunk fold and the device C-ABI copy_reduce: left fold in the given
    leaf order, every destination identical; compared with a sequential numpy fold."""
    count = 70001
    srcs_np = xorshift_inputs(nsrc, count, code, seed_base=991 + nsrc)
    want = srcs_np[0].copy()
    with np.errstate(over="ignore"):
        for x in srcs_np[1:]:
            want = want + x
    srcs = [_dev(x) for x in srcs_np]
    for how in ("handle", "copy_reduce"):
        dsts = [torch.full((count,), -1, dtype=TORCH[code], device="cuda") for _ in range(ndst)]
        if how == "handle":
            h = emac.fold_init([t.data_ptr() for t in srcs], [t.data_ptr() for t in dsts], count, code)
            emac.start(h)
            emac.wait(h)
            emac.done(h)
        else:
            L = emac.lib()
            L.ext_mpi_amd_gpu_copy_reduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                      ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                                      ctypes.POINTER(ctypes.c_void_p), ctypes.c_long, ctypes.c_void_p]
            sp = (ctypes.c_void_p * nsrc)(*[t.data_ptr() for t in srcs])
            dp = (ctypes.c_void_p * ndst)(*[t.data_ptr() for t in dsts])
            assert L.ext_mpi_amd_gpu_copy_reduce(code, emac.SUM, nsrc, sp, ndst, dp, count, None) == 0
        for d in dsts:
            assert np.array_equal(d.cpu().numpy().view(np.uint8), want.view(np.uint8)), (how, nsrc, ndst)


def test_copy_reduce_headline_instance():
    """The device C-ABI (ext_mpi_amd_gpu_copy_reduce, the reference's ext_mpi_gpu_copy_reduce,
    include/gpu/gpu_core.h:11-22, src/gpu/cuda_core.cu:88-106) and the persistent fold handle on
    the bench headline's kernel instance: float, 8 leaves folded and fanned out to 8 destinations,
    4 MiB per leaf -- the static schedule (U 4, staggered issue: fold_kernel<float, SUM, 8, 4,
    linear, 8, 5>) -- then the handle's tuned schedule on later Starts, every result bitwise
    equal to a sequential numpy left fold."""
    count, nsrc = 1 << 20, 8
    srcs_np = xorshift_inputs(nsrc, count, emac.FLOAT, seed_base=4242)
    want = srcs_np[0].copy()
    for x in srcs_np[1:]:
        want = want + x
    srcs = [_dev(x) for x in srcs_np]
    dsts = [torch.full((count,), -1.0, device="cuda") for _ in range(nsrc)]
    L = emac.lib()
    L.ext_mpi_amd_gpu_copy_reduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                              ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_long, ctypes.c_void_p]
    sp = (ctypes.c_void_p * nsrc)(*[t.data_ptr() for t in srcs])
    dp = (ctypes.c_void_p * nsrc)(*[t.data_ptr() for t in dsts])
    assert L.ext_mpi_amd_gpu_copy_reduce(emac.FLOAT, emac.SUM, nsrc, sp, nsrc, dp, count, None) == 0
    for d in dsts:
        assert np.array_equal(d.cpu().numpy().view(np.uint8), want.view(np.uint8))
    emac.tune_cache_clear()  # this shape tunes on this handle (engine_tune.c: kept schedules are shared)
    h = emac.fold_init([t.data_ptr() for t in srcs], [t.data_ptr() for t in dsts], count, emac.FLOAT)
    seen = set()
    for k in range(TUNE_STARTS):  # the static pick, 3 rounds of <= 8 candidates on three Starts each, then the kept one
        for d in dsts:
            d.fill_(-1.0)
        torch.cuda.synchronize()  # the fill runs on torch's stream, the fold on the handle's
        emac.start(h)
        emac.wait(h)
        sc = emac.handle_schedule(h)
        seen.add((sc["unroll"], sc["issue"], sc["tuned"]))
        for d in dsts:
            assert np.array_equal(d.cpu().numpy().view(np.uint8), want.view(np.uint8)), (k, sc)
    emac.done(h)
    assert (4, 5, 0) in seen  # the headline instance ran (static pick, before tuning kept one)
    assert any(t == 1 for _, _, t in seen)  # and the tuned schedule after it


DEFER_SHIFT = 11  # fold_kernel.hpp kDeferShift: deferred-store schedules (issue bits 11-12)
LEAF_MAJOR = 1 << 13  # fold_kernel.hpp kLeafMajor: leaf-major deferred groups
LM_OPEN_COPY = 1 << 16  # fold_kernel.hpp kLmOpenCopy: a chain's opening leaves copied into their accumulators
BUF_LOAD = 1 << 15  # fold_kernel.hpp kBufLoad: leaf loads as buffer loads


@pytest.mark.parametrize("copyin", ["6;1 -8 8", "6;1 -2 -2 -2 2 2 2"])
@pytest.mark.parametrize("code", [emac.FLOAT, emac.DOUBLE])
def test_every_tuned_schedule_bitwise(oracle, code, copyin):
    """The per-handle schedule tuner (engine.c emac_tune) runs every candidate on a handle's first
    Starts -- burst loads at U 2 / U 4, the staggered issue, and the deferred-store schedules
    (fold_kernel.hpp fold_deferred_kernel: 2 or 4 tiles folded into LDS, or leaf after leaf in
    registers, then stored in one burst) -- and
    keeps one. Every Start must give the oracle's bits: here a node form whose buckets end in a
    partial tile and whose last group of tiles is short (41000 elements per chunk: under 8 MiB per
    leaf, so (U 1, burst) among the candidates; 262147: above), and a local
    fold (8 leaves -> 1, fold_init) of 512040 elements, each over all the Starts of its tuning."""
    R = 8
    for chunk in ((41000, 262147) if code == emac.FLOAT else (20500, 131075)):
        count = R * chunk
        sends = xorshift_inputs(R, count, code, seed_base=0x7E57 + chunk)
        want = oracle.allreduce(sends, copyin)
        dsend = [_dev(x) for x in sends]
        drecv = [torch.full((count,), -1, dtype=TORCH[code], device="cuda") for _ in range(R)]
        emac.tune_cache_clear()  # every candidate runs on this handle (kept schedules are shared per shape)
        h = emac.node_allreduce_init([t.data_ptr() for t in dsend], [t.data_ptr() for t in drecv], count, code, copyin)
        cands = emac.handle_candidates(h)
        seen = set()
        try:
            for k in range(TUNE_STARTS):
                for t in drecv:
                    t.fill_(-1)
                torch.cuda.synchronize()
                emac.start(h)
                emac.wait(h)
                sc = emac.handle_schedule(h)
                seen.add((sc["unroll"], sc["issue"], sc["tuned"]))
                assert_bitwise([t.cpu().numpy() for t in drecv], want, f"node {copyin} chunk {chunk} Start {k} {sc}")
        finally:
            emac.done(h)
        assert any(t == 1 for _, _, t in seen), seen
        small = chunk * R * sends[0].itemsize < 8 << 20
        assert ((1, 1) in cands) == small, (chunk, cands)
        leaf = (2, 1 | 2 << DEFER_SHIFT | LEAF_MAJOR)  # leaf-major groups: linear fold and compile-time chains
        opencopy = (2, 1 | 2 << DEFER_SHIFT | LEAF_MAJOR | LM_OPEN_COPY)  # ... and for a chain its other form
        assert leaf in cands and (4, 1 | 1 << DEFER_SHIFT) in cands, cands
        assert (opencopy in cands) == (copyin != "6;1 -8 8"), cands
    # the local fold: one destination, one bucket -- under 8 MiB per leaf, and above it, where the
    # candidates are (U 4, burst), (U 4, staggered) with buffer loads and the LDS groups of (U 2, 4
    # tiles) and (U 4, 2 tiles) (engine_tune.c, round 6)
    big = ((8 << 20) // 4 + 1000) if code == emac.FLOAT else ((8 << 20) // 8 + 500)
    for n in ((8 * 64000 + 40 if code == emac.FLOAT else 4 * 64000 + 20), big):
        srcs_np = xorshift_inputs(R, n, code, seed_base=0x10CA1 + n)
        lwant = srcs_np[0].copy()
        for x in srcs_np[1:]:
            lwant = lwant + x
        srcs = [_dev(x) for x in srcs_np]
        dst = torch.full((n,), -1, dtype=TORCH[code], device="cuda")
        emac.tune_cache_clear()
        h = emac.fold_init([t.data_ptr() for t in srcs], [dst.data_ptr()], n, code)
        try:
            cands = emac.handle_candidates(h)
            if n == big:
                assert sorted(cands) == sorted([(4, 1), (4, 5 | BUF_LOAD), (2, 1 | 2 << DEFER_SHIFT),
                                                (4, 1 | 1 << DEFER_SHIFT)]), cands
            for k in range(TUNE_STARTS):
                dst.fill_(-1)
                torch.cuda.synchronize()
                emac.start(h)
                emac.wait(h)
                sc = emac.handle_schedule(h)
                assert_bitwise([dst.cpu().numpy()], [lwant], f"local fold {n} Start {k} {sc}")
        finally:
            emac.done(h)


@pytest.mark.parametrize("copyin", ["6;1 -2 -2 -2 2 2 2", "6;1 -4 -2 2 4", "6;1 -2 -4 4 2", "6;1 -8 8", "6;1 -2 -2 2 2",
                                    "6;-64 -8 8", "6;-4099 -8 8", "6;-64 -2 -2 -2 2 2 2"])
@pytest.mark.parametrize("form", ["plain", "opencopy"])
@pytest.mark.parametrize("code", [emac.FLOAT, emac.DOUBLE, emac.INT, emac.LONG])
def test_leaf_major_chains_forced_bitwise(oracle, monkeypatch, code, form, copyin):
    """Leaf-major groups over the compile-time radix chains (round 5, fold_kernel.hpp lm_leaves: one
    accumulator per open level, closed as the leaves complete their groups), forced as the only
    schedule (EXT_MPI_AMD_FOLD_SCHEDULE): every Start bitwise against the oracle's fold order.
    Sizes: whole groups (every bucket a multiple of the group), and a ragged one (partial last tile
    and group: the bounded buffer loads), both above the tuning threshold so the forced word is
    the handle's schedule. Both forms of the chains (the opening leaf of each level-0 group loaded into
    its accumulator, or copied there: kLmOpenCopy); the linear fold has the first only. The `-k`
    fractions (seven short chunks beside a long one: unequal buckets) run the groups through the
    layout's bucket map (layout.c, fold_kernel.hpp deferred_body MAP)."""
    R = 4 if copyin == "6;1 -2 -2 2 2" else 8
    tsize = 4 if code in (emac.FLOAT, emac.INT) else 8
    kb = 4
    word = 2 | (1 | 2 << DEFER_SHIFT | LEAF_MAJOR | (LM_OPEN_COPY if form == "opencopy" else 0)) << 4
    if copyin.endswith(" -8 8") and form == "opencopy":
        pytest.skip("the opening-copy form is instantiated for the chains only")
    monkeypatch.setenv("EXT_MPI_AMD_FOLD_SCHEDULE", str(word))
    group = 256 * 2 * kb * 16 // tsize  # elements per group and leaf
    m = max(8, (4 << 20) // (R * group * tsize))  # >= 4 MiB per rank: above the tuning threshold
    for chunk in (m * group, m * group + 3 * group // 4 + 5):  # equal chunks: every bucket the same tiles
        count = R * chunk
        sends = xorshift_inputs(R, count, code, seed_base=0x1EAF + len(form) + chunk + 7 * R)
        want = oracle.allreduce(sends, copyin)
        dsend = [_dev(x) for x in sends]
        drecv = [torch.full((count,), -1, dtype=TORCH[code], device="cuda") for _ in range(R)]
        emac.tune_cache_clear()
        h = emac.node_allreduce_init([t.data_ptr() for t in dsend], [t.data_ptr() for t in drecv], count, code, copyin)
        dwant = [_dev(w) for w in want]
        try:
            assert emac.handle_candidates(h) == [(2, word >> 4)], emac.handle_candidates(h)
            for k in range(TUNE_1):  # the static pick, the forced word's samples, then the word kept
                for t in drecv:
                    t.fill_(-1)
                torch.cuda.synchronize()
                emac.start(h)
                emac.wait(h)
                sc = emac.handle_schedule(h)
                for r, (g, w) in enumerate(zip(drecv, dwant)):  # bitwise, compared on the device
                    if not torch.equal(g.view(torch.uint8), w.view(torch.uint8)):
                        assert_bitwise([t.cpu().numpy() for t in drecv], want, f"{copyin} kb {kb} chunk {chunk} Start {k} {sc}")
            assert (sc["unroll"], sc["issue"], sc["tuned"]) == (2, word >> 4, 1), sc
        finally:
            emac.done(h)


def run_comm_loopback(sends, code, copyin, host=False, in_place=False, phase=None, op=emac.SUM, repeats=1, nodes=1,
                      ports=None, each=None):
    """COMM form (one rank per communicator) on the in-process loopback transport: the legs run
    on every rank in lock-step -- stage-in, reduce-scatter, fold, [the two-node legs,] all-gather,
    stage-out -- so the staging slots, fold buckets and leg programs of the multi-GPU path execute
    on one GPU. nodes > 1: consecutive blocks of R/nodes ranks are nodes, under the inter-node
    ports list `ports` (ext_mpi_amd_comm_set_node_ports; None: one port per step)."""
    R, count = len(sends), sends[0].size
    comms = emac.comm_init_loopback(R)
    if nodes > 1:
        for c in comms:
            emac.comm_set_nodes(c, nodes, ports)
    phase = phase or [0] * R
    keep = []
    if host == "pinned":  # page-locked host memory (staged through device mirrors like pageable memory)
        sbufs = [torch.from_numpy(s.copy()).pin_memory() for s in sends]
        rbufs = sbufs if in_place else [torch.full((count,), -1, dtype=TORCH[code]).pin_memory() for _ in sends]
        keep += sbufs + rbufs
        ptrs = [(s.data_ptr(), r.data_ptr()) for s, r in zip(sbufs, rbufs)]
    elif host:
        sbufs = [s.copy() for s in sends]
        rbufs = sbufs if in_place else [np.full(count, -1, dtype=s.dtype) for s in sends]
        ptrs = [(s.ctypes.data, r.ctypes.data) for s, r in zip(sbufs, rbufs)]
    else:
        # element offsets shift the 16-byte phase of each rank's buffers independently
        sb = [torch.zeros(count + 4, dtype=TORCH[code], device="cuda") for _ in range(R)]
        sbufs = [b[p:p + count] for b, p in zip(sb, phase)]
        for t, s in zip(sbufs, sends):
            t.copy_(torch.from_numpy(s))
        rbufs = sbufs if in_place else [torch.full((count,), -1, dtype=TORCH[code], device="cuda") for _ in range(R)]
        keep += sb
        ptrs = [(s.data_ptr(), r.data_ptr()) for s, r in zip(sbufs, rbufs)]
    hs = []
    try:
        for r in range(R):
            hs.append(emac.allreduce_init(ptrs[r][0], ptrs[r][1], count, code, comms[r], copyin, op=op))
        for rep in range(repeats):
            if rep and not host and not in_place:  # the receive buffers forget the previous result
                for t in rbufs:
                    t.fill_(-1)
            torch.cuda.synchronize()
            for leg in emac.lockstep_legs(nodes, ports):
                for h in hs:
                    emac.start_legs(h, leg)
                for h in hs:
                    emac.wait(h)
            if each is not None:  # every Start's results, with every rank's fold schedule
                each(rep, [np.asarray(r) if host else r.cpu().numpy() for r in rbufs],
                     [emac.handle_schedule(h) for h in hs])
    finally:
        for h in hs:
            emac.done(h)
        for c in comms:
            emac.comm_free(c)
    return [np.asarray(r) if host else r.cpu().numpy() for r in rbufs]


def test_comm_form_tuned_fold_every_start(oracle):
    """The COMM form's local fold (R staged slices of the owner chunk -> the receive buffer) is
    tuned per handle like the NODE form's (engine.c emac_tune: per-tile and deferred-store
    candidates, 3 rounds of three Starts each): 8 loopback ranks x 16 MiB float, every Start bitwise."""
    R, count = 8, (16 << 20) // 4
    sends = xorshift_inputs(R, count, emac.FLOAT, seed_base=0x7A11)
    want = oracle.allreduce(sends, "6;1 -8 8")
    seen = set()

    def each(rep, got, scheds):
        assert_bitwise(got, want, f"Start {rep}")
        seen.update((sc["unroll"], sc["issue"], sc["tuned"]) for sc in scheds)

    emac.tune_cache_clear()
    run_comm_loopback(sends, emac.FLOAT, "6;1 -8 8", repeats=TUNE_STARTS, each=each)
    assert any(t == 1 for _, _, t in seen), seen  # the tuning finished and kept a schedule


@pytest.mark.parametrize("R,copyin,in_place", [(2, "6;1 -2 2", False), (4, "6;1 -2 -2 2 2", True),
                                               (8, "6;1 -8 8", False), (3, "6;-64 -3 3", False)])
@pytest.mark.parametrize("code", CODES)
def test_comm_loopback_pinned_host_buffers(oracle, R, copyin, in_place, code):
    """COMM form with page-locked host send / receive buffers (torch pin_memory), staged through
    device mirrors on the handle's stream -- bitwise against the oracle, in place too."""
    for count in (1, 1031, 65536 + 5):
        sends = xorshift_inputs(R, count, code, seed_base=0x9140 + count)
        want = oracle.allreduce(sends, copyin, in_place=in_place)
        got = run_comm_loopback(sends, code, copyin, host="pinned", in_place=in_place)
        assert_bitwise(got, want, f"pinned comm R={R} {copyin} code={code} n={count}")


COMM_CONFIGS = [(2, "6;1 -2 2"), (3, "6;1 -3 3"), (4, "6;1 -2 -2 2 2"), (6, "6;1 -3 -2 2 3"), (8, "6;1 -8 8"),
                (8, "6;1 -2 -4 4 2"), (8, "6;-64 -8 8"), (16, "6;1 -4 -4 4 4"), (8, "6;1 -2 2 1 2 1 -4 4"),
                (8, "6;1 -2 2 1 2 1 -2 2 1 2 1 -2 2")]


@pytest.mark.parametrize("R,copyin", COMM_CONFIGS)
@pytest.mark.parametrize("code", CODES)
def test_comm_form_loopback_parity(oracle, R, copyin, code):
    for count in (0, 1, 7, 1031, 65536 + 5):
        sends = xorshift_inputs(R, count, code, seed_base=0xC0AA0000 + count)
        want = oracle.allreduce(sends, copyin)
        got = run_comm_loopback(sends, code, copyin, phase=[(r * 3) % 4 for r in range(R)])
        assert_bitwise(got, want, f"comm R={R} {copyin} code={code} n={count}")


@pytest.mark.parametrize("R,copyin", [(2, "6;1 -1 1"), (4, "6;1 -2 2"), (8, "6;1 -4 4"), (8, "6;1 -2 -2 2 2"),
                                      (16, "6;1 -8 8"), (8, "7;1 -4 4"), (6, "5;1 -3 3"), (8, "6;-64 -4 4")])
@pytest.mark.parametrize("code", CODES)
def test_comm_two_nodes_loopback_vs_oracle(oracle, R, copyin, code):
    """§8(f3): two nodes of R/2 ranks, one port -- the node's legs and fold, the node-pair swap of
    the owned chunk's halves, their two-leaf fold, the swap back, the node's allgather -- bitwise
    against the oracle's two-node emulation, with per-rank 16-byte phase shifts."""
    for count in (0, 1, 7, 1031, 65536 + 5):
        sends = xorshift_inputs(R, count, code, seed_base=0x20DE0000 + count)
        want = oracle.allreduce_nodes(sends, copyin, 2)
        got = run_comm_loopback(sends, code, copyin, phase=[(r * 3) % 4 for r in range(R)], nodes=2)
        assert_bitwise(got, want, f"two nodes R={R} {copyin} code={code} n={count}")


@pytest.mark.parametrize("R,nodes,copyin", [(4, 4, "6;1 -1 1"), (8, 4, "6;1 -2 2"), (16, 4, "6;1 -2 -2 2 2"),
                                             (8, 8, "6;1 -1 1"), (16, 8, "7;1 -2 2"), (16, 16, "6;1 -1 1"),
                                             (12, 4, "5;1 -3 3")])
@pytest.mark.parametrize("code", [emac.FLOAT, emac.DOUBLE, emac.INT])
def test_comm_many_nodes_loopback_vs_oracle(oracle, R, nodes, copyin, code):
    """2^k nodes, one port per step: the node-pair swaps and folds step by step (pairs by the
    lowest node bit first), the ranges back in reverse order -- bitwise vs the oracle."""
    for count in (0, 5, 1031, 65536 + 7):
        sends = xorshift_inputs(R, count, code, seed_base=0x4D0E0000 + count)
        want = oracle.allreduce_nodes(sends, copyin, nodes)
        got = run_comm_loopback(sends, code, copyin, phase=[(r * 3) % 4 for r in range(R)], nodes=nodes)
        assert_bitwise(got, want, f"{nodes} nodes R={R} {copyin} code={code} n={count}")


@pytest.mark.parametrize("R,nodes,ports,copyin", [(3, 3, [-2, 2], "6;1 -1 1"), (6, 3, [-2, 2], "6;1 -2 2"),
                                                   (12, 3, [-2, 2], "7;1 -2 -2 2 2"), (8, 4, [-3, 3], "6;1 -2 2"),
                                                   (6, 6, [-1, -2, 2, 1], "6;1 -1 1"),
                                                   (12, 6, [-2, -1, 1, 2], "5;1 -2 2"),
                                                   (16, 8, [-3, -1, 1, 3], "6;1 -2 2"), (9, 9, [-2, -2, 2, 2], "6;1 -1 1"),
                                                   (10, 5, [-4, 4], "6;1 -2 2"),
                                                   # allgather steps that reduce (README 4(3), 4(-1 1 1))
                                                   (4, 4, [3], "6;1 -1 1"), (8, 4, [-1, 1, 1], "6;1 -2 2"),
                                                   (8, 4, [1, 1], "6;1 -2 2"), (6, 6, [-1, 2, 1], "6;1 -1 1"),
                                                   (6, 3, [2], "6;1 -2 2"),
                                                   # radix-2 reduce-scatter steps, other allgather radices
                                                   (4, 4, [-1, -1, 3], "6;1 -1 1"),
                                                   (16, 8, [-1, -1, -1, 3, 1], "6;1 -2 2"),
                                                   (16, 16, [-15, 15], "6;1 -1 1")])  # 16 leaves
@pytest.mark.parametrize("code", [emac.FLOAT, emac.DOUBLE, emac.INT])
def test_comm_node_ports_loopback_vs_oracle(oracle, R, nodes, ports, copyin, code):
    """Several ports per step (radix 3-5 node steps, mixed radices): every task trades its
    sub-group's lines with its column peers and folds them in the reference's accumulator order
    (raw_code.c over allreduce_core's reducefrom lists) -- bitwise vs the oracle's restatement."""
    for count in (0, 5, 1031, 65536 + 7):
        sends = xorshift_inputs(R, count, code, seed_base=0x4D0F0000 + count)
        want = oracle.allreduce_nodes(sends, copyin, nodes, ports=ports)
        got = run_comm_loopback(sends, code, copyin, phase=[(r * 3) % 4 for r in range(R)], nodes=nodes, ports=ports)
        assert_bitwise(got, want, f"{nodes} nodes {ports} R={R} {copyin} code={code} n={count}")


def test_comm_node_ports_in_place_host_min(oracle):
    sends = xorshift_inputs(9, 100003, emac.FLOAT, seed_base=0x20DE8000)
    want = oracle.allreduce_nodes(sends, "6;1 -3 3", 3, in_place=True, ports=[-2, 2])
    assert_bitwise(run_comm_loopback(sends, emac.FLOAT, "6;1 -3 3", in_place=True, nodes=3, ports=[-2, 2]), want,
                   "three nodes in place")
    want = oracle.allreduce_nodes(sends, "6;1 -3 3", 3, ports=[-2, 2])
    assert_bitwise(run_comm_loopback(sends, emac.FLOAT, "6;1 -3 3", host=True, nodes=3, ports=[-2, 2]), want,
                   "three nodes host buffers")
    want = oracle.allreduce_nodes(sends, "6;1 -3 3", 3, op=oracle.MIN, ports=[-2, 2])
    assert_bitwise(run_comm_loopback(sends, emac.FLOAT, "6;1 -3 3", nodes=3, ports=[-2, 2], op=emac.MIN), want,
                   "three nodes MIN")


def test_comm_two_nodes_loopback_in_place_host_repeats(oracle):
    sends = xorshift_inputs(8, 100003, emac.FLOAT, seed_base=0x20DE7000)
    want = oracle.allreduce_nodes(sends, "6;1 -4 4", 2, in_place=True)
    assert_bitwise(run_comm_loopback(sends, emac.FLOAT, "6;1 -4 4", in_place=True, nodes=2), want,
                   "two nodes in place")
    want = oracle.allreduce_nodes(sends, "6;1 -2 -2 2 2", 2)
    assert_bitwise(run_comm_loopback(sends, emac.FLOAT, "6;1 -2 -2 2 2", host=True, nodes=2), want,
                   "two nodes host buffers")


@pytest.mark.parametrize("graph", ["0", "1"])
def test_comm_form_graph_and_eager(oracle, monkeypatch, graph):
    """The COMM form's legs captured into HIP graphs (one per subset of legs, replayed by
    hipGraphLaunch) and launched eagerly (EXT_MPI_AMD_GRAPH=0): both bit-exact against the oracle
    on the loopback transport, every leg's graph replayed three times (receive buffers reset
    between replays)."""
    monkeypatch.setenv("EXT_MPI_AMD_GRAPH", graph)
    for R, copyin, code in [(4, "6;1 -2 -2 2 2", emac.FLOAT), (8, "6;1 -8 8", emac.DOUBLE), (3, "6;-64 -3 3", emac.INT)]:
        sends = xorshift_inputs(R, 4099 + R, code, seed_base=0x6A0000 + R)
        want = oracle.allreduce(sends, copyin)
        got = run_comm_loopback(sends, code, copyin, phase=[(r * 3) % 4 for r in range(R)], repeats=3)
        assert_bitwise(got, want, f"graph={graph} R={R} {copyin}")


def test_comm_single_rank_rccl_graph_replays(monkeypatch):
    """One persistent handle on a 1-rank RCCL communicator started 5 times with new data: the
    graph captured at the first Start is replayed and sees every new input."""
    monkeypatch.setenv("EXT_MPI_AMD_GRAPH", "1")
    uid = emac.get_unique_id()
    comm = emac.comm_init(0, 1, uid, 0)
    x = torch.empty(70001, dtype=torch.float32, device="cuda")
    y = torch.empty_like(x)
    h = emac.allreduce_init(x.data_ptr(), y.data_ptr(), x.numel(), emac.FLOAT, comm)
    try:
        for it in range(5):
            x.uniform_(-1, 1)
            torch.cuda.synchronize()
            emac.start(h)
            emac.wait(h)
            assert torch.equal(x, y), it
    finally:
        emac.done(h)
        emac.comm_free(comm)


@pytest.mark.parametrize("in_place", [False, True])
def test_comm_form_loopback_host_and_in_place(oracle, in_place):
    sends = xorshift_inputs(4, 200003, emac.DOUBLE)
    want = oracle.allreduce(sends, "6;1 -4 4", in_place=in_place)
    for host in (False, True):
        got = run_comm_loopback(sends, emac.DOUBLE, "6;1 -4 4", host=host, in_place=in_place)
        assert_bitwise(got, want, f"comm host={host} in_place={in_place}")


# ---- MIN / MAX: the reference's CPU reduction (ext_mpi_native_exec.c:240-318), not its GPU kernel

def special_inputs(R, count, code, seed):
    """xorshift inputs with NaN, signed zeros and infinities planted on some ranks (floating
    point), so that the order-dependent compare-and-select rule is exercised, not only min()."""
    sends = xorshift_inputs(R, count, code, seed_base=seed)
    if code in (emac.FLOAT, emac.DOUBLE) and count:
        idx = np.arange(count)
        for r, x in enumerate(sends):
            x[(idx % 7 == 0) & (idx % R == r)] = np.nan
            x[(idx % 11 == 3)] = -0.0 if r % 2 else 0.0
            x[(idx % 13 == 5) & (idx % R == (r + 1) % R)] = np.inf
            x[(idx % 17 == 6) & (idx % R == (r + 2) % R)] = -np.inf
    return sends


MINMAX_CONFIGS = [(2, "6;1 -2 2"), (3, "6;1 -3 3"), (4, "6;1 -2 -2 2 2"), (8, "6;1 -8 8"), (8, "6;1 -2 -2 -2 2 2 2"),
                  (8, "6;-64 -8 8"), (8, "6;1 -4 4 1 4 1 -2 2"), (16, "6;1 -16 16")]


@pytest.mark.parametrize("op", [emac.MIN, emac.MAX])
@pytest.mark.parametrize("R,copyin", MINMAX_CONFIGS)
@pytest.mark.parametrize("code", CODES)
def test_node_min_max_vs_oracle(oracle, op, R, copyin, code):
    for count in (1, 1031, 65536 + 3):
        sends = special_inputs(R, count, code, 0x313A0000 + count)
        want = oracle.allreduce(sends, copyin, op=op)
        got = run_node(sends, code, copyin, op=op)
        assert_bitwise(got, want, f"op={op} R={R} {copyin} code={code} n={count}")


@pytest.mark.parametrize("op", [emac.MIN, emac.MAX])
@pytest.mark.parametrize("code", CODES)
def test_comm_loopback_min_max_vs_oracle(oracle, op, code):
    for R, copyin in [(4, "6;1 -2 -2 2 2"), (8, "6;1 -8 8")]:
        sends = special_inputs(R, 65536 + 5, code, 0x313B0000 + R)
        want = oracle.allreduce(sends, copyin, op=op)
        got = run_comm_loopback(sends, code, copyin, phase=[(r * 3) % 4 for r in range(R)], op=op)
        assert_bitwise(got, want, f"comm op={op} R={R} {copyin} code={code}")


@pytest.mark.parametrize("op", [emac.MIN, emac.MAX])
def test_node_min_max_in_place_and_full_size(oracle, op):
    sends = special_inputs(8, (16 << 20) // 4, emac.FLOAT, 0x313C0000)
    want = oracle.allreduce(sends, "6;1 -8 8", in_place=True, op=op)
    assert_bitwise(run_node(sends, emac.FLOAT, "6;1 -8 8", in_place=True, repeats=2, op=op), want, "in place")


def _radix_chain(R):
    fs, n = [], R
    for p in (2, 3, 5, 7, 11, 13):
        while n % p == 0:
            fs.append(p)
            n //= p
    return "6;1 " + " ".join(f"-{f}" for f in fs) + " " + " ".join(str(f) for f in reversed(fs)) if len(fs) > 1 else None


def test_node_random_cases_vs_oracle(oracle):
    """Seeded random node-form cases: node size, size, type, operation, copy-in variant, in place."""
    rng = np.random.default_rng(0x9A11)
    for _ in range(40):
        R = int(rng.integers(2, 17))
        variants = [f"6;1 -{R} {R}", f"6;-64 -{R} {R}", f"6;{int(rng.integers(2, 5))} -{R} {R}"]
        if _radix_chain(R):
            variants.append(_radix_chain(R))
        copyin = variants[int(rng.integers(len(variants)))]
        count = int(min(1 << 21, np.exp(rng.uniform(0, np.log(1 << 21)))))
        code = int(rng.choice(CODES))
        op = int(rng.choice([emac.SUM, emac.SUM, emac.MIN, emac.MAX]))
        in_place = bool(rng.random() < 0.3)
        sends = special_inputs(R, count, code, int(rng.integers(1 << 30)))
        want = oracle.allreduce(sends, copyin, in_place=in_place, op=op)
        got = run_node(sends, code, copyin, in_place=in_place, op=op)
        assert_bitwise(got, want, f"R={R} '{copyin}' code={code} op={op} n={count} in_place={in_place}")


def test_comm_loopback_random_cases_vs_oracle(oracle):
    """Seeded random COMM-form cases on the loopback transport (staging slots, leg programs and
    the owner's fold): node size, size, type, operation, copy-in variant, buffer phase."""
    rng = np.random.default_rng(0xC0BB)
    for _ in range(16):
        R = int(rng.integers(2, 9))
        variants = [f"6;1 -{R} {R}", f"6;-64 -{R} {R}"]
        if _radix_chain(R):
            variants.append(_radix_chain(R))
        copyin = variants[int(rng.integers(len(variants)))]
        count = int(min(1 << 20, np.exp(rng.uniform(0, np.log(1 << 20)))))
        code = int(rng.choice(CODES))
        op = int(rng.choice([emac.SUM, emac.MIN, emac.MAX]))
        sends = special_inputs(R, count, code, int(rng.integers(1 << 30)))
        want = oracle.allreduce(sends, copyin, op=op)
        got = run_comm_loopback(sends, code, copyin, phase=[int(x) for x in rng.integers(0, 4, R)], op=op)
        assert_bitwise(got, want, f"comm R={R} '{copyin}' code={code} op={op} n={count}")
