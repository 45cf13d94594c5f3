"""The NODE form over several nodes (ext_mpi_amd_node_comm_allreduce_init): every rank of a node
in one process on one GPU, the nodes joined by a communicator with one member per node, here the
in-process loopback transport (every node on the one GPU, the inter-node legs as device copies run
in lock-step). Bitwise against the oracle's multi-node restatement over nodes * R ranks
(oracle/ref_emulate.c ref_emulate_node_ports: each node's copy-in, allreduce_core between the
nodes under the EXT_MPI_NUM_PORTS list, the copy-out; src/core/allreduce_recursive.c:222-453,
src/mpi/ext_mpi_native.c:879-1000). This is the form bench.py measures at N > 1 GPUs (one node of
8 ranks per GPU, RCCL between them); the RCCL members run the same per-leg programs."""
import numpy as np
import pytest

import ext_mpi_collectives_amd as emac
from helpers import xorshift_inputs

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TORCH = {emac.FLOAT: torch.float32, emac.DOUBLE: torch.float64, emac.INT: torch.int32, emac.LONG: torch.int64}


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    emac.lib()


def assert_bitwise(got, want, what=""):
    for r, (g, w) in enumerate(zip(got, want)):
        if not np.array_equal(g.view(np.uint8), w.view(np.uint8)):
            bad = np.nonzero(g.view(np.uint8) != w.view(np.uint8))[0]
            raise AssertionError(f"{what}: rank {r}: {bad.size} differing bytes, first at byte {bad[0]}")


def run_node_comm_loopback(sends, code, copyin, nodes, ports=None, in_place=False, phase=None, op=emac.SUM,
                           repeats=1):
    """node-major ranks: sends[n * R + me] is rank me of node n"""
    W, count = len(sends), sends[0].size
    R = W // nodes
    comms = emac.comm_init_loopback(nodes)
    if ports is not None:
        for c in comms:
            emac.comm_set_nodes(c, nodes, ports)
    phase = phase or [0] * W
    sb = [torch.zeros(count + 4, dtype=TORCH[code], device="cuda") for _ in range(W)]
    sbufs = [b[p:p + count] for b, p in zip(sb, phase)]
    for t, s in zip(sbufs, sends):
        t.copy_(torch.from_numpy(s))
    rbufs = sbufs if in_place else [torch.full((count,), -1, dtype=TORCH[code], device="cuda") for _ in range(W)]
    hs = []
    try:
        for n in range(nodes):
            hs.append(emac.node_comm_allreduce_init([t.data_ptr() for t in sbufs[n * R:(n + 1) * R]],
                                                    [t.data_ptr() for t in rbufs[n * R:(n + 1) * R]], count, code,
                                                    comms[n], copyin, op=op))
        for rep in range(repeats):
            if rep and not in_place:
                for t in rbufs:
                    t.fill_(-1)
            torch.cuda.synchronize()
            for leg in emac.lockstep_legs(nodes, ports):
                for h in hs:
                    emac.start_legs(h, leg)
                for h in hs:
                    emac.wait(h)
    finally:
        for h in hs:
            emac.done(h)
        for c in comms:
            emac.comm_free(c)
    return [r.cpu().numpy() for r in rbufs]


def _want(oracle, sends, copyin, nodes, ports, **kw):
    if ports is None and nodes & (nodes - 1):
        ports = emac.default_node_ports(nodes)
    return oracle.allreduce_nodes(sends, copyin, nodes, ports=ports, **kw)


NODE_COMM_CONFIGS = [
    (2, 8, "6;1 -8 8", None),             # configs[1]'s node, two of them (one port)
    (4, 8, "6;1 -8 8", [-3, 3]),          # the bench's N = 4 shape: one radix-4 step
    (8, 8, "6;1 -8 8", [-7, 7]),          # ... N = 8: one radix-8 step
    (4, 8, "6;1 -2 -2 -2 2 2 2", None),   # radix chain in the node, one port per step between
    (3, 4, "6;1 -2 -2 2 2", None),        # three nodes: one radix-3 step by default
    (2, 3, "6;1 -3 3", None),
    (4, 2, "6;1 -2 2", [-1, -1, 1, 1]),
    (4, 4, "6;-64 -4 4", [3]),            # small-message fractions; an allgather step that reduces
    (2, 16, "6;1 -4 -4 4 4", None),
    (2, 4, "7;1 -4 4", None),             # tree method
    (6, 2, "6;1 -2 2", [-2, -1, 1, 2]),   # mixed radices
    (2, 1, "6;1 -1 1", None),             # one rank per node: the copy-in is a copy, no copy-out
]


@pytest.mark.parametrize("nodes,R,copyin,ports", NODE_COMM_CONFIGS)
@pytest.mark.parametrize("code", [emac.FLOAT, emac.DOUBLE, emac.INT, emac.LONG])
def test_node_comm_loopback_vs_oracle(oracle, nodes, R, copyin, ports, code):
    for count in (0, 1, 7, 1031, 65536 + 5):
        W = nodes * R
        sends = xorshift_inputs(W, count, code, seed_base=0x4C0C0000 + count + W)
        want = _want(oracle, sends, copyin, nodes, ports)
        got = run_node_comm_loopback(sends, code, copyin, nodes, ports, phase=[(r * 3) % 4 for r in range(W)])
        assert_bitwise(got, want, f"{nodes} nodes x {R} {copyin} {ports} code={code} n={count}")


def test_node_comm_in_place_min_repeats(oracle):
    sends = xorshift_inputs(12, 100003, emac.FLOAT, seed_base=0x4C0C8000)
    want = _want(oracle, sends, "6;1 -4 4", 3, None, in_place=True)
    assert_bitwise(run_node_comm_loopback(sends, emac.FLOAT, "6;1 -4 4", 3, in_place=True), want, "in place")
    want = _want(oracle, sends, "6;1 -4 4", 3, None, op=oracle.MIN)
    assert_bitwise(run_node_comm_loopback(sends, emac.FLOAT, "6;1 -4 4", 3, op=emac.MIN), want, "MIN")
    want = _want(oracle, sends, "6;1 -2 -2 2 2", 3, None)
    assert_bitwise(run_node_comm_loopback(sends, emac.FLOAT, "6;1 -2 -2 2 2", 3, repeats=3), want, "three Starts")


@pytest.mark.parametrize("nodes,ports", [(2, None), (4, [-3, 3])])
def test_node_comm_headline_shape(oracle, nodes, ports):
    """configs[1]'s node (8 ranks x 16 MiB float, '6;1 -8 8') on `nodes` nodes: the N-GPU bench
    workload at full size, bitwise."""
    count = (16 << 20) // 4
    sends = xorshift_inputs(8 * nodes, count, emac.FLOAT, seed_base=0x4C0C9000 + nodes)
    want = _want(oracle, sends, "6;1 -8 8", nodes, ports)
    assert_bitwise(run_node_comm_loopback(sends, emac.FLOAT, "6;1 -8 8", nodes, ports), want, f"{nodes} x 8 x 16 MiB")


def test_node_comm_refusals():
    """The members are the nodes: a communicator declared as nodes of several members is refused
    (ERROR_ARG), as are empty node sizes."""
    comms = emac.comm_init_loopback(4)
    a = torch.zeros(64, device="cuda")
    try:
        for c in comms:
            emac.comm_set_nodes(c, 2)
        with pytest.raises(emac.ExtMpiError) as e:
            emac.node_comm_allreduce_init([a.data_ptr()], [a.data_ptr()], 64, emac.FLOAT, comms[0], "6;1 -1 1")
        assert e.value.code == emac.ERROR_ARG
        with pytest.raises(emac.ExtMpiError) as e:
            emac.node_comm_allreduce_init([], [], 64, emac.FLOAT, comms[0])
        assert e.value.code == emac.ERROR_ARG
    finally:
        for c in comms:
            emac.comm_free(c)
