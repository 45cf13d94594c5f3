"""More than 16 nodes: the inter-node ports schedule of the COMM form over
up to 64 nodes, executed in ONE process -- every rank's point-to-point program replayed with its
messages matched in order per (sender, receiver) pair inside each leg, as RCCL matches the ops of
one group and as the loopback transport does (engine.c run_leg_loopback) -- and compared bitwise,
rank by rank, with the oracle's task-by-task restatement of allreduce_core
(oracle/ref_emulate.c ref_emulate_node_ports; src/core/allreduce_recursive.c:222-453).
Gloo with one process per rank (tests/test_dist_gloo.py) covers up to 8 nodes; 32-64 processes
would not fit the CPU suite's budget, and the program is the same data either way.
"""
import numpy as np
import pytest

import ext_mpi_collectives_amd as emac
from helpers import NP, xorshift_inputs


def _replay(nodes, R, count, code, copyin, ports):
    """Every rank's result of emac_comm_program_nodes (plan.c), run leg by leg in one process."""
    W = nodes * R
    dt = NP[code]
    isz = np.dtype(dt).itemsize
    sends = xorshift_inputs(W, count, code, seed_base=0x40DE5000 + count + nodes)
    progs = [emac.comm_program_nodes(nodes, R, r, count, code, copyin, ports=ports) for r in range(W)]
    bufs = []
    for r in range(W):
        stage = progs[r][2]
        bufs.append({emac.BUF_SEND: sends[r].view(np.uint8).copy(),
                     emac.BUF_RECV: np.full(count * isz, 0xAB, dtype=np.uint8),
                     emac.BUF_STAGE: np.zeros(max(stage, 1), dtype=np.uint8)})
    desc = emac.plan_describe(R, count, code, copyin, 0)

    def run_leg(leg):
        # a grouped exchange: every send reads its bytes before any receive of the leg lands
        queues = {}
        for r in range(W):
            for (lg, peer, is_send, b, off, n) in progs[r][0]:
                if lg == leg and is_send:
                    queues.setdefault((r, peer), []).append(bufs[r][b][off:off + n].copy())
        for r in range(W):
            for (lg, peer, is_send, b, off, n) in progs[r][0]:
                if lg == leg and not is_send:
                    data = queues[(peer, r)].pop(0)
                    assert data.size == n
                    bufs[r][b][off:off + n] = data
        assert all(not q for q in queues.values()), "unmatched sends"

    def node_fold(r, folds):
        for off, n, leaves in folds:
            xs = [bufs[r][b][lo:lo + n * isz].view(dt) for b, lo in leaves]
            acc, cur = [None] * desc["nlev"], None
            with np.errstate(over="ignore"):
                for t, x in enumerate(xs):
                    cur = x
                    for lvl in range(desc["nlev"]):
                        if lvl == 0 or desc["close"][t] >= lvl:
                            acc[lvl] = cur.copy() if (desc["first"][t] >> lvl) & 1 else acc[lvl] + cur
                        cur = acc[lvl]
            bufs[r][emac.BUF_RECV][off:off + n * isz].view(dt)[:] = cur

    nx, na = emac.node_steps(nodes, ports)
    SH = emac.LEG_STEP_SHIFT
    run_leg(emac.LEG_REDUCE_SCATTER)
    for r in range(W):
        node_fold(r, [f[:3] for f in progs[r][1] if f[3] == emac.LEG_FOLD])
    for st in range(nx):
        run_leg(emac.LEG_NODES_RS | st << SH)
        for r in range(W):
            for off, n, leaves, leg in progs[r][1]:
                if leg != emac.LEG_NODES_FOLD | st << SH:
                    continue
                xs = [bufs[r][b][o:o + n * isz].view(dt).copy() for b, o in leaves]
                acc = xs[0]
                with np.errstate(over="ignore"):
                    for x in xs[1:]:  # a left fold in the listed order
                        acc = acc + x
                bufs[r][emac.BUF_RECV][off:off + n * isz].view(dt)[:] = acc
    for j in range(na):
        run_leg(emac.LEG_NODES_AG | j << SH)
    run_leg(emac.LEG_ALLGATHER)
    return sends, [b[emac.BUF_RECV].view(dt) for b in bufs]


@pytest.mark.parametrize("nodes,R,ports,cases", [
    (32, 1, None, [(emac.FLOAT, 100003, "6;1 -1 1"), (emac.INT, 77, "6;1 -1 1")]),   # one port per step, 5 steps
    (64, 1, None, [(emac.FLOAT, 65536 + 37, "6;1 -1 1"), (emac.DOUBLE, 63, "6;1 -1 1")]),  # 6 steps
    (32, 2, [-1, -1, -1, -1, -1, 1, 1, 1, 1, 1], [(emac.FLOAT, 40009, "6;1 -2 2")]),
    (24, 1, [-2, -1, -1, -1, 1, 1, 1, 2], [(emac.FLOAT, 30011, "6;1 -1 1"), (emac.LONG, 999, "6;1 -1 1")]),
    (48, 1, [-2, -1, -1, -1, -1, 1, 1, 1, 1, 2], [(emac.DOUBLE, 20011, "6;1 -1 1")]),
    (20, 1, None, [(emac.FLOAT, 20011, "6;1 -1 1")]),       # no list, 20 nodes: steps 5, 2, 2 (prime factors)
    (48, 1, None, [(emac.FLOAT, 12001, "6;1 -1 1")]),       # 3, 2, 2, 2, 2
    (32, 1, [-3, -3, -1, 1, 3, 3], [(emac.FLOAT, 20011, "6;1 -1 1")]),                  # radix-4 steps, mixed
    (36, 1, [-2, -2, -1, -1, 1, 1, 2, 2], [(emac.FLOAT, 9001, "6;1 -1 1")]),            # 3 x 3 x 2 x 2
    (32, 1, [-1, -1, -1, -1, 1, 3, 1, 1], [(emac.FLOAT, 8009, "6;1 -1 1")]),             # 16 groups of 2 reduce in the allgather
])
def test_many_node_programs_vs_oracle(nodes, R, ports, cases):
    """The program of emac_comm_program_nodes over 20-64 nodes equals the oracle bitwise per rank
    (lists whose allgather radices multiply to the nodes; allgather steps that still reduce when
    the reduce-scatter radices cover fewer)."""
    for code, count, copyin in cases:
        try:
            sends, got = _replay(nodes, R, count, code, copyin, ports)
        except emac.ExtMpiError as e:
            pytest.fail(f"{nodes} nodes {ports}: program refused: {e}")
        from oracle import oracle
        oports = ports if ports is not None or nodes & (nodes - 1) == 0 else emac.default_node_ports(nodes)
        want = oracle.allreduce_nodes(sends, copyin, nodes, ports=oports)
        for r in range(nodes * R):
            assert np.array_equal(got[r].view(np.uint8), want[r].view(np.uint8)), (nodes, R, ports, code, count, r)


@pytest.mark.parametrize("nodes,ports", [
    (20, [-19, 19]),             # a step of radix 20: more partials than one fold launch takes (16)
    (34, None),                  # 2 x 17: no default schedule of steps of at most 16
    (32, [-1, -1, -1, -1, -1, -1, 1, 1, 1, 1, 1, 1]),  # 64 > 32 nodes' worth of steps
])
def test_many_node_lists_refused(nodes, ports):
    """Lists the path does not take are refused (ERROR_UNSUPPORTED / ERROR_ARG), never computed
    otherwise: radices above EXT_MPI_AMD_MAX_RANKS leaves, node counts with a prime factor above
    it when no list is given, radices that do not multiply to the nodes."""
    with pytest.raises(emac.ExtMpiError) as e:
        emac.comm_program_nodes(nodes, 1, 0, 1000, emac.FLOAT, "6;1 -1 1", ports=ports)
    assert e.value.code in (emac.ERROR_UNSUPPORTED, emac.ERROR_ARG)


@pytest.mark.parametrize("nodes", range(2, 65))
def test_default_node_ports_matches_c(nodes):
    """ext_mpi_collectives_amd.default_node_ports restates plan.c emac_node_sched_build's default
    list: the program the C library builds with no list (NULL) equals the one it builds from the
    Python list, rank by rank; where C refuses the default (a prime factor above 16 leaves per
    step), Python raises."""
    R, count = 1, 4 * nodes + 3
    try:
        ports = emac.default_node_ports(nodes)
    except ValueError:
        with pytest.raises(emac.ExtMpiError):
            emac.comm_program_nodes(nodes, R, 0, count, emac.FLOAT)
        return
    prod = 1
    for p in ports:
        if p < 0:
            prod *= 1 - p
    assert prod == nodes
    for r in sorted({0, nodes // 2, nodes - 1}):
        assert emac.comm_program_nodes(nodes, R, r, count, emac.FLOAT) == \
            emac.comm_program_nodes(nodes, R, r, count, emac.FLOAT, ports=ports)
