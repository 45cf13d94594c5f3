"""The peer-mapped node join's shares (plan.c emac_node_shares, via ext_mpi_amd_node_shares)
replayed on the CPU: every node's partial is its copy-in (the planner's fold trees,
helpers.replay_plan), every part of every node rank's chunk is ONE left fold of the N node partials
in the listed order, and the result must equal the oracle's multi-node restatement
(oracle/ref_emulate.c ref_emulate_node_ports: allreduce_core's line tables under the
EXT_MPI_NUM_PORTS list, src/core/allreduce_recursive.c:222-453) bit for bit, for every rank of every
node. The parts of each chunk must tile it exactly once. No GPU needed: the GPU runs the same
buckets (tests/test_gpu_node_ipc.py)."""
import numpy as np
import pytest

import ext_mpi_collectives_amd as emac
from helpers import replay_plan, xorshift_inputs

CASES = [
    (2, [-1, 1], 4, "6;1 -4 4"), (2, None, 2, "6;1 -2 2"), (3, [-2, 2], 4, "6;1 -4 4"), (3, None, 2, "6;1 -2 2"),
    (4, [-3, 3], 8, "6;1 -8 8"), (4, [-3, 3], 4, "6;1 -2 -2 2 2"), (5, [-4, 4], 3, "6;1 -3 3"),
    (6, [-5, 5], 2, "6;-64 -2 2"), (7, [-6, 6], 1, "6;1 -1 1"), (8, [-7, 7], 8, "6;1 -8 8"),
    (8, [-7, 7], 4, "7;1 -2 -2 2 2"), (3, [-2, 2], 4, "5;1 -4 4"), (4, [-3, 3], 4, "6;3 -4 4"),
    # one port per step over 2^k nodes (the default list there): pairs over the task bits
    (4, None, 4, "6;1 -4 4"), (8, None, 2, "6;1 -2 2"), (16, None, 2, "6;1 -2 2"), (4, [-1, -1, 1, 1], 3, "6;1 -3 3"),
]


def _node_join(sends, code, copyin, nodes, ports):
    W, count = len(sends), sends[0].size
    R = W // nodes
    part = [replay_plan(sends[n * R:(n + 1) * R], code, copyin) for n in range(nodes)]
    out = np.empty_like(sends[0])
    cover = np.zeros(count, np.int32)
    for me in range(R):
        levels, shares = emac.node_shares(nodes, ports, R, count, code, copyin, me)
        for off, ln, who, leaves in shares:
            seg = slice(off, off + ln)
            assert 0 <= who < nodes and sorted(leaves) == list(range(nodes))
            with np.errstate(over="ignore"):
                if levels == 1:  # a left fold in the listed order
                    acc = part[leaves[0]][seg].copy()
                    for n in leaves[1:]:
                        acc = acc + part[n][seg]
                else:  # levels of pairs of consecutive leaves
                    vals = [part[n][seg] for n in leaves]
                    for _ in range(levels):
                        vals = [vals[2 * i] + vals[2 * i + 1] for i in range(len(vals) // 2)]
                    assert len(vals) == 1
                    acc = vals[0]
            out[seg] = acc
            cover[seg] += 1
    assert np.all(cover == 1), "the parts do not tile the message"
    return out


@pytest.mark.parametrize("nodes,ports,R,copyin", CASES)
@pytest.mark.parametrize("code", [emac.FLOAT, emac.DOUBLE, emac.INT, emac.LONG])
def test_node_shares_replay_equals_oracle(oracle, nodes, ports, R, copyin, code):
    for count in (0, 1, 7, 1000, 4099, 65536 + 3):
        sends = xorshift_inputs(nodes * R, count, code, seed_base=0x5A4E0000 + count + nodes)
        want = oracle.allreduce_nodes(sends, copyin, nodes,
                                      ports=ports if ports is not None else
                                      (emac.default_node_ports(nodes) if nodes & (nodes - 1) else None))
        got = _node_join(sends, code, copyin, nodes, ports)
        for r, w in enumerate(want):
            assert np.array_equal(w.view(np.uint8), got.view(np.uint8)), (nodes, ports, R, copyin, code, count, r)


def test_node_shares_balanced_and_refused():
    """Every node folds an equal share (±1 element per piece); lists of several steps that are not
    one port each, or whose allgather steps reduce, are refused."""
    for nodes in (3, 4, 8):
        per = [0] * nodes
        for me in range(8):
            for off, ln, who, _ in emac.node_shares(nodes, [-(nodes - 1), nodes - 1], 8, 1 << 20, emac.FLOAT, "6;1 -8 8",
                                                    me)[1]:
                per[who] += ln
        assert max(per) - min(per) <= 8, per
    for ports in ([-1, -2, 2, 1], [-2, -1, 1, 2], [3]):  # several steps with larger radices, reducing allgathers
        with pytest.raises(emac.ExtMpiError) as e:
            emac.node_shares(6 if len(ports) > 1 else 4, ports, 2, 1000, emac.FLOAT, "6;1 -2 2", 0)
        assert e.value.code == emac.ERROR_UNSUPPORTED
