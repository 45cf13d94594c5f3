"""The N>1 (COMM form) path on CPU: world-size-2 and -4 gloo process groups execute exactly
the program the engine hands to RCCL (ext_mpi_amd_comm_program: reduce-scatter p2p ops, the
owner's folds, allgather p2p ops), with a numpy replay of the fold tree standing in for the
HIP kernel, and every rank's result is compared bit for bit with the oracle."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import ext_mpi_collectives_amd as emac
from helpers import NP, xorshift_inputs

LEG_RS, LEG_AG = emac.LEG_REDUCE_SCATTER, emac.LEG_ALLGATHER


def _bytes_view(buf, off, n):
    return torch.from_numpy(buf[off:off + n])


def _run_leg(ops, leg, bufs):
    reqs = []
    for (lg, peer, is_send, b, off, n) in ops:
        if lg != leg:
            continue
        t = _bytes_view(bufs[b], off, n)
        reqs.append(dist.isend(t, peer) if is_send else dist.irecv(t, peer))
    for r in reqs:
        r.wait()


def _fold(folds, bufs, code, desc):
    dt = NP[code]
    for off, count, leaves in folds:
        xs = [bufs[b][lo:lo + count * np.dtype(dt).itemsize].view(dt) for b, lo in leaves]
        acc, cur = [None] * desc["nlev"], None
        with np.errstate(over="ignore"):
            for t, x in enumerate(xs):
                cur = x
                for lvl in range(desc["nlev"]):
                    if lvl == 0 or desc["close"][t] >= lvl:
                        acc[lvl] = cur.copy() if (desc["first"][t] >> lvl) & 1 else acc[lvl] + cur
                    cur = acc[lvl]
        bufs[emac.BUF_RECV][off:off + count * np.dtype(dt).itemsize].view(dt)[:] = cur


def _worker(rank, world, port, cases, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    failures = []
    for code, count, copyin in cases:
        sends = xorshift_inputs(world, count, code)
        itemsize = np.dtype(NP[code]).itemsize
        ops, folds, stage = emac.comm_program(world, rank, count, code, copyin)
        bufs = {emac.BUF_SEND: sends[rank].view(np.uint8).copy(),
                emac.BUF_RECV: np.full(count * itemsize, 0xAB, dtype=np.uint8),
                emac.BUF_STAGE: np.zeros(max(stage, 1), dtype=np.uint8)}
        desc = emac.plan_describe(world, count, code, copyin, 0)
        _run_leg(ops, LEG_RS, bufs)
        _fold(folds, bufs, code, desc)
        _run_leg(ops, LEG_AG, bufs)
        want = oracle.allreduce(sends, copyin or f"6;1 -{world} {world}")[rank]
        if not np.array_equal(bufs[emac.BUF_RECV], want.view(np.uint8)):
            failures.append((rank, code, count, copyin))
    q.put(failures)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,cases", [
    (2, [(emac.FLOAT, 100003, None), (emac.DOUBLE, 7, "6;1 -2 2"), (emac.INT, 4099, "6;3 -2 2"),
         (emac.LONG, 1000, "6;-5 -2 2"), (emac.FLOAT, 0, None), (emac.FLOAT, 1, None)]),
    (4, [(emac.FLOAT, 65539, "6;1 -4 4"), (emac.DOUBLE, 4099, "6;1 -2 -2 2 2"), (emac.INT, 1001, "6;2 -2 -2 4"),
         (emac.LONG, 5000, "6;-7 -4 4"), (emac.FLOAT, 30011, "6;1 -2 2 1 2 1 -2 2"),
         (emac.DOUBLE, 999, "6;-5 -2 2 1 2 3 -2 2")]),
])
def test_comm_program_over_gloo(world, cases):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + world * 7 + os.getpid() % 200
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert [f for r in results for f in r] == []


def _nodes_worker(rank, world, port, cases, q, nodes=2, ports=None):
    """`nodes` nodes of world // nodes ranks: the node legs, per step the node-pair legs and
    their fold, the exchanges back in reverse step order"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    failures = []
    R = world // nodes
    nx, na = emac.node_steps(nodes, ports)
    SH = emac.LEG_STEP_SHIFT
    for code, count, copyin in cases:
        sends = xorshift_inputs(world, count, code, seed_base=0x2A0DE000 + count)
        dt = NP[code]
        itemsize = np.dtype(dt).itemsize
        ops, folds, stage = emac.comm_program_nodes(nodes, R, rank, count, code, copyin, ports=ports)
        bufs = {emac.BUF_SEND: sends[rank].view(np.uint8).copy(),
                emac.BUF_RECV: np.full(count * itemsize, 0xAB, dtype=np.uint8),
                emac.BUF_STAGE: np.zeros(max(stage, 1), dtype=np.uint8)}
        desc = emac.plan_describe(R, count, code, copyin, 0)
        _run_leg(ops, LEG_RS, bufs)
        _fold([f[:3] for f in folds if f[3] == emac.LEG_FOLD], bufs, code, desc)
        for st in range(nx):
            _run_leg(ops, emac.LEG_NODES_RS | st << SH, bufs)
            for off, n, leaves, leg in folds:
                if leg != emac.LEG_NODES_FOLD | st << SH:
                    continue
                xs = [bufs[b][o:o + n * itemsize].view(dt).copy() for b, o in leaves]
                acc = xs[0]
                with np.errstate(over="ignore"):
                    for x in xs[1:]:  # a left fold in the listed order
                        acc = acc + x
                bufs[emac.BUF_RECV][off:off + n * itemsize].view(dt)[:] = acc
        for j in range(na):  # the copying allgather steps, block growing
            _run_leg(ops, emac.LEG_NODES_AG | j << SH, bufs)
        _run_leg(ops, LEG_AG, bufs)
        want = oracle.allreduce_nodes(sends, copyin, nodes, ports=ports)[rank]
        if not np.array_equal(bufs[emac.BUF_RECV], want.view(np.uint8)):
            failures.append((rank, code, count, copyin))
    q.put(failures)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,cases", [
    (2, [(emac.FLOAT, 100003, "6;1 -1 1"), (emac.INT, 7, "6;1 -1 1"), (emac.DOUBLE, 1, "6;1 -1 1")]),
    (4, [(emac.FLOAT, 65539, "6;1 -2 2"), (emac.DOUBLE, 4099, "6;3 -2 2"), (emac.LONG, 1001, "6;-5 -2 2"),
         (emac.FLOAT, 0, "6;1 -2 2"), (emac.FLOAT, 3, "6;1 -2 2")]),
    (8, [(emac.FLOAT, 30011, "6;1 -2 -2 2 2"), (emac.DOUBLE, 9999, "7;1 -4 4"), (emac.INT, 5003, "5;1 -4 4"),
         (emac.FLOAT, 20000, "6;1 -2 2 1 2 1 -2 2")]),
])
def test_two_node_program_over_gloo(world, cases):
    """§8(f3), two nodes and one port: the COMM program of emac_comm_program_nodes executed over
    gloo (ranks [0, world/2) are node 0) equals the oracle's two-node emulation bitwise."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29800 + world * 7 + os.getpid() % 200
    procs = [ctx.Process(target=_nodes_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert [f for r in results for f in r] == []


@pytest.mark.parametrize("world,nodes,cases", [
    (4, 4, [(emac.FLOAT, 100003, "6;1 -1 1"), (emac.DOUBLE, 7, "6;1 -1 1")]),
    (8, 4, [(emac.FLOAT, 65539, "6;1 -2 2"), (emac.INT, 4099, "6;3 -2 2"), (emac.DOUBLE, 1001, "7;1 -2 2")]),
    (8, 8, [(emac.FLOAT, 30011, "6;1 -1 1"), (emac.LONG, 999, "6;1 -1 1")]),
])
def test_many_node_program_over_gloo(world, nodes, cases):
    """2^k nodes, one port per step: emac_comm_program_nodes over gloo equals the oracle bitwise."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29900 + world * 7 + nodes + os.getpid() % 200
    procs = [ctx.Process(target=_nodes_worker, args=(r, world, port, cases, q, nodes)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert [f for r in results for f in r] == []


def test_two_node_program_shape():
    # rank 5 = node 1, local rank 1 of 4: node legs with ranks 4..7, node-pair legs with rank 1
    ops, folds, stage = emac.comm_program_nodes(2, 4, 5, 4 * 1000, emac.FLOAT, "6;1 -4 4")
    assert {o[1] for o in ops if o[0] in (LEG_RS, LEG_AG)} == {4, 6, 7}
    pair = [o for o in ops if o[0] in (emac.LEG_NODES_RS, emac.LEG_NODES_AG)]
    assert {o[1] for o in pair} == {1} and len(pair) == 4
    node_folds = [f for f in folds if f[3] == emac.LEG_NODES_FOLD]
    assert len(node_folds) == 1
    off, n, leaves, _ = node_folds[0]
    assert (off, n) == ((1000 + 500) * 4, 500)  # node 1 finishes the second half of chunk 1
    # raw_code.c's accumulator at the last step: the partner's partial (received), then the own
    assert leaves[1] == (emac.BUF_RECV, off) and leaves[0][0] == emac.BUF_STAGE


def test_comm_program_shape():
    ops, folds, stage = emac.comm_program(8, 3, 8 * 1000, emac.FLOAT, "6;1 -8 8")
    rs = [o for o in ops if o[0] == LEG_RS]
    ag = [o for o in ops if o[0] == LEG_AG]
    assert len(rs) == 14 and len(ag) == 14  # one send + one recv per peer and leg, one round each
    assert sorted({o[1] for o in ops}) == [0, 1, 2, 4, 5, 6, 7]
    assert len(folds) == 1 and folds[0][0] == 3 * 1000 * 4 and folds[0][1] == 1000
    # leaf 0 of rank 3's chunk is its own send buffer; the others come from staging slots
    assert folds[0][2][0] == (emac.BUF_SEND, 12000)
    assert all(b == emac.BUF_STAGE for b, _ in folds[0][2][1:])
    assert all(off % 16 == 0 for b, off in folds[0][2][1:])
    assert stage >= 7 * 4000


def _ipc_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def ag(payload):
        calls.append(len(payload))
        return emac.torch_allgather()(payload)
    try:
        emac.comm_init_ipc(rank, world, ag, -1)
        q.put((rank, "no error", calls))
    except emac.ExtMpiError as e:
        q.put((rank, e.code, calls))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ipc_bootstrap_over_gloo_without_gpu(world):
    """The peer-mapped communicator's set-up is collective: without a device every rank still
    takes part in the same bootstrap exchanges (no rank left waiting) and all fail loudly with
    ERROR_DEVICE instead of falling back to the CPU."""
    if torch.cuda.is_available():
        pytest.skip("GPU present: tests/test_gpu_peer_mapped.py covers the working path")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + world * 7 + os.getpid() % 200
    procs = [ctx.Process(target=_ipc_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert [r[1] for r in results] == [-5] * world
    assert len({tuple(r[2]) for r in results}) == 1 and results[0][2]  # same exchanges on every rank


@pytest.mark.parametrize("world,nodes,ports,cases", [
    (3, 3, [-2, 2], [(emac.FLOAT, 100003, "6;1 -1 1"), (emac.DOUBLE, 7, "6;1 -1 1"), (emac.FLOAT, 2, "6;1 -1 1")]),
    (6, 3, [-2, 2], [(emac.FLOAT, 65539, "6;1 -2 2"), (emac.INT, 4099, "6;3 -2 2"), (emac.DOUBLE, 1001, "7;1 -2 2")]),
    (4, 4, [-3, 3], [(emac.FLOAT, 30011, "6;1 -1 1"), (emac.LONG, 999, "6;1 -1 1")]),
    (6, 6, [-1, -2, 2, 1], [(emac.FLOAT, 40009, "6;1 -1 1"), (emac.DOUBLE, 6007, "6;1 -1 1")]),
    (8, 8, [-3, -1, 1, 3], [(emac.FLOAT, 40009, "6;1 -1 1")]),
    (8, 4, [-1, -1, 1, 1], [(emac.FLOAT, 20011, "6;1 -2 2")]),
    # allgather steps that reduce (README "4(3)", "4(-1 1 1)", "4(1 1)"): nodes may disagree
    (4, 4, [3], [(emac.FLOAT, 30011, "6;1 -1 1"), (emac.INT, 77, "6;1 -1 1")]),
    (8, 4, [-1, 1, 1], [(emac.FLOAT, 20011, "6;1 -2 2")]),
    (4, 4, [1, 1], [(emac.DOUBLE, 9001, "6;1 -1 1")]),
    (6, 6, [-1, 2, 1], [(emac.FLOAT, 12001, "6;1 -1 1")]),
    (6, 3, [2], [(emac.FLOAT, 12001, "6;1 -2 2")]),
    # radix-2 reduce-scatter steps with other allgather radices: the lines are followed
    (4, 4, [-1, -1, 3], [(emac.FLOAT, 20011, "6;1 -1 1")]),
    (8, 8, [-1, -1, -1, 3, 1], [(emac.FLOAT, 20011, "6;1 -1 1")]),
])
def test_node_ports_program_over_gloo(world, nodes, ports, cases):
    """Several ports per step (EXT_MPI_NUM_PORTS "N(-p ... p ...)", radix-3/4 node steps, mixed
    radices): the program of emac_comm_program_nodes over gloo equals the oracle's task-by-task
    restatement of allreduce_core bitwise."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30100 + world * 7 + nodes * 3 + len(ports) + os.getpid() % 200
    procs = [ctx.Process(target=_nodes_worker, args=(r, world, port, cases, q, nodes, ports)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert [f for r in results for f in r] == []


def test_single_step_node_ports_program_is_balanced():
    """One reduce-scatter step over every node ("3(-2 2)"): each rank trades an equal share of its
    chunk -- (N-1)/N of it each way -- whatever lines the chunk lies in, and its folds follow the
    lines inside its share."""
    nodes, R, count = 3, 4, 3 * 4 * 1000 + 7
    for rank in range(nodes * R):
        ops, folds, _ = emac.comm_program_nodes(nodes, R, rank, count, emac.FLOAT, "6;1 -4 4", ports=[-2, 2])
        chunk = [f for f in folds if f[3] == emac.LEG_FOLD][0][1]
        sent = sum(o[5] for o in ops if o[0] == emac.LEG_NODES_RS and o[2]) // 4
        got = sum(o[5] for o in ops if o[0] == emac.LEG_NODES_RS and not o[2]) // 4
        assert abs(sent - 2 * chunk / 3) <= 2 and abs(got - 2 * chunk / 3) <= 2, (rank, chunk, sent, got)
        node_folds = [f for f in folds if f[3] == emac.LEG_NODES_FOLD]
        assert node_folds and all(len(f[2]) == nodes for f in node_folds)
        assert abs(sum(f[1] for f in node_folds) - chunk / 3) <= 1


@pytest.mark.parametrize("nodes,ports,code", [
    (4, [-1, -1], emac.ERROR_UNSUPPORTED),      # ends in a reduce-scatter port: reduce_scatter_core
    (4, [-1, 2, 1], emac.ERROR_ARG),            # allgather radices 3 x 2 != 4 nodes
    (4, [-3, 1, 1, 1], emac.ERROR_ARG),         # allgather radices multiply to 8
    (6, [-1, 2, 1], None), (4, [3], None), (4, [1, 1], None), (8, [-1, -1, -1, 1, 1, 1], None),
    (4, [-1, 2, 1, -1], emac.ERROR_UNSUPPORTED),  # a reduce-scatter port after the allgather ports
])
def test_node_ports_validation(nodes, ports, code):
    """The inter-node list is checked as allreduce_core needs it (emac_node_sched_build)."""
    if code is None:
        emac.comm_program_nodes(nodes, 2, 0, 1000, emac.FLOAT, "6;1 -2 2", ports=ports)
        return
    with pytest.raises(emac.ExtMpiError) as e:
        emac.comm_program_nodes(nodes, 2, 0, 1000, emac.FLOAT, "6;1 -2 2", ports=ports)
    assert e.value.code == code
