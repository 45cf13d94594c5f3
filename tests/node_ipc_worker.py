"""One node of the NODE form over peer-mapped nodes, run as its own process by test_gpu_node_ipc.py.

Every process is a node of R ranks (all their buffers in this process, on its GPU); the nodes are
joined by an ext_mpi_amd_comm_init_ipc communicator (engine.c node_ipc_init: the node's copy-in
into a partial block the peers map, the fold of this node's share of every node rank's chunk over
the N partials read in place, the pull of every share into the chunk owners' receive buffers, the
copy-out). Every node runs the same cases in the same order, regenerates every global rank's input
(node-major: rank me of node n is global rank n * R + me), checks its R receive buffers bit for bit
against the oracle's multi-node restatement (oracle.allreduce_nodes: reduce_copyin over the node,
allreduce_core between the nodes under the EXT_MPI_NUM_PORTS list, reduce_copyout) and prints one
line per case. Exit status 0 iff every case matched.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ext_mpi_collectives_amd as emac  # noqa: E402
from helpers import ipc_flags_problem, xorshift_inputs  # noqa: E402
from oracle import oracle  # noqa: E402

TORCH = {emac.FLOAT: torch.float32, emac.DOUBLE: torch.float64, emac.INT: torch.int32, emac.LONG: torch.int64}


def cases(N):
    """(dtype, count, R, copyin, ports, op, repeats, in_place, host); ports None = the default list"""
    single = [-(N - 1), N - 1]
    out = [(emac.FLOAT, 40961, 4, "6;1 -4 4", single, emac.SUM, 3, False, False),
           (emac.DOUBLE, 100003, 2, "6;1 -2 2", single, emac.SUM, 2, False, False),
           (emac.INT, 65536 * 4 + 5, 4, "6;1 -2 -2 2 2", single, emac.SUM, 1, False, False),
           (emac.LONG, 777, 1, "6;1 -1 1", single, emac.SUM, 1, False, False),
           (emac.FLOAT, 1, 2, "6;1 -2 2", single, emac.SUM, 1, False, False),
           (emac.FLOAT, 0, 2, "6;1 -2 2", single, emac.SUM, 1, False, False),
           (emac.FLOAT, 5, 8, "6;1 -8 8", single, emac.SUM, 1, False, False),
           (emac.FLOAT, 100000, 4, "6;1 -4 4", single, emac.SUM, 2, True, False),
           (emac.DOUBLE, 33333, 2, "6;1 -2 2", single, emac.SUM, 2, False, True),
           (emac.FLOAT, 5000, 4, "6;-64 -4 4", single, emac.SUM, 1, False, False),
           (emac.DOUBLE, 70001, 4, "6;3 -4 4", single, emac.SUM, 1, False, False),
           (emac.FLOAT, 100003, 4, "7;1 -2 -2 2 2", single, emac.SUM, 1, False, False),
           (emac.DOUBLE, 4099, 4, "5;1 -4 4", single, emac.SUM, 1, False, False),
           # configs[1]'s node (8 ranks x 16 MiB) on every process: the bench's N > 1 headline
           (emac.FLOAT, 4 << 20, 8, "6;1 -8 8", single, emac.SUM, 2, False, False)]
    if N > 2:  # MIN / MAX: one step over every node keeps the line's order (two nodes at one port: SUM only)
        out += [(emac.FLOAT, 100003, 4, "6;1 -4 4", single, emac.MIN, 1, False, False),
                (emac.LONG, 77777, 2, "6;1 -2 2", single, emac.MAX, 1, False, False)]
    if N == 3:  # the default list for 3 nodes is the one step
        out += [(emac.FLOAT, 65539, 4, "6;1 -4 4", None, emac.SUM, 1, False, False)]
    if N & (N - 1) == 0:  # one port per step (the default for 2^k nodes): pairs over the task bits, SUM
        out += [(emac.DOUBLE, 65539, 4, "6;1 -4 4", None, emac.SUM, 1, False, False),
                (emac.FLOAT, 100003, 2, "6;1 -2 2", None, emac.SUM, 2, False, False),
                (emac.FLOAT, 4 << 20, 8, "6;1 -8 8", None, emac.SUM, 1, False, False),
                (emac.FLOAT, 100, 4, "6;-64 -4 4", None, emac.SUM, 1, False, False)]  # ranks with no elements
    return out


def unsupported(N):
    """lists the peer-mapped join refuses (MIN / MAX at one port per step, allgather steps that
    reduce): every node gets ERROR_UNSUPPORTED from the same collective call and goes on"""
    out = [(emac.FLOAT, 1000, 2, "6;1 -2 2", None, emac.MIN)] if N & (N - 1) == 0 else []
    if N == 4:
        out += [(emac.FLOAT, 1000, 2, "6;1 -2 2", [3], emac.SUM)]  # '4(3)': the allgather steps reduce
    return out


def timeout_recovery(node, N, dev):
    """A late node costs one Start, not the communicator (ipc_sync.hpp), in the serial and in the
    pipelined join (every part's slot): on a communicator with a 0.3 s barrier timeout node 1 starts
    its second Allreduce 1 s late. Every node must report that Start as failed (ERROR_TRANSPORT) and
    the next Start on the same handle must be bit-exact again."""
    saved = os.environ.get("EXT_MPI_AMD_BARRIER_TIMEOUT")
    os.environ["EXT_MPI_AMD_BARRIER_TIMEOUT"] = "0.3"
    comm = emac.comm_init_ipc(node, N, emac.torch_allgather(), dev)
    os.environ["EXT_MPI_AMD_BARRIER_TIMEOUT"] = saved if saved is not None else ""
    if saved is None:
        del os.environ["EXT_MPI_AMD_BARRIER_TIMEOUT"]
    emac.comm_set_nodes(comm, N, [-(N - 1), N - 1])
    R, count = 2, 1 << 20  # 4 MiB per rank: the pipelined join's size by default
    sbufs = [torch.full((count,), float(node * R + me + 1), device="cuda") for me in range(R)]
    rbufs = [torch.empty_like(s) for s in sbufs]
    want = float(N * R * (N * R + 1) // 2)
    h = emac.node_comm_allreduce_init([s.data_ptr() for s in sbufs], [r.data_ptr() for r in rbufs], count, emac.FLOAT,
                                      comm, "6;1 -2 2")
    parts = emac.handle_join_parts(h)
    why = ipc_flags_problem(h, N, parts)
    verdicts = [why] if why else []
    for it in range(3):
        dist.barrier()
        for r in rbufs:
            r.fill_(-1.0)
        torch.cuda.synchronize()
        if it == 1 and node == 1:
            time.sleep(1.0)
        try:
            emac.start(h)
            emac.wait(h)
            verdicts.append("ok" if all(bool((r == want).all()) for r in rbufs) else "wrong")
        except emac.ExtMpiError as e:
            verdicts.append("failed" if e.code == emac.ERROR_TRANSPORT else str(e))
    dist.barrier()
    emac.done(h)
    emac.comm_free(comm)
    ok = verdicts == ["ok", "failed", "ok"]
    print(f"NODEIPC node {node}/{N} timeout recovery (join parts {parts}): "
          f"{'ok' if ok else verdicts}", flush=True)
    return ok


def main():
    node, N = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("IPC_DEVICE", "0"))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    comm = emac.comm_init_ipc(node, N, emac.torch_allgather(), dev)
    failures = 0
    for k, (code, count, R, copyin, ports, op, repeats, in_place, host) in enumerate(cases(N)):
        emac.comm_set_nodes(comm, N if ports is not None else 1, ports)  # 1: the default list
        W = N * R
        sbufs, rbufs, hbufs = [], [], []
        for me in range(R):
            if host:
                hs = np.zeros(count, dtype=xorshift_inputs(1, 1, code)[0].dtype)
                hr = np.full_like(hs, -1)
                hbufs.append((hs, hr))
                sbufs.append(hs.ctypes.data)
                rbufs.append(hr.ctypes.data)
            else:
                s = torch.zeros(count, dtype=TORCH[code], device="cuda")
                r = s if in_place else torch.full((count,), -1, dtype=TORCH[code], device="cuda")
                hbufs.append((s, r))
                sbufs.append(s.data_ptr())
                rbufs.append(r.data_ptr())
        h = emac.node_comm_allreduce_init(sbufs, rbufs, count, code, comm, copyin, op=op)
        parts = emac.handle_join_parts(h)
        ok = True
        why = ipc_flags_problem(h, N, parts)
        if why:
            print(f"node {node}/{N} case {k}: {why}", flush=True)
            ok = False
        for rep in range(repeats):
            sends = xorshift_inputs(W, count, code, seed_base=0x40DE0000 + 977 * k + 31 * rep)
            want = oracle.allreduce_nodes(sends, copyin, N, ports=ports if ports is not None else
                                          (emac.default_node_ports(N) if N & (N - 1) else None),
                                          in_place=in_place, op=op)
            for me in range(R):
                s, r = hbufs[me]
                if host:
                    s[:] = sends[node * R + me]
                    r[:] = -1
                else:
                    s.copy_(torch.from_numpy(sends[node * R + me]))
                    if not in_place:
                        r.fill_(-1)
            torch.cuda.synchronize()
            emac.start(h)
            emac.wait(h)
            for me in range(R):
                s, r = hbufs[me]
                got = r if host else r.cpu().numpy()
                w = want[node * R + me]
                if not np.array_equal(got.view(np.uint8), w.view(np.uint8)):
                    bad = np.flatnonzero(got.view(np.uint8) != w.view(np.uint8))
                    print(f"node {node}/{N} case {k} rep {rep} rank {me}: {bad.size} differing bytes, first at "
                          f"byte {bad[0]}", flush=True)
                    ok = False
        emac.done(h)
        failures += not ok
        print(f"NODEIPC node {node}/{N} case {k} code {code} op {op} count {count} R {R} '{copyin}' ports {ports} "
              f"in_place={in_place} host={host} x{repeats} join parts {parts}: {'ok' if ok else 'MISMATCH'}", flush=True)
    for k, (code, count, R, copyin, ports, op) in enumerate(unsupported(N)):
        emac.comm_set_nodes(comm, N if ports is not None else 1, ports)
        bufs = [torch.zeros(count, dtype=TORCH[code], device="cuda") for _ in range(2 * R)]
        try:
            h = emac.node_comm_allreduce_init([b.data_ptr() for b in bufs[:R]], [b.data_ptr() for b in bufs[R:]], count,
                                              code, comm, copyin, op=op)
            emac.done(h)
            res = "accepted"
        except emac.ExtMpiError as e:
            res = "refused" if "UNSUPPORTED" in str(e) else f"error {e}"
        ok = res == "refused"
        failures += not ok
        print(f"NODEIPC node {node}/{N} refusal {k} op {op} ports {ports}: {'ok' if ok else res}", flush=True)
    emac.comm_free(comm)
    if os.environ.get("NODEIPC_RECOVERY"):
        failures += not timeout_recovery(node, N, dev)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(1 if failures else 0)


if __name__ == "__main__":
    main()
