"""The NODE form over peer-mapped nodes on the GPU box: N processes sharing the one MI355X, each a
node of R ranks (tests/node_ipc_worker.py), joined by an ext_mpi_amd_comm_init_ipc communicator
(engine.c node_ipc_init). This is the form bench.py's N > 1 headline runs first (one node of 8
ranks per GPU); on one GPU the nodes' peer loads stay on the device, the bits are the same. Every
node checks its receive buffers bit for bit against the oracle's multi-node restatement."""
import os
import socket
import subprocess
import sys
import tempfile
import time

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_nodes(nodes, budget=180, **extra_env):
    port = _port()
    procs, logs = [], []
    for r in range(nodes):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(nodes), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), IPC_DEVICE="0", EXT_MPI_AMD_BARRIER_TIMEOUT="20", **extra_env)
        logs.append(tempfile.TemporaryFile(mode="w+"))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "node_ipc_worker.py")],
                                      env=env, stdout=logs[-1], stderr=subprocess.STDOUT, text=True))
    deadline = time.monotonic() + budget
    codes = []
    for p in procs:
        try:
            p.wait(timeout=max(1.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            p.wait()
        codes.append(p.returncode)
    outs = []
    for f in logs:
        f.seek(0)
        outs.append(f.read())
        f.close()
    bad = [l for o in outs for l in o.splitlines() if l.startswith("NODEIPC") and not l.endswith(": ok")]
    tails = "\n".join(f"--- node {r}: exit {c}\n" + "\n".join(o.splitlines()[-12:]) for r, (o, c) in
                      enumerate(zip(outs, codes)))
    assert codes == [0] * nodes and not bad, "\n".join(bad[:20]) + "\n" + tails
    lines = [l for o in outs for l in o.splitlines() if l.startswith("NODEIPC")]
    assert lines and len(lines) == nodes * sum(1 for l in lines if l.startswith("NODEIPC node 0/")), tails
    print("\n".join(l for l in lines if l.startswith("NODEIPC node 0/")))


@pytest.mark.parametrize("nodes", [2, 3, 4, 8])
def test_node_form_over_peer_mapped_nodes(nodes):
    """the default join: serial under 1 MiB per rank, the fused one of 2 parts from there
    (engine_join.c join_parts)"""
    _run_nodes(nodes, budget=300 if nodes >= 8 else 180)


@pytest.mark.parametrize("join", ["serial", "fused3", "fused4", "streams3"])
@pytest.mark.parametrize("nodes", [2, 3, 4, 8])
def test_node_join_serial_and_pipelined(nodes, join):
    """every case with the join serial (EXT_MPI_AMD_JOIN_PARTS=1) or pipelined by 3 or 4 parts at
    every size (parts of no element, buckets cut inside their tiles) -- in one launch per Start
    (join_fused.hip; shapes it has no kernel for fall back to the serial join) or on three streams
    (EXT_MPI_AMD_JOIN=streams) -- plus the timeout recovery of a late node over every part's slot"""
    parts = "1" if join == "serial" else join[-1]
    env = dict(EXT_MPI_AMD_JOIN_PARTS=parts, NODEIPC_RECOVERY="1")
    if join.startswith("streams"):
        env["EXT_MPI_AMD_JOIN"] = "streams"
    _run_nodes(nodes, budget=300 if nodes >= 8 else 180, **env)
