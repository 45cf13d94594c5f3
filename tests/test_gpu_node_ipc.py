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


def _run_nodes(nodes, budget=180, rank_env=None, **extra_env):
    """Run `nodes` node_ipc_worker processes (rank_env(r): extra environment of node r only); every
    case line of every node must end in ': ok'. Returns node 0's case lines."""
    port = _port()
    procs, logs = [], []
    for r in range(nodes):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(nodes), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), IPC_DEVICE="0", EXT_MPI_AMD_BARRIER_TIMEOUT="20", **extra_env)
        env.update(rank_env(r) if rank_env else {})
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
    for r in range(1, nodes):  # every node ran every case with the same join (parts agreed on rank 0's)
        assert [l.split("join parts")[-1] for l in lines if l.startswith(f"NODEIPC node {r}/") and "join parts" in l] == \
            [l.split("join parts")[-1] for l in lines if l.startswith("NODEIPC node 0/") and "join parts" in l], tails
    return [l for l in lines if l.startswith("NODEIPC node 0/")]


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


@pytest.mark.parametrize("join", ["default", "serial", "fused3", "fused4"])
@pytest.mark.parametrize("nodes", [2, 4, 8])
def test_node_join_cross_device_code(nodes, join):
    """The code an 8-GPU node runs, on one GPU: EXT_MPI_AMD_TEST_CROSS_DEVICE=1 makes the
    communicator's agreed verdict 'some node is on another device' (engine_ipc.c) while the nodes
    still share this GPU, so every Start records the system-scope release before phase 0 and the
    fused join runs join_fused_kernel<..., true> (system-scope partial stores), its grid still
    divided among the nodes on this GPU (by UUID). Every case bitwise against the oracle; every
    handle's flags (tests/helpers.py ipc_flags_problem) say the cross-GPU code ran; plus the
    timeout recovery over every part's slot. Reference synchronisation replaced:
    ext_mpi_native_exec.c:21-84, cuda_shmem.c:218-299."""
    env = dict(EXT_MPI_AMD_TEST_CROSS_DEVICE="1", NODEIPC_RECOVERY="1")
    if join != "default":
        env["EXT_MPI_AMD_JOIN_PARTS"] = "1" if join == "serial" else join[-1]
    _run_nodes(nodes, budget=300 if nodes >= 8 else 180, **env)


def test_node_join_settings_follow_rank0():
    """The join's settings are rank 0's: node 0 asks for 3 parts, the others for the
    serial join; every node must run 3 parts from 1 MiB per rank (and the same join on every case),
    bitwise -- a disagreement would run different slot protocols and time out every Start."""
    lines = _run_nodes(4, rank_env=lambda r: {"EXT_MPI_AMD_JOIN_PARTS": "3" if r == 0 else "1"})
    assert any(l.endswith("join parts 3: ok") for l in lines), lines
