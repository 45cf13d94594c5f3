"""Peer-mapped (IPC) form on the GPU box: R processes, one rank each, sharing the one MI355X.

Each rank is a separate process (tests/ipc_worker.py) with its own HIP context; the ranks
exchange hipIpc handles through a gloo bootstrap, map each other's send/receive buffers, and
run the persistent Allreduce: barrier kernel -> fold over the peers' leaves with the fan-out
stored into every peer's receive buffer -> barrier kernel. Every rank checks its result bit for
bit against the CPU oracle (float, double, int, long; repeats, in place, host buffers, empty and
one-element messages, -k fractions, pieces, radix chains, a sub-split) and several handles
in flight on separate streams.
"""
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


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


# The barrier does not depend on where its workgroups land (ipc_sync.hpp), so 8 processes sharing
# the one GPU -- the dispatcher interleaving their launches -- run the same cases as 2 to 4.
WORLDS = [int(w) for w in os.environ.get("IPC_TEST_WORLDS", "2,3,4,8").split(",")]


@pytest.mark.parametrize("world", WORLDS)
def test_ipc_ranks_share_one_gpu(world):
    port = _port()
    procs, logs = [], []
    # each rank writes to its own file: pipes read one after the other would fill up and block a
    # rank mid-print (then every peer waits for it in the next collective)
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), IPC_DEVICE="0", EXT_MPI_AMD_BARRIER_TIMEOUT="20")
        env.setdefault("IPC_FUZZ", "16")  # seeded random cases beside the fixed ones (ipc_worker.fuzz_cases)
        logs.append(tempfile.TemporaryFile(mode="w+"))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "ipc_worker.py")], env=env,
                                      stdout=logs[-1], stderr=subprocess.STDOUT, text=True))
    deadline = time.monotonic() + 150
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
    report = "\n".join(outs)
    print(report)
    assert codes == [0] * world, report
    lines = [l for l in report.splitlines() if l.startswith("IPC rank")]
    assert lines and all(l.endswith(": ok") for l in lines), report
    assert len(lines) == world * sum(1 for l in lines if l.startswith("IPC rank 0/")), report
