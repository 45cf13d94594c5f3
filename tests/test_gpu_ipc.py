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


def _digest(outs, codes, keep=40):
    """Per rank: its exit code, every line that is not a passing case (set-up retries, errors,
    tracebacks) -- repeated lines counted once -- and its last lines; bounded, so a failing run's
    report stays readable."""
    parts = []
    for r, (out, code) in enumerate(zip(outs, codes)):
        lines = out.splitlines()
        seen, odd = {}, []
        for l in lines:
            if l.endswith(": ok"):
                continue
            if l not in seen:
                odd.append(l)
            seen[l] = seen.get(l, 0) + 1
        odd = [f"{l}  (x{seen[l]})" if seen[l] > 1 else l for l in odd[:keep]]
        parts.append(f"--- rank {r}: exit {code}, {len(lines)} lines\n" + "\n".join(odd) +
                     "\n... last lines:\n" + "\n".join(lines[-8:]))
    return "\n".join(parts)


@pytest.mark.parametrize("world", WORLDS)
def test_ipc_ranks_share_one_gpu(world):
    port = _port()
    procs, logs = [], []
    # each rank writes to its own file: pipes read one after the other would fill up and block a
    # rank mid-print (then every peer waits for it in the next collective)
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), IPC_DEVICE="0", EXT_MPI_AMD_BARRIER_TIMEOUT="20")
        env.setdefault("EXT_MPI_AMD_DEBUG_IPC", "1")  # set-up retries are reported (silent when none)
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
    print(_digest(outs, codes))
    assert codes == [0] * world, _digest(outs, codes)
    lines = [l for l in report.splitlines() if l.startswith("IPC rank")]
    assert lines and all(l.endswith(": ok") for l in lines), _digest(outs, codes)
    assert len(lines) == world * sum(1 for l in lines if l.startswith("IPC rank 0/")), _digest(outs, codes)
