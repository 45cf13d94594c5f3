"""Peer-mapped (IPC) form on the GPU box: R processes, one rank each, sharing the one MI355X.

Each rank is a separate process (tests/ipc_worker.py) with its own HIP context; the ranks
exchange hipIpc handles through a gloo bootstrap, map each other's send buffers and result
buffers ("outboxes"), and run the persistent Allreduce: barrier -> fold of the owner chunks over
the peers' leaves into the outbox -> barrier -> pull of every owner's result into the own receive
buffer. Every rank checks its result bit for bit against the CPU oracle (float, double, int,
long; repeats, in place, host buffers, empty and one-element messages, -k fractions, pieces,
radix chains, a sub-split), freed and re-allocated buffers, and several handles in flight on
separate streams. (Named to sort after test_gpu_parity.py: the single-process parity suite runs
first under `pytest -x`.)
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


def _digest(outs, codes, keep=12):
    """First every rank's exit code and failing cases (so a truncated report still names every
    rank that failed), then per rank every other line that is not a passing case (set-up retries,
    errors, tracebacks) -- repeated lines counted once -- and its last lines."""
    head, parts = [], []
    for r, (out, code) in enumerate(zip(outs, codes)):
        lines = out.splitlines()
        bad = [l for l in lines if l.startswith("IPC rank") and not l.endswith(": ok")]
        head.append(f"rank {r}: exit {code}, {len(bad)} failing case(s)" + "".join("\n  " + l for l in bad[:6]))
        seen, odd = {}, []
        for l in lines:
            if l.endswith(": ok") or l in bad:
                continue
            if l not in seen:
                odd.append(l)
            seen[l] = seen.get(l, 0) + 1
        odd = [f"{l}  (x{seen[l]})" if seen[l] > 1 else l for l in odd[:keep]]
        parts.append(f"--- rank {r}: exit {code}, {len(lines)} lines\n" + "\n".join(odd) +
                     "\n... last lines:\n" + "\n".join(lines[-4:]))
    return "\n".join(head) + "\n" + "\n".join(parts)


def _run_world(world, extra_env=None, budget=None):
    port = _port()
    procs, logs = [], []
    # each rank writes to its own file: pipes read one after the other would fill up and block a
    # rank mid-print (then every peer waits for it in the next collective)
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), IPC_DEVICE="0", EXT_MPI_AMD_BARRIER_TIMEOUT="20")
        env.setdefault("EXT_MPI_AMD_DEBUG_IPC", "1")  # set-up retries are reported (silent when none)
        env.setdefault("IPC_FUZZ", "16")  # seeded random cases beside the fixed ones (ipc_worker.fuzz_cases)
        env.update(extra_env or {})
        logs.append(tempfile.TemporaryFile(mode="w+"))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "ipc_worker.py")], env=env,
                                      stdout=logs[-1], stderr=subprocess.STDOUT, text=True))
    # 8 processes time-share the one GPU: every set-up round trip and barrier is slower there
    deadline = time.monotonic() + (budget or (300 if world >= 8 else 150))
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
    return report


@pytest.mark.parametrize("world", WORLDS)
def test_ipc_ranks_share_one_gpu(world):
    _run_world(world)


@pytest.mark.parametrize("world", [3, 8])
def test_ipc_forced_mirror(world):
    """EXT_MPI_AMD_IPC_FORCE_MIRROR=1: every rank's exported send buffer is re-placed in
    the first set-up round of every handle (an arena mirror), so the mirror path -- staged send buffers, a second
    exchange, re-validated mappings -- runs on every case, bitwise against the oracle."""
    report = _run_world(world, {"EXT_MPI_AMD_IPC_FORCE_MIRROR": "1", "IPC_FUZZ": "4",
                                "IPC_SECTIONS": "realloc,newdata,concurrent,recycle"})
    assert "re-placing send" in report  # the forced round was taken (EXT_MPI_AMD_DEBUG_IPC)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ipc_cross_device_code(world):
    """EXT_MPI_AMD_TEST_CROSS_DEVICE=1: the ranks' agreed verdict is 'some peer on another device'
    though all share this GPU, so every Start records the system-scope release before phase 0 (the
    code one rank per GPU runs, engine_ipc.c); every case bitwise against the oracle and every
    handle's flags checked (ipc_worker.py), timeout recovery included."""
    _run_world(world, {"EXT_MPI_AMD_TEST_CROSS_DEVICE": "1"})
