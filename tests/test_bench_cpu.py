"""bench.py's N > 1 driver on the CPU: two torchrun ranks (gloo), no GPU.

Each transport runs in child processes of its own (one per rank, own gloo group); here both
children fail (no device), and the ranks must still agree on it, try the other transport, and
end with rank 0's single JSON line reporting that no transport completed -- the path a real node
takes when a transport fails, exercised without one.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_multi_rank_transport_isolation_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present: the real N > 1 path runs instead")
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    # stdout carries the one result line and nothing else (gloo / RCCL chatter goes to stderr)
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] == 0.0 and out["error"] == "no transport completed"
    ex = out["extras"]
    assert ex["process_per_transport"] is True
    assert "error" in ex["ipc_transport"] and "error" in ex["rccl_transport"]
