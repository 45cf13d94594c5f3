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
    # every failure is named with its transport, exit code and the child's last stderr lines
    fails = ex["failures"]
    assert {f["transport"] for f in fails} == {"node-ipc", "node-rccl", "ipc", "rccl"}
    assert all(f["rc"] != 0 and isinstance(f["stderr_tail"], list) and f["stderr_tail"] for f in fails), fails


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


class _Args:
    steps, warmup, dtype, transport, copyin, size_mib, ranks = 20, 5, "float", "ipc", None, 16.0, 8


MIB = 1 << 20


def _node_ok(world):
    S = 16 * MIB
    return {"wall": 20 * 50e-6, "checked": True, "ranks_per_gpu": 8, "bytes_per_rank": S, "copyin": "6;1 -8 8",
            "ports": [-(world - 1), world - 1], "transport": "ipc", "copy_in_fold_s": 25e-6, "node_legs_s": 20e-6,
            "copy_out_s": 0.0, "schedule": {"unroll": 4, "issue": 5, "tuned": 1}, "nsets": 3,
            "transports": {"ipc": {"ms_per_step": 0.05, "checked": True}}}


def _one_rank_ok(world):
    sweep = [{"dtype": "float", "bytes_per_rank": n, "us_per_allreduce": 10.0, "algbw_gbps": 1.0, "checked": True}
             for n in (8, 64 << 10, 1 << 20, 16 << 20, 64 << 20, 256 << 20, 512 << 20)]
    sweep.append({"dtype": "double", "bytes_per_rank": 256 << 20, "us_per_allreduce": 900.0, "algbw_gbps": 298.0,
                  "checked": True})  # BASELINE configs[3]
    return {"wall": 20 * 60e-6, "checked": True, "fold_s": 8e-6, "alone_s": 7.5e-6, "sweep": sweep,
            "radix_sweep": [], "local_fold": {"leaves": world, "chunk_bytes": 2 * MIB, "us_all_gpus": 4.0,
                                              "us_rank0_alone": 3.9, "rate_retained": 0.975, "schedule": None},
            "host_buffers": {"checked": True}}


REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "config", "roofline", "extras")


@pytest.mark.parametrize("world", [2, 8])
def test_multi_gpu_line_from_fabricated_children(world):
    """multi_gpu's assembly (bench.py multi_gpu_line / node_form_line) from fabricated child
    results: every child ok; the node child failed (exit code, stderr tail); the node child timed
    out and one transport failed; everything timed out. Each case yields one valid line with the
    contract's keys that names what failed."""
    b = _bench()
    S = 16 * MIB
    order = ["ipc", "rccl"]
    ok_line = b.multi_gpu_line(_Args, world, "f32", S, f"6;1 -{world} {world}", _node_ok(world),
                               {"ipc": _one_rank_ok(world), "rccl": {"wall": 1e-3, "checked": True}}, order, world, [])
    json.dumps(ok_line)
    assert all(k in ok_line for k in REQUIRED)
    assert "configs[1]'s node" in ok_line["config"]["workload"] and ok_line["config"]["layout"] == "node-per-gpu"
    assert ok_line["value"] == pytest.approx(world * 8 * S * 20 / (20 * 50e-6) / 1e9, rel=1e-3)
    one = ok_line["extras"]["one_rank_per_gpu"]
    assert any(p["dtype"] == "double" and p["bytes_per_rank"] == 256 << 20 for p in one["extras"]["sweep"])  # configs[3]
    assert "failures" not in ok_line["extras"]

    # the peer-mapped node children failed, RCCL's ran: its line, the failure beside it
    rc_fail, fail = b.child_outcome("node-ipc", 1, 12.5, ["Traceback ...", "RuntimeError: boom"], None)
    assert rc_fail == {} and fail["rc"] == 1 and fail["stderr_tail"][-1] == "RuntimeError: boom"
    rn = b.node_result({"ipc": fail, "rccl": dict(_node_ok(world), transport="rccl")}, _Args.steps)
    assert rn["transport"] == "rccl" and rn["transports"]["ipc"]["rc"] == 1
    line = b.multi_gpu_line(_Args, world, "f32", S, f"6;1 -{world} {world}", rn,
                            {"ipc": _one_rank_ok(world), "rccl": {"wall": 1e-3, "checked": True}}, order, world,
                            [dict(fail, rank=1)])
    assert line["config"]["layout"] == "node-per-gpu" and line["config"]["transport"] == "rccl"
    assert line["extras"]["failures"][0]["transport"] == "node-ipc"
    # both node children failed on one rank: the one-rank-per-GPU line, the node failures named
    rn = b.node_result({"ipc": fail, "rccl": {"error": "failed on another rank"}}, _Args.steps)
    assert rn["checked"] is False and "ipc: node-ipc child exited with 1" in rn["error"]
    line = b.multi_gpu_line(_Args, world, "f32", S, f"6;1 -{world} {world}", rn,
                            {"ipc": _one_rank_ok(world), "rccl": {"wall": 1e-3, "checked": True}}, order, world,
                            [dict(fail, rank=1)])
    json.dumps(line)
    assert all(k in line for k in REQUIRED) and line["config"]["layout"] == "rank-per-gpu" and line["value"] > 0
    assert line["extras"]["node_form_per_gpu"]["transports"]["ipc"]["transport"] == "node-ipc"
    assert line["extras"]["failures"][0]["stderr_tail"][-1] == "RuntimeError: boom"

    # the node child timed out, ipc failed its check, rccl ran: rccl's line
    _, tmo = b.child_outcome("node-ipc", "timeout", 480.0, ["rank 0: node form ..."], None)
    _, bad = b.child_outcome("ipc", 0, 30.0, [], {"wall": 1.0, "checked": False})
    assert tmo["rc"] == "timeout" and "timed out" in tmo["error"] and bad["error"] == "result check failed"
    line = b.multi_gpu_line(_Args, world, "f32", S, f"6;1 -{world} {world}", b.node_result({"ipc": tmo}, 20),
                            {"ipc": bad, "rccl": _one_rank_ok(world)}, order, world, [tmo, bad])
    assert line["config"]["transport"] == "rccl" and line["extras"]["ipc_transport"]["error"] == "result check failed"
    assert line["extras"]["node_form_per_gpu"]["transports"]["ipc"]["rc"] == "timeout"

    # everything timed out: a zero line naming every failure
    fails = [b.child_outcome(t, "timeout", 100.0, ["..."], None)[1] for t in ("node-ipc", "node-rccl", "ipc", "rccl")]
    line = b.multi_gpu_line(_Args, world, "f32", S, f"6;1 -{world} {world}",
                            b.node_result({"ipc": fails[0], "rccl": fails[1]}, 20),
                            {"ipc": fails[2], "rccl": fails[3]}, order, world, fails)
    json.dumps(line)
    assert all(k in line for k in REQUIRED)
    assert line["value"] == 0.0 and line["error"] == "no transport completed"
    assert "ipc: ipc child timed out" in line["config"]["workload"]
    assert [f["transport"] for f in line["extras"]["failures"]] == ["node-ipc", "node-rccl", "ipc", "rccl"]


def test_child_process_limit_kills_and_reports():
    """run_child_process: a child that outlives its limit is killed (its process group) and
    reported as "timeout" with its last stderr lines; one that fails reports its exit code."""
    b = _bench()
    code = "import sys, time\nfor i in range(3): print('line', i, file=sys.stderr, flush=True)\ntime.sleep(60)"
    rc, el, tail = b.run_child_process([sys.executable, "-c", code], dict(os.environ), 3.0)
    assert rc == "timeout" and el < 30 and tail[-1] == "line 2"
    rc, el, tail = b.run_child_process([sys.executable, "-c", "import sys; print('bad', file=sys.stderr); sys.exit(7)"],
                                       dict(os.environ), 30.0)
    assert rc == 7 and tail == ["bad"]


@pytest.mark.parametrize("read_mib", [4 * 8, 16 * 8, 64 * 8, 256 * 8, 512 * 8])
def test_rotation_keeps_every_read_in_hbm(monkeypatch, read_mib):
    """bench.rotation_sets: between two uses of one buffer set, at least READ_REUSE_BYTES (2.5x the
    256 MiB Infinity Cache) of other sets' inputs are read, with no more sets than that needs;
    EXT_MPI_AMD_BENCH_ROTATION=legacy gives rounds 1-3's whole-working-set rule."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv("EXT_MPI_AMD_BENCH_ROTATION", raising=False)
    rd = read_mib * bench.MIB
    n = bench.rotation_sets(rd, 2 * rd)
    assert (n - 1) * rd >= bench.READ_REUSE_BYTES and (n - 2) * rd < bench.READ_REUSE_BYTES and n >= 2
    monkeypatch.setenv("EXT_MPI_AMD_BENCH_ROTATION", "legacy")
    legacy = bench.rotation_sets(rd, 2 * rd)
    assert legacy == max(2, -(-640 * bench.MIB // (2 * rd)))
    if read_mib == 16 * 8:  # the headline: 6 sets now, 3 before
        assert (n, legacy) == (6, 3)


def test_radix_crossover_and_vs_linear():
    """bench.py's configs[4] summary: each point against the linear fold at the same size, and each
    variant's fixed cost, streaming rate and latency -> bandwidth crossover from synthetic times
    t = fixed + R * bytes / rate."""
    sys.path.insert(0, ROOT)
    import bench
    R, pts = 8, []
    for cp, fixed, rate in (("6;1 -8 8", 3.0, 3.0e12), ("6;-64 -8 8", 4.0, 2.0e12)):
        for b in bench.RADIX_SWEEP_BYTES:
            pts.append({"copyin": cp, "bytes_per_rank": b, "us": fixed + R * b / rate * 1e6})
    bench.radix_vs_linear(pts, "6;1 -8 8", "us")
    assert all(p["vs_linear"] == 1.0 for p in pts if p["copyin"] == "6;1 -8 8")
    assert [p["vs_linear"] for p in pts if p["copyin"] != "6;1 -8 8"][0] == 0.75  # 3 / 4 us at 8 B
    x = bench.radix_crossovers(pts, "us", R)
    assert x["6;1 -8 8"]["fixed_us"] == 3.0 and x["6;1 -8 8"]["streaming_gbps_reduced"] == 3000.0
    # fixed cost == streaming time at 3 us * 3 TB/s / 8 ranks per rank
    assert abs(x["6;1 -8 8"]["crossover_bytes_per_rank"] - 3e-6 * 3e12 / 8) < 16
    assert abs(x["6;-64 -8 8"]["crossover_bytes_per_rank"] - 4e-6 * 2e12 / 8) < 16


def test_shared_hw_queues():
    """ranks sharing a GPU get at most 2 hardware queues each, whatever the environment exports
    (the boxes export 4); one rank per GPU leaves the setting alone"""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.shared_hw_queues(8, 8, None) is None
    assert bench.shared_hw_queues(8, 8, "4") is None
    assert bench.shared_hw_queues(1, 8, None) == "2"
    assert bench.shared_hw_queues(1, 8, "4") == "2"
    assert bench.shared_hw_queues(1, 2, "1") == "1"
    assert bench.shared_hw_queues(1, 4, "junk") == "2"
