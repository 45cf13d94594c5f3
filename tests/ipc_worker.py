"""One rank of the peer-mapped (IPC) form, run as its own process by test_gpu_peer_mapped.py.

Every rank runs the same cases in the same order; for each it regenerates every rank's input
(seeded per rank), checks its own receive buffer bit for bit against the CPU oracle and prints
one line per case. Several ranks may share one GPU: the hipIpc mappings, the barrier kernels and
the fan-out stores are then the same code the 8-GPU node runs, over the one device's memory.
Exit status 0 iff every case matched.
"""
import ctypes
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


def cases(R):
    full = f"6;1 -{R} {R}"
    out = [(emac.FLOAT, 40961, full, False, False, 3), (emac.DOUBLE, 1000003, full, False, False, 2),
           (emac.INT, 65536 * R + 5, full, False, False, 1), (emac.LONG, 777, full, False, False, 1),
           (emac.FLOAT, 1, full, False, False, 1), (emac.FLOAT, 0, full, False, False, 1),
           (emac.FLOAT, 100000, full, True, False, 2), (emac.DOUBLE, 33333, full, False, True, 2),
           (emac.FLOAT, 5000, f"6;-64 -{R} {R}", False, False, 1), (emac.FLOAT, 70001, f"6;3 -{R} {R}", False, False, 1),
           # small raw hipMalloc buffers (sub-allocated by the runtime: not exported, staged through mirrors)
           (emac.INT, 12345, full, False, "raw", 2), (emac.FLOAT, 3001, full, True, "raw", 1),
           # MIN / MAX (the reference's CPU reduction, ext_mpi_native_exec.c:240-318)
           (emac.FLOAT, 100003, full, False, False, 2, emac.MIN), (emac.LONG, 77777, full, False, False, 1, emac.MAX),
           (emac.DOUBLE, 4099, f"6;-64 -{R} {R}", True, False, 1, emac.MAX)]
    if R == 4:
        out += [(emac.FLOAT, 123457, "6;1 -2 -2 2 2", False, False, 2), (emac.DOUBLE, 54321, "6;1 -2 2 1 2 1 -2 2", False, False, 1)]
    if R == 8:
        out += [(emac.FLOAT, 262147, "6;1 -2 -2 -2 2 2 2", False, False, 2), (emac.DOUBLE, 100001, "6;1 -4 -2 2 4", False, False, 1),
                (emac.LONG, 65539, "6;1 -4 4 1 4 1 -2 2", False, False, 1), (emac.FLOAT, 4 << 20, full, False, False, 1)]
    if R == 2 and os.environ.get("IPC_BIG"):  # 256 MiB per rank, float then double (same bytes: reused addresses)
        out += [(emac.FLOAT, 64 << 20, full, False, False, 1), (emac.DOUBLE, 32 << 20, full, False, False, 1),
                (emac.FLOAT, 64 << 20, full, False, False, 1)]
    if R == 3:
        out += [(emac.DOUBLE, 99999, "6;2 -3 3", True, False, 2)]
    if R == 8 and os.environ.get("IPC_BIG8"):  # BASELINE configs[3]: double, 256 MiB per rank, random values
        out += [(emac.DOUBLE, 32 << 20, full, False, False, 2), (emac.DOUBLE, 32 << 20, "6;1 -2 -2 -2 2 2 2", False, False, 1)]
    # copy-in methods 5 cyclic / 7 tree (reduce_copyin.c:531-634, :844-968)
    if R == 4:
        out += [(emac.FLOAT, 100003, "7;1 -2 -2 2 2", False, False, 1), (emac.DOUBLE, 4099, "5;1 -4 4", True, False, 1)]
    if R == 8:
        out += [(emac.DOUBLE, 100001, "7;1 -4 -2 2 4", False, False, 1),
                (emac.FLOAT, 65539, "5;1 -2 -2 -2 2 2 2", False, False, 1)]
    return out + fuzz_cases(R, int(os.environ.get("IPC_FUZZ", "0")))


def fuzz_cases(R, n):
    """n random cases (IPC_FUZZ=n), the same on every rank: sizes log-uniform up to 4 Mi elements,
    every type and operation, copy-in variants of R, in place, host and raw device buffers."""
    rng = np.random.default_rng(0xF022 + R)
    variants = [f"6;1 -{R} {R}", f"6;-64 -{R} {R}", f"6;2 -{R} {R}", f"6;3 -{R} {R}"]
    variants += {4: ["6;1 -2 -2 2 2"], 8: ["6;1 -2 -2 -2 2 2 2", "6;1 -4 -2 2 4"], 6: ["6;1 -2 -3 3 2"]}.get(R, [])
    out = []
    for _ in range(n):
        count = int(min(4 << 20, np.exp(rng.uniform(0, np.log(4 << 20)))))
        code = int(rng.choice([emac.FLOAT, emac.DOUBLE, emac.INT, emac.LONG]))
        op = int(rng.choice([emac.SUM, emac.SUM, emac.MIN, emac.MAX]))
        in_place = bool(rng.random() < 0.3)
        host = [False, False, True, "raw"][int(rng.integers(4))]
        in_place = in_place and host is not True  # the host branch below has no in-place form
        out.append((code, count, variants[int(rng.integers(len(variants)))], in_place, host, int(rng.integers(1, 3)), op))
    return out


def _report_mismatch(rank, world, k, got, want):
    """stderr: how many elements differ, the first few (index, got, want) and the owner chunks
    (equal split) they fall in -- enough to tell a stale leaf from a lost pull"""
    g, w = got.view(np.uint8).reshape(-1, got.itemsize), want.view(np.uint8).reshape(-1, want.itemsize)
    bad = np.nonzero(np.any(g != w, axis=1))[0]
    n = got.size
    chunks = sorted({int(i * world // max(n, 1)) for i in bad[:1000]})
    print(f"rank {rank}: case {k}: {bad.size} of {n} differ; first {bad[:6].tolist()} got {got[bad[:6]].tolist()} "
          f"want {want[bad[:6]].tolist()}; owner chunks {chunks[:8]}", file=sys.stderr, flush=True)


def arena_fault(rank, world, dev):
    """A rank that cannot validate its peers' new arena segments (engine_ipc.c
    arena_grow) fails the set-up on EVERY rank -- none left waiting in an exchange the failed rank
    skipped -- and the communicator stays usable: on a fresh communicator, whose first handle
    grows every rank's arena, the last rank's validation sample is failed on purpose
    (EXT_MPI_AMD_TEST_FAIL_ARENA_SAMPLE); every rank must see its allreduce_init refused, then the
    same init again, with the fault cleared, must give the bit-exact sum."""
    comm = emac.comm_init_ipc(rank, world, emac.torch_allgather(), dev)
    n = 4099
    x = torch.full((n,), float(rank + 1), device="cuda")
    y = torch.full_like(x, -1.0)
    if rank == world - 1:
        os.environ["EXT_MPI_AMD_TEST_FAIL_ARENA_SAMPLE"] = "1"
    try:
        h = emac.allreduce_init(x.data_ptr(), y.data_ptr(), n, emac.FLOAT, comm)
        emac.done(h)
        refused = False
    except emac.ExtMpiError as e:
        refused = True
        code = e.code
    os.environ.pop("EXT_MPI_AMD_TEST_FAIL_ARENA_SAMPLE", None)
    h = emac.allreduce_init(x.data_ptr(), y.data_ptr(), n, emac.FLOAT, comm)
    emac.start(h)
    emac.wait(h)
    good = bool(torch.all(y == world * (world + 1) / 2).item())
    emac.done(h)
    emac.comm_free(comm)
    if not (refused and good):
        print(f"rank {rank}: arena fault: refused {refused}{f' ({code})' if refused else ''}, retry good {good}",
              file=sys.stderr, flush=True)
    print(f"IPC rank {rank}/{world} arena validation failure: {'ok' if refused and good else 'MISMATCH'}", flush=True)
    return refused and good


def timeout_recovery(rank, world):
    """A late rank costs one Start, not the communicator (ipc_sync.hpp): on a communicator with a
    0.3 s barrier timeout, rank 1 starts its second Allreduce 1 s late. Every rank must report
    that Start as failed (ERROR_TRANSPORT: the others time out and skip their folds, rank 1 finds
    their marks), and the next Start on the same handle must be bit-exact again. Both the fused
    one-launch path (small message) and barrier -> fold -> barrier (4 MiB per rank)."""
    saved = os.environ.get("EXT_MPI_AMD_BARRIER_TIMEOUT")
    os.environ["EXT_MPI_AMD_BARRIER_TIMEOUT"] = "0.3"
    comm = emac.comm_init_ipc(rank, world, emac.torch_allgather(), int(os.environ.get("IPC_DEVICE", "0")))
    if saved is None:
        del os.environ["EXT_MPI_AMD_BARRIER_TIMEOUT"]
    else:
        os.environ["EXT_MPI_AMD_BARRIER_TIMEOUT"] = saved
    ok = True
    for n in (1000, 1 << 20):
        x = torch.full((n,), float(rank + 1), device="cuda")
        y = torch.empty_like(x)
        h = emac.allreduce_init(x.data_ptr(), y.data_ptr(), n, emac.FLOAT, comm)
        verdicts = []
        for it in range(3):
            dist.barrier()
            y.fill_(-1.0)
            torch.cuda.synchronize()
            if it == 1 and rank == 1:
                time.sleep(1.0)
            try:
                emac.start(h)
                emac.wait(h)
                bad = (y != world * (world + 1) / 2).nonzero().flatten()
                if bad.numel():
                    print(f"rank {rank}: recovery n={n} it={it}: {bad.numel()} wrong, first {bad[:4].tolist()} "
                          f"values {y[bad[:4]].tolist()}", file=sys.stderr, flush=True)
                verdicts.append("wrong" if bad.numel() else "ok")
            except emac.ExtMpiError as e:
                verdicts.append("failed" if e.code == emac.ERROR_TRANSPORT else str(e))
        dist.barrier()
        emac.done(h)
        good = verdicts == ["ok", "failed", "ok"]
        if not good:
            print(f"rank {rank}: timeout recovery n={n}: {verdicts}", file=sys.stderr, flush=True)
        ok &= good
    emac.comm_free(comm)
    print(f"IPC rank {rank}/{world} timeout recovery: {'ok' if ok else 'MISMATCH'}", flush=True)
    return ok


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("IPC_DEVICE", "0"))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    comm = emac.comm_init_ipc(rank, world, emac.torch_allgather(), dev)
    failures = 0
    if os.environ.get("IPC_RECOVERY_ONLY"):  # diagnosis
        failures += not timeout_recovery(rank, world)
        emac.comm_free(comm)
        dist.barrier()
        dist.destroy_process_group()
        sys.exit(1 if failures else 0)
    only = os.environ.get("IPC_CASES")  # diagnosis: comma-separated case indices, in order, repeats allowed
    order = [int(x) for x in only.split(",")] if only else list(range(len(cases(world))))
    for k in order:
        code, count, copyin, in_place, host, repeats = cases(world)[k][:6]
        op = cases(world)[k][6] if len(cases(world)[k]) > 6 else emac.SUM
        sends = xorshift_inputs(world, count, code, seed_base=0x1C0000 + 97 * k)
        want = oracle.allreduce(sends, copyin, in_place=in_place, op=op)[rank]
        raw = host == "raw"
        if raw:
            L, nbytes = emac.lib(), sends[rank].nbytes
            dsend, drecv = ctypes.c_void_p(), ctypes.c_void_p()
            assert L.ext_mpi_amd_gpu_malloc(ctypes.byref(dsend), nbytes) == 0
            if in_place:
                drecv = dsend
            else:
                assert L.ext_mpi_amd_gpu_malloc(ctypes.byref(drecv), nbytes) == 0
            h = emac.allreduce_init(dsend.value, drecv.value, count, code, comm, copyin, op=op)
        elif host:
            hsend = sends[rank].copy()
            hrecv = np.full_like(hsend, -1)
            h = emac.allreduce_init(hsend.ctypes.data, hrecv.ctypes.data, count, code, comm, copyin, op=op)
        else:
            send = torch.from_numpy(sends[rank].copy()).cuda()
            recv = send if in_place else torch.full((count,), -1, dtype=TORCH[code], device="cuda")
            h = emac.allreduce_init(send.data_ptr(), recv.data_ptr(), count, code, comm, copyin, op=op)
        ok = True
        why = ipc_flags_problem(h, world)
        if why:
            print(f"IPC rank {rank}/{world} case {k}: {why}", flush=True)
            ok = False
        for _ in range(repeats):
            if raw:
                src = np.ascontiguousarray(sends[rank])
                assert L.ext_mpi_amd_gpu_memcpy_hd(dsend, src.ctypes.data, nbytes) == 0
            elif in_place:
                send.copy_(torch.from_numpy(sends[rank]))
            torch.cuda.synchronize()
            emac.start(h)
            emac.wait(h)
            if raw:
                got = np.empty_like(want)
                assert L.ext_mpi_amd_gpu_memcpy_dh(got.ctypes.data, drecv, nbytes) == 0
            else:
                got = hrecv if host else recv.cpu().numpy()
            good = bool(np.array_equal(got.view(np.uint8), want.view(np.uint8)))
            if not good and ok:
                _report_mismatch(rank, world, k, got, want)
            ok &= good
        emac.done(h)
        if os.environ.get("IPC_SYNC_AFTER_DONE"):  # diagnosis: surface an asynchronous fault at its case
            torch.cuda.synchronize()
        if raw:
            L.ext_mpi_amd_gpu_free(dsend)
            if not in_place:
                L.ext_mpi_amd_gpu_free(drecv)
        failures += not ok
        print(f"IPC rank {rank}/{world} case {k} code {code} op {op} count {count} '{copyin}' in_place={in_place} "
              f"host={host} x{repeats}: {'ok' if ok else 'MISMATCH'}", flush=True)
    sections = os.environ.get("IPC_SECTIONS", "realloc,newdata,concurrent,recycle,arenafault,recovery").split(",")
    if os.environ.get("IPC_CASES_ONLY"):
        emac.comm_free(comm)
        dist.barrier()
        dist.destroy_process_group()
        sys.exit(1 if failures else 0)
    # Freed and re-allocated user buffers: the same 64 MiB hipMalloc address comes back with
    # new memory while a slower rank still maps the old one. The runtime's IPC handle of the new
    # allocation can then equal the old one's, so a handle exported before every peer has
    # dropped its old mapping would import the old memory (stale leaves, lost fan-out).
    L, n = emac.lib(), 16 << 20
    ok = True
    for it in range(4 if "realloc" in sections else 0):
        bufs = []
        for _ in range(2):
            p = ctypes.c_void_p()
            assert L.ext_mpi_amd_gpu_malloc(ctypes.byref(p), 4 * n) == 0
            bufs.append(p)
        # the same contents in every re-allocation (a stale mapping of the previous
        # allocation would pass the set-up's read-only sample), then new data before a second
        # Start: a peer still reading the old memory would fold the old values
        fill = np.full(n, float(rank + 1), np.float32)
        assert L.ext_mpi_amd_gpu_memcpy_hd(bufs[0], fill.ctypes.data, 4 * n) == 0
        h = emac.allreduce_init(bufs[0].value, bufs[1].value, n, emac.FLOAT, comm)
        got = np.empty(n, np.float32)
        for second in (False, True):
            if second:
                fill = np.full(n, float((rank + 1) * (it + 2)), np.float32)
                assert L.ext_mpi_amd_gpu_memcpy_hd(bufs[0], fill.ctypes.data, 4 * n) == 0
            emac.start(h)
            emac.wait(h)
            assert L.ext_mpi_amd_gpu_memcpy_dh(got.ctypes.data, bufs[1], 4 * n) == 0
            ok &= bool(np.all(got == (it + 2 if second else 1) * world * (world + 1) / 2))
        if os.environ.get("EXT_MPI_AMD_DEBUG_IPC"):
            q = [got[j * n // world: (j + 1) * n // world] for j in range(world)]
            print(f"rank {rank} re-allocation {it}: {ok}; per chunk first/last/n_bad: "
                  f"{[(float(c[0]), float(c[-1]), int(np.sum(c != (it + 1) * world * (world + 1) / 2))) for c in q]}",
                  file=sys.stderr, flush=True)
        if rank == 0:
            time.sleep(0.3)  # the others reach Done first: it is collective, none frees before rank 0 closes
        emac.done(h)
        for p in bufs:
            L.ext_mpi_amd_gpu_free(p)
    failures += not ok
    print(f"IPC rank {rank}/{world} re-allocated buffers: {'ok' if ok else 'MISMATCH'}", flush=True)
    # new send data before every Start (the fold must never see a previous iteration's lines)
    ok = True
    for in_place in ((False, True) if "newdata" in sections else ()):
        x = torch.empty(100003, device="cuda")
        y = x if in_place else torch.empty_like(x)
        h = emac.allreduce_init(x.data_ptr(), y.data_ptr(), x.numel(), emac.FLOAT, comm)
        for it in range(5):
            x.fill_(float((rank + 1) * (it + 1)))
            torch.cuda.synchronize()
            emac.start(h)
            emac.wait(h)
            ok &= bool(torch.all(y == (it + 1) * world * (world + 1) / 2).item())
        emac.done(h)
    failures += not ok
    print(f"IPC rank {rank}/{world} new data every Start: {'ok' if ok else 'MISMATCH'}", flush=True)
    # several handles in flight on separate streams, started in the same order on every rank
    hs, bufs = [], []
    for j in range(3 if "concurrent" in sections else 0):
        s = torch.full((4099,), float(rank + 1 + j), device="cuda")
        r = torch.empty_like(s)
        bufs.append((s, r))
        hs.append(emac.allreduce_init(s.data_ptr(), r.data_ptr(), 4099, emac.FLOAT, comm))
    for _ in range(5):
        for h in hs:
            emac.start(h)
    for h in hs:
        emac.wait(h)
    tri = world * (world + 1) / 2
    ok = True
    for j, (_, r) in enumerate(bufs):
        good = bool(torch.all(r == tri + world * j).item())
        if not good:
            bad = (r != tri + world * j).nonzero().flatten()
            print(f"rank {rank}: concurrent handle {j}: {bad.numel()} of {r.numel()} wrong, first {bad[:6].tolist()} "
                  f"values {r[bad[:6]].tolist()} want {tri + world * j}", file=sys.stderr, flush=True)
        ok &= good
    for h in hs:
        emac.done(h)
    failures += not ok
    print(f"IPC rank {rank}/{world} concurrent handles: {'ok' if ok else 'MISMATCH'}", flush=True)
    # synchronisation slots are recycled: more handle lifetimes than slots, released in a
    # rank-dependent order, each still synchronising correctly (epochs continue per slot)
    ok = True
    x = torch.full((64,), float(rank + 1), device="cuda")
    y = torch.empty_like(x)
    # (past EMAC_SYNC_SLOTS = 1024 lifetimes with up to 4 processes; 8 processes time-sharing the
    # one GPU take 100 s for it, so there 200 lifetimes check the same protocol)
    for it in range((600 if world <= 4 else 100) if "recycle" in sections else 0):
        pair = [emac.allreduce_init(x.data_ptr(), y.data_ptr(), 64, emac.FLOAT, comm) for _ in range(2)]
        for h in pair:
            emac.start(h)
            emac.wait(h)
        if it % 50 == 0:
            good = bool(torch.all(y == world * (world + 1) / 2).item())
            if not good and ok:
                print(f"rank {rank}: slot recycling iteration {it}: y[:4] = {y[:4].tolist()}", file=sys.stderr, flush=True)
            ok &= good
        for h in (pair if rank % 2 else pair[::-1]):
            emac.done(h)
    failures += not ok
    print(f"IPC rank {rank}/{world} slot recycling ({1200 if world <= 4 else 200} handles): {'ok' if ok else 'MISMATCH'}",
          flush=True)
    if "arenafault" in sections:
        failures += not arena_fault(rank, world, dev)
    if "recovery" in sections:
        failures += not timeout_recovery(rank, world)
    emac.comm_free(comm)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(1 if failures else 0)


if __name__ == "__main__":
    main()
