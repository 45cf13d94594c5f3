#!/usr/bin/env python3
"""bench.py -- device-resident GB/s reduced (float32 MPI_SUM) per GPU and % of the HBM3E roofline.

Workload (BASELINE.json configs[1]): persistent Allreduce, float32 MPI_SUM, 16 MiB per rank,
EXT_MPI_COPYIN '6;1 -R R' (copy-in method 6), device-resident synthetic buffers.

  N = 1  (python bench.py): 8 node ranks whose send/recv buffers all live in the one GPU's HBM
         (the reference's XPMEM / IPC-mapped node, ext_mpi_xpmem.c:68-133), one fused
         copy-in + copy-out fold launch per step. Buffer sets are rotated so the working set
         between re-uses (1 GiB) exceeds the 256 MiB Infinity Cache.
  N > 1  (torchrun, one rank per GPU): each GPU holds one rank's 16 MiB. Default transport: the
         peer-mapped form (hipIpc over xGMI, the reference's cudaIpc design): barrier kernel, fold
         of the owned chunk reading the peers' send buffers, fan-out stored into every peer's
         receive buffer, barrier kernel. --transport rccl: reduce-scatter and allgather legs as
         RCCL point-to-point rounds; the other transport is also timed as an extra.

A step is one full Allreduce. value = bytes folded by all ranks (R x 16 MiB per step at N = 1,
N x 16 MiB at N > 1) / wall time of K steps (max over ranks), inputs already in HBM.
The roofline object prices the fold kernel: algorithmic bytes per launch (R reads + D writes
per owner chunk) / its average launch time from HIP events on the
stream it runs on. cpu_baseline times the oracle's threaded restatement of the reference's
CPU path (oracle/ref_cpu_threads.c) on this host, rank 0 at N = 1 only.
"""
import argparse
import ctypes
import json
import math
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
HBM_GUIDE_COPY_GBPS = 6290.0  # the same guide's measured float4 copy (79 % of spec, "~6.3 TB/s achievable")
MIB = 1 << 20


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--size-mib", type=float, default=16.0, help="message bytes per rank")
    ap.add_argument("--ranks", type=int, default=8, help="node ranks resident in one GPU (N = 1)")
    ap.add_argument("--dtype", default="float", choices=["float", "double", "int", "long"])
    ap.add_argument("--copyin", default=None, help="EXT_MPI_COPYIN (default '6;1 -R R')")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the 256 MiB and host-buffer points")
    ap.add_argument("--cpu-seconds", type=float, default=30.0, help="bound of the CPU baseline sample")
    ap.add_argument("--transport", default="ipc", choices=["ipc", "rccl"],
                    help="N > 1: peer-mapped hipIpc form (default) or RCCL point-to-point legs")
    ap.add_argument("--shape", default=None, choices=["local256", "node16", "node64", "node256", "node512", "copy256",
                                                      "int4", "long4", "small", "joinci"],
                    help="profiling: run only this fold shape (40 launches) and exit (PMC passes, tools/gpu_r06_localfp.sh)")
    ap.add_argument("--schedules", default=None,
                    help="--shape node* / local256: comma-separated fold schedule words (U | issue << 4) to run in turn")
    ap.add_argument("--child-transport", default=None, choices=["ipc", "rccl", "node-ipc", "node-rccl"],
                    help=argparse.SUPPRESS)
    ap.add_argument("--child-full", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--child-result", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--child-deadline", type=float, default=600.0, help=argparse.SUPPRESS)
    ap.add_argument("--alloc", default="hip", choices=["hip", "torch", "contig"],
                    help="device buffers from hipMalloc (library device ABI, like the reference's "
                         "tests/benchmark_gpu.c cudaMalloc) or torch's caching allocator")
    return ap.parse_args()


def dtype_info(name):
    import torch
    import ext_mpi_collectives_amd as emac
    return {"float": (torch.float32, emac.FLOAT, "f32", 4), "double": (torch.float64, emac.DOUBLE, "f64", 8),
            "int": (torch.int32, emac.INT, "i32", 4), "long": (torch.int64, emac.LONG, "i64", 8)}[name]


def fill(t, seed):
    import torch
    g = torch.Generator(device=t.device)
    g.manual_seed(seed)
    if t.dtype.is_floating_point:
        t.uniform_(-1.0, 1.0, generator=g)
    else:
        t.random_(-(1 << 20), (1 << 20), generator=g)


DEFER_SHIFT = 11  # fold_kernel.hpp kDeferShift: issue bits 11-12 select the deferred-store kernel


def fold_kernel_name(schedule):
    """the kernel a fold schedule runs (fold_kernel.hpp launch_one): the per-tile loop, or
    fold_deferred_kernel when the issue word carries deferred-store bits"""
    return "fold_deferred_kernel" if schedule and (schedule.get("issue", 0) >> DEFER_SHIFT) & 3 else "fold_kernel"


def traffic_from_profiles(tag):
    """HBM bytes per launch measured by rocprofv3 PMC (profiles/traffic_<tag>.json), or None."""
    path = os.path.join(ROOT, "profiles", f"traffic_{tag}.json")
    if os.path.exists(path):
        try:
            return json.load(open(path)).get("hbm_bytes_per_launch")
        except (ValueError, OSError):
            return None
    return None


class DevBuf:
    """A device buffer from the library's device ABI (hipMalloc), filled from host data.
    CONTIG (bench.py --alloc contig): physically contiguous memory instead (hipExtMallocWithFlags
    hipDeviceMallocContiguous through tools/libceiling.so), an A/B of address translation."""
    CONTIG = False

    def __init__(self, nbytes):
        import ext_mpi_collectives_amd as emac
        self.ptr = ctypes.c_void_p()
        self.nbytes = nbytes
        self.contig = DevBuf.CONTIG
        if self.contig:
            C = _ceiling_lib()
            if C is None or C.ceiling_malloc(ctypes.byref(self.ptr), ctypes.c_size_t(nbytes), 0x4) != 0:
                raise MemoryError("contiguous device allocation failed")
            return
        L = emac.lib()
        if L.ext_mpi_amd_gpu_malloc(ctypes.byref(self.ptr), ctypes.c_size_t(nbytes)) != 0:
            raise MemoryError("ext_mpi_amd_gpu_malloc failed")

    def data_ptr(self):
        return self.ptr.value

    def upload(self, arr):
        import ext_mpi_collectives_amd as emac
        emac.lib().ext_mpi_amd_gpu_memcpy_hd(self.ptr, arr.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(arr.nbytes))

    def download(self, arr):
        import ext_mpi_collectives_amd as emac
        emac.lib().ext_mpi_amd_gpu_memcpy_dh(arr.ctypes.data_as(ctypes.c_void_p), self.ptr, ctypes.c_size_t(arr.nbytes))

    def free(self):
        import ext_mpi_collectives_amd as emac
        if self.ptr.value:
            if self.contig:
                _ceiling_lib().ceiling_free(self.ptr)
            else:
                emac.lib().ext_mpi_amd_gpu_free(self.ptr)
            self.ptr = ctypes.c_void_p()


class HostBuf:
    """A page-locked host buffer (torch pin_memory) with DevBuf's interface: the path's real start
    and end (the reference's XPMEM-mapped MPI buffers)."""

    def __init__(self, nbytes):
        import torch
        self.t = torch.empty(max(1, nbytes), dtype=torch.uint8).pin_memory()

    def data_ptr(self):
        return self.t.data_ptr()

    def upload(self, arr):
        ctypes.memmove(self.t.data_ptr(), arr.ctypes.data, arr.nbytes)

    def download(self, arr):
        ctypes.memmove(arr.ctypes.data, self.t.data_ptr(), arr.nbytes)

    def free(self):
        self.t = None


def host_random(count, np_dtype, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    if np.dtype(np_dtype).kind == "f":
        return (rng.random(count, dtype=np.float64) * 2 - 1).astype(np_dtype)
    lim = 1 << (40 if np.dtype(np_dtype).itemsize == 8 else 20)  # sums cannot overflow
    return rng.integers(-lim, lim, count).astype(np_dtype)


def poison(buf, nbytes):
    """every byte of a receive buffer (DevBuf, HostBuf or tensor) set to 0xFF"""
    if isinstance(buf, DevBuf):
        buf.upload(np.full(nbytes, 0xFF, np.uint8))
    elif isinstance(buf, HostBuf):
        ctypes.memset(buf.data_ptr(), 0xFF, nbytes)
    else:
        buf.view(-1).view(__import__("torch").uint8)[:nbytes].fill_(0xFF)


def free_sets(sets):
    for sends, recvs in sets:
        for b in list(sends) + list(recvs):
            if isinstance(b, DevBuf):
                b.free()


def free_pool(pool):
    for sets in pool.values():
        free_sets(sets)
    pool.clear()


TUNE_STARTS = 1 + 3 * 3 * 8 + 1  # a handle's first Start, 3 rounds of at most 8 candidates on three Starts each, and the keeping one

# Rotated buffer sets: between two uses of one set, at least this many bytes of OTHER sets' inputs
# are read (2.5x the 256 MiB Infinity Cache). Round 4 measured that a rotation sized by the whole
# working set (>= 640 MiB, e.g. 3 sets of 8 x 16 MiB send + receive) still let the Infinity Cache
# serve part of the reads: the time followed the send sets alone -- 3 send sets 45.3 us, 6 or 8
# sets 49.7-50.3 us, whatever the receive rotation (tools/setsweep.hip, profiles/r04/rotation/).
READ_REUSE_BYTES = 640 * MIB


def rotation_sets(read_bytes_per_set, set_bytes=None):
    """Buffer sets to rotate so every read comes from HBM: 1 + READ_REUSE_BYTES / the bytes one set's
    launch reads. EXT_MPI_AMD_BENCH_ROTATION=legacy: rounds 1-3's rule (>= 640 MiB of whole sets,
    `set_bytes`), for A/B runs only."""
    if os.environ.get("EXT_MPI_AMD_BENCH_ROTATION") == "legacy" and set_bytes:
        return max(2, math.ceil(640 * MIB / max(1, set_bytes)))
    return 1 + math.ceil(READ_REUSE_BYTES / max(1, read_bytes_per_set))


def node_run(R, count, tdtype, code, copyin, steps, warmup, min_set_bytes=640 * MIB, host=False, alloc="torch", hold=None,
             pool=None, launch_times=False, isolate=False):
    """Time `steps` node-form Allreduces (R ranks in this GPU). Returns dict of timings. `pool`: a
    dict that keeps the device buffer sets for the next call of the same shape (freed by the caller,
    free_pool) instead of making and filling them again. `launch_times`: also each Start's own time,
    between fence-free events recorded before and after every launch ("launch_us"). `isolate`: the
    host waits for each Start before queuing the next, so no launch overlaps its neighbours' head or
    tail (the lease fingerprint's isolated times)."""
    import torch
    import ext_mpi_collectives_amd as emac
    tsize = torch.empty((), dtype=tdtype).element_size()
    set_bytes = 2 * R * count * tsize
    if host or min_set_bytes <= 0:
        nsets = 1
    else:  # every read from HBM: R send buffers read per launch (READ_REUSE_BYTES)
        nsets = rotation_sets(R * count * tsize, set_bytes)
    stream = torch.cuda.Stream()
    sets, handles = [], []
    key = (R, count, str(tdtype), nsets, host, alloc)
    pooled = pool is not None and key in pool
    if pooled:
        sets = pool[key]
    for s in range(nsets):
        if pooled:
            sends, recvs = sets[s]
        elif host:
            sends = [torch.empty(count, dtype=tdtype).pin_memory() for _ in range(R)]
            recvs = [torch.empty(count, dtype=tdtype).pin_memory() for _ in range(R)]
            for r, t in enumerate(sends):
                t.copy_(torch.rand(count, dtype=torch.float64).mul_(2).sub_(1).to(tdtype))
        elif alloc == "hip":
            np_dtype = {torch.float32: np.float32, torch.float64: np.float64, torch.int32: np.int32,
                        torch.int64: np.int64}[tdtype]
            sends, recvs = [], []
            # EXT_MPI_AMD_BENCH_FAST_FILL (the lease fingerprint's placement runs): one random array
            # for every buffer of the set, so fresh allocations cost a copy, not a generation each
            same = host_random(count, np_dtype, 0x5EED0000 + 97 * s) if os.environ.get("EXT_MPI_AMD_BENCH_FAST_FILL") else None
            for r in range(R):
                b = DevBuf(count * tsize)
                b.upload(same if same is not None else host_random(count, np_dtype, 0x5EED0000 + 97 * s + r))
                sends.append(b)
                recvs.append(DevBuf(count * tsize))
        else:
            sends = [torch.empty(count, dtype=tdtype, device="cuda") for _ in range(R)]
            recvs = [torch.empty(count, dtype=tdtype, device="cuda") for _ in range(R)]
            for r, t in enumerate(sends):
                fill(t, 0x5EED0000 + 97 * s + r)
        h = emac.node_allreduce_init([t.data_ptr() for t in sends], [t.data_ptr() for t in recvs], count, code, copyin)
        emac.set_stream(h, stream.cuda_stream)
        if not pooled:
            sets.append((sends, recvs))
        handles.append(h)
    if pool is not None:
        pool[key] = sets
    torch.cuda.synchronize()
    # W untimed Starts -- and at least enough for every handle to finish its launch-schedule
    # tuning (its first TUNE_STARTS Starts, engine.c emac_tune): the timed Starts run the kept schedule
    for k in range(max(warmup, nsets * TUNE_STARTS)):
        emac.start(handles[k % nsets])
    stream.synchronize()
    sched = emac.handle_schedule(handles[0])
    scheds = [emac.handle_schedule(h) for h in handles]
    # sanity: set 0 against a float64 sum (parity proper is tests/test_gpu_parity.py). Its receive
    # buffers are poisoned first (all bytes 0xFF: NaN / -1), so a schedule that writes nothing or
    # only part of the result cannot pass on an earlier Start's output
    stream.synchronize()
    for b in sets[0][1]:
        poison(b, count * tsize)
    torch.cuda.synchronize()
    emac.start(handles[0])
    stream.synchronize()
    sends, recvs = sets[0]
    if isinstance(sends[0], DevBuf):
        np_dtype = {torch.float32: np.float32, torch.float64: np.float64, torch.int32: np.int32,
                    torch.int64: np.int64}[tdtype]
        hs = [np.empty(count, np_dtype) for _ in range(R)]
        hr = [np.empty(count, np_dtype) for _ in range(R)]
        for b, a in zip(sends, hs):
            b.download(a)
        for b, a in zip(recvs, hr):
            b.download(a)
        sends = [torch.from_numpy(a) for a in hs]
        recvs = [torch.from_numpy(a) for a in hr]
    ref = torch.stack([t.to("cuda", torch.float64) for t in sends]).sum(0)
    got = recvs[0].to("cuda", torch.float64)
    tol = 1e-5 * R if tdtype.is_floating_point else 0.0
    checked = bool(torch.allclose(got, ref, rtol=0, atol=tol)) and all(
        torch.equal(recvs[0], recvs[r]) for r in range(1, R))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    # the timed region: the stream is held while the start event and the first two Starts are
    # enqueued, then runs; the wall clock starts when it is let go
    C = _ceiling_lib() if launch_times else None
    evs = [C.ceiling_event_create() for _ in range(steps + 1)] if C is not None else []
    if evs and not all(evs):
        for ev in evs:
            C.ceiling_event_destroy(ev)
        evs = []

    # per-launch events only in the isolated mode here; back to back they are taken in a second pass
    # below (an event record between two launches adds about a microsecond to the pair)
    def one(k, ev=False):
        if ev and (k == 0 or isolate):
            C.ceiling_event_record(evs[k], stream.cuda_stream)
        emac.start(handles[k % nsets])
        if ev:
            C.ceiling_event_record(evs[k + 1], stream.cuda_stream)
        if isolate:
            stream.synchronize()

    gate = StreamGate(stream.cuda_stream)
    host_us = None
    try:
        e0.record(stream)
        # (isolated launches wait for each other: nothing behind the gate; the latency sweeps hold 2
        # launches only, so their wall clock keeps the host's cost of each Start)
        pre = 0 if isolate else min(GATE_HOLD if hold is None else hold, steps)
        h0 = time.perf_counter()
        for k in range(pre):
            one(k, isolate and bool(evs))
        if pre and gate.g:
            host_us = (time.perf_counter() - h0) / pre * 1e6
    finally:  # a held stream must never outlive an error
        t0 = time.perf_counter()
        gate.open()
    for k in range(pre, steps):
        one(k, isolate and bool(evs))
    e1.record(stream)
    stream.synchronize()
    t1 = time.perf_counter()
    gate.free()
    if evs and not isolate:  # the per-launch pass, held the same way
        gate = StreamGate(stream.cuda_stream)
        try:
            for k in range(min(GATE_HOLD, steps)):
                one(k, True)
        finally:
            gate.open()
        for k in range(min(GATE_HOLD, steps), steps):
            one(k, True)
        stream.synchronize()
        gate.free()
    launch_us = []
    if evs:
        ms = ctypes.c_float()
        for k in range(steps):
            if C.ceiling_event_ms(evs[k], evs[k + 1], ctypes.byref(ms)) == 0:
                launch_us.append(ms.value * 1e3)
    for ev in evs:
        C.ceiling_event_destroy(ev)
    for h in handles:
        emac.done(h)
    if pool is None:
        free_sets(sets)
    del sets
    return {"wall_s": t1 - t0, "event_ms": e0.elapsed_time(e1), "nsets": nsets, "checked": checked,
            "set_bytes": set_bytes, "schedule": sched, "schedules": scheds, "launch_us": launch_us,
            "host_start_us": None if host_us is None else round(host_us, 2)}


def launch_stats(us):
    """median / min / max / count of per-launch times (microseconds), or {} without them"""
    if not us:
        return {}
    v = sorted(us)
    return {"launches_timed": len(v), "median_launch_us": round(statistics.median(v), 1),
            "min_launch_us": round(v[0], 1), "max_launch_us": round(v[-1], 1)}


def comm_shape_fold(R, chunk, tdtype, code, steps, launch_times=False):
    """The COMM form's per-GPU fold (R leaves of one chunk -> 1 destination) on this one GPU, at
    the chunk size an R-GPU run of the same message uses: the 1-GPU reference for the
    'per-GPU rate retained at N GPUs' comparison. Buffer sets rotate past the
    Infinity Cache."""
    import torch
    import ext_mpi_collectives_amd as emac
    tsize = torch.empty((), dtype=tdtype).element_size()
    nbytes = chunk * tsize
    nsets = rotation_sets(R * nbytes, (R + 1) * nbytes)  # R leaves read per launch
    np_dtype = {torch.float32: np.float32, torch.float64: np.float64, torch.int32: np.int32,
                torch.int64: np.int64}[tdtype]
    bufs, handles = [], []
    stream = torch.cuda.Stream()
    for st in range(nsets):
        srcs = [DevBuf(nbytes) for _ in range(R)]
        for i, b in enumerate(srcs):
            b.upload(host_random(chunk, np_dtype, 77 * st + i))
        dst = DevBuf(nbytes)
        h = emac.fold_init([b.data_ptr() for b in srcs], [dst.data_ptr()], chunk, code)
        emac.set_stream(h, stream.cuda_stream)
        bufs += srcs + [dst]
        handles.append(h)
    for k in range(max(10, nsets * TUNE_STARTS)):  # every handle past its schedule tuning (engine.c emac_tune)
        emac.start(handles[k % nsets])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stream.synchronize()
    sched = emac.handle_schedule(handles[0])
    gate = StreamGate(stream.cuda_stream)
    try:
        e0.record(stream)
        for k in range(min(GATE_HOLD, steps)):
            emac.start(handles[k % nsets])
    finally:
        gate.open()
    for k in range(min(GATE_HOLD, steps), steps):
        emac.start(handles[k % nsets])
    e1.record(stream)
    stream.synchronize()
    gate.free()
    t = e0.elapsed_time(e1) * 1e-3 / steps
    # then (launch_times) the same launches again, each between its own fence-free events: an event
    # record between two launches adds about a microsecond to the pair, so the average above is
    # taken without them and only the per-launch spread comes from this pass
    C = _ceiling_lib() if launch_times else None
    evs = [C.ceiling_event_create() for _ in range(steps + 1)] if C is not None else []
    if evs and not all(evs):
        for ev in evs:
            C.ceiling_event_destroy(ev)
        evs = []
    if evs:
        gate = StreamGate(stream.cuda_stream)
        try:
            C.ceiling_event_record(evs[0], stream.cuda_stream)
            for k in range(min(GATE_HOLD, steps)):
                emac.start(handles[k % nsets])
                C.ceiling_event_record(evs[k + 1], stream.cuda_stream)
        finally:
            gate.open()
        for k in range(min(GATE_HOLD, steps), steps):
            emac.start(handles[k % nsets])
            C.ceiling_event_record(evs[k + 1], stream.cuda_stream)
        stream.synchronize()
        gate.free()
    launch_us = []
    if evs:
        ms = ctypes.c_float()
        for k in range(steps):
            if C.ceiling_event_ms(evs[k], evs[k + 1], ctypes.byref(ms)) == 0:
                launch_us.append(ms.value * 1e3)
    # and (launch_times) a third pass in blocks of BLOCK launches back to back, a fence-free event
    # only between blocks: the per-launch events above add about a microsecond to each launch they
    # separate, which this pass spreads over BLOCK launches
    block_us = []
    BLOCK = 5
    if evs and steps >= 2 * BLOCK:
        nb = steps // BLOCK
        gate = StreamGate(stream.cuda_stream)
        try:
            C.ceiling_event_record(evs[0], stream.cuda_stream)
            for j in range(nb):
                for k in range(j * BLOCK, (j + 1) * BLOCK):
                    emac.start(handles[k % nsets])
                C.ceiling_event_record(evs[j + 1], stream.cuda_stream)
                if j + 1 == min(nb, GATE_HOLD // BLOCK):
                    gate.open()
        finally:
            gate.open()
        stream.synchronize()
        gate.free()
        ms = ctypes.c_float()
        for j in range(nb):
            if C.ceiling_event_ms(evs[j], evs[j + 1], ctypes.byref(ms)) == 0:
                block_us.append(ms.value * 1e3 / BLOCK)
    for ev in evs:
        C.ceiling_event_destroy(ev)
    scheds = [emac.handle_schedule(h) for h in handles]
    for h in handles:
        emac.done(h)
    for b in bufs:
        b.free()
    return {"chunk_bytes": nbytes, "leaves": R, "avg_launch_us": round(t * 1e6, 2),
            "gbps_reduced": round(R * nbytes / t / 1e9, 1), "achieved_gbps": round((R + 1) * nbytes / t / 1e9, 1),
            "schedule": sched, "schedules_per_set": schedule_counts(scheds), **launch_stats(launch_us),
            **({"blocks_timed": len(block_us), "block_launches": BLOCK,
                "median_of_block_means_us": round(statistics.median(block_us), 2)} if block_us else {})}


def schedule_counts(scheds):
    """{"U<u>/<issue>": number of handles that kept it}: every rotated set tunes on its own"""
    out = {}
    for sc in scheds:
        k = f"U{sc['unroll']}/{sc['issue']}"
        out[k] = out.get(k, 0) + 1
    return out


def _ceiling_lib():
    """tools/libceiling.so (built by __graft_entry__.build()): measured-ceiling kernels, or None."""
    path = os.path.join(ROOT, "tools", "libceiling.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.ceiling_read_glds.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.ceiling_read_vgpr.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_void_p]
    L.ceiling_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.ceiling_write.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_void_p]
    L.ceiling_event_create.restype = ctypes.c_void_p
    L.ceiling_event_record.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.ceiling_event_ms.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
    L.ceiling_event_destroy.argtypes = [ctypes.c_void_p]
    L.ceiling_gate_arm.argtypes = [ctypes.c_void_p]
    L.ceiling_gate_arm.restype = ctypes.c_void_p
    L.ceiling_gate_open.argtypes = [ctypes.c_void_p]
    L.ceiling_gate_free.argtypes = [ctypes.c_void_p]
    L.ceiling_malloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    L.ceiling_free.argtypes = [ctypes.c_void_p]
    return L


# launches enqueued behind the gate before it opens: all of a timed region's (up to this many), so
# the GPU never waits for the host's next Start (a Start costs the host several microseconds:
# `host_start_us`; configs[2]'s launch is only 11 us) -- well below the stream's packet ring
GATE_HOLD = 64


class StreamGate:
    """Holds `stream` (tools/ceiling.hip ceiling_gate_arm) while the host enqueues the first
    launches of a timed region, so its start event does not time the host's submission latency;
    open() lets it run. A no-op without tools/libceiling.so."""

    def __init__(self, stream_ptr):
        self.L = _ceiling_lib()
        self.g = self.L.ceiling_gate_arm(stream_ptr) if self.L else None

    def open(self):
        if self.g:
            self.L.ceiling_gate_open(self.g)

    def free(self):
        if self.g:
            self.L.ceiling_gate_free(self.g)
            self.g = None


def measured_ceilings(steps=10, launch_bytes=256 * MIB):
    """Best HBM rates measured on this GPU in this run (tools/ceiling.hip), GB/s of algorithmic bytes:
    read -- the best of three read-only streams over 4 GiB: LDS-DMA (global_load_lds_dwordx4 nt)
    and nontemporal global_load_dwordx4 into VGPRs with 4 or 8 vectors per lane in flight; write --
    a nontemporal store stream over 4 GiB and at the launch's written bytes; copy -- the best of a nontemporal and a default-policy 1:1 copy
    (K = 4 vectors per lane) and a nontemporal copy in phases (tools/ceiling.hip copy_phased), each timed over 4 GiB and over `launch_bytes` (read + written, the
    headline launch's bytes, buffer sets rotated as the launches' are, rotation_sets): the rate
    of the node-form fold's 1:1 read/write mix."""
    import torch
    L = _ceiling_lib()
    if L is None:
        return {}
    n = 4 << 30
    a = torch.empty(n // 4, dtype=torch.float32, device="cuda")
    a.uniform_(-1, 1)
    sink = torch.zeros(4, device="cuda")
    stream = torch.cuda.current_stream()
    out = {}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reads = {}
    for vname, fn in (("glds", lambda it: L.ceiling_read_glds(a.data_ptr(), n, it, sink.data_ptr(), stream.cuda_stream)),
                      ("vgpr_k4", lambda it: L.ceiling_read_vgpr(a.data_ptr(), n, it, 4, sink.data_ptr(), stream.cuda_stream)),
                      ("vgpr_k8", lambda it: L.ceiling_read_vgpr(a.data_ptr(), n, it, 8, sink.data_ptr(), stream.cuda_stream))):
        fn(2)
        e0.record(stream)
        assert fn(steps) == 0
        e1.record(stream)
        torch.cuda.synchronize()
        reads[vname] = round(steps * n / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
    out["read_ceiling_gbps"] = max(reads.values())
    out["read_variants_gbps"] = reads
    # write-only: over 4 GiB and at the launch's written bytes (three buffers rotated)
    writes = {}
    L.ceiling_write(a.data_ptr(), n, 2, stream.cuda_stream)
    e0.record(stream)
    assert L.ceiling_write(a.data_ptr(), n, steps, stream.cuda_stream) == 0
    e1.record(stream)
    torch.cuda.synchronize()
    writes["write_4GiB"] = round(steps * n / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
    half = launch_bytes // 2
    k = rotation_sets(half, launch_bytes)  # buffers rotated (as the launches' sets)
    e0.record(stream)
    for i in range(k * steps):
        assert L.ceiling_write(a.data_ptr() + (i % k) * launch_bytes, half, 1, stream.cuda_stream) == 0
    e1.record(stream)
    torch.cuda.synchronize()
    writes["write_launch"] = round(k * steps * half / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
    out["write_ceiling_gbps"] = max(writes.values())
    out["write_variants_gbps"] = writes
    copies = {}
    for variant, vname in ((0, "nt"), (1, "plain"), (2, "phased")):
        half = n // 2
        L.ceiling_copy(a.data_ptr(), a.data_ptr() + half, half, 2, variant, stream.cuda_stream)
        e0.record(stream)
        assert L.ceiling_copy(a.data_ptr(), a.data_ptr() + half, half, steps, variant, stream.cuda_stream) == 0
        e1.record(stream)
        torch.cuda.synchronize()
        copies[f"copy_{vname}_4GiB"] = round(steps * 2 * half / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
        half = launch_bytes // 2  # k sets of (src, dst) rotated, every source read from HBM
        k = rotation_sets(half, launch_bytes)
        L.ceiling_copy(a.data_ptr(), a.data_ptr() + half, half, 1, variant, stream.cuda_stream)
        e0.record(stream)
        for i in range(k * steps):
            base = a.data_ptr() + (i % k) * launch_bytes
            assert L.ceiling_copy(base, base + half, half, 1, variant, stream.cuda_stream) == 0
        e1.record(stream)
        torch.cuda.synchronize()
        copies[f"copy_{vname}_launch"] = round(k * steps * 2 * half / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
    out["copy_gbps"] = max(copies.values())
    out["copy_variants_gbps"] = copies
    del a, sink
    torch.cuda.empty_cache()
    return out


def read_write_floor_s(ceil, read_bytes, write_bytes):
    """The shortest time HBM can read `read_bytes` and write `write_bytes` on this GPU: the two
    streams' times at the measured read and write ceilings, added (HBM does not read and write at
    once; tools/nodevar.hip: the node fold at 256 MiB per rank took 0.97 of that sum)."""
    return read_bytes / (ceil["read_ceiling_gbps"] * 1e9) + write_bytes / (ceil["write_ceiling_gbps"] * 1e9)


def stream_copy_peak():
    """Measured device copy rate (read + write bytes / s) of a 2 GiB buffer, for context."""
    import torch
    n = (1 << 31) // 4
    a = torch.empty(n, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    a.fill_(1.0)
    for _ in range(3):
        b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbps = 10 * 2 * a.numel() * 4 / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return gbps


def host_l3_bytes():
    """Total L3 of this host (sum over distinct L3 domains), or None."""
    base, seen, total = "/sys/devices/system/cpu", set(), 0
    try:
        for cpu in os.listdir(base):
            idx = os.path.join(base, cpu, "cache", "index3")
            if not cpu.startswith("cpu") or not os.path.isdir(idx):
                continue
            shared = open(os.path.join(idx, "shared_cpu_list")).read().strip()
            if shared in seen:
                continue
            seen.add(shared)
            size = open(os.path.join(idx, "size")).read().strip()
            total += int(size[:-1]) * (1024 if size.endswith("K") else 1 << 20 if size.endswith("M") else 1)
    except (OSError, ValueError):
        return None
    return total or None


def cpu_baseline(R, count, np_dtype, copyin, seconds):
    """The oracle's threaded CPU restatement of the reference path on a bounded sample. Buffer
    sets rotate every Allreduce so the working set (>= 2x the host's L3, at least 1 GiB) is
    memory-resident, as the GPU leg's rotated sets are HBM-resident."""
    from oracle import oracle
    rng = np.random.default_rng(0x5EED0000)
    set_bytes = 2 * R * count * np.dtype(np_dtype).itemsize
    l3 = host_l3_bytes()
    nsets = max(2, math.ceil(max(1 << 30, 2 * (l3 or 0)) / max(1, set_bytes)))
    base = [(rng.random(count) * 2 - 1).astype(np_dtype) for _ in range(R)]
    sets = [([b.copy() for b in base], [np.empty_like(b) for b in base]) for _ in range(nsets)]
    iters, t = nsets, 0.0
    budget_left = seconds
    # tests/benchmark.c:92-157 doubles the iteration count until a run takes >= 2 s; here until
    # >= 8 s (a 10-30 s sample of CPU work in all, bounded by `seconds`)
    while True:
        t = oracle.cpu_allreduce_threads_sets(sets, copyin, iters)
        budget_left -= t
        if t >= 8.0 or budget_left < 2.5 * t:
            break
        iters *= 2
    return {"value": round(iters * R * count * np.dtype(np_dtype).itemsize / t / 1e9, 3), "unit": "GB/s",
            "cores": R, "kind": "port",
            "sample": f"{iters} Allreduce(s) of {R} ranks x {count * np.dtype(np_dtype).itemsize // MIB} MiB "
                      f"'{copyin}' in {t:.2f} s over {nsets} rotated buffer sets ({nsets * set_bytes // MIB} MiB; "
                      f"host L3 {l3 // MIB if l3 else '?'} MiB): R pthreads replaying each rank's SMEMCPY/SREDUCE "
                      f"program (gcc -O3 restatement of ext_mpi_native_exec.c:207-234) with spin barriers, one "
                      f"thread per rank as the reference runs one process per rank; host nproc={os.cpu_count()}"}


def cpu_config0():
    """BASELINE configs[0] on the host: the CPU restatement at tests/benchmark.c's shape (4 ranks,
    64 KiB float, '6;1 -4 4'), iteration count doubled until a run takes >= 2 s (benchmark.c:150)."""
    from oracle import oracle
    rng = np.random.default_rng(0x5EED0000)
    sends = [(rng.random(16384) * 2 - 1).astype(np.float32) for _ in range(4)]
    recvs = [np.empty_like(s) for s in sends]
    iters = 1
    while True:
        t = oracle.cpu_allreduce_threads(sends, recvs, "6;1 -4 4", iters)
        if t >= 2.0 or iters >= (1 << 24):
            break
        iters *= 2
    return {"us_per_allreduce": round(t * 1e6 / iters, 3), "gbps_reduced": round(iters * 4 * 65536 / t / 1e9, 3),
            "cores": 4, "kind": "port", "sample": f"{iters} Allreduce(s) in {t:.2f} s"}


def single_gpu(args):
    import torch
    import ext_mpi_collectives_amd as emac
    tdtype, code, dname, tsize = dtype_info(args.dtype)
    R = args.ranks
    count = int(args.size_mib * MIB) // tsize
    S = count * tsize
    copyin = args.copyin or f"6;1 -{R} {R}"
    emac.lib()
    main = node_run(R, count, tdtype, code, copyin, args.steps, args.warmup, alloc=args.alloc)
    kernel_s = main["event_ms"] * 1e-3 / args.steps
    bytes_reduced_per_step = R * S
    algo_bytes = 2 * R * S  # R buckets x (R leaf reads + R fan-out writes) x chunk S/R
    achieved = algo_bytes / kernel_s / 1e9
    out = {
        "metric": "device-resident GB/s reduced (float32 MPI_SUM) per GPU; % HBM3E roofline",
        "value": round(bytes_reduced_per_step * args.steps / main["wall_s"] / 1e9, 2),
        "unit": "GB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(main["wall_s"] * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dname,
        "data": f"synthetic: uniform [-1,1) per rank (seeded), device-resident, {main['nsets']} rotated buffer sets "
                f"({main['nsets'] * main['set_bytes'] // MIB} MiB; {(main['nsets'] - 1) * main['set_bytes'] // 2 // MIB} "
                f"MiB of other sets' inputs read between two uses of one set, 2.5x the 256 MiB Infinity Cache)",
        "config": {"workload": f"persistent Allreduce {args.dtype} MPI_SUM, {S // MIB} MiB per rank, {R} node ranks "
                               f"resident in one MI355X (BASELINE configs[1]), EXT_MPI_COPYIN '{copyin}', fused "
                               f"reduce_copyin + reduce_copyout fold",
                   "ranks": R, "message_bytes_per_rank": S, "copyin": copyin, "layout": "node-in-one-HBM",
                   "buffers": "hipMalloc" if args.alloc == "hip" else "torch caching allocator",
                   "checked_vs_fp64_sum": main["checked"],
                   "warmup_starts": max(args.warmup, main["nsets"] * TUNE_STARTS),
                   "fold_schedule": main["schedule"],
                   "fold_schedules_per_set": schedule_counts(main["schedules"])},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic_from_profiles(f"node_r{R}_{S // MIB}mib_{args.dtype}"),
                     "kernel": fold_kernel_name(main["schedule"]), "algorithmic_bytes_per_launch": algo_bytes,
                     "avg_launch_us": round(kernel_s * 1e6, 2),
                     "guide_measured_copy": HBM_GUIDE_COPY_GBPS,
                     "frac_of_guide_measured_copy": round(achieved / HBM_GUIDE_COPY_GBPS, 4)},
        # the timed region's Starts are enqueued behind a stream gate and run back to back once it opens
        # (StreamGate); host_start_us is what one Start cost the host meanwhile
        "timing": {"launches_held_behind_gate": min(GATE_HOLD, args.steps), "host_start_us": main["host_start_us"]},
    }
    if not args.no_extras:
        extras = {}
        try:
            extras["stream_copy_gbps"] = round(stream_copy_peak(), 1)
            ceil = measured_ceilings()
            extras.update(ceil)
            if ceil:
                out["roofline"]["measured_read_ceiling"] = ceil["read_ceiling_gbps"]
                out["roofline"]["frac_of_measured_read_ceiling"] = round(achieved / ceil["read_ceiling_gbps"], 4)
                out["roofline"]["measured_copy_ceiling"] = ceil["copy_gbps"]
                # the fold against the best measured 1:1 copy of the same mix; a fold faster than
                # every copy kernel measured makes that copy no ceiling: then only the flag is kept
                if achieved <= ceil["copy_gbps"]:
                    out["roofline"]["frac_of_measured_copy_ceiling"] = round(achieved / ceil["copy_gbps"], 4)
                else:
                    out["roofline"]["kernel_above_measured_copy"] = True
                # HBM does not read and write at once: a launch that reads B_r and writes B_w bytes
                # takes at least B_r / read ceiling + B_w / write ceiling (both measured here)
                fl = read_write_floor_s(ceil, algo_bytes / 2, algo_bytes / 2)
                out["roofline"]["read_write_floor_us"] = round(fl * 1e6, 2)
                out["roofline"]["frac_of_read_write_floor"] = round(fl / kernel_s, 4)
        except (RuntimeError, AssertionError) as e:
            log("ceiling probes failed:", e)
        big = (256 * MIB) // tsize
        # at least 20 timed launches, each also between its own fence-free events (4
        # launches could not tell a slow lease from noise); the median is the point's figure
        n256 = max(20, args.steps // 5)
        r256 = node_run(R, big, tdtype, code, copyin, n256, 2, alloc=args.alloc, launch_times=True)
        k256 = r256["event_ms"] * 1e-3 / n256
        st256 = launch_stats(r256["launch_us"])
        extras["point_256MiB"] = {
            "gbps_reduced": round(R * big * tsize / k256 / 1e9, 1),
            "achieved_gbps": round(2 * R * big * tsize / k256 / 1e9, 1),
            "frac_of_peak": round(2 * R * big * tsize / k256 / 1e9 / HBM_PEAK_GBPS, 4),
            "frac_of_guide_measured_copy": round(2 * R * big * tsize / k256 / 1e9 / HBM_GUIDE_COPY_GBPS, 4),
            "frac_of_measured_read_ceiling": round(2 * R * big * tsize / k256 / 1e9 / extras["read_ceiling_gbps"], 4)
            if "read_ceiling_gbps" in extras else None,
            "read_gbps": round(R * big * tsize / k256 / 1e9, 1),
            "avg_launch_us": round(k256 * 1e6, 1), **st256,
            "frac_of_peak_at_median": round(2 * R * big * tsize / (st256["median_launch_us"] * 1e-6) / 1e9 /
                                            HBM_PEAK_GBPS, 4) if st256 else None,
            "checked": r256["checked"], "fold_schedule": r256["schedule"],
            "schedules_per_set": schedule_counts(r256["schedules"]),
            "traffic": traffic_from_profiles(f"node_r{R}_256mib_{args.dtype}")}
        if "write_ceiling_gbps" in extras:
            fl = read_write_floor_s(extras, R * big * tsize, R * big * tsize)
            extras["point_256MiB"].update(read_write_floor_us=round(fl * 1e6, 1),
                                          frac_of_read_write_floor=round(fl / k256, 4))
        # latency -> bandwidth crossover of the node form (cf. BASELINE configs[4] on 8 GPUs);
        # small points reuse one buffer set (as the reference's latency runs do), large ones rotate
        sweep = []
        # (to configs[4]'s 512 MiB endpoint: one buffer set of 8 GiB is far past the Infinity Cache)
        for nbytes in (8, 1024, 64 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 512 << 20):
            cnt = max(1, nbytes // tsize)
            st = 200 if nbytes <= (1 << 20) else 40 if nbytes <= (64 << 20) else 5
            r = node_run(R, cnt, tdtype, code, copyin, st, 2 if nbytes > (64 << 20) else 5,
                         min_set_bytes=0 if nbytes < (16 << 20) or nbytes > (64 << 20) else 640 * MIB,
                         alloc=args.alloc, hold=2)
            sweep.append({"bytes_per_rank": cnt * tsize, "us_per_allreduce": round(r["wall_s"] * 1e6 / st, 2),
                          "gpu_us_per_allreduce": round(r["event_ms"] * 1e3 / st, 2),
                          "gbps_reduced": round(R * cnt * tsize * st / r["wall_s"] / 1e9, 2),
                          "checked": r["checked"], "fold_schedule": r.get("schedule")})
        extras["sweep_node_form"] = sweep
        # BASELINE configs[4]'s EXT_MPI_COPYIN radix sweep on the node form (8 ranks in this GPU): the
        # linear fold, the radix chains and the -64 fractions -- which the reference offers for small
        # messages (reduce_copyin.c:410-425) -- from latency to bandwidth sizes, each point against the
        # linear fold measured in the same sweep, and each variant's latency -> bandwidth crossover
        rsweep = []
        for cp in (copyin,) + RADIX_VARIANTS.get(R, ()):
            for nbytes in RADIX_SWEEP_BYTES:
                cnt = max(1, nbytes // tsize)
                st = 200 if nbytes <= (1 << 20) else 40
                r = node_run(R, cnt, tdtype, code, cp, st, 5, min_set_bytes=0 if nbytes < (16 << 20) else 640 * MIB,
                             alloc=args.alloc, hold=2)
                rsweep.append({"copyin": cp, "bytes_per_rank": cnt * tsize,
                               "us_per_allreduce": round(r["wall_s"] * 1e6 / st, 2),
                               "gpu_us_per_allreduce": round(r["event_ms"] * 1e3 / st, 2), "checked": r["checked"]})
        radix_vs_linear(rsweep, copyin, "gpu_us_per_allreduce")
        extras["radix_crossover_node_form"] = radix_crossovers(rsweep, "gpu_us_per_allreduce", R)
        extras["radix_sweep_node_form"] = rsweep
        # radix chains (compile-time fold trees) against the linear fold, measured alike and
        # alternated twice (median of each), so a drifting clock does not favour either
        chains, runs = {}, {}
        for rep in range(2):
            for cp in (copyin, "6;1 -2 -2 -2 2 2 2", "6;1 -4 -2 2 4", "6;1 -2 -4 4 2"):  # (-k: small messages only)
                r = node_run(R, count, tdtype, code, cp, args.steps, args.warmup, alloc=args.alloc)
                runs.setdefault(cp, []).append((r["event_ms"] * 1e-3 / args.steps, r["checked"]))
        lin = min(t for t, _ in runs[copyin])
        for cp, v in runs.items():
            k = min(t for t, _ in v)
            chains[cp] = {"gbps_reduced": round(R * S / k / 1e9, 1), "avg_launch_us": round(k * 1e6, 2),
                          "vs_linear": round(lin / k, 4), "checked": all(c for _, c in v)}
        extras["radix_chains_16MiB"] = chains
        extras["fold_comm_shape"] = comm_shape_fold(R, count // R, tdtype, code, 200)
        # SURVEY.md 8(d)'s local fold at the north-star size: the owner's fold of the COMM / IPC
        # forms (R leaves of C = 256 MiB / R -> one destination, read-dominated), where the
        # ">= 80 % of HBM read bandwidth" target is defined
        lf = comm_shape_fold(R, big // R, tdtype, code, 40, launch_times=True)
        lf["frac_of_peak"] = round(lf["achieved_gbps"] / HBM_PEAK_GBPS, 4)
        if "median_launch_us" in lf:
            lf["frac_of_peak_at_median"] = round((R + 1) * lf["chunk_bytes"] / (lf["median_launch_us"] * 1e-6) / 1e9 /
                                                 HBM_PEAK_GBPS, 4)
        if "median_of_block_means_us" in lf:
            lf["frac_of_peak_at_block_median"] = round((R + 1) * lf["chunk_bytes"] / (lf["median_of_block_means_us"] * 1e-6) /
                                                       1e9 / HBM_PEAK_GBPS, 4)
        lf["algorithmic_bytes_per_launch"] = (R + 1) * lf["chunk_bytes"]
        lf["traffic"] = traffic_from_profiles(f"local_r{R}_{lf['chunk_bytes'] // MIB}mib_{args.dtype}")
        if "write_ceiling_gbps" in extras:
            fl = read_write_floor_s(extras, R * lf["chunk_bytes"], lf["chunk_bytes"])
            lf["read_write_floor_us"] = round(fl * 1e6, 2)
            lf["frac_of_read_write_floor"] = round(fl / (lf["avg_launch_us"] * 1e-6), 4)
        if "read_ceiling_gbps" in extras:
            lf["frac_of_measured_read_ceiling"] = round(lf["achieved_gbps"] / extras["read_ceiling_gbps"], 4)
        extras["local_fold_256MiB"] = lf
        hst = node_run(R, count, tdtype, code, copyin, 10, 3, host=True, hold=2)
        os.environ["EXT_MPI_AMD_HOST_DIRECT"] = "0"  # staged through device mirrors, for comparison
        hst0 = node_run(R, count, tdtype, code, copyin, 10, 3, host=True, hold=2)
        del os.environ["EXT_MPI_AMD_HOST_DIRECT"]
        extras["host_buffers_pcie_inclusive"] = {
            "gbps_reduced": round(R * S * 10 / hst["wall_s"] / 1e9, 2),
            "ms_per_step": round(hst["wall_s"] * 1e3 / 10, 3),
            "checked": hst["checked"] and hst0["checked"],
            "staged_gbps_reduced": round(R * S * 10 / hst0["wall_s"] / 1e9, 2),
            "note": "pinned host send/recv buffers read and written by the fold kernel over PCIe (default); "
                    "staged: EXT_MPI_AMD_HOST_DIRECT=0, H2D -> fold -> D2H on one stream, 3 warm-up Starts"}
        # BASELINE configs[2]: int and long, 4 MiB per rank, 8 ranks; integer sums are exact in any
        # order, so the check against the float64 sum of the inputs is bit-exact (|values| <= 2^20
        # int, 2^40 long: every partial sum is exact in float64)
        ints = {}
        for dn, td, cd in (("int", torch.int32, emac.INT), ("long", torch.int64, emac.LONG)):
            ts = torch.empty((), dtype=td).element_size()
            r = node_run(R, (4 * MIB) // ts, td, cd, copyin, 50, 5, alloc=args.alloc)
            k = r["event_ms"] * 1e-3 / 50
            ints[dn] = {"gbps_reduced": round(R * 4 * MIB / k / 1e9, 1), "avg_launch_us": round(k * 1e6, 2),
                        "achieved_gbps": round(2 * R * 4 * MIB / k / 1e9, 1), "bitexact": r["checked"],
                        "host_start_us": r["host_start_us"]}
        extras["config3_int_long_4MiB"] = ints
        # BASELINE configs[0] shape (tests/benchmark.c: 4 ranks, 64 KiB float, '6;1 -4 4') on this path
        c0 = (64 << 10) // 4
        d0 = node_run(4, c0, torch.float32, emac.FLOAT, "6;1 -4 4", 400, 20, min_set_bytes=0, alloc=args.alloc, hold=2)
        h0 = node_run(4, c0, torch.float32, emac.FLOAT, "6;1 -4 4", 200, 20, host=True, hold=2)
        os.environ["EXT_MPI_AMD_HOST_DIRECT"] = "0"
        h1 = node_run(4, c0, torch.float32, emac.FLOAT, "6;1 -4 4", 200, 20, host=True, hold=2)
        del os.environ["EXT_MPI_AMD_HOST_DIRECT"]
        extras["config0_64KiB_4ranks"] = {
            "device_us_per_allreduce": round(d0["wall_s"] * 1e6 / 400, 2),
            "host_buffers_us_per_allreduce": round(h0["wall_s"] * 1e6 / 200, 2),
            "host_buffers_staged_us_per_allreduce": round(h1["wall_s"] * 1e6 / 200, 2),
            "checked": d0["checked"] and h0["checked"] and h1["checked"],
            "note": "4 node ranks in one MI355X; host_buffers = pinned host send/recv read and written by the "
                    "fold kernel over PCIe; staged = H2D -> fold -> D2H (EXT_MPI_AMD_HOST_DIRECT=0)"}
        out["extras"] = extras
    if not args.no_cpu_baseline:
        np_dtype = {"float": np.float32, "double": np.float64, "int": np.int32, "long": np.int64}[args.dtype]
        out["cpu_baseline"] = cpu_baseline(R, count, np_dtype, copyin, args.cpu_seconds)
        if not args.no_extras:
            out["cpu_baseline"]["config0_64KiB_4ranks"] = cpu_config0()
    emit(out)


def _comm_run(emac, comm, count, tdtype, code, dname, copyin, steps, warmup, rank, world, dist, torch, check=True,
              host=False):
    """Persistent Allreduce of `count` elements per rank on communicator `comm`; returns the max-over-ranks
    wall time of `steps` Starts (one stream), the handle's fold time alone, and the check."""
    tsize = torch.empty((), dtype=tdtype).element_size()
    np_dtype = {torch.float32: np.float32, torch.float64: np.float64, torch.int32: np.int32,
                torch.int64: np.int64}[tdtype]
    Buf = HostBuf if host else DevBuf
    send, recv = Buf(max(1, count * tsize)), Buf(max(1, count * tsize))
    mine = host_random(count, np_dtype, 0x5EED0000 + rank)
    send.upload(mine)
    h = emac.allreduce_init(send.data_ptr(), recv.data_ptr(), count, code, comm, copyin)
    # the handle's own HIP stream (on the 1-GPU rehearsal box the first handle put on a torch
    # pool stream ran its barriers ~8x slower, tools/ipc_latency.py IPC_LAT_OWN_STREAM)
    stream = torch.cuda.ExternalStream(emac.stream(h))
    for _ in range(warmup):
        emac.start(h)
    emac.wait(h)
    checked = True
    if check:
        got = np.empty(count, np_dtype)
        recv.download(got)
        idx = np.arange(0, count, max(1, count // (1 << 20)))  # <= 1 Mi samples spread over every chunk
        allin = [None] * world
        dist.all_gather_object(allin, mine[idx])
        got = got[idx]
        ref = np.sum(np.stack([a.astype(np.float64) for a in allin]), axis=0)
        tol = 1e-5 * world if np.dtype(np_dtype).kind == "f" else 0.0
        good = np.isclose(got.astype(np.float64), ref, rtol=0, atol=tol)
        if not good.all():
            bad = np.flatnonzero(~good)
            log(f"rank {rank}: {dname} {count} elements: {bad.size}/{idx.size} samples differ, first at element "
                f"{idx[bad[0]]} (chunk {idx[bad[0]] * world // count}), last at {idx[bad[-1]]}: got {got[bad[0]]} "
                f"want {ref[bad[0]]}")
        ok = torch.tensor([int(good.all())])
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        checked = bool(ok.item())
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        emac.start(h)
    emac.wait(h)
    torch.cuda.synchronize()
    # each rank's own completion time (the barrier above aligned the starts); the slowest rank's
    # is the job's. The trailing barrier stays outside the timed region: a gloo round trip is
    # 100-300 us, as long as dozens of small Allreduces.
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.barrier()
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return h, send, recv, stream, el.item(), checked


def _fold_only(emac, h, stream, steps, torch):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        emac.start_legs(h, emac.LEG_FOLD)
    e1.record(stream)
    stream.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / steps


def _rccl_allreduce_baseline(rank, world, dist, torch):
    """RCCL's own float Allreduce at the sweep's sizes (the reference's tests/benchmark_nccl.c
    comparison), through torch's RCCL process group; max over ranks. A reported
    baseline: its summation order is RCCL's, not the reference's."""
    try:
        g = dist.new_group(backend="nccl")
        pts = []
        for nbytes in (8, 64 << 10, 1 << 20, 16 << 20, 64 << 20, 256 << 20):
            n = max(1, nbytes // 4)
            x = torch.ones(n, device="cuda")
            st = 100 if nbytes <= (1 << 20) else 10
            for _ in range(5):
                dist.all_reduce(x, group=g)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(st):
                dist.all_reduce(x, group=g)
            torch.cuda.synchronize()
            el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            pts.append({"bytes_per_rank": n * 4, "us_per_allreduce": round(el.item() * 1e6 / st, 2),
                        "algbw_gbps": round(n * 4 * st / el.item() / 1e9, 2)})
            del x
        dist.destroy_process_group(g)
        return pts
    except Exception as e:  # noqa: BLE001 -- a baseline, never the measurement
        log(f"rank {rank}: RCCL Allreduce baseline failed: {e}")
        return {"error": str(e)[:200]}


def _node_point(emac, rank, world, dev, count, tdtype, code, dname, dist, torch, nodes=2, ports=None):
    """§8(f3): the same ranks as `nodes` logical nodes of world/nodes (ext_mpi_amd_comm_set_nodes;
    the reference's one-port inter-node schedule between the node legs) on a second RCCL
    communicator, at the run's size; checked against the float64 sum like the headline."""
    R = world // nodes
    try:
        uid = [emac.get_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm2 = emac.comm_init(rank, world, uid[0], dev)
        try:
            emac.comm_set_nodes(comm2, nodes, ports)
            st = 20
            h2, sb, rb, _, el, ok = _comm_run(emac, comm2, count, tdtype, code, dname, f"6;1 -{R} {R}", st, 3, rank,
                                              world, dist, torch)
            emac.done(h2)
            sb.free()
            rb.free()
        finally:
            emac.comm_free(comm2)
        log(f"rank {rank}: {nodes} nodes of {R}: {el * 1e6 / st:.2f} us, checked {ok}")
        return {"nodes": nodes, "ports": ports or "one per step", "ranks_per_node": R, "copyin": f"6;1 -{R} {R}", "bytes_per_rank": count * tdtype.itemsize,
                "us_per_allreduce": round(el * 1e6 / st, 2),
                "algbw_gbps": round(count * tdtype.itemsize * st / el / 1e9, 2), "checked": ok}
    except Exception as e:  # noqa: BLE001 -- an extra point, never the headline
        log(f"rank {rank}: {nodes}-node schedule failed: {e}")
        return {"error": str(e)[:200]}


def _node_form_run(emac, comm, R, count, tdtype, code, copyin, steps, warmup, rank, world, dist, torch):
    """N > 1 headline: configs[1]'s node (R ranks x count elements resident in this GPU) on every
    GPU, the GPUs joined as nodes (ext_mpi_amd_node_comm_allreduce_init over an RCCL communicator
    of one member per GPU): the node's copy-in fold, the inter-node legs over xGMI, the copy-out.
    Returns the max-over-ranks wall time of `steps` Starts, the check, and each part's time."""
    tsize = torch.empty((), dtype=tdtype).element_size()
    np_dtype = {torch.float32: np.float32, torch.float64: np.float64, torch.int32: np.int32,
                torch.int64: np.int64}[tdtype]
    set_bytes = 2 * R * count * tsize
    nsets = rotation_sets(R * count * tsize, set_bytes)  # every read from HBM (READ_REUSE_BYTES)
    stream = torch.cuda.Stream()
    sets, handles, mine = [], [], None
    for s in range(nsets):
        sends, recvs = [], []
        for r in range(R):
            b = DevBuf(count * tsize)
            a = host_random(count, np_dtype, 0x5EED0000 + 4099 * s + rank * R + r)  # global rank rank * R + r
            b.upload(a)
            if s == 0:
                mine = (mine or []) + [a]
            sends.append(b)
            recvs.append(DevBuf(count * tsize))
        h = emac.node_comm_allreduce_init([b.data_ptr() for b in sends], [b.data_ptr() for b in recvs], count, code,
                                          comm, copyin)
        emac.set_stream(h, stream.cuda_stream)
        sets.append((sends, recvs))
        handles.append(h)
    try:
        for k in range(max(warmup, nsets * TUNE_STARTS)):  # every handle past its fold tuning
            emac.start(handles[k % nsets])
        emac.start(handles[0])
        stream.synchronize()
        sched = emac.handle_schedule(handles[0])
        join_parts = emac.handle_join_parts(handles[0])
        # how many distinct GPUs the nodes ran on (1 in the shared-GPU rehearsal; N on a real node)
        devs = [None] * world
        dist.all_gather_object(devs, str(torch.cuda.get_device_properties(torch.cuda.current_device()).uuid))
        # check set 0 against a float64 sum over every rank of every node (sampled)
        idx = np.arange(0, count, max(1, count // (1 << 18)))
        got = []
        for b in (sets[0][1][0], sets[0][1][R - 1]):
            a = np.empty(count, np_dtype)
            b.download(a)
            got.append(a[idx])
        allin = [None] * world
        dist.all_gather_object(allin, [a[idx] for a in mine])
        ref = np.sum(np.stack([x.astype(np.float64) for node in allin for x in node]), axis=0)
        tol = 1e-5 * world * R if np.dtype(np_dtype).kind == "f" else 0.0
        good = bool(np.allclose(got[0].astype(np.float64), ref, rtol=0, atol=tol)) and np.array_equal(
            got[0].view(np.uint8), got[1].view(np.uint8))
        if not good:
            log(f"rank {rank}: node form over {world} GPUs: result check failed")
        ok = torch.tensor([int(good)])
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            emac.start(handles[k % nsets])
        stream.synchronize()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.barrier()
        dist.all_reduce(el, op=dist.ReduceOp.MAX)

        def part(legs, n):  # one part of the Start alone on every GPU at once; max over ranks
            dist.barrier()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for k in range(n):
                emac.start_legs(handles[k % nsets], legs)
            e1.record(stream)
            stream.synchronize()
            t = torch.tensor([e0.elapsed_time(e1) * 1e-3 / n], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return t.item()

        parts = {"copy_in_fold_s": part(emac.LEG_FOLD, steps),
                 "node_legs_s": part(emac.LEG_NODES_RS | emac.LEG_NODES_FOLD | emac.LEG_NODES_AG, steps),
                 "copy_out_s": part(emac.LEG_ALLGATHER, steps)}
        return {"wall": el.item(), "checked": bool(ok.item()), "schedule": sched, "nsets": nsets, "join_parts": join_parts,
                "distinct_devices": len(set(devs)), **parts}
    finally:
        for h in handles:
            emac.done(h)
        for sends, recvs in sets:
            for b in sends + recvs:
                b.free()


def node_child(args, emac, rank, world, dev, dist, torch, transport):
    """--child-transport node-ipc / node-rccl: the N > 1 headline (see _node_form_run), the nodes
    joined by one inter-node step of radix N (EXT_MPI_NUM_PORTS '-(N-1) (N-1)': every GPU trades
    with all N - 1 others at once, one xGMI link each) over a peer-mapped communicator (engine_join.c
    node_ipc_init: the nodes' partials read in place over xGMI) or over RCCL (the node legs as
    point-to-point groups). Each transport runs in a child of its own (multi_gpu), so one that hangs
    or faults cannot take the other down; every rank agrees on the outcome. Returns the result (with
    "checked") or {"error": ...}."""
    tdtype, code, dname, tsize = dtype_info(args.dtype)
    R = args.ranks
    count = int(args.size_mib * MIB) // tsize
    copyin = f"6;1 -{R} {R}"  # the node's own split (configs[1]); --copyin is the one-rank-per-GPU runs'
    ports = [-(world - 1), world - 1] if world > 1 else []
    out = {}
    for transport in (transport,):
        comm, res = None, None
        try:
            if transport == "ipc":
                comm = emac.comm_init_ipc(rank, world, emac.torch_allgather(), dev)
            else:
                uid = [emac.get_unique_id() if rank == 0 else None]
                dist.broadcast_object_list(uid, src=0)
                comm = emac.comm_init(rank, world, uid[0], dev)
            if world > 1:
                emac.comm_set_nodes(comm, world, ports)
            t_run = time.monotonic()
            res = _node_form_run(emac, comm, R, count, tdtype, code, copyin, args.steps, args.warmup, rank, world, dist,
                                 torch)
            log(f"rank {rank}: node form over {world} GPUs ({transport}): {args.steps} steps in "
                f"{res['wall'] * 1e3:.3f} ms, checked {res['checked']}")
            # beside the default (fused, pipelined) peer-mapped join, the serial one on the same node,
            # when the child's deadline leaves room for a second run (rank 0 decides for all): which
            # join is faster across GPUs is measured, not assumed
            again = torch.tensor([int(transport == "ipc" and world > 1 and res.get("join_parts", 1) > 1 and
                                      (time.monotonic() - t_run) < 0.3 * args.child_deadline)])
            dist.broadcast(again, src=0)
            if again.item():
                saved = os.environ.get("EXT_MPI_AMD_JOIN_PARTS")
                os.environ["EXT_MPI_AMD_JOIN_PARTS"] = "1"
                try:
                    ser = _node_form_run(emac, comm, R, count, tdtype, code, copyin, args.steps, args.warmup, rank,
                                         world, dist, torch)
                finally:
                    if saved is None:
                        del os.environ["EXT_MPI_AMD_JOIN_PARTS"]
                    else:
                        os.environ["EXT_MPI_AMD_JOIN_PARTS"] = saved
                res["serial_join"] = {"ms_per_step": round(ser["wall"] * 1e3 / args.steps, 4), "checked": ser["checked"],
                                      "join_parts": ser["join_parts"],
                                      "parts_us": {k: round(ser[k] * 1e6, 2) for k in ("copy_in_fold_s", "node_legs_s",
                                                                                      "copy_out_s")}}
                log(f"rank {rank}: serial join over {world} GPUs: {res['serial_join']}")
            res.update(ranks_per_gpu=R, copyin=copyin, ports=ports, bytes_per_rank=count * tsize, transport=transport)
        except Exception as e:  # noqa: BLE001 -- every rank reports and agrees below
            log(f"rank {rank}: node form over {world} GPUs ({transport}) failed: {e}")
            res = {"error": str(e)[:200]}
        finally:
            if comm is not None:
                try:
                    emac.comm_free(comm)
                except Exception:  # noqa: BLE001
                    pass
        ok = torch.tensor([int("wall" in res)])
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        out[transport] = res if ok.item() else (res if "error" in res else {"error": "failed on another rank"})
    res = out[transport]
    if "wall" not in res:
        res["checked"] = False
    return res


def transport_child(args):
    """One transport's N > 1 measurement in a process of its own (spawned by multi_gpu): its own
    gloo group, its own HIP context. Writes this rank's results as JSON to --child-result."""
    import torch
    import torch.distributed as dist
    import ext_mpi_collectives_amd as emac
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    import signal
    signal.signal(signal.SIGALRM, lambda *_: (log(f"rank {rank}: watchdog expired"), os._exit(3)))
    signal.alarm(max(1, int(args.child_deadline)))  # a rank stuck in a collective must not hang the job
    ndev = torch.cuda.device_count()
    dev = local % ndev  # one rank per GPU; ranks share a GPU only when there are fewer GPUs (rehearsal)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    tdtype, code, dname, tsize = dtype_info(args.dtype)
    count = int(args.size_mib * MIB) // tsize
    copyin = args.copyin or f"6;1 -{world} {world}"
    transport, full = args.child_transport, args.child_full
    res = {}
    log(f"rank {rank}: {transport} child on GPU {dev}: communicator set-up")
    if transport.startswith("node-"):  # the N > 1 headline over one transport (node_child)
        res = node_child(args, emac, rank, world, dev, dist, torch, transport[5:])
        with open(args.child_result.replace("{rank}", str(rank)), "w") as f:
            json.dump(res, f)
        dist.barrier()
        dist.destroy_process_group()
        signal.alarm(0)
        return
    if transport == "ipc":
        comm = emac.comm_init_ipc(rank, world, emac.torch_allgather(), dev)
    else:
        uid = [emac.get_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = emac.comm_init(rank, world, uid[0], dev)
    log(f"rank {rank}: {transport} child: communicator ready")
    try:
        h, send, recv, stream, wall, checked = _comm_run(emac, comm, count, tdtype, code, dname, copyin,
                                                         args.steps, args.warmup, rank, world, dist, torch)
        res.update(wall=wall, checked=checked)
        log(f"rank {rank}: {transport}: {args.steps} steps in {wall * 1e3:.3f} ms, checked {checked}")
        if full:
            # the fold leg alone on every GPU at once, then on rank 0's GPU while the others idle
            dist.barrier()
            fold_s = torch.tensor([_fold_only(emac, h, stream, args.steps, torch)], dtype=torch.float64)
            dist.all_reduce(fold_s, op=dist.ReduceOp.MAX)
            dist.barrier()
            alone_s = torch.zeros(1, dtype=torch.float64)
            if rank == 0:
                alone_s[0] = _fold_only(emac, h, stream, args.steps, torch)
            dist.barrier()
            dist.broadcast(alone_s, src=0)
            res.update(fold_s=fold_s.item(), alone_s=alone_s.item())
            # SURVEY.md 8(d)'s 'per-GPU rate retained': the LOCAL fold kernel (R leaves of this
            # run's chunk size -> 1 destination, all in this GPU's HBM) on every GPU at once
            # inside the N-GPU job, against the same kernel on rank 0's GPU while the others idle
            chunk = max(1, count // world)
            dist.barrier()
            lfr = comm_shape_fold(world, chunk, tdtype, code, 100)
            lf = torch.tensor([lfr["avg_launch_us"]], dtype=torch.float64)
            dist.all_reduce(lf, op=dist.ReduceOp.MAX)
            dist.barrier()
            lf_alone = torch.zeros(1, dtype=torch.float64)
            if rank == 0:
                lf_alone[0] = comm_shape_fold(world, chunk, tdtype, code, 100)["avg_launch_us"]
            dist.barrier()
            dist.broadcast(lf_alone, src=0)
            res["local_fold"] = {"leaves": world, "chunk_bytes": chunk * tsize, "us_all_gpus": lf.item(),
                                 "us_rank0_alone": lf_alone.item(),
                                 "rate_retained": round(lf_alone.item() / lf.item(), 3), "schedule": lfr["schedule"]}
        emac.done(h)
        send.free()
        recv.free()
        if transport == "rccl":
            res["rccl_allreduce_baseline"] = _rccl_allreduce_baseline(rank, world, dist, torch)
            if world >= 2 and world % 2 == 0:
                res["two_node_schedule"] = _node_point(emac, rank, world, dev, count, tdtype, code, dname, dist,
                                                       torch)
            if world >= 4 and world % 4 == 0:  # two radix-2 node steps (4 nodes), and one radix-4 step
                res["four_node_schedule"] = _node_point(emac, rank, world, dev, count, tdtype, code, dname, dist,
                                                        torch, nodes=4)
                res["four_node_three_ports"] = _node_point(emac, rank, world, dev, count, tdtype, code, dname, dist,
                                                           torch, nodes=4, ports=[-3, 3])
        if full:
            # BASELINE configs[3] (double, 256 MiB per rank) and a configs[4]-style size sweep
            points = [(args.dtype, n) for n in (8, 64 << 10, 1 << 20, 16 << 20, 64 << 20, 256 << 20, 512 << 20)]
            points.append(("double", 256 << 20))
            sweep = []
            for dname_p, nbytes in points:
                tdt, cde, _, tsz = dtype_info(dname_p)
                cnt = max(1, nbytes // tsz)
                st = 100 if nbytes <= (1 << 20) else 10
                hp, sb, rb, _, el_p, ok_p = _comm_run(emac, comm, cnt, tdt, cde, dname_p, copyin, st, 3, rank,
                                                      world, dist, torch)
                emac.done(hp)
                sb.free()
                rb.free()
                sweep.append({"dtype": dname_p, "bytes_per_rank": cnt * tsz,
                              "us_per_allreduce": round(el_p * 1e6 / st, 2),
                              "algbw_gbps": round(cnt * tsz * st / el_p / 1e9, 2), "checked": ok_p})
                log(f"rank {rank}: {transport}: sweep {dname_p} {cnt * tsz} B: {el_p * 1e6 / st:.2f} us, checked {ok_p}")
            res["sweep"] = sweep
            # BASELINE configs[4]: EXT_MPI_COPYIN radix variants of this node size (radix chains and
            # the small-message -64 fraction) beside the linear fold, latency to bandwidth sizes
            radix = []
            for cp in (copyin,) + RADIX_VARIANTS.get(world, ()):
                for nbytes in RADIX_SWEEP_BYTES:
                    cnt, st = max(1, nbytes // tsize), 100 if nbytes <= (1 << 20) else 20
                    hp, sb, rb, _, el_p, ok_p = _comm_run(emac, comm, cnt, tdtype, code, dname, cp, st, 3, rank, world,
                                                          dist, torch)
                    emac.done(hp)
                    sb.free()
                    rb.free()
                    radix.append({"copyin": cp, "bytes_per_rank": cnt * tsize, "us_per_allreduce": round(el_p * 1e6 / st, 2),
                                  "algbw_gbps": round(cnt * tsize * st / el_p / 1e9, 2), "checked": ok_p})
                    log(f"rank {rank}: {transport}: '{cp}' {nbytes} B: {el_p * 1e6 / st:.2f} us, checked {ok_p}")
            radix_vs_linear(radix, copyin, "us_per_allreduce")
            res["radix_crossover"] = radix_crossovers(radix, "us_per_allreduce", world)
            res["radix_sweep"] = radix
            # the path's real start and end: page-locked host send / receive buffers, staged through
            # device mirrors on each rank's own PCIe link (H2D, legs, D2H on the handle's stream)
            hp, sb, rb, _, el_p, ok_p = _comm_run(emac, comm, count, tdtype, code, dname, copyin, 10, 3, rank, world,
                                                  dist, torch, host=True)
            emac.done(hp)
            sb.free()
            rb.free()
            res["host_buffers"] = {"bytes_per_rank": count * tsize, "us_per_allreduce": round(el_p * 1e6 / 10, 2),
                                   "gbps_reduced_job": round(world * count * tsize * 10 / el_p / 1e9, 2),
                                   "checked": ok_p}
            log(f"rank {rank}: {transport}: host buffers {count * tsize} B: {el_p * 1e5:.2f} us, checked {ok_p}")
    finally:
        emac.comm_free(comm)
    with open(args.child_result.replace("{rank}", str(rank)), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()
    signal.alarm(0)


MULTI_DEADLINE_S = 1200.0  # the whole N > 1 bench (every child of every rank), EXT_MPI_AMD_BENCH_DEADLINE overrides
CHILD_MAX_S = 600.0  # one child at most (its own watchdog, --child-deadline, fires first)


def run_child_process(cmd, env, timeout_s, tail_lines=12):
    """Run one child (its stderr passed through line by line, its last lines kept) under a time
    limit; returns (rc or "timeout", elapsed seconds, last stderr lines). A child that outlives its
    limit is killed with its whole process group."""
    import collections
    import signal
    import subprocess
    import threading
    tail = collections.deque(maxlen=tail_lines)
    t0 = time.monotonic()
    p = subprocess.Popen(cmd, env=env, stderr=subprocess.PIPE, start_new_session=True)

    def pump():
        for raw in iter(p.stderr.readline, b""):
            line = raw.decode(errors="replace").rstrip()
            tail.append(line[:300])
            print(line, file=sys.stderr, flush=True)

    th = threading.Thread(target=pump, daemon=True)
    th.start()
    try:
        rc = p.wait(timeout=max(1.0, timeout_s))
    except subprocess.TimeoutExpired:
        rc = "timeout"
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
        p.wait()
    th.join(timeout=5)
    return rc, round(time.monotonic() - t0, 1), list(tail)


def child_outcome(transport, rc, elapsed, tail, result):
    """(result or {}, None) for a child that completed and checked, else ({}, failure record): the
    transport, the exit code ("timeout" when killed at its limit), its time and last stderr lines."""
    if rc == 0 and result is not None:
        if result.get("checked"):
            return result, None
        return result, {"transport": transport, "rc": 0, "error": result.get("error") or "result check failed",
                        "elapsed_s": elapsed, "stderr_tail": tail}
    what = "timed out" if rc == "timeout" else f"exited with {rc}" if rc != 0 else "wrote no result"
    return {}, {"transport": transport, "rc": rc, "error": f"{transport} child {what}", "elapsed_s": elapsed,
                "stderr_tail": tail}


def multi_gpu(args):
    """N > 1 driver rank. It never touches the GPU itself: each transport runs in a child process
    per rank (own gloo group, own HIP context), so a transport that fails -- even by a GPU fault
    that ends its processes -- leaves these ranks alive to agree on it and try the other one. The
    whole run is bounded (MULTI_DEADLINE_S): each child gets at most what is left of it, and a
    child killed at its limit, or one that fails, is reported with its exit code and last stderr
    lines in the line's extras -- a valid JSON line comes out either way."""
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    tdtype, code, dname, tsize = dtype_info(args.dtype)
    count = int(args.size_mib * MIB) // tsize
    S = count * tsize
    copyin = args.copyin or f"6;1 -{world} {world}"
    base_port = int(os.environ.get("MASTER_PORT", "29500"))
    deadline = time.monotonic() + float(os.environ.get("EXT_MPI_AMD_BENCH_DEADLINE", MULTI_DEADLINE_S))

    def everyone(ok):
        t = torch.tensor([int(bool(ok))])
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    # ranks sharing a GPU (a rehearsal on fewer GPUs than ranks): at HIP's default of 4 hardware queues
    # per process, 8 processes oversubscribe the GPU's queue slots and the scheduler time-slices them,
    # ~22.5 ms per Allreduce whatever its size; 2 queues each keep every queue resident
    # (profiles/r06/rehearsal/: 22.9 ms against 0.50 ms per Start). One process per GPU is untouched.
    shared_hwq = shared_hw_queues(torch.cuda.device_count(), world, os.environ.get("GPU_MAX_HW_QUEUES"))

    def run_child(i, transport, full, share):
        out = os.path.join("/tmp", f"emac_bench_{base_port}_{i}_{rank}.json")
        if os.path.exists(out):
            os.remove(out)
        # this child's share of what is left of the run (every rank computes the same budget)
        budget = min(CHILD_MAX_S, max(30.0, (deadline - time.monotonic()) * share))
        cmd = [sys.executable, os.path.abspath(__file__), "--gpus", str(args.gpus), "--steps", str(args.steps),
               "--warmup", str(args.warmup), "--size-mib", str(args.size_mib), "--dtype", args.dtype,
               "--ranks", str(args.ranks), "--child-transport", transport, "--child-result", out,
               "--child-deadline", str(int(budget))] + (["--child-full"] if full else []) + \
              (["--copyin", args.copyin] if args.copyin else [])
        env = dict(os.environ, MASTER_PORT=str(base_port + 101 + i))
        if shared_hwq:
            env["GPU_MAX_HW_QUEUES"] = shared_hwq
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)  # the children's rank 0 hosts their own store
        rc, elapsed, tail = run_child_process(cmd, env, budget + 20)  # the child's watchdog fires first
        result = None
        if rc == 0 and os.path.exists(out):
            with open(out) as f:
                result = json.load(f)
            os.remove(out)
        return child_outcome(transport, rc, elapsed, tail, result)

    failures = []
    # the headline: configs[1]'s node (8 ranks x 16 MiB resident in one GPU) on every GPU, the GPUs
    # joined as nodes -- the N = 1 workload scaled weakly -- peer-mapped first, then over RCCL,
    # each in its own children
    node = {}
    for i, (t, share) in enumerate((("ipc", 0.3), ("rccl", 0.35))):
        r, fail = run_child(9 + i, f"node-{t}", False, share)
        if fail:
            failures.append(dict(fail, rank=rank))
        if not everyone(fail is None):
            r = fail or {"error": "failed on another rank"}
        node[t] = r
    rn = node_result(node, args.steps)
    # BASELINE configs[3] / [4] (one rank per GPU): the requested transport first; if it fails on
    # any rank (every rank agrees before moving on), the other one
    order = [args.transport, "rccl" if args.transport == "ipc" else "ipc"]
    results = {}
    for i, transport in enumerate(order):
        full = not any("wall" in r for r in results.values())
        r, fail = run_child(i, transport, full, 0.6 if i == 0 else 0.9)
        if fail:
            failures.append(dict(fail, rank=rank))
        if not everyone(fail is None):
            r = fail or {"error": "failed on another rank"}
        results[transport] = r
    allf = [None] * world
    dist.all_gather_object(allf, failures)
    if rank == 0:
        line = multi_gpu_line(args, world, dname, S, copyin, rn, results, order, torch.cuda.device_count(),
                              [f for fs in allf for f in fs])
        if shared_hwq:
            line.setdefault("extras", {})["gpu_max_hw_queues_per_process"] = int(shared_hwq)
        emit(line)
    dist.barrier()
    dist.destroy_process_group()


def shared_hw_queues(devices, world, env_value):
    """GPU_MAX_HW_QUEUES for the N > 1 children: None (left alone) with one rank per GPU, else at most
    2 -- an exported value is capped, not kept, since the GPU boxes export HIP's default of 4, at which
    8 processes sharing one GPU time-slice (profiles/r06/rehearsal/)."""
    if devices >= world:
        return None
    try:
        v = int(env_value) if env_value else 4
    except ValueError:
        v = 4
    return str(max(1, min(2, v)))


def node_result(node, steps):
    """The headline's node-form result from the per-transport ones: the peer-mapped one when it ran
    and checked, else RCCL's, else an error naming both; `transports` keeps each one's summary."""
    head = next((node[t] for t in ("ipc", "rccl") if t in node and "wall" in node[t] and node[t].get("checked")), None)
    res = dict(head or {"error": "; ".join(f"{t}: {r.get('error', 'unchecked')}" for t, r in node.items()),
                        "checked": False})
    res["transports"] = {t: ({"ms_per_step": round(r["wall"] * 1e3 / steps, 4), "checked": r["checked"],
                              "parts_us": {k: round(r[k] * 1e6, 2) for k in ("copy_in_fold_s", "node_legs_s",
                                                                            "copy_out_s")}}
                             if "wall" in r else r) for t, r in node.items()}
    return res


def multi_gpu_line(args, world, dname, S, copyin, rn, results, order, gpus_visible, failures):
    """The N > 1 JSON line from the children's results (pure: tests/test_bench_cpu.py feeds it
    fabricated ones): the node form's line when its child ran and checked, else the one-rank-per-GPU
    line of the first transport that completed, else a zero line naming every failure."""
    primary = next((t for t in order if "wall" in results[t] and "fold_s" in results[t]), None)
    extras = {"gpus_visible": gpus_visible, "process_per_transport": True}
    if failures:
        extras["failures"] = failures  # per rank: transport, exit code or "timeout", last stderr lines
    for t in order:
        if t != primary:
            r = results[t]
            extras[f"{t}_transport"] = r if "wall" not in r else {
                "ms_per_step": round(r["wall"] * 1e3 / args.steps, 4),
                "value": round(world * S * args.steps / r["wall"] / 1e9, 2), "checked": r["checked"]}
        if "rccl_allreduce_baseline" in results[t]:  # whichever role RCCL had
            extras["rccl_allreduce_baseline"] = results[t]["rccl_allreduce_baseline"]
        for key in ("two_node_schedule", "four_node_schedule", "four_node_three_ports"):
            if key in results[t]:
                extras[key] = results[t][key]
    metric = "device-resident GB/s reduced (float32 MPI_SUM) per GPU; % HBM3E roofline"
    if primary is None:
        legacy = {"metric": metric, "value": 0.0, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                  "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
                  "vs_baseline": None, "dtype": dname, "data": "synthetic", "error": "no transport completed",
                  "config": {"workload": f"persistent Allreduce {args.dtype} MPI_SUM, {S // MIB} MiB per rank, one rank "
                                         f"per GPU, EXT_MPI_COPYIN '{copyin}' (no transport completed: "
                                         + "; ".join(f"{t}: {results[t].get('error', 'unchecked')}" for t in order)
                                         + ")",
                             "ranks": world, "message_bytes_per_rank": S, "copyin": copyin, "layout": "rank-per-gpu"},
                  "roofline": None, "extras": extras}
    else:
        r = results[primary]
        wall, checked, kf = r["wall"], r["checked"], r["fold_s"]
        extras["transport"] = primary
        extras["sweep"] = r.get("sweep", [])
        extras["radix_sweep"] = r.get("radix_sweep", [])
        extras["radix_crossover"] = r.get("radix_crossover", {})
        extras["local_fold_rate_retained"] = r.get("local_fold")
        extras["host_buffers_pcie_inclusive"] = r.get("host_buffers")
        chunk = S / world
        # the fold leg of the run's own transport: R leaf reads (R-1 of them over xGMI in the IPC
        # form, from staging in the RCCL form) + 1 write of the owned chunk
        algo = (world + 1) * chunk
        remote = (world - 1) * chunk if primary == "ipc" else 0
        extras.update({
            "fold_us_all_gpus": round(kf * 1e6, 2), "fold_us_rank0_alone": round(r["alone_s"] * 1e6, 2),
            "fold_algorithmic_bytes": int(algo),
            "per_gpu_fold_rate_retained": round(r["alone_s"] / kf, 3),
            "fold_xgmi_gbps_per_gpu": round(remote / kf / 1e9, 1) if remote else None,
            "value_per_gpu_gbps": round(S * args.steps / wall / 1e9, 2),
            "end_to_end_algbw_gbps_per_gpu": round(S * args.steps / wall / 1e9, 2),
            "xgmi_bound_us": round(2 * (world - 1) / world * S / (min(world - 1, 7) * 153e9) * 1e6, 1)})
        # roofline: the LOCAL fold kernel of SURVEY.md 8(d) (R leaves of this run's chunk -> 1
        # destination, all in this GPU's HBM) timed on every GPU at once inside the N-GPU job: the
        # HBM-bound kernel. The transport's own fold reads R-1 leaves over xGMI and is priced
        # against the xGMI links in extras (fold_xgmi_gbps_per_gpu, xgmi_bound_us).
        lfd = r.get("local_fold") or {}
        kl = lfd.get("us_all_gpus", kf * 1e6) * 1e-6
        achieved = algo / kl / 1e9
        # the N > 1 Allreduce is bound by xGMI (each GPU moves 2(N-1)/N S over its links), not by
        # HBM as the N = 1 kernel-only workload (8 node ranks in one HBM) is: its fraction of
        # that bound, and what N = 1 measures instead
        extras["end_to_end_frac_of_xgmi_bound"] = (
            round(extras["xgmi_bound_us"] / (wall * 1e6 / args.steps), 3)
            if gpus_visible >= world else None)  # ranks sharing a GPU cross no xGMI
        extras["note_vs_n1"] = ("N = 1 is BASELINE configs[1]: 8 node ranks resident in one GPU's HBM, HBM-bound; "
                                "N > 1 is one rank per GPU, every rank's chunk crossing xGMI (bound: xgmi_bound_us)")
        form = ("peer-mapped (hipIpc over xGMI): barrier kernel, fold of the owned chunk over the peers' send "
                "buffers into the own receive buffer, barrier kernel, pull of the other owners' chunks"
                if primary == "ipc" else
                "reduce-scatter + allgather legs over RCCL/xGMI, fold on the owner GPU")
        legacy = {
            "metric": metric,
            "value": round(world * S * args.steps / wall / 1e9, 2),
            "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall * 1e3 / args.steps, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": dname,
            "data": "synthetic: uniform [-1,1) per rank (seeded), device-resident (hipMalloc)",
            "config": {"workload": f"persistent Allreduce {args.dtype} MPI_SUM, {S // MIB} MiB per rank, one rank per "
                                   f"GPU, EXT_MPI_COPYIN '{copyin}': {form}; value = bytes reduced by the whole job "
                                   f"per second (N x {S // MIB} MiB per step), extras.value_per_gpu_gbps = value / N",
                       "ranks": world, "message_bytes_per_rank": S, "copyin": copyin, "layout": "rank-per-gpu",
                       "transport": primary, "checked_vs_fp64_sum": checked},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
                         "kernel": f"{fold_kernel_name(lfd.get('schedule'))} (local fold: R leaves of the run's chunk -> 1, "
                                   "this GPU's HBM)",
                         "algorithmic_bytes_per_launch": int(algo), "avg_launch_us": round(kl * 1e6, 2)},
            "extras": extras,
        }
    if "wall" in rn and rn.get("checked"):
        line = node_form_line(args, world, dname, rn, legacy)
        if failures:
            line["extras"]["failures"] = failures
        return line
    legacy["extras"]["node_form_per_gpu"] = rn
    return legacy


def node_form_line(args, world, dname, rn, one_rank_per_gpu):
    """The N > 1 JSON line: configs[1]'s node on each of the N GPUs (weak scaling of the N = 1
    workload), the nodes joined over xGMI (peer-mapped, else RCCL). value = bytes reduced by the whole job per second
    (N GPUs x R ranks x S bytes per Start); roofline = the node's copy-in fold (R leaves -> the
    owner chunks, this GPU's HBM) timed on every GPU at once inside the job."""
    R, S, steps = rn["ranks_per_gpu"], rn["bytes_per_rank"], args.steps
    wall = rn["wall"]
    t_in, t_x, t_out = rn["copy_in_fold_s"], rn["node_legs_s"], rn["copy_out_s"]
    algo_in = (R + 1) * S  # R leaf reads of every owner chunk + one write of each (SURVEY.md 8d B_in)
    achieved = algo_in / t_in / 1e9
    xb = 2 * (world - 1) / world * S  # the node partial crosses xGMI out and back (reduce-scatter + allgather)
    xgmi_bound = xb / (min(world - 1, 7) * 153e9)
    extras = {
        "form": ("NODE form over peer-mapped nodes (ext_mpi_amd_node_comm_allreduce_init on an IPC communicator): "
                 "per GPU one node of R ranks; copy-in fold into the node's partial block, barrier, fold of this "
                 "node's share of every chunk over the N partials read in place over xGMI (EXT_MPI_NUM_PORTS one "
                 "step of radix N), barrier, pull of every share, the copy-out fan-out"
                 if rn.get("transport") == "ipc" else
                 "NODE form over nodes (ext_mpi_amd_node_comm_allreduce_init): per GPU one node of R ranks; "
                 "copy-in fold of the node in place, the inter-node legs of every node rank as one RCCL group per "
                 "leg (EXT_MPI_NUM_PORTS one step of radix N), the copy-out fan-out"),
        "node_transports": rn.get("transports"),
        "parts_us": {"copy_in_fold": round(t_in * 1e6, 2), "node_legs_xgmi": round(t_x * 1e6, 2),
                     "copy_out": round(t_out * 1e6, 2), "sum": round((t_in + t_x + t_out) * 1e6, 2),
                     "start_to_wait": round(wall * 1e6 / steps, 2)},
        # (peer-mapped members: the copy-out is fused into the node legs' pull, its part is empty)
        "copy_out_achieved_gbps": round(R * S / t_out / 1e9, 1) if t_out > 1e-6 else None,
        # the peer-mapped join pipelined by parts (engine_join.c emac_join; 1: serial): its copy-ins
        # overlap the node legs, so start_to_wait can fall below the sum of the parts timed alone
        "join_parts": rn.get("join_parts"),
        "serial_join": rn.get("serial_join"),
        "distinct_devices": rn.get("distinct_devices"),
        "node_legs_xgmi_bound_us": round(xgmi_bound * 1e6, 1),
        "node_legs_frac_of_xgmi_bound": round(xgmi_bound / t_x, 3) if t_x > 0 else None,
        "value_per_gpu_gbps": round(R * S * steps / wall / 1e9, 2),
        "fold_schedule": rn.get("schedule"), "buffer_sets": rn.get("nsets"),
        "one_rank_per_gpu": one_rank_per_gpu,
    }
    return {
        "metric": "device-resident GB/s reduced (float32 MPI_SUM) per GPU; % HBM3E roofline",
        "value": round(world * R * S * steps / wall / 1e9, 2),
        "unit": "GB/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
        "ms_per_step": round(wall * 1e3 / steps, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": dname,
        "data": "synthetic: uniform [-1,1) per rank (seeded), device-resident (hipMalloc), "
                f"{rn.get('nsets')} rotated buffer sets per GPU",
        "config": {"workload": f"persistent Allreduce {args.dtype} MPI_SUM over {world} x {R} ranks: BASELINE "
                               f"configs[1]'s node ({R} ranks x {S // MIB} MiB resident in one MI355X, "
                               f"EXT_MPI_COPYIN '{rn['copyin']}') on each of {world} GPUs, the GPUs joined as "
                               f"nodes over xGMI ({'peer-mapped' if rn.get('transport') == 'ipc' else 'RCCL'}, "
                               f"EXT_MPI_NUM_PORTS {rn['ports']}); value = bytes reduced by "
                               f"the whole job per second ({world} x {R} x {S // MIB} MiB per step)",
                   "ranks": world * R, "ranks_per_gpu": R, "message_bytes_per_rank": S, "copyin": rn["copyin"],
                   "node_ports": rn["ports"], "layout": "node-per-gpu", "transport": rn.get("transport", "rccl"),
                   "checked_vs_fp64_sum": rn["checked"]},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None,
                     "kernel": f"{fold_kernel_name(rn.get('schedule'))} (the node's copy-in: R leaves -> owner chunk, this GPU's HBM)",
                     "algorithmic_bytes_per_launch": int(algo_in), "avg_launch_us": round(t_in * 1e6, 2)},
        "extras": extras,
    }


# BASELINE configs[4]'s EXT_MPI_COPYIN variants per node size (beside the linear '6;1 -R R'), and the
# sizes per rank they are swept at: the -k fractions are the reference's small-message split
RADIX_VARIANTS = {8: ("6;1 -2 -2 -2 2 2 2", "6;1 -4 -2 2 4", "6;-64 -8 8"), 4: ("6;1 -2 -2 2 2", "6;-64 -4 4"),
                  2: ("6;-64 -2 2",)}
RADIX_SWEEP_BYTES = (8, 1 << 10, 64 << 10, 1 << 20, 16 << 20)


def radix_vs_linear(points, linear, key):
    """Each point's time against the linear fold's at the same size (linear / variant: > 1 faster)."""
    lin = {p["bytes_per_rank"]: p[key] for p in points if p["copyin"] == linear}
    for p in points:
        if p["bytes_per_rank"] in lin and p[key] > 0:
            p["vs_linear"] = round(lin[p["bytes_per_rank"]] / p[key], 4)


def radix_crossovers(points, key, R):
    """Per EXT_MPI_COPYIN variant, its latency -> bandwidth crossover: the fixed cost (the shortest time
    of the points up to 1 KiB per rank), the streaming rate (GB/s reduced between the two largest
    points) and the size per rank at which streaming time equals the fixed cost."""
    out = {}
    for cp in dict.fromkeys(p["copyin"] for p in points):
        pts = sorted((p["bytes_per_rank"], p[key]) for p in points if p["copyin"] == cp)
        small = sorted(t for b, t in pts if b <= 1024)
        if len(pts) < 3 or not small or pts[-1][1] <= pts[-2][1]:
            continue
        fixed = small[0]
        (b1, t1), (b2, t2) = pts[-2], pts[-1]
        rate = R * (b2 - b1) / ((t2 - t1) * 1e-6)  # bytes reduced per second
        out[cp] = {"fixed_us": round(fixed, 2), "streaming_gbps_reduced": round(rate / 1e9, 1),
                   "crossover_bytes_per_rank": int(fixed * 1e-6 * rate / R)}
    return out


def _fit_line(xs, ys):
    """least-squares y = a + b x: (a, b)"""
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    return my - b * mx, b


def small_sweep(emac, torch):
    """BASELINE configs[2]'s launch size class: the int node form (8 ranks, MPI_SUM, tuned schedule)
    at 0.5 - 16 MiB per rank against a 1:1 copy of the same bytes (tools/ceiling.hip, the best of
    its three variants) on the same lease, both rotated past the 256 MiB Infinity Cache. A straight
    line through launch time against bytes separates the fixed cost of a launch (its intercept:
    dispatch, first-load latency, store drain) from the streaming rate (its slope)."""
    L = _ceiling_lib()
    stream = torch.cuda.current_stream()
    pts = []
    for mb in (0.5, 1, 2, 4, 8, 16):
        per_rank = int(mb * MIB)
        x = node_run(8, per_rank // 4, torch.int32, emac.INT, "6;1 -8 8", 50, 5, alloc="hip")
        fold_us = x["event_ms"] * 1e3 / 50
        n = 8 * per_rank  # the fold reads 8 x per_rank and writes 8 x per_rank: a copy of n bytes
        pairs = rotation_sets(n, 2 * n)
        a = DevBuf(pairs * 2 * n)
        best = None
        for variant in (0, 1, 2):
            for i in range(pairs):
                L.ceiling_copy(a.data_ptr() + i * 2 * n, a.data_ptr() + i * 2 * n + n, n, 1, variant, stream.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(50):
                b = a.data_ptr() + (i % pairs) * 2 * n
                assert L.ceiling_copy(b, b + n, n, 1, variant, stream.cuda_stream) == 0
            e1.record(stream)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 50
            best = us if best is None else min(best, us)
        a.free()
        pts.append({"mib_per_rank": mb, "bytes_per_launch": 2 * n, "fold_us": round(fold_us, 2),
                    "copy_us": round(best, 2), "fold_frac_8tbs": round(2 * n / fold_us / 1e3 / HBM_PEAK_GBPS, 4),
                    "fold_over_copy": round(best / fold_us, 3), "schedule": x["schedule"], "checked": x["checked"]})
        log(f"small sweep {mb} MiB/rank: {pts[-1]}")
    out = {"points": pts}
    for k in ("fold", "copy"):
        a0, b0 = _fit_line([p["bytes_per_launch"] for p in pts], [p[f"{k}_us"] for p in pts])
        out[f"{k}_fit"] = {"fixed_us": round(a0, 2), "streaming_gbps": round(1e-3 / b0, 1)}
    return out


def join_copyin_alone(emac, torch, steps=40):
    """The peer-mapped node join's copy-in alone on a one-node communicator (configs[1]'s node, 8 ranks
    x 16 MiB): the fused join's (join_fused_kernel, mode 1: CI segments only; EXT_MPI_AMD_JOIN_PARTS,
    default 2) beside the serial join's tuned fold over the same bytes. Rotated buffer sets as the
    headline. For rocprofv3 PMC passes every join_fused_kernel dispatch of this run is a copy-in."""
    R, count = 8, 16 * MIB // 4
    parts = os.environ.get("EXT_MPI_AMD_JOIN_PARTS", "2")
    comm = emac.comm_init_ipc(0, 1, lambda p: [p], torch.cuda.current_device())
    out = {}
    try:
        for label, p in (("fused", parts), ("serial", "1")):
            os.environ["EXT_MPI_AMD_JOIN_PARTS"] = p
            nsets = rotation_sets(R * count * 4, 2 * R * count * 4)
            stream = torch.cuda.Stream()
            sets, handles = [], []
            for s in range(nsets):
                sends = [DevBuf(count * 4) for _ in range(R)]
                recvs = [DevBuf(count * 4) for _ in range(R)]
                for r, b in enumerate(sends):
                    b.upload(host_random(count, np.float32, 0x5EED0000 + 4099 * s + r))
                h = emac.node_comm_allreduce_init([b.data_ptr() for b in sends], [b.data_ptr() for b in recvs], count,
                                                  emac.FLOAT, comm, "6;1 -8 8")
                emac.set_stream(h, stream.cuda_stream)
                sets.append(sends + recvs)
                handles.append(h)
            try:
                for k in range(nsets * TUNE_STARTS):  # the serial join's fold past its tuning
                    emac.start_legs(handles[k % nsets], emac.LEG_FOLD)
                stream.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for k in range(steps):
                    emac.start_legs(handles[k % nsets], emac.LEG_FOLD)
                e1.record(stream)
                stream.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / steps
                out[label] = {"join_parts": emac.handle_join_parts(handles[0]), "avg_launch_us": round(us, 2),
                              "achieved_gbps": round((R + 1) * count * 4 / (us * 1e-6) / 1e9, 1),
                              "schedule": emac.handle_schedule(handles[0])}
                log(f"joinci {label}: {out[label]}")
            finally:
                for h in handles:
                    emac.done(h)
                for bs in sets:
                    for b in bs:
                        b.free()
    finally:
        os.environ["EXT_MPI_AMD_JOIN_PARTS"] = parts
        emac.comm_free(comm)
    return {"bytes_per_launch": (R + 1) * count * 4, **out}


def shape_only(args):
    """One fold shape alone (for rocprofv3 PMC passes): the local fold (8 x 32 MiB -> 1) or the
    node-form Allreduce at 256 / 16 MiB per rank, 40 launches after warm-up."""
    import torch
    import ext_mpi_collectives_amd as emac
    emac.lib()
    DevBuf.CONTIG = args.alloc == "contig"
    MB = {"node16": 16, "node64": 64, "node512": 512, "int4": 4, "long4": 4}.get(args.shape, 256) * MIB
    if args.shape == "local256" and args.schedules:  # every listed schedule in turn (EXT_MPI_AMD_FOLD_SCHEDULE)
        r = {}
        for w in args.schedules.split(","):
            os.environ["EXT_MPI_AMD_FOLD_SCHEDULE"] = w
            x = comm_shape_fold(8, MB // 8 // 4, torch.float32, emac.FLOAT, 40)
            r[w] = {"avg_launch_us": x["avg_launch_us"], "schedule": x["schedule"]}
            log(f"{args.shape} schedule {w}: {r[w]}")
        del os.environ["EXT_MPI_AMD_FOLD_SCHEDULE"]
        r = {"by_schedule": r}
    elif args.shape == "local256":
        r = comm_shape_fold(8, MB // 8 // 4, torch.float32, emac.FLOAT, 40, launch_times=True)
    elif args.shape == "small":
        r = small_sweep(emac, torch)
    elif args.shape == "joinci":
        r = join_copyin_alone(emac, torch)
    elif args.shape == "copy256":  # the node256 launch's bytes as a 1:1 copy (tools/ceiling.hip), same lease
        L = _ceiling_lib()
        n = 8 * MB  # 2 GiB read + 2 GiB written per launch, 3 buffer pairs rotated
        if DevBuf.CONTIG:
            a = DevBuf(3 * 2 * n)  # contents do not matter to a copy
        else:
            a = torch.empty(3 * 2 * n // 4, dtype=torch.float32, device="cuda")
            a.uniform_(-1, 1)
        stream = torch.cuda.current_stream()
        best = {}
        for variant in (0, 1, 2):  # nontemporal, default policy, phased (tools/ceiling.hip)
            for i in range(3):
                L.ceiling_copy(a.data_ptr() + i * 2 * n, a.data_ptr() + i * 2 * n + n, n, 1, variant, stream.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(20):
                b = a.data_ptr() + (i % 3) * 2 * n
                assert L.ceiling_copy(b, b + n, n, 1, variant, stream.cuda_stream) == 0
            e1.record(stream)
            torch.cuda.synchronize()
            best[("nt", "plain", "phased")[variant]] = round(e0.elapsed_time(e1) * 1e3 / 20, 2)
        r = {"avg_launch_us": best, "bytes_per_launch": 2 * n}
    else:  # the node form: float at 16 - 512 MiB per rank, or BASELINE configs[2]'s int / long launch
        if args.shape in ("int4", "long4"):  # (4 MiB per rank x 8)
            td, cd, ts, steps = (torch.int32, emac.INT, 4, 50) if args.shape == "int4" else (torch.int64, emac.LONG, 8, 50)
        else:
            td, cd, ts, steps = torch.float32, emac.FLOAT, 4, 40
        if args.schedules:  # every listed fold schedule in turn (EXT_MPI_AMD_FOLD_SCHEDULE), one handle set each
            r, pool = {}, {}
            for w in args.schedules.split(","):
                os.environ["EXT_MPI_AMD_FOLD_SCHEDULE"] = w
                x = node_run(8, MB // ts, td, cd, args.copyin or "6;1 -8 8", steps, 4, alloc="hip", pool=pool)
                r[w] = {"avg_launch_us": round(x["event_ms"] * 1e3 / steps, 2), "checked": x["checked"],
                        "schedule": x["schedule"]}
                log(f"{args.shape} schedule {w}: {r[w]}")
            del os.environ["EXT_MPI_AMD_FOLD_SCHEDULE"]
            free_pool(pool)
            r = {"by_schedule": r}
        else:
            pool = {}  # the isolated run reuses the buffer sets (filling 8 GiB from host takes minutes)
            x = node_run(8, MB // ts, td, cd, args.copyin or "6;1 -8 8", steps, 5, alloc="hip", launch_times=True,
                         pool=pool)
            r = {"avg_launch_us": round(x["event_ms"] * 1e3 / steps, 2), "checked": x["checked"], "schedule": x["schedule"],
                 **launch_stats(x["launch_us"])}
            log(f"{args.shape}: back to back {r}")
            if os.environ.get("EXT_MPI_AMD_BENCH_ISOLATED"):  # each launch alone (lease fingerprint)
                y = node_run(8, MB // ts, td, cd, args.copyin or "6;1 -8 8", 20, 5, alloc="hip", launch_times=True,
                             isolate=True, pool=pool)
                r["isolated"] = launch_stats(y["launch_us"])
            free_pool(pool)
            # EXT_MPI_AMD_BENCH_PLACEMENTS=k: k more runs, each on freshly allocated buffer sets (the
            # lease fingerprint: does the time move with the allocation inside one lease?)
            for i in range(int(os.environ.get("EXT_MPI_AMD_BENCH_PLACEMENTS", "0"))):
                z = node_run(8, MB // ts, td, cd, args.copyin or "6;1 -8 8", 20, 5, alloc="hip", launch_times=True)
                r.setdefault("placements", []).append(launch_stats(z["launch_us"]).get("median_launch_us"))
                log(f"{args.shape}: placement {i}: {r['placements'][-1]}")
    emit({"shape": args.shape, **r})


_RESULT_FD = None


def emit(obj):
    """The result line, on the real stdout: everything else -- library banners, gloo and RCCL
    chatter of this process and its children -- goes to stderr (see main)."""
    line = (json.dumps(obj) + "\n").encode()
    if _RESULT_FD is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_RESULT_FD, line)


def main():
    global _RESULT_FD
    args = parse()
    # keep stdout for the one result line: fd 1 (C-level writers included, and every child
    # process) goes to stderr, the line is written to a saved copy of the original stdout
    sys.stdout.flush()
    _RESULT_FD = os.dup(1)
    os.dup2(2, 1)
    if args.shape:
        shape_only(args)
    elif args.child_transport:
        transport_child(args)
    elif int(os.environ.get("WORLD_SIZE", "1")) > 1:
        multi_gpu(args)
    else:
        single_gpu(args)


if __name__ == "__main__":
    main()
