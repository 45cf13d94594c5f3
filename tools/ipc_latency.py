"""Latency breakdown of the peer-mapped (IPC) form: full Allreduce, barriers only, fold only.

Run one process per rank (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment);
ranks may share one GPU (rehearsal) or sit on separate GPUs. Prints one JSON line from rank 0."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ext_mpi_collectives_amd as emac  # noqa: E402


def timed(h, legs, n, stream):
    for _ in range(10):
        emac.start_legs(h, legs)
    stream.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(n):
        emac.start_legs(h, legs)
    stream.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return el.item() / n * 1e6


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    if os.environ.get("IPC_LAT_EARLY_POOL"):  # diagnosis: torch's stream pool created before the communicator
        torch.cuda.Stream()
    comm = emac.comm_init_ipc(rank, world, emac.torch_allgather(), dev)
    out = {"world": world, "gpus": torch.cuda.device_count(), "points": []}
    sizes = [int(v) for v in os.environ.get("IPC_LAT_SIZES", "8,65536,1048576").split(",")]
    for nbytes in sizes:
        n = max(1, nbytes // 4)
        x = torch.ones(n, device="cuda")
        y = torch.empty_like(x)
        h = emac.allreduce_init(x.data_ptr(), y.data_ptr(), n, emac.FLOAT, comm)
        if os.environ.get("IPC_LAT_OWN_STREAM"):  # diagnosis: the handle's own HIP stream
            s = torch.cuda.ExternalStream(emac.lib().ext_mpi_amd_stream(h))
        else:
            for _ in range(int(os.environ.get("IPC_LAT_SKIP_STREAMS", "0"))):  # diagnosis: pool position
                torch.cuda.Stream()
            s = torch.cuda.Stream()
            if os.environ.get("IPC_LAT_WARM"):  # diagnosis: the stream used once before the handle gets it
                with torch.cuda.stream(s):
                    torch.zeros(1, device="cuda").add_(1)
                s.synchronize()
            emac.set_stream(h, s.cuda_stream)
        full = timed(h, emac.LEG_ALL, 200, s)
        if os.environ.get("IPC_LAT_TWICE"):  # diagnosis: the same handle and stream timed again
            out.setdefault("first_timing_us", []).append(round(full, 2))
            full = timed(h, emac.LEG_ALL, 2000, s)
        bars = timed(h, emac.LEG_REDUCE_SCATTER | emac.LEG_ALLGATHER, 200, s)
        fold = timed(h, emac.LEG_FOLD, 200, s)
        emac.wait(h)
        emac.done(h)
        out["points"].append({"bytes": nbytes, "full_us": round(full, 2), "two_barriers_us": round(bars, 2),
                              "fold_us": round(fold, 2)})
    emac.comm_free(comm)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
