"""Start -> Wait latency of the COMM form on a 1-rank RCCL communicator (the fold leg only: the
transport legs are empty at one rank), eager launches vs the captured HIP graph
(EXT_MPI_AMD_GRAPH). Prints one JSON line. N > 1 latency needs several GPUs (unmeasured here)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import ext_mpi_collectives_amd as emac  # noqa: E402


def timed(h, n):
    for _ in range(20):
        emac.start(h)
        emac.wait(h)
    t0 = time.perf_counter()
    for _ in range(n):
        emac.start(h)
        emac.wait(h)
    return (time.perf_counter() - t0) / n * 1e6


def main():
    torch.cuda.set_device(0)
    comm = emac.comm_init(0, 1, emac.get_unique_id(), 0)
    out = {"what": "1-rank RCCL communicator, Start+Wait per Allreduce (us), host wall", "points": []}
    for nbytes in (8, 65536, 1 << 20):
        x = torch.ones(max(1, nbytes // 4), device="cuda")
        y = torch.empty_like(x)
        pt = {"bytes": nbytes}
        for g in ("0", "1"):
            os.environ["EXT_MPI_AMD_GRAPH"] = g
            h = emac.allreduce_init(x.data_ptr(), y.data_ptr(), x.numel(), emac.FLOAT, comm)
            pt["graph_us" if g == "1" else "eager_us"] = round(timed(h, 2000), 2)
            emac.done(h)
        out["points"].append(pt)
    emac.comm_free(comm)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
