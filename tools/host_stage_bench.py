"""Host-buffer rates of the NODE form (8 ranks x 16 MiB float, pinned host send / receive buffers):
read and written by the fold kernel over PCIe (default), or staged through device mirrors
(EXT_MPI_AMD_HOST_DIRECT=0: H2D copies, the fold, D2H copies on one stream). Prints one JSON line.
(Round 3 also tried copying the staged receive side out with a kernel instead of the D2H DMA: 4.99
against 4.94 ms -- the 16 MiB D2H copies already ran at ~53 GB/s -- and dropped it.)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import ext_mpi_collectives_amd as emac  # noqa: E402


def run(env, R=8, mib=16, steps=10):
    os.environ.pop("EXT_MPI_AMD_HOST_DIRECT", None)
    os.environ.update(env)
    count = (mib << 20) // 4
    sends = [torch.rand(count).pin_memory() for _ in range(R)]
    recvs = [torch.empty(count).pin_memory() for _ in range(R)]
    h = emac.node_allreduce_init([t.data_ptr() for t in sends], [t.data_ptr() for t in recvs], count, emac.FLOAT)
    for _ in range(3):
        emac.start(h)
        emac.wait(h)
    want = torch.stack(sends).double().sum(0)
    ok = bool(torch.allclose(recvs[R - 1].double(), want, atol=1e-4 * R))
    t0 = time.perf_counter()
    for _ in range(steps):
        emac.start(h)
        emac.wait(h)
    el = time.perf_counter() - t0
    emac.done(h)
    return {"ms_per_allreduce": round(el * 1e3 / steps, 3), "gbps_reduced": round(R * count * 4 * steps / el / 1e9, 2),
            "checked": ok}


def main():
    out = {"direct": run({}), "staged": run({"EXT_MPI_AMD_HOST_DIRECT": "0"})}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
