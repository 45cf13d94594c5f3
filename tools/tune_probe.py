"""The per-handle schedule tuner at large node-form sizes (8 ranks x S float, one buffer set):
every candidate's shortest sample (EXT_MPI_AMD_DEBUG_TUNE=1 on stderr), then 5 timed Starts of the
kept schedule. Usage: tune_probe.py [MiB per rank ...]"""
import os
import sys
import time

os.environ.setdefault("EXT_MPI_AMD_DEBUG_TUNE", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import ext_mpi_collectives_amd as emac  # noqa: E402


def main():
    R = 8
    for mib in [int(a) for a in sys.argv[1:]] or [256, 512]:
        count = (mib << 20) // 4
        sends = [torch.rand(count, device="cuda") for _ in range(R)]
        recvs = [torch.empty(count, device="cuda") for _ in range(R)]
        h = emac.node_allreduce_init([t.data_ptr() for t in sends], [t.data_ptr() for t in recvs], count, emac.FLOAT)
        for _ in range(21):
            emac.start(h)
        emac.wait(h)
        t0 = time.perf_counter()
        for _ in range(5):
            emac.start(h)
        emac.wait(h)
        el = (time.perf_counter() - t0) / 5
        print(f"{mib} MiB per rank: kept {emac.handle_schedule(h)}, {el * 1e6:.1f} us per Start, "
              f"{2 * R * count * 4 / el / 1e12:.3f} TB/s", flush=True)
        emac.done(h)
        del sends, recvs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
