"""PCIe-inclusive NODE-form rate with host buffers (the path's real start and end): R ranks x S
bytes of pinned (or pageable) host send/recv buffers, H2D + fold + D2H per Start. Prints one
JSON line. EXT_MPI_AMD_PIPELINE=1 / EXT_MPI_AMD_PIPE_PARTS select the staging schedule."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import ext_mpi_collectives_amd as emac  # noqa: E402


def main():
    R, mib, steps = 8, int(os.environ.get("HOST_MIB", "16")), 10
    pinned = os.environ.get("HOST_PAGEABLE") is None
    count = (mib << 20) // 4
    mk = (lambda: torch.empty(count, dtype=torch.float32).pin_memory()) if pinned else \
        (lambda: torch.empty(count, dtype=torch.float32))
    keep = []
    for _ in range(int(os.environ.get("HOST_PRE_STREAMS", "0"))):  # diagnosis: shift the HW-queue mapping
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            keep.append(torch.zeros(1, device="cuda") + 1)
        st.synchronize()
        keep.append(st)
    sends = [mk() for _ in range(R)]
    recvs = [mk() for _ in range(R)]
    for r, t in enumerate(sends):
        t.fill_(float(r + 1))
    h = emac.node_allreduce_init([t.data_ptr() for t in sends], [t.data_ptr() for t in recvs], count, emac.FLOAT)
    if os.environ.get("HOST_TORCH_STREAM"):  # the caller's stream, as bench.py's node_run sets it
        s = torch.cuda.Stream()
        emac.set_stream(h, s.cuda_stream)
    for _ in range(2):
        emac.start(h)
    emac.wait(h)
    t0 = time.perf_counter()
    for _ in range(steps):
        emac.start(h)
    emac.wait(h)
    dt = (time.perf_counter() - t0) / steps
    ok = all(bool(torch.all(r == R * (R + 1) / 2)) for r in recvs)
    emac.done(h)
    print(json.dumps({"ranks": R, "mib_per_rank": mib, "pinned": pinned, "ms_per_allreduce": round(dt * 1e3, 3),
                      "gbps_reduced": round(R * (mib << 20) / dt / 1e9, 2), "checked": ok,
                      "pipeline": os.environ.get("EXT_MPI_AMD_PIPELINE", "0") != "0",
                      "parts": os.environ.get("EXT_MPI_AMD_PIPE_PARTS", "8")}), flush=True)


if __name__ == "__main__":
    main()
