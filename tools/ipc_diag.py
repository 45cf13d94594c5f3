"""Diagnosis of the peer-mapped form: one rank per process (RANK / WORLD_SIZE / MASTER_* from the
environment, ranks may share one GPU). For several message sizes, fill the receive buffer with
-1 before every Start (as an application reusing it would), run the Allreduce and report, per
iteration, how many elements differ from the exact sum and where the first ones are."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ext_mpi_collectives_amd as emac  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    pre = None
    if os.environ.get("DIAG_PRE_COMM"):  # a first communicator, used and kept alive
        pre = emac.comm_init_ipc(rank, world, emac.torch_allgather(), 0)
        a = torch.full((4099,), 1.0, device="cuda")
        b = torch.empty_like(a)
        hp = emac.allreduce_init(a.data_ptr(), b.data_ptr(), a.numel(), emac.FLOAT, pre)
        for _ in range(3):
            emac.start(hp)
            emac.wait(hp)
        emac.done(hp)
    if os.environ.get("DIAG_TIMEOUT"):
        os.environ["EXT_MPI_AMD_BARRIER_TIMEOUT"] = os.environ["DIAG_TIMEOUT"]
    comm = emac.comm_init_ipc(rank, world, emac.torch_allgather(), 0)
    late = int(os.environ.get("DIAG_LATE", "-1"))
    out = []
    want = world * (world + 1) / 2
    sizes = [int(v) for v in os.environ.get("DIAG_SIZES", "1000,4096,40961,262144").split(",")]
    reads = os.environ.get("DIAG_READ", "torch")
    for n in sizes:
        x = torch.full((n,), float(rank + 1), device="cuda")
        y = torch.empty_like(x)
        h = emac.allreduce_init(x.data_ptr(), y.data_ptr(), n, emac.FLOAT, comm)
        rec = {"n": n, "iters": []}
        for it in range(int(os.environ.get("DIAG_ITERS", "4"))):
            dist.barrier()
            y.fill_(-1.0)
            torch.cuda.synchronize()
            if it == late and rank == 1:
                import time
                time.sleep(1.0)
            err = None
            try:
                emac.start(h)
                emac.wait(h)
            except emac.ExtMpiError as e:
                err = e.code
            if reads == "torch":
                bad = (y != want).nonzero().flatten()
                vals = y[bad[:6]].tolist() if bad.numel() else []
                nbad = int(bad.numel())
                first = bad[:6].tolist()
            else:
                yh = y.cpu()
                bad = (yh != want).nonzero().flatten()
                vals = yh[bad[:6]].tolist() if bad.numel() else []
                nbad = int(bad.numel())
                first = bad[:6].tolist()
            rec["iters"].append({"err": err, "nbad": nbad, "first": first, "vals": vals})
        emac.done(h)
        out.append(rec)
    emac.comm_free(comm)
    if pre is not None:
        emac.comm_free(pre)
    print(json.dumps({"rank": rank, "world": world, "read": reads, "res": out}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
