"""Probe (GPU box): can the COMM form run with 2 ranks sharing one GPU? Launched by torchrun.
Prints PROBE lines; any failure is reported, not retried."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ext_mpi_collectives_amd as emac  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
uid = [emac.get_unique_id() if rank == 0 else None]
dist.broadcast_object_list(uid, src=0)
try:
    comm = emac.comm_init(rank, world, uid[0], 0)
    n = 100003
    x = torch.full((n,), float(rank + 1), device="cuda")
    y = torch.empty_like(x)
    h = emac.allreduce_init(x.data_ptr(), y.data_ptr(), n, emac.FLOAT, comm)
    emac.start(h)
    emac.wait(h)
    ok = bool(torch.all(y == world * (world + 1) / 2).item())
    emac.done(h)
    emac.comm_free(comm)
    print(f"PROBE rank {rank}: comm form with {world} ranks on one GPU -> {'ok' if ok else 'WRONG'}", flush=True)
except Exception as e:  # noqa: BLE001
    print(f"PROBE rank {rank}: failed: {e}", flush=True)
dist.destroy_process_group()
