"""Probe (GPU box): bench.py's RCCL Allreduce baseline helper in one rank (torchrun, 1 process)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
print(json.dumps(bench._rccl_allreduce_baseline(rank, world, dist, torch)), flush=True)
dist.destroy_process_group()
