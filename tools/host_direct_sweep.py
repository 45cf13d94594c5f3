"""Pinned-host NODE form across message sizes: the fold kernel over PCIe (default) vs staged
through device mirrors (EXT_MPI_AMD_HOST_DIRECT=0). One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import ext_mpi_collectives_amd as emac  # noqa: E402

R = int(os.environ.get("HDS_RANKS", "8"))
out = {"ranks": R, "points": []}
for nbytes in (8, 4096, 65536, 1 << 20, 4 << 20, 16 << 20, 64 << 20):
    cnt = max(1, nbytes // 4)
    st = 200 if nbytes <= (1 << 20) else 10
    pt = {"bytes_per_rank": cnt * 4}
    for mode in ("1", "0"):
        os.environ["EXT_MPI_AMD_HOST_DIRECT"] = mode
        r = bench.node_run(R, cnt, torch.float32, emac.FLOAT, f"6;1 -{R} {R}", st, 5, host=True)
        key = "direct" if mode == "1" else "staged"
        pt[key + "_us"] = round(r["wall_s"] * 1e6 / st, 2)
        pt[key + "_gbps_reduced"] = round(R * cnt * 4 * st / r["wall_s"] / 1e9, 2)
        pt[key + "_checked"] = r["checked"]
    out["points"].append(pt)
    print(json.dumps(pt), file=sys.stderr, flush=True)
print(json.dumps(out), flush=True)
