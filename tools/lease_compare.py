"""The 256 MiB point's lease fingerprints side by side (tools/gpu_r05_lease.sh): per lease, the node
launch's event time under its usual kept schedule and under leaf-major groups, the best 1:1 copy of
its 4 GiB, and, per kernel, the DRAM credit stall cycles and L2->memory cycles in flight per request
(the counters round 4 found bounding the fold), next to the busy time. Sorted by the node launch's
time, so the counters of slow and fast leases line up.
Usage: lease_compare.py <gpurun_out/r05/lease> [--json OUT]"""
import csv
import glob
import json
import os
import re
import sys

CLOCK_GHZ = 2.4  # GRBM_GUI_ACTIVE counts engine cycles on each of the 8 XCDs


def label(name):
    """a short kernel label: the fold's template arguments, or which copy ceiling kernel"""
    if "copy_phased" in name:
        return "copy phased"
    if "copy_k4<true>" in name:
        return "copy nt"
    if "copy_k4<false>" in name:
        return "copy plain"
    m = re.search(r"(fold_\w*kernel<[^>]*>)", name)
    return m.group(1) if m else None


def merged(d, prefix):
    """{kernel label: {counter: median}} over the lease's PMC pass directories <prefix>_*"""
    vals = {}
    for path in glob.glob(os.path.join(d, prefix + "_*", "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            k = label(row.get("Kernel_Name", ""))
            if k:
                vals.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    out = {k: {c: sorted(v)[len(v) // 2] for c, v in cs.items()} for k, cs in vals.items()}
    if not out:  # a lease whose large CSVs were dropped: the medians tools/pmc_counters.py kept
        try:
            for per_dir in json.load(open(os.path.join(d, "pmc_fold.json" if prefix == "node256" else "pmc_copy.json"))).values():
                for k, cs in per_dir.items():
                    if label(k):
                        out.setdefault(label(k), {}).update(cs)
        except (OSError, ValueError):
            pass
    return out


def per_request(cs):
    rd, wr = cs.get("TCC_EA0_RDREQ_sum"), cs.get("TCC_EA0_WRREQ_sum")
    f = {}
    if rd:
        if "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" in cs:
            f["rd_credit_stall_per_req"] = round(cs["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"] / rd, 3)
        if "TCC_EA0_RDREQ_LEVEL_sum" in cs:
            f["rd_level_per_req"] = round(cs["TCC_EA0_RDREQ_LEVEL_sum"] / rd, 1)
        f["rd_mib"] = round(rd * 128 / 2 ** 20, 1)
    if wr:
        if "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" in cs:
            f["wr_credit_stall_per_req"] = round(cs["TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"] / wr, 3)
        if "TCC_EA0_WRREQ_LEVEL_sum" in cs:
            f["wr_level_per_req"] = round(cs["TCC_EA0_WRREQ_LEVEL_sum"] / wr, 1)
        f["wr_mib"] = round(wr * 64 / 2 ** 20, 1)
    if "GRBM_GUI_ACTIVE" in cs:
        f["busy_us"] = round(cs["GRBM_GUI_ACTIVE"] / 8 / CLOCK_GHZ / 1e3, 1)
    return f


def lease(d):
    out = {"lease": os.path.basename(d)}
    try:
        out["host"] = open(os.path.join(d, "host.txt")).read().strip()
    except OSError:
        pass
    try:
        t = json.load(open(os.path.join(d, "time_node256.json")))
        out["node256_us"] = {w: v["avg_launch_us"] for w, v in t["by_schedule"].items()}
    except (OSError, ValueError, KeyError):
        return None
    try:
        t = json.load(open(os.path.join(d, "time_node256_iso.json")))
        out["node256_back_to_back_median_us"] = t.get("median_launch_us")
        out["node256_isolated_median_us"] = t.get("isolated", {}).get("median_launch_us")
        out["node256_placements_median_us"] = t.get("placements")
    except (OSError, ValueError):
        pass
    try:
        out["copy256_us"] = json.load(open(os.path.join(d, "time_copy256.json")))["avg_launch_us"]
    except (OSError, ValueError, KeyError):
        pass
    out["fold_pmc"] = {k: per_request(cs) for k, cs in merged(d, "node256").items()}
    out["copy_pmc"] = {k: per_request(cs) for k, cs in merged(d, "copy256").items()}
    return out


def main():
    root = sys.argv[1]
    rows = [r for r in (lease(d) for d in sorted(glob.glob(os.path.join(root, "*")))) if r]
    rows.sort(key=lambda r: min(r["node256_us"].values()))
    for r in rows:
        fold = next(iter(r["fold_pmc"].values()), {})
        copy = r["copy_pmc"].get("copy phased", {})
        print(f"{r['lease']:>12} node {r['node256_us']} b2b/isolated {r.get('node256_back_to_back_median_us')} / "
              f"{r.get('node256_isolated_median_us')} fresh allocations {r.get('node256_placements_median_us')} "
              f"copy {r.get('copy256_us')} | fold {fold} | phased copy {copy}")
    if "--json" in sys.argv:
        json.dump(rows, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
