"""Summary of the round-4 PMC campaign (tools/gpu_r04_pmc.sh): per shape (node fold at 16 / 64 /
256 / 512 MiB per rank, the 1:1 copies of the 256 MiB launch's 4 GiB) and kernel instance, the
memory-side request counts, DRAM credit stalls per request, in-flight levels (Little's law: cycles a
request spends between the L2 and the memory), UTCL1 translation miss rate and UTCL2 busy share,
next to the event-timed launch time of the same lease.
Usage: pmc_r04_summary.py <gpurun_out/pmc4>  -> JSON on stdout."""
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_counters import medians  # noqa: E402

CLOCK_GHZ = 2.4  # MI355X engine clock: GRBM_GUI_ACTIVE counts cycles on each of the 8 XCDs


def schedule_of(kname):
    """'fold_kernel<float, 0, 8, 4, 0, 8, 1>' -> 'U4 issue 1'; deferred kernels carry their tile count"""
    m = re.search(r"<([^>]*)>", kname)
    if not m:
        return kname
    a = [x.strip() for x in m.group(1).split(",")]
    if kname.startswith("fold") and len(a) >= 7:
        return f"U{a[3]} issue {a[6]}" + (" whole" if len(a) > 7 and a[7] == "true" else "")
    return kname


def summarize(d):
    out = {}
    for shape_dir in sorted(glob.glob(os.path.join(d, "*_ea"))):
        shape = os.path.basename(shape_dir)[:-3]
        kernel = r"copy_k4|copy_phased" if shape.startswith("copy") else r"\bfold_(deferred_)?kernel<"
        per = {}
        for group in ("ea", "stall", "level", "tlb", "utcl2", "tlbcontig"):
            path = os.path.join(d, f"{shape}_{group}")
            if not os.path.isdir(path):
                continue
            for kname, c in medians(path, kernel, by_kernel=True).items():
                k = per.setdefault(kname, {})
                for name, v in c.items():
                    if name == "dispatches":
                        continue
                    key = f"{name}@contig" if group == "tlbcontig" else name
                    k.setdefault(key, v)
        rows = {}
        for kname, c in per.items():
            rd, wr = c.get("TCC_EA0_RDREQ_sum"), c.get("TCC_EA0_WRREQ_sum")
            row = {"schedule": schedule_of(kname)}
            if c.get("GRBM_GUI_ACTIVE"):
                row["busy_us"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (CLOCK_GHZ * 1e3), 1)
            if rd:
                row["read_MiB"] = round(rd * 128 / 2 ** 20, 1)
            if wr:
                row["write_MiB"] = round(wr * 64 / 2 ** 20, 1)
                if c.get("TCC_EA0_WRREQ_64B_sum") is not None:
                    row["write_64B_share"] = round(c["TCC_EA0_WRREQ_64B_sum"] / wr, 3)
            if rd and "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" in c:
                row["rd_credit_stall_per_req"] = round(c["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"] / rd, 3)
            if wr and "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" in c:
                row["wr_credit_stall_per_req"] = round(c["TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"] / wr, 3)
            if rd and "TCC_EA0_RDREQ_LEVEL_sum" in c:
                row["rd_cycles_in_flight_per_req"] = round(c["TCC_EA0_RDREQ_LEVEL_sum"] / rd, 1)
            if wr and "TCC_EA0_WRREQ_LEVEL_sum" in c:
                row["wr_cycles_in_flight_per_req"] = round(c["TCC_EA0_WRREQ_LEVEL_sum"] / wr, 1)
            for sfx in ("", "@contig"):
                h, m = c.get("TCP_UTCL1_TRANSLATION_HIT_sum" + sfx), c.get("TCP_UTCL1_TRANSLATION_MISS_sum" + sfx)
                if h is not None and m is not None and h + m > 0:
                    row["utcl1_miss_rate" + sfx] = round(m / (h + m), 5)
                oc = c.get("TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum" + sfx)
                if oc is not None:
                    row["utcl1_stall_utcl2_out_of_credits" + sfx] = oc
            if "GRBM_UTCL2_BUSY" in c and c.get("GRBM_GUI_ACTIVE"):
                row["utcl2_busy_share"] = round(c["GRBM_UTCL2_BUSY"] / c["GRBM_GUI_ACTIVE"], 3)
            rows[kname] = row
        out[shape] = rows
    times = {}
    for f in sorted(glob.glob(os.path.join(d, "time_*.json"))):
        try:
            times[os.path.basename(f)[5:-5]] = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            pass
    return {"pmc": out, "event_timing": times}


if __name__ == "__main__":
    print(json.dumps(summarize(sys.argv[1]), indent=1))
