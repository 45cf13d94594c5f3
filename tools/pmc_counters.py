"""Median per-dispatch value of every counter rocprofv3 --pmc wrote for the profiled kernel.
Usage: pmc_counters.py [--kernel=REGEX] <dir> [<dir> ...] -> one JSON object {dir: {counter: median}}
(default: fold_kernel or fold_deferred_kernel; the copy ceiling is copy_k4)"""
import csv
import glob
import json
import re
import sys


def medians(d, kernel, by_kernel=False):
    vals = {}
    for path in glob.glob(f"{d}/**/*counter_collection*.csv", recursive=True):
        for row in csv.DictReader(open(path)):
            name = row.get("Kernel_Name", "")
            if re.search(kernel, name):
                key = (re.sub(r"\(.*", "", name), row["Counter_Name"]) if by_kernel else row["Counter_Name"]
                vals.setdefault(key, []).append(float(row["Counter_Value"]))
    if not by_kernel:
        return {k: sorted(v)[len(v) // 2] for k, v in vals.items()}
    out = {}
    for (kname, c), v in vals.items():  # per kernel instance (template arguments = the schedule)
        out.setdefault(kname, {})[c] = sorted(v)[len(v) // 2]
        out[kname]["dispatches"] = len(v)
    return out


if __name__ == "__main__":
    kernel = r"\bfold_(deferred_)?kernel<"
    dirs, by_kernel = [], False
    for a in sys.argv[1:]:
        if a.startswith("--kernel="):
            kernel = a.split("=", 1)[1]
        elif a == "--by-kernel":
            by_kernel = True
        else:
            dirs.append(a)
    print(json.dumps({d: medians(d, kernel, by_kernel) for d in dirs}, indent=1))
