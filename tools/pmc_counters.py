"""Median per-dispatch value of every counter rocprofv3 --pmc wrote for the profiled kernel.
Usage: pmc_counters.py [--kernel=REGEX] <dir> [<dir> ...] -> one JSON object {dir: {counter: median}}
(default: fold_kernel or fold_deferred_kernel; the copy ceiling is copy_k4)"""
import csv
import glob
import json
import re
import sys


def medians(d, kernel):
    vals = {}
    for path in glob.glob(f"{d}/**/*counter_collection*.csv", recursive=True):
        for row in csv.DictReader(open(path)):
            if re.search(kernel, row.get("Kernel_Name", "")):
                vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: sorted(v)[len(v) // 2] for k, v in vals.items()}


if __name__ == "__main__":
    kernel = r"\bfold_(deferred_)?kernel<"
    dirs = []
    for a in sys.argv[1:]:
        if a.startswith("--kernel="):
            kernel = a.split("=", 1)[1]
        else:
            dirs.append(a)
    print(json.dumps({d: medians(d, kernel) for d in dirs}, indent=1))
