"""Median per-dispatch value of every counter rocprofv3 --pmc wrote for fold_kernel launches.
Usage: pmc_counters.py <dir> [<dir> ...] -> one JSON object {dir: {counter: median}}"""
import csv
import glob
import json
import sys


def medians(d):
    vals = {}
    for path in glob.glob(f"{d}/**/*counter_collection*.csv", recursive=True):
        for row in csv.DictReader(open(path)):
            if "fold_kernel" in row.get("Kernel_Name", ""):
                vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: sorted(v)[len(v) // 2] for k, v in vals.items()}


if __name__ == "__main__":
    print(json.dumps({d: medians(d) for d in sys.argv[1:]}, indent=1))
