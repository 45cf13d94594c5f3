"""Per-dispatch durations of one kernel family from a rocprofv3 --kernel-trace CSV, grouped by
(kernel name, grid size): which launch shape took how long, and the gaps between consecutive
dispatches of the same group (launch-boundary cost). Usage:
  prof_dispatches.py run_kernel_trace.csv [name regex = fold_(deferred_)?kernel<] [min calls = 5]"""
import csv
import re
import statistics
import sys


def main():
    path = sys.argv[1]
    sub = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"\bfold_(deferred_)?kernel<")
    minc = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rows = [r for r in csv.DictReader(open(path)) if sub.search(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    groups = {}
    for r in rows:
        key = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
        groups.setdefault(key, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    print(f"{'kernel':70s} {'WGs':>6s} {'calls':>6s} {'median_us':>10s} {'mean_us':>9s} {'gap_median_us':>13s}")
    for (name, wgs), ds in sorted(groups.items(), key=lambda kv: -len(kv[1])):
        if len(ds) < minc:
            continue
        dur = [(e - s) / 1e3 for s, e in ds]
        gaps = [(ds[i + 1][0] - ds[i][1]) / 1e3 for i in range(len(ds) - 1) if ds[i + 1][0] - ds[i][1] < 20000]
        gap = statistics.median(gaps) if gaps else float("nan")
        print(f"{name[-70:]:70s} {wgs:6d} {len(ds):6d} {statistics.median(dur):10.2f} {statistics.mean(dur):9.2f} {gap:13.2f}")


if __name__ == "__main__":
    main()
