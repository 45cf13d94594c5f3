"""Per-dispatch summary of a kernel trace (rocprofv3 --kernel-trace database, tools/gpu_r04_small.sh):
runs of consecutive dispatches of one kernel at one grid size, each with its dispatch count, median
and minimum duration, median gap to the next dispatch and median start-to-start interval, in the
trace's order; then, for the runs whose dispatches queue back to back (median gap < 0.5 us: the
kernel's duration is the whole per-launch cost), a straight line through duration against bytes
moved per launch for the fold and for each copy variant -- its intercept is the fixed cost of a
launch (dispatch, first-load latency, store drain), its slope the streaming rate.
Usage: small_trace_summary.py <run_results.db> <sweep.json>  -> JSON on stdout."""
import json
import re
import sqlite3
import statistics as st
import sys


NAME = re.compile(r"^(?:void )?(?:\(anonymous namespace\)::)?([\w:]+(?:<[^>]*>)?)")


def runs(db):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, grid_x / workgroup_x, start, end, duration from kernels order by start"))
    out = []
    for name, groups, s, e, d in rows:
        m = NAME.match(name)
        key = (m.group(1) if m else name[:60], groups)
        if out and out[-1][0] == key:
            out[-1][1].append((s, e, d))
        else:
            out.append([key, [(s, e, d)]])
    res = []
    for (name, groups), rs in out:
        if len(rs) < 20 or "rocclr" in name:
            continue
        last = rs[-50:]
        res.append({"kernel": name, "workgroups": groups, "dispatches": len(rs),
                    "dur_med_us": round(st.median(x[2] for x in last) / 1e3, 2),
                    "dur_min_us": round(min(x[2] for x in last) / 1e3, 2),
                    "gap_med_us": round(st.median((last[i + 1][0] - last[i][1]) for i in range(len(last) - 1)) / 1e3, 2),
                    "start_to_start_med_us": round(st.median((last[i + 1][0] - last[i][0]) for i in range(len(last) - 1)) / 1e3, 2)})
    return res


def fit(pts):
    n = len(pts)
    mx, my = sum(p[0] for p in pts) / n, sum(p[1] for p in pts) / n
    b = sum((x - mx) * (y - my) for x, y in pts) / sum((x - mx) ** 2 for x, _ in pts)
    return {"fixed_us": round(my - b * mx, 2), "streaming_gbps": round(1e-3 / b, 1), "points": n}


def main(db, sweep):
    rs = runs(db)
    # bytes per launch by fold grid size: the sweep's tuned schedules (last run of each size)
    pts = json.loads(open(sweep).read().strip().splitlines()[-1])["points"]
    groups = {}
    for r in rs:
        if r["gap_med_us"] >= 0.5:  # host-bound runs: the duration is not the per-launch cost
            continue
        k = r["kernel"]
        if k.startswith("emac::fold_kernel") or k.startswith("emac::fold_deferred_kernel"):
            # tiles of 256 lanes x U x 16 B (deferred groups: KB tiles each); 8 leaves read, 8 written
            a = k.split("<")[1].split(",")
            u, kb = int(a[3]), 1
            if "deferred" in k:
                kb = {0: 1, 1: 2, 2: 4, 3: 8}[(int(a[6]) >> 11) & 3]
            groups.setdefault("fold (tuned schedule)", {})[r["workgroups"] * kb * 256 * u * 16 * 16] = r
        elif k.startswith("copy_phased"):  # a group per 2048 vectors of 16 B, read and written
            groups.setdefault(k, {})[r["workgroups"] * 2048 * 16 * 2] = r
        elif k.startswith("copy_k4"):  # a fixed grid: its back-to-back runs come in size order
            g = groups.setdefault(k, {})
            g[len(g)] = r
    fits = {}
    sweep_bytes = [p["bytes_per_launch"] for p in pts]
    for k, by in groups.items():
        if k.startswith("copy_k4"):  # size order -> the sweep's largest sizes
            by = dict(zip(sweep_bytes[-len(by):], [by[i] for i in sorted(by)]))
        xy = sorted((b, r["dur_med_us"]) for b, r in by.items())
        fits[k] = {"by_bytes": [{"bytes": x, "dur_med_us": y} for x, y in xy], **(fit(xy) if len(xy) > 1 else {})}
    return {"runs": rs, "back_to_back_fits": fits}


if __name__ == "__main__":
    print(json.dumps(main(sys.argv[1], sys.argv[2]), indent=1))
