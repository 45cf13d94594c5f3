"""Summarise EXT_MPI_AMD_JOIN_TRACE files (join_fused.hip kTraceSlots records): per launch, for every
recorded event (start, each segment left or gate passed, end), the spread over workgroups of its time
after the launch's first workgroup started, in microseconds, and the items the workgroups took.

Usage: join_trace_summary.py <trace file> [launch indices to show, default: the last 3 of each mode]"""
import collections
import statistics
import sys

STAGE = {0: "CI", 1: "SF-gate", 2: "SF", 3: "PL-gate", 4: "PL", 14: "start", 15: "end"}


def launches(path):
    cur = None
    for line in open(path):
        p = line.split()
        if not p:
            continue
        if p[0] == "launch":
            if cur:
                yield cur
            cur = {"n": int(p[1]), "mode": int(p[3]), "grid": int(p[5]), "wg": []}
        elif cur is not None:
            cur["wg"].append([int(x) for x in p[1:]])
    if cur:
        yield cur


def summary(L):
    t0 = min(r[0] >> 16 for r in L["wg"] if r)
    ev = collections.OrderedDict()
    for r in L["wg"]:
        for v in r:
            tag, items, t = v & 0xFF, (v >> 8) & 0xFF, ((v >> 16) - t0) / 100.0  # 100 MHz -> us
            name = STAGE.get(tag >> 4, "?") + ("" if tag >> 4 >= 14 else f"[{tag & 15}]")
            ev.setdefault(name, []).append((t, items))
    out = [f"launch {L['n']} mode {L['mode']} grid {L['grid']} workgroups {len(L['wg'])}"]
    for name, v in ev.items():
        ts = sorted(t for t, _ in v)
        its = [i for _, i in v]
        out.append(f"  {name:10s} min {ts[0]:8.2f}  median {statistics.median(ts):8.2f}  max {ts[-1]:8.2f} us"
                   f"   items: total {sum(its)}, per workgroup {min(its)}-{max(its)}")
    return "\n".join(out)


def main():
    ls = list(launches(sys.argv[1]))
    if len(sys.argv) > 2:
        pick = [int(x) for x in sys.argv[2:]]
        show = [L for L in ls if L["n"] in pick]
    else:
        by = collections.defaultdict(list)
        for L in ls:
            by[L["mode"]].append(L)
        show = [L for m in sorted(by) for L in by[m][-3:]]
    for L in show:
        print(summary(L))


if __name__ == "__main__":
    main()
