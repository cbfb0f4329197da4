#!/usr/bin/env python3
"""Per-grid kernel statistics from a rocprofv3 --kernel-trace CSV, split by overlap.

rocprofv3 --stats averages every launch of a kernel name together: 2^22 and 2^24 MSMs, and
launches that ran alone with launches that shared the chip with another stream's kernels
(a launch's duration then counts time the chip spent on the other kernel).  This groups
the launches of each kernel by grid size and by whether any other kernel ran during them,
so a bench line's per-launch figure can be recomputed from a committed file.

    python tools/trace_grid_stats.py kernel_trace.csv [name_filter ...] > stats.csv
Columns: kernel, grid, launches, overlap ("lone" / "overlapped"), total_ms, mean_ms,
median_ms, min_ms, max_ms.
"""
import csv
import statistics
import sys
from collections import defaultdict


def grid_of(r):
    for k in ("Grid_Size_X", "Grid_Size", "grid_size_x"):
        if k in r and r[k] != "":
            x = int(r[k])
            y = int(r.get("Grid_Size_Y", 1) or 1)
            return x if y == 1 else f"{x}x{y}"
    return "?"


def main():
    path, filters = sys.argv[1], sys.argv[2:]
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], grid_of(r)) for r in rows)
    # overlap: was any other launch in flight at some point of [s, e)?  sweep the
    # endpoints with the set of launches in flight (a few at most)
    lone = [True] * len(ev)
    pts = sorted([(s, 1, i) for i, (s, e, _, _) in enumerate(ev)] + [(e, 0, i) for i, (s, e, _, _) in enumerate(ev)])
    active = set()
    for _, start, i in pts:  # at equal times ends (0) come before starts (1)
        if start:
            if active:
                lone[i] = False
                for j in active:
                    lone[j] = False
            active.add(i)
        else:
            active.discard(i)
    groups = defaultdict(list)
    for (s, e, name, g), alone in zip(ev, lone):
        short = name.split("(")[0]
        if filters and not any(f in short for f in filters):
            continue
        groups[(short, g, "lone" if alone else "overlapped")].append((e - s) / 1e6)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid", "overlap", "launches", "total_ms", "mean_ms", "median_ms", "min_ms", "max_ms"])
    for (name, g, ov), d in sorted(groups.items(), key=lambda kv: (-sum(kv[1]), kv[0])):
        w.writerow([name, g, ov, len(d), round(sum(d), 4), round(sum(d) / len(d), 5),
                    round(statistics.median(d), 5), round(min(d), 5), round(max(d), 5)])


if __name__ == "__main__":
    main()
