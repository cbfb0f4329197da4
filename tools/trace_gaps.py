"""Timeline analysis of a rocprofv3 kernel trace: GPU busy time (union of kernel
intervals) vs wall time over the last proof-sized window, the largest idle gaps and
the per-kernel time inside that window.  usage: trace_gaps.py kernel_trace.csv [window_ms]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
win_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
t_end = max(e for _, e, _ in ev)
t0 = t_end - int(win_ms * 1e6)
ev = [x for x in ev if x[0] >= t0]
busy, cur_s, cur_e = 0, None, None
gaps = []
for s, e, name in ev:
    if cur_e is None:
        cur_s, cur_e = s, e
        continue
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, name))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = ev[-1][1] - ev[0][0]
print(f"window {span / 1e6:.2f} ms: GPU busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f}%), idle {(span - busy) / 1e6:.2f} ms")
gaps.sort(reverse=True)
print("largest idle gaps (ms, next kernel):")
for g, name in gaps[:12]:
    print(f"  {g / 1e6:7.3f}  {name[:90]}")
per = defaultdict(float)
cnt = defaultdict(int)
for s, e, name in ev:
    short = name.split("(")[0][:80]
    per[short] += (e - s) / 1e6
    cnt[short] += 1
print("kernel time in window (ms, calls):")
for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:20]:
    print(f"  {v:8.3f}  {cnt[k]:4d}  {k}")
