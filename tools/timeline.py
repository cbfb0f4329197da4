"""Per-kernel attribution over the last proof-sized window of a rocprofv3 kernel trace:
time with 0/1/2/3 kernels in flight, and for each kernel the time it ran alone plus
its share (1/k) of the time it overlapped k-1 others.
usage: timeline.py kernel_trace.csv [window_ms] [top] [anchor:index:before_ms]
anchor: the window is [t - before_ms, t - before_ms + window_ms] around the start of the
index-th kernel whose name contains `anchor` (e.g. evaluate_h:-2:56 for the last timed proof
when the bench's 2^24 MSMs follow it)"""
import csv
import sys
from collections import Counter, defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
win = float(sys.argv[2]) if len(sys.argv) > 2 else 110.0
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-44:]) for r in rows)
t0 = ev[-1][1] - int(win * 1e6)
t1 = ev[-1][1]
if len(sys.argv) > 4:
    name, idx, before = sys.argv[4].split(":")
    anchors = [s for s, e, n in ev if name in n]
    t0 = anchors[int(idx)] - int(float(before) * 1e6)
    t1 = t0 + int(win * 1e6)
ev = [(max(s, t0), min(e, t1), n) for s, e, n in ev if e > t0 and s < t1]
pts = sorted([(s, 1, n) for s, e, n in ev] + [(e, -1, n) for s, e, n in ev])
active, last = Counter(), pts[0][0]
conc, alone, shared, calls = defaultdict(int), defaultdict(int), defaultdict(float), Counter(n for _, _, n in ev)
for t, d, n in pts:
    dt, k = t - last, sum(active.values())
    conc[k] += dt
    if k == 1:
        alone[next(iter(active))] += dt
    elif k > 1:
        for nm, c in active.items():
            shared[nm] += dt * c / k
    active[n] += d
    if active[n] == 0:
        del active[n]
    last = t
tot = sum(conc.values())
print(f"window {tot / 1e6:.2f} ms; in flight:", {k: round(v / 1e6, 2) for k, v in sorted(conc.items())})
for n in sorted(set(alone) | set(shared), key=lambda n: -(alone[n] + shared[n]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{n:46s} calls {calls[n]:4d}  alone {alone[n] / 1e6:7.2f}  shared {shared[n] / 1e6:7.2f}  sum {(alone[n] + shared[n]) / 1e6:7.2f} ms")
