"""The last proof of a rocprofv3 kernel trace (tools/prove_bench.py: three copy_columns
launches open each proof) as a sequence: start / end / duration (ms from the proof's
start), stream and queue of every kernel over 30 us and of every accumulation -- which
MSM phase waits for which, and where no accumulation is in flight.
usage: python tools/proof_sequence.py kernel_trace.csv"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ","").replace("h2g::","")[:40], r["Stream_Id"], r["Queue_Id"]) for r in rows)
starts = [s for s, e, n, st, q in ev if n.startswith("copy_columns")]
t0 = starts[-3]
last = [x for x in ev if x[0] >= t0]
# merge consecutive kernels by (stream) into segments of names for compactness
for s, e, n, st, q in last:
    if (e - s) < 30000 and not n.startswith("msm_acc") : continue
    print(f"{(s - t0)/1e6:8.3f} {(e - t0)/1e6:8.3f} {(e-s)/1e6:7.3f} st{st} q{q} {n}")
