#!/usr/bin/env python3
"""HBM traffic of the MSM bucket partition kernels from PMC counters, against their
algorithmic bytes.

Two rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE: they cannot share a pass) over
tools/ab_env.py's child running lone fixed-base MSMs of 2^log_n resident SRS points
with random scalars.  Per kernel: mean counters per launch, the calibrated traffic
(profiles/r03/pmc_calibration.json: FETCH_SIZE counts 0.5 of a coalesced stream's bytes
and 1.0 of 64-B gathers, WRITE_SIZE 1.0 of written bytes; every partition read is a
coalesced stream, so traffic = 2 FETCH + WRITE) and its ratio to the algorithmic bytes.

    python tools/pmc_partition.py --log-n 22 --out profiles/r04/pmc_partition_2p22.json
"""
import argparse
import csv
import json
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("msm_coarse_hist_kernel", "msm_coarse_scatter_kernel", "msm_fine_hist_kernel",
           "msm_fine_scatter_kernel", "msm_fine_hist_staged_kernel", "msm_fine_scatter_staged_kernel",
           "msm_acc_kernel")


def windows_for(c):
    return (255 + c - 1) // c


def choose_c_fixed(n):  # msm.hip msm_choose_c_fixed
    best_c, best = 2, 1e300
    for c in range(2, 23):
        cost = windows_for(c) * n + 3.0 * (1 << (c - 1))
        if cost < best * 0.98:
            best, best_c = cost, c
    return best_c


def algorithmic(name, n, total):
    """bytes each kernel must move: scalars 32 B, u64 entries (key << 32 | value), u32
    values; the fine histogram needs only the keys but they sit interleaved with the
    values, so its lines carry the whole entries"""
    if name == "msm_coarse_hist_kernel":
        return {"read": 32 * n, "write": 0}
    if name == "msm_coarse_scatter_kernel":
        return {"read": 32 * n, "write": 8 * total}
    if name.startswith("msm_fine_hist"):
        return {"read": 8 * total, "write": 0, "note": "keys only would be 4 B per entry"}
    if name.startswith("msm_fine_scatter"):
        return {"read": 8 * total, "write": 4 * total}
    if name == "msm_acc_kernel":
        return {"read": 4 * total + 64 * total, "write": 0, "note": "values + one 64-B table point per entry"}
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=22)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    n = 1 << args.log_n
    c = choose_c_fixed(n)
    W = windows_for(c)
    total = n * W  # nonzero signed digits of random scalars: all but ~n W / 2^c
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix=f"h2g_pmcpart_{ctr}_", dir="/tmp")
        cmd = ["timeout", "-s", "KILL", "120", prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "pmc",
               "--", sys.executable, os.path.join(REPO, "tools", "ab_env.py"), "--child", "--msm", str(args.log_n)]
        subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL,
                       stderr=subprocess.DEVNULL, check=True)
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    for r in csv.DictReader(open(os.path.join(root, f))):
                        nm = r["Kernel_Name"].split("(")[0].split("::")[-1]
                        if nm in KERNELS and r["Counter_Name"] == ctr:
                            vals.setdefault(nm, {}).setdefault(ctr, []).append(float(r["Counter_Value"]) * 1024.0)
        shutil.rmtree(d, ignore_errors=True)
    out = {"log_n": args.log_n, "c": c, "windows": W, "entries_per_msm": total,
           "calibration": "profiles/r03/pmc_calibration.json: FETCH_SIZE = 0.5 x coalesced-stream bytes, 1.0 x 64-B "
                          "gathers; WRITE_SIZE = 1.0 x written bytes",
           "kernels": {}}
    for nm, cs in vals.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
        write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
        alg = algorithmic(nm, n, total)
        # the accumulation's table points are gathers (x1), its values a stream (x2)
        if nm == "msm_acc_kernel":
            traffic = fetch + 0.5 * 4 * total + write
        else:
            traffic = 2 * fetch + write
        e = {"launches": len(cs["FETCH_SIZE"]), "fetch_size_bytes": round(fetch), "write_size_bytes": round(write),
             "traffic_calibrated_bytes": round(traffic)}
        if alg:
            a = alg["read"] + alg["write"]
            e["algorithmic_bytes"] = a
            e["algorithmic"] = alg
            e["counted_over_algorithmic"] = round(traffic / a, 3)
            e["read_counted_over_algorithmic"] = round((traffic - write) / alg["read"], 3) if alg["read"] else None
            e["write_counted_over_algorithmic"] = round(write / alg["write"], 3) if alg["write"] else None
        out["kernels"][nm] = e
    s = json.dumps(out, indent=1)
    print(s)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
