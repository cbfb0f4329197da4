#!/usr/bin/env python3
"""Benchmark: BN254 G1 MSM throughput (Mscalar-mul/s) at 2^24 points per GPU.

BASELINE.json metric: "create_proof wall-seconds at k=22 (BN254/KZG); MSM
Mscalar-mul/s at 2^24".  This round the bench line reports the MSM half of it:
one step = one MSM of 2^24 (scalar, SRS point) pairs resident in HBM, through
the C ABI (h2g_msm_dev) on torch's current stream.

N > 1 (torchrun, one process per GPU): the MSM is sharded by point slabs
(weak scaling: every rank owns its own 2^24-point slab of a 2^24*N MSM); the
per-rank partial sums (64 B affine points) are exchanged with an RCCL
all_gather and summed on the host -- the one real exchange step of a sharded
MSM.

Also printed in the same JSON line:
  roofline     : dominant kernel (bucket accumulation) from live HIP events;
                 algorithmic bytes = 96 B/point
  cpu_baseline : the CPU restatement oracle (halo2curves best_multiexp
                 algorithm, oracle/) timed on a bounded sample on this host
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "yet-another-halo2-fork_amd"))

HBM_PEAK_GBS = 8000.0
MSM_BYTES_PER_POINT = 96  # 32 B scalar + 64 B affine base
MADD_MODMUL = 10          # XYZZ mixed add: 8M + 2S


def random_scalars(rng, n):
    """Uniform values < 2^253 < r: valid Montgomery-form Fr elements."""
    c = rng.integers(0, 2**63, size=(n, 4), dtype=np.int64).astype(np.uint64)
    c[:, 0] = c[:, 0] * np.uint64(2) + (rng.integers(0, 2, size=n, dtype=np.int64).astype(np.uint64))
    c[:, 3] &= np.uint64((1 << 61) - 1)
    return c


def cpu_baseline(log_n=20, reps=2):
    """Oracle (CPU restatement, halo2curves best_multiexp algorithm) on a bounded
    sample: one MSM of 2^log_n points with all host threads (<= 16)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle as O

    threads = min(16, os.cpu_count() or 1)
    rng = np.random.default_rng(5)
    n = 1 << log_n
    # bases: any valid points work for timing; reuse a small SRS tiled
    s = O.random_fr(rng, 1)[0]
    small = O.srs_powers(s, 1 << 10)
    bases = np.ascontiguousarray(np.tile(small, (n >> 10, 1)))
    sc = O.random_fr(rng, n)
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        O.msm_best(sc, bases, threads)
        best = min(best, time.perf_counter() - t0)
    return {"value": round(n / best / 1e6, 4), "unit": "Mscalar-mul/s", "cores": threads, "kind": "port",
            "sample": f"one 2^{log_n}-point MSM, oracle best_multiexp (Booth-window Pippenger), "
                      f"{threads} threads, best of {reps}"}


def pmc_traffic(log_n, window_bits):
    """HBM traffic of the dominant kernel from PMC counters, per the MI355X guide:
    one rocprofv3 --pmc pass per counter (FETCH_SIZE and WRITE_SIZE cannot share a
    pass), values in KiB, FETCH_SIZE doubled (gfx950 reports half of a 16-B/lane
    read stream).  Runs child processes BEFORE this process touches the GPU."""
    import csv
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    vals = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix=f"h2g_pmc_{ctr}_", dir="/tmp")
        cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--log-n", str(log_n),
               "--window-bits", str(window_bits)]
        try:
            subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           timeout=240, check=True)
            rows = []
            for root, _, files in os.walk(d):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        rows += [r for r in csv.DictReader(open(os.path.join(root, f)))
                                 if "msm_acc_kernel" in r["Kernel_Name"] and r["Counter_Name"] == ctr]
            if not rows:
                return None, f"no {ctr} rows for msm_acc_kernel"
            vals[ctr] = sum(float(r["Counter_Value"]) for r in rows) / len(rows)
        except Exception as e:  # profiling is best-effort; the timed result stands alone
            return None, f"{ctr} pass failed: {type(e).__name__}"
        finally:
            shutil.rmtree(d, ignore_errors=True)
    traffic = (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
    return traffic, (f"rocprofv3 --pmc per launch of msm_acc_kernel: FETCH_SIZE {vals['FETCH_SIZE']:.0f} KiB (x2 gfx950 "
                     f"correction), WRITE_SIZE {vals['WRITE_SIZE']:.0f} KiB")


def pmc_child(args):
    """Minimal profiled workload: SRS + 2 MSMs (no torch)."""
    import h2g

    h2g.init([0])
    n = 1 << args.log_n
    rng = np.random.default_rng(1000)
    bases = h2g.DevBuf(n * 64)
    h2g.srs_setup_dev(random_scalars(rng, 1)[0], n, bases.ptr)
    sc = h2g.DevBuf.from_array(random_scalars(rng, n))
    for _ in range(2):
        h2g.msm_dev_host(sc.ptr, bases.ptr, n, args.window_bits)
    h2g.shutdown()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-n", type=int, default=24)
    ap.add_argument("--window-bits", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the PMC traffic passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.pmc_child:
        return pmc_child(args)

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    traffic, traffic_note = (None, "skipped (--no-pmc)")
    if not args.no_pmc and world_env == 1:
        traffic, traffic_note = pmc_traffic(args.log_n, args.window_bits)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    import h2g

    h2g.init([torch.cuda.current_device()])
    dev = torch.device("cuda", torch.cuda.current_device())
    stream = torch.cuda.current_stream().cuda_stream
    n = 1 << args.log_n

    # inputs resident in HBM: SRS slab [s^i]G (generated on device) + random scalars
    rng = np.random.default_rng(1000 + rank)
    s = random_scalars(rng, 1)[0]
    bases = torch.empty((n, 8), dtype=torch.int64, device=dev)
    h2g.srs_setup_dev(s, n, bases.data_ptr(), stream)
    scalars = torch.from_numpy(random_scalars(rng, n).view(np.int64)).to(dev)
    torch.cuda.synchronize()
    result = {}

    def step():
        # MsmAccel::msm path: inputs resident in HBM, affine result returned to the host
        result["p"] = h2g.msm_dev_host(scalars.data_ptr(), bases.data_ptr(), n, args.window_bits, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    h2g.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if world > 1:
            part = torch.from_numpy(result["p"].view(np.int64)).to(dev)
            gathered = [torch.empty_like(part) for _ in range(world)]
            dist.all_gather(gathered, part)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    h2g.profile_enable(False)
    calls, phases = h2g.profile_msm_collect()

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # combine the per-rank partial sums (host EC adds), once, outside timing
        total = np.zeros(8, dtype=np.uint64)
        for g in gathered:
            total = h2g.g1_add_affine(total, g.cpu().numpy().view(np.uint64))

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = world * n * args.steps / elapsed / 1e6
        acc_ms = phases.get("accumulate", 0.0) / max(calls, 1)
        total_phase_ms = sum(phases.values()) / max(calls, 1)
        achieved = (n * MSM_BYTES_PER_POINT) / (acc_ms * 1e-3) / 1e9 if acc_ms > 0 else None
        W = None
        try:
            c = args.window_bits or h2g_choose_c(n)
            W = (255 + c - 1) // c
        except Exception:
            c = None
        modmul_rate = (n * W * MADD_MODMUL) / (acc_ms * 1e-3) if (acc_ms > 0 and W) else None
        line = {
            "metric": "MSM Mscalar-mul/s at 2^24 (BN254 G1)",
            "value": round(value, 3),
            "unit": "Mscalar-mul/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 limbs (BN254 Fr/Fq Montgomery, 256-bit modular integer)",
            "data": "synthetic: uniform random Fr scalars, SRS bases [s^i]G generated on device",
            "config": {"workload": f"BN254 G1 MSM, 2^{args.log_n} points per GPU (BASELINE configs[1]/metric)",
                       "points_per_gpu": n, "window_bits": c, "windows": W,
                       "parallelism": f"point-slab shard x{world} + RCCL all_gather of partials"},
            "roofline": {
                "bound": "hbm",
                "kernel": "msm_acc_kernel (bucket accumulation)",
                "achieved": round(achieved, 2) if achieved else None,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
                "traffic": round(traffic) if traffic else None,
                "traffic_note": traffic_note,
                "kernel_ms": round(acc_ms, 4),
                "note": "VALU-bound 256-bit modular arithmetic (no MFMA); HBM fraction is low by construction",
                "valu_modmul_per_s": round(modmul_rate, 1) if modmul_rate else None,
            },
            "phases_ms": {k: round(v / max(calls, 1), 4) for k, v in phases.items()},
            "msm_device_ms": round(total_phase_ms, 4),
        }
        line["ntt"] = ntt_extras(h2g, torch, dev, stream)
        if not args.no_cpu_baseline and world == 1:
            cb = cpu_baseline()
            line["cpu_baseline"] = cb
            line["gpu_vs_cpu"] = round(value / cb["value"], 1)
        print(json.dumps(line), flush=True)

    h2g.shutdown()
    if world > 1:
        dist.destroy_process_group()


def ntt_extras(h2g, torch, dev, stream, reps=5):
    """Side measurements (not the headline value): device-resident radix-2^m NTT
    (best_fft) at 2^20 (BASELINE configs[1]) and 2^22, and coeff_to_extended
    k=22 -> 2^23 (the quotient-domain coset NTT of configs[2..3]).
    Algorithmic bytes: 64 B/element (read + write once)."""
    out = {}
    rng = np.random.default_rng(9)
    for log_n in (20, 22):
        n = 1 << log_n
        a = torch.from_numpy(random_scalars(rng, n).view(np.int64)).to(dev)
        d = h2g.Domain(2, log_n)
        w = d.consts[0]
        h2g.fft_dev(a.data_ptr(), log_n, w, stream)
        torch.cuda.synchronize()
        t = h2g.Timer(stream)
        t.start()
        for _ in range(reps):
            h2g.fft_dev(a.data_ptr(), log_n, w, stream)
        ms = t.stop_ms() / reps
        d.close()
        out[f"fft_2^{log_n}_ms"] = round(ms, 4)
        out[f"fft_2^{log_n}_GBs"] = round(64 * n / (ms * 1e-3) / 1e9, 1)
        out[f"fft_2^{log_n}_modmul_per_s"] = round((n // 2) * log_n / (ms * 1e-3), 1)
    k = 22
    d = h2g.Domain(3, k)
    a = torch.from_numpy(random_scalars(rng, 1 << k).view(np.int64)).to(dev)
    o = torch.empty((d.extended_len, 4), dtype=torch.int64, device=dev)
    h2g.check(h2g.lib().h2g_coeff_to_extended_dev(d.h, h2g.VP(a.data_ptr()), h2g.VP(o.data_ptr()), h2g.VP(stream)))
    torch.cuda.synchronize()
    t = h2g.Timer(stream)
    t.start()
    for _ in range(reps):
        h2g.check(h2g.lib().h2g_coeff_to_extended_dev(d.h, h2g.VP(a.data_ptr()), h2g.VP(o.data_ptr()),
                                                      h2g.VP(stream)))
    ms = t.stop_ms() / reps
    d.close()
    out["coeff_to_extended_k22_ms"] = round(ms, 4)
    return out


def h2g_choose_c(n):
    # mirror of msm_choose_c (msm.hip) for reporting
    best, bc = 1e300, 2
    for c in range(2, 23):
        W = (255 + c - 1) // c
        cost = W * (n + 2.8 * (1 << (c - 1)))
        if cost < best:
            best, bc = cost, c
    return bc


if __name__ == "__main__":
    main()
