#!/usr/bin/env python3
"""The metric's MSM half over N GPUs, emulated on one GPU.

One 2^log_n MSM strong-scaled over N ranks is what bench.py's msm_2p24 runs at N > 1: rank
r holds point slab [n r / N, n (r + 1) / N) with its scalars and fixed-base windows sized
for the slab, runs a whole MSM on it, and the 64-B partials are all-gathered and summed on
the host.  Every rank does the same work, so one GPU measures a rank: the slab MSM (HIP
events, median of `steps`), plus the all-gather's modelled wire time (latency + 64 B per
link over xGMI, --comm-model) and the host sum of the N partials (measured,
h2g_g1_add_affine).  The full 2^log_n MSM on the same box is the baseline.

    python tools/msm_scale_emulate.py --log-n 24 --worlds 2,4,8 [--comm-model 50,40]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "yet-another-halo2-fork_amd"))
sys.path.insert(0, REPO)

import h2g  # noqa: E402
import h2g_circuit as hc  # noqa: E402


def msm_ms(n, steps, warmup, seed):
    """median wall ms of one fixed-base MSM of n resident points (windows built for n)"""
    import torch
    stream = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(seed)
    bases = torch.empty((n, 8), dtype=torch.int64, device="cuda")
    h2g.srs_setup_dev(np.asarray(hc.fr_to_limbs(0x1234567 + seed), dtype=np.uint64), n, bases.data_ptr(), stream)
    c = rng.integers(0, 2**63, size=(n, 4), dtype=np.int64).astype(np.uint64)
    c[:, 3] &= np.uint64((1 << 61) - 1)
    sc = torch.from_numpy(c.view(np.int64)).cuda()
    torch.cuda.synchronize()
    base = h2g.base_descriptor_dev(bases.data_ptr(), n, 0)
    part = None
    for _ in range(warmup):
        part = h2g.msm_with_cached_base_dev(sc.data_ptr(), n, base, 0, stream)
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        part = h2g.msm_with_cached_base_dev(sc.data_ptr(), n, base, 0, stream)
        ts.append(time.perf_counter() - t0)
    h2g.descriptor_free(base)
    del bases, sc
    torch.cuda.empty_cache()
    ts.sort()
    return 1e3 * ts[len(ts) // 2], part


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=24)
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--comm-model", default="50,40", help="GB/s,us per xGMI link (all-gather of the partials)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    h2g.init([0])
    n = 1 << args.log_n
    gbs, lat = (float(x) for x in args.comm_model.split(","))
    full, _ = msm_ms(n, args.steps, args.warmup, 0)
    out = {"log_n": args.log_n, "full_ms": round(full, 3), "comm_model": args.comm_model, "worlds": {}}
    print(json.dumps({"full_ms": out["full_ms"]}), flush=True)
    for N in [int(x) for x in args.worlds.split(",")]:
        slab = n // N
        t, part = msm_ms(slab, args.steps, args.warmup, N)
        # the all-gather of 9 words per rank (partial + identity flag): every rank receives
        # 72 B from each peer over its own link
        comm = 1e3 * (lat * 1e-6 + 72 / (gbs * 1e9))
        parts = [part] * N  # the host sum of N partials (their values do not change its cost)
        t0 = time.perf_counter()
        tot = np.zeros(8, dtype=np.uint64)
        for _ in range(20):
            tot = np.zeros(8, dtype=np.uint64)
            for p in parts:
                tot = h2g.g1_add_affine(tot, p)
        host = 1e3 * (time.perf_counter() - t0) / 20
        step = t + comm + host
        out["worlds"][N] = {"slab_points": slab, "slab_msm_ms": round(t, 3), "allgather_ms_modelled": round(comm, 4),
                            "host_sum_ms": round(host, 4), "step_ms": round(step, 3),
                            "mscalar_mul_per_s": round(n / (step * 1e-3) / 1e6, 1),
                            "speedup": round(full / step, 3), "efficiency": round(full / step / N, 3)}
        print(json.dumps({"N": N, **out["worlds"][N]}), flush=True)
    h2g.shutdown()
    print("MSMSCALE " + json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
