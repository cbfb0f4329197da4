#!/usr/bin/env python3
"""Fixed-base MSM time against the window size c at a given length (resident SRS points,
random scalars): per-phase HIP-event times, median of `--steps` after warm-ups.
    python tools/msm_window_sweep.py --log-n 15,19,22 --c 8-20"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "yet-another-halo2-fork_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", default="15,19")
    ap.add_argument("--c", default="8-18")
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import h2g
    import h2g_circuit as hc
    h2g.init([0])
    lo, hi = (int(x) for x in args.c.split("-"))
    rng = np.random.default_rng(7)
    for ln in [int(x) for x in args.log_n.split(",")]:
        n = 1 << ln
        bases = h2g.DevBuf(n * 64)
        h2g.srs_setup_dev(np.asarray(hc.fr_to_limbs(0x1234567), dtype=np.uint64), n, bases.ptr)
        c = rng.integers(0, 2**63, size=(n, 4), dtype=np.int64).astype(np.uint64)
        c[:, 3] &= np.uint64((1 << 61) - 1)
        sc = h2g.DevBuf.from_array(c)
        ref = None
        for cw in list(range(lo, hi + 1)) + [0]:
            if cw and (cw > ln + 2):
                continue
            h = h2g.base_descriptor_dev(bases.ptr, n, cw)
            for _ in range(2):
                res = h2g.msm_with_cached_base_dev(sc.ptr, n, h, 0)
            torch.cuda.synchronize()
            h2g.profile_enable(True)
            import time
            ts = []
            for _ in range(args.steps):
                t0 = time.perf_counter()
                h2g.msm_with_cached_base_dev(sc.ptr, n, h, 0)
                ts.append(time.perf_counter() - t0)
            h2g.profile_enable(False)
            calls, phases = h2g.profile_msm_collect()
            ts.sort()
            ref = res if ref is None else ref
            print(json.dumps({"log_n": ln, "c": cw or "auto", "ms": round(ts[len(ts) // 2] * 1e3, 4),
                              "same": bool(np.array_equal(res, ref)),
                              "phases": {k: round(v / max(calls, 1), 4) for k, v in phases.items()}}), flush=True)
            h2g.descriptor_free(h)
        sc.close()
        bases.close()
    h2g.shutdown()


if __name__ == "__main__":
    main()
