#!/usr/bin/env python3
"""The bench's strong-scaled MSM (one 2^log_n fixed-base MSM over N GPUs) measured one rank
at a time on one GPU: per world size, every rank's part (h2g_msm_with_cached_base_dev_shard,
bucket ranges) and, for comparison, round 2's point slabs (a whole MSM of n / N points);
the slowest rank's time before the all-gather of the partials is the predicted per-MSM
time.  usage: msm_shard_emulate.py [log_n] [worlds]   (default 24, 1,2,4,8)"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "yet-another-halo2-fork_amd"))


def main():
    import torch
    torch.cuda.set_device(0)
    import h2g
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    worlds = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4,8").split(",")]
    h2g.init([0])
    stream = torch.cuda.current_stream().cuda_stream
    n = 1 << log_n
    rng = np.random.default_rng(1000)
    s = rng.integers(0, 2**62, size=4, dtype=np.int64).astype(np.uint64)
    bases = torch.empty((n, 8), dtype=torch.int64, device="cuda")
    h2g.srs_setup_dev(s, n, bases.data_ptr(), stream)
    sc = rng.integers(0, 2**63, size=(n, 4), dtype=np.int64).astype(np.uint64)
    sc[:, 3] &= np.uint64((1 << 61) - 1)
    scalars = torch.from_numpy(sc.view(np.int64)).cuda()
    torch.cuda.synchronize()
    base = h2g.base_descriptor_dev(bases.data_ptr(), n, 0)
    whole = h2g.msm_with_cached_base_dev(scalars.data_ptr(), n, base, 0, stream)

    def timed(fn, reps=8):
        fn()
        torch.cuda.synchronize()
        h2g.profile_enable(True)
        t0 = time.perf_counter()
        for _ in range(reps):
            r = fn()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / reps * 1e3
        h2g.profile_enable(False)
        calls, phases = h2g.profile_msm_collect()
        return el, {k: round(v / max(calls, 1), 4) for k, v in phases.items()}, r

    out = {"log_n": log_n, "whole_ms": None, "worlds": {}}
    out["whole_ms"], _, _ = timed(lambda: h2g.msm_with_cached_base_dev(scalars.data_ptr(), n, base, 0, stream))
    for world in worlds:
        ranks, total = [], np.zeros(8, dtype=np.uint64)
        for r in range(world):
            ms, ph, res = timed(lambda: h2g.msm_with_cached_base_dev_shard(scalars.data_ptr(), n, base, world, r, 0,
                                                                           stream))
            total = h2g.g1_add_affine(total, res[0])
            ranks.append({"rank": r, "ms": round(ms, 4), "range": list(res[2]), "phases": ph})
        slab = None
        if world > 1:  # round 2's point slab: a whole MSM of n / world points (its own windows)
            m = n // world
            bslab = h2g.base_descriptor_dev(bases.data_ptr(), m, 0)
            slab, _, _ = timed(lambda: h2g.msm_with_cached_base_dev(scalars.data_ptr(), m, bslab, 0, stream))
            h2g.descriptor_free(bslab)
        slowest = max(x["ms"] for x in ranks)
        out["worlds"][world] = {"slowest_rank_ms": round(slowest, 4), "speedup": round(out["whole_ms"] / slowest, 2),
                                "point_slab_ms": round(slab, 4) if slab else None,
                                "point_slab_speedup": round(out["whole_ms"] / slab, 2) if slab else None,
                                "sum_equals_whole": bool(np.array_equal(total, whole)), "ranks": ranks}
        print(json.dumps({"world": world, **{k: v for k, v in out["worlds"][world].items() if k != "ranks"}}),
              flush=True)
    print("RESULT " + json.dumps(out), flush=True)
    h2g.descriptor_free(base)
    h2g.shutdown()


if __name__ == "__main__":
    main()
