#!/usr/bin/env python3
"""Interleaved A/B of environment switches (H2G_MSM_FINE, H2G_MSM_Q4_MAX, ...) on one box.

Each variant runs in its own child process, variants alternate for `--reps` rounds, and
the child measures lone fixed-base MSMs (2^log_n resident points, per-phase HIP-event
times) and/or the C3 create_proof at k.  Prints one JSON line per child and a summary.

    python tools/ab_env.py --variants 'H2G_MSM_FINE=tile' '' --msm 19,21,22,24 --prove 22 --reps 2
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "yet-another-halo2-fork_amd"))


def child(args):
    import torch
    torch.cuda.set_device(0)
    import h2g
    import h2g_circuit as hc
    h2g.init([0])
    out = {"msm": {}, "prove": {}}
    rng = np.random.default_rng(1000)
    for ln in [int(x) for x in args.msm.split(",") if x]:
        n = 1 << ln
        bases = h2g.DevBuf(n * 64)
        h2g.srs_setup_dev(np.asarray(hc.fr_to_limbs(0x1234567), dtype=np.uint64), n, bases.ptr)
        c = rng.integers(0, 2**63, size=(n, 4), dtype=np.int64).astype(np.uint64)
        c[:, 3] &= np.uint64((1 << 61) - 1)
        sc = h2g.DevBuf.from_array(c)
        base = h2g.base_descriptor_dev(bases.ptr, n, 0)
        for _ in range(2):
            res = h2g.msm_with_cached_base_dev(sc.ptr, n, base, 0)
        torch.cuda.synchronize()
        h2g.profile_enable(True)
        steps = 10
        t0 = time.perf_counter()
        for _ in range(steps):
            h2g.msm_with_cached_base_dev(sc.ptr, n, base, 0)
        el = time.perf_counter() - t0
        h2g.profile_enable(False)
        calls, phases = h2g.profile_msm_collect()
        out["msm"][ln] = {"ms": round(el / steps * 1e3, 4),
                          "sha": __import__("hashlib").sha256(res.tobytes()).hexdigest()[:16],
                          "phases": {k: round(v / max(calls, 1), 4) for k, v in phases.items()}}
        h2g.descriptor_free(base)
        sc.close()
        bases.close()
    for spec in [x for x in args.prove.split(",") if x]:  # "22" (C3) or "keccak:18"
        kind, _, kk = spec.rpartition(":")
        k = int(kk)
        if kind == "keccak":
            circ, wit = hc.keccak_style(k, words=16, seed=5)
        else:
            circ, wit = hc.synthetic_c3(k, h2g.DeviceOps, seed=3)
        params = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(0x1234567), dtype=np.uint64))
        pk = h2g.ProvingKey(params, circ)
        adv = torch.from_numpy(np.ascontiguousarray(wit.advice).view(np.int64)).cuda()
        torch.cuda.synchronize()
        for _ in range(3):
            p0 = pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
        ts = []
        h2g.profile_enable(True)
        for _ in range(10):
            t0 = time.perf_counter()
            p = pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
            ts.append(time.perf_counter() - t0)
            assert p == p0
        h2g.profile_enable(False)
        calls, phases = h2g.profile_msm_collect()
        ts.sort()
        out["prove"][spec] = {"median_ms": round(ts[len(ts) // 2] * 1e3, 3), "min_ms": round(ts[0] * 1e3, 3),
                           "msm_phases": {kk: round(v / max(calls, 1), 4) for kk, v in phases.items()},
                           "proof_sha": __import__("hashlib").sha256(p0).hexdigest()[:16]}
        pk.close()
        params.close()
        del adv
    h2g.shutdown()
    print("AB " + json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", default=[""])
    ap.add_argument("--msm", default="")
    ap.add_argument("--prove", default="")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        return child(args)
    res = {v: [] for v in args.variants}
    for rep in range(args.reps):
        for v in args.variants:
            env = dict(os.environ)
            for kv in v.split():
                k, val = kv.split("=", 1)
                env[k] = val
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--msm", args.msm,
                                "--prove", args.prove], env=env, capture_output=True, text=True, timeout=600)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("AB ")]
            if p.returncode != 0 or not line:
                print(f"variant {v!r} failed rc={p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}", flush=True)
                return 1
            r = json.loads(line[-1][3:])
            res[v].append(r)
            print(json.dumps({"rep": rep, "variant": v or "(default)", **r}), flush=True)
    print("SUMMARY", flush=True)
    for v, rs in res.items():
        msm = {ln: [r["msm"][ln]["ms"] for r in rs] for ln in rs[0]["msm"]}
        prove = {k: [r["prove"][k]["median_ms"] for r in rs] for k in rs[0]["prove"]}
        print(json.dumps({"variant": v or "(default)", "msm_ms": msm, "prove_median_ms": prove}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
