"""CPU baseline study: the oracle's create_proof (C restatement of
halo2_backend's prover) of the bench's C3 circuit, in both modes, at several k, median of
`--reps` runs after one warm-up run, keygen excluded.

  all-cores : MSM / FFT and the parallelize-style loops on T OpenMP threads
  faithful  : MSM / FFT single-threaded (halo2curves without its `multicore` feature,
              SURVEY finding 3), the parallelize-style loops on T threads

The SRS comes from the device (h2g_params_setup, tested bit-exact against the oracle's);
only the CPU prover is timed.  Writes one JSON object (stdout and --out).
usage: python tools/cpu_baseline.py [--ks 18,20,22] [--reps 3] [--modes all,faithful]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "yet-another-halo2-fork_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="18,20,22")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="all,faithful")
    ap.add_argument("--faithful-max-k", type=int, default=20)
    ap.add_argument("--out", default="")
    ap.add_argument("--no-warmup", action="store_true")
    a = ap.parse_args()
    import _oracle as O  # the checker's CPU restatement, timed here as the baseline
    import bench
    import h2g
    import h2g_circuit as hc

    import threading

    def heartbeat():  # a progress line every minute (long faithful-mode runs)
        t0 = time.time()
        while True:
            time.sleep(60)
            print(f"  ... {time.time() - t0:.0f} s", flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    h2g.init()
    model, ncpu = bench.cpu_info()
    T, how = bench.cpu_threads()
    res = {"cpu_model": model, "nproc": ncpu, "threads": T, "threads_from": how, "reps": a.reps, "runs": []}
    for k in [int(x) for x in a.ks.split(",")]:
        circ, wit = hc.synthetic_c3(k, h2g.DeviceOps, seed=3)
        params = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(0x1234567), dtype=np.uint64))
        g, gl = params.export()
        params.close()
        kg = O.Keygen(circ, wit, g, gl, threads=T)
        for mode in a.modes.split(","):
            if mode == "faithful" and k > a.faithful_max_k:
                continue
            O.lib().or_set_kernel_threads(1 if mode == "faithful" else 0)
            if not a.no_warmup:
                O.create_proof(circ, wit, g, gl, threads=T, keygen=kg)  # warm-up
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                O.create_proof(circ, wit, g, gl, threads=T, keygen=kg)
                ts.append(time.perf_counter() - t0)
                print(f"  k={k} {mode}: {ts[-1]:.3f} s", flush=True)
            run = {"k": k, "mode": mode, "median_s": round(sorted(ts)[len(ts) // 2], 3),
                   "runs_s": [round(t, 3) for t in ts]}
            res["runs"].append(run)
            print(json.dumps(run), flush=True)
        O.lib().or_set_kernel_threads(0)
        kg.close()
    h2g.shutdown()
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
