"""Time the device create_proof on the C3 synthetic circuit or the C5-shaped
keccak-style circuit at the given k values; prints per-stage wall times.
usage: python tools/prove_bench.py [c3|keccak] [--dev] [--sync] 20 22
--dev: the witness resident in HBM (bench.py's `value` path) instead of host memory
--sync: the prover drains its streams at every stage mark (per-stage GPU time; slower)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "yet-another-halo2-fork_amd")]
import numpy as np  # noqa: E402

import h2g  # noqa: E402
import h2g_circuit as hc  # noqa: E402


def main():
    args = sys.argv[1:]
    kind = "c3"
    dev = "--dev" in args
    sync = "--sync" in args
    args = [a for a in args if a not in ("--dev", "--sync")]
    if args and not args[0].isdigit():
        kind = args.pop(0)
    ks = [int(a) for a in args] or [20]
    if dev:
        import torch  # noqa: F401 -- before h2g.init (h2g.init: torch's HIP runtime first)
    h2g.init()
    if sync:
        h2g.prover_stage_sync(True)
    for k in ks:
        t0 = time.time()
        circ, wit = hc.synthetic_c3(k, h2g.DeviceOps) if kind == "c3" else hc.keccak_style(k)
        t1 = time.time()
        params = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(0x1234567 + k), dtype=np.uint64))
        t2 = time.time()
        pk = h2g.ProvingKey(params, circ)
        adv = None
        if dev:
            import torch
            adv = torch.from_numpy(np.ascontiguousarray(wit.advice).view(np.int64)).cuda()
            torch.cuda.synchronize()
        t3 = time.time()
        print(f"k={k}: witness {t1 - t0:.2f}s  srs {t2 - t1:.2f}s  keygen {t3 - t2:.2f}s", flush=True)
        times = []
        for it in range(4):
            a = time.time()
            proof = pk.create_proof(wit) if adv is None else pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
            times.append(time.time() - a)
            st = h2g.prover_stages()
            print(f"  prove {times[-1] * 1e3:.1f} ms, {len(proof)} B: " +
                  ", ".join(f"{nm} {ms:.1f}" for nm, ms in st), flush=True)
        print(f"k={k} best {min(times) * 1e3:.1f} ms", flush=True)
        pk.close()
        params.close()


if __name__ == "__main__":
    main()
