#!/usr/bin/env python3
"""Where a proof's wall time goes on the host: per proof, the Python-measured time of
create_proof against the prover's own (unsynchronised) stage clock, whose sum spans
prove_impl from its StageClock to the final commitment -- the difference is the entry
(argument checks, RNG, Python/ctypes) and exit cost.  usage: host_gap.py [k] [proofs]"""
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
    import h2g_circuit as hc
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    h2g.init([0])
    circ, wit = hc.synthetic_c3(k, h2g.DeviceOps, seed=3)
    params = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(0x1234567), dtype=np.uint64))
    pk = h2g.ProvingKey(params, circ)
    adv = torch.from_numpy(np.ascontiguousarray(wit.advice).view(np.int64)).cuda()
    torch.cuda.synchronize()
    for _ in range(3):
        pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
    rows = []
    for _ in range(reps):
        t0 = time.perf_counter()
        pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
        wall = (time.perf_counter() - t0) * 1e3
        st = h2g.prover_stages()
        rows.append((wall, sum(ms for _, ms in st), st))
    for wall, inner, st in rows:
        print(f"wall {wall:7.2f} ms  stage clock {inner:7.2f} ms  outside {wall - inner:5.2f} ms  "
              + " ".join(f"{nm}={ms:.2f}" for nm, ms in st), flush=True)
    h2g.shutdown()


if __name__ == "__main__":
    main()
