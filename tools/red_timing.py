#!/usr/bin/env python3
"""Phase stamps inside the MSM reduction kernels (diagnostic build):
    python tools/build_variant.py redts --src msm.hip -DH2G_RED_TIMING
    H2G_LIB=.../libh2g_redts.so python tools/red_timing.py --msm 15,19
Prints, per MSM size, the median over runs of each stamp's offset (us) from the start of
msm_rgroup_plane_kernel's block 0 (stamps: see RED_TS in csrc/msm.hip)."""
import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "yet-another-halo2-fork_amd"))

NAMES = {0: "rgp b0 start", 1: "rgp b0 loaded", 2: "rgp b0 tree done", 3: "rgp b0 end", 4: "rgp last start",
         5: "rgp last end", 8: "mid sum start", 9: "mid sum loaded", 10: "mid sum tree done", 11: "mid fold start",
         12: "mid fold loaded", 13: "mid fold done", 14: "mid last block", 15: "mid doublings done",
         16: "mid final tree done", 20: "fixup b0 start", 22: "fixup last start"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msm", default="15,19")
    ap.add_argument("--runs", type=int, default=8)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import h2g
    import h2g_circuit as hc
    h2g.init([0])
    f = h2g.lib().h2g_dbg_red_ts
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 64)()
    rng = np.random.default_rng(5)
    for ln in [int(x) for x in args.msm.split(",")]:
        n = 1 << ln
        bases = h2g.DevBuf(n * 64)
        h2g.srs_setup_dev(np.asarray(hc.fr_to_limbs(0x1234567), dtype=np.uint64), n, bases.ptr)
        c = rng.integers(0, 2**63, size=(n, 4), dtype=np.int64).astype(np.uint64)
        c[:, 3] &= np.uint64((1 << 61) - 1)
        sc = h2g.DevBuf.from_array(c)
        base = h2g.base_descriptor_dev(bases.ptr, n, 0)
        rows = []
        for r in range(args.runs + 2):
            h2g.msm_with_cached_base_dev(sc.ptr, n, base, 0)
            torch.cuda.synchronize()
            assert f(buf) == 0
            if r >= 2:
                rows.append(np.array(buf[:], dtype=np.int64))
        a = np.stack(rows)
        ref = a[:, 0:1]
        rel = np.where(a > 0, (a - ref) * 0.01, np.nan)  # 100 MHz -> us
        med = np.nanmedian(rel, axis=0)
        print(f"2^{ln}:", {NAMES[i]: round(float(med[i]), 1) for i in sorted(NAMES) if not np.isnan(med[i])},
              flush=True)
        h2g.descriptor_free(base)
        sc.close()
        bases.close()
    h2g.shutdown()


if __name__ == "__main__":
    main()
