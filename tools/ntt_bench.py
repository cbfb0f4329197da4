"""Time device NTTs through the C ABI (for rocprofv3 --kernel-trace --stats)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "yet-another-halo2-fork_amd"))
import h2g  # noqa: E402

h2g.init([0])
rng = np.random.default_rng(1)
for log_n in [int(x) for x in (sys.argv[1:] or ["20", "22"])]:
    n = 1 << log_n
    a = rng.integers(0, 2**62, size=(n, 4), dtype=np.int64).astype(np.uint64)
    d = h2g.DevBuf.from_array(a)
    dom = h2g.Domain(2, log_n)
    w = dom.consts[0]
    h2g.fft_dev(d.ptr, log_n, w)
    h2g.check(h2g.lib().h2g_synchronize())
    t = h2g.Timer()
    t.start()
    for _ in range(10):
        h2g.fft_dev(d.ptr, log_n, w)
    ms = t.stop_ms() / 10
    print(f"fft 2^{log_n}: {ms:.4f} ms  {(n // 2) * log_n / ms / 1e6:.1f} Mbfly/s")
    # lagrange_to_coeff (inverse, scaled by 1/n) and coeff_to_extended (coset, 2n points)
    ext = h2g.DevBuf(2 * n * 32)
    L = h2g.lib()
    h2g.check(L.h2g_lagrange_to_coeff_dev(dom.h, h2g.VP(d.ptr), None))
    h2g.check(L.h2g_coeff_to_extended_dev(dom.h, h2g.VP(d.ptr), h2g.VP(ext.ptr), None))
    h2g.check(L.h2g_synchronize())
    for nm, fn in (("lagrange_to_coeff", lambda: L.h2g_lagrange_to_coeff_dev(dom.h, h2g.VP(d.ptr), None)),
                   ("coeff_to_extended", lambda: L.h2g_coeff_to_extended_dev(dom.h, h2g.VP(d.ptr), h2g.VP(ext.ptr),
                                                                              None))):
        t.start()
        for _ in range(10):
            h2g.check(fn())
        print(f"{nm} 2^{log_n}: {t.stop_ms() / 10:.4f} ms")
    # a degree-5 circuit's coset extension (j = 5: 4x the points, a quarter of them nonzero)
    dom5 = h2g.Domain(5, log_n)
    ext4 = h2g.DevBuf(dom5.extended_len * 32)
    h2g.check(L.h2g_coeff_to_extended_dev(dom5.h, h2g.VP(d.ptr), h2g.VP(ext4.ptr), None))
    h2g.check(L.h2g_synchronize())
    t.start()
    for _ in range(10):
        h2g.check(L.h2g_coeff_to_extended_dev(dom5.h, h2g.VP(d.ptr), h2g.VP(ext4.ptr), None))
    print(f"coeff_to_extended_x4 2^{log_n}: {t.stop_ms() / 10:.4f} ms")
h2g.shutdown()
