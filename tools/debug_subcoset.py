"""Debug: compare the SPMD sub-coset arrays with the single-GPU full cosets (H2G_DUMP)."""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
case = sys.argv[1] if len(sys.argv) > 1 else "mixed_k10"
base = os.path.join(REPO, "gpurun_out", "dbg")
os.makedirs(base, exist_ok=True)
# single GPU (world 1 via the case runner with --nproc 1 is not SPMD): use h2g directly
code = f"""
import os, sys
sys.path[:0] = [{os.path.join(REPO, 'yet-another-halo2-fork_amd')!r}, {os.path.join(REPO, 'tests')!r}, {os.path.join(REPO, 'oracle', 'py')!r}]
import numpy as np, h2g, h2g_circuit as hc
sys.argv = ['x']
import _shard_prove as S
h2g.init([0])
case = S.CASES[{case!r}]()
circ = case[0]
params = h2g.Params(circ.k, s=np.asarray(hc.fr_to_limbs(0x5eed + circ.k), dtype=np.uint64))
pk = h2g.ProvingKey(params, circ)
S._prove(pk, case, seed=bytes(range(32)), vanishing_threads=3)
"""
env = dict(os.environ, H2G_DUMP=os.path.join(base, "full"))
os.makedirs(env["H2G_DUMP"], exist_ok=True)
subprocess.run([sys.executable, "-c", code], check=True, env=env, timeout=300)
print("full done", flush=True)

port = 29611
env = dict(os.environ, H2G_DUMP_BASE=os.path.join(base, "spmd"), HSA_ENABLE_IPC_MODE_LEGACY="0")
subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                "--master-addr", "127.0.0.1", "--master-port", str(port),
                os.path.join(REPO, "tests", "_shard_prove.py"), "--backend", "gloo", "--mode", "spmd"]
               + os.environ.get("DBG_PRE", "").split() + [case],
               check=False, env=env, timeout=600)
print("spmd done", flush=True)


def load(d, name):
    p = os.path.join(d, name + ".bin")
    return np.fromfile(p, dtype=np.uint64).reshape(-1, 4) if os.path.exists(p) else None


full = os.path.join(base, "full")
hf = load(full, "h_ext")
ext = len(hf)
for name in ("adv_coset0", "z_coset0", "inst_coset0"):
    f = load(full, name)
    for r in range(2):
        sd = load(os.path.join(base, "spmd", f"r{r}"), name)
        if f is None or sd is None:
            print(name, "missing")
            continue
        E = int(sys.argv[2]) if len(sys.argv) > 2 else 4
        n = ext // E
        # sub-coset slots t = r, r + 2, ...
        for i, t in enumerate(range(r, E, 2)):
            ok = np.array_equal(sd[i * n:(i + 1) * n], f[t::E])
            print(name, "rank", r, "slot", i, "t", t, "ok", ok, flush=True)
for r in range(2):
    hs = load(os.path.join(base, "spmd", f"r{r}"), "h_ext")
    print("h_ext rank", r, "equal", np.array_equal(hs, hf), flush=True)
    if not np.array_equal(hs, hf):
        for E in (2, 4):
            if ext % E == 0:
                for t in range(E):
                    print("  E", E, "t", t, np.array_equal(hs[t::E], hf[t::E]))
