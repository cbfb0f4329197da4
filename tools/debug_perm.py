"""Debug: dump device permutation intermediates for simple_example(6), recompute in Python."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, d) for d in ("tests", "oracle/py", "yet-another-halo2-fork_amd")]
os.makedirs(os.path.join(REPO, "gpurun_out/dump"), exist_ok=True)
os.environ["H2G_DUMP"] = os.path.join(REPO, "gpurun_out/dump")
import numpy as np
import _oracle as O, h2g, h2g_circuit as hc, verifier as V
h2g.init()
circ, wit = hc.simple_example(6)
s, g, gl = O.srs(6)
params = h2g.Params(6, g, gl)
pk = h2g.ProvingKey(params, circ)
proof = pk.create_proof(wit)
D = os.environ["H2G_DUMP"]
ld = lambda nm: hc.mont_to_ints(np.fromfile(os.path.join(D, nm + ".bin"), dtype=np.uint64))
R = hc.R_MOD
beta, gamma = ld("beta")[0], ld("gamma")[0]
from bn254_ref import Domain
dom = Domain(3, 6)
sig = V.sigma_values(circ, dom)
n = 64
print("sigma0 ok", ld("sigma0") == sig[0])
v0 = hc.mont_to_ints(wit.instance[0])
print("v0 ok", ld("v0") == v0)
den = [(beta * sig[0][r] + gamma + v0[r]) % R for r in range(n)]
print("den ok", ld("den0") == den)
inv = [pow(x, -1, R) for x in den]
print("inv ok", ld("inv0") == inv)
w = [pow(dom.omega, r, R) for r in range(n)]
mod = [inv[r] * (beta * w[r] + gamma + v0[r]) % R for r in range(n)]
got = ld("mod0")
print("mod ok", got == mod, [i for i in range(n) if got[i] != mod[i]][:5])
pre = []
acc = 1
for r in range(n):
    acc = acc * mod[r] % R
    pre.append(acc)
gp = ld("pre0")
print("pre ok", gp == pre, [i for i in range(n) if gp[i] != pre[i]][:5])
z = ld("z0")
print("z[0..] head ok", z[:n - 5] == [1] + pre[:n - 6])
