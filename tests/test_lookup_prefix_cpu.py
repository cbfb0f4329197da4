"""The identity behind the lookup commitments' prefix basis (prover.cpp params_prefix,
SRS_LAGRANGE_PREFIX): with P_i = L_0 + ... + L_i,

    sum_i a_i L_i  ==  sum_i (a_i - a_{i+1}) P_i      (a_n = 0),

so a lookup's permuted columns A', S' (runs of equal values after permute_expression_pair,
halo2_backend/src/plonk/lookup/prover.rs:410-494) commit to the same point from scalars
that vanish inside every run.  Checked on the CPU with the reference group law
(oracle/py/bn254_ref.py) for a run-structured column, a dense one and one ending in
blinding rows; the device path is covered by the GPU proof-bytes tests."""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle", "py"))

from bn254_ref import G1_GEN, R, g1_add, g1_mul, msm_naive  # noqa: E402


def _prefix(points):
    out, acc = [], None
    for p in points:
        acc = p if acc is None else g1_add(acc, p)
        out.append(acc)
    return out


def _diffs(a):
    return [(a[i] - (a[i + 1] if i + 1 < len(a) else 0)) % R for i in range(len(a))]


def test_prefix_basis_commitment_identity():
    rnd = random.Random(11)
    n = 24
    lag = [g1_mul(G1_GEN, rnd.randrange(1, R)) for _ in range(n)]  # stand-ins for L_i = [L_i(s)] G
    pre = _prefix(lag)
    runs = sorted(rnd.choice([3, 5, 7, 11]) for _ in range(n - 3)) + [rnd.randrange(R) for _ in range(3)]
    dense = [rnd.randrange(R) for _ in range(n)]
    for a in (runs, dense, [0] * n, [5] * n):
        d = _diffs(a)
        assert msm_naive(d, pre) == msm_naive(a, lag)
    # the run column's scalars are zero inside its runs: the MSM's work follows the runs
    assert sum(1 for x in _diffs(runs) if x) <= 4 + 3 + 1
