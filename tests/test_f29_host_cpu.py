"""csrc/f29.h's primitives and XYZZ formulas at the worst-case operands of the bounds model.

A host program (tests/native/f29_host.cpp, built from the kernels' own header with hipcc
for the host side only) runs mul29, sqr29, mul29x2, sub29, reduce29, is_zero29 and the
XYZZ madd / add / dbl on operands chosen at the limits tools/f29_bounds.py derives:
limbs at their maxima, values carrying the largest multiple of M the data flow allows,
the accumulation's coordinates at the model's fixpoint, the back-end's at 1.2 M.
Every result is checked with Python big integers: the Montgomery congruence (R = 2^261),
the output bound REDC(x) < x / R + M, normalised limbs, and for the curve formulas the
affine BN254 group law of oracle/py/bn254_ref.py.  Random-input parity on the GPU cannot
reach these operands; an overflow near the bounds shows up here.
"""
import os
import random
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# H2G_F29_CSRC: build the harness against another copy of the headers (mutation checks)
CSRC = os.environ.get("H2G_F29_CSRC") or os.path.join(REPO, "yet-another-halo2-fork_amd", "csrc")
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "oracle", "py"))
import bn254_ref as B  # noqa: E402
import f29_bounds as F  # noqa: E402

MQ, MR_ = F.M, F.MR
RR = 1 << 261
N29 = 1 << 29
MASK = N29 - 1
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


# ------------------------------------------------------------------ limb helpers
def limbs(v):
    """normalised 29-bit limbs of v >= 0 (limbs 0..7 < 2^29, the rest in the top limb)"""
    assert 0 <= v
    out = [(v >> (29 * i)) & MASK for i in range(8)] + [v >> 232]
    assert out[8] < 1 << 32, v.bit_length()
    return out


def val(ls):
    return sum(int(x) << (29 * i) for i, x in enumerate(ls))


def km29_safe(k, off, m):
    """kmul_safe (f29.h) restated: k M with limbs 0..7 raised by 2^off, the top lowered"""
    n = limbs(k * m)
    unit = 1 << (off - 29)
    return [n[0] + (1 << off)] + [n[i] + (1 << off) - unit for i in range(1, 8)] + [n[8] - unit]


@pytest.fixture(scope="module")
def run(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not found")
    exe = tmp_path_factory.mktemp("f29host") / "f29_host"
    subprocess.run([HIPCC, "--offload-host-only", "-O2", "-std=c++17", "-I", CSRC,
                    os.path.join(REPO, "tests", "native", "f29_host.cpp"), "-o", str(exe)],
                   check=True, cwd=str(exe.parent))

    def go(cmds):
        text = "\n".join(op + " " + " ".join(str(x) for x in args) for op, args in cmds) + "\n"
        out = subprocess.run([str(exe)], input=text, check=True, capture_output=True, text=True).stdout
        rows = out.splitlines()
        assert len(rows) == len(cmds)
        for r in rows:
            assert not r.startswith("ERR"), r
        return [[int(x) for x in r.split()] for r in rows]
    return go


def redc_ok(out, x, m):
    """out = REDC(x) as the kernels produce it: congruent, < x / R + M, limbs 0..7 normalised"""
    v = val(out)
    assert all(l < N29 for l in out[:8]), out
    assert (v - x * pow(RR, -1, m)) % m == 0
    assert v < x // RR + m + 1, (v.bit_length(), (x // RR + m).bit_length())


# ------------------------------------------------------------------ field primitives
def _operands(m, rng):
    top_norm = [MASK] * 9                            # 2^261 - 1: the largest normalised value
    sum2 = [2 * MASK] * 9                            # a limb-wise add of two of them (< 2^262)
    near = [limbs(k * m + d) for k in (1, 7, 32, 57, 64) for d in (-1, 0, 1)]
    rnd = [[rng.getrandbits(29) for _ in range(8)] + [rng.getrandbits(29)] for _ in range(24)]
    return [top_norm, sum2, limbs(0), limbs(1), limbs(m - 1)] + near + rnd


@pytest.mark.parametrize("fld", ["q", "r"])
def test_mul29_sqr29_at_the_limb_bounds(run, fld):
    m = MQ if fld == "q" else MR_
    rng = random.Random(1)
    ops = _operands(m, rng)
    pairs = [(a, b) for a in ops for b in ops[:12]]
    # mul29's column bound: limbs 0..7 < 2^30 and a top limb < 2^31 against a small operand
    # (the NTT's stage values times a twiddle)
    wide = [(1 << 30) - 1] * 8 + [(1 << 31) - 1]
    pairs += [(wide, limbs(m - 1)), (limbs(m - 1), wide), (wide, [MASK] * 8 + [limbs(m)[8]])]
    got = run([("mul" + fld, a + b) for a, b in pairs])
    for (a, b), o in zip(pairs, got):
        redc_ok(o, val(a) * val(b), m)
    # sqr29 takes normalised operands (top limb up to 2^30: U = 2 Y of the doubling)
    sq = [a for a in ops if all(l < N29 for l in a[:8]) and a[8] < 1 << 30] + [[MASK] * 8 + [(1 << 30) - 1]]
    got_s = run([("sqr" + fld, a) for a in sq])
    got_m = run([("mul" + fld, a + a) for a in sq])
    for a, s, mm in zip(sq, got_s, got_m):
        redc_ok(s, val(a) ** 2, m)
        assert s == mm  # the same REDC as mul29(a, a), bit for bit


@pytest.mark.parametrize("fld", ["q", "r"])
def test_mul29x2_at_its_column_bound(run, fld):
    """a, c normalised, b, d limbs just below 1.5 * 2^30: the middle column sits at ~2^63.98"""
    m = MQ if fld == "q" else MR_
    rng = random.Random(2)
    big = [3 * (1 << 29) - 1] * 9
    cases = [([MASK] * 9, big, [MASK] * 9, big)]
    for _ in range(40):
        a = [rng.choice((MASK, rng.getrandbits(29))) for _ in range(9)]
        c = [rng.choice((MASK, rng.getrandbits(29))) for _ in range(9)]
        b = [rng.choice((3 * (1 << 29) - 1, rng.randrange(3 << 29))) for _ in range(9)]
        d = [rng.choice((3 * (1 << 29) - 1, rng.randrange(3 << 29))) for _ in range(9)]
        cases.append((a, b, c, d))
    got = run([("mulx2" + fld, a + b + c + d) for a, b, c, d in cases])
    for (a, b, c, d), o in zip(cases, got):
        redc_ok(o, val(a) * val(b) + val(c) * val(d), m)


SUBS = [("q", 64, 29), ("q", 32, 31), ("q", 16, 29), ("q", 4, 31), ("q", 4, 29), ("q", 2, 29),
        ("r", 64, 29), ("r", 4, 29), ("r", 8, 29), ("r", 16, 29), ("r", 32, 29), ("r", 128, 29)]


def test_sub29_instantiations_cover_the_sources():
    used = set()
    for key, v in F.source_constants().items():
        if key == "is_zero29":
            continue
        fld = "r" if key.startswith(("ntt.hip", "prover_kernels.hip")) else "q"
        for k, off in v:
            ks = [F.k_of(k, s) for s in range(6)] if "S" in k else [F.k_of(k)]
            used |= {(fld, kk, int(off)) for kk in ks}
    assert used <= set(SUBS), used - set(SUBS)


@pytest.mark.parametrize("fld,K,OFF", SUBS)
def test_sub29_never_borrows_at_its_bounds(run, fld, K, OFF):
    """b with every low limb at 2^OFF - 1 and the largest top limb kmul_safe leaves room for"""
    m = MQ if fld == "q" else MR_
    L = km29_safe(K, OFF, m)
    rng = random.Random(K * 100 + OFF)
    bmax = [(1 << OFF) - 1] * 8 + [L[8]]
    cases = [([MASK] * 9, bmax), (limbs(0), bmax), ([MASK] * 9, limbs(0)), (limbs(0), limbs(0))]
    for _ in range(30):
        a = [rng.getrandbits(29) for _ in range(9)]
        b = [rng.randrange(1 << OFF) for _ in range(8)] + [rng.randrange(L[8] + 1)]
        cases.append((a, b))
    got = run([(f"sub{fld}_{K}_{OFF}", a + b) for a, b in cases])
    for (a, b), o in zip(cases, got):
        assert val(o) == val(a) - val(b) + K * m  # as integers: no limb wrapped
        assert all(0 <= x < 1 << 32 for x in o)
        assert o == [a[i] + L[i] - b[i] for i in range(9)]


@pytest.mark.parametrize("fld", ["q", "r"])
def test_reduce29_over_the_whole_top_limb(run, fld):
    m = MQ if fld == "q" else MR_
    rng = random.Random(3)
    vs = [[MASK] * 8 + [(1 << 32) - 1], limbs(0), limbs(m - 1), limbs(m)]
    vs += [limbs(k * m + d) for k in (1, 2, 31, 64, 96, 255) for d in (-1, 0, 1)]
    vs += [[rng.getrandbits(29) for _ in range(8)] + [rng.getrandbits(32)] for _ in range(60)]
    got = run([("red" + fld, v) for v in vs])
    mt = limbs(m)[8] + 1
    for v, o in zip(vs, got):
        x, y = val(v), val(o)
        q = v[8] // mt
        assert (x - y) % m == 0 and 0 <= y < m + (q + 2) * (1 << 232), (x.bit_length(), y / m)
        assert all(l < N29 for l in o[:8])


@pytest.mark.parametrize("fld", ["q", "r"])
def test_is_zero29_up_to_its_threshold(run, fld):
    m = MQ if fld == "q" else MR_
    thr = F.source_constants()["is_zero29"]
    ks = list(range(0, 70)) + [127, 128, 255, 256, 511, 512, 1000, thr - 1, thr]
    cases = [(limbs(k * m), 1) for k in ks]
    cases += [(limbs(k * m + 1), 0) for k in ks] + [(limbs(k * m - 1), 0) for k in ks if k]
    cases += [(limbs(k * m + (1 << 232)), 0) for k in (0, 5, 64)]
    got = run([("isz" + fld, v) for v, _ in cases])
    for (v, want), o in zip(cases, got):
        assert o == [want], (val(v) // m, want)


# ------------------------------------------------------------------ curve formulas
def _points(n, seed):
    """n distinct affine points kG (consecutive multiples from a random start)"""
    rng = random.Random(seed)
    p = B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))
    out = []
    for _ in range(n):
        out.append(p)
        p = B.g1_add(p, B.G1_GEN)
    return out


def _mont(e):
    return e * RR % MQ


def _rep(e, bound, rng, top=True):
    """an F29 value of the field element e carrying the largest multiple of M below bound
    (or a random one when top is False)"""
    v = _mont(e)
    kmax = max(0, (bound - 1 - v) // MQ)
    return limbs(v + (kmax if top else rng.randrange(kmax + 1)) * MQ)


def _xyzz(pt, z, bounds, rng, top=True):
    x, y = pt
    zz, zzz = z * z % MQ, z * z * z % MQ
    es = (x * zz % MQ, y * zzz % MQ, zz, zzz)
    return [l for e, bd in zip(es, bounds) for l in _rep(e, bd, rng, top)]


def _affine(ls):
    X, Y, ZZ, ZZZ = (val(ls[9 * i:9 * i + 9]) for i in range(4))
    if all(l == 0 for l in ls[18:27]):
        return None
    rinv = pow(RR, -1, MQ)
    x, y, zz, zzz = (v * rinv % MQ for v in (X, Y, ZZ, ZZZ))
    return (x * pow(zz, -1, MQ) % MQ, y * pow(zzz, -1, MQ) % MQ)


def _coords(ls):
    return [val(ls[9 * i:9 * i + 9]) for i in range(4)]


def _q29(pt):
    """the madd operand: to29 of the canonical storage form = 32 x_st"""
    return limbs(32 * (pt[0] * (1 << 256) % MQ)) + limbs(32 * (pt[1] * (1 << 256) % MQ))


@pytest.fixture(scope="module")
def model():
    return F.check()


def test_xyzz29_madd_at_the_accumulation_fixpoint(run, model):
    """p's coordinates carry the largest multiple of M below the model's fixpoint (X near
    2^259.46, Y near 2^258.6), q is an affine point in to29 form (< 32 M)"""
    fix = model["madd_fixpoint"]
    rng = random.Random(5)
    pts = _points(48, 11)
    cases, want = [], []
    for i in range(0, 48, 2):
        p, q = pts[i], pts[i + 1]
        z = rng.randrange(1, MQ)
        cases.append(_xyzz(p, z, fix, rng, top=(i % 4 == 0)) + _q29(q))
        want.append(B.g1_add(p, q))
    # p == q (the doubling path), p == -q (the identity), p the identity
    for p in pts[:4]:
        z = rng.randrange(1, MQ)
        cases.append(_xyzz(p, z, fix, rng) + _q29(p))
        want.append(B.g1_add(p, p))
        cases.append(_xyzz(p, z, fix, rng) + _q29(B.g1_neg(p)))
        want.append(None)
        cases.append([0] * 36 + _q29(p))
        want.append(p)
    got = run([("madd", c) for c in cases])
    for c, w, o in zip(cases, want, got):
        assert _affine(o) == w
        if w is not None:
            assert all(l < N29 for k in range(4) for l in o[9 * k:9 * k + 8])
    # outputs of the non-special cases stay inside the model's fixpoint bounds
    for o in got[:24]:
        for v, bd in zip(_coords(o), fix):
            assert v < bd, (v.bit_length(), bd.bit_length())


def test_xyzz29_madd_chain_stays_in_bounds(run, model):
    """the kernel's data flow: 300 mixed additions into one accumulator, every output fed
    back in; bounds checked after every step, the sum against the affine group law"""
    fix = model["madd_fixpoint"]
    pts = _points(300, 13)
    acc = [0] * 36
    ref = None
    for q in pts:
        acc = run([("madd", acc + _q29(q))])[0]
        ref = B.g1_add(ref, q)
        for v, bd in zip(_coords(acc), fix):
            assert v < bd
    assert _affine(acc) == ref


def _small_z(pt, rng, frac):
    """a z for which all four XYZZ coordinates of pt are below frac M (so that adding M
    puts each near the back-end class bound)"""
    x, y = pt
    while True:
        z = rng.randrange(1, MQ)
        zz, zzz = z * z % MQ, z * z * z % MQ
        es = [_mont(x * zz % MQ), _mont(y * zzz % MQ), _mont(zz), _mont(zzz)]
        if all(e < frac * MQ for e in es):
            return z


def test_xyzz29_add_dbl_at_the_back_end_class_bound(run, model):
    """coordinates near 1.2 M (an element below 0.2 M plus M): outputs stay in the class
    (the model's bound) and match the group law; identity, p + p and p + (-p) too"""
    C = int(1.2 * MQ)
    rng = random.Random(7)
    pts = _points(24, 17)
    cases, want = [], []
    for i in range(0, 24, 2):
        p, q = pts[i], pts[i + 1]
        zp = _small_z(p, rng, 0.2) if i < 6 else rng.randrange(1, MQ)
        zq = _small_z(q, rng, 0.2) if i < 6 else rng.randrange(1, MQ)
        P29, Q29 = _xyzz(p, zp, [C] * 4, rng), _xyzz(q, zq, [C] * 4, rng)
        if i < 6:
            assert all(v > MQ for v in _coords(P29) + _coords(Q29))
        cases += [("add", P29 + Q29), ("dbl", P29), ("add", P29 + P29), ("add", P29 + _xyzz(B.g1_neg(p), zq, [C] * 4, rng)),
                  ("add", P29 + [0] * 36), ("add", [0] * 36 + Q29), ("dbl", [0] * 36)]
        want += [B.g1_add(p, q), B.g1_add(p, p), B.g1_add(p, p), None, p, q, None]
    got = run(cases)
    for j, ((op, c), w, o) in enumerate(zip(cases, want, got)):
        assert _affine(o) == w, op
        # a sum or a doubling lands below the model's output bound; an identity operand
        # hands the other point back unchanged (< C)
        bound = C if j % 7 in (4, 5) else model["backend_out"] + 1
        if w is not None:
            for v in _coords(o):
                assert v < bound, (op, j % 7, v / MQ)


def test_xyzz29_back_end_chain_closed(run, model):
    """200 additions and doublings with every output fed back (the bucket reduction's
    data flow): the class bound holds at every step"""
    C = int(1.2 * MQ)
    rng = random.Random(9)
    pts = _points(100, 19)
    acc_ref = pts[0]
    acc = _xyzz(pts[0], _small_z(pts[0], rng, 0.2), [C] * 4, rng)
    for q in pts[1:]:
        acc = run([("add", acc + _xyzz(q, rng.randrange(1, MQ), [C] * 4, rng))])[0]
        acc = run([("dbl", acc)])[0]
        acc_ref = B.g1_add(B.g1_add(acc_ref, q), B.g1_add(acc_ref, q))
        for v in _coords(acc):
            assert v < C
    assert _affine(acc) == acc_ref
