"""BN254 optimal ate pairing in Python ints (TEST INFRASTRUCTURE ONLY).

The verifier's last step, DualMSM::check (halo2_backend/src/poly/kzg/msm.rs, via
VerifierSHPLONK / VerifierGWC, kzg/multiopen/*/verifier.rs), is the pairing equation
e(left, [s]G2) == e(right, G2).  With this module oracle/py/verifier.py decides it from
the params' G2 elements alone, as the reference does, instead of from the secret s.

Tower: Fq2 = Fq[i] / (i^2 + 1), Fq12 = Fq2[w] / (w^6 - xi), xi = 9 + i; G2 lives on the
D-type twist y^2 = x^3 + 3 / xi (bn254_ref.G2_B) and maps into E(Fq12) as
(x w^2, y w^3).  Miller loop over 6u + 2 (u = 0x44e992b44a6909f1) with the two
Frobenius-twisted extra lines, then the full final exponentiation (p^12 - 1) / r.
Pinned by bilinearity, non-degeneracy and order r (tests/test_pairing_ref.py); any
error in the tower, the lines or the loop breaks bilinearity.
"""
from bn254_ref import G2_GEN, P, R, fq2_add, fq2_inv, fq2_mul, fq2_sub

XI = (9, 1)
ATE_LOOP = 29793968203157093288  # 6u + 2


def fq2_conj(a):
    return (a[0], (-a[1]) % P)


def fq2_pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = fq2_mul(r, a)
        a = fq2_mul(a, a)
        e >>= 1
    return r


def fq2_scale(a, k):
    return (a[0] * k % P, a[1] * k % P)


# ------------------------------------------------------------------ Fq12 = Fq2[w]/(w^6 - xi)
ONE12 = [(1, 0)] + [(0, 0)] * 5


def f12_mul(a, b):
    t = [(0, 0)] * 11
    for i in range(6):
        if a[i] == (0, 0):
            continue
        for j in range(6):
            if b[j] == (0, 0):
                continue
            t[i + j] = fq2_add(t[i + j], fq2_mul(a[i], b[j]))
    return [fq2_add(t[k], fq2_mul(t[k + 6], XI)) if k + 6 < 11 else t[k] for k in range(6)]


def f12_pow(a, e):
    r = ONE12
    while e:
        if e & 1:
            r = f12_mul(r, a)
        a = f12_mul(a, a)
        e >>= 1
    return r


def f12_is_one(a):
    return a[0] == (1, 0) and all(c == (0, 0) for c in a[1:])


# ------------------------------------------------------------------ Miller loop
def _line(t, q, p):
    """the line through twisted points t, q (or the tangent at t) at the G1 point p, and
    t + q; in E(Fq12) coordinates the slope is lam * w with lam in Fq2:
    l = -yp + (lam xp) w + (yt - lam xt) w^3"""
    (xt, yt), (xq, yq) = t, q
    if xt == xq and yt == yq:
        lam = fq2_mul(fq2_scale(fq2_mul(xt, xt), 3), fq2_inv(fq2_scale(yt, 2)))
    elif xt == xq:
        raise ValueError("vertical line in the Miller loop (points not in the r-torsion)")
    else:
        lam = fq2_mul(fq2_sub(yq, yt), fq2_inv(fq2_sub(xq, xt)))
    xp, yp = p
    line = [((-yp) % P, 0), fq2_scale(lam, xp), (0, 0), fq2_sub(yt, fq2_mul(lam, xt)), (0, 0), (0, 0)]
    # t + q on the twist: x3 = lam^2 xi^-1 ... in twisted coordinates the slope is lam w, so
    # x3' w^2 = (lam w)^2 - (xt + xq) w^2  ->  x3' = lam^2 - xt - xq (w^2 cancels)
    x3 = fq2_sub(fq2_sub(fq2_mul(lam, lam), xt), xq)
    # y3' w^3 = lam w (xt' w^2 - x3' w^2) - yt' w^3  ->  y3' = lam (xt - x3) - yt
    y3 = fq2_sub(fq2_mul(lam, fq2_sub(xt, x3)), yt)
    return line, (x3, y3)


_G2_FROB_X = fq2_pow(XI, (P - 1) // 3)
_G2_FROB_Y = fq2_pow(XI, (P - 1) // 2)


def _frob_twist(q):
    """the p-power Frobenius of E(Fq12) restricted to the twisted G2 image"""
    return fq2_mul(fq2_conj(q[0]), _G2_FROB_X), fq2_mul(fq2_conj(q[1]), _G2_FROB_Y)


def miller_loop(p, q):
    """p: G1 affine (x, y) ints or None; q: G2 affine ((x0, x1), (y0, y1)) or None"""
    if p is None or q is None:
        return ONE12
    f = ONE12
    t = q
    for i in range(ATE_LOOP.bit_length() - 2, -1, -1):
        ln, t = _line(t, t, p)
        f = f12_mul(f12_mul(f, f), ln)
        if (ATE_LOOP >> i) & 1:
            ln, t = _line(t, q, p)
            f = f12_mul(f, ln)
    q1 = _frob_twist(q)
    q2 = _frob_twist(q1)
    nq2 = (q2[0], ((-q2[1][0]) % P, (-q2[1][1]) % P))
    ln, t = _line(t, q1, p)
    f = f12_mul(f, ln)
    ln, _ = _line(t, nq2, p)
    return f12_mul(f, ln)


FINAL_EXP = (P ** 12 - 1) // R


def final_exponentiation(f):
    return f12_pow(f, FINAL_EXP)


def pairing(p, q):
    return final_exponentiation(miller_loop(p, q))


def pairing_check(pairs):
    """prod_i e(p_i, q_i) == 1 (one final exponentiation)"""
    f = ONE12
    for p, q in pairs:
        f = f12_mul(f, miller_loop(p, q))
    return f12_is_one(final_exponentiation(f))


G2 = G2_GEN
