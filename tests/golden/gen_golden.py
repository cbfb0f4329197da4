#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ from the Python
big-integer oracle (oracle/py/bn254_ref.py).  Run once in the build container:

    python tests/golden/gen_golden.py

The fixtures are data only (uint64 limb arrays, Montgomery form, halo2curves'
in-memory layout) and are loaded with numpy.load(allow_pickle=False).
Inputs are drawn from a seeded random.Random, so the files are reproducible.
"""
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))
import bn254_ref as B  # noqa: E402


def fr_arr(vals):
    return np.array([B.fr_mont_limbs(v) for v in vals], dtype=np.uint64).reshape(-1, 4)


def pt_arr(pts):
    return np.array([B.g1_affine_mont_limbs(p) for p in pts], dtype=np.uint64).reshape(-1, 8)


def gen_msm(rng):
    out = {}
    s = rng.randrange(1, B.R)
    srs = B.srs_powers(s, 1 << 10)
    rand_pts = [B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)) for _ in range(64)]
    cases = []
    for k in (0, 1, 3, 5, 8, 10):
        n = 1 << k
        cases.append((f"srs_random_k{k}", [rng.randrange(B.R) for _ in range(n)], srs[:n]))
    n = 256
    cases += [
        ("zeros", [0] * n, srs[:n]),
        ("ones", [1] * n, srs[:n]),
        ("small64", [rng.randrange(1 << 64) for _ in range(n)], srs[:n]),
        ("r_minus_1", [B.R - 1] * n, srs[:n]),
        ("half_zero", [rng.randrange(B.R) if i % 2 else 0 for i in range(n)], srs[:n]),
        ("same_scalar", [0xDEADBEEF12345] * n, srs[:n]),
        ("repeated_point", [rng.randrange(B.R) for _ in range(64)], [rand_pts[0]] * 64),
        ("with_identity_bases", [rng.randrange(B.R) for _ in range(64)],
         [None if i % 5 == 0 else rand_pts[i] for i in range(64)]),
        ("cancel_to_identity", [3, B.R - 3], [rand_pts[1], rand_pts[1]]),
        ("top_bits", [(B.R - 1) - rng.randrange(1 << 200) for _ in range(128)], srs[:128]),
        ("sparse_high", [1 << rng.randrange(253) for _ in range(128)], srs[:128]),
    ]
    names = []
    for name, sc, pts in cases:
        res = B.msm_naive(sc, pts)
        out[f"{name}__scalars"] = fr_arr(sc)
        out[f"{name}__bases"] = pt_arr(pts)
        out[f"{name}__result"] = pt_arr([res])[0]
        out[f"{name}__is_identity"] = np.array([1 if res is None else 0], dtype=np.uint64)
        names.append(name)
        print("msm", name, len(sc), "identity" if res is None else "ok")
    out["__names"] = np.array(names)
    out["srs_s"] = fr_arr([s])[0]
    np.savez_compressed(os.path.join(HERE, "msm_golden.npz"), **out)


def gen_ntt(rng):
    out = {}
    names = []
    for k in range(0, 11):
        n = 1 << k
        a = [rng.randrange(B.R) for _ in range(n)]
        w = B.omega_for(k)
        name = f"k{k}"
        out[f"{name}__input"] = fr_arr(a)
        out[f"{name}__omega"] = fr_arr([w])[0]
        out[f"{name}__fft"] = fr_arr(B.fft(a, w) if k > 6 else B.dft(a, w))
        names.append(name)
    out["__names"] = np.array(names)
    # domain operations (domain.rs) for j in {3, 5} -> ext = 2n, 4n
    dnames = []
    for (j, k) in ((3, 2), (3, 5), (3, 8), (5, 4), (5, 7), (9, 5)):
        d = B.Domain(j, k)
        name = f"j{j}_k{k}"
        lag = [rng.randrange(B.R) for _ in range(d.n)]
        coeff = d.lagrange_to_coeff(lag)
        ext = d.coeff_to_extended(coeff)
        ext_in = [rng.randrange(B.R) for _ in range(d.extended_len)]
        out[f"{name}__lagrange"] = fr_arr(lag)
        out[f"{name}__coeff"] = fr_arr(coeff)
        out[f"{name}__extended"] = fr_arr(ext)
        out[f"{name}__ext_in"] = fr_arr(ext_in)
        out[f"{name}__divided"] = fr_arr(d.divide_by_vanishing_poly(ext_in))
        out[f"{name}__ext_to_coeff"] = fr_arr(d.extended_to_coeff(ext_in))
        out[f"{name}__roundtrip"] = fr_arr(d.extended_to_coeff(ext))  # == coeff padded
        out[f"{name}__t_evaluations"] = fr_arr(d.t_evaluations)
        out[f"{name}__consts"] = fr_arr([d.omega, d.omega_inv, d.extended_omega, d.extended_omega_inv,
                                         d.g_coset, d.g_coset_inv, d.ifft_divisor,
                                         d.extended_ifft_divisor, d.barycentric_weight])
        out[f"{name}__meta"] = np.array([j, k, d.extended_k], dtype=np.uint64)
        dnames.append(name)
        print("domain", name, d.n, d.extended_len)
    out["__domains"] = np.array(dnames)
    np.savez_compressed(os.path.join(HERE, "ntt_golden.npz"), **out)


def gen_poly(rng):
    out = {}
    names = []
    for n in (1, 2, 7, 64, 1000):
        a = [rng.randrange(B.R) for _ in range(n)]
        b = [rng.randrange(B.R) for _ in range(n)]
        x = rng.randrange(B.R)
        name = f"n{n}"
        out[f"{name}__a"] = fr_arr(a)
        out[f"{name}__b"] = fr_arr(b)
        out[f"{name}__x"] = fr_arr([x])[0]
        out[f"{name}__add"] = fr_arr([(u + v) % B.R for u, v in zip(a, b)])
        out[f"{name}__sub"] = fr_arr([(u - v) % B.R for u, v in zip(a, b)])
        out[f"{name}__mul"] = fr_arr([(u * v) % B.R for u, v in zip(a, b)])
        out[f"{name}__scale"] = fr_arr([(u * x) % B.R for u in a])
        out[f"{name}__eval"] = fr_arr([B.eval_polynomial(a, x)])[0]
        out[f"{name}__inv"] = fr_arr([pow(u, -1, B.R) if u else 0 for u in a])
        pp = []
        acc = 1
        for u in a:
            acc = acc * u % B.R
            pp.append(acc)
        out[f"{name}__prefix_product"] = fr_arr(pp)
        if n > 1:
            # a(X) - a(x) is divisible by (X - x)
            a2 = list(a)
            a2[0] = (a2[0] - B.eval_polynomial(a, x)) % B.R
            out[f"{name}__kate_in"] = fr_arr(a2)
            out[f"{name}__kate_q"] = fr_arr(B.kate_division(a2, x))
        names.append(name)
    out["__names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "poly_golden.npz"), **out)


if __name__ == "__main__":
    gen_poly(random.Random(0x505))
    gen_ntt(random.Random(0x177))
    gen_msm(random.Random(0x3553))
