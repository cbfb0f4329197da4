#!/usr/bin/env python3
"""Value bounds of the F29 lazy reduction (csrc/f29.h and its users), checked.

The subtraction constants are read from the sources, not restated: every
`sub29<P, K, OFF>` the kernels instantiate (f29.h's XYZZ formulas, msm.hip's quad
variants, ntt.hip's stage subtraction and sparse first pass, prover_kernels.hip's
evaluate_h helpers) and is_zero29's early-out threshold are parsed
(`source_constants`) and the model below runs on exactly those numbers.  `EXPECTED` is
the snapshot this model was last reviewed against; tests/test_f29_bounds_cpu.py fails
when the sources drift from it (any edit of a K, OFF or the threshold) and when the
model rejects the sources' constants.

Every quantity is tracked as an integer upper bound; a Montgomery product (R = 2^261) of
x < A and y < B is < A B / R + M.  Starting from each state the accumulation can begin in
(a fresh point: X, Y < 32 M, ZZ = ZZZ = one < M; the doubling path: all four < 32 M) the
madd map is iterated to its fixpoint, and at every step the model asserts what the
kernel relies on:
  * each subtraction a - b + k M has k M > b with a top-limb margin (kmul_safe's borrow of
    1 (offset 29) or 4 (offset 31) from the top limb: the top limb of k M minus it still
    covers b's top limb), and b's low limbs are below 2^OFF, so no limb goes negative;
  * every value stays below 2^261 (normalised 29-bit limbs, top limb < 2^29);
  * every product's column sums stay below 2^64 (limb bounds of the operands);
  * every value is_zero29 tests is below (T + 1) M, T its early-out threshold, so a
    multiple of M it holds is k M with k <= T and the early-out never hides a zero.
    python tools/f29_bounds.py
"""
import math
import os
import re

M = 0x30644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd47  # BN254 Fq
MR = 0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001  # BN254 Fr
R = 2 ** 261
LG = math.log2
N29 = 1 << 29

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "yet-another-halo2-fork_amd", "csrc")
SOURCES = ("f29.h", "msm.hip", "ntt.hip", "prover_kernels.hip")

# the constants this model was last reviewed against ("file:function": [(K, OFF), ...] in
# source order; K as written, e.g. ntt.hip's stage expression)
EXPECTED = {
    "f29.h:xyzz29_madd": [("64", "29"), ("64", "29"), ("32", "31"), ("64", "29"), ("16", "29")],
    "f29.h:xyzz29_dbl": [("4", "31"), ("4", "29"), ("2", "29")],
    "f29.h:xyzz29_add": [("2", "29"), ("2", "29"), ("4", "31"), ("4", "29"), ("2", "29")],
    "msm.hip:xyzz29_dbl_q4": [("4", "31"), ("4", "29"), ("2", "29")],
    "msm.hip:xyzz29_add_q4": [("2", "29"), ("2", "29"), ("4", "31"), ("4", "29"), ("2", "29")],
    "ntt.hip:nsub29": [("(4u << S)", "29")],
    "ntt.hip:ntt_first_sparse29_kernel": [("4", "29")],
    "prover_kernels.hip:eh_sub": [("64", "29")],
    "prover_kernels.hip:eh_subn": [("64", "29")],
    "is_zero29": 1024,
}

_SUB = re.compile(r"\bsub29<\s*\w+\s*,\s*(\([^()]*\)|[^,<>]+?)\s*,\s*(\d+)\s*>")
_FUNC = re.compile(r"([A-Za-z_]\w*)\s*\(")
_NOT_FUNC = {"__launch_bounds__", "if", "for", "while", "switch", "return", "sizeof", "static_assert", "defined"}


def _enclosing_functions(text):
    """(line start offset, function name) for every line that begins a top-level definition"""
    out, pos = [], 0
    for line in text.splitlines(keepends=True):
        if line[:1].isalpha() or line[:1] == "_":
            if not line.startswith(("template", "struct", "static constexpr", "using", "namespace", "typedef")):
                for m in _FUNC.finditer(line):
                    if m.group(1) not in _NOT_FUNC:
                        out.append((pos, m.group(1)))
                        break
        pos += len(line)
    return out


def source_constants(texts=None):
    """{"file:function": [(K, OFF), ...]} for every sub29<P, K, OFF> outside comments, and
    "is_zero29": the threshold of its early-out.  `texts` ({file: text}) replaces the
    files on disk (the mutation tests)."""
    texts = texts or {}
    found = {}
    for fn in SOURCES:
        text = texts.get(fn)
        if text is None:
            with open(os.path.join(CSRC, fn)) as f:
                text = f.read()
        code = re.sub(r"//[^\n]*", lambda m: " " * len(m.group(0)), text)  # keep offsets
        funcs = _enclosing_functions(code)
        for m in _SUB.finditer(code):
            name = None
            for start, nm in funcs:
                if start > m.start():
                    break
                name = nm
            found.setdefault(f"{fn}:{name}", []).append((m.group(1).strip(), m.group(2)))
        if fn == "f29.h":
            z = re.search(r"is_zero29\(const F29& a\)\s*\{.*?if \(k > (\d+)\) return false;", code, re.S)
            assert z, "is_zero29's early-out not found in f29.h"
            found["is_zero29"] = int(z.group(1))
    return found


def k_of(expr, s=None):
    """the integer K of a parsed constant (ntt.hip's stage form "(4u << S)" at stage s)"""
    e = expr.replace("u", "")
    if "S" in e:
        assert s is not None, expr
        e = e.replace("S", str(s))
    assert re.fullmatch(r"[\d\s()<+*-]+", e), expr
    return int(eval(e))  # digits and shifts only (checked above)


def top(v):
    return v >> 232


def mul(a, b):
    return a * b // R + M + 1


def sub_ok(b, k, off, b_limb=N29, m=M):
    """a - b + k M limb-wise: b's limbs 0..7 (< b_limb) below 2^OFF, and the top limb of
    k M minus the borrow covers b's top limb"""
    unit = 1 << (off - 29)
    assert b_limb <= 1 << off, ("sub29 low limbs of b above 2^OFF", k, off)
    assert top(k * m) - unit >= top(b), ("sub29 K too small", k, off, LG(b), LG(k * m))


def sub_limb(off, a_limb=N29):
    """limb bound of a sub29<K, OFF> result before norm29: a_i + (k M)_i + 2^OFF"""
    return a_limb + N29 + (1 << off)


def column_ok(la, lb, lc=0, ld=0):
    """max column sum of REDC(a b [+ c d]) with limb bounds la, lb (lc, ld), m M < 2^58"""
    s = 9 * la * lb + 9 * lc * ld + 9 * (1 << 58) + (1 << 35)
    assert s < 1 << 64, LG(s)


def iszero_ok(v, thr, m=M):
    """is_zero29 on a value < v: a multiple of M there is k M with k <= thr"""
    assert v <= (thr + 1) * m, ("is_zero29 input may exceed its early-out", LG(v), thr)


def madd(st, xq, yq, ks, thr):
    """xyzz29_madd (f29.h) on bounds; ks: its five sub29 constants in source order"""
    (k0, o0), (k1, o1), (k2, o2), (k3, o3), (k4, o4) = [(k_of(k), int(o)) for k, o in ks]
    X, Y, ZZ, ZZZ = st
    U2, S2 = mul(xq, ZZ), mul(yq, ZZZ)
    sub_ok(X, k0, o0)
    sub_ok(Y, k1, o1)
    P, Rr = U2 + k0 * M, S2 + k1 * M
    iszero_ok(P, thr)
    iszero_ok(Rr, thr)
    PP, R2 = mul(P, P), mul(Rr, Rr)
    PPP, Q = mul(P, PP), mul(X, PP)
    T = PPP + 2 * Q
    sub_ok(T, k2, o2, b_limb=3 * (N29 - 1))  # add29(add29(PPP, Q), Q): unnormalised
    X3 = R2 + k2 * M
    sub_ok(X3, k3, o3)
    D = Q + k3 * M
    sub_ok(PPP, k4, o4)
    E = k4 * M
    column_ok(N29, N29)  # normalised operands
    column_ok(N29, sub_limb(o3), N29, sub_limb(o4, a_limb=0))  # R (Q - X3 + K M) + Y (K M - PPP)
    Y3 = (Rr * D + Y * E) // R + M + 1
    ZZ3, ZZZ3 = mul(ZZ, PP), mul(ZZZ, PPP)
    inter = dict(U2=U2, S2=S2, P=P, R=Rr, PP=PP, PPP=PPP, Q=Q, R2=R2, X3=X3, D=D, E=E, Y3=Y3)
    for k, v in inter.items():
        assert v < 1 << 261, (k, LG(v))
    return (X3, Y3, ZZ3, ZZZ3), inter


def madd_fixpoint(st, ks, thr):
    xq = yq = 32 * M
    worst = 0
    for _ in range(60):
        nxt, inter = madd(st, xq, yq, ks, thr)
        worst = max(worst, *nxt, *inter.values())
        st = tuple(max(a, b) for a, b in zip(st, nxt))  # bounds only grow
    return st, worst


def reduce29(vmax, m=M):
    """bound of csrc/f29.h reduce29(v) over v < vmax: v - q M with q = floor(v_8 / (M_8 + 1))
    is >= 0 and < M + (q + 2) 2^232"""
    q = top(vmax) // (top(m) + 1)
    return m + (q + 2) * (1 << 232)


def backend_class(C, add_ks, dbl_ks, thr):
    """the MSM back-end's class (every coordinate < C): closed under xyzz29_add / xyzz29_dbl
    (and their quad-cooperative forms in msm.hip) with the given sub29 constants"""
    (a0, p0), (a1, p1), (a2, p2), (a3, p3), (a4, p4) = [(k_of(k), int(o)) for k, o in add_ks]
    (d0, q0), (d1, q1), (d2, q2) = [(k_of(k), int(o)) for k, o in dbl_ks]
    # add-2008-s
    U = mul(C, C)
    sub_ok(U, a0, p0)
    sub_ok(U, a1, p1)
    P = U + max(a0, a1) * M
    iszero_ok(P, thr)
    PP = mul(P, P)
    PPP, Q = mul(P, PP), mul(U, PP)
    sub_ok(PPP + 2 * Q, a2, p2, b_limb=3 * (N29 - 1))
    X3 = reduce29(mul(P, P) + a2 * M)
    sub_ok(X3, a3, p3)
    sub_ok(PPP, a4, p4)
    column_ok(N29, sub_limb(p3), N29, sub_limb(p4, a_limb=0))
    Y3 = (P * (Q + a3 * M) + U * a4 * M) // R + M + 1
    ZZ3 = mul(mul(C, C), PP)
    out_add = (X3, Y3, ZZ3, mul(mul(C, C), PPP))
    # dbl-2008-s-1
    Uy = 2 * C
    V = mul(Uy, Uy)
    W, S, X2 = mul(Uy, V), mul(C, V), mul(C, C)
    Mm = 3 * X2
    sub_ok(2 * S, d0, q0, b_limb=2 * (N29 - 1))
    X3d = reduce29(mul(Mm, Mm) + d0 * M)
    sub_ok(X3d, d1, q1)
    sub_ok(W, d2, q2)
    column_ok(N29, sub_limb(q1), N29, sub_limb(q2, a_limb=0))
    Y3d = (Mm * (S + d1 * M) + C * d2 * M) // R + M + 1
    out_dbl = (X3d, Y3d, mul(V, C), mul(W, C))
    for v in out_add + out_dbl:
        assert v < C, (LG(v), LG(C))
    return max(out_add + out_dbl)


def ntt_pass(stages, b0, kexpr, off, tw=MR):
    """one NTT pass in F29 (csrc/ntt.hip ntt_pass29_kernel / ntt_last29_kernel): inputs <
    b0; stage s: sums a + b, differences a - b + K_s M (nsub29<S>) into a product with a
    twiddle < M, or kept (normalised) for the j = 0 butterflies; closing product with a
    constant < M.  Returns the bound of the pass's outputs."""
    B = b0
    for s in range(stages):
        k = k_of(kexpr, s)
        sub_ok(B, k, off, m=MR)
        B = max(2 * B, B + k * MR)        # sums; kept differences
        # a product's operand: limbs 0..7 < 2^29 + 2^30, the twiddle normalised
        column_ok(N29, sub_limb(off))
    assert top(B) < 1 << 31, LG(B)         # top limb of a normalised value fits its 32 bits
    return B * tw // R + MR + 1


def check(consts=None, verbose=False):
    """run the whole model on `consts` (default: parsed from the sources); AssertionError
    names the first violated bound"""
    c = consts if consts is not None else source_constants()
    say = print if verbose else (lambda *a, **k: None)
    thr = c["is_zero29"]
    madd_ks = c["f29.h:xyzz29_madd"]
    fx, w1 = madd_fixpoint((32 * M, 32 * M, M, M), madd_ks, thr)
    say(f"fresh point: fixpoint log2 X Y ZZ ZZZ = {[round(LG(v), 3) for v in fx]}, largest intermediate 2^{LG(w1):.3f}")
    d = mul(32 * M, M)
    fd, w2 = madd_fixpoint((d, d, d, d), madd_ks, thr)
    say(f"doubling path: fixpoint log2 X Y ZZ ZZZ = {[round(LG(v), 3) for v in fd]}, largest intermediate 2^{LG(w2):.3f}")
    acc_max = max(fx + fd)
    assert acc_max < 1 << 260
    assert reduce29(1 << 260) < 1.001 * M
    bworst = 0
    for add_key, dbl_key in (("f29.h:xyzz29_add", "f29.h:xyzz29_dbl"), ("msm.hip:xyzz29_add_q4", "msm.hip:xyzz29_dbl_q4")):
        bworst = max(bworst, backend_class(int(1.2 * M), c[add_key], c[dbl_key], thr))
    say(f"back-end class: coordinates < 1.2 M closed under add and dbl (outputs < {bworst / M:.3f} M); "
        f"reduce29 of an accumulator < 2^260 gives < {reduce29(1 << 260) / M:.4f} M")
    (nk, no), = c["ntt.hip:nsub29"]
    no = int(no)
    b0 = 3 * MR  # stored values of the NTT passes
    for st in (3, 4, 5, 6):
        out = ntt_pass(st, b0, nk, no)
        assert out < b0 and out < 1 << 256, (st, out / MR)
        say(f"ntt pass of {st} stages: inputs < 3 M, outputs < {out / MR:.3f} M (packable, below the input bound)")
    say(f"last pass: outputs < {ntt_pass(6, b0, nk, no) / MR:.3f} M before two conditional subtractions of M")
    # the last pass without an epilogue product (ntt_last29_kernel ONE): reduce29 of the
    # stage outputs, then one conditional subtraction, must land below 2 M
    Bl = b0
    for s_ in range(6):
        Bl = max(2 * Bl, Bl + k_of(nk, s_) * MR)
    ql = top(Bl) // (top(MR) + 1)
    red = MR + (ql + 2) * (1 << 232)
    assert red < 2 * MR and top(Bl) < 1 << 32, (LG(Bl), red / MR)
    say(f"last pass without a product: stage outputs < {Bl / MR:.0f} M, reduce29 -> < {red / MR:.6f} M")
    # the sparse first pass (ntt_first_sparse29_kernel): x0 < 1.01 M, p = x1 w < 1.01 M;
    # x0 - p + K M feeds the closing product with the pass twiddle
    (sk, so), = c["ntt.hip:ntt_first_sparse29_kernel"]
    sk, so = k_of(sk), int(so)
    pj = MR * MR // R + MR + 1
    sub_ok(pj, sk, so, m=MR)
    ys = MR * 101 // 100 + sk * MR
    column_ok(N29, sub_limb(so))
    out_sp = ys * MR // R + MR + 1
    assert out_sp < b0
    say(f"sparse first pass: outputs < {out_sp / MR:.3f} M")
    tw_live = MR * MR // R + MR + 1  # a twiddle formed in the pass: lo x hi, both < M (H2G_NTT_TW_LIVE)
    for st in (3, 4, 5, 6):
        out = ntt_pass(st, b0, nk, no, tw_live)
        assert out < b0 and out < 1 << 256, (st, out / MR)
    say(f"passes with twiddles formed in the pass (< {tw_live / MR:.4f} M): outputs < {ntt_pass(6, b0, nk, no, tw_live) / MR:.3f} M")
    # evaluate_h29_kernel's unreduced sums / differences (eh_addn / eh_add3n / eh_subn): each
    # feeds one product; loads < 32 M, constants < M, reduced values < 1.001 M, Horner
    # accumulators reduced after every step
    (ek, eo), = c["prover_kernels.hip:eh_subn"]
    assert c["prover_kernels.hip:eh_sub"] == c["prover_kernels.hip:eh_subn"]
    ek, eo = k_of(ek), int(eo)

    def prod(a, b):  # bound of REDC(a b) for a < aM, b < bM, in units of MR
        return a * b * MR // R + 1
    LD, C, RED = 32, 1, 1.001

    def sub_ok_fr(bm):  # a - b + K M: K M covers b's top limb
        sub_ok(int(bm * MR), ek, eo, m=MR)
    worst = 0
    # permutation block
    lo_hi = prod(LD, LD)
    cur = max(prod(C, prod(C, lo_hi)), prod(prod(C, lo_hi), C))
    add3 = LD + prod(C, LD) + C
    left = LD
    for _ in range(8):
        left = max(left, prod(left, add3))
    right = LD
    for _ in range(8):
        right = max(right, prod(right, LD + cur + C))
    sub_ok_fr(right)
    worst = max(worst, left + ek, ek + 1, prod(LD, LD) + ek, LD + ek)
    # lookup block
    tv = prod(RED + C, RED + C)
    a1 = prod(prod(LD, LD + C), LD + C)
    sub_ok_fr(prod(LD, tv))
    sub_ok_fr(LD)
    worst = max(worst, a1 + ek, LD + ek, prod(LD + ek, LD + ek))
    # shuffle block
    sub_ok_fr(prod(LD, RED + C))
    worst = max(worst, prod(LD, RED + C) + ek)
    assert worst * MR < 1 << 261, worst
    # every such operand times a load (< 32 M) -- the largest product input pairing
    assert prod(worst, LD) < 64, prod(worst, LD)
    say(f"evaluate_h unreduced operands < {worst:.1f} M (< 2^261), their products < {prod(worst, LD):.1f} M")
    # lincomb29_kernel: up to 6 pairs REDC(a c + b d) (a, b storage integers < M, c, d < M)
    # plus the accumulated storage value, then reduce29 + one subtraction
    pair = 2 * MR * MR // R + MR + 1
    tot = 6 * pair + MR
    column_ok(N29, N29, N29, N29)
    assert tot < 1 << 260
    qv = top(tot) // (top(MR) + 1)
    assert MR + (qv + 2) * (1 << 232) < 2 * MR
    say(f"lincomb: pairs < {pair / MR:.4f} M, sum < {tot / MR:.2f} M, reduced below 2 M before the subtraction")
    # H2G_HORNER29 (eval_level1, kate_phase1/3): acc <- REDC(acc x) + a with x < M and a
    # storage integer a < 2^256; kate_phase3 (ACC) adds one more stored value before reducing
    h = 0
    for _ in range(200):
        h = max(h, h * MR // R + MR + 1 + (1 << 256))
    column_ok(1 << 30, N29)  # acc: a limb-wise add of two normalised values
    stored = h + (1 << 256)
    assert stored < 1 << 260
    qh = top(stored) // (top(MR) + 1)
    assert MR + (qh + 2) * (1 << 232) < 2 * MR
    say(f"Horner chains: accumulator < {h / MR:.2f} M, stored sums < {stored / MR:.2f} M, reduced below 2 M")
    return {"madd_fixpoint": tuple(max(a, b) for a, b in zip(fx, fd)), "madd_intermediate": max(w1, w2),
            "backend_out": bworst}


def main():
    c = source_constants()
    if c != EXPECTED:
        print("WARNING: the sources' constants differ from EXPECTED (the reviewed snapshot):")
        for k in sorted(set(c) | set(EXPECTED)):
            if c.get(k) != EXPECTED.get(k):
                print(f"  {k}: sources {c.get(k)} snapshot {EXPECTED.get(k)}")
    check(c, verbose=True)
    print("ok")


if __name__ == "__main__":
    main()
