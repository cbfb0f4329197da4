#!/usr/bin/env python3
"""Value bounds of the F29 XYZZ mixed addition (csrc/f29.h xyzz29_madd), checked.

Every quantity is tracked as an integer upper bound; a Montgomery product (R = 2^261) of
x < A and y < B is < A B / R + M.  Starting from each state the accumulation can begin in
(a fresh point: X, Y < 32 M, ZZ = ZZZ = one < M; the doubling path: all four < 32 M) the
madd map is iterated to its fixpoint, and at every step the script asserts what the
kernel relies on:
  * each subtraction a - b + k M has k M > b with a top-limb margin (kmul_safe's borrow of
    1 (offset 29) or 4 (offset 31) from the top limb: the top limb of k M minus it still
    covers b's top limb), so no limb goes negative;
  * every value stays below 2^261 (normalised 29-bit limbs, top limb < 2^29);
  * every product's column sums stay below 2^64 (limb bounds of the operands).
    python tools/f29_bounds.py
"""
import math

M = 0x30644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd47  # BN254 Fq
R = 2 ** 261
LG = math.log2


def top(v):
    return v >> 232


def mul(a, b):
    return a * b // R + M + 1


def sub_ok(b, k, off):
    """a - b + k M limb-wise: the top limb of k M minus the borrow must cover b's top limb"""
    unit = 1 << (off - 29)
    assert top(k * M) - unit >= top(b), (k, off, LG(b), LG(k * M))


def column_ok(la, lb, lc=0, ld=0):
    """max column sum of REDC(a b [+ c d]) with limb bounds la, lb (lc, ld), m M < 2^58"""
    s = 9 * la * lb + 9 * lc * ld + 9 * (1 << 58) + (1 << 35)
    assert s < 1 << 64, LG(s)


def madd(st, xq, yq):
    X, Y, ZZ, ZZZ = st
    n29 = 1 << 29
    U2, S2 = mul(xq, ZZ), mul(yq, ZZZ)
    sub_ok(X, 64, 29)
    sub_ok(Y, 64, 29)
    P, Rr = U2 + 64 * M, S2 + 64 * M
    PP, R2 = mul(P, P), mul(Rr, Rr)
    PPP, Q = mul(P, PP), mul(X, PP)
    T = PPP + 2 * Q
    sub_ok(T, 32, 31)
    X3 = R2 + 32 * M
    sub_ok(X3, 64, 29)
    D = Q + 64 * M
    sub_ok(PPP, 16, 29)
    E = 16 * M
    column_ok(n29, n29)                                  # normalised operands
    column_ok(n29, n29 + (1 << 30), n29, 1 << 30)        # R (Q - X3 + 64M) + Y (16M - PPP)
    Y3 = (Rr * D + Y * E) // R + M + 1
    ZZ3, ZZZ3 = mul(ZZ, PP), mul(ZZZ, PPP)
    inter = dict(U2=U2, S2=S2, P=P, R=Rr, PP=PP, PPP=PPP, Q=Q, R2=R2, X3=X3, D=D, E=E, Y3=Y3)
    for k, v in inter.items():
        assert v < 1 << 261, (k, LG(v))
    return (X3, Y3, ZZ3, ZZZ3), inter


def run(name, st):
    xq = yq = 32 * M
    worst = 0
    for _ in range(60):
        nxt, inter = madd(st, xq, yq)
        worst = max(worst, *nxt, *inter.values())
        st = tuple(max(a, b) for a, b in zip(st, nxt))  # bounds only grow
    print(f"{name}: fixpoint log2 X Y ZZ ZZZ = {[round(LG(v), 3) for v in st]}, "
          f"largest intermediate 2^{LG(worst):.3f}")


def reduce29(vmax):
    """bound of csrc/f29.h reduce29(v) over v < vmax: v - q M with q = floor(v_8 / (M_8 + 1))
    is >= 0 and < M + (q + 2) 2^232"""
    q = top(vmax) // (top(M) + 1)
    return M + (q + 2) * (1 << 232)


def backend_class(C):
    """the MSM back-end's class (every coordinate < C): closed under xyzz29_add / xyzz29_dbl"""
    n29, n30 = 1 << 29, 1 << 30
    # add-2008-s
    U = mul(C, C)
    sub_ok(U, 2, 29)
    P = U + 2 * M
    PP = mul(P, P)
    PPP, Q = mul(P, PP), mul(U, PP)
    sub_ok(PPP + 2 * Q, 4, 31)
    X3 = reduce29(mul(P, P) + 4 * M)
    sub_ok(X3, 4, 29)
    sub_ok(PPP, 2, 29)
    column_ok(n29, n29 + n30, n29, n30)
    Y3 = (P * (Q + 4 * M) + U * 2 * M) // R + M + 1
    ZZ3 = mul(mul(C, C), PP)
    out_add = (X3, Y3, ZZ3, mul(mul(C, C), PPP))
    # dbl-2008-s-1
    Uy = 2 * C
    V = mul(Uy, Uy)
    W, S, X2 = mul(Uy, V), mul(C, V), mul(C, C)
    Mm = 3 * X2
    sub_ok(2 * S, 4, 31)
    X3d = reduce29(mul(Mm, Mm) + 4 * M)
    sub_ok(X3d, 4, 29)
    sub_ok(W, 2, 29)
    Y3d = (Mm * (S + 4 * M) + C * 2 * M) // R + M + 1
    out_dbl = (X3d, Y3d, mul(V, C), mul(W, C))
    for v in out_add + out_dbl:
        assert v < C, (LG(v), LG(C))
    return max(out_add + out_dbl)


MR = 0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001  # BN254 Fr


def ntt_pass(stages, b0, tw=MR):
    """one NTT pass in F29 (csrc/ntt.hip ntt_pass29_kernel / ntt_last29_kernel): inputs <
    b0; stage s: sums a + b, differences a - b + K_s M with K_s = 2^(s+2) into a product
    with a twiddle < M, or kept (normalised) for the j = 0 butterflies; closing product
    with a constant < M.  Returns the bound of the pass's outputs."""
    B = b0
    for s in range(stages):
        k = 4 << s
        assert top(k * MR) - 1 >= top(B), ("NTT K_s too small", s, LG(B), LG(k * MR))
        B = max(2 * B, B + k * MR)        # sums; kept differences
        # a product's operand: limbs 0..7 < 2^29 + 2^30, the twiddle normalised
        column_ok(1 << 29, (1 << 29) + (1 << 30))
    assert top(B) < 1 << 31, LG(B)         # top limb of a normalised value fits its 32 bits
    return B * tw // R + MR + 1


if __name__ == "__main__":
    run("fresh point", (32 * M, 32 * M, M, M))
    d = mul(32 * M, M)
    run("doubling path", (d, d, d, d))
    acc_max = (1 << 260)  # above every accumulation output (fixpoints above)
    assert reduce29(acc_max) < 1.001 * M
    worst = backend_class(int(1.2 * M))
    print(f"back-end class: coordinates < 1.2 M closed under add and dbl (outputs < {worst / M:.3f} M); "
          f"reduce29 of an accumulator < 2^260 gives < {reduce29(acc_max) / M:.4f} M")
    b0 = 3 * MR  # stored values of the NTT passes
    for st in (3, 4, 5, 6):
        out = ntt_pass(st, b0)
        assert out < b0 and out < 1 << 256, (st, out / MR)
        print(f"ntt pass of {st} stages: inputs < 3 M, outputs < {out / MR:.3f} M (packable, below the input bound)")
    print(f"last pass: outputs < {ntt_pass(6, b0) / MR:.3f} M before two conditional subtractions of M")
    # the last pass without an epilogue product (ntt_last29_kernel ONE): reduce29 of the
    # stage outputs, then one conditional subtraction, must land below 2 M
    Bl = b0
    for s_ in range(6):
        Bl = max(2 * Bl, Bl + (4 << s_) * MR)
    ql = top(Bl) // (top(MR) + 1)
    red = MR + (ql + 2) * (1 << 232)
    assert red < 2 * MR and top(Bl) < 1 << 32, (LG(Bl), red / MR)
    print(f"last pass without a product: stage outputs < {Bl / MR:.0f} M, reduce29 -> < {red / MR:.6f} M")
    # the sparse first pass (ntt_first_sparse29_kernel): x0 < 1.01 M, p = x1 w < 1.01 M;
    # x0 - p + 4M feeds the closing product with the pass twiddle
    pj = MR * MR // R + MR + 1
    assert top(4 * MR) - 1 >= top(pj)
    ys = MR * 101 // 100 + 4 * MR
    column_ok(1 << 29, (1 << 29) + (1 << 30))
    out_sp = ys * MR // R + MR + 1
    assert out_sp < b0
    print(f"sparse first pass: outputs < {out_sp / MR:.3f} M")
    tw_live = MR * MR // R + MR + 1  # a twiddle formed in the pass: lo x hi, both < M (H2G_NTT_TW_LIVE)
    for st in (3, 4, 5, 6):
        out = ntt_pass(st, b0, tw_live)
        assert out < b0 and out < 1 << 256, (st, out / MR)
    print(f"passes with twiddles formed in the pass (< {tw_live / MR:.4f} M): outputs < {ntt_pass(6, b0, tw_live) / MR:.3f} M")
    # evaluate_h29_kernel's unreduced sums / differences (eh_addn / eh_add3n / eh_subn): each
    # feeds one product; loads < 32 M, constants < M, reduced values < 1.001 M, Horner
    # accumulators reduced after every step
    def prod(a, b):  # bound of REDC(a b) for a < aM, b < bM, in units of MR
        return a * b * MR // R + 1
    LD, C, RED = 32, 1, 1.001
    def sub_ok_fr(bm):  # a - b + 64 M: 64 M covers b's top limb
        assert top(64 * MR) - 1 >= top(int(bm * MR)), bm
    worst = 0
    # permutation block
    lo_hi = prod(LD, LD); cur = max(prod(C, prod(C, lo_hi)), prod(prod(C, lo_hi), C))
    add3 = LD + prod(C, LD) + C
    left = LD
    for _ in range(8):
        left = max(left, prod(left, add3))
    right = LD
    for _ in range(8):
        right = max(right, prod(right, LD + cur + C))
    sub_ok_fr(right)
    worst = max(worst, left + 64, 65, prod(LD, LD) + 64, LD + 64)
    # lookup block
    tv = prod(RED + C, RED + C)
    a1 = prod(prod(LD, LD + C), LD + C)
    sub_ok_fr(prod(LD, tv)); sub_ok_fr(LD)
    worst = max(worst, a1 + 64, LD + 64, prod(LD + 64, LD + 64))
    # shuffle block
    sub_ok_fr(prod(LD, RED + C))
    worst = max(worst, prod(LD, RED + C) + 64)
    assert worst * MR < 1 << 261, worst
    # every such operand times a load (< 32 M) -- the largest product input pairing
    assert prod(worst, LD) < 64, prod(worst, LD)
    print(f"evaluate_h unreduced operands < {worst:.1f} M (< 2^261), their products < {prod(worst, LD):.1f} M")
    # lincomb29_kernel: up to 6 pairs REDC(a c + b d) (a, b storage integers < M, c, d < M)
    # plus the accumulated storage value, then reduce29 + one subtraction
    pair = 2 * MR * MR // R + MR + 1
    tot = 6 * pair + MR
    column_ok(1 << 29, 1 << 29, 1 << 29, 1 << 29)
    assert tot < 1 << 260
    qv = top(tot) // (top(MR) + 1)
    assert MR + (qv + 2) * (1 << 232) < 2 * MR
    print(f"lincomb: pairs < {pair / MR:.4f} M, sum < {tot / MR:.2f} M, reduced below 2 M before the subtraction")
    # H2G_HORNER29 (eval_level1, kate_phase1/3): acc <- REDC(acc x) + a with x < M and a
    # storage integer a < 2^256; kate_phase3 (ACC) adds one more stored value before reducing
    h = 0
    for _ in range(200):
        h = max(h, h * MR // R + MR + 1 + (1 << 256))
    column_ok(1 << 30, 1 << 29)  # acc: a limb-wise add of two normalised values
    stored = h + (1 << 256)
    assert stored < 1 << 260
    qh = top(stored) // (top(MR) + 1)
    assert MR + (qh + 2) * (1 << 232) < 2 * MR
    print(f"Horner chains: accumulator < {h / MR:.2f} M, stored sums < {stored / MR:.2f} M, reduced below 2 M")
    print("ok")
