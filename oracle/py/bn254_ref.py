"""BN254 big-integer reference (TEST INFRASTRUCTURE ONLY -- never on the product path).

Pure-Python restatement of the arithmetic the halo2 prover hot path relies on,
written from the public BN254 definitions and from the reference's own use of
it.  It is deliberately slow and obviously-correct (affine formulas, O(n^2)
DFTs) and is used only to generate the small golden fixtures committed under
``tests/golden/`` and to cross-check the C restatement in ``oracle/``.

Reference behaviour followed (paths relative to the reference snapshot):
  * Fr/Fq Montgomery, 4 x u64 little-endian limbs, R = 2^256
        -- halo2curves 0.6 (third-party, not vendored)
  * EvaluationDomain::new constants          halo2_backend/src/poly/domain.rs:38-144
  * lagrange_to_coeff / ifft                 halo2_backend/src/poly/domain.rs:216-226, 343-351
  * coeff_to_extended                        halo2_backend/src/poly/domain.rs:230-244
  * extended_to_coeff                        halo2_backend/src/poly/domain.rs:271-293
  * divide_by_vanishing_poly                 halo2_backend/src/poly/domain.rs:297-316
  * distribute_powers_zeta                   halo2_backend/src/poly/domain.rs:325-341
  * MsmAccel::msm == best_multiexp           halo2_middleware/src/zal.rs:57-58, 136-138
  * eval_polynomial / kate_division          halo2_backend/src/arithmetic.rs:57-82, 101-120

Parity pinning: the reference holds no BN254 golden vectors; this
module is pinned to public BN254 constants (generator, 2G, S=28 root of unity,
DELTA = 7^(2^28), ZETA^3 = 1) in tests/test_oracle_golden.py.
"""
from __future__ import annotations

P = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47  # Fq
R = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001  # Fr
MONT_R = 1 << 256
S = 28
GENERATOR = 7
ROOT_OF_UNITY = pow(GENERATOR, (R - 1) >> S, R)
DELTA = pow(GENERATOR, 1 << S, R)
# halo2curves bn256 Fr::ZETA (cube root of unity); parity-neutral choice
ZETA = 0xB3C4D79D41A917585BFC41088D8DAAA78B17EA66B99C90DD
G1_GEN = (1, 2)
G1_B = 3

# ---------------------------------------------------------------- encodings


def to_limbs(x: int, n: int = 4) -> list[int]:
    return [(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(n)]


def from_limbs(l) -> int:
    return sum(int(v) << (64 * i) for i, v in enumerate(l))


def to_mont(x: int, m: int) -> int:
    return (x * MONT_R) % m


def from_mont(x: int, m: int) -> int:
    return (x * pow(MONT_R, -1, m)) % m


def fr_mont_limbs(x: int) -> list[int]:
    return to_limbs(to_mont(x % R, R))


def fq_mont_limbs(x: int) -> list[int]:
    return to_limbs(to_mont(x % P, P))


def g1_affine_mont_limbs(pt) -> list[int]:
    """halo2curves G1Affine in-memory layout: x[4], y[4] Montgomery; identity = (0, 0)."""
    if pt is None:
        return [0] * 8
    return fq_mont_limbs(pt[0]) + fq_mont_limbs(pt[1])


# ---------------------------------------------------------------- G1 (affine, None = identity)


def g1_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - G1_B) % P == 0


def g1_neg(pt):
    return None if pt is None else (pt[0], (-pt[1]) % P)


def g1_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    x1, y1 = a
    x2, y2 = b
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, -1, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    y3 = (lam * (x1 - x3) - y1) % P
    return (x3, y3)


def g1_mul(pt, k: int):
    k %= R
    acc = None
    add = pt
    while k:
        if k & 1:
            acc = g1_add(acc, add)
        add = g1_add(add, add)
        k >>= 1
    return acc


def msm_naive(scalars, points):
    """sum_i s_i * P_i -- the mathematical contract of MsmAccel::msm (zal.rs:58)."""
    acc = None
    for s, pt in zip(scalars, points):
        acc = g1_add(acc, g1_mul(pt, s))
    return acc


def srs_powers(s: int, n: int):
    """g_i = [s^i] G, as ParamsKZG::setup (halo2_backend/src/poly/kzg/commitment.rs:64-90)."""
    out = []
    cur = G1_GEN
    for _ in range(n):
        out.append(cur)
        cur = g1_mul(cur, s)
    return out


# ---------------------------------------------------------------- Fr polynomials


def omega_for(k: int) -> int:
    """2^k-th root of unity: ROOT_OF_UNITY^(2^(S-k)) (domain.rs:56-75)."""
    w = ROOT_OF_UNITY
    for _ in range(k, S):
        w = w * w % R
    return w


def dft(a, omega: int):
    """y_j = sum_i a_i omega^(ij) -- what best_fft computes in natural order (domain.rs:238,344)."""
    n = len(a)
    out = []
    for j in range(n):
        wj = pow(omega, j, R)
        acc = 0
        x = 1
        for i in range(n):
            acc += a[i] * x
            x = x * wj % R
        out.append(acc % R)
    return out


def fft(a, omega: int):
    """Recursive radix-2 DFT (same result as dft, O(n log n)) for moderate n."""
    n = len(a)
    if n == 1:
        return [a[0] % R]
    w2 = omega * omega % R
    ev = fft(a[0::2], w2)
    od = fft(a[1::2], w2)
    out = [0] * n
    w = 1
    for i in range(n // 2):
        t = od[i] * w % R
        out[i] = (ev[i] + t) % R
        out[i + n // 2] = (ev[i] - t) % R
        w = w * omega % R
    return out


class Domain:
    """EvaluationDomain::new(j, k) constants (domain.rs:38-144)."""

    def __init__(self, j: int, k: int):
        self.k = k
        self.n = 1 << k
        self.quotient_poly_degree = j - 1
        ek = k
        while (1 << ek) < self.n * self.quotient_poly_degree:
            ek += 1
        self.extended_k = ek
        self.extended_omega = omega_for(ek)
        self.omega = omega_for(k)
        self.omega_inv = pow(self.omega, -1, R)
        self.extended_omega_inv = pow(self.extended_omega, -1, R)
        self.g_coset = ZETA
        self.g_coset_inv = ZETA * ZETA % R
        orig = pow(ZETA, self.n, R)
        step = pow(self.extended_omega, self.n, R)
        t = []
        cur = orig
        while True:
            t.append(cur)
            cur = cur * step % R
            if cur == orig:
                break
        assert len(t) == 1 << (ek - k)
        self.t_evaluations = [pow((v - 1) % R, -1, R) for v in t]
        self.ifft_divisor = pow(1 << k, -1, R)
        self.extended_ifft_divisor = pow(1 << ek, -1, R)
        self.barycentric_weight = pow(self.n, -1, R)

    @property
    def extended_len(self):
        return 1 << self.extended_k

    def distribute_powers_zeta(self, a, into_coset: bool):
        pw = [1, self.g_coset, self.g_coset_inv] if into_coset else [1, self.g_coset_inv, self.g_coset]
        return [v * pw[i % 3] % R for i, v in enumerate(a)]

    def lagrange_to_coeff(self, a):
        assert len(a) == self.n
        return [v * self.ifft_divisor % R for v in fft(a, self.omega_inv)]

    def coeff_to_extended(self, a):
        assert len(a) == self.n
        b = self.distribute_powers_zeta(a, True) + [0] * (self.extended_len - self.n)
        return fft(b, self.extended_omega)

    def extended_to_coeff(self, a):
        assert len(a) == self.extended_len
        b = [v * self.extended_ifft_divisor % R for v in fft(a, self.extended_omega_inv)]
        b = self.distribute_powers_zeta(b, False)
        return b[: self.n * self.quotient_poly_degree]

    def divide_by_vanishing_poly(self, a):
        assert len(a) == self.extended_len
        t = self.t_evaluations
        return [v * t[i % len(t)] % R for i, v in enumerate(a)]


def eval_polynomial(poly, x: int) -> int:
    acc = 0
    for c in reversed(poly):
        acc = (acc * x + c) % R
    return acc


def kate_division(a, b: int):
    """arithmetic.rs:101-120: divide a(X) by (X - b), no remainder."""
    b = (-b) % R
    q = [0] * (len(a) - 1)
    tmp = 0
    for idx in range(len(a) - 1, 0, -1):
        lead = (a[idx] - tmp) % R
        q[idx - 1] = lead
        tmp = lead * b % R
    return q


# ---------------------------------------------------------------- G2 (twist over Fq2 = Fq[u]/(u^2 + 1))
# ParamsKZG keeps g2 and s_g2 = [s] g2 (halo2_backend/src/poly/kzg/commitment.rs:122-123).
# Elements of Fq2 are (c0, c1) = c0 + c1 u; the twist is y^2 = x^3 + 3 / (9 + u).


def fq2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def fq2_inv(a):
    t = pow(a[0] * a[0] + a[1] * a[1], P - 2, P)
    return (a[0] * t % P, (-a[1]) * t % P)


def fq2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def fq2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


G2_B = fq2_mul((3, 0), fq2_inv((9, 1)))
# the standard BN254 G2 generator (EIP-197; halo2curves G2_GENERATOR_X / _Y)
G2_GEN = ((10857046999023057135944570762232829481370756359578518086990519993285655852781,
           11559732032986387107991004021392285783925812861821192530917403151452391805634),
          (8495653923123431417604973247489272438418190587263600148770280649306958101930,
           4082367875863433681332203403145435568316851327593401208105741076214120093531))


def g2_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return fq2_mul(y, y) == fq2_add(fq2_mul(fq2_mul(x, x), x), G2_B)


def g2_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    (x1, y1), (x2, y2) = a, b
    if x1 == x2:
        if fq2_add(y1, y2) == (0, 0):
            return None
        lam = fq2_mul(fq2_mul((3, 0), fq2_mul(x1, x1)), fq2_inv(fq2_add(y1, y1)))
    else:
        lam = fq2_mul(fq2_sub(y2, y1), fq2_inv(fq2_sub(x2, x1)))
    x3 = fq2_sub(fq2_sub(fq2_mul(lam, lam), x1), x2)
    return (x3, fq2_sub(fq2_mul(lam, fq2_sub(x1, x3)), y1))


def g2_mul(pt, k: int):
    k %= R
    acc, add = None, pt
    while k:
        if k & 1:
            acc = g2_add(acc, add)
        add = g2_add(add, add)
        k >>= 1
    return acc


def g2_affine_mont_limbs(pt) -> list[int]:
    """halo2curves G2Affine raw layout: x.c0, x.c1, y.c0, y.c1 Montgomery (4 u64 each)."""
    if pt is None:
        return [0] * 16
    return fq_mont_limbs(pt[0][0]) + fq_mont_limbs(pt[0][1]) + fq_mont_limbs(pt[1][0]) + fq_mont_limbs(pt[1][1])


# ---------------------------------------------------------------- SerdeFormat::Processed
# halo2_backend/src/helpers.rs:36-100: curve points as GroupEncoding::to_bytes (halo2curves
# 0.6 bn256, the encoding the transcript's write_point also uses: x canonical LE, bit 7 of
# the last byte = parity of canonical y -- of y.c0 for G2 --, identity all zero), field
# elements as PrimeField::to_repr (canonical LE).  halo2curves is not vendored in the
# reference, so the flag convention is restated, not pinned by a reference vector.


def fq_sqrt(a: int):
    """a^((p+1)/4) (p = 3 mod 4), None for a non-residue"""
    y = pow(a % P, (P + 1) // 4, P)
    return y if y * y % P == a % P else None


def fq2_pow(a, e: int):
    acc = (1, 0)
    for bit in bin(e)[2:]:
        acc = fq2_mul(acc, acc)
        if bit == "1":
            acc = fq2_mul(acc, a)
    return acc


def fq2_sqrt(a):
    """a square root in Fq2 (eprint 2012/685 Algorithm 9), None for a non-residue"""
    if a == (0, 0):
        return (0, 0)
    a1 = fq2_pow(a, (P - 3) // 4)
    alpha = fq2_mul(fq2_mul(a1, a1), a)
    x0 = fq2_mul(a1, a)
    if alpha == (P - 1, 0):
        x = ((-x0[1]) % P, x0[0])
    else:
        x = fq2_mul(fq2_pow(fq2_add(alpha, (1, 0)), (P - 1) // 2), x0)
    return x if fq2_mul(x, x) == a else None


def g1_to_bytes(pt) -> bytes:
    if pt is None:
        return bytes(32)
    b = bytearray(pt[0].to_bytes(32, "little"))
    b[31] |= (pt[1] & 1) << 7
    return bytes(b)


def g1_from_bytes(b: bytes):
    """(ok, point): GroupEncoding::from_bytes"""
    ysign = b[31] >> 7
    x = int.from_bytes(bytes(b[:31]) + bytes([b[31] & 0x7F]), "little")
    if x >= P:
        return False, None
    if x == 0 and not ysign:
        return True, None
    y = fq_sqrt(x * x * x + G1_B)
    if y is None:
        return False, None
    if (y & 1) != ysign:
        y = (-y) % P
    return True, (x, y)


def g2_to_bytes(pt) -> bytes:
    if pt is None:
        return bytes(64)
    b = bytearray(pt[0][0].to_bytes(32, "little") + pt[0][1].to_bytes(32, "little"))
    b[63] |= (pt[1][0] & 1) << 7
    return bytes(b)


def g2_from_bytes(b: bytes):
    ysign = b[63] >> 7
    x0 = int.from_bytes(b[:32], "little")
    x1 = int.from_bytes(bytes(b[32:63]) + bytes([b[63] & 0x7F]), "little")
    if x0 >= P or x1 >= P:
        return False, None
    if x0 == 0 and x1 == 0 and not ysign:
        return True, None
    x = (x0, x1)
    y = fq2_sqrt(fq2_add(fq2_mul(fq2_mul(x, x), x), G2_B))
    if y is None:
        return False, None
    if (y[0] & 1) != ysign:
        y = ((-y[0]) % P, (-y[1]) % P)
    return True, (x, y)


def fr_to_repr(x: int) -> bytes:
    return (x % R).to_bytes(32, "little")
