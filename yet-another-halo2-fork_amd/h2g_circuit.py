"""Backend circuit description consumed by keygen / create_proof, and the synthetic
circuits the tests and the bench prove.

This mirrors what the reference's backend receives from its frontend
(`halo2_middleware/src/circuit.rs`): `ConstraintSystemMid` (column counts, gates as
`ExpressionMid` trees, the permutation `ArgumentMid.columns`, unblinded advice
columns) plus `Preprocessing` (fixed column values and `PermutationMid.copies`), and
the witness of one proof (advice columns, instance columns).  Circuit authoring
(chips, layouters, floor planners) is the frontend and out of scope; the generators
below lay cells out directly.

Expressions are flattened for the C ABI into nodes of 4 int32 `(op, a, b, c)`:
  CONST (a = constant index) | QUERY (a = column type, b = column index, c = rotation)
  | NEG (a = child) | SUM / PROD (a = lhs, b = rhs) | CHALLENGE (a = challenge index).
Column types follow `halo2_middleware::circuit::Any` as used here: 0 advice,
1 fixed, 2 instance.  Field elements travel as numpy uint64 arrays in halo2curves'
layout (Montgomery form, 4 little-endian limbs).
"""
import hashlib

import numpy as np

ADVICE, FIXED, INSTANCE = 0, 1, 2
OP_CONST, OP_QUERY, OP_NEG, OP_SUM, OP_PROD, OP_CHALLENGE = 0, 1, 2, 3, 4, 5

R_MOD = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
_MONT = (1 << 256) % R_MOD


def fr_to_limbs(x: int) -> list:
    """canonical int -> Montgomery limbs"""
    m = (x % R_MOD) * _MONT % R_MOD
    return [(m >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)]


def fr_from_limbs(l) -> int:
    m = sum(int(l[i]) << (64 * i) for i in range(4))
    return m * pow(_MONT, -1, R_MOD) % R_MOD


def ints_to_mont(vals) -> np.ndarray:
    out = np.zeros((len(vals), 4), dtype=np.uint64)
    for i, v in enumerate(vals):
        if v:
            out[i] = fr_to_limbs(v)
    return out


def mont_to_ints(arr) -> list:
    arr = np.asarray(arr, dtype=np.uint64).reshape(-1, 4)
    return [fr_from_limbs(r) for r in arr]


# ----------------------------------------------------------------------------- expressions
class Expr:
    """ExpressionMid (halo2_middleware/src/expression.rs), challenges included."""

    __slots__ = ("op", "a", "b", "c")

    def __init__(self, op, a=0, b=0, c=0):
        self.op, self.a, self.b, self.c = op, a, b, c

    def __add__(self, o):
        return Expr(OP_SUM, self, _e(o))

    def __radd__(self, o):
        return Expr(OP_SUM, _e(o), self)

    def __sub__(self, o):
        return Expr(OP_SUM, self, Expr(OP_NEG, _e(o)))

    def __rsub__(self, o):
        return Expr(OP_SUM, _e(o), Expr(OP_NEG, self))

    def __mul__(self, o):
        return Expr(OP_PROD, self, _e(o))

    def __rmul__(self, o):
        return Expr(OP_PROD, _e(o), self)

    def __neg__(self):
        return Expr(OP_NEG, self)

    def degree(self):
        if self.op in (OP_CONST, OP_CHALLENGE):
            return 0
        if self.op == OP_QUERY:
            return 1
        if self.op == OP_NEG:
            return self.a.degree()
        if self.op == OP_SUM:
            return max(self.a.degree(), self.b.degree())
        return self.a.degree() + self.b.degree()

    def evaluate(self, const, query, mod=R_MOD, challenge=None):
        """Expression::evaluate with closures for constants, queries and challenges (ints mod r)."""
        if self.op == OP_CONST:
            return const(self.a) % mod
        if self.op == OP_CHALLENGE:
            return challenge(self.a) % mod
        if self.op == OP_QUERY:
            return query(self.a, self.b, self.c) % mod
        if self.op == OP_NEG:
            return (-self.a.evaluate(const, query, mod, challenge)) % mod
        x = self.a.evaluate(const, query, mod, challenge)
        y = self.b.evaluate(const, query, mod, challenge)
        return (x + y) % mod if self.op == OP_SUM else (x * y) % mod


def _e(x):
    return x if isinstance(x, Expr) else const(int(x))


def const(v: int) -> Expr:
    return Expr(OP_CONST, int(v) % R_MOD)


def challenge(index):
    """ExpressionMid::Challenge (the value squeezed after its phase's advice commitments)"""
    return Expr(OP_CHALLENGE, int(index))


def advice(col, rot=0):
    return Expr(OP_QUERY, ADVICE, col, rot)


def fixed(col, rot=0):
    return Expr(OP_QUERY, FIXED, col, rot)


def instance(col, rot=0):
    return Expr(OP_QUERY, INSTANCE, col, rot)


# ----------------------------------------------------------------------------- circuit
class Circuit:
    """ConstraintSystemMid + Preprocessing (one compiled circuit)."""

    def __init__(self, k, num_advice, num_fixed, num_instance, gates, perm_columns, copies,
                 fixed_values, unblinded=None, name="circuit", lookups=(), shuffles=(), advice_phase=None,
                 challenge_phase=None):
        """lookups: [(input_exprs, table_exprs)], shuffles: [(input_exprs, shuffle_exprs)]
        (halo2_middleware circuit.rs LookupArgument / ShuffleArgument); advice_phase /
        challenge_phase: ConstraintSystemMid advice_column_phase / challenge_phase"""
        self.lookups = [(list(a), list(b)) for a, b in lookups]
        self.shuffles = [(list(a), list(b)) for a, b in shuffles]
        for a, b in self.lookups + self.shuffles:
            assert len(a) == len(b) and len(a) > 0
        self.k = int(k)
        self.n = 1 << self.k
        self.num_advice, self.num_fixed, self.num_instance = num_advice, num_fixed, num_instance
        self.gates = list(gates)
        self.perm_columns = [tuple(c) for c in perm_columns]
        self.copies = np.asarray(copies, dtype=np.int32).reshape(-1, 6)
        self.fixed_values = np.ascontiguousarray(fixed_values, dtype=np.uint64).reshape(num_fixed, self.n, 4)
        self.unblinded = np.zeros(max(num_advice, 1), dtype=np.uint8)
        for c in unblinded or []:
            self.unblinded[c] = 1
        self.name = name
        self.advice_phase = np.zeros(max(num_advice, 1), dtype=np.uint8)
        if advice_phase is not None:
            self.advice_phase[:num_advice] = advice_phase
        self.challenge_phase = np.asarray(list(challenge_phase or []) or [0], dtype=np.uint8)
        self.num_challenges = len(challenge_phase or [])
        self.max_phase = int(self.advice_phase[:num_advice].max()) if num_advice else 0
        assert all(int(p) <= self.max_phase for p in self.challenge_phase[:self.num_challenges])
        self._flatten()

    # -- ConstraintSystem facts (halo2_backend/src/plonk/circuit.rs, keygen.rs) --
    def degree(self):
        """ConstraintSystem::degree: permutation (3), lookups max(4, 2 + deg(in) + deg(table)),
        shuffles 2 + max(deg(in), deg(shuffle)), gates -- circuit.rs:100-139,292-389"""
        d = [3] + [g.degree() for g in self.gates]
        for a, b in self.lookups:
            d.append(max(4, 2 + max([1] + [e.degree() for e in a]) + max([1] + [e.degree() for e in b])))
        for a, b in self.shuffles:
            d.append(2 + max([1] + [e.degree() for e in a] + [e.degree() for e in b]))
        return max(d)

    def queries(self):
        """(advice, fixed, instance) query lists in first-appearance order: gate
        expressions depth first (lhs before rhs), then permutation columns at
        Rotation::cur() -- keygen.rs:191-260."""
        lists = {ADVICE: [], FIXED: [], INSTANCE: []}

        def add(t, i, r):
            if (i, r) not in lists[t]:
                lists[t].append((i, r))

        def walk(e):
            if e.op == OP_QUERY:
                add(e.a, e.b, e.c)
            elif e.op == OP_NEG:
                walk(e.a)
            elif e.op in (OP_SUM, OP_PROD):
                walk(e.a)
                walk(e.b)

        for g in self.gates:
            walk(g)
        for a, b in self.lookups + self.shuffles:
            for e in a + b:
                walk(e)
        for t, i in self.perm_columns:
            add(t, i, 0)
        return lists[ADVICE], lists[FIXED], lists[INSTANCE]

    def blinding_factors(self):
        """max(3, max advice queries per column) + 2 -- circuit.rs:143-170"""
        adv, _, _ = self.queries()
        per_col = [sum(1 for (c, _) in adv if c == col) for col in range(self.num_advice)]
        return max([3] + per_col) + 2 if self.num_advice else 5

    def usable_rows(self):
        return self.n - (self.blinding_factors() + 1)

    def _flatten(self):
        nodes, consts, const_idx = [], [], {}

        def rec(e):
            if e.op == OP_CONST:
                if e.a not in const_idx:
                    const_idx[e.a] = len(consts)
                    consts.append(e.a)
                nodes.append((OP_CONST, const_idx[e.a], 0, 0))
            elif e.op == OP_QUERY:
                nodes.append((OP_QUERY, e.a, e.b, e.c))
            elif e.op == OP_CHALLENGE:
                nodes.append((OP_CHALLENGE, e.a, 0, 0))
            elif e.op == OP_NEG:
                a = rec(e.a)
                nodes.append((OP_NEG, a, 0, 0))
            else:
                a = rec(e.a)
                b = rec(e.b)
                nodes.append((e.op, a, b, 0))
            return len(nodes) - 1

        roots = [rec(g) for g in self.gates]
        self.lookup_sizes = np.asarray([len(a) for a, _ in self.lookups] or [0], dtype=np.uint32)
        self.lookup_roots = np.asarray([rec(e) for a, b in self.lookups for e in a + b] or [0], dtype=np.int32)
        self.shuffle_sizes = np.asarray([len(a) for a, _ in self.shuffles] or [0], dtype=np.uint32)
        self.shuffle_roots = np.asarray([rec(e) for a, b in self.shuffles for e in a + b] or [0], dtype=np.int32)
        self.nodes = np.asarray(nodes, dtype=np.int32).reshape(-1, 4)
        self.gate_roots = np.asarray(roots, dtype=np.int32)
        self.constants = ints_to_mont(consts) if consts else np.zeros((1, 4), dtype=np.uint64)
        self.num_constants = len(consts)
        self.perm_array = np.asarray(self.perm_columns, dtype=np.int32).reshape(-1, 2)

    def transcript_repr(self) -> np.ndarray:
        """vk.transcript_repr.  The reference hashes the Debug text of the pinned VK
        (plonk.rs:189-200: Blake2b-512, personal "Halo2-Verify-Key", length-prefixed,
        from_uniform_bytes); that text cannot be reproduced outside Rust, so the same
        construction is applied to this description's canonical bytes."""
        h = hashlib.blake2b(digest_size=64, person=b"Halo2-Verify-Key")
        desc = b"".join([
            np.asarray([self.k, self.num_advice, self.num_fixed, self.num_instance], dtype=np.int64).tobytes(),
            self.nodes.tobytes(), self.gate_roots.tobytes(), self.constants.tobytes(),
            self.perm_array.tobytes(), self.copies.tobytes(), self.unblinded.tobytes(),
            self.lookup_sizes.tobytes(), self.lookup_roots.tobytes(), self.shuffle_sizes.tobytes(),
            self.shuffle_roots.tobytes(),
            hashlib.blake2b(self.fixed_values.tobytes()).digest(),
        ] + ([self.advice_phase.tobytes(), self.challenge_phase[:self.num_challenges].tobytes()]
             if self.max_phase or self.num_challenges else []))
        h.update(len(desc).to_bytes(8, "little"))
        h.update(desc)
        v = int.from_bytes(h.digest(), "little") % R_MOD
        return np.asarray(fr_to_limbs(v), dtype=np.uint64)


class Witness:
    """One proof's advice and instance columns (Lagrange values, length n each)."""

    def __init__(self, advice_values, instance_values, instance_lens):
        self.advice = np.ascontiguousarray(advice_values, dtype=np.uint64)
        self.instance = np.ascontiguousarray(instance_values, dtype=np.uint64)
        self.instance_lens = np.ascontiguousarray(instance_lens, dtype=np.uint32)
        if self.instance_lens.size == 0:
            self.instance_lens = np.zeros(1, dtype=np.uint32)


# ----------------------------------------------------------------------------- generators
def _rand_ints(rng, count):
    return [int.from_bytes(rng.bytes(32), "little") % R_MOD for _ in range(count)]


def simple_example(k=8, seed=1, blocks=None):
    """C1: the simple-example constraint system (halo2_proofs/examples/simple-example.rs:
    98-117,266-277): advice a0, a1; instance i; fixed `constant` (enable_constant) and
    the s_mul selector (as a fixed column); gate s_mul * (a0 * a1 - a0[next]);
    equality on instance, constant, a0, a1.  Cells are laid out in 4-row blocks
    computing c = constant * (a*b)^2 and exposing c in the instance column."""
    n = 1 << k
    rng = np.random.default_rng(seed)
    a0, a1 = [0] * n, [0] * n
    fconst, smul = [0] * n, [0] * n
    inst = [0] * n
    copies = []
    gates = [fixed(1) * (advice(0) * advice(1) - advice(0, 1))]
    perm = [(INSTANCE, 0), (FIXED, 0), (ADVICE, 0), (ADVICE, 1)]
    # a0 has 2 queries (cur, next) -> bf = 5, usable = n - 6
    usable = n - 6
    nblocks = blocks if blocks is not None else max(1, (usable - 1) // 4)
    for blk in range(nblocks):
        r = 4 * blk
        if r + 4 > usable:
            break
        a, b = _rand_ints(rng, 2)
        cst = 7 + blk
        ab = a * b % R_MOD
        absq = ab * ab % R_MOD
        c = cst * absq % R_MOD
        a0[r], a1[r], smul[r] = a, b, 1          # ab = a * b
        a0[r + 1], a1[r + 1], smul[r + 1] = ab, ab, 1   # absq = ab * ab
        a0[r + 2], a1[r + 2], smul[r + 2] = absq, cst, 1  # c = absq * constant
        a0[r + 3] = c
        fconst[blk] = cst
        inst[blk] = c
        copies += [(ADVICE, 0, r + 1, ADVICE, 1, r + 1),
                   (FIXED, 0, blk, ADVICE, 1, r + 2),
                   (ADVICE, 0, r + 3, INSTANCE, 0, blk)]
    fixed_vals = np.stack([ints_to_mont(fconst), ints_to_mont(smul)])
    circ = Circuit(k, 2, 2, 1, gates, perm, copies, fixed_vals, name=f"simple-example k={k}")
    wit = Witness(np.stack([ints_to_mont(a0), ints_to_mont(a1)]), ints_to_mont(inst)[None],
                  [nblocks])
    return circ, wit


def mixed_circuit(k=7, seed=2):
    """A circuit exercising every expression/argument feature the backend supports:
    degree 5 (extended domain 4n), rotations -1/+1/+2, constants, negation, instance
    queries inside gates, fixed and instance columns in the permutation, two
    permutation sets (chunk_len 3), an unblinded advice column."""
    n = 1 << k
    rng = np.random.default_rng(seed)
    A, B, C, D, E = range(5)
    Q1, Q2, Q3, K = range(4)
    gates = [
        fixed(Q1) * (advice(A) * advice(B) * advice(C) - advice(D) + 7),
        fixed(Q2) * (advice(A, 1) - advice(A) - advice(B, -1)),
        fixed(Q3) * (advice(C) * advice(D) * advice(A, 2) * advice(B) - const(5) * instance(0)),
        -(fixed(Q1) * (advice(D) - instance(1))),
        fixed(Q2) * advice(E) * (advice(E) - 1),   # E boolean on q2 rows; E is unblinded
    ]
    perm = [(ADVICE, A), (FIXED, K), (INSTANCE, 0), (ADVICE, C), (ADVICE, B), (ADVICE, D)]
    circ0 = Circuit(k, 5, 4, 2, gates, perm, [], np.zeros((4, n, 4), np.uint64))
    u = circ0.usable_rows()
    va = _rand_ints(rng, n)
    vb = _rand_ints(rng, n)
    vc = _rand_ints(rng, n)
    vd = _rand_ints(rng, n)
    ve = [0] * n
    for r in range(n):
        va[r] = va[r] if r < u else 0
        vb[r] = vb[r] if r < u else 0
        vc[r] = vc[r] if r < u else 0
        vd[r] = vd[r] if r < u else 0
    q1, q2, q3, kf = [0] * n, [0] * n, [0] * n, [0] * n
    for r in range(u):
        if r % 3 == 0:
            q1[r] = 1
        elif r % 3 == 1 and r + 1 < u:
            q2[r] = 1
            ve[r] = int(rng.integers(0, 2))
        elif r % 3 == 2 and r + 2 < u:
            q3[r] = 1
    i0, i1 = [0] * n, [0] * n
    copies = []
    # copies between free cells (set before the constrained cells are derived)
    used_b, used_a = set(), set()
    for r in range(1, u - 3, 7):
        r2 = (r * 5 + 3) % (u - 2)
        if r2 % 3 == 0 or r2 in used_b:
            continue
        used_b.add(r2)
        vb[r2] = vc[r]
        copies.append((ADVICE, C, r, ADVICE, B, r2))
    # c[r] == a[r3] for a few free a cells (r3 % 3 in {0,1}); joins the cycles above
    for r in range(2, u - 3, 11):
        r3 = (r * 3 + 1) % (u - 3)
        if r3 % 3 == 2 or r3 in used_a:
            continue
        used_a.add(r3)
        va[r3] = vc[r]
        copies.append((ADVICE, A, r3, ADVICE, C, r))
    # fixed constants copied into c cells
    for j, r in enumerate(range(5, u, 13)):
        kf[j] = vc[r]
        copies.append((FIXED, K, j, ADVICE, C, r))
    # constrained cells
    for r in range(u):
        if r % 3 == 2 and r >= 2:
            va[r] = (va[r - 1] + vb[r - 2]) % R_MOD if q2[r - 1] else va[r]
    for r in range(u):
        if q1[r]:
            vd[r] = (va[r] * vb[r] % R_MOD * vc[r] + 7) % R_MOD
            i1[r] = vd[r]
    inv5 = pow(5, -1, R_MOD)
    for r in range(u):
        if q3[r]:
            i0[r] = vc[r] * vd[r] % R_MOD * va[r + 2] % R_MOD * vb[r] % R_MOD * inv5 % R_MOD
        elif r % 3 == 0:
            i0[r] = va[r]
            copies.append((INSTANCE, 0, r, ADVICE, A, r))
    fixed_vals = np.stack([ints_to_mont(q1), ints_to_mont(q2), ints_to_mont(q3), ints_to_mont(kf)])
    circ = Circuit(k, 5, 4, 2, gates, perm, copies, fixed_vals, unblinded=[E], name=f"mixed k={k}")
    wit = Witness(np.stack([ints_to_mont(v) for v in (va, vb, vc, vd, ve)]),
                  np.stack([ints_to_mont(i0), ints_to_mont(i1)]), [u, u])
    return circ, wit


def lookup_circuit(k=8, seed=4, table_bits=None):
    """Lookup + shuffle circuit (the argument shapes of BASELINE configs[4]): advice a (bytes),
    b = a^2, c, d = a permutation of c; fixed q, t = range table 0..2^bits-1, t2 = t^2,
    q2.  gate q (b - a a); lookup [q a] in [t]; lookup [q a, q b] in [t, t2] (two-column
    table); lookup [q a[next]] in [t] (rotation inside a lookup); shuffle [q2 c] ~ [q2 d];
    permutation over a, c with copies between equal cells."""
    n = 1 << k
    rng = np.random.default_rng(seed)
    A, B, C, D = range(4)
    Q, T, T2, Q2 = range(4)
    gates = [fixed(Q) * (advice(B) - advice(A) * advice(A))]
    lookups = [([fixed(Q) * advice(A)], [fixed(T)]),
               ([fixed(Q) * advice(A), fixed(Q) * advice(B)], [fixed(T), fixed(T2)]),
               ([fixed(Q) * advice(A, 1)], [fixed(T)])]
    shuffles = [([fixed(Q2) * advice(C)], [fixed(Q2) * advice(D)])]
    perm = [(ADVICE, A), (ADVICE, C)]
    probe = Circuit(k, 4, 4, 0, gates, perm, [], np.zeros((4, n, 4), np.uint64), lookups=lookups,
                    shuffles=shuffles)
    u = probe.usable_rows()
    tsize = 1 << (table_bits if table_bits is not None else min(8, k - 1))
    assert tsize <= u, "the range table must fit in the usable rows"
    va = [0] * n
    vc = [0] * n
    for r in range(u):
        va[r] = int(rng.integers(0, tsize))
        vc[r] = int.from_bytes(rng.bytes(32), "little") % R_MOD
    vb = [v * v % R_MOD for v in va]
    perm_idx = rng.permutation(u)
    vd = [vc[int(perm_idx[r])] for r in range(u)] + [0] * (n - u)
    q = [1 if r < u - 1 else 0 for r in range(n)]   # a[next] must stay inside the usable rows
    q2 = [1 if r < u else 0 for r in range(n)]
    t = [r % tsize if r < u else 0 for r in range(n)]
    t2 = [v * v % R_MOD for v in t]
    copies = []
    seen = {}
    for r in range(u):
        if va[r] in seen and len(copies) < 20:
            copies.append((ADVICE, A, seen[va[r]], ADVICE, A, r))
        seen[va[r]] = r
    copies.append((ADVICE, C, 3, ADVICE, C, 3))   # trivial self-copy (no-op in Assembly)
    fixed_vals = np.stack([ints_to_mont(q), ints_to_mont(t), ints_to_mont(t2), ints_to_mont(q2)])
    circ = Circuit(k, 4, 4, 0, gates, perm, copies, fixed_vals, name=f"lookup k={k}", lookups=lookups,
                   shuffles=shuffles)
    wit = Witness(np.stack([ints_to_mont(v) for v in (va, vb, vc, vd)]), np.zeros((0, n, 4), np.uint64), [])
    return circ, wit


def synthetic_c3(k, ops, seed=3):
    """C3: 3 advice a, b, c; 1 fixed f; gate f * (a * b - c); a, b, c in
    the permutation (3 sets); copies c_i -> a_{i+1} chain every usable row.
    Witness: random b, a_0; a_{i+1} = c_i = a_i * b_i (a prefix product), f = 1 on
    usable rows.  `ops` supplies vectorised Montgomery arithmetic (mul, prefix_product)
    so that k = 20..24 builds in seconds (GPU ops on the bench box, the C oracle in CPU
    tests)."""
    n = 1 << k
    gates = [fixed(0) * (advice(0) * advice(1) - advice(2))]
    perm = [(ADVICE, 0), (ADVICE, 1), (ADVICE, 2)]
    bf = 5
    u = n - (bf + 1)
    rng = np.random.default_rng(seed)
    b = random_mont(rng, n)
    b[u:] = 0
    a0 = random_mont(rng, 1)
    # a_i = a0 * prod_{j<i} b_j  for i < u
    pp = ops.prefix_product(b)              # pp_i = prod_{j<=i} b_j
    a = np.empty_like(b)
    a[0] = a0[0]
    a[1:] = ops.mul(pp[:-1], np.broadcast_to(a0, (n - 1, 4)).copy())
    a[u:] = 0
    c = ops.mul(a, b)
    f = np.zeros((1, n, 4), dtype=np.uint64)
    one = np.asarray(fr_to_limbs(1), dtype=np.uint64)
    f[0, :u] = one
    rows = np.arange(u - 1, dtype=np.int32)
    copies = np.stack([np.full(u - 1, ADVICE, np.int32), np.full(u - 1, 2, np.int32), rows,
                       np.full(u - 1, ADVICE, np.int32), np.zeros(u - 1, np.int32), rows + 1], axis=1)
    circ = Circuit(k, 3, 1, 0, gates, perm, copies, f, name=f"synthetic-c3 k={k}")
    wit = Witness(np.stack([a, b, c]), np.zeros((0, n, 4), dtype=np.uint64), [])
    return circ, wit


def random_mont(rng, count):
    """uniform-ish field elements already in Montgomery form (top limb < r's top limb)"""
    x = rng.integers(0, 2**63, size=(count, 4), dtype=np.int64).astype(np.uint64) * np.uint64(2)
    x += rng.integers(0, 2, size=(count, 4), dtype=np.int64).astype(np.uint64)
    x[:, 3] %= np.uint64(0x30644E72E131A029)
    return x


def keccak_style(k, words=16, seed=5):
    """C5-shaped circuit (BASELINE configs[4]: many advice columns + lookup arguments, the
    shape of keccak's nibble-xor tables): advice x_0..x_{W-1}, y_0..y_{W-1}; fixed q, qc,
    Ta, Tb, Tc with (Ta, Tb, Tc) = (a, b, a ^ b) over 4-bit nibbles; W lookups
    [q x_i, q x_{i+1 mod W}, q y_i] in [Ta, Tb, Tc] (y_i = x_i ^ x_{i+1}, degree 5 ->
    extended domain 4n); gate qc (x_0[next] - y_0) (a xor chain down x_0); permutation
    over y_0, x_4 with copies y_0[r] = x_4[r] every 5th row.  Witness generation is
    vectorised (numpy), so k = 18 builds in seconds."""
    n = 1 << k
    W = words
    assert W >= 5
    X = list(range(W))
    Y = list(range(W, 2 * W))
    Q, QC, TA, TB, TC = range(5)
    lookups = [([fixed(Q) * advice(X[i]), fixed(Q) * advice(X[(i + 1) % W]), fixed(Q) * advice(Y[i])],
                [fixed(TA), fixed(TB), fixed(TC)]) for i in range(W)]
    gates = [fixed(QC) * (advice(X[0], 1) - advice(Y[0]))]
    perm = [(ADVICE, Y[0]), (ADVICE, X[4])]
    probe = Circuit(k, 2 * W, 5, 0, gates, perm, [], np.zeros((5, n, 4), np.uint64), lookups=lookups)
    u = probe.usable_rows()
    assert u >= 256, "the nibble-xor table needs 256 usable rows"
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 16, size=(W, n), dtype=np.int64)
    x[:, u:] = 0
    # x_0 chain: x0[r+1] = x0[r] ^ x1[r] for r < u - 1
    acc = np.bitwise_xor.accumulate(x[1, : u - 1])
    x[0, 1:u] = x[0, 0] ^ acc
    y = np.zeros_like(x)
    rows_c = np.arange(0, u, 5)
    for i in range(W):
        if i == 4:  # copies: x_4 = y_0 on the copy rows (y_0 is final by now)
            x[4, rows_c] = y[0, rows_c]
        if i < W - 1:
            y[i, :u] = x[i, :u] ^ x[i + 1, :u]
    y[3, :u] = x[3, :u] ^ x[4, :u]
    y[W - 1, :u] = x[W - 1, :u] ^ x[0, :u]
    small = ints_to_mont(list(range(16)))
    adv = np.concatenate([small[x], small[y]], axis=0)
    q = np.zeros(n, np.int64)
    q[:u] = 1
    qc = np.zeros(n, np.int64)
    qc[: u - 1] = 1
    r = np.arange(n)
    ta = np.where(r < u, r % 16, 0)
    tb = np.where(r < u, (r // 16) % 16, 0)
    tc = ta ^ tb
    fixed_vals = np.stack([small[q], small[qc], small[ta], small[tb], small[tc]])
    copies = np.stack([np.full(len(rows_c), ADVICE, np.int32), np.full(len(rows_c), Y[0], np.int32),
                       rows_c.astype(np.int32), np.full(len(rows_c), ADVICE, np.int32),
                       np.full(len(rows_c), X[4], np.int32), rows_c.astype(np.int32)], axis=1)
    circ = Circuit(k, 2 * W, 5, 0, gates, perm, copies, fixed_vals, name=f"keccak-style k={k} W={W}",
                   lookups=lookups)
    wit = Witness(adv, np.zeros((0, n, 4), np.uint64), [])
    return circ, wit


def challenge_circuit(k=6, seed=6, extended=False):
    """C6: two advice phases and two challenges (ConstraintSystemMid advice_column_phase /
    challenge_phase; Prover::commit_phase, halo2_backend/src/plonk/prover.rs:309-494).
    Phase 0: advice a (values 0..15); challenge c0 squeezed after it.  Phase 1: advice
    z, the running random linear combination z[i+1] = z[i] c0 + a[i] (z[0] = 0 by a copy
    from a cell holding 0); challenge c1 squeezed after it.  Gates: q (z[next] - z c0 - a)
    c1 and q0 z; lookup (a c0) in (t c0) over a fixed table t = 0..15, so challenges
    also enter the compressed lookup expressions.
    extended: adds an unblinded phase-1 column w = a c1-free copy of a shifted (w[i] = a[i+1])
    whose rows are shuffled against a (shuffle (w) ~ (a) over the usable rows), an instance
    column, and a third phase with a column holding z scaled by the phase-1 challenge.
    -> (circuit, phase-0 witness (instance only), fill(phase, challenges) -> {column: values})"""
    n = 1 << k
    rng = np.random.default_rng(seed)
    c0, c1 = challenge(0), challenge(1)
    gates = [fixed(0) * (advice(1, 1) - advice(1) * c0 - advice(0)) * c1, fixed(1) * advice(1)]
    lookups = [([advice(0) * c0], [fixed(2) * c0])]
    # z has 2 queries (cur, next) -> bf = 5, usable = n - 6
    usable = n - 6
    a = [int(v) for v in rng.integers(0, 16, size=n)]
    a[4] = 0
    q = [1 if i < usable - 1 else 0 for i in range(n)]
    q0 = [1 if i == 0 else 0 for i in range(n)]
    t = [i % 16 for i in range(n)]
    copies = [(ADVICE, 1, 0, ADVICE, 0, 4), (ADVICE, 0, 2, ADVICE, 0, 6)]
    a[6] = a[2]
    fixed_vals = np.stack([ints_to_mont(q), ints_to_mont(q0), ints_to_mont(t)])
    if not extended:
        circ = Circuit(k, 2, 3, 0, gates, [(ADVICE, 0), (ADVICE, 1)], copies, fixed_vals,
                       name=f"challenge k={k}", lookups=lookups, advice_phase=[0, 1], challenge_phase=[0, 1])
    else:
        # w (col 2, phase 1, unblinded): a permutation of a's active rows (rotated by one);
        # y (col 3, phase 2): y = z c1 on the q rows; instance 0 = a[0..4)
        gates.append(fixed(0) * (advice(3) - advice(1) * c1))
        shuffles = [([fixed(3) * advice(2)], [fixed(3) * advice(0)])]
        fixed_vals = np.concatenate([fixed_vals, ints_to_mont([1 if i < usable else 0 for i in range(n)])[None]])
        copies = copies + [(ADVICE, 0, i, INSTANCE, 0, i) for i in range(4)]
        circ = Circuit(k, 4, 4, 1, gates, [(ADVICE, 0), (ADVICE, 1), (INSTANCE, 0)], copies, fixed_vals,
                       unblinded=[2], name=f"challenge+ k={k}", lookups=lookups, shuffles=shuffles,
                       advice_phase=[0, 1, 1, 2], challenge_phase=[0, 1])

    def z_values(ch):
        z = [0] * n
        for i in range(usable - 1):
            z[i + 1] = (z[i] * ch[0] + a[i]) % R_MOD
        return z

    w = [a[(i + 1) % usable] if i < usable else 0 for i in range(n)]

    def y_values(ch):
        z = z_values(ch)
        return [z[i] * ch[1] % R_MOD if q[i] else 0 for i in range(n)]

    def fill(phase, ch):
        if phase == 0:
            return {0: ints_to_mont(a)}
        if phase == 1:
            out = {1: ints_to_mont(z_values(ch))}
            if extended:
                out[2] = ints_to_mont(w)
            return out
        return {3: ints_to_mont(y_values(ch))}

    def full(ch):
        """the complete witness once the challenges are known"""
        cols = [a, z_values(ch)] + ([w, y_values(ch)] if extended else [])
        return Witness(np.stack([ints_to_mont(c) for c in cols]), wit.instance, wit.instance_lens)

    fill.z_values = z_values
    fill.a = a
    fill.full = full
    if extended:
        inst = ints_to_mont(a[:4] + [0] * (n - 4))[None]
        wit = Witness(np.zeros((4, n, 4), dtype=np.uint64), inst, [4])
    else:
        wit = Witness(np.zeros((2, n, 4), dtype=np.uint64), np.zeros((0, n, 4), dtype=np.uint64), [])
    return circ, wit, fill


def my_circuit(k=6, input_value=42):
    """The MyCircuit shape of halo2_proofs/tests/frontend_backend_split.rs:33-465 (WIDTH_FACTOR
    1, one synthesize_unit), compiled by hand: advice a, b, c (first phase), e (second phase);
    fixed d, s_lookup, s_ltable, s_shuffle, s_stable and the selectors s_gate, s_rlc as fixed
    columns (the frontend's selector compression is not restated); one instance column.
      gate_a   s_gate (a + b c d - a[next])
      lookup   [s_lookup, s_lookup a, s_lookup b] in [s_ltable, s_ltable d, s_ltable c]
      shuffle  [s_shuffle, s_shuffle a] ~ [s_stable, s_stable b]
      gate_rlc s_rlc (a + ch b - e), s_rlc (c + ch d - e)   (ch: a FirstPhase challenge)
    equality on a, b, d, instance; the unit's cells and copies as synthesize_unit assigns them
    (:236-409); the instance column is MyCircuit::instance() (:114-131).
    -> (circuit, instance-only witness, fill(phase, challenges) -> {column: values})"""
    n = 1 << k
    A, B, C, E = range(4)
    D, SL, ST, SS, SSt, SG, SR = range(7)
    ch = challenge(0)
    one = const(1)
    gates = [fixed(SG) * (advice(A) + advice(B) * advice(C) * fixed(D) - advice(A, 1)),
             fixed(SR) * (advice(A) + ch * advice(B) - advice(E)),
             fixed(SR) * (advice(C) + ch * fixed(D) - advice(E))]
    lookups = [([one * fixed(SL), advice(A) * fixed(SL), advice(B) * fixed(SL)],
                [one * fixed(ST), fixed(D) * fixed(ST), advice(C) * fixed(ST)])]
    shuffles = [([one * fixed(SS), advice(A) * fixed(SS)], [one * fixed(SSt), advice(B) * fixed(SSt)])]
    perm = [(ADVICE, A), (ADVICE, B), (FIXED, D), (INSTANCE, 0)]
    a, b, c = [0] * n, [0] * n, [0] * n
    fx = [[0] * n for _ in range(7)]
    rlc_rows = []
    copies = [(INSTANCE, 0, 0, ADVICE, A, 0)]   # assign_advice_from_instance(instance, 0, a, 0)
    off = 0

    def gate(av, bv, cv, dv):
        nonlocal off
        fx[SG][off] = 1
        if av is not None:
            a[off] = av
        b[off], c[off], fx[D][off] = bv, cv, dv
        a[off + 1] = (a[off] + bv * cv * dv) % R_MOD
        cells = (off, off)
        off += 1
        return cells

    a[0] = input_value
    inst_rows = []
    for bcd in ((3, 4, 1), (6, 7, 1), (8, 9, 1)):
        gate(None, *bcd)
        inst_rows.append((ADVICE, A, off))
    gate(None, 0xffffffff, 0xdeadbeef, 1)
    gate(None, 0xabad1d3a, 0x12345678, 0x42424242)
    off += 1
    r1 = off
    gate(5, 2, 1, 1)
    off += 1
    r2 = off
    gate(2, 3, 1, 1)
    off += 1
    r3 = off
    gate(4, 2, 1, 1)
    off += 1
    copies += [(ADVICE, B, r1, ADVICE, A, r2), (ADVICE, A, r2, ADVICE, B, r3)]
    inst_rows += [(ADVICE, B, r1), (ADVICE, A, r2)]
    r1 = off
    gate(5, 9, 1, 9)
    off += 1
    r2 = off
    gate(2, 9, 1, 1)
    off += 1
    r3 = off
    gate(9, 2, 1, 1)
    off += 1
    copies += [(ADVICE, B, r1, FIXED, D, r1), (ADVICE, B, r2, FIXED, D, r1), (ADVICE, A, r3, FIXED, D, r1)]
    lk = [(2, 4), (2, 4), (10, 1024), (0, 1), (2, 4)]
    for i in range(11):
        fx[SL][off] = fx[ST][off] = 1
        a[off], b[off] = lk[i] if i < len(lk) else (0, 1)
        fx[D][off], c[off] = i, 2 ** i
        off += 1
    for abcd in ((3, 5, 3, 5), (8, 9, 8, 9), (111, 222, 111, 222)):
        fx[SR][off] = 1
        rlc_rows.append((off, abcd[0], abcd[1]))
        gate(*abcd)
        off += 1
    shuf = [0, 2, 4, 6, 8, 10, 12, 14, 1, 3, 5, 7, 9, 11, 13, 15]
    for i in range(16):
        fx[SS][off] = fx[SSt][off] = 1
        a[off], b[off] = shuf[i], i
        off += 1
    # layouter.constrain_instance(instance_copy[i], instance, 1 + i)
    copies += [(t, col, r, INSTANCE, 0, 1 + i) for i, (t, col, r) in enumerate(inst_rows)]
    inst = [input_value]
    for bcd in ((3, 4, 1), (6, 7, 1), (8, 9, 1)):
        inst.append((inst[-1] + bcd[0] * bcd[1] * bcd[2]) % R_MOD)
    inst += [2, 2]
    circ = Circuit(k, 4, 7, 1, gates, perm, copies, np.stack([ints_to_mont(v) for v in fx]),
                   name=f"MyCircuit shape k={k}", lookups=lookups, shuffles=shuffles,
                   advice_phase=[0, 0, 0, 1], challenge_phase=[0])
    assert off <= circ.usable_rows(), "the unit must fit in the usable rows"
    wit = Witness(np.zeros((4, n, 4), dtype=np.uint64), ints_to_mont(inst + [0] * (n - len(inst)))[None],
                  [len(inst)])

    def e_values(chs):
        e = [0] * n
        for r, av, bv in rlc_rows:
            e[r] = (av + chs[0] * bv) % R_MOD
        return e

    def fill(phase, chs):
        if phase == 0:
            return {A: ints_to_mont(a), B: ints_to_mont(b), C: ints_to_mont(c)}
        return {E: ints_to_mont(e_values(chs))}

    def full(chs):
        return Witness(np.stack([ints_to_mont(v) for v in (a, b, c, e_values(chs))]), wit.instance,
                       wit.instance_lens)

    fill.full = full
    return circ, wit, fill


# OneNg (halo2_proofs/tests/frontend_backend_split.rs:477-489): a BlockRng whose every u32
# is 1, so every Fr::random is LE512(01 00 00 00 x 16) mod r
ONE_NG_FR = 0x0fdd950c1da3e00b1d2fb9cf61452b1ec0c9dfb910ecfb36b574601aedf0313b


class OneNg:
    """the reference's deterministic test RNG as an h2g_rng source (fill_bytes only)"""

    def fill_bytes(self, n):
        return (b"\x01\x00\x00\x00" * ((n + 3) // 4))[:n]


class OneNgFr(OneNg):
    """OneNg with F::random answered directly (the shim's random_fr path)"""

    def random_fr(self):
        return np.asarray(fr_to_limbs(ONE_NG_FR), dtype=np.uint64)
