"""Python restatement of halo2's verify_proof for BN254 / KZG / SHPLONK with the
Blake2b transcript.  TEST INFRASTRUCTURE ONLY: it pins the prover restatement
(oracle/c/prover.c) and, through it, the device prover, by the reference's own
relational test -- prove then verify (halo2_proofs/tests/plonk_api.rs,
frontend_backend_split.rs).

Restated reference code (paths relative to the reference root):
  verify_proof                     halo2_backend/src/plonk/verifier.rs:58-512
  vanishing verifier               halo2_backend/src/plonk/vanishing/verifier.rs:40-137
  permutation verifier             halo2_backend/src/plonk/permutation/verifier.rs:33-253
  VerifierSHPLONK::verify_proof    halo2_backend/src/poly/kzg/multiopen/shplonk/verifier.rs:45-140
  VerifierGWC::verify_proof        halo2_backend/src/poly/kzg/multiopen/gwc/verifier.rs:42-123, gwc.rs:25-50
  construct_intermediate_sets      halo2_backend/src/poly/kzg/multiopen/shplonk.rs:48-140
  l_i_range                        halo2_backend/src/poly/domain.rs:425-450
  DualMSM::check                   halo2_backend/src/poly/kzg/msm.rs:188-206
  permutation Assembly             halo2_backend/src/plonk/permutation/keygen.rs:16-213
  lookup / shuffle verifiers       halo2_backend/src/plonk/lookup/verifier.rs, shuffle/verifier.rs

Pairings: the test setup knows the SRS secret s, so the pairing equation
e(left, [s]G2) = e(right, G2) of DualMSM::check is decided by the BN254 optimal ate
pairing (pairing_ref.py) from the params' G2 elements when they are passed (`g2=`),
else exactly as [s]·left == right in G1 with the secret.  VK commitments are computed as [f(s)]G the same way.

Independent of the C code: field/curve arithmetic (Python ints), Blake2b (hashlib),
the permutation Assembly and the query collection are restated again here.
"""
import hashlib

from bn254_ref import G1_GEN, P, R, DELTA, Domain, eval_polynomial, g1_add, g1_mul, g1_neg

ADVICE, FIXED, INSTANCE = 0, 1, 2


class VerifyError(Exception):
    pass


# ----------------------------------------------------------------------------- transcript
class Blake2bRead:
    """Blake2bRead (transcript.rs:120-130,214-245): personal "Halo2-Transcript";
    prefixes challenge 0, point 1, scalar 2; squeeze = update([0]) then finalize a
    clone; points are compressed (x LE, bit 7 of byte 31 = y parity)."""

    def __init__(self, proof: bytes):
        self.h = hashlib.blake2b(digest_size=64, person=b"Halo2-Transcript")
        self.buf = proof
        self.pos = 0

    def squeeze(self) -> int:
        self.h.update(b"\x00")
        return int.from_bytes(self.h.copy().digest(), "little") % R

    def common_point(self, pt):
        if pt is None:
            raise VerifyError("point at infinity in transcript")
        self.h.update(b"\x01" + pt[0].to_bytes(32, "little") + pt[1].to_bytes(32, "little"))

    def common_scalar(self, s: int):
        self.h.update(b"\x02" + (s % R).to_bytes(32, "little"))

    def _take(self):
        if self.pos + 32 > len(self.buf):
            raise VerifyError("proof too short")
        b = self.buf[self.pos:self.pos + 32]
        self.pos += 32
        return b

    def read_point(self):
        b = bytearray(self._take())
        sign = b[31] >> 7
        b[31] &= 0x7F
        x = int.from_bytes(bytes(b), "little")
        if x >= P:
            raise VerifyError("x not canonical")
        t = (x * x * x + 3) % P
        y = pow(t, (P + 1) // 4, P)
        if y * y % P != t:
            raise VerifyError("not on curve")
        if (y & 1) != sign:
            y = P - y
        pt = (x, y)
        self.common_point(pt)
        return pt

    def read_scalar(self) -> int:
        v = int.from_bytes(self._take(), "little")
        if v >= R:
            raise VerifyError("scalar not canonical")
        self.common_scalar(v)
        return v


class Keccak256Read(Blake2bRead):
    """Keccak256Read (transcript.rs:109-150,248-288): the state starts with
    "Halo2-Transcript"; the same prefixes; squeeze = update([0]), then two clones
    finalized after the extra bytes 10 and 11 (not kept in the state) give the low and
    high 32 of the 64 uniform bytes.  Keccak-256 from keccak_ref (Python ints)."""

    def __init__(self, proof: bytes):
        from keccak_ref import Keccak
        self.h = Keccak(0x01).update(b"Halo2-Transcript")
        self.buf = proof
        self.pos = 0

    def squeeze(self) -> int:
        self.h.update(b"\x00")
        lo = self.h.copy().update(b"\x0a").digest()
        hi = self.h.copy().update(b"\x0b").digest()
        return int.from_bytes(lo + hi, "little") % R


TRANSCRIPTS = {"blake2b": Blake2bRead, "keccak256": Keccak256Read}


# ----------------------------------------------------------------------------- keygen restated
def permutation_mapping(circ):
    """Assembly::copy over the copies in order (permutation/keygen.rs:48-97);
    returns mapping[col][row] = (col', row')."""
    n = circ.n
    cols = circ.perm_columns
    pos = {c: i for i, c in enumerate(cols)}
    mapping = [[(c, r) for r in range(n)] for c in range(len(cols))]
    aux = [[(c, r) for r in range(n)] for c in range(len(cols))]
    sizes = [[1] * n for _ in range(len(cols))]
    for lt, li, lr, rt, ri, rr in circ.copies.tolist():
        lc, rc = pos[(lt, li)], pos[(rt, ri)]
        lcyc, rcyc = aux[lc][lr], aux[rc][rr]
        if lcyc == rcyc:
            continue
        if sizes[lcyc[0]][lcyc[1]] < sizes[rcyc[0]][rcyc[1]]:
            lcyc, rcyc = rcyc, lcyc
        sizes[lcyc[0]][lcyc[1]] += sizes[rcyc[0]][rcyc[1]]
        i = rcyc
        while True:
            aux[i[0]][i[1]] = lcyc
            i = mapping[i[0]][i[1]]
            if i == rcyc:
                break
        mapping[lc][lr], mapping[rc][rr] = mapping[rc][rr], mapping[lc][lr]
    return mapping


def sigma_values(circ, dom):
    """permutation polynomials in Lagrange form: delta^col' * omega^row'"""
    mapping = permutation_mapping(circ)
    wp = [1] * circ.n
    for i in range(1, circ.n):
        wp[i] = wp[i - 1] * dom.omega % R
    dp = [pow(DELTA, i, R) for i in range(len(circ.perm_columns) + 1)]
    return [[dp[c] * wp[r] % R for (c, r) in col] for col in mapping]


def lagrange_at(dom, s):
    """L_i(s) for all i (the scalars behind g_lagrange)"""
    n = dom.n
    mult = (pow(s, n, R) - 1) * pow(n, -1, R) % R
    out, w = [], 1
    for _ in range(n):
        out.append(mult * w % R * pow((s - w) % R, -1, R) % R)
        w = w * dom.omega % R
    return out


def rotate_omega(dom, x, rot):
    return x * pow(dom.omega if rot >= 0 else dom.omega_inv, abs(rot), R) % R


def l_i_range(dom, x, xn, rotations):
    common = (xn - 1) * dom.barycentric_weight % R
    out = []
    for rot in rotations:
        w = rotate_omega(dom, 1, rot)
        out.append(rotate_omega(dom, pow((x - w) % R, -1, R) * common % R, rot))
    return out


def vanishing_poly_eval(points, z):
    acc = 1
    for p in points:
        acc = acc * (z - p) % R
    return acc


def lagrange_interpolate(points, evals):
    m = len(points)
    coeffs = [0] * m
    for j in range(m):
        num = [1]
        den = 1
        for k in range(m):
            if k == j:
                continue
            num = [((num[i - 1] if i > 0 else 0) - points[k] * (num[i] if i < len(num) else 0)) % R
                   for i in range(len(num) + 1)]
            den = den * (points[j] - points[k]) % R
        sc = evals[j] * pow(den, -1, R) % R
        for i in range(m):
            coeffs[i] = (coeffs[i] + num[i] * sc) % R
    return coeffs


# ----------------------------------------------------------------------------- MSM helper
class Msm:
    """linear combination of points (MSMKZG), evaluated exactly"""

    def __init__(self):
        self.terms = []

    def add(self, scalar, pt):
        self.terms.append([scalar % R, pt])

    def add_msm(self, other):
        self.terms.extend([list(t) for t in other.terms])

    def scale(self, f):
        for t in self.terms:
            t[0] = t[0] * f % R

    def eval(self):
        acc = None
        for s, pt in self.terms:
            acc = g1_add(acc, g1_mul(pt, s))
        return acc


# ----------------------------------------------------------------------------- verify
def affine_from_limbs(a):
    """G1Affine in the halo2curves layout (8 u64 Montgomery limbs; identity = zeros) ->
    (x, y) ints or None"""
    from bn254_ref import from_limbs, from_mont
    a = [int(v) for v in a]
    if not any(a):
        return None
    return (from_mont(from_limbs(a[:4]), P), from_mont(from_limbs(a[4:8]), P))


def verify(circ, instances, proof: bytes, s: int, instance_lens=None, multiopen="shplonk", vk=None,
           instances_multi=None, transcript="blake2b", g2=None):
    """Returns True iff the proof verifies (raises VerifyError on malformed input).
    multiopen: "shplonk" (VerifierSHPLONK) or "gwc" (VerifierGWC).
    transcript: "blake2b" (Blake2bRead) or "keccak256" (Keccak256Read).
    g2: the params' (g2, s_g2) as G2 affine int pairs: DualMSM::check is then decided by
    the pairing equation e(left, s_g2) == e(right, g2) (pairing_ref) as the reference
    does, and s is needed only to compute the VK when `vk` is not given.
    vk: optional (fixed commitments, permutation commitments) -- each a list of (x, y) ints
    or 8-limb affine arrays -- taken instead of recomputing [f(s)]G here (large k).
    instances_multi: per-circuit instance columns of a proof over several circuits
    (verify_proof's instances: &[&[&[F]]], verifier.rs:58-140); `instances` is then unused."""
    from h2g_circuit import fr_from_limbs
    adv_q, fix_q, ins_q = circ.queries()
    degree = circ.degree()
    bf = circ.blinding_factors()
    dom = Domain(degree, circ.k)
    n = circ.n
    chunk_len = degree - 2
    nsets = (len(circ.perm_columns) + chunk_len - 1) // chunk_len
    insts = instances_multi if instances_multi is not None else [instances]
    NC = len(insts)

    # vk: fixed and permutation commitments, [f(s)]G
    if vk is not None:
        def pt(c):
            return c if c is None or isinstance(c, tuple) else affine_from_limbs(c)
        fixed_cm = [pt(c) for c in vk[0]]
        sigma_cm = [pt(c) for c in vk[1]]
        if len(fixed_cm) != circ.num_fixed or len(sigma_cm) != len(circ.perm_columns):
            raise VerifyError("verifying key does not match the circuit")
    else:
        L = lagrange_at(dom, s)

        def commit_lagrange(vals):
            acc = 0
            for v, l in zip(vals, L):
                if v:
                    acc = (acc + v * l) % R
            return g1_mul(G1_GEN, acc)

        fixed_vals = [[fr_from_limbs(r) for r in col] for col in circ.fixed_values]
        fixed_cm = [commit_lagrange(v) for v in fixed_vals]
        sig = sigma_values(circ, dom)
        sigma_cm = [commit_lagrange(v) for v in sig]

    T = TRANSCRIPTS[transcript](proof)
    T.common_scalar(fr_from_limbs(circ.transcript_repr()))
    for inst in insts:
        for col in inst:
            for v in col:
                T.common_scalar(v)
    # advice commitments per phase, circuit by circuit, each phase followed by its
    # challenges (verifier.rs:104-140)
    adv_cm = [[None] * circ.num_advice for _ in range(NC)]
    chal = [0] * circ.num_challenges
    for ph in range(circ.max_phase + 1):
        for c in range(NC):
            for col in range(circ.num_advice):
                if int(circ.advice_phase[col]) == ph:
                    adv_cm[c][col] = T.read_point()
        for i in range(circ.num_challenges):
            if int(circ.challenge_phase[i]) == ph:
                chal[i] = T.squeeze()
    theta = T.squeeze()
    lk_perm_cm = [[(T.read_point(), T.read_point()) for _ in circ.lookups] for _ in range(NC)]   # A', S'
    beta = T.squeeze()
    gamma = T.squeeze()
    perm_cm = [[T.read_point() for _ in range(nsets)] for _ in range(NC)]
    lk_z_cm = [[T.read_point() for _ in circ.lookups] for _ in range(NC)]
    sh_z_cm = [[T.read_point() for _ in circ.shuffles] for _ in range(NC)]
    random_cm = T.read_point()
    y = T.squeeze()
    h_cm = [T.read_point() for _ in range(dom.quotient_poly_degree)]
    x = T.squeeze()
    xn = pow(x, n, R)
    # instance evals (QUERY_INSTANCE = false): inner product with l_i_range
    rots = [r for (_, r) in ins_q] or [0]
    min_rot, max_rot = min(0, min(rots)), max(0, max(rots))
    max_len = max([len(c) for inst in insts for c in inst] or [0])
    l_is = l_i_range(dom, x, xn, range(-max_rot, max_len + abs(min_rot)))
    ins_evals = []
    for inst in insts:
        ev_c = []
        for (col, rot) in ins_q:
            off = max_rot - rot
            vals = inst[col]
            ev_c.append(sum(v * l for v, l in zip(vals, l_is[off:off + len(vals)])) % R)
        ins_evals.append(ev_c)
    adv_evals = [[T.read_scalar() for _ in adv_q] for _ in range(NC)]
    fix_evals = [T.read_scalar() for _ in fix_q]
    random_eval = T.read_scalar()
    perm_evals = [T.read_scalar() for _ in circ.perm_columns]
    sets = []
    for _ in range(NC):
        sc = []
        for i in range(nsets):
            e0 = T.read_scalar()
            e1 = T.read_scalar()
            e2 = T.read_scalar() if i + 1 < nsets else None
            sc.append((e0, e1, e2))
        sets.append(sc)
    lk_ev = [[tuple(T.read_scalar() for _ in range(5)) for _ in circ.lookups] for _ in range(NC)]   # z, z_next, A', A'_inv, S'
    sh_ev = [[tuple(T.read_scalar() for _ in range(2)) for _ in circ.shuffles] for _ in range(NC)]  # z, z_next

    # vanishing argument: every circuit's expressions at x, one Horner chain in y
    l_evals = l_i_range(dom, x, xn, range(-(bf + 1), 1))
    l_last, l_blind, l_0 = l_evals[0], sum(l_evals[1:1 + bf]) % R, l_evals[1 + bf]
    active = (1 - (l_last + l_blind)) % R
    exprs = []
    for c in range(NC):
        def qeval(t, i, r, c=c):
            if t == ADVICE:
                return adv_evals[c][adv_q.index((i, r))]
            if t == FIXED:
                return fix_evals[fix_q.index((i, r))]
            return ins_evals[c][ins_q.index((i, r))]

        exprs += [g.evaluate(lambda v: v, qeval, challenge=lambda i: chal[i]) for g in circ.gates]
        st = sets[c]
        if nsets:
            exprs.append(l_0 * (1 - st[0][0]) % R)
            exprs.append((st[-1][0] * st[-1][0] - st[-1][0]) * l_last % R)
            for i in range(1, nsets):
                exprs.append((st[i][0] - st[i - 1][2]) * l_0 % R)
            for ci in range(nsets):
                cols = circ.perm_columns[ci * chunk_len:(ci + 1) * chunk_len]
                pev = perm_evals[ci * chunk_len:(ci + 1) * chunk_len]
                left = st[ci][1]
                for (t, i), pe in zip(cols, pev):
                    left = left * (qeval(t, i, 0) + beta * pe + gamma) % R
                right = st[ci][0]
                cur = beta * x % R * pow(DELTA, ci * chunk_len, R) % R
                for (t, i) in cols:
                    right = right * (qeval(t, i, 0) + cur + gamma) % R
                    cur = cur * DELTA % R
                exprs.append((left - right) * active % R)

        def compress(es, qeval=qeval):
            acc = 0
            for e in es:
                acc = (acc * theta + e.evaluate(lambda v: v, qeval, challenge=lambda i: chal[i])) % R
            return acc

        for (ins_e, tab_e), (z, zn, ap, api, sp) in zip(circ.lookups, lk_ev[c]):   # lookup/verifier.rs:98-160
            exprs.append(l_0 * (1 - z) % R)
            exprs.append(l_last * (z * z - z) % R)
            left = zn * (ap + beta) % R * (sp + gamma) % R
            right = z * (compress(ins_e) + beta) % R * (compress(tab_e) + gamma) % R
            exprs.append((left - right) * active % R)
            exprs.append(l_0 * (ap - sp) % R)
            exprs.append((ap - sp) * (ap - api) % R * active % R)
        for (ins_e, sh_e), (z, zn) in zip(circ.shuffles, sh_ev[c]):   # shuffle/verifier.rs
            exprs.append(l_0 * (1 - z) % R)
            exprs.append(l_last * (z * z - z) % R)
            exprs.append(active * (zn * (compress(sh_e) + gamma) - z * (compress(ins_e) + gamma)) % R)
    h_eval = 0
    for v in exprs:
        h_eval = (h_eval * y + v) % R
    expected_h_eval = h_eval * pow((xn - 1) % R, -1, R) % R
    h_msm = Msm()
    for c in reversed(h_cm):
        h_msm.scale(xn)
        h_msm.add(1, c)

    # queries: (key, commitment-or-msm, point, eval), circuit by circuit then the common ones
    x_next = rotate_omega(dom, x, 1)
    x_last = rotate_omega(dom, x, -(bf + 1))
    x_prev = rotate_omega(dom, x, -1)
    queries = []
    for c in range(NC):
        for qi, (col, rot) in enumerate(adv_q):
            queries.append((("adv", c, col), adv_cm[c][col], rotate_omega(dom, x, rot), adv_evals[c][qi]))
        for i in range(nsets):
            queries.append((("z", c, i), perm_cm[c][i], x, sets[c][i][0]))
            queries.append((("z", c, i), perm_cm[c][i], x_next, sets[c][i][1]))
        for i in reversed(range(nsets - 1)):
            queries.append((("z", c, i), perm_cm[c][i], x_last, sets[c][i][2]))
        for l, (zc, (apc, spc), (z, zn, ap, api, sp)) in enumerate(zip(lk_z_cm[c], lk_perm_cm[c], lk_ev[c])):
            queries.append((("lz", c, l), zc, x, z))
            queries.append((("la", c, l), apc, x, ap))
            queries.append((("ls", c, l), spc, x, sp))
            queries.append((("la", c, l), apc, x_prev, api))
            queries.append((("lz", c, l), zc, x_next, zn))
        for l, (zc, (z, zn)) in enumerate(zip(sh_z_cm[c], sh_ev[c])):
            queries.append((("sz", c, l), zc, x, z))
            queries.append((("sz", c, l), zc, x_next, zn))
    for qi, (col, rot) in enumerate(fix_q):
        queries.append((("fix", col), fixed_cm[col], rotate_omega(dom, x, rot), fix_evals[qi]))
    for i in range(len(circ.perm_columns)):
        queries.append((("sigma", i), sigma_cm[i], x, perm_evals[i]))
    queries.append((("h",), h_msm, x, expected_h_eval))
    queries.append((("random",), random_cm, x, random_eval))

    if multiopen == "gwc":
        return _verify_gwc(T, queries, proof, s, g2)

    # SHPLONK (construct_intermediate_sets + VerifierSHPLONK::verify_proof)
    super_points = sorted({q[2] for q in queries})
    order, cm_points, cm_obj, evals = [], {}, {}, {}
    for key, obj, pt, ev in queries:
        if key not in cm_points:
            order.append(key)
            cm_points[key] = set()
            cm_obj[key] = obj
        cm_points[key].add(pt)
        evals[(key, pt)] = ev
    rot_sets = []   # [(points sorted, [keys])]
    for key in order:
        pts = sorted(cm_points[key])
        for rs in rot_sets:
            if rs[0] == pts:
                rs[1].append(key)
                break
        else:
            rot_sets.append((pts, [key]))
    sy = T.squeeze()
    v = T.squeeze()
    h1 = T.read_point()
    u = T.squeeze()
    h2 = T.read_point()
    z0_diff_inv = z0 = 0
    outer = Msm()
    r_outer = 0
    vpow = 1
    for i, (pts, keys) in enumerate(rot_sets):
        diffs = [p for p in super_points if p not in pts]
        z_diff = vanishing_poly_eval(diffs, u)
        if i == 0:
            z0 = vanishing_poly_eval(pts, u)
            z0_diff_inv = pow(z_diff, -1, R)
            z_diff = 1
        else:
            z_diff = z_diff * z0_diff_inv % R
        inner = Msm()
        r_inner = 0
        ypow = 1
        for key in keys:
            r_x = lagrange_interpolate(pts, [evals[(key, p)] for p in pts])
            r_inner = (r_inner + ypow * eval_polynomial(r_x, u)) % R
            obj = cm_obj[key]
            if isinstance(obj, Msm):
                m = Msm()
                m.add_msm(obj)
                m.scale(ypow)
                inner.add_msm(m)
            else:
                inner.add(ypow, obj)
            ypow = ypow * sy % R
        inner.scale(vpow * z_diff)
        outer.add_msm(inner)
        r_outer = (r_outer + vpow * r_inner % R * z_diff) % R
        vpow = vpow * v % R
    outer.add(-r_outer, G1_GEN)
    outer.add(-z0, h1)
    outer.add(u, h2)
    if T.pos != len(proof):
        raise VerifyError(f"trailing proof bytes: read {T.pos} of {len(proof)}")
    right = outer.eval()
    return _dual_msm_check(h2, right, s, g2)


def g2_from_limbs(a):
    """a G2 affine point from 16 u64 (x.c0, x.c1, y.c0, y.c1, Montgomery limbs; the layout of
    h2g_params_g2 and of halo2curves' G2Affine)"""
    from bn254_ref import from_limbs, from_mont
    v = [from_mont(from_limbs([int(t) for t in a[4 * i:4 * i + 4]]), P) for i in range(4)]
    return (v[0], v[1]), (v[2], v[3])


def _dual_msm_check(left, right, s, g2):
    """DualMSM::check: e(left, [s]G2) == e(right, G2) -- by the pairing when the params'
    G2 elements are given, else exactly as [s] left == right with the secret"""
    if g2 is None:
        return g1_mul(left, s) == right
    from pairing_ref import pairing_check
    g2_gen, s_g2 = g2
    return pairing_check([(left, s_g2), (g1_neg(right) if right is not None else None, g2_gen)])


def _verify_gwc(T, queries, proof, s, g2=None):
    """VerifierGWC::verify_proof (gwc/verifier.rs:42-123): queries grouped by point in
    first-appearance order (gwc.rs:25-50); one witness point per group; then
    DualMSM::check, decided as [s]·left == right."""
    v = T.squeeze()
    groups = []  # [(point, [(commitment-or-msm, eval)])]
    for _key, obj, pt, ev in queries:
        for g in groups:
            if g[0] == pt:
                g[1].append((obj, ev))
                break
        else:
            groups.append((pt, [(obj, ev)]))
    ws = [T.read_point() for _ in groups]
    u = T.squeeze()
    if T.pos != len(proof):
        raise VerifyError(f"trailing proof bytes: read {T.pos} of {len(proof)}")
    commitment_multi, eval_multi = Msm(), 0
    left, right = Msm(), Msm()
    upow = 1
    for (z, items), wi in zip(groups, ws):
        batch, evb, vpow = Msm(), 0, 1
        for obj, ev in items:
            m = Msm()
            if isinstance(obj, Msm):
                m.add_msm(obj)
            else:
                m.add(1, obj)
            m.scale(vpow)
            batch.add_msm(m)
            evb = (evb + vpow * ev) % R
            vpow = vpow * v % R
        batch.scale(upow)
        commitment_multi.add_msm(batch)
        eval_multi = (eval_multi + upow * evb) % R
        right.add(upow * z, wi)   # witness_with_aux
        left.add(upow, wi)        # witness
        upow = upow * u % R
    right.add_msm(commitment_multi)
    right.add(-eval_multi, G1_GEN)
    return _dual_msm_check(left.eval(), right.eval(), s, g2)


def sigma_lagrange(circ):
    """exported for the keygen parity test (C keygen vs this restatement)"""
    return sigma_values(circ, Domain(circ.degree(), circ.k))
