"""ctypes view of the C restatement oracle (oracle/build/liboracle.so).

Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module.  All arrays are numpy uint64 in the
halo2curves layout (Montgomery limbs; Fr = 4 limbs, G1Affine = 8 limbs).
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(REPO, "oracle", "build", "liboracle.so")

_lib = None
U64P = ctypes.POINTER(ctypes.c_uint64)


def _p(a):
    if a is None:
        return None
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data_as(U64P)


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u64, u32, i32 = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        sig = {
            "or_g1_is_on_curve": ([U64P], i32),
            "or_g1_mul": ([U64P, U64P, U64P], None),
            "or_g1_add": ([U64P, U64P, U64P], None),
            "or_srs_powers": ([U64P, u64, U64P], None),
            "or_msm_naive": ([U64P, U64P, u64, U64P], None),
            "or_msm_best": ([U64P, U64P, u64, i32, U64P], None),
            "or_fft": ([U64P, u32, U64P, i32], None),
            "or_domain_constants": ([u32, u32, U64P, U64P], u32),
            "or_lagrange_to_coeff": ([U64P, u32, u32, i32], None),
            "or_coeff_to_extended": ([U64P, U64P, u32, u32, i32], None),
            "or_extended_to_coeff": ([U64P, U64P, u32, u32, i32], None),
            "or_divide_by_vanishing_poly": ([U64P, u32, u32], None),
            "or_fr_add": ([U64P, U64P, U64P, u64], None),
            "or_fr_sub": ([U64P, U64P, U64P, u64], None),
            "or_fr_mul": ([U64P, U64P, U64P, u64], None),
            "or_fr_scale": ([U64P, U64P, U64P, u64], None),
            "or_fr_from_canonical": ([U64P, U64P, u64], None),
            "or_fr_to_canonical": ([U64P, U64P, u64], None),
            "or_fq_from_canonical": ([U64P, U64P, u64], None),
            "or_fr_eval": ([U64P, u64, U64P, U64P], None),
            "or_kate_division": ([U64P, u64, U64P, U64P], None),
            "or_fr_batch_invert": ([U64P, u64], None),
            "or_fr_prefix_product": ([U64P, U64P, u64], None),
            "or_num_threads": ([], i32),
            "or_keygen": ([ctypes.c_void_p, i32], ctypes.c_void_p),
            "or_prove": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p, u64, U64P, i32], i32),
            "or_pk_free": ([ctypes.c_void_p], None),
            "or_pk_info": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)], None),
            "or_pk_sigma": ([ctypes.c_void_p, i32, U64P], None),
            "or_create_proof": ([ctypes.c_void_p, ctypes.c_char_p, u64, U64P, i32], i32),
            "or_srs_lagrange": ([U64P, u32, U64P], None),
            "or_blake2b": ([ctypes.c_char_p, u64, ctypes.c_char_p, ctypes.c_char_p], None),
            "or_chacha20_block": ([ctypes.c_char_p, u64, ctypes.c_char_p], None),
            "or_keccak": ([ctypes.c_char_p, u64, ctypes.c_uint8, ctypes.c_char_p], None),
            "or_fr_random_stream": ([ctypes.c_char_p, u64, U64P], None),
            "or_set_kernel_threads": ([i32], None),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def keccak(data, pad=0x01):
    """the oracle's Keccak sponge: pad 0x01 = Keccak-256, 0x06 = SHA3-256"""
    out = ctypes.create_string_buffer(32)
    lib().or_keccak(bytes(data), len(data), pad, out)
    return out.raw


def fr_arr(n):
    return np.zeros((n, 4), dtype=np.uint64)


def msm_naive(scalars, bases):
    out = np.zeros(8, dtype=np.uint64)
    lib().or_msm_naive(_p(np.ascontiguousarray(scalars)), _p(np.ascontiguousarray(bases)), len(scalars), _p(out))
    return out


def msm_best(scalars, bases, threads=1):
    out = np.zeros(8, dtype=np.uint64)
    lib().or_msm_best(_p(np.ascontiguousarray(scalars)), _p(np.ascontiguousarray(bases)), len(scalars), threads, _p(out))
    return out


def fft(a, omega, threads=1):
    a = np.ascontiguousarray(a.copy())
    k = int(len(a)).bit_length() - 1
    lib().or_fft(_p(a), k, _p(np.ascontiguousarray(omega)), threads)
    return a


def domain_constants(j, k):
    c = np.zeros((9, 4), dtype=np.uint64)
    t = np.zeros((1 << 12, 4), dtype=np.uint64)
    ek = lib().or_domain_constants(j, k, _p(c), _p(t))
    return ek, c, t[: 1 << (ek - k)].copy()


def lagrange_to_coeff(a, j, k, threads=1):
    a = np.ascontiguousarray(a.copy())
    lib().or_lagrange_to_coeff(_p(a), j, k, threads)
    return a


def coeff_to_extended(a, j, k, threads=1):
    ek = domain_constants(j, k)[0]
    out = fr_arr(1 << ek)
    lib().or_coeff_to_extended(_p(np.ascontiguousarray(a)), _p(out), j, k, threads)
    return out


def extended_to_coeff(a, j, k, threads=1):
    a = np.ascontiguousarray(a.copy())
    out = fr_arr((1 << k) * (j - 1))
    lib().or_extended_to_coeff(_p(a), _p(out), j, k, threads)
    return out


def divide_by_vanishing_poly(a, j, k):
    a = np.ascontiguousarray(a.copy())
    lib().or_divide_by_vanishing_poly(_p(a), j, k)
    return a


def binop(name, a, b):
    out = fr_arr(len(a))
    getattr(lib(), name)(_p(np.ascontiguousarray(a)), _p(np.ascontiguousarray(b)), _p(out), len(a))
    return out


def scale(a, x):
    out = fr_arr(len(a))
    lib().or_fr_scale(_p(np.ascontiguousarray(a)), _p(np.ascontiguousarray(x)), _p(out), len(a))
    return out


def eval_poly(a, x):
    out = np.zeros(4, dtype=np.uint64)
    lib().or_fr_eval(_p(np.ascontiguousarray(a)), len(a), _p(np.ascontiguousarray(x)), _p(out))
    return out


def kate_division(a, b):
    q = fr_arr(len(a) - 1)
    lib().or_kate_division(_p(np.ascontiguousarray(a)), len(a), _p(np.ascontiguousarray(b)), _p(q))
    return q


def batch_invert(a):
    a = np.ascontiguousarray(a.copy())
    lib().or_fr_batch_invert(_p(a), len(a))
    return a


def prefix_product(a):
    out = fr_arr(len(a))
    lib().or_fr_prefix_product(_p(np.ascontiguousarray(a)), _p(out), len(a))
    return out


def srs_powers(s, n):
    out = np.zeros((n, 8), dtype=np.uint64)
    lib().or_srs_powers(_p(np.ascontiguousarray(s)), n, _p(out))
    return out


def g1_mul(pt, s):
    out = np.zeros(8, dtype=np.uint64)
    lib().or_g1_mul(_p(np.ascontiguousarray(pt)), _p(np.ascontiguousarray(s)), _p(out))
    return out


def g1_add(a, b):
    out = np.zeros(8, dtype=np.uint64)
    lib().or_g1_add(_p(np.ascontiguousarray(a)), _p(np.ascontiguousarray(b)), _p(out))
    return out


def fr_from_canonical(c):
    c = np.ascontiguousarray(c, dtype=np.uint64).reshape(-1, 4)
    out = fr_arr(len(c))
    lib().or_fr_from_canonical(_p(c), _p(out), len(c))
    return out


def random_fr(rng, n):
    """Uniform-ish Fr elements (Montgomery form) from a numpy Generator: canonical
    values below 2^253 < r, then converted to Montgomery form by the oracle."""
    c = rng.integers(0, 2**63, size=(n, 4), dtype=np.int64).astype(np.uint64)
    c[:, 3] &= np.uint64((1 << 61) - 1)  # < 2^253 < r
    c[:, 0] = rng.integers(0, 2**63, size=n, dtype=np.int64).astype(np.uint64) * np.uint64(2) + (c[:, 0] & np.uint64(1))
    return fr_from_canonical(c)


# ----------------------------------------------------------------------------- prover
I32P = ctypes.POINTER(ctypes.c_int32)
U8P = ctypes.POINTER(ctypes.c_uint8)
U32P = ctypes.POINTER(ctypes.c_uint32)


class OrSpec(ctypes.Structure):
    """struct or_spec (oracle/c/prover.c)"""
    _fields_ = [
        ("k", ctypes.c_uint32), ("num_advice", ctypes.c_uint32), ("num_fixed", ctypes.c_uint32),
        ("num_instance", ctypes.c_uint32),
        ("num_gates", ctypes.c_uint32), ("gate_roots", I32P),
        ("num_nodes", ctypes.c_uint32), ("nodes", I32P),
        ("num_constants", ctypes.c_uint32), ("constants", U64P),
        ("num_perm_columns", ctypes.c_uint32), ("perm_columns", I32P),
        ("num_copies", ctypes.c_uint32), ("copies", I32P),
        ("fixed_values", U64P), ("advice_values", U64P), ("instance_values", U64P),
        ("instance_lens", U32P), ("transcript_repr", U64P), ("rng_seed", U8P),
        ("vanishing_threads", ctypes.c_uint32), ("srs_g", U64P), ("srs_g_lagrange", U64P),
        ("unblinded", U8P),
        ("num_lookups", ctypes.c_uint32), ("lookup_sizes", U32P), ("lookup_roots", I32P),
        ("num_shuffles", ctypes.c_uint32), ("shuffle_sizes", U32P), ("shuffle_roots", I32P),
        ("multiopen", ctypes.c_uint32),
        ("advice_phase", U8P), ("num_challenges", ctypes.c_uint32), ("challenge_phase", U8P),
        ("fill", ctypes.c_void_p), ("fill_ctx", ctypes.c_void_p), ("challenges_out", U64P),
        ("challenge_values", U64P),
        ("num_circuits", ctypes.c_uint32), ("advice_c", ctypes.POINTER(ctypes.c_void_p)),
        ("instance_c", ctypes.POINTER(ctypes.c_void_p)), ("instance_lens_c", ctypes.POINTER(ctypes.c_void_p)),
        ("fill_multi", ctypes.c_void_p),
        ("rng_fill_bytes", ctypes.c_void_p), ("rng_random_fr", ctypes.c_void_p), ("rng_ctx", ctypes.c_void_p),
        ("transcript", ctypes.c_uint32),
    ]


MULTIOPEN = {"shplonk": 0, "gwc": 1}


def _ptr(a, t):
    return a.ctypes.data_as(t) if a is not None and a.size else None


def make_spec(circ, wit, srs_g, srs_gl, seed=bytes([7] * 32), vanishing_threads=8, multiopen="shplonk"):
    """Builds the or_spec; returns (struct, keepalive list)."""
    keep = [np.ascontiguousarray(x) for x in (
        circ.gate_roots, circ.nodes, circ.constants, circ.perm_array, circ.copies, circ.fixed_values,
        wit.advice, wit.instance, wit.instance_lens, circ.transcript_repr(),
        np.frombuffer(bytes(seed), dtype=np.uint8).copy(), srs_g, srs_gl, circ.unblinded,
        circ.lookup_sizes, circ.lookup_roots, circ.shuffle_sizes, circ.shuffle_roots, circ.advice_phase,
        circ.challenge_phase)]
    (roots, nodes, consts, perm, copies, fixed, adv, ins, lens, tr, sd, g, gl, unb, lks, lkr, shs, shr, aph,
     chph) = keep
    s = OrSpec(circ.k, circ.num_advice, circ.num_fixed, circ.num_instance,
               len(roots), _ptr(roots, I32P), len(nodes), _ptr(nodes, I32P),
               circ.num_constants, _ptr(consts, U64P), len(perm), _ptr(perm, I32P),
               len(copies), _ptr(copies, I32P), _ptr(fixed, U64P), _ptr(adv, U64P), _ptr(ins, U64P),
               _ptr(lens, U32P), _ptr(tr, U64P), _ptr(sd, U8P), vanishing_threads,
               _ptr(g, U64P), _ptr(gl, U64P), _ptr(unb, U8P),
               len(circ.lookups), _ptr(lks, U32P), _ptr(lkr, I32P),
               len(circ.shuffles), _ptr(shs, U32P), _ptr(shr, I32P), MULTIOPEN[multiopen],
               _ptr(aph, U8P), circ.num_challenges, _ptr(chph, U8P), None, None, None, None,
               0, None, None, None, None, None, None, None)
    return s, keep


def srs_lagrange(s, k):
    out = np.zeros((1 << k, 8), dtype=np.uint64)
    lib().or_srs_lagrange(_p(np.ascontiguousarray(s)), k, _p(out))
    return out


_SRS_CACHE = {}


def srs(k, s_int=None):
    """(s (Montgomery limbs), g, g_lagrange) for a known toxic s (test setup)."""
    import h2g_circuit as hc
    if s_int is None:
        s_int = 0x1234567890ABCDEF1122334455667788 * 3 + k
    key = (k, s_int)
    if key not in _SRS_CACHE:
        s = np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64)
        _SRS_CACHE[key] = (s_int, srs_powers(s, 1 << k), srs_lagrange(s, k))
    return _SRS_CACHE[key]


class Keygen:
    def __init__(self, circ, wit, srs_g, srs_gl, threads=8):
        self.spec, self.keep = make_spec(circ, wit, srs_g, srs_gl)
        self.pk = lib().or_keygen(ctypes.byref(self.spec), threads)
        if not self.pk:
            raise ValueError("or_keygen failed")
        info = (ctypes.c_int32 * 8)()
        lib().or_pk_info(self.pk, info)
        self.degree, self.bf, self.extended_k, self.P, self.n_adv_q, self.n_fix_q, self.n_ins_q, self.nsets = list(info)
        self.n = 1 << circ.k

    def sigma(self, i):
        out = np.zeros((self.n, 4), dtype=np.uint64)
        lib().or_pk_sigma(self.pk, i, _p(out))
        return out

    def close(self):
        if self.pk:
            lib().or_pk_free(self.pk)
            self.pk = None

    def __del__(self):
        self.close()


def create_proof(circ, wit, srs_g, srs_gl, seed=bytes([7] * 32), vanishing_threads=8, threads=8, keygen=None,
                 multiopen="shplonk", fill=None, challenges_out=None, wits=None, rng=None, fills=None,
                 transcript="blake2b"):
    """Oracle create_proof -> proof bytes (multiopen: "shplonk" = ProverSHPLONK, "gwc" = ProverGWC).
    fill: the per-phase witness source fill(phase, challenges) -> {column: values}
    (h2g.witness_fill); challenges_out: a list that receives the squeezed challenges.
    wits: several circuits' witnesses in one proof (create_proof's circuits: &[C]; `wit`
    is then only used for the spec's shapes), fills: their per-circuit witness sources;
    rng: the caller's RngCore (fill_bytes(n), optionally random_fr()) instead of the seed.
    transcript: "blake2b" (Blake2bWrite) or "keccak256" (Keccak256Write)."""
    spec, keep = make_spec(circ, wit, srs_g, srs_gl, seed, vanishing_threads, multiopen)
    spec.transcript = {"blake2b": 0, "keccak256": 1}[transcript]
    ch = np.zeros((max(circ.num_challenges, 1), 4), dtype=np.uint64)
    spec.challenges_out = _ptr(ch, U64P)
    import h2g
    if fill is not None:
        cb = h2g.witness_fill(circ.num_advice, circ.n, fill)
        cb.num_challenges = circ.num_challenges
        cfn = h2g.WITNESS_FILL(cb)
        keep.append(cfn)
        spec.fill = ctypes.cast(cfn, ctypes.c_void_p)
    if wits is not None:
        nc = len(wits)
        arrs = [(ctypes.c_void_p * nc)() for _ in range(3)]
        for c, w in enumerate(wits):
            a = np.ascontiguousarray(w.advice, dtype=np.uint64)
            ins = np.ascontiguousarray(w.instance, dtype=np.uint64) if circ.num_instance else np.zeros(4, np.uint64)
            ln_ = np.ascontiguousarray(w.instance_lens if circ.num_instance else np.zeros(1), dtype=np.uint32)
            keep += [a, ins, ln_]
            arrs[0][c], arrs[1][c], arrs[2][c] = a.ctypes.data, ins.ctypes.data, ln_.ctypes.data
        keep += arrs
        spec.num_circuits = nc
        spec.advice_c, spec.instance_c, spec.instance_lens_c = (ctypes.cast(x, ctypes.POINTER(ctypes.c_void_p))
                                                               for x in arrs)
    if fills is not None:
        cbm = h2g.witness_fill_multi(circ.num_advice, circ.n, fills)
        cbm.num_challenges = circ.num_challenges
        cfm = h2g.WITNESS_FILL_MULTI(cbm)
        keep += [cbm, cfm]
        spec.fill_multi = ctypes.cast(cfm, ctypes.c_void_p)
    if rng is not None:
        fb, fr = h2g.rng_callbacks(rng)
        keep += [fb, fr]
        spec.rng_fill_bytes = ctypes.cast(fb, ctypes.c_void_p)
        spec.rng_random_fr = ctypes.cast(fr, ctypes.c_void_p) if fr else None
    cap = 1 << 20
    buf = ctypes.create_string_buffer(cap)
    ln = np.zeros(1, dtype=np.uint64)
    if keygen is not None:
        rc = lib().or_prove(keygen.pk, ctypes.byref(spec), buf, cap, _p(ln), threads)
    else:
        rc = lib().or_create_proof(ctypes.byref(spec), buf, cap, _p(ln), threads)
    if rc != 0:
        raise ValueError(f"oracle create_proof failed: {rc}")
    if challenges_out is not None:
        import h2g_circuit as hc
        challenges_out[:] = hc.mont_to_ints(ch[: circ.num_challenges])
    return buf.raw[: int(ln[0])]


class OracleOps:
    """vectorised Montgomery arithmetic for witness generation (h2g_circuit.synthetic_c3)"""

    @staticmethod
    def mul(a, b):
        return binop("or_fr_mul", np.ascontiguousarray(a), np.ascontiguousarray(b))

    @staticmethod
    def prefix_product(a):
        return prefix_product(np.ascontiguousarray(a))


def commit_lagrange_at_s(values, s_int, degree, k, threads=8):
    """[f(s)]G for a Lagrange-form column f (ParamsKZG::commit_lagrange against an SRS whose
    secret s is known): the column's coefficients by the oracle's iNTT, Horner at s, one
    scalar multiplication -- independent of any SRS array.  -> (x, y) ints or None."""
    import h2g_circuit as hc
    from bn254_ref import G1_GEN, g1_mul

    coeff = lagrange_to_coeff(np.ascontiguousarray(values, dtype=np.uint64), degree, k, threads)
    e = eval_poly(coeff, np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64))
    return g1_mul(G1_GEN, hc.fr_from_limbs(e))


def vk_commitments(circ, wit, s_int, srs_g, srs_gl, threads=8):
    """The verifying key's (fixed, permutation) commitments computed on the CPU: sigma
    columns from the oracle keygen (C restatement of permutation/keygen.rs), fixed
    columns from the circuit, each committed as [f(s)]G."""
    kg = Keygen(circ, wit, srs_g, srs_gl, threads=threads)
    try:
        d, k = circ.degree(), circ.k
        fixed = [commit_lagrange_at_s(circ.fixed_values[i], s_int, d, k, threads) for i in range(circ.num_fixed)]
        sigma = [commit_lagrange_at_s(kg.sigma(i), s_int, d, k, threads) for i in range(len(circ.perm_columns))]
    finally:
        kg.close()
    return fixed, sigma
