"""ctypes binding of libh2g.so (include/h2g.h) -- what a Python host (tests,
bench.py, smoke) uses to call the MI355X hot path through the C ABI.

No fallback: if the library or a GPU is missing, calls raise.  Arrays are numpy
uint64 in the halo2curves layout (Fr = 4 Montgomery limbs, G1Affine = 8 limbs);
device buffers are raw pointers (ints) from h2g_dev_alloc or torch tensors'
data_ptr().
"""
import ctypes
import sys
import os
import re

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
LIB_PATH = os.environ.get("H2G_LIB") or os.path.join(PKG, "lib", "libh2g.so")  # H2G_LIB: A/B builds
HEADER = os.path.join(REPO, "include", "h2g.h")

U64P = ctypes.POINTER(ctypes.c_uint64)
VP = ctypes.c_void_p
SZ = ctypes.c_size_t
I32 = ctypes.c_int
U32 = ctypes.c_uint32
U64 = ctypes.c_uint64

OP_ADD, OP_SUB, OP_MUL, OP_SCALE, OP_SUB_CONST, OP_ADD_CONST, OP_AXPY = range(7)

_SIGS = {
    "h2g_abi_version": ([], I32),
    "h2g_last_error": ([], ctypes.c_char_p),
    "h2g_init": ([ctypes.POINTER(I32), I32], I32),
    "h2g_shutdown": ([], I32),
    "h2g_device_count": ([ctypes.POINTER(I32)], I32),
    "h2g_device_mem_info": ([ctypes.POINTER(U64), ctypes.POINTER(U64)], I32),
    "h2g_set_device": ([I32], I32),
    "h2g_msm": ([U64P, U64P, SZ, U64P, ctypes.POINTER(I32)], I32),
    "h2g_msm_coeffs_descriptor": ([U64P, SZ, ctypes.POINTER(U64)], I32),
    "h2g_msm_base_descriptor": ([U64P, SZ, ctypes.POINTER(U64)], I32),
    "h2g_msm_descriptor_free": ([U64], I32),
    "h2g_msm_base_descriptor_dev": ([VP, SZ, I32, ctypes.POINTER(U64)], I32),
    "h2g_msm_with_cached_base_dev": ([VP, SZ, U64, SZ, U64P, ctypes.POINTER(I32), VP], I32),
    "h2g_msm_with_cached_scalars": ([U64, U64P, SZ, U64P, ctypes.POINTER(I32)], I32),
    "h2g_msm_with_cached_base": ([U64P, SZ, U64, SZ, U64P, ctypes.POINTER(I32)], I32),
    "h2g_msm_with_cached_inputs": ([U64, U64, SZ, U64P, ctypes.POINTER(I32)], I32),
    "h2g_msm_dev": ([VP, VP, SZ, VP, VP], I32),
    "h2g_msm_dev_cfg": ([VP, VP, SZ, I32, VP, VP], I32),
    "h2g_msm_dev_host": ([VP, VP, SZ, I32, U64P, ctypes.POINTER(I32), VP], I32),
    "h2g_descriptor_device_ptr": ([U64, ctypes.POINTER(VP), ctypes.POINTER(SZ)], I32),
    "h2g_srs_setup_dev": ([U64P, SZ, VP, VP], I32),
    "h2g_fft": ([U64P, U32, U64P], I32),
    "h2g_fft_dev": ([VP, U32, U64P, VP], I32),
    "h2g_domain_create": ([U32, U32, ctypes.POINTER(U64)], I32),
    "h2g_domain_free": ([U64], I32),
    "h2g_domain_info": ([U64, ctypes.POINTER(U32), ctypes.POINTER(U32), U64P], I32),
    "h2g_lagrange_to_coeff": ([U64, U64P], I32),
    "h2g_lagrange_to_coeff_dev": ([U64, VP, VP], I32),
    "h2g_coeff_to_extended": ([U64, U64P, U64P], I32),
    "h2g_coeff_to_extended_dev": ([U64, VP, VP, VP], I32),
    "h2g_extended_to_coeff": ([U64, U64P, U64P], I32),
    "h2g_extended_to_coeff_dev": ([U64, VP, VP, VP], I32),
    "h2g_divide_by_vanishing_poly": ([U64, U64P], I32),
    "h2g_divide_by_vanishing_poly_dev": ([U64, VP, VP], I32),
    "h2g_fr_op": ([I32, U64P, U64P, U64P, U64P, SZ], I32),
    "h2g_fr_op_dev": ([I32, VP, VP, U64P, VP, SZ, VP], I32),
    "h2g_fr_batch_invert": ([U64P, SZ], I32),
    "h2g_fr_batch_invert_dev": ([VP, SZ, VP], I32),
    "h2g_fr_prefix_product": ([U64P, U64P, SZ], I32),
    "h2g_fr_prefix_product_dev": ([VP, VP, SZ, VP], I32),
    "h2g_u32_exclusive_scan_dev": ([VP, VP, SZ, VP], I32),
    "h2g_dev_alloc": ([SZ, ctypes.POINTER(VP)], I32),
    "h2g_dev_free": ([VP], I32),
    "h2g_memcpy_htod": ([VP, VP, SZ], I32),
    "h2g_memcpy_dtoh": ([VP, VP, SZ], I32),
    "h2g_synchronize": ([], I32),
    "h2g_event_create": ([ctypes.POINTER(VP)], I32),
    "h2g_event_destroy": ([VP], I32),
    "h2g_event_record": ([VP, VP], I32),
    "h2g_event_elapsed_ms": ([VP, VP, ctypes.POINTER(ctypes.c_float)], I32),
    "h2g_g1_add_affine": ([U64P, U64P, U64P], I32),
    "h2g_profile_enable": ([I32], I32),
    "h2g_profile_msm_collect": ([ctypes.POINTER(ctypes.c_float), I32, ctypes.POINTER(I32), ctypes.POINTER(I32)], I32),
    "h2g_profile_msm_entries": ([ctypes.POINTER(U64), ctypes.POINTER(I32)], I32),
    "h2g_profile_box_calibrate": ([ctypes.POINTER(ctypes.c_double), I32], I32),
    "h2g_params_create": ([U32, U64P, U64P, ctypes.POINTER(U64)], I32),
    "h2g_params_setup": ([U32, U64P, ctypes.POINTER(U64)], I32),
    "h2g_params_export": ([U64, U64P, U64P], I32),
    "h2g_params_free": ([U64], I32),
    "h2g_params_g2": ([U64, U64P, U64P], I32),
    "h2g_params_set_g2": ([U64, U64P, U64P], I32),
    "h2g_params_write": ([U64, I32, VP, SZ, ctypes.POINTER(SZ)], I32),
    "h2g_params_read": ([ctypes.c_char_p, SZ, I32, ctypes.POINTER(U64)], I32),
    "h2g_pk_write": ([U64, I32, VP, SZ, ctypes.POINTER(SZ)], I32),
    "h2g_pk_read": ([U64, VP, ctypes.c_char_p, SZ, I32, ctypes.POINTER(U64)], I32),
    "h2g_keygen": ([U64, VP, ctypes.POINTER(U64)], I32),
    "h2g_pk_free": ([U64], I32),
    "h2g_pk_info": ([U64, ctypes.POINTER(ctypes.c_int32)], I32),
    "h2g_pk_vk_commitments": ([U64, U64P, U64P], I32),
    "h2g_pk_set_multiopen": ([U64, I32], I32),
    "h2g_pk_set_transcript": ([U64, I32], I32),
    "h2g_create_proof": ([U64, U64, VP, I32, U64P, ctypes.POINTER(U32), ctypes.c_char_p, U32, ctypes.c_char_p, SZ,
                          ctypes.POINTER(SZ)], I32),
    "h2g_create_proof_phased": ([U64, U64, VP, U64P, ctypes.POINTER(U32), ctypes.c_char_p, U32, ctypes.c_char_p,
                                 SZ, ctypes.POINTER(SZ)], I32),
    "h2g_create_proof_multi": ([U64, U64, VP, ctypes.c_char_p, SZ, ctypes.POINTER(SZ)], I32),
    "h2g_last_challenges": ([U64P, I32, ctypes.POINTER(I32)], I32),
    "h2g_prover_stages": ([ctypes.POINTER(ctypes.c_double), I32, ctypes.POINTER(I32)], I32),
    "h2g_prover_stage_name": ([I32], ctypes.c_char_p),
    "h2g_prover_stage_sync": ([I32], I32),
    "h2g_set_shard_transport": ([VP], I32),
    "h2g_params_set_slab": ([U64, U64, U64], I32),
    "h2g_params_msm_dev": ([U64, ctypes.c_int32, U64, U64, VP, U64P, ctypes.POINTER(ctypes.c_int32)], I32),
    "h2g_params_table_bytes": ([U64, U64P], I32),
    "h2g_memcpy_dtod": ([VP, VP, SZ], I32),
    "h2g_comm_unique_id": ([ctypes.c_char_p], I32),
    "h2g_comm_init": ([ctypes.c_char_p, I32, I32], I32),
    "h2g_comm_set_timeout": ([ctypes.c_double], I32),
    "h2g_comm_set_serve_timeout": ([ctypes.c_double], I32),
    "h2g_comm_keepalive": ([], I32),
    "h2g_comm_set_exchange_overlap": ([ctypes.c_int32], I32),
    "h2g_comm_install": ([U64], I32),
    "h2g_comm_serve": ([U64, ctypes.POINTER(U64)], I32),
    "h2g_comm_stop": ([], I32),
    "h2g_comm_destroy": ([], I32),
    "h2g_set_spmd_transport": ([VP], I32),
    "h2g_spmd_set_weights": ([VP, I32], I32),
    "h2g_comm_spmd_install": ([I32], I32),
    "h2g_comm_spmd_uninstall": ([], I32),
    "h2g_spmd_set_column_owners": ([I32], I32),
    "h2g_spmd_stats": ([ctypes.POINTER(ctypes.c_double), I32, I32], I32),
    "h2g_rng_chacha20": ([ctypes.POINTER(ctypes.c_uint8), VP, U64P], I32),
    "h2g_rng_free": ([U64], I32),
    "h2g_comm_info": ([ctypes.POINTER(I32), ctypes.POINTER(I32)], I32),
    "h2g_set_spmd_exchange_async": ([VP, VP], I32),
    "h2g_event_wait": ([VP], I32),
    "h2g_debug_link_delay": ([VP, VP, ctypes.c_double], I32),
}

TRANSCRIPTS = {"blake2b": 0, "keccak256": 1}  # Blake2bWrite / Keccak256Write (h2g_pk_set_transcript)
MSM_PHASES = ("partition_coarse", "partition_fine", "bucket_bounds", "accumulate", "bucket_fixup", "reduce")

_lib = None


class H2GError(RuntimeError):
    pass


def header_symbols():
    """Function names declared in include/h2g.h."""
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(?:int|const char\*)\s+(h2g_\w+)\s*\(", text)))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise H2GError(f"{LIB_PATH} not built: run __graft_entry__.build() "
                           "(yet-another-halo2-fork_amd/build_lib.py)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            if os.environ.get("H2G_LIB") and not hasattr(L, name):
                continue  # an older A/B build lacks newer entry points
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        raise H2GError(f"h2g error {rc}: {lib().h2g_last_error().decode()}")


def p64(a):
    if a is None:
        return None
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"], "need C-contiguous uint64"
    return a.ctypes.data_as(U64P)


_inited = False


def init(devices=None):
    """h2g_init.  libh2g runs on /opt/rocm's HIP runtime; a torch wheel carries its own
    copy, and in one process the copy initialised second must be torch's (torch started
    after libh2g finds no GPU: "No HIP GPUs are available").  So when the caller has
    imported torch, its CUDA state is initialised first."""
    global _inited
    tm = sys.modules.get("torch")
    if tm is not None and tm.cuda.device_count() > 0:
        tm.cuda.init()
    if devices:
        arr = (I32 * len(devices))(*devices)
        check(lib().h2g_init(arr, len(devices)))
    else:
        check(lib().h2g_init(None, 0))
    _inited = True


def shutdown():
    global _inited
    check(lib().h2g_shutdown())
    _inited = False


# ----------------------------------------------------------------- MSM (host API)
def msm(scalars, bases):
    sc = np.ascontiguousarray(scalars, dtype=np.uint64)
    bs = np.ascontiguousarray(bases, dtype=np.uint64)
    assert sc.shape[0] == bs.shape[0]
    out = np.zeros(8, dtype=np.uint64)
    ident = I32(0)
    check(lib().h2g_msm(p64(sc), p64(bs), sc.shape[0], p64(out), ctypes.byref(ident)))
    return out


def base_descriptor(bases):
    h = U64(0)
    bs = np.ascontiguousarray(bases, dtype=np.uint64)
    check(lib().h2g_msm_base_descriptor(p64(bs), bs.shape[0], ctypes.byref(h)))
    return h.value


def coeffs_descriptor(scalars):
    h = U64(0)
    sc = np.ascontiguousarray(scalars, dtype=np.uint64)
    check(lib().h2g_msm_coeffs_descriptor(p64(sc), sc.shape[0], ctypes.byref(h)))
    return h.value


def base_descriptor_dev(d_bases, n, window_bits=0):
    """fixed-base descriptor over device-resident bases (precomputed windows)"""
    h = U64()
    check(lib().h2g_msm_base_descriptor_dev(VP(d_bases), n, window_bits, ctypes.byref(h)))
    return h.value


def msm_with_cached_base_dev(d_scalars, n, base_handle, offset=0, stream=None):
    out = np.zeros(8, dtype=np.uint64)
    is_id = I32()
    check(lib().h2g_msm_with_cached_base_dev(VP(d_scalars), n, base_handle, offset, p64(out), ctypes.byref(is_id),
                                             VP(stream) if stream else None))
    return out


def descriptor_free(h):
    check(lib().h2g_msm_descriptor_free(h))


def msm_with_cached_base(scalars, base_handle, offset=0):
    sc = np.ascontiguousarray(scalars, dtype=np.uint64)
    out = np.zeros(8, dtype=np.uint64)
    ident = I32(0)
    check(lib().h2g_msm_with_cached_base(p64(sc), sc.shape[0], base_handle, offset, p64(out), ctypes.byref(ident)))
    return out


def msm_with_cached_scalars(coeff_handle, bases):
    bs = np.ascontiguousarray(bases, dtype=np.uint64)
    out = np.zeros(8, dtype=np.uint64)
    ident = I32(0)
    check(lib().h2g_msm_with_cached_scalars(coeff_handle, p64(bs), bs.shape[0], p64(out), ctypes.byref(ident)))
    return out


def msm_with_cached_inputs(coeff_handle, base_handle, offset=0):
    out = np.zeros(8, dtype=np.uint64)
    ident = I32(0)
    check(lib().h2g_msm_with_cached_inputs(coeff_handle, base_handle, offset, p64(out), ctypes.byref(ident)))
    return out


# ----------------------------------------------------------------- device buffers
class DevBuf:
    """Device allocation owned by Python (freed on close / GC)."""

    def __init__(self, nbytes):
        p = VP()
        check(lib().h2g_dev_alloc(nbytes, ctypes.byref(p)))
        self.ptr = p.value
        self.nbytes = nbytes

    @classmethod
    def from_array(cls, a):
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        b.upload(a)
        return b

    def upload(self, a):
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        check(lib().h2g_memcpy_htod(VP(self.ptr), a.ctypes.data_as(VP), a.nbytes))

    def download(self, shape, dtype=np.uint64):
        out = np.empty(shape, dtype=dtype)
        check(lib().h2g_memcpy_dtoh(out.ctypes.data_as(VP), VP(self.ptr), out.nbytes))
        return out

    def close(self):
        if self.ptr:
            try:
                lib().h2g_dev_free(VP(self.ptr))
            finally:
                self.ptr = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def msm_dev(d_scalars, d_bases, n, d_out, window_bits=0, stream=None):
    check(lib().h2g_msm_dev_cfg(VP(d_scalars), VP(d_bases), n, window_bits, VP(d_out), VP(stream) if stream else None))


def msm_dev_host(d_scalars, d_bases, n, window_bits=0, stream=None):
    out = np.zeros(8, dtype=np.uint64)
    ident = I32(0)
    check(lib().h2g_msm_dev_host(VP(d_scalars), VP(d_bases), n, window_bits, p64(out), ctypes.byref(ident),
                                 VP(stream) if stream else None))
    return out


def srs_setup_dev(s, n, d_out, stream=None):
    s = np.ascontiguousarray(s, dtype=np.uint64)
    check(lib().h2g_srs_setup_dev(p64(s), n, VP(d_out), VP(stream) if stream else None))


# ----------------------------------------------------------------- FFT / domain
def fft(a, omega):
    a = np.ascontiguousarray(a, dtype=np.uint64).copy()
    k = int(a.shape[0]).bit_length() - 1
    assert a.shape[0] == 1 << k
    check(lib().h2g_fft(p64(a), k, p64(np.ascontiguousarray(omega, dtype=np.uint64))))
    return a


def fft_dev(d_a, log_n, omega, stream=None):
    check(lib().h2g_fft_dev(VP(d_a), log_n, p64(np.ascontiguousarray(omega, dtype=np.uint64)),
                            VP(stream) if stream else None))


class Domain:
    """EvaluationDomain::new(j, k) mirror (halo2_backend/src/poly/domain.rs:38-144)."""

    def __init__(self, j, k):
        h = U64(0)
        check(lib().h2g_domain_create(j, k, ctypes.byref(h)))
        self.h = h.value
        self.j = j
        kk, ek = U32(0), U32(0)
        self.consts = np.zeros((9, 4), dtype=np.uint64)
        check(lib().h2g_domain_info(self.h, ctypes.byref(kk), ctypes.byref(ek), p64(self.consts)))
        self.k, self.extended_k = kk.value, ek.value
        self.n = 1 << self.k
        self.extended_len = 1 << self.extended_k

    def lagrange_to_coeff(self, a):
        a = np.ascontiguousarray(a, dtype=np.uint64).copy()
        assert a.shape[0] == self.n
        check(lib().h2g_lagrange_to_coeff(self.h, p64(a)))
        return a

    def coeff_to_extended(self, a):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        assert a.shape[0] == self.n
        out = np.zeros((self.extended_len, 4), dtype=np.uint64)
        check(lib().h2g_coeff_to_extended(self.h, p64(a), p64(out)))
        return out

    def extended_to_coeff(self, a):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        assert a.shape[0] == self.extended_len
        out = np.zeros((self.n * (self.j - 1), 4), dtype=np.uint64)
        check(lib().h2g_extended_to_coeff(self.h, p64(a), p64(out)))
        return out

    def divide_by_vanishing_poly(self, a):
        a = np.ascontiguousarray(a, dtype=np.uint64).copy()
        assert a.shape[0] == self.extended_len
        check(lib().h2g_divide_by_vanishing_poly(self.h, p64(a)))
        return a

    def close(self):
        if self.h:
            lib().h2g_domain_free(self.h)
            self.h = 0


# ----------------------------------------------------------------- poly ops
def fr_op(op, a, b=None, c=None):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    out = np.zeros_like(a)
    bb = np.ascontiguousarray(b, dtype=np.uint64) if b is not None else None
    cc = np.ascontiguousarray(c, dtype=np.uint64) if c is not None else None
    check(lib().h2g_fr_op(op, p64(a), p64(bb), p64(cc), p64(out), a.shape[0]))
    return out


def batch_invert(a):
    a = np.ascontiguousarray(a, dtype=np.uint64).copy()
    check(lib().h2g_fr_batch_invert(p64(a), a.shape[0]))
    return a


def u32_exclusive_scan_dev(d_in, d_out, n, stream=None):
    """exclusive prefix sum of n u32 on the device (in place when d_in == d_out)"""
    check(lib().h2g_u32_exclusive_scan_dev(VP(d_in), VP(d_out), n, VP(stream) if stream else None))


def prefix_product(a):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    out = np.zeros_like(a)
    check(lib().h2g_fr_prefix_product(p64(a), p64(out), a.shape[0]))
    return out


def g1_add_affine(a, b):
    out = np.zeros(8, dtype=np.uint64)
    check(lib().h2g_g1_add_affine(p64(np.ascontiguousarray(a, dtype=np.uint64)),
                                  p64(np.ascontiguousarray(b, dtype=np.uint64)), p64(out)))
    return out


def profile_enable(on=True):
    check(lib().h2g_profile_enable(1 if on else 0))


def profile_msm_collect(with_union=False):
    """-> (calls, {phase: total_ms}) for MSMs run since profiling was enabled; with_union:
    (calls, phases, {"accumulate": ms, "msm": ms}) adding the busy time (union of the
    intervals) of the overlapping MSMs' accumulate phases and of the whole MSMs."""
    ms = (ctypes.c_float * 8)()
    npz, calls = I32(0), I32(0)
    ent, unc = U64(0), I32(0)
    check(lib().h2g_profile_msm_entries(ctypes.byref(ent), ctypes.byref(unc)))
    check(lib().h2g_profile_msm_collect(ms, 8, ctypes.byref(npz), ctypes.byref(calls)))
    phases = {MSM_PHASES[i]: ms[i] for i in range(npz.value)}
    if not with_union:
        return calls.value, phases
    return calls.value, phases, {"accumulate": ms[npz.value], "msm": ms[npz.value + 1],
                                 "entries": ent.value if unc.value == 0 else None}


def box_calibrate():
    """this GPU's Montgomery product throughput now (G/s): the round-4 reference kernel
    (tools/microbench/modmul_bench.hip's FIPS product, one chain per thread), the F29
    product and the FIPS product (two chains per thread each); the shader clock during the
    F29 run (GHz) and the ms spent (h2g_profile_box_calibrate)"""
    out = (ctypes.c_double * 5)()
    check(lib().h2g_profile_box_calibrate(out, 5))
    return {"modmul_ref_gps": round(out[0], 2), "modmul_f29_gps": round(out[1], 2),
            "modmul_fips2_gps": round(out[4], 2), "sclk_ghz_in_kernel": round(out[2], 3),
            "calibration_ms": round(out[3], 1)}


class Timer:
    """HIP-event timing on the library stream (or a given stream)."""

    def __init__(self, stream=None):
        self.stream = VP(stream) if stream else None
        a, b = VP(), VP()
        check(lib().h2g_event_create(ctypes.byref(a)))
        check(lib().h2g_event_create(ctypes.byref(b)))
        self.a, self.b = a, b

    def start(self):
        check(lib().h2g_event_record(self.a, self.stream))

    def stop_ms(self):
        check(lib().h2g_event_record(self.b, self.stream))
        ms = ctypes.c_float(0)
        check(lib().h2g_event_elapsed_ms(self.a, self.b, ctypes.byref(ms)))
        return ms.value


# ----------------------------------------------------------------------------- prover
I32P_ = ctypes.POINTER(ctypes.c_int32)


class H2gCircuit(ctypes.Structure):
    """struct h2g_circuit (include/h2g.h)"""
    _fields_ = [
        ("k", U32), ("num_advice", U32), ("num_fixed", U32), ("num_instance", U32),
        ("num_gates", U32), ("gate_roots", I32P_),
        ("num_nodes", U32), ("nodes", I32P_),
        ("num_constants", U32), ("constants", U64P),
        ("num_perm_columns", U32), ("perm_columns", I32P_),
        ("num_copies", U32), ("copies", I32P_),
        ("fixed_values", U64P), ("unblinded", ctypes.POINTER(ctypes.c_uint8)),
        ("transcript_repr", U64P),
        ("num_lookups", U32), ("lookup_sizes", ctypes.POINTER(U32)), ("lookup_roots", I32P_),
        ("num_shuffles", U32), ("shuffle_sizes", ctypes.POINTER(U32)), ("shuffle_roots", I32P_),
        ("advice_phase", ctypes.POINTER(ctypes.c_uint8)), ("num_challenges", U32),
        ("challenge_phase", ctypes.POINTER(ctypes.c_uint8)),
    ]


# h2g_witness_source.fill(ctx, phase, challenges, advice)
WITNESS_FILL = ctypes.CFUNCTYPE(ctypes.c_int, VP, U32, U64P, U64P)


class WitnessSource(ctypes.Structure):
    """struct h2g_witness_source (include/h2g.h)"""
    _fields_ = [("ctx", VP), ("fill", WITNESS_FILL)]


def witness_fill(num_advice, n, fn):
    """Wraps fn(phase, challenges: list[int] (canonical, 0 for later phases)) -> {column:
    m x 4 Montgomery array, m <= n (rows [0, m) are written: at least the usable rows)} as a
    WITNESS_FILL callback (Prover::commit_phase's witness)."""
    import h2g_circuit as hc

    def cb(_ctx, phase, ch_p, adv_p):
        try:
            nch = cb.num_challenges
            ch = np.ctypeslib.as_array(ch_p, shape=(max(nch, 1), 4))[:nch] if nch else np.zeros((0, 4), np.uint64)
            adv = np.ctypeslib.as_array(adv_p, shape=(num_advice, n, 4))
            for col, vals in fn(int(phase), hc.mont_to_ints(ch)).items():
                adv[col, : len(vals)] = vals  # a prefix of rows: the usable ones at least
            return 0
        except Exception:  # noqa: BLE001 -- reported to the prover as a failed witness
            import traceback
            traceback.print_exc()
            return 1

    cb.num_challenges = 0
    return cb


# h2g_witness_source_multi.fill(ctx, circuit, phase, challenges, advice)
WITNESS_FILL_MULTI = ctypes.CFUNCTYPE(ctypes.c_int, VP, U32, U32, U64P, U64P)


class WitnessSourceMulti(ctypes.Structure):
    """struct h2g_witness_source_multi (include/h2g.h)"""
    _fields_ = [("ctx", VP), ("fill", WITNESS_FILL_MULTI)]


def witness_fill_multi(num_advice, n, fns):
    """fns[c](phase, challenges) -> {column: values} per circuit c (see witness_fill) as a
    WITNESS_FILL_MULTI callback"""
    single = [witness_fill(num_advice, n, f) for f in fns]

    def cb(ctx, circuit, phase, ch_p, adv_p):
        if circuit >= len(single):
            return 1
        single[circuit].num_challenges = cb.num_challenges
        return single[circuit](ctx, phase, ch_p, adv_p)

    cb.num_challenges = 0
    return cb


# h2g_rng: RngCore::fill_bytes and F::random of the caller's RNG
RNG_FILL = ctypes.CFUNCTYPE(ctypes.c_int, VP, ctypes.POINTER(ctypes.c_uint8), SZ)
RNG_FR = ctypes.CFUNCTYPE(ctypes.c_int, VP, U64P)


class Rng(ctypes.Structure):
    """struct h2g_rng (include/h2g.h)"""
    _fields_ = [("ctx", VP), ("fill_bytes", RNG_FILL), ("random_fr", RNG_FR)]


def rng_callbacks(rng):
    """(RNG_FILL, RNG_FR or None) of a Python RNG object: rng.fill_bytes(n) -> bytes, and
    optionally rng.random_fr() -> 4 Montgomery limbs (F::random)"""
    def fill(_ctx, out, n):
        try:
            b = bytes(rng.fill_bytes(int(n)))
            if len(b) != n:
                return 1
            ctypes.memmove(out, b, n)
            return 0
        except Exception:  # noqa: BLE001 -- reported to the prover as a failed draw
            return 1

    def fr(_ctx, out):
        try:
            v = np.ascontiguousarray(rng.random_fr(), dtype=np.uint64)
            ctypes.memmove(out, v.ctypes.data, 32)
            return 0
        except Exception:  # noqa: BLE001
            return 1

    return RNG_FILL(fill), (RNG_FR(fr) if hasattr(rng, "random_fr") else RNG_FR())


class ProveInputs(ctypes.Structure):
    """struct h2g_prove_inputs (include/h2g.h)"""
    _fields_ = [("num_circuits", U32), ("advice", ctypes.POINTER(VP)), ("advice_on_device", I32),
                ("witness", ctypes.POINTER(WitnessSourceMulti)), ("instance", ctypes.POINTER(VP)),
                ("instance_lens", ctypes.POINTER(VP)), ("rng", ctypes.POINTER(Rng)),
                ("rng_seed", ctypes.POINTER(ctypes.c_uint8)), ("vanishing_threads", U32)]


def _ptr(a, t):
    return a.ctypes.data_as(t) if a is not None and a.size else None


# SerdeFormat (halo2_backend/src/helpers.rs:8-21)
PROCESSED, RAW_BYTES, RAW_BYTES_UNCHECKED = 0, 1, 2


def _write_bytes(fn, handle, fmt):
    ln = SZ()
    check(fn(handle, fmt, None, 0, ctypes.byref(ln)))
    buf = ctypes.create_string_buffer(max(ln.value, 1))
    check(fn(handle, fmt, ctypes.cast(buf, VP), ln.value, ctypes.byref(ln)))
    return buf.raw[: ln.value]


class Params:
    """ParamsKZG resident on the device (g, g_lagrange; g2, s_g2 on the host)."""

    def __init__(self, k, g=None, g_lagrange=None, s=None, _handle=None):
        self.k = k
        h = U64()
        if _handle is not None:
            h.value = _handle
        elif s is not None:
            s = np.ascontiguousarray(s, dtype=np.uint64)
            check(lib().h2g_params_setup(k, p64(s), ctypes.byref(h)))
        else:
            g = np.ascontiguousarray(g, dtype=np.uint64)
            gl = np.ascontiguousarray(g_lagrange, dtype=np.uint64)
            check(lib().h2g_params_create(k, p64(g), p64(gl), ctypes.byref(h)))
        self.handle = h.value

    @classmethod
    def read(cls, data, fmt=RAW_BYTES):
        """ParamsKZG::read_custom (kzg/commitment.rs:183-267)"""
        h = U64()
        check(lib().h2g_params_read(bytes(data), len(data), fmt, ctypes.byref(h)))
        k = int.from_bytes(bytes(data[:4]), "little")
        return cls(k, _handle=h.value)

    def write(self, fmt=RAW_BYTES):
        """ParamsKZG::write_custom (kzg/commitment.rs:166-181) -> bytes"""
        return _write_bytes(lib().h2g_params_write, self.handle, fmt)

    def g2(self):
        """(g2, s_g2) as 16 u64 each (x.c0, x.c1, y.c0, y.c1 Montgomery)"""
        a = np.zeros(16, dtype=np.uint64)
        b = np.zeros(16, dtype=np.uint64)
        check(lib().h2g_params_g2(self.handle, p64(a), p64(b)))
        return a, b

    def set_g2(self, g2, s_g2):
        a = np.ascontiguousarray(g2, dtype=np.uint64)
        b = np.ascontiguousarray(s_g2, dtype=np.uint64)
        check(lib().h2g_params_set_g2(self.handle, p64(a), p64(b)))

    def set_slab(self, lo, hi):
        """fixed-base windows for this rank's point slab [lo, hi) (one proof over several GPUs)"""
        check(lib().h2g_params_set_slab(self.handle, lo, hi))

    def export(self):
        n = 1 << self.k
        g = np.zeros((n, 8), dtype=np.uint64)
        gl = np.zeros((n, 8), dtype=np.uint64)
        check(lib().h2g_params_export(self.handle, p64(g), p64(gl)))
        return g, gl

    def close(self):
        if self.handle:
            lib().h2g_params_free(self.handle)
            self.handle = 0


class ProvingKey:
    """keygen_vk + keygen_pk on the device for an h2g_circuit.Circuit."""

    def __init__(self, params, circ, data=None, fmt=RAW_BYTES):
        """keygen, or -- with `data` -- ProvingKey::read of serialised bytes (plonk.rs:334-359)"""
        self.params = params
        self.circ = circ
        keep = [np.ascontiguousarray(x) for x in (circ.gate_roots, circ.nodes, circ.constants, circ.perm_array,
                                                  circ.copies, circ.fixed_values, circ.unblinded,
                                                  circ.transcript_repr(), circ.lookup_sizes, circ.lookup_roots,
                                                  circ.shuffle_sizes, circ.shuffle_roots, circ.advice_phase,
                                                  circ.challenge_phase)]
        roots, nodes, consts, perm, copies, fixed, unb, tr, lks, lkr, shs, shr, aph, chph = keep
        c = H2gCircuit(circ.k, circ.num_advice, circ.num_fixed, circ.num_instance,
                       len(roots), _ptr(roots, I32P_), len(nodes), _ptr(nodes, I32P_),
                       circ.num_constants, _ptr(consts, U64P), len(perm), _ptr(perm, I32P_),
                       len(copies), _ptr(copies, I32P_), _ptr(fixed, U64P),
                       _ptr(unb, ctypes.POINTER(ctypes.c_uint8)), _ptr(tr, U64P),
                       len(circ.lookups), _ptr(lks, ctypes.POINTER(U32)), _ptr(lkr, I32P_),
                       len(circ.shuffles), _ptr(shs, ctypes.POINTER(U32)), _ptr(shr, I32P_),
                       _ptr(aph, ctypes.POINTER(ctypes.c_uint8)), circ.num_challenges,
                       _ptr(chph, ctypes.POINTER(ctypes.c_uint8)))
        h = U64()
        if data is None:
            check(lib().h2g_keygen(params.handle, ctypes.byref(c), ctypes.byref(h)))
        else:
            check(lib().h2g_pk_read(params.handle, ctypes.byref(c), bytes(data), len(data), fmt, ctypes.byref(h)))
        self.handle = h.value
        info = (ctypes.c_int32 * 8)()
        check(lib().h2g_pk_info(self.handle, info))
        (self.degree, self.bf, self.extended_k, self.nsets, self.n_adv_q, self.n_fix_q, self.n_ins_q,
         self.n_slots) = list(info)

    def vk_commitments(self):
        """(fixed commitments, permutation commitments): uint64 arrays (F, 8), (P, 8) affine
        Montgomery (VerifyingKey::fixed_commitments, the permutation VerifyingKey)"""
        f = np.zeros((max(self.circ.num_fixed, 1), 8), dtype=np.uint64)
        p = np.zeros((max(len(self.circ.perm_columns), 1), 8), dtype=np.uint64)
        check(lib().h2g_pk_vk_commitments(self.handle, p64(f), p64(p)))
        return f[: self.circ.num_fixed], p[: len(self.circ.perm_columns)]

    def write(self, fmt=RAW_BYTES):
        """ProvingKey::write (plonk.rs:311-321) -> bytes"""
        return _write_bytes(lib().h2g_pk_write, self.handle, fmt)

    def create_proof(self, wit=None, seed=bytes([7] * 32), vanishing_threads=8, advice_dev_ptr=None,
                     multiopen="shplonk", transcript="blake2b"):
        """-> proof bytes.  advice_dev_ptr: device pointer to num_advice x n Fr (resident inputs).
        multiopen: "shplonk" (ProverSHPLONK) or "gwc" (ProverGWC)."""
        if multiopen != "shplonk" or hasattr(lib(), "h2g_pk_set_multiopen"):
            check(lib().h2g_pk_set_multiopen(self.handle, {"shplonk": 0, "gwc": 1}[multiopen]))
        check(lib().h2g_pk_set_transcript(self.handle, TRANSCRIPTS[transcript]))
        circ = self.circ
        n = 1 << circ.k
        if advice_dev_ptr is not None:
            adv_p, on_dev = VP(advice_dev_ptr), 1
            adv = None
        else:
            adv = np.ascontiguousarray(wit.advice, dtype=np.uint64)
            adv_p, on_dev = VP(adv.ctypes.data) if adv.size else None, 0
        ins = np.ascontiguousarray(wit.instance, dtype=np.uint64) if circ.num_instance else np.zeros(4, np.uint64)
        lens = np.ascontiguousarray(wit.instance_lens if circ.num_instance else np.zeros(1), dtype=np.uint32)
        cap = 32 * (64 + 8 * (circ.num_advice + circ.num_fixed + 4 * len(circ.perm_columns)) + 64 * 64
                    + 16 * (len(circ.lookups) + len(circ.shuffles)))
        buf = ctypes.create_string_buffer(cap)
        ln = SZ()
        check(lib().h2g_create_proof(self.params.handle, self.handle, adv_p, on_dev, p64(ins),
                                     lens.ctypes.data_as(ctypes.POINTER(U32)), bytes(seed), vanishing_threads,
                                     buf, cap, ctypes.byref(ln)))
        del adv
        return buf.raw[: ln.value]

    def create_proof_phased(self, fill, wit, seed=bytes([7] * 32), vanishing_threads=8, multiopen="shplonk",
                            transcript="blake2b"):
        """Prover::commit_phase per phase with the witness from fill(phase, challenges) ->
        {column: values} (see witness_fill); wit supplies the instance columns.
        -> (proof bytes, challenges as ints)"""
        check(lib().h2g_pk_set_multiopen(self.handle, {"shplonk": 0, "gwc": 1}[multiopen]))
        check(lib().h2g_pk_set_transcript(self.handle, TRANSCRIPTS[transcript]))
        circ = self.circ
        ins = np.ascontiguousarray(wit.instance, dtype=np.uint64) if circ.num_instance else np.zeros(4, np.uint64)
        lens = np.ascontiguousarray(wit.instance_lens if circ.num_instance else np.zeros(1), dtype=np.uint32)
        cb = witness_fill(circ.num_advice, circ.n, fill)
        cb.num_challenges = circ.num_challenges
        cfn = WITNESS_FILL(cb)
        src = WitnessSource(None, cfn)
        cap = 32 * (64 + 8 * (circ.num_advice + circ.num_fixed + 4 * len(circ.perm_columns)) + 64 * 64
                    + 16 * (len(circ.lookups) + len(circ.shuffles)))
        buf = ctypes.create_string_buffer(cap)
        ln = SZ()
        check(lib().h2g_create_proof_phased(self.params.handle, self.handle, ctypes.byref(src), p64(ins),
                                            lens.ctypes.data_as(ctypes.POINTER(U32)), bytes(seed),
                                            vanishing_threads, buf, cap, ctypes.byref(ln)))
        ch = np.zeros((max(circ.num_challenges, 1), 4), dtype=np.uint64)
        cnt = ctypes.c_int()
        check(lib().h2g_last_challenges(p64(ch), circ.num_challenges, ctypes.byref(cnt)))
        import h2g_circuit as hc
        return buf.raw[: ln.value], hc.mont_to_ints(ch[: cnt.value])

    def create_proof_multi(self, wits, seed=bytes([7] * 32), rng=None, fills=None, vanishing_threads=8,
                           multiopen="shplonk", advice_dev_ptrs=None, transcript="blake2b"):
        """create_proof(params, pk, circuits, instances, rng, transcript) over several circuits
        (halo2_proofs/src/plonk/prover.rs:19-36) -> proof bytes.  wits: one witness per circuit
        (advice, or -- with fills -- only the instance columns); rng: None = ChaCha20Rng::from_seed(
        seed), "native" = the same generator behind the h2g_rng callbacks (h2g_rng_chacha20: the
        caller-RNG path), else an object with fill_bytes(n) (and optionally random_fr()); fills: per-circuit
        fill(phase, challenges) -> {column: values} witness sources."""
        check(lib().h2g_pk_set_multiopen(self.handle, {"shplonk": 0, "gwc": 1}[multiopen]))
        check(lib().h2g_pk_set_transcript(self.handle, TRANSCRIPTS[transcript]))
        circ = self.circ
        nc = len(wits)
        keep = []
        adv_arr = (VP * nc)()
        ins_arr = (VP * nc)()
        lens_arr = (VP * nc)()
        for c, wit in enumerate(wits):
            if advice_dev_ptrs is not None:
                adv_arr[c] = advice_dev_ptrs[c]
            elif fills is None:
                a = np.ascontiguousarray(wit.advice, dtype=np.uint64)
                keep.append(a)
                adv_arr[c] = a.ctypes.data if a.size else None
            ins = np.ascontiguousarray(wit.instance, dtype=np.uint64) if circ.num_instance else np.zeros(4, np.uint64)
            lens = np.ascontiguousarray(wit.instance_lens if circ.num_instance else np.zeros(1), dtype=np.uint32)
            keep += [ins, lens]
            ins_arr[c] = ins.ctypes.data
            lens_arr[c] = lens.ctypes.data
        inp = ProveInputs()
        inp.num_circuits = nc
        inp.advice = ctypes.cast(adv_arr, ctypes.POINTER(VP))
        inp.advice_on_device = 1 if advice_dev_ptrs is not None else 0
        inp.instance = ctypes.cast(ins_arr, ctypes.POINTER(VP))
        inp.instance_lens = ctypes.cast(lens_arr, ctypes.POINTER(VP))
        inp.vanishing_threads = vanishing_threads
        if fills is not None:
            cb = witness_fill_multi(circ.num_advice, circ.n, fills)
            cb.num_challenges = circ.num_challenges
            cfn = WITNESS_FILL_MULTI(cb)
            src = WitnessSourceMulti(None, cfn)
            keep += [cb, cfn, src]
            inp.witness = ctypes.pointer(src)
        native_rng = None
        if isinstance(rng, str) and rng == "native":  # the library's ChaCha20Rng behind the callbacks
            r = Rng()
            native_rng = U64()
            sd0 = (ctypes.c_uint8 * 32)(*bytes(seed))
            check(lib().h2g_rng_chacha20(sd0, ctypes.byref(r), ctypes.byref(native_rng)))
            keep += [r, sd0]
            inp.rng = ctypes.pointer(r)
        elif rng is not None:
            fb, fr = rng_callbacks(rng)
            r = Rng(None, fb, fr)
            keep += [fb, fr, r]
            inp.rng = ctypes.pointer(r)
        sd = (ctypes.c_uint8 * 32)(*bytes(seed))
        keep.append(sd)
        inp.rng_seed = ctypes.cast(sd, ctypes.POINTER(ctypes.c_uint8))
        cap = nc * 32 * (64 + 8 * (circ.num_advice + 4 * len(circ.perm_columns)) + 64 * 64
                         + 16 * (len(circ.lookups) + len(circ.shuffles))) + 32 * 8 * circ.num_fixed
        buf = ctypes.create_string_buffer(cap)
        ln = SZ()
        try:
            check(lib().h2g_create_proof_multi(self.params.handle, self.handle, ctypes.byref(inp), buf, cap,
                                               ctypes.byref(ln)))
        finally:
            if native_rng is not None:
                lib().h2g_rng_free(native_rng.value)
        del keep
        return buf.raw[: ln.value]

    def close(self):
        if self.handle:
            lib().h2g_pk_free(self.handle)
            self.handle = 0


# ----------------------------------------------------------- multi-GPU MSM slabs
SHARD_LAUNCH = ctypes.CFUNCTYPE(ctypes.c_int, VP, U64, ctypes.c_int32, U64, VP)
SHARD_COLLECT = ctypes.CFUNCTYPE(ctypes.c_int, VP, U64, U64P, ctypes.POINTER(ctypes.c_int32))


class ShardTransport(ctypes.Structure):
    """struct h2g_shard_transport (include/h2g.h)"""
    _fields_ = [("ctx", VP), ("world", ctypes.c_int32), ("launch", SHARD_LAUNCH), ("collect", SHARD_COLLECT)]


_transport_keep = None


def set_shard_transport(world, launch=None, collect=None):
    """Install the MSM slab transport of create_proof: launch(seq, base_set, n, d_scalars)
    and collect(seq) -> [(affine uint64[8], is_identity)] * (world - 1).  world <= 1
    removes it.  Exceptions inside the callbacks fail the proof (nonzero status)."""
    global _transport_keep
    if world <= 1:
        check(lib().h2g_set_shard_transport(None))
        _transport_keep = None
        return

    def _launch(ctx, seq, base_set, n, d_scalars):
        try:
            launch(int(seq), int(base_set), int(n), int(d_scalars or 0))
            return 0
        except Exception as e:  # noqa: BLE001 -- reported through the C status
            _transport_keep[-1].append(e)
            return 1

    def _collect(ctx, seq, partials, ids):
        try:
            parts = collect(int(seq))
            assert len(parts) == world - 1
            for i, (pt, is_id) in enumerate(parts):
                pt = np.ascontiguousarray(pt, dtype=np.uint64).reshape(8)
                for j in range(8):
                    partials[8 * i + j] = int(pt[j])
                ids[i] = 1 if is_id else 0
            return 0
        except Exception as e:  # noqa: BLE001
            _transport_keep[-1].append(e)
            return 1

    cl, cc = SHARD_LAUNCH(_launch), SHARD_COLLECT(_collect)
    t = ShardTransport(None, world, cl, cc)
    _transport_keep = (t, cl, cc, [])
    check(lib().h2g_set_shard_transport(ctypes.byref(t)))


def transport_errors():
    """exceptions raised inside the installed transport's callbacks (cleared)"""
    if _transport_keep is None:
        return []
    errs = list(_transport_keep[-1])
    _transport_keep[-1].clear()
    return errs


SPMD_WORDS = 13  # H2G_SPMD_WORDS (include/h2g.h)
_spmd_world = 1
SPMD_ALLGATHER = ctypes.CFUNCTYPE(ctypes.c_int, VP, U64, U64P, U64P)
SPMD_BCAST = ctypes.CFUNCTYPE(ctypes.c_int, VP, VP, SZ, ctypes.c_int)
SPMD_ALLGATHER_HOST = ctypes.CFUNCTYPE(ctypes.c_int, VP, VP, SZ, VP)
SPMD_EXCHANGE = ctypes.CFUNCTYPE(ctypes.c_int, VP, VP, ctypes.POINTER(SZ), VP, ctypes.POINTER(SZ))


class SpmdTransport(ctypes.Structure):
    """struct h2g_spmd_transport (include/h2g.h)"""
    _fields_ = [("ctx", VP), ("world", ctypes.c_int32), ("rank", ctypes.c_int32), ("allgather", SPMD_ALLGATHER),
                ("bcast", SPMD_BCAST), ("allgather_host", SPMD_ALLGATHER_HOST), ("exchange", SPMD_EXCHANGE)]


def set_spmd_transport(world, rank=0, allgather=None, bcast=None, allgather_host=None, exchange=None):
    """SPMD sharding: every rank runs the same create_proof and computes its point slab of
    each commitment MSM; allgather(seq, mine: uint64[SPMD_WORDS]) -> uint64[world, SPMD_WORDS]
    (rank order) collects the partials (8 affine limbs, identity flag, 4 words of the
    rank's transcript / RNG digest, which the library compares across ranks).  bcast(d_ptr, nbytes, root) (optional) divides the extended
    domain's sub-cosets over the ranks and broadcasts each one's h evaluations (device
    memory, in place).  allgather_host(data: bytes) -> world byte strings in rank order
    (optional) runs the evaluations and the SHPLONK multi-open on coefficient slabs.
    exchange(d_send, send_bytes, d_recv, recv_bytes) (optional, with both): all-to-all of
    device memory with per-peer byte lists -- h(X) then travels as coefficient slabs.
    world <= 1 removes it.  Exceptions fail the proof."""
    global _transport_keep, _spmd_world, _xasync_keep
    _xasync_keep = None  # the library removes the overlapped exchange with the transport
    if world <= 1:
        check(lib().h2g_set_spmd_transport(None))
        _transport_keep = None
        return
    _spmd_world = world

    def _ag(ctx, seq, mine, out):
        try:
            got = np.ascontiguousarray(allgather(int(seq), np.ctypeslib.as_array(mine, shape=(SPMD_WORDS,)).copy()),
                                       dtype=np.uint64).reshape(world * SPMD_WORDS)
            ctypes.memmove(out, got.ctypes.data, world * SPMD_WORDS * 8)
            return 0
        except Exception as e:  # noqa: BLE001 -- reported through the C status
            _transport_keep[-1].append(e)
            return 1

    def _bc(ctx, d_ptr, nbytes, root):
        try:
            bcast(int(d_ptr or 0), int(nbytes), int(root))
            return 0
        except Exception as e:  # noqa: BLE001
            _transport_keep[-1].append(e)
            return 1

    def _agh(ctx, d_in, nbytes, d_out):
        try:
            parts = allgather_host(ctypes.string_at(d_in, nbytes))
            if len(parts) != world or any(len(p) != nbytes for p in parts):
                raise ValueError("allgather_host: world x bytes expected")
            ctypes.memmove(d_out, b"".join(bytes(p) for p in parts), world * nbytes)
            return 0
        except Exception as e:  # noqa: BLE001
            _transport_keep[-1].append(e)
            return 1

    def _ex(ctx, d_send, sbytes, d_recv, rbytes):
        try:
            exchange(int(d_send or 0), [int(sbytes[i]) for i in range(world)], int(d_recv or 0),
                     [int(rbytes[i]) for i in range(world)])
            return 0
        except Exception as e:  # noqa: BLE001
            _transport_keep[-1].append(e)
            return 1

    cb = SPMD_ALLGATHER(_ag)
    cbb = SPMD_BCAST(_bc) if bcast is not None else ctypes.cast(None, SPMD_BCAST)
    cbh = SPMD_ALLGATHER_HOST(_agh) if allgather_host is not None else ctypes.cast(None, SPMD_ALLGATHER_HOST)
    cbx = SPMD_EXCHANGE(_ex) if exchange is not None else ctypes.cast(None, SPMD_EXCHANGE)
    t = SpmdTransport(None, world, rank, cb, cbb, cbh, cbx)
    _transport_keep = (t, cb, cbb, cbh, cbx, [])
    check(lib().h2g_set_spmd_transport(ctypes.byref(t)))


SPMD_XPOST = ctypes.CFUNCTYPE(ctypes.c_int, VP, VP, ctypes.POINTER(SZ), VP, ctypes.POINTER(SZ), VP, VP)
SPMD_XWAIT = ctypes.CFUNCTYPE(ctypes.c_int, VP, VP)
_xasync_keep = None


def set_spmd_exchange_async(post=None, wait=None):
    """the column-ownership exchanges overlapped with the later stages
    (h2g_set_spmd_exchange_async; after set_spmd_transport with an exchange, which removes
    it again): post(d_send, send_bytes, d_recv, recv_bytes, stream, done) queues the
    all-to-all behind the work on `stream` so far and has `done` recorded (event_record /
    debug_link_delay) once the bytes are in place; wait(done) returns when it has been.
    post=None: exchanges complete on return.  Exceptions fail the proof."""
    global _xasync_keep
    if post is None:
        check(lib().h2g_set_spmd_exchange_async(None, None))
        _xasync_keep = None
        return
    errs = _transport_keep[-1] if _transport_keep is not None else []

    def _post(ctx, d_send, sbytes, d_recv, rbytes, stream, done):
        try:
            w = _spmd_world
            post(int(d_send or 0), [int(sbytes[i]) for i in range(w)], int(d_recv or 0),
                 [int(rbytes[i]) for i in range(w)], int(stream or 0), int(done or 0))
            return 0
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            return 1

    def _wait(ctx, done):
        try:
            if wait is not None:
                wait(int(done or 0))
            return 0
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            return 1

    # no wait callable: NULL, so the library itself waits on `done` (hipEventSynchronize in
    # xp_flush) instead of a callback that returns before the transfer has landed
    cp = SPMD_XPOST(_post)
    cw = SPMD_XWAIT(_wait) if wait is not None else None
    check(lib().h2g_set_spmd_exchange_async(ctypes.cast(cp, VP), ctypes.cast(cw, VP) if cw is not None else None))
    _xasync_keep = (cp, cw)


def event_record(done, stream):
    check(lib().h2g_event_record(VP(done), VP(stream)))


def event_wait(done):
    check(lib().h2g_event_wait(VP(done)))


def debug_link_delay(stream, done, us):
    """`done` recorded `us` microseconds of device time after the work on `stream` (a
    modelled transfer for the one-GPU SPMD emulation)"""
    check(lib().h2g_debug_link_delay(VP(stream), VP(done), float(us)))


SPMD_COLLECTIVES = ("msm_allgather", "host_allgather", "exchange", "bcast")


def spmd_stats(reset=True):
    """time / calls / bytes inside the SPMD transport per collective kind (h2g_spmd_stats)"""
    out = (ctypes.c_double * 12)()
    check(lib().h2g_spmd_stats(out, 12, 1 if reset else 0))
    return {k: {"ms": out[3 * i], "calls": int(out[3 * i + 1]), "bytes": int(out[3 * i + 2])}
            for i, k in enumerate(SPMD_COLLECTIVES)}


def comm_info():
    """(ncclCommCount, ncclCommUserRank) of the library's communicator, (0, -1) without one"""
    c, r = I32(), I32()
    check(lib().h2g_comm_info(ctypes.byref(c), ctypes.byref(r)))
    return c.value, r.value


def spmd_set_column_owners(on):
    """SPMD column ownership of wide stages (h2g_spmd_set_column_owners; on by default)"""
    check(lib().h2g_spmd_set_column_owners(1 if on else 0))


def spmd_set_weights(weights):
    """SPMD slab weights (h2g_spmd_set_weights): rank r's slab is [P S_r / S, P S_{r+1} / S);
    None restores the uniform partition.  Every rank passes the same list, and sets its
    params slab to h2g_dist.slab(P, world, rank, weights=...)."""
    if not weights:
        check(lib().h2g_spmd_set_weights(None, 0))
        return
    w = np.ascontiguousarray(weights, dtype=np.uint32)
    check(lib().h2g_spmd_set_weights(VP(w.ctypes.data), len(w)))


# ------------------------------------------------- native RCCL transport (csrc/comm.cpp)
def comm_unique_id():
    buf = ctypes.create_string_buffer(256)
    check(lib().h2g_comm_unique_id(buf))
    return buf.raw


def comm_init(uid, world, rank):
    check(lib().h2g_comm_init(bytes(uid), world, rank))


def comm_set_timeout(seconds):
    """deadline of every wait on the library's RCCL communicators (h2g_comm_set_timeout)"""
    check(lib().h2g_comm_set_timeout(float(seconds)))


def comm_set_serve_timeout(seconds):
    """a serving peer's idle deadline for rank 0's next request (h2g_comm_set_serve_timeout)"""
    check(lib().h2g_comm_set_serve_timeout(float(seconds)))


def comm_keepalive():
    """rank 0: renew the serving peers' idle deadline (h2g_comm_keepalive)"""
    check(lib().h2g_comm_keepalive())


def comm_set_exchange_overlap(on):
    """SPMD over the library's communicators: overlapped column exchanges (opt-in)"""
    check(lib().h2g_comm_set_exchange_overlap(1 if on else 0))


def comm_install(params):
    check(lib().h2g_comm_install(params.handle))


def comm_serve(params):
    served = U64()
    check(lib().h2g_comm_serve(params.handle, ctypes.byref(served)))
    return served.value


def comm_stop():
    check(lib().h2g_comm_stop())


def comm_destroy():
    check(lib().h2g_comm_destroy())


def comm_spmd_install(subcosets=True):
    """SPMD sharding over the library's communicator (RCCL all-gather of the partials;
    subcosets: the extended domain's sub-cosets divided over the ranks, h broadcast)"""
    check(lib().h2g_comm_spmd_install(1 if subcosets else 0))


def comm_spmd_uninstall():
    check(lib().h2g_comm_spmd_uninstall())


def device_mem_info():
    """(free, total) bytes of the current device (hipMemGetInfo after a synchronize)"""
    f, t = U64(), U64()
    check(lib().h2g_device_mem_info(ctypes.byref(f), ctypes.byref(t)))
    return f.value, t.value


def params_table_bytes(params):
    """(full g/g_lagrange, their slab, full prefix basis, slab prefix basis) window bytes"""
    out = np.zeros(4, dtype=np.uint64)
    check(lib().h2g_params_table_bytes(params.handle, p64(out)))
    return tuple(int(v) for v in out)


def params_msm_dev(params, base_set, offset, n, d_scalars):
    """peer side of the slab transport: MSM of n device scalars against params'
    base set (0 = g, 1 = g_lagrange) at [offset, offset + n) -> (affine, is_identity)"""
    out = np.zeros(8, dtype=np.uint64)
    is_id = ctypes.c_int32()
    check(lib().h2g_params_msm_dev(params.handle, base_set, offset, n, VP(d_scalars) if n else None, p64(out),
                                   ctypes.byref(is_id)))
    return out, bool(is_id.value)


def memcpy_dtod(d_dst, d_src, nbytes):
    check(lib().h2g_memcpy_dtod(VP(d_dst), VP(d_src), nbytes))


def memcpy_dtoh(h_dst, d_src, nbytes):
    check(lib().h2g_memcpy_dtoh(VP(h_dst), VP(d_src), nbytes))


def memcpy_htod(d_dst, h_src, nbytes):
    check(lib().h2g_memcpy_htod(VP(d_dst), VP(h_src), nbytes))


def prover_stage_sync(on=True):
    """stage boundaries synchronise the prover stream (GPU completion times; diagnostics)"""
    check(lib().h2g_prover_stage_sync(1 if on else 0))


def prover_stages():
    ms = (ctypes.c_double * 64)()
    cnt = I32()
    check(lib().h2g_prover_stages(ms, 64, ctypes.byref(cnt)))
    return [(lib().h2g_prover_stage_name(i).decode(), ms[i]) for i in range(min(cnt.value, 64))]


class DeviceOps:
    """vectorised Montgomery arithmetic on the device (witness generation for
    h2g_circuit.synthetic_c3 at bench sizes)"""

    @staticmethod
    def mul(a, b):
        return fr_op(OP_MUL, a, b)

    @staticmethod
    def prefix_product(a):
        return prefix_product(a)
