"""The F29 lazy-reduction bounds (tools/f29_bounds.py) as a tested invariant.

The model reads every sub29<P, K, OFF> constant and is_zero29's early-out from the
kernel sources.  These tests fail when
  * the model rejects the constants the sources hold (a K too small for what it
    subtracts, a column sum at 2^64, a value above 2^261, an is_zero29 input that can
    exceed its early-out);
  * the sources drift from the snapshot the model was last reviewed against (any edit
    of a K, an OFF or the threshold, in f29.h, msm.hip, ntt.hip or prover_kernels.hip).
The arithmetic itself at the model's worst-case operands is tests/test_f29_host_cpu.py.
"""
import copy
import os
import re
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import f29_bounds as F  # noqa: E402


def _texts():
    out = {}
    for fn in F.SOURCES:
        with open(os.path.join(F.CSRC, fn)) as f:
            out[fn] = f.read()
    return out


def test_model_accepts_the_sources_constants():
    res = F.check()
    # the accumulation's coordinates stay below 2^259.5 (the bound f29.h's comment quotes)
    assert max(res["madd_fixpoint"]) < 2 ** 259.5
    assert res["madd_intermediate"] < 2 ** 260
    assert res["backend_out"] < 1.2 * F.M


def test_sources_match_the_reviewed_snapshot():
    got = F.source_constants()
    assert got == F.EXPECTED, {k: (got.get(k), F.EXPECTED.get(k)) for k in set(got) | set(F.EXPECTED)
                               if got.get(k) != F.EXPECTED.get(k)}


def test_every_sub29_site_is_parsed():
    """each sub29<...> instantiation in the sources lands in exactly one snapshot entry"""
    texts = _texts()
    n_src = sum(len(re.findall(r"\bsub29<", re.sub(r"//[^\n]*", "", t))) for t in texts.values())
    n_snap = sum(len(v) for k, v in F.EXPECTED.items() if k != "is_zero29")
    assert n_src == n_snap


def _sites():
    texts = _texts()
    out = []
    for fn, t in texts.items():
        code = re.sub(r"//[^\n]*", lambda m: " " * len(m.group(0)), t)
        for m in F._SUB.finditer(code):
            out.append((fn, m.start(1), m.end(1), m.group(1)))
    return texts, out


@pytest.mark.parametrize("how", ["half", "double"])
def test_editing_any_K_fails_a_check(how):
    """every K edited in place (halved or doubled) in its source file fails: the snapshot
    always, and the model too wherever the new K is unsafe"""
    texts, sites = _sites()
    assert len(sites) >= 20
    rejected_by_model = 0
    for fn, a, b, k in sites:
        if "S" in k:
            new = "(2u << S)" if how == "half" else "(8u << S)"
        else:
            new = str(int(k) // 2) if how == "half" else str(int(k) * 2)
        t = dict(texts)
        t[fn] = texts[fn][:a] + new + texts[fn][b:]
        c = F.source_constants(t)
        assert c != F.EXPECTED, (fn, a, k, new)
        try:
            F.check(c)
        except AssertionError:
            rejected_by_model += 1
    if how == "half":
        # the subtractions whose K is the smallest safe power of two (all but the back-end's
        # Q - X3 / S - X3 and the sparse pass, which keep a spare factor of 2)
        assert rejected_by_model >= len(sites) - 5, rejected_by_model


def test_halving_a_tight_K_is_rejected_by_the_model():
    """the model itself (not the snapshot) rejects K / 2 at the accumulation's subtractions,
    the NTT stages and evaluate_h"""
    c0 = F.source_constants()
    for key in ("f29.h:xyzz29_madd", "ntt.hip:nsub29", "prover_kernels.hip:eh_subn"):
        for i, (k, off) in enumerate(c0[key]):
            c = copy.deepcopy(c0)
            c[key][i] = ("(2u << S)" if "S" in k else str(int(k) // 2), off)
            if key == "prover_kernels.hip:eh_subn":
                c["prover_kernels.hip:eh_sub"] = c[key]
            with pytest.raises(AssertionError):
                F.check(c)


def test_is_zero29_threshold_is_asserted():
    c = copy.deepcopy(F.source_constants())
    F.check(c)
    c["is_zero29"] = 64  # the accumulation's P = U2 - X + 64 M reaches ~76 M
    with pytest.raises(AssertionError, match="early-out"):
        F.check(c)
    t = _texts()
    t["f29.h"] = t["f29.h"].replace("if (k > 1024) return false;", "if (k > 32) return false;")
    c2 = F.source_constants(t)
    assert c2["is_zero29"] == 32 and c2 != F.EXPECTED
    with pytest.raises(AssertionError):
        F.check(c2)


def test_script_runs_as_a_program(capsys):
    F.main()
    out = capsys.readouterr().out
    assert out.rstrip().endswith("ok") and "WARNING" not in out
