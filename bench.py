#!/usr/bin/env python3
"""Benchmark of the MI355X prover hot path (BASELINE.json metric:
"create_proof wall-seconds at k=22 (BN254/KZG); MSM Mscalar-mul/s at 2^24").

--workload keccak: the same over the keccak256-style circuit of BASELINE configs[4]
(32 advice columns, 16 three-column lookups, degree 5) at k = 18.

Default workload (--workload prove): one step = one full create_proof
(KZG + SHPLONK + Blake2b) of the C3 synthetic circuit at k=22 (BASELINE configs[2]/[3]:
3 advice a,b,c + 1 fixed f, gate f*(a*b - c), a,b,c in the permutation, copies
c_i -> a_{i+1}) through the C ABI (h2g_create_proof), witness resident in HBM when the
timed region starts.  value = wall-seconds per proof (lower is better).  The proof
bytes of this exact pipeline are tested identical to the CPU restatement prover
(tests/test_gpu_prover.py).
N > 1 (torchrun, one process per GPU), --mode spmd (default): ONE proof at a time over
all ranks -- every rank runs the same prover (same key, witness and seed) and computes
point slab `rank` of each commitment MSM; the 64-B partials are all-gathered (libh2g's
RCCL communicator, --transport native, or torch.distributed) so every rank writes the
same proof; value = max-over-ranks wall time / steps, "scaling": "strong".  --mode shard:
rank 0 proves and sends each MSM's scalar slabs to the peers.  --mode
replicas: every rank proves its own instance; value = max-over-ranks time / (steps * N).

--workload msm: one step = one MSM of 2^24 resident (scalar, SRS point) pairs
(h2g_msm_dev_host); N > 1 shards point slabs and all_gathers the 64-B partials (RCCL).

`python bench.py --gpus N` without WORLD_SIZE starts torchrun with N ranks as a child
process (before any GPU call) and exits with its status.

Also in the JSON line (prove workload, outside the timed region):
  roofline     : dominant kernel = msm_acc_kernel (bucket accumulation), average
                 launch time from HIP events on the library stream over the timed
                 region; algorithmic bytes = 96 B/point x points per launch; PMC
                 traffic from rocprofv3 --pmc child passes (MI355X guide recipe);
                 bound "valu" with the modmul rate against the measured and modelled peaks
  verified     : the timed proof accepted by the checker's verifier (oracle/py/verifier.py)
  msm_2p24     : the metric's MSM half, 2^24 resident points, Mscalar-mul/s
  cpu_baseline : the CPU restatement (oracle/, halo2 algorithms, all cores) proving the
                 same circuit, witness and SRS at the same k, measured directly
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "yet-another-halo2-fork_amd"))

HBM_PEAK_GBS = 8000.0
MSM_BYTES_PER_POINT = 96  # 32 B scalar + 64 B affine base
MADD_MODMUL = 10          # XYZZ mixed add: 8M + 2S
PROVE_K = 22
KECCAK_K = 18  # BASELINE configs[4]: keccak256-style circuit (many columns, lookups) at k = 18
METRIC = "create_proof wall-seconds at k=22 (BN254/KZG); MSM Mscalar-mul/s at 2^24"


def random_scalars(rng, n):
    """Uniform values < 2^253 < r: valid Montgomery-form Fr elements."""
    c = rng.integers(0, 2**63, size=(n, 4), dtype=np.int64).astype(np.uint64)
    c[:, 0] = c[:, 0] * np.uint64(2) + (rng.integers(0, 2, size=n, dtype=np.int64).astype(np.uint64))
    c[:, 3] &= np.uint64((1 << 61) - 1)
    return c


def fixed_c(n):
    # mirror of msm_choose_c_fixed (msm.hip): one shared bucket set
    best, bc = 1e300, 2
    for c in range(2, 23):
        cost = ((255 + c - 1) // c) * n + 3.0 * (1 << (c - 1))
        if cost < best * 0.98:
            best, bc = cost, c
    return bc


def h2g_choose_c(n):
    # mirror of msm_choose_c (msm.hip) for reporting
    best, bc = 1e300, 2
    for c in range(2, 23):
        W = (255 + c - 1) // c
        cost = W * (n + 2.8 * (1 << (c - 1)))
        if cost < best:
            best, bc = cost, c
    return bc


# ----------------------------------------------------------------------------- CPU baselines
def _oracle():
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle as O
    return O


def cpu_info():
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model, os.cpu_count() or 1


def cpu_threads():
    """host threads the CPU baseline may use: this process's CPU affinity, capped by the
    OMP_NUM_THREADS the pool sets (the box's share of its cores) -> (threads, how)"""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < aff:
        return int(omp), f"OMP_NUM_THREADS={omp} (sched_getaffinity: {aff} CPUs)"
    return aff, f"sched_getaffinity: {aff} CPUs"


T_START = time.perf_counter()


def progress(msg):
    """a progress line on stderr (the JSON line alone goes to stdout): long legs -- the CPU
    baselines run for minutes -- must not look like a hang to a watchdog"""
    print(f"[bench {time.perf_counter() - T_START:7.1f} s] {msg}", file=sys.stderr, flush=True)


def box_smi():
    """clocks, power and power cap of the GPUs as rocm-smi reports them (best effort)"""
    import subprocess
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--showmaxpower", "--showperflevel", "--json"],
                           capture_output=True, text=True, timeout=30)
        d = json.loads(r.stdout[r.stdout.index("{"):])
    except Exception as e:  # the line stands without it
        return {"error": f"{type(e).__name__}"}
    out = {}
    for card, v in d.items():
        if not card.startswith("card"):
            continue
        keep = {}
        for k, val in v.items():
            kl = k.lower()
            if any(t in kl for t in ("sclk", "mclk", "fclk", "power", "perf")):
                keep[k] = val
        out[card] = keep
    return out


def box_block(h2g):
    """box calibration, measured before the timed region: this GPU's
    Montgomery product rate now (tools/microbench kernels, csrc/calib.hip), its shader
    clock under that load, and rocm-smi's clocks / power / power cap"""
    b = h2g.box_calibrate()
    b["reference_gps"] = MODMUL_REF_GPS
    b["reference_f29_gps"] = MODMUL_F29_REF_GPS
    b["smi"] = box_smi()
    return b


def cpu_baseline_prove(circ, wit, g, gl, k, reps=1):
    """The oracle's create_proof (C restatement of halo2's prover: best_multiexp /
    best_fft / parallelize, OpenMP over `threads` cores) of the SAME circuit, witness and
    SRS as the timed GPU proofs, measured directly at the bench's k (keygen excluded,
    untimed); median of `reps` runs.  Both modes of SURVEY 8d at several k, median of 3:
    tools/cpu_baseline.py (profiles/r02/cpu_baseline.json)."""
    O = _oracle()
    model, ncpu = cpu_info()
    threads, how = cpu_threads()
    kg = O.Keygen(circ, wit, g, gl, threads=threads)
    times = []
    for i in range(reps):
        progress(f"cpu baseline, all-cores mode, k={k}, run {i + 1} of {reps}")
        t0 = time.perf_counter()
        O.create_proof(circ, wit, g, gl, threads=threads, keygen=kg)
        times.append(time.perf_counter() - t0)
    kg.close()
    med = sorted(times)[len(times) // 2]
    return {"value": round(med, 3), "unit": "s", "cores": threads, "kind": "port",
            "sample": f"oracle create_proof (C restatement of halo2_backend's prover, all-cores mode: MSM/FFT and "
                      f"parallelize on {threads} OpenMP threads) of the bench's own C3 circuit, witness and SRS at "
                      f"k={k}, measured directly (no scaling), median of {reps} run(s), keygen excluded",
            "runs_s": [round(t, 3) for t in times],
            "host": {"cpu_model": model, "nproc": ncpu, "threads_used": threads, "threads_from": how}}


def cpu_baseline_faithful(h2g, k=20, reps=1):
    """SURVEY 8d's faithful mode beside the all-cores one: the oracle's
    create_proof with MSM and FFT single-threaded (halo2curves built without its `multicore`
    feature, as the reference's Cargo.toml selects -- SURVEY finding 3) and the
    parallelize-style loops on the box's threads, C3 at k (20: about 80 s), SRS from the
    device params, keygen excluded"""
    import h2g_circuit as hc
    O = _oracle()
    threads, how = cpu_threads()
    circ, wit = hc.synthetic_c3(k, h2g.DeviceOps, seed=3)
    params = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(0x1234567 + k), dtype=np.uint64))
    g, gl = params.export()
    params.close()
    kg = O.Keygen(circ, wit, g, gl, threads=threads)
    times = []
    O.lib().or_set_kernel_threads(1)
    try:
        for _ in range(reps):
            progress(f"cpu baseline, faithful mode, k={k}")
            t0 = time.perf_counter()
            O.create_proof(circ, wit, g, gl, threads=threads, keygen=kg)
            times.append(time.perf_counter() - t0)
    finally:
        O.lib().or_set_kernel_threads(0)
        kg.close()
    med = sorted(times)[len(times) // 2]
    return {"value": round(med, 3), "unit": "s", "k": k, "msm_fft_threads": 1, "parallelize_threads": threads,
            "kind": "port", "runs_s": [round(t, 3) for t in times], "threads_from": how,
            "sample": f"oracle create_proof of the C3 circuit at k={k}, faithful mode (SURVEY 8d (i)): best_multiexp "
                      f"and best_fft on 1 thread, parallelize on {threads}; median of {reps} run(s), keygen excluded"}


def cpu_baseline_msm(log_n=20, reps=2):
    """Oracle best_multiexp (halo2curves algorithm) on one 2^log_n MSM."""
    O = _oracle()
    threads, _ = cpu_threads()
    rng = np.random.default_rng(5)
    n = 1 << log_n
    s = O.random_fr(rng, 1)[0]
    small = O.srs_powers(s, 1 << 10)
    bases = np.ascontiguousarray(np.tile(small, (n >> 10, 1)))
    sc = O.random_fr(rng, n)
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        O.msm_best(sc, bases, threads)
        best = min(best, time.perf_counter() - t0)
    return {"value": round(n / best / 1e6, 4), "unit": "Mscalar-mul/s", "cores": threads, "kind": "port",
            "sample": f"one 2^{log_n}-point MSM, oracle best_multiexp (Booth-window Pippenger), "
                      f"{threads} threads, best of {reps}"}


# ----------------------------------------------------------------------------- PMC traffic
def pmc_traffic(args):
    """HBM traffic of the dominant kernel from PMC counters, per the MI355X guide:
    one rocprofv3 --pmc pass per counter (FETCH_SIZE and WRITE_SIZE cannot share a
    pass), values in KiB, FETCH_SIZE doubled (gfx950 reports half of a 16-B/lane
    read stream).  Child processes run BEFORE this process touches the GPU."""
    import csv
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    vals = {}
    env = dict(os.environ, TMPDIR="/tmp")
    # one pass per TCC counter (FETCH_SIZE and WRITE_SIZE cannot share one), then one pass
    # of 5 SQ counters (8 SQ slots): where the accumulation's wave cycles go
    sq_ctrs = ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU")
    for ctrs in (("FETCH_SIZE",), ("WRITE_SIZE",), sq_ctrs):
        d = tempfile.mkdtemp(prefix=f"h2g_pmc_{ctrs[0]}_", dir="/tmp")
        cmd = [prof, "--pmc", *ctrs, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--workload", args.workload,
               "--log-n", str(args.log_n), "--k", str(args.k)]
        try:
            subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           timeout=300, check=True)
            rows = []
            for root, _, files in os.walk(d):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        rows += [r for r in csv.DictReader(open(os.path.join(root, f)))
                                 if "msm_acc_kernel" in r["Kernel_Name"] and r["Counter_Name"] in ctrs]
            for ctr in ctrs:
                cr = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == ctr]
                if not cr:
                    raise RuntimeError(f"no {ctr} rows for msm_acc_kernel")
                vals[ctr] = sum(cr) / len(cr)
        except Exception as e:  # profiling is best-effort; the timed result stands alone
            if ctrs == sq_ctrs:  # the traffic passes stand without the SQ one
                vals["sq_error"] = f"SQ pass failed: {type(e).__name__}"
                continue
            return None, f"{ctrs[0]} pass failed: {type(e).__name__}"
        finally:
            shutil.rmtree(d, ignore_errors=True)
    sq = None
    if "SQ_WAVE_CYCLES" in vals and vals["SQ_WAVE_CYCLES"] > 0:
        wc = vals["SQ_WAVE_CYCLES"]
        sq = {"issue_stall_frac": round(vals["SQ_WAIT_INST_ANY"] / wc, 3),
              "waitcnt_frac": round(vals["SQ_WAIT_ANY"] / wc, 3),
              "active_frac": round(vals["SQ_ACTIVE_INST_ANY"] / wc, 3),
              "valu_insts_per_launch": round(vals["SQ_INSTS_VALU"]),
              "counters_per_launch": {c: round(vals[c]) for c in sq_ctrs},
              "note": "SQ_WAIT_INST_ANY: a wave had an instruction ready but the VALU was taken (issue-bound); "
                      "SQ_WAIT_ANY: parked on s_waitcnt (memory); SQ_ACTIVE_INST_ANY: issuing. The three add up "
                      "to SQ_WAVE_CYCLES (MI355X guide, PMC slots)"}
    elif "sq_error" in vals:
        sq = {"error": vals["sq_error"]}
    # the raw counters (bytes); roofline_from_phases applies the calibration per access kind
    return {"fetch": vals["FETCH_SIZE"] * 1024.0, "write": vals["WRITE_SIZE"] * 1024.0, "sq": sq}, (
        f"rocprofv3 --pmc, mean per launch of msm_acc_kernel: FETCH_SIZE {vals['FETCH_SIZE']:.0f} KiB, WRITE_SIZE "
        f"{vals['WRITE_SIZE']:.0f} KiB.  Calibration (tools/microbench/pmc_calib.hip, profiles/r03/pmc_calibration.json): "
        "FETCH_SIZE counts one 64-B unit per read request -- 1.01 of random 64-B point gathers, 0.50 of a coalesced "
        "8-B / 16-B per lane stream -- so `traffic` counts the gathers x1 and the sorted-value stream x2 "
        "(FETCH + 0.5 x the stream's bytes) + WRITE; `traffic_upper` prices every request as a 128-B line (2 FETCH + WRITE)")


def pmc_child(args):
    """Minimal profiled workload (no torch): one proof, or SRS + 2 MSMs."""
    import h2g

    h2g.init([0])
    if args.workload in ("prove", "keccak"):
        import h2g_circuit as hc
        circ, wit = (hc.keccak_style(args.k, words=16) if args.workload == "keccak"
                     else hc.synthetic_c3(args.k, h2g.DeviceOps))
        params = h2g.Params(args.k, s=np.asarray(hc.fr_to_limbs(0x1234567), dtype=np.uint64))
        pk = h2g.ProvingKey(params, circ)
        pk.create_proof(wit)
        pk.close()
        params.close()
    else:
        n = 1 << args.log_n
        rng = np.random.default_rng(1000)
        bases = h2g.DevBuf(n * 64)
        h2g.srs_setup_dev(random_scalars(rng, 1)[0], n, bases.ptr)
        sc = h2g.DevBuf.from_array(random_scalars(rng, n))
        base = h2g.base_descriptor_dev(bases.ptr, n, 0)
        for _ in range(2):
            h2g.msm_with_cached_base_dev(sc.ptr, n, base, 0)
        h2g.descriptor_free(base)
    h2g.shutdown()


# ----------------------------------------------------------------------------- roofline
# tools/microbench/modmul_bench.hip's FIPS product rate on the round-4 boxes:
# value_normalised_fips = value x (this box's rate of that same kernel / this)
MODMUL_REF_GPS = 125.0
# the F29 product rate (h2g_profile_box_calibrate, 9 x 29-bit limbs: the arithmetic the hot
# kernels run since round 5) of a reference MI355X box: value_normalised = value x (this
# box's F29 rate / this), the proof time scaled to a box of that rate.  Boxes of this pool
# measure 161.9-169.1 G/s at 2.30-2.35 GHz shader clock; 165.0 is the stated reference.
MODMUL_F29_REF_GPS = 165.0


def roofline_from_phases(calls, phases, points_per_launch, traffic, traffic_note, window_bits=0, union=None,
                         peak_gps=None):
    acc_ms = phases.get("accumulate", 0.0) / max(calls, 1)
    achieved = (points_per_launch * MSM_BYTES_PER_POINT) / (acc_ms * 1e-3) / 1e9 if acc_ms > 0 else None
    c = window_bits or fixed_c(points_per_launch)
    W = (255 + c - 1) // c
    # mixed additions per MSM: the device's count of sorted entries (nonzero signed digits)
    # when recorded -- W x n overstates it for scalars with zero digits (small witness
    # values, e.g. the keccak-style circuit's nibbles)
    entries = (union or {}).get("entries")
    madds = entries / max(calls, 1) if entries else points_per_launch * W
    madd_source = "counted (sorted entries)" if entries else f"{W} windows x n"
    modmul_rate = (madds * MADD_MODMUL) / (acc_ms * 1e-3) if acc_ms > 0 else None
    out = {
        "bound": "valu",
        "kernel": "msm_acc_kernel (Pippenger bucket accumulation)",
        "achieved": round(achieved, 2) if achieved else None,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
        "traffic": None,
        "traffic_note": traffic_note,
        "kernel_ms": round(acc_ms, 4),
        "launches": calls,
        "bytes_per_launch": points_per_launch * MSM_BYTES_PER_POINT,
        "note": "VALU-bound 256-bit modular arithmetic (no MFMA applies): achieved/peak/frac are the HBM view the "
                "contract asks for (algorithmic 96 B/point), low by construction; `valu` is the bound that applies",
        "valu_modmul_per_s": round(modmul_rate, 1) if modmul_rate else None,
        "valu": {"achieved": round(modmul_rate / 1e9, 2) if modmul_rate else None, "unit": "G modmul/s",
                 "per_point": f"{W} windows x 1 XYZZ mixed add (8M + 2S = {MADD_MODMUL} modmul)",
                 "madds_per_launch": round(madds), "madds": madd_source},
        "window_bits": c,
    }
    if peak_gps and modmul_rate:  # this box's product rate, measured before the timed region
        out["valu"].update({"peak": round(peak_gps, 2), "frac": round(modmul_rate / (peak_gps * 1e9), 4),
                            "peak_note": "this GPU's F29 Montgomery products/s (h2g_profile_box_calibrate: "
                                         "9 x 29-bit limbs, the arithmetic the accumulation runs), measured "
                                         "before the timed region; the madd's 10 products counted as full "
                                         "products (its two squarings and one merged reduction are cheaper)"})
    if traffic and traffic.get("sq"):  # where the accumulation's wave cycles go (PMC SQ pass)
        out["valu"]["pmc"] = traffic["sq"]
    if traffic:  # PMC bytes per launch, calibrated per access kind (pmc_traffic)
        stream = madds * 4.0  # the u32 bucket-ordered values, read once
        cal = traffic["fetch"] + 0.5 * stream + traffic["write"]
        gathered = madds * 64.0  # one 64-B table point per mixed addition
        out.update({"traffic": round(cal), "traffic_upper": round(2 * traffic["fetch"] + traffic["write"]),
                    "traffic_vs_algorithmic": round(cal / (points_per_launch * MSM_BYTES_PER_POINT), 2),
                    "traffic_vs_gathered_table_bytes": round(cal / gathered, 3),
                    "gathered_table_bytes": round(gathered)})
    if union and union.get("accumulate", 0) > 0:
        # MSMs on the two MSM streams overlap each other, so a launch's duration counts the
        # chip's time twice while they do: the chip-level rate is the work over the busy time
        agg = calls * madds * MADD_MODMUL / (union["accumulate"] * 1e-3)
        out["valu"].update({"aggregate": round(agg / 1e9, 2),
                            "aggregate_note": "all launches' modmuls / union of their accumulate intervals"})
        out["valu_modmul_per_s_aggregate"] = round(agg, 1)
    return out


# ----------------------------------------------------------------------------- collectives
# a gloo group beside the RCCL default group (N > 1): the bench's own small agreements
# (timing max, transport fallback, proof digests) do not depend on the transport under test
CTRL = None


def ctrl_all_reduce(value, dist, op):
    import torch
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=op, group=CTRL)
    return float(t.item())


def max_over_ranks(elapsed, dist, world, device):
    """the job's time is the slowest rank's (contract: max over ranks)"""
    if world == 1:
        return elapsed
    return ctrl_all_reduce(elapsed, dist, dist.ReduceOp.MAX)


# set when the SPMD proof had to fall back to the gloo transport: RCCL is then not trusted
# for the MSM partials either
RCCL_SUSPECT = False


def gather_partials(part, dist, world, device):
    """all_gather of the per-rank MSM partial sums (64-B affine points; RCCL has no
    EC-add reduction) -> list of numpy uint64[8]"""
    import torch
    group = None
    if dist.get_backend() == "gloo" or RCCL_SUSPECT:
        device, group = "cpu", CTRL
    t = torch.from_numpy(np.ascontiguousarray(part, dtype=np.uint64).view(np.int64)).to(device)
    gathered = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(gathered, t, group=group)
    return [g.cpu().numpy().view(np.uint64) for g in gathered]


def combine_partials(parts, add):
    """sum of the gathered partials with a host EC add (h2g_g1_add_affine)"""
    total = np.zeros(8, dtype=np.uint64)
    for p in parts:
        total = add(total, p)
    return total


# ----------------------------------------------------------------------------- workloads
def run_prove(args, h2g, torch, dist, world, rank, dev, traffic, traffic_note):
    global RCCL_SUSPECT
    import h2g_circuit as hc
    import h2g_dist

    k = args.k
    n = 1 << k
    shard = world > 1 and args.mode == "shard"  # rank 0 proves, peers serve slabs
    spmd = world > 1 and args.mode == "spmd"    # every rank proves its slab of each MSM
    one_proof = shard or spmd
    worker = shard and rank != 0
    seed_off = 0 if one_proof else rank  # ranks of one proof hold the same SRS and witness
    spmd_weights = {"w": None}
    s_int = 0x1234567 + seed_off
    params = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(s_int), dtype=np.uint64))
    if shard:  # fixed-base windows sized for this rank's point slab (spmd: after keygen, weighted)
        params.set_slab(*h2g_dist.slab(n, world, rank))
    native = one_proof and args.transport == "native"
    transport_note = None
    if one_proof:  # every wait on the library's RCCL communicators has a deadline (fail soft)
        h2g.comm_set_timeout(args.comm_timeout)
        h2g.comm_set_serve_timeout(args.comm_timeout)  # shard peers: rank 0's next request
    if native and shard:  # the library's own RCCL communicators (csrc/comm.cpp); the id travels over torch
        import torch as _t
        tdev = dev if dist.get_backend() == "nccl" else "cpu"
        uid = _t.zeros(256, dtype=_t.uint8, device=tdev)
        if rank == 0:
            uid.copy_(_t.frombuffer(bytearray(h2g.comm_unique_id()), dtype=_t.uint8))
        dist.broadcast(uid, 0)
        ok = 1
        try:
            h2g.comm_init(bytes(uid.cpu().numpy().tobytes()), world, rank)
        except h2g.H2GError as e:  # every rank learns of any failure and falls back together
            ok, transport_note = 0, f"native communicator failed ({e}); torch.distributed transport used"
        flag = _t.tensor([ok], dtype=_t.int64, device=tdev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if not int(flag.item()):
            if ok:
                h2g.comm_destroy()
            native = False
            transport_note = transport_note or "a peer's native communicator failed; torch.distributed transport used"
    if worker:
        slabs = None if native else h2g_dist.SlabWorker(dist, params=params)
    else:
        if args.workload == "keccak":
            circ, wit = hc.keccak_style(k, words=16, seed=5 + seed_off)
        else:
            circ, wit = hc.synthetic_c3(k, h2g.DeviceOps, seed=3 + seed_off)
        pk = h2g.ProvingKey(params, circ)
        if spmd:  # lighter slabs for the ranks that own extended-domain sub-cosets
            weights = h2g_dist.owner_weights(world, pk.extended_k, k,
                                             None if args.spmd_owner_weight < 0 else args.spmd_owner_weight) \
                if args.spmd_owner_weight != 0 else None
            h2g.spmd_set_weights(weights)
            params.set_slab(*h2g_dist.slab(n, world, rank, weights=weights))
            spmd_weights["w"] = weights
        adv = torch.from_numpy(np.ascontiguousarray(wit.advice).view(np.int64)).to(dev)  # resident witness
        client = h2g_dist.SlabClient(dist, points=n) if shard and not native else None
        gather = None
    torch.cuda.synchronize()
    proofs = []

    def step():
        proofs.append(pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr()))

    # SPMD transport, first that proves on every rank: the library's RCCL communicators
    # with the column exchanges overlapped on the second one ("native"), the same with
    # blocking exchanges ("native-sync"), torch.distributed over RCCL ("torch"),
    # torch.distributed over the gloo group with host-staged exchanges ("host" -- the form
    # the one-GPU tests exercise).  A transport "proves" when its first proof equals, on
    # every rank, the single-GPU proof the rank made before (same key, witness and seed):
    # a hang ends at the communicator deadline, a wrong exchange at the comparison.
    spmd_kind = {"kind": None}

    native_setup_failed = {"v": False}

    def spmd_open(kind):
        nonlocal gather
        if kind.startswith("native"):
            h2g.comm_set_exchange_overlap(kind == "native")
            try:
                spmd_native_init()
            except Exception:
                native_setup_failed["v"] = True  # the blocking form would fail the same way
                raise
            h2g.comm_spmd_install(not args.no_subcosets)
        else:
            gather = h2g_dist.SpmdGather(dist, group=CTRL if kind == "host" else None,
                                         subcosets=not args.no_subcosets)
            gather.install()

    def spmd_close(kind):
        if kind.startswith("native"):
            h2g.comm_spmd_uninstall()
        else:
            gather.uninstall()

    def spmd_native_init():
        import torch as _t
        uid = _t.zeros(256, dtype=_t.uint8)
        if rank == 0:
            uid.copy_(_t.frombuffer(bytearray(h2g.comm_unique_id()), dtype=_t.uint8))
        dist.broadcast(uid, 0, group=CTRL)
        h2g.comm_init(bytes(uid.numpy().tobytes()), world, rank)

    if spmd:
        # ranks sharing a GPU (a gloo rehearsal on a smaller box): RCCL refuses them (a
        # communicator per GPU), so the native kinds are not tried there
        shared_gpus = torch.cuda.device_count() < world
        kinds = [kd for kd in args.spmd_transports.split(",")
                 if (not kd.startswith("native") or args.transport == "native" or
                     (args.dist_backend == "gloo" and not shared_gpus))
                 and (kd != "native" or not args.sync_exchange)
                 and (kd != "torch" or dist.get_backend() == "nccl")]
        notes = []
        progress("spmd: this rank's single-GPU reference proof")
        ref = pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())  # this rank alone
        for kind in kinds:
            if kind == "native-sync" and int(ctrl_all_reduce(1 if native_setup_failed["v"] else 0, dist,
                                                              dist.ReduceOp.MAX)):
                notes.append("native-sync: skipped (the communicators could not be set up)")
                continue
            progress(f"spmd: trying the {kind} transport")
            ok = 1
            try:
                spmd_open(kind)
                try:
                    step()  # the first warm-up proof doubles as the transport check
                finally:
                    spmd_close(kind)
                if proofs[-1] != ref:
                    ok = 0
                    proofs.pop()
                    notes.append(f"{kind}: proof bytes differ from this rank's single-GPU proof")
            except Exception as e:  # every rank learns of any failure and tries the next
                ok = 0
                notes.append(f"{kind}: {type(e).__name__}: {str(e)[:200]}")
            if int(ctrl_all_reduce(ok, dist, dist.ReduceOp.MIN)):
                spmd_kind["kind"] = kind
                break
            if kind.startswith("native"):
                h2g.comm_destroy()
        if spmd_kind["kind"] is None:
            raise RuntimeError("no SPMD transport proved on every rank: " + "; ".join(notes))
        native = spmd_kind["kind"].startswith("native")
        if spmd_kind["kind"] == "host" and dist.get_backend() == "nccl":
            RCCL_SUSPECT = True
        if notes:
            transport_note = "fell back to the " + spmd_kind["kind"] + " transport after: " + "; ".join(notes)

    def session(body):
        """shard: rank 0 proves with the slab transport installed, peers serve until it
        stops; spmd: every rank proves with the all-gather installed"""
        if spmd:
            kind = spmd_kind["kind"]
            if kind.startswith("native"):
                h2g.comm_spmd_install(not args.no_subcosets)
            else:
                gather.install()
            try:
                body()
            finally:
                spmd_close(kind)
            return
        if worker:
            if native:
                h2g.comm_serve(params)
            else:
                slabs.serve()
            return
        if native:
            h2g.comm_install(params)
        elif client:
            client.install()
        try:
            body()
        finally:
            if native:
                h2g.comm_stop()
            elif client:
                client.uninstall()
                client.stop()

    def warm():
        for _ in range(args.warmup):
            step()

    def timed():
        for _ in range(args.steps):
            step()

    box = box_block(h2g) if rank == 0 else None  # before the timed region
    progress(f"prove workload: {args.warmup} warm-up proofs")
    session(warm)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier(group=CTRL)
    torch.cuda.synchronize()
    h2g.profile_enable(True)
    if spmd:
        h2g.spmd_stats(reset=True)
    t0 = time.perf_counter()
    progress(f"prove workload: {args.steps} timed proofs")
    session(timed)
    torch.cuda.synchronize()
    t_local = time.perf_counter() - t0  # this rank's proofs, before the closing barrier
    if world > 1:
        dist.barrier(group=CTRL)
    elapsed = time.perf_counter() - t0
    h2g.profile_enable(False)
    calls, phases, union = h2g.profile_msm_collect(with_union=True)
    per_rank = None
    if spmd:  # attribution: each rank's proof time, and the part of it inside each collective kind
        st_ = h2g.spmd_stats(reset=True)
        mine = [t_local / args.steps * 1e3] + [st_[k]["ms"] / args.steps for k in h2g.SPMD_COLLECTIVES] + \
               [st_[k]["calls"] / args.steps for k in h2g.SPMD_COLLECTIVES] + \
               [st_[k]["bytes"] / args.steps for k in h2g.SPMD_COLLECTIVES]
        t = torch.tensor(mine, dtype=torch.float64)
        allt = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(allt, t, group=CTRL)
        per_rank = []
        nk = len(h2g.SPMD_COLLECTIVES)
        for r, v in enumerate(allt):
            v = v.tolist()
            coll = {k: {"ms": round(v[1 + i], 3), "calls": v[1 + nk + i], "mb": round(v[1 + 2 * nk + i] / 1e6, 2)}
                    for i, k in enumerate(h2g.SPMD_COLLECTIVES)}
            cms = sum(c["ms"] for c in coll.values())
            per_rank.append({"rank": r, "proof_ms": round(v[0], 3), "in_collectives_ms": round(cms, 3),
                             "compute_ms": round(v[0] - cms, 3), "collectives_per_proof": coll})
    elapsed = max_over_ranks(elapsed, dist, world, dev)
    line = None
    extra = {}
    if spmd:  # every rank wrote the proof: the same bytes on all ranks
        import hashlib
        hd = torch.frombuffer(bytearray(hashlib.sha256(proofs[0]).digest()), dtype=torch.uint8).to(torch.int64)
        allh = [torch.empty_like(hd) for _ in range(world)]
        dist.all_gather(allh, hd, group=CTRL)
        extra["ranks_equal"] = all(bool(torch.equal(a, allh[0])) for a in allh)
    if rank == 0:
        assert all(p == proofs[0] for p in proofs), "non-deterministic proof bytes"
        # outside the timed region: the proof checked by the independent verifier
        # (oracle/py/verifier.py, the checker), and one proof with synchronised stage
        # boundaries for a per-stage GPU time breakdown
        extra["verified"] = verify_proof(h2g, circ, pk, params, proofs[0])
        stages = []
        pcie = None
        rngcore = None
        if not one_proof:
            h2g.prover_stage_sync(True)
            step()
            h2g.prover_stage_sync(False)
            stages = h2g.prover_stages()
            assert proofs[-1] == proofs[0]
            # PCIe-inclusive (the metric includes host <-> device transfers): the
            # advice handed over in host memory, as a Rust host holding the witness would;
            # as many proofs as the timed steps, each timed alone, median reported
            pts = []
            for _ in range(args.steps):
                t0 = time.perf_counter()
                pp = pk.create_proof(wit)
                pts.append(time.perf_counter() - t0)
                assert pp == proofs[0]
            pcie = {"median_s": round(sorted(pts)[len(pts) // 2], 4), "min_s": round(min(pts), 4),
                    "max_s": round(max(pts), 4), "proofs": len(pts),
                    "note": "advice uploaded from pageable host memory inside each proof (the random polynomial's "
                            "commitment runs under the first column's upload, each later upload under the previous "
                            "column's commitment MSM); same proof bytes.  This is SURVEY 8d's timing convention "
                            "(create_proof including host<->device transfers); `value` keeps the witness resident "
                            "in HBM as the bench contract asks"}
            # the caller-RNG form (create_proof(..., rng: R: RngCore, ...)): the same
            # ChaCha20 stream drawn through the h2g_rng callback struct by h2g_create_proof_multi,
            # advice device-resident as in `value`; as many proofs as the timed steps, median
            rts = []
            for _ in range(args.steps):
                t0 = time.perf_counter()
                pp = pk.create_proof_multi([wit], rng="native", advice_dev_ptrs=[adv.data_ptr()])
                rts.append(time.perf_counter() - t0)
                assert pp == proofs[0]
            rngcore = {"median_s": round(sorted(rts)[len(rts) // 2], 4), "min_s": round(min(rts), 4),
                       "max_s": round(max(rts), 4), "proofs": len(rts),
                       "note": "h2g_create_proof_multi with an h2g_rng callback (ChaCha20Rng from [7; 32] drawn "
                               "through fill_bytes); advice device-resident; same proof bytes"}
        ms_per_step = elapsed / args.steps * 1e3
        msm_ms = sum(phases.values()) / max(calls, 1)
        n_local = h2g_dist.slab(n, world, 1)[0] if one_proof else n  # rank 0's points per MSM
        line = {
            "metric": METRIC,
            "value": round(elapsed / (args.steps * (1 if one_proof else world)), 4),
            "unit": "s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": False,
            "scaling": "strong" if one_proof else "weak",
            "vs_baseline": None,
            "dtype": "u32 limbs (BN254 Fr/Fq Montgomery, 256-bit modular integer)",
            "data": ("synthetic keccak-style witness (nibble xor chains, 16 lookups into a 3-column table)"
                     if args.workload == "keccak" else
                     "synthetic C3 witness (random b, a_0; a_{i+1} = c_i = a_i b_i)")
                    + ", SRS from a fixed s generated on device, prover rng ChaCha20([7; 32])",
            "config": {"workload": (f"create_proof (KZG/SHPLONK/Blake2b) of the keccak256-style circuit (32 advice, "
                                    f"5 fixed, 16 lookups) at k={k} (BASELINE configs[4])"
                                    if args.workload == "keccak" else
                                    f"create_proof (KZG/SHPLONK/Blake2b) of the C3 synthetic circuit at k={k} "
                                    "(BASELINE configs[2]/[3])"),
                       "k": k, "advice": circ.num_advice, "fixed": circ.num_fixed,
                       "lookups": len(circ.lookups), "permutation_columns": len(circ.perm_columns), "degree": pk.degree,
                       "extended_k": pk.extended_k, "proof_bytes": len(proofs[0]),
                       "parallelism": ("single GPU per proof" if world == 1 else
                                       f"one proof over {world} GPUs, SPMD: every rank runs the prover and "
                                       "computes its point slab of each commitment MSM, partials all-gathered ("
                                       + ("libh2g RCCL all-gather" if native else
                                          "torch.distributed all_gather over "
                                          + ("RCCL" if spmd_kind["kind"] == "torch" else "gloo, host-staged"))
                                       + ("); extended-domain cosets + evaluate_h replicated" if args.no_subcosets else
                                          "); extended-domain sub-cosets + evaluate_h divided over the ranks, h "
                                          "broadcast; other transforms and SHPLONK replicated") if spmd else
                                       f"one proof over {world} GPUs: commitment MSMs in point slabs ("
                                       + ("libh2g RCCL communicators" if native else "torch.distributed p2p")
                                       + " slabs + partials), NTT/evaluate_h/SHPLONK on rank 0" if shard else
                                       f"{world} independent provers")},
            "roofline": roofline_from_phases(calls, phases, n_local, traffic, traffic_note, union=union,
                                             peak_gps=box["modmul_f29_gps"]),
            "box": box,
            "value_normalised": round(elapsed / (args.steps * (1 if one_proof else world)) *
                                      box["modmul_f29_gps"] / MODMUL_F29_REF_GPS, 4),
            "value_normalised_basis": f"value x box.modmul_f29_gps / {MODMUL_F29_REF_GPS} G/s (F29 products, the "
                                      "hot kernels' arithmetic)",
            "value_normalised_fips": round(elapsed / (args.steps * (1 if one_proof else world)) *
                                           box["modmul_ref_gps"] / MODMUL_REF_GPS, 4),
            "msm_in_prover": {"launches_per_proof": calls // max(args.steps, 1), "avg_ms": round(msm_ms, 4),
                              "busy_ms_per_proof": round(union["msm"] / args.steps, 3),
                              "accumulate_busy_ms_per_proof": round(union["accumulate"] / args.steps, 3),
                              "points_per_launch": n_local,
                              "mscalar_mul_per_s": round(n_local / (msm_ms * 1e-3) / 1e6, 2) if msm_ms else None,
                              "phases_ms": {kk: round(v / max(calls, 1), 4) for kk, v in phases.items()}},
            "verified": extra["verified"],
            "stages_ms_synced_proof": {nm: round(ms, 3) for nm, ms in stages},
        }
        if world == 1 and args.workload == "prove":
            # the roofline's kernel figure from lone launches of the same MSM shape (no other
            # stream's kernels inside a launch); the in-proof launches' figures stay beside it
            rp = line["roofline"]
            progress("lone MSM leg (roofline kernel time)")
            lcalls, lphases, lunion = lone_msm_leg(h2g, torch, dev, k)
            roof = roofline_from_phases(lcalls, lphases, n, traffic, traffic_note,
                                        union={"entries": lunion.get("entries")}, peak_gps=box["modmul_f29_gps"])
            roof["kernel_ms_source"] = (f"mean HIP-event duration of msm_acc_kernel over {lcalls} lone 2^{k} "
                                        "fixed-base MSMs (lone_msm_leg, outside the timed region; one stream, "
                                        "nothing else in flight)")
            roof["in_proof"] = {"kernel_ms": rp["kernel_ms"], "launches": rp["launches"],
                                "valu_achieved": rp["valu"]["achieved"], "valu_aggregate": rp["valu"].get("aggregate"),
                                "note": "the timed proofs' launches, HIP events on the two MSM streams: a launch "
                                        "that shares the chip with the other stream's MSM runs longer; aggregate = "
                                        "all launches' modmuls / the union of their intervals"}
            line["roofline"] = roof
            progress("NTT leg")
            line["ntt"] = ntt_leg(h2g, box)
        if pcie:
            line["pcie_inclusive"] = pcie
            line["pcie_inclusive_s"] = pcie["median_s"]
            line["rngcore"] = rngcore
            line["rngcore_s"] = rngcore["median_s"]
        if spmd:
            line["proof_bytes_equal_across_ranks"] = extra["ranks_equal"]
            line["config"]["spmd_slab_weights"] = spmd_weights["w"]
            line["per_rank"] = per_rank
            line["transport"] = {"kind": spmd_kind["kind"],
                                 "column_exchanges": ("overlapped (second RCCL communicator)"
                                                      if spmd_kind["kind"] == "native" else
                                                      "blocking" if spmd_kind["kind"] == "native-sync" else
                                                      "deferred, host transport"),
                                 "checked_against": "each rank's single-GPU proof (bytes equal)",
                                 "torch_backend": dist.get_backend(),
                                 "torch_world": dist.get_world_size()}
            if native:
                cnt, rk = h2g.comm_info()
                line["transport"]["rccl_comm_count"] = cnt
                line["transport"]["rccl_comm_rank0"] = rk
        if transport_note:
            line["transport_note"] = transport_note
    if args.workload == "prove" and (world == 1 or dist.get_backend() == "nccl"):
        # every rank takes part when sharded (collectives inside)
        progress("MSM 2^24 leg")
        m = measure_msm(h2g, torch, dev, 24, steps=10, warmup=2, dist=dist, world=world, rank=rank)
        if line is not None:
            line["msm_2p24"] = m
    if native:
        h2g.comm_destroy()
    if not worker:
        pk.close()
        del adv
    want_cpu = line is not None and world == 1 and not args.no_cpu_baseline and args.workload == "prove"
    g = gl = None
    if want_cpu:
        g, gl = params.export()
    params.close()
    torch.cuda.empty_cache()
    if line is not None and world == 1 and args.workload == "prove" and not args.no_krange:
        progress("k-range proofs")
        line["k_range"] = k_range(h2g, torch, dev, args)
    if want_cpu:
        cb = cpu_baseline_prove(circ, wit, g, gl, k, reps=args.cpu_reps)
        if not args.no_cpu_faithful:
            cb["faithful"] = cpu_baseline_faithful(h2g, k=args.cpu_faithful_k)
        line["cpu_baseline"] = cb
        line["gpu_vs_cpu"] = round(cb["value"] / line["value"], 1)
    return line


def lone_msm_leg(h2g, torch, dev, log_n, steps=10, warmup=2):
    """the dominant kernel measured alone: `steps` fixed-base MSMs of 2^log_n resident SRS
    points (the proof's commitment shape: same n, same window bits, same table layout), one
    at a time on one stream, so the accumulation's HIP events bracket a launch with no other
    kernel in flight -- the figure tools/trace_grid_stats.py recomputes from the trace
    ("lone" rows of msm_acc_kernel at that grid)"""
    import h2g_circuit as hc
    stream = torch.cuda.current_stream().cuda_stream
    n = 1 << log_n
    rng = np.random.default_rng(4242)
    bases = torch.empty((n, 8), dtype=torch.int64, device=dev)
    h2g.srs_setup_dev(np.asarray(hc.fr_to_limbs(0x1234567), dtype=np.uint64), n, bases.data_ptr(), stream)
    scalars = torch.from_numpy(random_scalars(rng, n).view(np.int64)).to(dev)
    torch.cuda.synchronize()
    base = h2g.base_descriptor_dev(bases.data_ptr(), n, 0)
    for _ in range(warmup):
        h2g.msm_with_cached_base_dev(scalars.data_ptr(), n, base, 0, stream)
    torch.cuda.synchronize()
    h2g.profile_enable(True)
    for _ in range(steps):
        h2g.msm_with_cached_base_dev(scalars.data_ptr(), n, base, 0, stream)
    torch.cuda.synchronize()
    h2g.profile_enable(False)
    calls, phases, union = h2g.profile_msm_collect(with_union=True)
    h2g.descriptor_free(base)
    del bases, scalars
    torch.cuda.empty_cache()
    return calls, phases, union


def ntt_split(L):
    """mirror of ntt_split (csrc/ntt.hip): the passes' radix bits, 3..6 each, last pass 6"""
    if L <= 11:  # NTT_SMALL_MAX_LOG: one block in LDS
        return [L]
    p = (L + 5) // 6
    r = L - 6 * (p - 1)
    lg = [r] if r >= 3 else [3, r + 3]
    return lg + [6] * (p - len(lg))


def ntt_pass_products(M, last, one, first_sparse=False):
    """Montgomery products one lane (8 elements) of a radix-2^M F29 pass executes
    (csrc/ntt.hip WaveDif29): round A's 3 stages x 4 butterflies (stage_a), round B's
    butterflies with a nonzero twiddle index (stage_b: 0 / 2 / 3 for its row bits 0 / 1 / 2),
    then the 8 inter-pass twiddles -- or the last pass's 8 epilogue constants, none when
    the constant is one (ntt_last29_kernel ONE: a reduce29 instead).  The sparse first
    pass: 3 products for y_k = x_0 + w_8^k x_1 and the 8 twiddles."""
    if first_sparse:
        return 3 + 8
    b = sum((0, 2, 3)[t] for t in range(M - 3))
    return 12 + b + (0 if (last and one) else 8)


def ntt_products(L, n_in=None, distribute=False, one=True):
    """(per-pass products, butterflies) of one transform of 2^L elements; n_in < 2^L is a
    zero-padded input (a coset extension), `distribute` multiplies the inputs by the coset
    powers in the first pass (2 of every 3)"""
    N = 1 << L
    n_in = N if n_in is None else n_in
    lg = ntt_split(L)
    per = []
    for i, M in enumerate(lg):
        sparse = i == 0 and M == 3 and n_in <= N // 4
        prod = N // 8 * ntt_pass_products(M, i == len(lg) - 1, one, sparse)
        if i == 0 and distribute:
            prod += 2 * n_in // 3
        per.append(prod)
    return per, N // 2 * L


def ntt_leg(h2g, box, sizes=(20, 22), reps=20):
    """the NTT row of the bench line: device transforms of 2^20 and
    2^22 elements -- the FFT, lagrange_to_coeff (1/n folded into the first pass) and the 2x
    coset extension (coeff_to_extended of a degree-3 domain, 2^(k+1) points) -- each the mean
    of `reps` back-to-back calls between HIP events on the library stream, with the F29
    products its passes execute (ntt_products) against this box's F29 product rate"""
    L = h2g.lib()
    rng = np.random.default_rng(77)
    out = {}
    for log_n in sizes:
        n = 1 << log_n
        a = random_scalars(rng, n)
        d = h2g.DevBuf.from_array(a)
        dom = h2g.Domain(3, log_n)
        ext = h2g.DevBuf(dom.extended_len * 32)
        w = dom.consts[0]
        tm = h2g.Timer()
        rows = {}
        cases = (("fft", lambda: h2g.fft_dev(d.ptr, log_n, w), log_n, ntt_products(log_n)),
                 ("lagrange_to_coeff", lambda: h2g.check(L.h2g_lagrange_to_coeff_dev(dom.h, h2g.VP(d.ptr), None)),
                  log_n, ntt_products(log_n)),
                 ("coeff_to_extended_x2",
                  lambda: h2g.check(L.h2g_coeff_to_extended_dev(dom.h, h2g.VP(d.ptr), h2g.VP(ext.ptr), None)),
                  dom.extended_k, ntt_products(dom.extended_k, n_in=n, distribute=True)))
        for name, fn, tl, (per, bfly) in cases:
            for _ in range(3):
                fn()
            h2g.check(L.h2g_synchronize())
            tm.start()
            for _ in range(reps):
                fn()
            ms = tm.stop_ms() / reps
            prods = sum(per)
            gps = prods / (ms * 1e-3) / 1e9
            rows[name] = {"points": 1 << tl, "ms": round(ms, 4), "passes": ntt_split(tl),
                          "products_per_pass": per, "products": prods, "radix2_butterflies": bfly,
                          "g_products_per_s": round(gps, 2),
                          "frac_of_box_f29": round(gps / box["modmul_f29_gps"], 3) if box else None,
                          "hbm_gbs_64B_per_element_pass": round(64 * (1 << tl) * len(per) / (ms * 1e-3) / 1e9, 1)}
        out[f"2^{log_n}"] = rows
        d.close()
        ext.close()
        dom.close()
    return {"transforms": out,
            "note": "products counted per pass as the F29 kernels execute them (round A 12 + round B's nonzero "
                    "twiddles + 8 inter-pass twiddles or epilogue constants per 8 elements; the last pass of these "
                    "transforms has constant one: reduce29, no products); frac = products/s over box.modmul_f29_gps "
                    "(a lone mul29 loop): the passes' adds, shuffles and loads share the same VALU"}


def k_range(h2g, torch, dev, args):
    """north_star's "prove-time on synthetic circuits at k=20..24": one GPU, C3 at k = 20
    and 24 (the bench line's value is k = 22) and the keccak-style circuit of configs[4]
    at k = 18 -- per workload `steps` proofs (witness resident in HBM) after `warmup`,
    each timed alone (host clock around the synchronous call), median / min reported, the
    proof verified by the checker's verifier.  Outside the main timed region."""
    import h2g_circuit as hc
    out = {}
    for name, k in (("c3_k20", 20), ("c3_k24", 24), ("keccak_k18", KECCAK_K)):
        if name.startswith("keccak"):
            circ, wit = hc.keccak_style(k, words=16, seed=5)
        else:
            circ, wit = hc.synthetic_c3(k, h2g.DeviceOps, seed=3)
        params = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(0x1234567 + k), dtype=np.uint64))
        pk = h2g.ProvingKey(params, circ)
        adv = torch.from_numpy(np.ascontiguousarray(wit.advice).view(np.int64)).to(dev)
        torch.cuda.synchronize()
        steps = max(3, min(args.steps, 10))
        for _ in range(max(1, min(args.warmup, 3))):
            proof = pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
        ts = []
        for _ in range(steps):
            t0 = time.perf_counter()
            p = pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
            ts.append(time.perf_counter() - t0)
            assert p == proof, f"{name}: non-deterministic proof bytes"
        ts.sort()
        out[name] = {"k": k, "median_s": round(ts[len(ts) // 2], 4), "min_s": round(ts[0], 4), "proofs": steps,
                     "extended_k": pk.extended_k, "advice": circ.num_advice, "lookups": len(circ.lookups),
                     "proof_bytes": len(proof), "verified": verify_proof(h2g, circ, pk, params, proof)}
        pk.close()
        params.close()
        del adv
        torch.cuda.empty_cache()
    return out


def verify_proof(h2g, circ, pk, params, proof):
    """prove -> verify (halo2_proofs/tests/plonk_api.rs): the checker's verifier with the
    device key's VK commitments (the device VK equals the CPU-computed one in
    tests/test_gpu_baseline_sizes.py) and the params' G2 elements -- DualMSM::check by the
    pairing (oracle/py/pairing_ref.py), no SRS secret involved"""
    sys.path.insert(0, os.path.join(REPO, "oracle", "py"))
    import verifier as V
    f, p = pk.vk_commitments()
    vk = ([V.affine_from_limbs(c) for c in f], [V.affine_from_limbs(c) for c in p])
    g2, s_g2 = params.g2()
    return bool(V.verify(circ, [], proof, None, vk=vk, g2=(V.g2_from_limbs(g2), V.g2_from_limbs(s_g2))))


def measure_msm(h2g, torch, dev, log_n, steps, warmup, dist=None, world=1, rank=0):
    """the metric's MSM half: one MSM of 2^log_n resident (scalar, SRS point) pairs through
    the base-descriptor path (fixed-base windows), HIP-event timed on the MSM stream.
    world > 1: the same MSM strong-scaled over the ranks -- rank r holds point slab
    [n r / world, n (r + 1) / world) and its scalars and runs a whole MSM on it, each step
    ending with the all_gather of the 64-B partials and their host sum; the time is the
    slowest rank's."""
    stream = torch.cuda.current_stream().cuda_stream
    n = 1 << log_n
    n_loc = n if world == 1 else n // world
    rng = np.random.default_rng(1000 + rank)
    bases = torch.empty((n_loc, 8), dtype=torch.int64, device=dev)
    h2g.srs_setup_dev(random_scalars(rng, 1)[0], n_loc, bases.data_ptr(), stream)
    scalars = torch.from_numpy(random_scalars(rng, n_loc).view(np.int64)).to(dev)
    torch.cuda.synchronize()
    base = h2g.base_descriptor_dev(bases.data_ptr(), n_loc, 0)
    out = {}

    def step():
        out["p"] = h2g.msm_with_cached_base_dev(scalars.data_ptr(), n_loc, base, 0, stream)
        if world > 1:
            out["total"] = combine_partials(gather_partials(out["p"], dist, world, dev), h2g.g1_add_affine)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier(group=CTRL)
    torch.cuda.synchronize()
    h2g.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier(group=CTRL)
    el = time.perf_counter() - t0
    h2g.profile_enable(False)
    calls, phases = h2g.profile_msm_collect()
    el = max_over_ranks(el, dist, world, dev)
    h2g.descriptor_free(base)
    del bases, scalars
    torch.cuda.empty_cache()
    return {"value": round(n * steps / el / 1e6, 2), "unit": "Mscalar-mul/s", "points": n, "steps": steps,
            "ms_per_msm": round(el / steps * 1e3, 3), "window_bits": fixed_c(n_loc),
            "n_gpus": world, "points_per_gpu": n_loc,
            "scaling": ("strong (one 2^%d MSM split into %d point slabs, all_gather of partials)" % (log_n, world))
                       if world > 1 else "single GPU",
            "phases_ms": {kk: round(v / max(calls, 1), 4) for kk, v in phases.items()}}


def run_msm(args, h2g, torch, dist, world, rank, dev, traffic, traffic_note):
    stream = torch.cuda.current_stream().cuda_stream
    n = 1 << args.log_n
    rng = np.random.default_rng(1000 + rank)
    s = random_scalars(rng, 1)[0]
    bases = torch.empty((n, 8), dtype=torch.int64, device=dev)
    h2g.srs_setup_dev(s, n, bases.data_ptr(), stream)
    scalars = torch.from_numpy(random_scalars(rng, n).view(np.int64)).to(dev)
    torch.cuda.synchronize()
    # resident bases registered once (MsmAccel base descriptor): fixed-base windows
    base = h2g.base_descriptor_dev(bases.data_ptr(), n, args.window_bits)
    result = {}

    def step():
        result["p"] = h2g.msm_with_cached_base_dev(scalars.data_ptr(), n, base, 0, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier(group=CTRL)
    torch.cuda.synchronize()
    h2g.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if world > 1:
            result["parts"] = gather_partials(result["p"], dist, world, dev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier(group=CTRL)
    elapsed = time.perf_counter() - t0
    h2g.profile_enable(False)
    calls, phases, union = h2g.profile_msm_collect(with_union=True)
    elapsed = max_over_ranks(elapsed, dist, world, dev)
    if world > 1:  # the job's MSM result (outside the timed region)
        result["total"] = combine_partials(result["parts"], h2g.g1_add_affine)
    if rank != 0:
        return None
    h2g.descriptor_free(base)
    c = args.window_bits or fixed_c(n)
    return {
        "metric": METRIC,
        "value": round(world * n * args.steps / elapsed / 1e6, 3),
        "unit": "Mscalar-mul/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 limbs (BN254 Fr/Fq Montgomery, 256-bit modular integer)",
        "data": "synthetic: uniform random Fr scalars, SRS bases [s^i]G generated on device",
        "config": {"workload": f"BN254 G1 MSM, 2^{args.log_n} resident points per GPU (the metric's MSM half), "
                               "fixed-base windows via the base descriptor",
                   "points_per_gpu": n, "window_bits": c, "windows": (255 + c - 1) // c,
                   "parallelism": f"point-slab shard x{world} + RCCL all_gather of partials"},
        "roofline": roofline_from_phases(calls, phases, n, traffic, traffic_note,
                                         union={"entries": union.get("entries")}),
        "phases_ms": {kk: round(v / max(calls, 1), 4) for kk, v in phases.items()},
    }


def spawn_ranks(n):
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=("prove", "keccak", "msm"), default="prove")
    ap.add_argument("--k", type=int, default=0, help="prove: 22 (C3), keccak: 18")
    ap.add_argument("--log-n", type=int, default=24)
    ap.add_argument("--window-bits", type=int, default=0, help="MSM workload: fixed-base window bits (0: auto)")
    ap.add_argument("--mode", choices=("spmd", "shard", "replicas"), default="spmd",
                    help="prove workload, N > 1: one proof over all GPUs -- every rank proves its MSM slabs "
                         "(spmd) or rank 0 proves and peers serve slabs (shard) -- or one proof per GPU (replicas)")
    ap.add_argument("--no-subcosets", action="store_true",
                    help="spmd: replicate the extended-domain work instead of splitting its sub-cosets")
    ap.add_argument("--spmd-owner-weight", type=float, default=-1,
                    help="spmd: slab weight of the sub-coset owners against 1 for the other ranks "
                         "(0: uniform, -1: measured default for the ratio of ranks to owners)")
    ap.add_argument("--comm-timeout", type=float, default=120.0,
                    help="N > 1: seconds any wait on libh2g's RCCL communicators may take (setup, each "
                         "collective); past it they are aborted, the proof fails on that rank, and every "
                         "rank moves to the next transport of --spmd-transports")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sync-exchange", action="store_true",
                    help="spmd over the library's RCCL communicators: skip the overlapped column exchanges (the "
                         "'native' transport) and start from 'native-sync' (blocking exchanges)")
    ap.add_argument("--cpu-reps", type=int, default=3, help="CPU baseline runs (median)")
    ap.add_argument("--no-cpu-faithful", action="store_true", help="skip the faithful-mode CPU baseline")
    ap.add_argument("--cpu-faithful-k", type=int, default=20, help="k of the faithful-mode CPU baseline")
    ap.add_argument("--no-krange", action="store_true",
                    help="prove workload: skip the k = 20 / 24 and keccak-style k = 18 timings")
    ap.add_argument("--no-pmc", action="store_true", help="skip the PMC traffic passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl", help=argparse.SUPPRESS)
    ap.add_argument("--transport", choices=("native", "torch"), default="native",
                    help="shard mode: libh2g's own RCCL communicators, or torch.distributed slabs (h2g_dist)")
    ap.add_argument("--spmd-transports", default="native,native-sync,torch,host",
                    help="spmd: transports to try in order, the first that proves on every rank is used "
                         "(native = libh2g's RCCL communicator, torch = torch.distributed over RCCL, "
                         "host = torch.distributed over gloo with host-staged exchanges)")
    args = ap.parse_args()
    if not args.k:
        args.k = KECCAK_K if args.workload == "keccak" else PROVE_K
    if args.pmc_child:
        return pmc_child(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: torchrun as a CHILD process, started before anything here
        # touches the GPU; its rank 0 prints the JSON line
        return spawn_ranks(args.gpus)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world_env:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        return 2
    traffic, traffic_note = (None, "skipped (--no-pmc)")
    if not args.no_pmc and world_env == 1:
        traffic, traffic_note = pmc_traffic(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    global CTRL
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if args.dist_backend == "gloo":  # rehearsal: ranks may share GPUs, host-staged exchanges
            args.transport = "torch"  # RCCL refuses two ranks on one GPU
            local %= torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
            CTRL = dist.group.WORLD
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            CTRL = dist.new_group(backend="gloo")
    else:
        torch.cuda.set_device(0)

    import h2g

    h2g.init([torch.cuda.current_device()])
    dev = torch.device("cuda", torch.cuda.current_device())
    run = run_msm if args.workload == "msm" else run_prove
    line = run(args, h2g, torch, dist, world, rank, dev, traffic, traffic_note)
    if rank == 0:
        if not args.no_cpu_baseline and world == 1 and args.workload == "msm":
            cb = cpu_baseline_msm()
            line["cpu_baseline"] = cb
            line["gpu_vs_cpu"] = round(line["value"] / cb["value"], 1)
        print(json.dumps(line), flush=True)
    h2g.shutdown()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
