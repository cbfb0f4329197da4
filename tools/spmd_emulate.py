#!/usr/bin/env python3
"""Per-rank cost of one SPMD proof at world N, measured on ONE GPU.

The driver's 8-GPU node is the only place the SPMD prover runs at N > 1 on RCCL.  This
tool measures what one rank of an N-rank proof computes: it installs an SPMD transport
with (world = N, rank = r) whose collectives return at once -- the all-gather hands back
this rank's own partial and digest for itself and the generator for the peers, broadcasts
and exchanges are no-ops -- so the rank runs exactly its share of the kernels (its MSM
slabs, its sub-cosets, its coefficient slabs) and the proof bytes are meaningless.  The
column-ownership exchanges are posted and waited for as over RCCL (h2g_set_spmd_exchange_async):
their modelled wire time is a wait kernel on a side stream, so it overlaps the stages after
them exactly as far as the prover lets it (--sync-exchange: charged on the host instead).  The
time per proof of the slowest rank plus a communication model (comm_model below) is the
predicted N-GPU proof time.

    python tools/spmd_emulate.py --k 22 --world 8 [--ranks 0,1,2] [--workload c3|keccak]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "yet-another-halo2-fork_amd"))

import h2g  # noqa: E402
import h2g_circuit as hc  # noqa: E402
import h2g_dist as D  # noqa: E402

FQ_P = 0x30644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd47


def _fq_mont_limbs(v):
    m = (v << 256) % FQ_P
    return [(m >> (64 * i)) & (2**64 - 1) for i in range(4)]


COMMIT_TAG = 0x54494d4d4f433248  # prover.cpp kSpmdCommitTag
G1_GEN_MONT = np.array(_fq_mont_limbs(1) + _fq_mont_limbs(2), dtype=np.uint64)  # (1, 2), Montgomery form


def spin(seconds):
    """busy-wait (time.sleep is too coarse for tens of microseconds)"""
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        pass


class CommModel:
    """a collective's modelled wire time on the node's xGMI (point-to-point links, every
    pair of GPUs on its own link): latency + the bytes the busiest link carries / link
    bandwidth.  All-gather of b bytes per rank: each rank receives b from every peer over
    a separate link -> b per link; exchange: the largest per-peer block; broadcast: b on
    each of the root's links.  Charged on the host inside the collective's callback, where
    the real transport blocks the prover (the exchanges drain the stream first)."""

    def __init__(self, gbs, lat_us):
        self.bw = gbs * 1e9
        self.lat = lat_us * 1e-6
        self.charged = 0.0
        self.by_kind = {}

    def charge(self, link_bytes, kind):
        t = self.lat + link_bytes / self.bw
        self.charged += t
        c = self.by_kind.setdefault(kind, [0.0, 0, 0])
        c[0] += t
        c[1] += 1
        c[2] = max(c[2], int(link_bytes))
        return t

    def wait(self, link_bytes, kind):
        spin(self.charge(link_bytes, kind))


class FakeCollectives:
    """world x the rank's own payload; the peers' partials are a fixed nonzero point so
    the sum never degenerates to the identity (which the transcript refuses).  With a
    CommModel every collective also waits its modelled wire time."""

    def __init__(self, world, rank, gen, model=None):
        self.world, self.rank, self.gen = world, rank, gen
        self.model = model
        self.calls = self.bcasts = self.exchanges = self.xchg = self.xchg_bytes = 0
        self.log = None  # recording: [(kind, enter_s, exit_s, link_bytes)], times from self.t0
        self.t0 = 0.0

    def _rec(self, kind, enter, link):
        if self.log is not None:
            self.log.append((kind, enter - self.t0, time.perf_counter() - self.t0, int(link)))

    def _wait(self, link_bytes, kind):
        if self.model is not None:
            self.model.wait(link_bytes, kind)

    def allgather(self, seq, mine):
        t = time.perf_counter()
        self._rec("coll", t, np.asarray(mine).nbytes)
        self._wait(np.asarray(mine).nbytes, "msm_allgather")
        out = np.tile(mine, (self.world, 1))
        for r in range(self.world):
            if r != self.rank:
                out[r, :8] = self.gen
                out[r, 8] = 0
        self.calls += 1
        return out

    def bcast(self, d_ptr, nbytes, root):
        self._rec("coll", time.perf_counter(), nbytes)
        self._wait(nbytes, "bcast")
        self.bcasts += 1

    def allgather_host(self, data):
        self._rec("coll", time.perf_counter(), len(data))
        self._wait(len(data), "host_allgather")
        self.exchanges += 1
        out = [data] * self.world
        w = np.frombuffer(bytes(data), dtype=np.uint64) if len(data) % 8 == 0 and len(data) >= 16 else None
        if w is not None and int(w[0]) == COMMIT_TAG:  # a stage's commitments (commit_collect_all)
            peer = w.copy()
            rec = peer[2:].reshape(int(w[1]), -1)
            rec[:, :8] = self.gen  # the peers' partials: the generator, as in allgather
            rec[:, 8] = 0
            out = [data if r == self.rank else peer.tobytes() for r in range(self.world)]
        return out

    def exchange(self, d_send, send_bytes, d_recv, recv_bytes):
        peers = [r for r in range(self.world) if r != self.rank]
        link = max([int(send_bytes[r]) for r in peers] + [int(recv_bytes[r]) for r in peers] + [0])
        self._rec("coll", time.perf_counter(), link)
        self._wait(link, "exchange")
        self.xchg += 1
        self.xchg_bytes += sum(recv_bytes)

    def exchange_post(self, d_send, send_bytes, d_recv, recv_bytes, stream, done):
        """the overlapped exchange (h2g_set_spmd_exchange_async): its modelled wire time
        runs on the device, a wait kernel on a side stream behind the packed bytes, as the
        native transport's RCCL exchange runs on its communicator's stream; the host goes on
        at once and waits for `done` before h(X)"""
        peers = [r for r in range(self.world) if r != self.rank]
        link = max([int(send_bytes[r]) for r in peers] + [int(recv_bytes[r]) for r in peers] + [0])
        us = 1e6 * self.model.charge(link, "exchange_overlapped") if self.model is not None else 0.0
        t = time.perf_counter()
        h2g.debug_link_delay(stream, done, us)
        self._rec("post", t, link)
        self.xchg += 1
        self.xchg_bytes += sum(recv_bytes)

    def exchange_wait(self, done):
        t = time.perf_counter()
        h2g.event_wait(done)
        self._rec("wait", t, 0)


def replay(logs, gbs, lat_us):
    """The ranks' recorded proofs replayed against each other: rank r's host reaches its
    k-th collective after the local time it spent since its previous one (as measured when
    it ran alone), a blocking collective completes for every rank when the last rank has
    arrived plus its modelled wire time (the busiest rank's link), an overlapped exchange's
    wait completes no earlier than the last rank's post plus its wire time.  Returns the
    predicted proof time (ms) -- the synchronising collectives' effect that the independent
    per-rank times leave out -- or None if the ranks' collective sequences differ."""
    return replay_detail(logs, gbs, lat_us)[0]


def replay_detail(logs, gbs, lat_us):
    """replay() and, per collective, (index, kind, rank 0's local time ms, the latest
    rank, the wait it causes: latest arrival - earliest arrival, ms)"""
    bw, lat = gbs * 1e9, lat_us * 1e-6
    W = len(logs)
    skew = []
    evs = [lg["events"] for lg in logs]
    if any(len(e) != len(evs[0]) or [k for k, *_ in e] != [k for k, *_ in evs[0]] for e in evs):
        return None, []
    T = [0.0] * W
    last = [0.0] * W
    posts = []  # per posted exchange: (latest post time over ranks, its wire time)
    nwait = 0
    for k in range(len(evs[0])):
        kind = evs[0][k][0]
        arrive = [T[r] + (evs[r][k][1] - last[r]) for r in range(W)]
        wire = lat + max(evs[r][k][3] for r in range(W)) / bw
        if kind != "post":
            late = max(range(W), key=lambda r: arrive[r])
            skew.append((k, kind, round(1e3 * evs[0][k][1], 3), late, round(1e3 * (max(arrive) - min(arrive)), 3)))
        if kind == "coll":
            done = max(arrive) + wire
            T = [done + (evs[r][k][2] - evs[r][k][1]) for r in range(W)]
        elif kind == "post":
            posts.append((max(arrive), wire))
            T = [arrive[r] + (evs[r][k][2] - evs[r][k][1]) for r in range(W)]
        else:  # wait: FIFO with the posts
            pt, pw = posts[nwait]
            nwait += 1
            T = [max(arrive[r] + (evs[r][k][2] - evs[r][k][1]), pt + pw) for r in range(W)]
        last = [evs[r][k][2] for r in range(W)]
    end = [T[r] + (logs[r]["proof_s"] - last[r]) for r in range(W)]
    return 1e3 * max(end), skew


def run(args):
    import torch
    torch.cuda.set_device(0)  # torch's HIP context first (as bench.py), then the library's
    h2g.init([0])
    k = args.k
    if args.workload == "keccak":
        circ, wit = hc.keccak_style(k, words=16, seed=5)
    else:
        circ, wit = hc.synthetic_c3(k, h2g.DeviceOps, seed=3)
    params = h2g.Params(k, s=np.asarray(hc.fr_to_limbs(0x1234567), dtype=np.uint64))
    gen = G1_GEN_MONT
    pk = h2g.ProvingKey(params, circ)
    adv = torch.from_numpy(np.ascontiguousarray(wit.advice).view(np.int64)).cuda()
    torch.cuda.synchronize()
    n = 1 << k
    ranks = [int(r) for r in args.ranks.split(",")] if args.ranks else list(range(args.world))
    out = {"k": k, "workload": args.workload, "world": args.world, "comm_model": args.comm_model or None,
           "column_owners": not args.no_column_owners, "overlapped_exchanges": not args.sync_exchange,
           "ranks": {}}
    single = []
    for _ in range(args.warmup):
        pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
    for _ in range(args.steps):
        t0 = time.perf_counter()
        pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
        single.append(time.perf_counter() - t0)
    out["single_gpu_ms"] = round(1e3 * sorted(single)[len(single) // 2], 3)
    weights = None
    if args.weights:
        weights = [int(x) for x in args.weights.split(",")]
    elif args.owner_weight:
        weights = D.owner_weights(args.world, pk.extended_k, k, args.owner_weight)
    out["weights"] = weights
    h2g.spmd_set_weights(weights)
    if args.no_column_owners:
        h2g.spmd_set_column_owners(0)
    logs = {}
    for r in ranks:
        if args.world > 1:
            params.set_slab(*D.slab(n, args.world, r, weights=weights))
        model = None
        if args.comm_model:
            gbs, lat = (float(x) for x in args.comm_model.split(","))
            model = CommModel(gbs, lat)
        fc = FakeCollectives(args.world, r, gen, model)
        xchg = not (args.no_slabs or args.no_subcosets or args.bcast_h)
        h2g.set_spmd_transport(args.world, r, fc.allgather, None if args.no_subcosets else fc.bcast,
                               None if args.no_slabs else fc.allgather_host, fc.exchange if xchg else None)
        if xchg and not args.sync_exchange:
            h2g.set_spmd_exchange_async(fc.exchange_post, fc.exchange_wait)
        try:
            for _ in range(args.warmup):
                pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
            ts = []
            for _ in range(args.steps):
                t0 = time.perf_counter()
                pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
                ts.append(time.perf_counter() - t0)
            h2g.prover_stage_sync(True)
            pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
            h2g.prover_stage_sync(False)
            stages = h2g.prover_stages()
            recs = []
            if args.replay and not args.comm_model:  # the collective timeline of 3 proofs
                for _ in range(3):
                    fc.log = []
                    fc.t0 = time.perf_counter()
                    pk.create_proof(wit=wit, advice_dev_ptr=adv.data_ptr())
                    recs.append({"proof_s": time.perf_counter() - fc.t0, "events": fc.log})
                    fc.log = None
        finally:
            h2g.set_spmd_transport(1)
        ts.sort()
        out["ranks"][r] = {"median_ms": round(1e3 * ts[len(ts) // 2], 3), "min_ms": round(1e3 * ts[0], 3),
                           "gathers_per_proof": fc.calls // (args.warmup + args.steps + 1),
                           "bcasts_per_proof": fc.bcasts // (args.warmup + args.steps + 1),
                           "host_gathers_per_proof": fc.exchanges // (args.warmup + args.steps + 1),
                           "h_exchanges_per_proof": fc.xchg // (args.warmup + args.steps + 1),
                           "h_exchange_recv_bytes": fc.xchg_bytes // max(fc.xchg, 1),
                           "modelled_comm_ms_per_proof": round(1e3 * model.charged / (args.warmup + args.steps + 1), 3)
                           if model else None,
                           "modelled_comm_by_kind": {kd: {"ms_per_proof": round(1e3 * v[0] / (args.warmup + args.steps + 1), 3),
                                                          "calls_per_proof": v[1] // (args.warmup + args.steps + 1),
                                                          "max_link_mb": round(v[2] / 1e6, 2)}
                                                     for kd, v in model.by_kind.items()} if model else None,
                           "stages_ms_synced": {nm: round(ms, 3) for nm, ms in stages}}
        print(json.dumps({"rank": r, **out["ranks"][r]}), flush=True)
        if recs:
            logs.setdefault(r, recs)
    if args.world > 1:
        params.set_slab(0, 0)
    worst = max(v["median_ms"] for v in out["ranks"].values())
    out["slowest_rank_ms"] = worst
    if logs and len(logs) == args.world:  # every rank recorded: replay them against each other
        out["replay"] = {}
        for model in args.replay.split(";"):
            gbs, lat = (float(x) for x in model.split(","))
            preds = [replay([logs[r][i] for r in range(args.world)], gbs, lat) for i in range(3)]
            preds = sorted(p for p in preds if p is not None)
            out["replay"][model] = {"predicted_ms": round(preds[len(preds) // 2], 3) if preds else None,
                                    "speedup": round(out["single_gpu_ms"] / preds[len(preds) // 2], 3)
                                    if preds else None}
        _, sk = replay_detail([logs[r][0] for r in range(args.world)], 1e9, 0)
        out["replay_skew_top"] = sorted(sk, key=lambda x: -x[4])[:10]
        out["replay_note"] = ("ranks replayed against each other at their collectives (tools/spmd_emulate.py "
                              "replay): GB/s,us of the link model -> predicted proof time")
    pk.close()
    params.close()
    h2g.shutdown()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=22)
    ap.add_argument("--workload", choices=("c3", "keccak"), default="c3")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", default="")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-subcosets", action="store_true")
    ap.add_argument("--no-slabs", action="store_true", help="replicate the multi-open tail")
    ap.add_argument("--bcast-h", action="store_true", help="broadcast h evaluations (no slab exchange)")
    ap.add_argument("--weights", default="", help="SPMD slab weights, comma separated")
    ap.add_argument("--owner-weight", type=float, default=0.0,
                    help="slab weight of the sub-coset owners (h2g_dist.owner_weights), others 1")
    ap.add_argument("--no-column-owners", action="store_true",
                    help="h2g_spmd_set_column_owners(0): wide stages keep point slabs, no row pieces")
    ap.add_argument("--sync-exchange", action="store_true",
                    help="the column exchanges complete on return (charged on the host) instead of overlapped")
    ap.add_argument("--comm-model", default="",
                    help="GB/s,us: every collective waits latency + its busiest link's bytes / bandwidth "
                         "(e.g. 50,40 for xGMI); empty: collectives return at once (compute only)")
    ap.add_argument("--replay", default="",
                    help="with every rank and no --comm-model: record each rank's collective timeline and replay "
                         "the ranks against each other, one prediction per 'GB/s,us' model (';'-separated, "
                         "e.g. '1e9,0;50,40': no wire time / xGMI)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    res = run(args)
    print("EMULATE " + json.dumps(res), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
