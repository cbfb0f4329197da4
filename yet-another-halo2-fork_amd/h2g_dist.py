"""One create_proof across several GPUs: the proof's commitment MSMs are
split into contiguous point slabs, one per rank, over torch.distributed -- backend
"nccl" (RCCL over xGMI) with one process per GPU, or "gloo" with host staging (CPU
tests; several ranks sharing one GPU).

Rank 0 runs h2g_create_proof with a slab transport installed
(h2g_set_shard_transport, include/h2g.h); ranks 1.. run SlabWorker.serve(), which
answers each MSM with the affine partial sum of its slab.  The reference's MSM call
sites (MsmAccel::msm, halo2_middleware/src/zal.rs:58, via ParamsKZG::commit /
commit_lagrange, poly/kzg/commitment.rs:305-317,354-366) are unchanged in meaning: the
group sum of the slabs is the MSM, so the proof bytes do not depend on the rank count.

Messages rank 0 -> rank r per MSM: header int64[5] = (op, seq, base_set, lo, count), then
the `count` scalars of slab r = points [lo, lo + count) (int64 view of the Fr limbs).  Reply r -> 0: int64[9] = the
affine partial (8 limbs) and its identity flag.  op 0 ends a serve() session.
"""
import numpy as np

OP_STOP, OP_MSM = 0, 1


def slab(n, world, r, P=None, weights=None):
    """[lo, hi) of rank r's points in an MSM of length n: the slab of the params' P = 2^k
    points, clipped to n (the C prover's shard_lo, csrc/prover.cpp); with SPMD weights
    (h2g.spmd_set_weights) [P S_r / S, P S_{r+1} / S)"""
    P = n if P is None else P
    if weights:
        pre = [0]
        for w in weights:
            pre.append(pre[-1] + int(w))
        return min(n, P * pre[r] // pre[-1]), min(n, P * pre[r + 1] // pre[-1])
    return min(n, P * r // world), min(n, P * (r + 1) // world)


def auto_owner_weight(world, extended_k, k):
    """the sub-coset owners' slab weight measured best on one GPU (tools/spmd_emulate.py,
    C3 at k = 22, profiles/r03/s3/spmd_owner_weights): with twice as many ranks as
    sub-coset owners 0.5 (N = 4: 0.4 / 0.5 / 0.65 / 0.8 -> slowest rank 29.1 / 27.8 / 29.6
    / 30.0 ms), with four times as many or more 0.1 (N = 8: 0.1 / 0.15 / 0.2 / 0.3 / 0.4 ->
    17.5 / 17.9 / 18.2 / 19.5 / 20.4 ms)"""
    E = 1 << (extended_k - k)
    return 0.5 if world <= 2 * E else 0.1


COLSHARD_MIN_WORLD = 4  # prover.cpp kColshardMinWorld


def row_pieces_active(world, extended_k, k, column_owners=True, multiopen="shplonk"):
    """whether the library cuts sub-cosets into row pieces for this world -- the condition
    prove_impl uses (prover.cpp: column owners on, SHPLONK, world >= kColshardMinWorld,
    more ranks than sub-cosets and a multiple of them)"""
    E = 1 << (extended_k - k)
    return (column_owners and multiopen == "shplonk" and world >= COLSHARD_MIN_WORLD and world > E
            and world % E == 0)


def owner_weights(world, extended_k, k, owner_weight=None, scale=100, row_pieces=None, column_owners=True,
                  multiopen="shplonk"):
    """SPMD slab weights that lighten the ranks owning extended-domain sub-cosets: with
    2^(extended_k - k) = E < world sub-cosets, ranks r < E evaluate h on a sub-coset each
    (its n-point coset NTTs, evaluate_h, the h interpolation) on top of their MSM slabs;
    they get weight owner_weight (None: auto_owner_weight), the other ranks 1.  None when
    every rank owns one, and when the library cuts the sub-cosets into row pieces (then
    every rank evaluates h on a row piece of one sub-coset, the same share of the work).
    row_pieces None: derived from the library's own condition for the given column-owner
    mode (h2g_spmd_set_column_owners) and multi-open (row_pieces_active)"""
    E = 1 << (extended_k - k)
    if row_pieces is None:
        row_pieces = row_pieces_active(world, extended_k, k, column_owners, multiopen)
    if world <= E or (row_pieces and world % E == 0):
        return None
    if owner_weight is None:
        owner_weight = auto_owner_weight(world, extended_k, k)
    return [int(round(scale * owner_weight)) if r < E else scale for r in range(world)]


def _staging(dist, group):
    """device tensors for RCCL, host tensors for gloo"""
    import torch
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class SlabClient:
    """rank 0: sends each MSM's slabs to the peers and collects their partials"""

    def __init__(self, dist, points=None, group=None):
        """points: the params' P = 2^k (slab partition); None = each MSM's own length"""
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.device = _staging(dist, group)
        self.points = points
        self.pending = {}

    def _send(self, seq, base_set, n, fill):
        import torch
        dist, dev = self.dist, self.device
        works, keep, replies = [], [], []
        for r in range(1, self.world):
            lo, hi = slab(n, self.world, r, self.points)
            hdr = torch.tensor([OP_MSM, seq, base_set, lo, hi - lo], dtype=torch.int64, device=dev)
            keep.append(hdr)
            works.append(dist.isend(hdr, r, group=self.group))
            if hi > lo:
                buf = torch.empty((hi - lo) * 4, dtype=torch.int64, device=dev)
                fill(buf, lo, hi)
                keep.append(buf)
                works.append(dist.isend(buf, r, group=self.group))
            rep = torch.empty(9, dtype=torch.int64, device=dev)
            replies.append(rep)
            works.append(dist.irecv(rep, r, group=self.group))
        self.pending[seq] = (works, keep, replies)

    def launch(self, seq, base_set, n, d_scalars):
        """transport launch: d_scalars = device pointer to n Fr (the prover's buffer)"""
        import h2g

        def fill(buf, lo, hi):
            src = d_scalars + lo * 32
            if buf.is_cuda:
                h2g.memcpy_dtod(buf.data_ptr(), src, (hi - lo) * 32)
            else:
                h2g.memcpy_dtoh(buf.data_ptr(), src, (hi - lo) * 32)

        self._send(seq, base_set, n, fill)

    def launch_host(self, seq, base_set, scalars):
        """the same from host scalars (numpy (n, 4) uint64): CPU tests / host callers"""
        import torch
        sc = np.ascontiguousarray(scalars, dtype=np.uint64)

        def fill(buf, lo, hi):
            buf.copy_(torch.from_numpy(sc[lo:hi].reshape(-1).view(np.int64)))

        self._send(seq, base_set, len(sc), fill)

    def collect(self, seq):
        """transport collect: [(affine uint64[8], is_identity)] for ranks 1.."""
        works, _keep, replies = self.pending.pop(seq)
        for w in works:
            w.wait()
        out = []
        for rep in replies:
            a = rep.cpu().numpy().view(np.uint64)
            out.append((a[:8].copy(), bool(a[8])))
        return out

    def drain(self):
        """complete every outstanding exchange (after a failed proof) so the peers stay
        in step"""
        for seq in sorted(self.pending):
            self.collect(seq)

    def stop(self):
        """end the peers' serve() session"""
        import torch
        self.drain()
        works = []
        for r in range(1, self.world):
            hdr = torch.tensor([OP_STOP, 0, 0, 0, 0], dtype=torch.int64, device=self.device)
            works.append((hdr, self.dist.isend(hdr, r, group=self.group)))
        for _, w in works:
            w.wait()

    def install(self):
        """make this client h2g_create_proof's slab transport"""
        import h2g
        h2g.set_shard_transport(self.world, self.launch, self.collect)

    @staticmethod
    def uninstall():
        import h2g
        h2g.set_shard_transport(1)


class SlabWorker:
    """ranks 1..: serve MSM slabs until rank 0 stops the session.  engine(base_set, lo,
    n, buf) -> (affine uint64[8], is_identity), buf = the slab's int64 tensor; the default
    engine is the device MSM against the params' resident fixed-base windows."""

    def __init__(self, dist, params=None, engine=None, group=None):
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = _staging(dist, group)
        self.params = params
        self.engine = engine or self._device_engine
        self._stage = None

    def _device_engine(self, base_set, lo, n, buf):
        import h2g
        import torch
        if buf.is_cuda:
            torch.cuda.current_stream().synchronize()  # the received slab is complete
            ptr = buf.data_ptr()
        else:  # gloo: stage the host slab into a reusable device buffer
            if self._stage is None or self._stage.nbytes < n * 32:
                self._stage = h2g.DevBuf(n * 32)
            h2g.memcpy_htod(self._stage.ptr, buf.data_ptr(), n * 32)
            ptr = self._stage.ptr
        return h2g.params_msm_dev(self.params, base_set, lo, n, ptr)

    def serve(self):
        """-> number of MSM slabs served in this session"""
        import torch
        dist, dev = self.dist, self.device
        count = 0
        while True:
            hdr = torch.empty(5, dtype=torch.int64, device=dev)
            dist.recv(hdr, 0, group=self.group)
            op, seq, base_set, lo, cnt = hdr.cpu().tolist()
            if op == OP_STOP:
                return count
            if op != OP_MSM:
                raise RuntimeError(f"slab worker: unknown op {op}")
            hi = lo + cnt
            if hi > lo:
                buf = torch.empty((hi - lo) * 4, dtype=torch.int64, device=dev)
                dist.recv(buf, 0, group=self.group)
                pt, is_id = self.engine(base_set, lo, hi - lo, buf)
            else:
                pt, is_id = np.zeros(8, dtype=np.uint64), True
            rep = np.zeros(9, dtype=np.uint64)
            rep[:8] = pt
            rep[8] = 1 if is_id else 0
            dist.send(torch.from_numpy(rep.view(np.int64)).to(dev), 0, group=self.group)
            count += 1


def host_all_to_all(dist, group, rank, world, sb, send_bytes, rb, recv_bytes):
    """all-to-all of host byte tensors by point-to-point messages (gloo): peer p's bytes are
    contiguous in peer order in sb / rb; `rank` and p index the group's members, while
    P2POp takes the peer's global rank"""
    so = [sum(send_bytes[:p]) for p in range(world)]
    ro = [sum(recv_bytes[:p]) for p in range(world)]
    ops = []
    for p in range(world):
        if p == rank:
            rb[ro[p]:ro[p] + recv_bytes[p]] = sb[so[p]:so[p] + send_bytes[p]]
            continue
        peer = p if group is None else dist.get_global_rank(group, p)
        if send_bytes[p]:
            ops.append(dist.P2POp(dist.isend, sb[so[p]:so[p] + send_bytes[p]], peer, group))
        if recv_bytes[p]:
            ops.append(dist.P2POp(dist.irecv, rb[ro[p]:ro[p] + recv_bytes[p]], peer, group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()


class SpmdGather:
    """SPMD sharding over torch.distributed (h2g_set_spmd_transport): every rank runs the
    same create_proof and computes point slab `rank` of each commitment MSM; the 9-word
    partials (affine limbs + identity flag) are all-gathered in rank order and every rank
    sums them, so no scalars travel; with `slabs` the evaluations and SHPLONK run on
    coefficient slabs joined by small host all-gathers (allgather_host).
    h2g_comm_spmd_install is the same over the library's own RCCL communicator."""

    def __init__(self, dist, group=None, subcosets=True, slabs=True, h_exchange=True, exchange_async=True):
        self.dist = dist
        self.exchange_async = exchange_async
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = _staging(dist, group)
        self.subcosets = subcosets
        self.slabs = slabs
        self.h_exchange = h_exchange
        self.calls = 0
        self.bcasts = 0
        self.host_gathers = 0
        self.exchanges = 0

    def allgather_host(self, data):
        """the multi-open tail's scalars: `data` (bytes) from every rank, rank order"""
        import torch
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(self.device)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        self.host_gathers += 1
        return [o.cpu().numpy().tobytes() for o in out]

    def allgather(self, seq, mine):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(mine, dtype=np.uint64).view(np.int64)).to(self.device)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        self.calls += 1
        return np.stack([o.cpu().numpy().view(np.uint64) for o in out])

    def bcast(self, d_ptr, nbytes, root):
        """in-place broadcast of device memory from `root` (a sub-coset's h evaluations):
        staged through a torch tensor (RCCL) or host memory (gloo)"""
        import h2g
        import torch
        t = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        if self.rank == root:
            h2g.memcpy_dtod(t.data_ptr(), d_ptr, nbytes)
        if self.device.type == "cuda":
            self.dist.broadcast(t, root, group=self.group)
        else:
            h = t.cpu()
            self.dist.broadcast(h, root, group=self.group)
            t.copy_(h)
        torch.cuda.synchronize()
        if self.rank != root:
            h2g.memcpy_dtod(d_ptr, t.data_ptr(), nbytes)
        self.bcasts += 1

    def exchange(self, d_send, send_bytes, d_recv, recv_bytes):
        """all-to-all of device bytes (h(X)'s coefficient slabs from the sub-coset owners):
        torch device tensors over RCCL (all_to_all_single), host tensors and point-to-point
        messages over gloo"""
        import h2g
        import torch
        W = self.world
        tot_s, tot_r = sum(send_bytes), sum(recv_bytes)
        if self.device.type == "cuda":
            sb = torch.empty(max(tot_s, 1), dtype=torch.uint8, device="cuda")
            rb = torch.empty(max(tot_r, 1), dtype=torch.uint8, device="cuda")
            if tot_s:
                h2g.memcpy_dtod(sb.data_ptr(), d_send, tot_s)
            self.dist.all_to_all_single(rb[:tot_r], sb[:tot_s], list(recv_bytes), list(send_bytes), group=self.group)
            torch.cuda.synchronize()
            if tot_r:
                h2g.memcpy_dtod(d_recv, rb.data_ptr(), tot_r)
        else:
            sb = torch.empty(max(tot_s, 1), dtype=torch.uint8)
            rb = torch.empty(max(tot_r, 1), dtype=torch.uint8)
            if tot_s:
                h2g.memcpy_dtoh(sb.data_ptr(), d_send, tot_s)
            host_all_to_all(self.dist, self.group, self.rank, W, sb, send_bytes, rb, recv_bytes)
            if tot_r:
                h2g.memcpy_htod(d_recv, rb.data_ptr(), tot_r)
        self.exchanges += 1

    def exchange_post(self, d_send, send_bytes, d_recv, recv_bytes, stream, done):
        """the overlapped exchange (h2g_set_spmd_exchange_async) over torch.distributed:
        torch's collectives cannot wait on the library's stream, so the packed bytes are
        waited for, the exchange runs to completion, and `done` is recorded behind it -- no
        overlap (that is the native transport's, comm_exchange_post), but the prover's
        deferred receive path runs the same as over RCCL"""
        import h2g
        h2g.event_record(done, stream)
        h2g.event_wait(done)
        self.exchange(d_send, send_bytes, d_recv, recv_bytes)
        h2g.event_record(done, stream)

    def install(self):
        import h2g
        xchg = self.subcosets and self.slabs and self.h_exchange
        h2g.set_spmd_transport(self.world, self.rank, self.allgather, self.bcast if self.subcosets else None,
                               self.allgather_host if self.slabs else None, self.exchange if xchg else None)
        if xchg and self.exchange_async:
            h2g.set_spmd_exchange_async(self.exchange_post)

    @staticmethod
    def uninstall():
        import h2g
        h2g.set_spmd_transport(1)
