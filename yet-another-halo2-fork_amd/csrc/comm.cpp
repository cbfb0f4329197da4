// comm.cpp -- native RCCL exchange of create_proof's MSM slabs across GPUs (see comm.h).
//
// The reference has no multi-GPU path; SURVEY 8e places the exchange at the commitment MSMs
// (MsmAccel::msm, halo2_middleware/src/zal.rs:58, via ParamsKZG::commit / commit_lagrange,
// halo2_backend/src/poly/kzg/commitment.rs:305-317,354-366): a sum over independent points,
// so point slabs on different GPUs and one exchange of 64-B partials.  RCCL has no
// elliptic-curve reduction, so the partials travel point-to-point and rank 0 adds them.
#include "comm.h"

#include <rccl/rccl.h>

#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "comm_wait.h"
#include "runtime.h"

namespace h2g {
namespace rt {
namespace {

#define NCCLCHK(expr)                                                                              \
  do {                                                                                            \
    ncclResult_t _r = (expr);                                                                     \
    if (_r != ncclSuccess) return fail(H2G_ERR_DEVICE, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

static constexpr int RING = 16;  // outstanding MSMs on rank 0

// the deadline of every RCCL wait (communicator setup, enqueue, completion), seconds; <= 0:
// none.  Past it the communicators are aborted and the call fails (comm_wait.h).
double g_timeout_s = 300.0;
// a serving peer's idle deadline: the longest wait for rank 0's next request header (<= 0:
// none).  Rank 0 aborting its communicators need not surface as an RCCL error on the peer,
// whose pending receive would then wait forever; past this deadline the peer aborts and
// h2g_comm_serve returns an error (rank 0 renews it with comm_keepalive when it idles)
double g_serve_timeout_s = 0.0;

struct Slot {
  bool busy = false;
  uint64_t seq = 0;
  void* stage = nullptr;  // the peers' scalars (device copy)
  size_t cap = 0;
  hipEvent_t copied = nullptr, done = nullptr;
};

struct Comm {
  int world = 1, rank = 0, device = 0;
  ncclComm_t tx = nullptr, rx = nullptr;
  hipStream_t stx = nullptr, srx = nullptr;
  // rank 0
  uint64_t points = 0;             // the params' P (slab partition)
  Slot slots[RING];
  int64_t* h_hdr = nullptr;        // pinned [RING][world][5]
  int64_t* d_hdr = nullptr;        // device mirror
  int64_t* h_part = nullptr;       // pinned [RING][world][9]
  int64_t* d_part = nullptr;
  // ranks 1..
  void* rstage[2] = {nullptr, nullptr};
  size_t rcap[2] = {0, 0};
  int rnext = 0;
  int64_t *h_rhdr = nullptr, *d_rhdr = nullptr;  // one header
  int64_t *h_rpart = nullptr, *d_rpart = nullptr;
  // SPMD all-gather of partials: pinned [world][H2G_SPMD_WORDS], device in / out
  bool broken = false;  // aborted after a failed or timed-out wait: every later call fails
  uint64_t* h_ag = nullptr;
  uint64_t *d_ag_in = nullptr, *d_ag_out = nullptr;
  // SPMD host all-gather (multi-open tail): pinned / device staging, world x bytes + bytes
  void *h_hg = nullptr, *d_hg = nullptr;
  size_t hg_cap = 0;
  // overlapped exchanges (comm_exchange_post): on the second communicator and its stream,
  // so the stages' all-gathers on the first do not queue behind them; xready gates them
  // on the prover's stream
  hipEvent_t xready = nullptr;
};
Comm* g_comm = nullptr;

size_t slab_lo(uint64_t P, uint64_t n, int world, int r) {  // prover.cpp shard_lo
  const uint64_t b = (uint64_t)((unsigned __int128)P * (unsigned)r / (unsigned)world);
  return b < n ? b : n;
}

int grow(void** p, size_t* cap, size_t bytes) {
  if (bytes <= *cap) return H2G_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  HIPCHK(hipMalloc(p, bytes ? bytes : 16));
  *cap = bytes;
  return H2G_OK;
}

// ---- non-blocking communicators, every wait against g_timeout_s
using commwait::poll_until;
int nccl_poll(ncclComm_t comm) {  // a communicator's asynchronous state
  if (!comm) return commwait::POLL_ERROR;
  ncclResult_t st = ncclSuccess;
  if (ncclCommGetAsyncError(comm, &st) != ncclSuccess) return commwait::POLL_ERROR;
  return st == ncclSuccess ? commwait::POLL_DONE : (st == ncclInProgress ? commwait::POLL_PENDING : commwait::POLL_ERROR);
}
void comm_abort(Comm* c) {
  if (c->tx) (void)ncclCommAbort(c->tx);
  if (c->rx) (void)ncclCommAbort(c->rx);
  c->tx = c->rx = nullptr;
  c->broken = true;
}
int wait_failed(Comm* c, int w, const std::string& what) {
  comm_abort(c);
  return fail(H2G_ERR_DEVICE, what + (w == commwait::WAIT_TIMEOUT
                                          ? ": no progress within " + std::to_string(g_timeout_s) + " s"
                                          : ": RCCL reported an error") + "; communicators aborted");
}
// an RCCL call on a non-blocking communicator: an error aborts; ncclInProgress is polled
// until the communicator is ready for the next call
int nccl_call(Comm* c, ncclComm_t comm, ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return H2G_OK;
  if (r != ncclInProgress) {
    comm_abort(c);
    return fail(H2G_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r) + "; communicators aborted");
  }
  const int w = poll_until([&] { return nccl_poll(comm); }, g_timeout_s);
  return w == commwait::WAIT_OK ? H2G_OK : wait_failed(c, w, what);
}
#define NCCLQ(c, comm, expr) RCCHK(nccl_call(c, comm, (expr), #expr))
// the work queued on `st` (RCCL kernels among it) has finished; RCCL errors on either
// communicator end the wait early
int wait_stream(Comm* c, hipStream_t st, const char* what, double timeout_s) {
  int hip_err = 0;
  const int w = poll_until(
      [&] {
        const hipError_t e = hipStreamQuery(st);
        if (e == hipSuccess) return (int)commwait::POLL_DONE;
        if (e != hipErrorNotReady) {
          hip_err = (int)e;
          return (int)commwait::POLL_ERROR;
        }
        if (nccl_poll(c->tx) == commwait::POLL_ERROR || nccl_poll(c->rx) == commwait::POLL_ERROR)
          return (int)commwait::POLL_ERROR;
        return (int)commwait::POLL_PENDING;
      },
      timeout_s);
  if (w == commwait::WAIT_OK) return H2G_OK;
  if (hip_err) {
    comm_abort(c);
    return fail(H2G_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString((hipError_t)hip_err));
  }
  return wait_failed(c, w, what);
}
int wait_event(Comm* c, hipEvent_t ev, const char* what) {
  const int w = poll_until(
      [&] {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return (int)commwait::POLL_DONE;
        if (e != hipErrorNotReady) return (int)commwait::POLL_ERROR;
        if (nccl_poll(c->tx) == commwait::POLL_ERROR || nccl_poll(c->rx) == commwait::POLL_ERROR)
          return (int)commwait::POLL_ERROR;
        return (int)commwait::POLL_PENDING;
      },
      g_timeout_s);
  return w == commwait::WAIT_OK ? H2G_OK : wait_failed(c, w, what);
}
Comm* usable(void* ctx) {
  Comm* c = static_cast<Comm*>(ctx);
  return c && c == g_comm && !c->broken ? c : nullptr;
}

}  // namespace

int comm_set_timeout(double seconds) {
  g_timeout_s = seconds;
  return H2G_OK;
}
int comm_set_serve_timeout(double seconds) {
  g_serve_timeout_s = seconds;
  return H2G_OK;
}

int comm_unique_id(uint8_t id[COMM_ID_BYTES]) {
  ncclUniqueId a, b;
  NCCLCHK(ncclGetUniqueId(&a));
  NCCLCHK(ncclGetUniqueId(&b));
  std::memcpy(id, &a, sizeof(a));
  std::memcpy(id + 128, &b, sizeof(b));
  return H2G_OK;
}

int comm_init(const uint8_t id[COMM_ID_BYTES], int world, int rank) {
  if (g_comm) return fail(H2G_ERR_STATE, "comm_init: a communicator exists (h2g_comm_destroy first)");
  if (world < 2 || rank < 0 || rank >= world) return fail(H2G_ERR_ARG, "comm_init: bad world / rank");
  Device* d = cur();
  if (!d) return fail(H2G_ERR_STATE, "h2g_init has not been called");
  HIPCHK(hipSetDevice(d->id));
  auto c = std::make_unique<Comm>();
  c->world = world;
  c->rank = rank;
  c->device = d->id;
  ncclUniqueId a, b;
  std::memcpy(&a, id, sizeof(a));
  std::memcpy(&b, id + 128, sizeof(b));
  // non-blocking setup: both communicators connect in the background, polled against the
  // deadline (a peer that never arrives fails this call instead of hanging it)
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t r = ncclCommInitRankConfig(&c->tx, world, a, rank, &cfg);
  if (r == ncclSuccess || r == ncclInProgress) r = ncclCommInitRankConfig(&c->rx, world, b, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    comm_abort(c.get());
    return fail(H2G_ERR_DEVICE, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
  }
  const int w = poll_until(
      [&] {
        const int a1 = nccl_poll(c->tx), b1 = nccl_poll(c->rx);
        if (a1 == commwait::POLL_ERROR || b1 == commwait::POLL_ERROR) return (int)commwait::POLL_ERROR;
        return a1 == commwait::POLL_DONE && b1 == commwait::POLL_DONE ? (int)commwait::POLL_DONE
                                                                      : (int)commwait::POLL_PENDING;
      },
      g_timeout_s);
  if (w != commwait::WAIT_OK) return wait_failed(c.get(), w, "communicator setup (ncclCommInitRankConfig)");
  HIPCHK(hipStreamCreateWithFlags(&c->stx, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&c->srx, hipStreamNonBlocking));
  if (rank == 0) {
    const size_t nh = (size_t)RING * world;
    HIPCHK(hipHostMalloc((void**)&c->h_hdr, nh * 5 * 8, hipHostMallocDefault));
    HIPCHK(hipHostMalloc((void**)&c->h_part, nh * 9 * 8, hipHostMallocDefault));
    HIPCHK(hipMalloc((void**)&c->d_hdr, nh * 5 * 8));
    HIPCHK(hipMalloc((void**)&c->d_part, nh * 9 * 8));
    for (auto& s : c->slots) {
      HIPCHK(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    }
  } else {
    HIPCHK(hipHostMalloc((void**)&c->h_rhdr, 5 * 8, hipHostMallocDefault));
    HIPCHK(hipHostMalloc((void**)&c->h_rpart, 9 * 8, hipHostMallocDefault));
    HIPCHK(hipMalloc((void**)&c->d_rhdr, 5 * 8));
    HIPCHK(hipMalloc((void**)&c->d_rpart, 9 * 8));
  }
  g_comm = c.release();
  return H2G_OK;
}

int comm_destroy() {
  Comm* c = g_comm;
  if (!c) return H2G_OK;
  g_comm = nullptr;
  (void)hipSetDevice(c->device);
  for (hipStream_t st : {c->stx, c->srx})  // bounded: an aborted communicator's work may not drain
    if (st) (void)poll_until([&] { return hipStreamQuery(st) == hipErrorNotReady ? 0 : 1; }, 10.0);
  if (c->tx) (void)ncclCommDestroy(c->tx);
  if (c->rx) (void)ncclCommDestroy(c->rx);
  for (auto& s : c->slots) {
    if (s.stage) (void)hipFree(s.stage);
    if (s.copied) (void)hipEventDestroy(s.copied);
    if (s.done) (void)hipEventDestroy(s.done);
  }
  for (void* p : c->rstage)
    if (p) (void)hipFree(p);
  for (int64_t* p : {c->h_hdr, c->h_part, c->h_rhdr, c->h_rpart})
    if (p) (void)hipHostFree(p);
  for (int64_t* p : {c->d_hdr, c->d_part, c->d_rhdr, c->d_rpart})
    if (p) (void)hipFree(p);
  if (c->h_ag) (void)hipHostFree(c->h_ag);
  if (c->h_hg) (void)hipHostFree(c->h_hg);
  if (c->d_hg) (void)hipFree(c->d_hg);
  for (uint64_t* p : {c->d_ag_in, c->d_ag_out})
    if (p) (void)hipFree(p);
  if (c->xready) (void)hipEventDestroy(c->xready);
  if (c->stx) (void)hipStreamDestroy(c->stx);
  if (c->srx) (void)hipStreamDestroy(c->srx);
  delete c;
  return H2G_OK;
}

int comm_world() { return g_comm ? g_comm->world : 1; }
// RCCL's own view of the slab communicator: ncclCommCount / ncclCommUserRank (0 / -1 without one)
int comm_rccl_info(int* count, int* rank) {
  *count = 0;
  *rank = -1;
  if (!g_comm || g_comm->broken) return H2G_OK;
  NCCLCHK(ncclCommCount(g_comm->tx, count));
  NCCLCHK(ncclCommUserRank(g_comm->tx, rank));
  return H2G_OK;
}
int comm_rank() { return g_comm ? g_comm->rank : 0; }

void* comm_spmd_ctx() { return g_comm; }

// SPMD: every rank's partial of MSM `seq` and its consistency digest, in rank order (one
// ncclAllGather of H2G_SPMD_WORDS words per rank on the slab communicator; every rank calls
// it for the same MSMs in the same order)
int comm_allgather_partial(void* ctx, uint64_t seq, const uint64_t in[H2G_SPMD_WORDS], uint64_t* out) {
  (void)seq;
  Comm* c = usable(ctx);
  if (!c) return fail(H2G_ERR_STATE, "comm: no (live) communicator for the SPMD all-gather");
  HIPCHK(hipSetDevice(c->device));
  const size_t W = (size_t)c->world;
  constexpr size_t SW = H2G_SPMD_WORDS;
  if (!c->h_ag) {
    HIPCHK(hipHostMalloc((void**)&c->h_ag, W * SW * 8, hipHostMallocDefault));
    HIPCHK(hipMalloc((void**)&c->d_ag_in, SW * 8));
    HIPCHK(hipMalloc((void**)&c->d_ag_out, W * SW * 8));
  }
  std::memcpy(c->h_ag, in, SW * 8);
  HIPCHK(hipMemcpyAsync(c->d_ag_in, c->h_ag, SW * 8, hipMemcpyHostToDevice, c->stx));
  NCCLQ(c, c->tx, ncclAllGather(c->d_ag_in, c->d_ag_out, SW, ncclUint64, c->tx, c->stx));
  HIPCHK(hipMemcpyAsync(c->h_ag, c->d_ag_out, W * SW * 8, hipMemcpyDeviceToHost, c->stx));
  RCCHK(wait_stream(c, c->stx, "SPMD all-gather of the MSM partials", g_timeout_s));
  std::memcpy(out, c->h_ag, W * SW * 8);
  return H2G_OK;
}

// the multi-open tail's scalars (partial evaluations, kate carries): staged through
// grow-only pinned / device buffers, one ncclAllGather of bytes
int comm_allgather_host(void* ctx, const void* in, size_t bytes, void* out) {
  Comm* c = usable(ctx);
  if (!c) return fail(H2G_ERR_STATE, "comm: no (live) communicator for the SPMD host all-gather");
  if (bytes == 0) return H2G_OK;
  HIPCHK(hipSetDevice(c->device));
  const size_t W = (size_t)c->world, total = W * bytes;
  if (total > c->hg_cap) {
    if (c->h_hg) (void)hipHostFree(c->h_hg);
    if (c->d_hg) (void)hipFree(c->d_hg);
    c->h_hg = nullptr;
    c->d_hg = nullptr;
    c->hg_cap = 0;
    HIPCHK(hipHostMalloc(&c->h_hg, total + bytes, hipHostMallocDefault));
    HIPCHK(hipMalloc(&c->d_hg, total + bytes));
    c->hg_cap = total;
  }
  uint8_t* hin = static_cast<uint8_t*>(c->h_hg) + total;  // the send staging follows the receive buffer
  uint8_t* din = static_cast<uint8_t*>(c->d_hg) + total;
  std::memcpy(hin, in, bytes);
  HIPCHK(hipMemcpyAsync(din, hin, bytes, hipMemcpyHostToDevice, c->stx));
  NCCLQ(c, c->tx, ncclAllGather(din, c->d_hg, bytes, ncclUint8, c->tx, c->stx));
  HIPCHK(hipMemcpyAsync(c->h_hg, c->d_hg, total, hipMemcpyDeviceToHost, c->stx));
  RCCHK(wait_stream(c, c->stx, "SPMD host all-gather", g_timeout_s));
  std::memcpy(out, c->h_hg, total);
  return H2G_OK;
}

// one group of sends and receives on `comm` / `st`, the rank's own block a device copy
int enqueue_exchange(Comm* c, ncclComm_t comm, hipStream_t st, const void* d_send, const size_t* send_bytes,
                     void* d_recv, const size_t* recv_bytes) {
  const int W = c->world;
  if (send_bytes[c->rank] != recv_bytes[c->rank]) return fail(H2G_ERR_ARG, "comm_exchange: own block sizes differ");
  size_t so = 0, ro = 0;
  NCCLQ(c, comm, ncclGroupStart());
  for (int p = 0; p < W; p++) {
    const uint8_t* sp = static_cast<const uint8_t*>(d_send) + so;
    uint8_t* rp = static_cast<uint8_t*>(d_recv) + ro;
    if (p == c->rank) {
      if (send_bytes[p]) HIPCHK(hipMemcpyAsync(rp, sp, send_bytes[p], hipMemcpyDeviceToDevice, st));
    } else {
      if (send_bytes[p]) NCCLQ(c, comm, ncclSend(sp, send_bytes[p], ncclUint8, p, comm, st));
      if (recv_bytes[p]) NCCLQ(c, comm, ncclRecv(rp, recv_bytes[p], ncclUint8, p, comm, st));
    }
    so += send_bytes[p];
    ro += recv_bytes[p];
  }
  NCCLQ(c, comm, ncclGroupEnd());
  return H2G_OK;
}

// h(X)'s coefficient slabs from the sub-coset owners (and the exchanges the prover waits
// for at once): on the slab communicator, complete on return
int comm_exchange(void* ctx, const void* d_send, const size_t* send_bytes, void* d_recv, const size_t* recv_bytes) {
  Comm* c = usable(ctx);
  if (!c) return fail(H2G_ERR_STATE, "comm: no (live) communicator for the SPMD exchange");
  HIPCHK(hipSetDevice(c->device));
  RCCHK(enqueue_exchange(c, c->tx, c->stx, d_send, send_bytes, d_recv, recv_bytes));
  return wait_stream(c, c->stx, "SPMD exchange", g_timeout_s);
}

// the column-ownership exchanges, overlapped with the stages after them: queued on the
// second communicator behind the prover's stream, `done` recorded behind them; the host
// does not wait here (comm_exchange_wait does, against the deadline)
int comm_exchange_post(void* ctx, const void* d_send, const size_t* send_bytes, void* d_recv, const size_t* recv_bytes,
                       void* stream, void* done) {
  Comm* c = usable(ctx);
  if (!c) return fail(H2G_ERR_STATE, "comm: no (live) communicator for the SPMD exchange");
  HIPCHK(hipSetDevice(c->device));
  if (!c->xready) HIPCHK(hipEventCreateWithFlags(&c->xready, hipEventDisableTiming));
  HIPCHK(hipEventRecord(c->xready, static_cast<hipStream_t>(stream)));
  HIPCHK(hipStreamWaitEvent(c->srx, c->xready, 0));
  RCCHK(enqueue_exchange(c, c->rx, c->srx, d_send, send_bytes, d_recv, recv_bytes));
  HIPCHK(hipEventRecord(static_cast<hipEvent_t>(done), c->srx));
  return H2G_OK;
}

int comm_exchange_wait(void* ctx, void* done) {
  Comm* c = usable(ctx);
  if (!c) return fail(H2G_ERR_STATE, "comm: no (live) communicator for the SPMD exchange");
  return wait_event(c, static_cast<hipEvent_t>(done), "SPMD exchange (overlapped)");
}

int comm_bcast(void* ctx, void* d_buf, size_t bytes, int root) {
  Comm* c = usable(ctx);
  if (!c) return fail(H2G_ERR_STATE, "comm: no (live) communicator for the SPMD broadcast");
  HIPCHK(hipSetDevice(c->device));
  NCCLQ(c, c->tx, ncclBroadcast(d_buf, d_buf, bytes, ncclUint8, root, c->tx, c->stx));
  return wait_stream(c, c->stx, "SPMD broadcast", g_timeout_s);
}

void* comm_transport_ctx(uint64_t points) {
  if (!g_comm || g_comm->rank != 0) return nullptr;
  g_comm->points = points;
  return g_comm;
}

// rank 0: one MSM's slabs to the peers.  The scalars are final when this is called (the
// prover synchronises its stream first); the prover stream is made to wait for the staging
// copy, so later in-place work cannot race the sends.
int comm_launch(void* ctx, uint64_t seq, int32_t base_set, uint64_t n, const void* d_scalars) {
  Comm* c = usable(ctx);
  if (!c || c->rank != 0) return fail(H2G_ERR_STATE, "comm_launch: no (live) rank-0 communicator");
  int si = -1;
  for (int i = 0; i < RING; i++)
    if (!c->slots[(seq + i) % RING].busy) {
      si = (int)((seq + i) % RING);
      break;
    }
  if (si < 0) return fail(H2G_ERR_STATE, "comm_launch: too many outstanding sharded MSMs");
  Slot& s = c->slots[si];
  const int W = c->world;
  const uint64_t lo1 = slab_lo(c->points, n, W, 1);
  const size_t bytes = (size_t)(n - lo1) * 32;
  RCCHK(grow(&s.stage, &s.cap, bytes));
  if (bytes) HIPCHK(hipMemcpyAsync(s.stage, (const uint8_t*)d_scalars + lo1 * 32, bytes, hipMemcpyDeviceToDevice, c->stx));
  HIPCHK(hipEventRecord(s.copied, c->stx));
  Device* d = cur();
  HIPCHK(hipStreamWaitEvent(d->stream, s.copied, 0));
  int64_t* hh = c->h_hdr + (size_t)si * W * 5;
  int64_t* dh = c->d_hdr + (size_t)si * W * 5;
  for (int r = 1; r < W; r++) {
    const uint64_t lo = slab_lo(c->points, n, W, r), hi = slab_lo(c->points, n, W, r + 1);
    const int64_t h[5] = {COMM_OP_MSM, (int64_t)seq, base_set, (int64_t)lo, (int64_t)(hi - lo)};
    std::memcpy(hh + 5 * r, h, sizeof(h));
  }
  HIPCHK(hipMemcpyAsync(dh + 5, hh + 5, (size_t)(W - 1) * 5 * 8, hipMemcpyHostToDevice, c->stx));
  // headers, then slabs (a peer reads its header before it posts the slab's receive)
  NCCLQ(c, c->tx, ncclGroupStart());
  for (int r = 1; r < W; r++) NCCLQ(c, c->tx, ncclSend(dh + 5 * r, 5 * 8, ncclUint8, r, c->tx, c->stx));
  NCCLQ(c, c->tx, ncclGroupEnd());
  NCCLQ(c, c->tx, ncclGroupStart());
  for (int r = 1; r < W; r++) {
    const uint64_t lo = slab_lo(c->points, n, W, r), hi = slab_lo(c->points, n, W, r + 1);
    if (hi > lo)
      NCCLQ(c, c->tx, ncclSend((const uint8_t*)s.stage + (lo - lo1) * 32, (hi - lo) * 32, ncclUint8, r, c->tx, c->stx));
  }
  NCCLQ(c, c->tx, ncclGroupEnd());
  int64_t* dp = c->d_part + (size_t)si * W * 9;
  NCCLQ(c, c->rx, ncclGroupStart());
  for (int r = 1; r < W; r++) NCCLQ(c, c->rx, ncclRecv(dp + 9 * r, 9 * 8, ncclUint8, r, c->rx, c->srx));
  NCCLQ(c, c->rx, ncclGroupEnd());
  HIPCHK(hipMemcpyAsync(c->h_part + (size_t)si * W * 9 + 9, dp + 9, (size_t)(W - 1) * 9 * 8, hipMemcpyDeviceToHost,
                        c->srx));
  HIPCHK(hipEventRecord(s.done, c->srx));
  s.busy = true;
  s.seq = seq;
  return H2G_OK;
}

int comm_collect(void* ctx, uint64_t seq, uint64_t* partials, int32_t* is_identity) {
  Comm* c = usable(ctx);
  if (!c) return fail(H2G_ERR_STATE, "comm_collect: no (live) communicator");
  for (int i = 0; i < RING; i++) {
    Slot& s = c->slots[i];
    if (!s.busy || s.seq != seq) continue;
    RCCHK(wait_event(c, s.done, "slab partials of a sharded MSM"));
    const int64_t* hp = c->h_part + (size_t)i * c->world * 9;
    for (int r = 1; r < c->world; r++) {
      std::memcpy(partials + 8 * (r - 1), hp + 9 * r, 64);
      is_identity[r - 1] = hp[9 * r + 8] != 0;
    }
    s.busy = false;
    return H2G_OK;
  }
  return fail(H2G_ERR_STATE, "comm_collect: unknown MSM " + std::to_string(seq));
}

// rank 0: one header of `op` to every peer, outside any MSM (no launch in flight)
static int send_control(Comm* c, int64_t op, const char* what) {
  for (auto& s : c->slots)
    if (s.busy) RCCHK(wait_event(c, s.done, "slab partials before a control header"));
  const int W = c->world;
  int64_t* hh = c->h_hdr;  // slot 0's header row (no launch is in flight)
  for (int r = 1; r < W; r++) {
    const int64_t h[5] = {op, 0, 0, 0, 0};
    std::memcpy(hh + 5 * r, h, sizeof(h));
  }
  HIPCHK(hipMemcpyAsync(c->d_hdr + 5, hh + 5, (size_t)(W - 1) * 5 * 8, hipMemcpyHostToDevice, c->stx));
  NCCLQ(c, c->tx, ncclGroupStart());
  for (int r = 1; r < W; r++) NCCLQ(c, c->tx, ncclSend(c->d_hdr + 5 * r, 5 * 8, ncclUint8, r, c->tx, c->stx));
  NCCLQ(c, c->tx, ncclGroupEnd());
  RCCHK(wait_stream(c, c->stx, what, g_timeout_s));
  return H2G_OK;
}

int comm_stop() {
  Comm* c = usable(g_comm);
  if (!c || c->rank != 0) return fail(H2G_ERR_STATE, "comm_stop: no (live) rank-0 communicator");
  RCCHK(send_control(c, COMM_OP_STOP, "stop headers"));
  for (auto& s : c->slots) s.busy = false;
  return H2G_OK;
}

int comm_keepalive() {
  Comm* c = usable(g_comm);
  if (!c || c->rank != 0) return fail(H2G_ERR_STATE, "comm_keepalive: no (live) rank-0 communicator");
  return send_control(c, COMM_OP_PING, "keep-alive headers");
}

int comm_next_request(int32_t* op, int32_t* base_set, uint64_t* lo, uint64_t* count, const void** d_slab,
                      hipStream_t* ready) {
  Comm* c = usable(g_comm);
  if (!c || c->rank == 0) return fail(H2G_ERR_STATE, "comm_next_request: no (live) peer communicator");
  NCCLQ(c, c->tx, ncclRecv(c->d_rhdr, 5 * 8, ncclUint8, 0, c->tx, c->stx));
  HIPCHK(hipMemcpyAsync(c->h_rhdr, c->d_rhdr, 5 * 8, hipMemcpyDeviceToHost, c->stx));
  // the serve loop's idle deadline (rank 0 decides when the next request comes; it renews
  // the deadline with keep-alive headers while idle): past it rank 0 is taken to be gone
  RCCHK(wait_stream(c, c->stx, "next request header from rank 0", g_serve_timeout_s));
  const int64_t* h = c->h_rhdr;
  *op = (int32_t)h[0];
  *base_set = (int32_t)h[2];
  *lo = (uint64_t)h[3];
  *count = (uint64_t)h[4];
  *d_slab = nullptr;
  *ready = c->stx;
  if (*op != COMM_OP_MSM || *count == 0) return H2G_OK;
  const int b = c->rnext;
  c->rnext ^= 1;
  RCCHK(grow(&c->rstage[b], &c->rcap[b], (size_t)*count * 32));
  NCCLQ(c, c->tx, ncclRecv(c->rstage[b], (size_t)*count * 32, ncclUint8, 0, c->tx, c->stx));
  *d_slab = c->rstage[b];
  return H2G_OK;
}

int comm_send_partial(const uint64_t partial[8], int32_t is_identity) {
  Comm* c = usable(g_comm);
  if (!c || c->rank == 0) return fail(H2G_ERR_STATE, "comm_send_partial: no (live) peer communicator");
  RCCHK(wait_stream(c, c->srx, "previous partial", g_timeout_s));  // it left the pinned buffer
  std::memcpy(c->h_rpart, partial, 64);
  c->h_rpart[8] = is_identity ? 1 : 0;
  HIPCHK(hipMemcpyAsync(c->d_rpart, c->h_rpart, 9 * 8, hipMemcpyHostToDevice, c->srx));
  NCCLQ(c, c->rx, ncclSend(c->d_rpart, 9 * 8, ncclUint8, 0, c->rx, c->srx));
  return H2G_OK;
}

}  // namespace rt
}  // namespace h2g
