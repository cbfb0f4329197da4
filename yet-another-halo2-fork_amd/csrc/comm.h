// comm.h -- native multi-GPU exchange over RCCL (xGMI) for one create_proof across several
// GPUs, one process per GPU.  Rank 0 (the prover) splits every commitment MSM
// into point slabs [P r / world, P (r + 1) / world) of the params' P points; the scalars of
// slab r go to rank r, which answers with the 64-B affine partial sum of its slab.  Two
// communicators keep the directions independent, so the slabs of later MSMs stream while
// the peers compute earlier ones:
//   tx (rank 0 -> r): header int64[5] = (op, seq, base_set, lo, count), then the slab
//                     (count x 32 B, from a device staging copy of the prover's scalars)
//   rx (r -> rank 0): int64[9] = affine partial (8 limbs) + identity flag
// SPMD mode all-gathers H2G_SPMD_WORDS words per rank instead (partial, flag, digest).
// Definitions in comm.cpp; the peers' serve loop (h2g_comm_serve) lives in prover.cpp next
// to the params it computes against.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "h2g.h"

namespace h2g {
namespace rt {

enum { COMM_OP_STOP = 0, COMM_OP_MSM = 1, COMM_OP_PING = 2 };
static constexpr int COMM_ID_BYTES = 256;  // two ncclUniqueIds (tx, rx)

int comm_unique_id(uint8_t id[COMM_ID_BYTES]);
int comm_init(const uint8_t id[COMM_ID_BYTES], int world, int rank);
int comm_set_timeout(double seconds);  // deadline of every RCCL wait (<= 0: none)
// a peer's longest wait for rank 0's next request in the serve loop (<= 0: none); rank 0
// renews it with comm_keepalive while it idles between proofs
int comm_set_serve_timeout(double seconds);
int comm_keepalive();  // rank 0: a PING header to every peer
int comm_destroy();
int comm_world();
int comm_rccl_info(int* count, int* rank);
int comm_rank();

// rank 0 (the h2g_shard_transport callbacks of a native transport; ctx = Comm state)
int comm_launch(void* ctx, uint64_t seq, int32_t base_set, uint64_t n, const void* d_scalars);
int comm_collect(void* ctx, uint64_t seq, uint64_t* partials, int32_t* is_identity);
void* comm_transport_ctx(uint64_t points);  // the params' P of the slab partition
int comm_stop();  // ends the peers' serve loops

// ranks 1..: next request from rank 0.  op COMM_OP_MSM: *d_slab (device, count Fr) is
// complete after the work queued on the stream *ready (the receive), until the next call.
int comm_next_request(int32_t* op, int32_t* base_set, uint64_t* lo, uint64_t* count, const void** d_slab,
                      hipStream_t* ready);
int comm_send_partial(const uint64_t partial[8], int32_t is_identity);

// SPMD (every rank proves): all-gather of the ranks' 9-word partials in rank order
// (h2g_spmd_transport.allgather; ctx = Comm state from comm_spmd_ctx)
void* comm_spmd_ctx();
int comm_allgather_partial(void* ctx, uint64_t seq, const uint64_t in[H2G_SPMD_WORDS], uint64_t* out);
// SPMD: `bytes` host bytes from every rank, out = world x bytes in rank order
int comm_allgather_host(void* ctx, const void* in, size_t bytes, void* out);
// SPMD: all-to-all of device bytes with per-peer counts (grouped send / receive)
int comm_exchange(void* ctx, const void* d_send, const size_t* send_bytes, void* d_recv, const size_t* recv_bytes);
int comm_exchange_post(void* ctx, const void* d_send, const size_t* send_bytes, void* d_recv, const size_t* recv_bytes,
                       void* stream, void* done);
int comm_exchange_wait(void* ctx, void* done);
// in-place broadcast of device memory from `root` (the sub-coset h evaluations)
int comm_bcast(void* ctx, void* d_buf, size_t bytes, int root);

}  // namespace rt
}  // namespace h2g
