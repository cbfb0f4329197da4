// runtime.h -- host-side device runtime shared by the C ABI (abi.cpp) and the
// prover orchestrator (prover.cpp): per-device state (stream, MSM workspace,
// grow-only scratch buffers, NTT twiddle tables), evaluation domains, error
// reporting.  Definitions live in abi.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/h2g.h"
#include "bn254.h"
#include "msm.h"
#include "ntt.h"

namespace h2g {
namespace rt {

extern thread_local std::string g_err;
extern std::recursive_mutex g_mu;

int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define HIPCHK(expr)                                                \
  do {                                                              \
    hipError_t _e = (expr);                                         \
    if (_e != hipSuccess) return ::h2g::rt::hip_fail(_e, #expr);    \
  } while (0)

#define RCCHK(expr)         \
  do {                      \
    int _rc = (expr);       \
    if (_rc) return _rc;    \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

struct NttKey {  // omega, and the scale folded into the first pass's twiddles (ntt.h NttTables::fold)
  int L;
  uint32_t w[8];
  uint32_t f[8];
  bool operator<(const NttKey& o) const {
    if (L != o.L) return L < o.L;
    const int c = std::memcmp(w, o.w, sizeof(w));
    if (c) return c < 0;
    return std::memcmp(f, o.f, sizeof(f)) < 0;
  }
};

// EvaluationDomain constants (halo2_backend/src/poly/domain.rs:38-144)
struct Domain {
  uint32_t j = 0, k = 0, ek = 0;
  Fr omega, omega_inv, ext_omega, ext_omega_inv, g_coset, g_coset_inv, ifft_div, ext_ifft_div, bary;
  std::vector<Fr> t_evals;
  Fr* d_t = nullptr;
};

struct Descriptor {
  int device;
  void* d = nullptr;  // scalars, or bases (= window 0 of fb.table when present)
  size_t n = 0;
  bool is_base = false;
  MsmFixedBase fb;    // fixed-base windows of resident bases (owned: d aliases fb.table)
};

// Asynchronous fixed-base MSMs: whole MSMs on two streams with a workspace each, so that
// one MSM's latency-bound phases (partition tail, fixup, reduction) overlap another's
// accumulation.  (Pipelining by stage instead -- partitions, accumulations and reductions
// on three streams -- measured slower: a partition beside an accumulation gets CUs only
// as the accumulation's blocks retire; profiles/r03/s3/ab_msm_pipe.)  Results land in a
// pinned ring (one XYZZ point each).
static constexpr int MSM_STREAMS = 2;
static constexpr int MSM_RING = 64;
struct MsmTicket {
  int slot = -1;
  int ring = -1;
  int c = 0;
  hipEvent_t done = nullptr;
  int64_t shard_seq = -1;  // >= 0: the peers' slabs of this MSM are pending (h2g_shard_transport)
  bool remote = false;     // SPMD column ownership: another rank computes this MSM whole
};

struct Device {
  int id = 0;
  hipStream_t stream = nullptr;
  MsmWorkspace msm;
  DevBuf a, b, c, work, out;
  std::map<NttKey, NttTables> ntt_tables;
  void* h_windows = nullptr;  // pinned host copy of MSM window sums
  // async MSM slots
  MsmWorkspace mws[MSM_STREAMS];
  hipStream_t mstream[MSM_STREAMS] = {};
  int next_slot = 0;
  void* h_ring = nullptr;  // pinned G1xyzz[MSM_RING]
  hipEvent_t ring_ev[MSM_RING] = {};
  bool ring_busy[MSM_RING] = {};
  int next_ring = 0;
  // the prover's column-transform stream (prove_impl: xs) and its NTT work buffer -- an NTT
  // on it must not share `work` with the prover's stream
  hipStream_t xstream = nullptr;
  DevBuf xwork;
  hipEvent_t xev_in = nullptr, xev_done = nullptr;
};

extern std::vector<std::unique_ptr<Device>> g_devs;
extern bool g_profile;
extern std::vector<MsmPhaseEvents> g_msm_prof;
extern int g_cur;
extern std::map<uint64_t, Descriptor> g_desc;
extern std::map<uint64_t, std::unique_ptr<Domain>> g_dom;
extern uint64_t g_next_handle;

Device* cur();
inline hipStream_t pick_stream(Device* d, void* s) { return s ? reinterpret_cast<hipStream_t>(s) : d->stream; }

Fr fr_from_limbs(const uint64_t* v);
void fr_to_limbs(const Fr& a, uint64_t* v);
Fr root_of_unity();
Fr zeta();
Fr fr_delta();
constexpr uint32_t FR_S = 28;

int domain_init(Domain* dm, uint32_t j, uint32_t k);  // host constants + device t-evaluations
void domain_release(Domain* dm);
Domain* get_dom(uint64_t h);

int get_tables(Device* d, const Fr& omega, int L, hipStream_t st, NttTables* out, const Fr& fold = Fr::one());
int msm_dev_impl(Device* d, const void* sc, const void* bs, size_t n, int c, void* out, hipStream_t st);
int msm_host_impl(Device* d, const void* sc, const void* bs, size_t n, int c, uint64_t* out, int* is_id,
                  hipStream_t st);
int msm_fixed_host_impl(Device* d, const void* sc, const MsmFixedBase& fb, size_t off, size_t n, uint64_t* out,
                        int* is_id, hipStream_t st);
// launch sum_{i<n} sc[i] * bases[off+i] after the work already queued on `producer`
int msm_fixed_launch(Device* d, const void* sc, const MsmFixedBase& fb, size_t off, size_t n, hipStream_t producer,
                     MsmTicket* t);
// nb (<= MSM_MAX_BATCH) MSMs against the same windows as one batched pipeline; t[nb]
int msm_ring_init(Device* d);  // the asynchronous MSMs' streams, ring and events (once)
int msm_fixed_launch_batch(Device* d, const void* const* sc, int nb, const MsmFixedBase& fb, size_t off, size_t n,
                           hipStream_t producer, MsmTicket* t);
// wait for a launched MSM, affine result
int msm_collect(Device* d, MsmTicket* t, uint64_t* out_affine);
int msm_collect_xyzz(Device* d, MsmTicket* t, G1xyzz* out);
// make `consumer` wait until every launched MSM has finished reading its scalars
int msm_fence(Device* d, hipStream_t consumer);
int msm_desc_impl(Device* d, const void* sc, const Descriptor& ds, size_t off, size_t n, uint64_t* out, int* is_id,
                  hipStream_t st);
int ntt_dev_impl_batch(Device* d, const Fr* const* src, uint64_t n_in, Fr* const* dst, int count, uint64_t out_len,
                       int L, const Fr& omega, int in_dist, const Fr& iz1, const Fr& iz2, int has_scale,
                       const Fr& scale, int out_dist, const Fr& oz1, const Fr& oz2, hipStream_t st);
int ntt_dev_impl(Device* d, const Fr* src, uint64_t n_in, Fr* dst, uint64_t out_len, int L, const Fr& omega,
                 int in_dist, const Fr& iz1, const Fr& iz2, int has_scale, const Fr& scale, int out_dist,
                 const Fr& oz1, const Fr& oz2, hipStream_t st);

// EvaluationDomain maps on device pointers (domain.rs:216-316)
int lagrange_to_coeff(Device* d, const Domain& dm, const Fr* src, Fr* dst, hipStream_t st);
int coeff_to_extended(Device* d, const Domain& dm, const Fr* src, Fr* dst, hipStream_t st);
// `count` independent transforms, NTT_MAX_BATCH per launch (work buffer grows to match)
int lagrange_to_coeff_batch(Device* d, const Domain& dm, const Fr* const* src, Fr* const* dst, int count,
                            hipStream_t st);
int coeff_to_extended_batch(Device* d, const Domain& dm, const Fr* const* src, Fr* const* dst, int count,
                            hipStream_t st);
int extended_to_coeff(Device* d, const Domain& dm, const Fr* src, Fr* dst, hipStream_t st);

}  // namespace rt
}  // namespace h2g
