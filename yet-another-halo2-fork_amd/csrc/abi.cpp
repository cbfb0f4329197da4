// abi.cpp -- implementation of include/h2g.h (the FFI boundary).
//
// Host-side plumbing only: device selection, descriptor/domain handle tables,
// grow-only device buffers for the host-pointer entry points, and argument
// validation mirroring the reference's assertions (best_multiexp's equal
// lengths, commit's `bases.len() >= size`, EvaluationDomain's length asserts).
// All arithmetic runs in the HIP kernels (msm.hip, ntt.hip, poly.hip, srs.hip);
// there is no CPU fallback: without a usable device every call fails loudly.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/h2g.h"
#include "radix.h"
#include "runtime.h"
#include "bn254.h"
#include "msm.h"
#include "ntt.h"
#include "poly.h"
#include "srs.h"

using namespace h2g;
using namespace h2g::rt;

namespace h2g {
namespace rt {

thread_local std::string g_err;
std::recursive_mutex g_mu;
std::vector<std::unique_ptr<Device>> g_devs;
bool g_profile = false;
std::vector<MsmPhaseEvents> g_msm_prof;
// pinned words receiving each profiled MSM's sorted-entry count (nonzero digits); beyond
// the capacity an MSM goes uncounted and h2g_profile_msm_entries reports it
static constexpr size_t PROF_ENTRY_CAP = 1 << 16;
uint32_t* g_prof_entries = nullptr;
int prof_entries_slot(MsmPhaseEvents* ev) {
  if (!g_prof_entries) HIPCHK(hipHostMalloc((void**)&g_prof_entries, PROF_ENTRY_CAP * 4, hipHostMallocDefault));
  ev->entries = g_msm_prof.size() < PROF_ENTRY_CAP ? g_prof_entries + g_msm_prof.size() : nullptr;
  if (ev->entries) *ev->entries = 0;
  return H2G_OK;
}
int g_cur = 0;
std::map<uint64_t, Descriptor> g_desc;
std::map<uint64_t, std::unique_ptr<Domain>> g_dom;
uint64_t g_next_handle = 1;




int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int hip_fail(hipError_t e, const char* what) {
  return fail(H2G_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}















Device* cur() {
  if (g_devs.empty()) return nullptr;
  return g_devs[g_cur].get();
}



Fr fr_from_limbs(const uint64_t* v) {
  Fr r;
  for (int i = 0; i < 4; i++) {
    r.l[2 * i] = (uint32_t)v[i];
    r.l[2 * i + 1] = (uint32_t)(v[i] >> 32);
  }
  return r;
}
void fr_to_limbs(const Fr& a, uint64_t* v) {
  for (int i = 0; i < 4; i++) v[i] = (uint64_t)a.l[2 * i] | ((uint64_t)a.l[2 * i + 1] << 32);
}

// halo2curves bn256::Fr constants (Montgomery form, 32-bit limbs) -- SURVEY A.1
Fr root_of_unity() {
  const uint64_t v[4] = {0x9632c7c5b639feb8ULL, 0x985ce3400d0ff299ULL, 0xb2dd880001b0ecd8ULL, 0x1d69070d6d98ce29ULL};
  return fr_from_limbs(v);
}
Fr zeta() {
  const uint64_t v[4] = {0x93e7cede4a0329b3ULL, 0x7d4fdca77a96c167ULL, 0x8be4ba08b19a750aULL, 0x1cbd5653a5661c25ULL};
  return fr_from_limbs(v);
}


int get_tables(Device* d, const Fr& omega, int L, hipStream_t st, NttTables* out, const Fr& fold) {
  NttKey key{L, {}, {}};
  std::memcpy(key.w, omega.l, sizeof(key.w));
  std::memcpy(key.f, fold.l, sizeof(key.f));
  auto it = d->ntt_tables.find(key);
  if (it != d->ntt_tables.end()) {
    *out = it->second;
    return H2G_OK;
  }
  NttTables t;
  hipError_t e = ntt_build_tables(&t, omega, L, st, fold);
  // built once per key; finished before any stream may use it (the prover's transform
  // stream and its own stream share the tables)
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "ntt_build_tables");
  d->ntt_tables[key] = t;
  *out = t;
  return H2G_OK;
}

int msm_dev_impl(Device* d, const void* sc, const void* bs, size_t n, int c, void* out, hipStream_t st) {
  if (n == 0) {
    if (out) HIPCHK(hipMemsetAsync(out, 0, 64, st));
    return H2G_OK;
  }
  if (n > 0x7fffffffULL) return fail(H2G_ERR_ARG, "msm: n too large");
  MsmConfig cfg;
  cfg.c = c;
  MsmPhaseEvents* pe = nullptr;
  if (g_profile) {
    MsmPhaseEvents ev;
    for (auto& e : ev.ev) HIPCHK(hipEventCreate(&e));
    RCCHK(prof_entries_slot(&ev));
    g_msm_prof.push_back(ev);
    pe = &g_msm_prof.back();
  }
  HIPCHK(msm_run(reinterpret_cast<const Fr*>(sc), reinterpret_cast<const G1Affine*>(bs), n, &d->msm, cfg,
                 reinterpret_cast<G1Affine*>(out), st, pe));
  return H2G_OK;
}

// Host-returning MSM: device phases, then the W window sums (W x 128 B) come back
// to the host and are combined there (msm_windows_host_finish); synchronous.
int msm_host_impl(Device* d, const void* sc, const void* bs, size_t n, int c, uint64_t* out, int* is_id,
                  hipStream_t st) {
  if (n == 0) {
    std::memset(out, 0, 64);
    if (is_id) *is_id = 1;
    return H2G_OK;
  }
  int rc = msm_dev_impl(d, sc, bs, n, c, nullptr, st);
  if (rc) return rc;
  const int W = d->msm.last_W;
  if (!d->h_windows) HIPCHK(hipHostMalloc(&d->h_windows, 256 * sizeof(G1xyzz), hipHostMallocDefault));
  HIPCHK(hipMemcpyAsync(d->h_windows, d->msm.windows, (size_t)W * sizeof(G1xyzz), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const G1Affine r = msm_windows_host_finish(reinterpret_cast<const G1xyzz*>(d->h_windows), W, d->msm.last_c);
  std::memcpy(out, &r, 64);
  if (is_id) {
    uint64_t x = 0;
    for (int i = 0; i < 8; i++) x |= out[i];
    *is_id = x == 0;
  }
  return H2G_OK;
}

int msm_fixed_host_impl(Device* d, const void* sc, const MsmFixedBase& fb, size_t off, size_t n, uint64_t* out,
                        int* is_id, hipStream_t st) {
  if (n == 0) {
    std::memset(out, 0, 64);
    if (is_id) *is_id = 1;
    return H2G_OK;
  }
  MsmPhaseEvents* pe = nullptr;
  if (g_profile) {
    MsmPhaseEvents ev;
    for (auto& e : ev.ev) HIPCHK(hipEventCreate(&e));
    RCCHK(prof_entries_slot(&ev));
    g_msm_prof.push_back(ev);
    pe = &g_msm_prof.back();
  }
  HIPCHK(msm_run_fixed(reinterpret_cast<const Fr*>(sc), fb, off, n, &d->msm, nullptr, st, pe));
  if (!d->h_windows) HIPCHK(hipHostMalloc(&d->h_windows, 256 * sizeof(G1xyzz), hipHostMallocDefault));
  HIPCHK(hipMemcpyAsync(d->h_windows, d->msm.windows, sizeof(G1xyzz), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const G1Affine r = msm_windows_host_finish(reinterpret_cast<const G1xyzz*>(d->h_windows), 1, d->msm.last_c);
  std::memcpy(out, &r, 64);
  if (is_id) {
    uint64_t x = 0;
    for (int i = 0; i < 8; i++) x |= out[i];
    *is_id = x == 0;
  }
  return H2G_OK;
}

#ifndef H2G_MSM_HIPRIO
#define H2G_MSM_HIPRIO 0
#endif
// the asynchronous MSMs' streams, result ring and events (h2g_init creates them, right
// after the device stream: see there)
int msm_ring_init(Device* d) {
  if (d->h_ring) return H2G_OK;
  HIPCHK(hipHostMalloc(&d->h_ring, MSM_RING * sizeof(G1xyzz), hipHostMallocDefault));
  if (H2G_MSM_HIPRIO) {  // A/B: the MSM streams at the device's greatest stream priority
    int least = 0, greatest = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    for (int i = 0; i < MSM_STREAMS; i++)
      HIPCHK(hipStreamCreateWithPriority(&d->mstream[i], hipStreamNonBlocking, greatest));
  } else {
    for (int i = 0; i < MSM_STREAMS; i++) HIPCHK(hipStreamCreateWithFlags(&d->mstream[i], hipStreamNonBlocking));
  }
  for (int i = 0; i < MSM_RING; i++) HIPCHK(hipEventCreateWithFlags(&d->ring_ev[i], hipEventDisableTiming));
  return H2G_OK;
}

// nb MSMs of n scalars each against the same fixed-base windows, launched as one batched
// pipeline (msm_run_fixed_batch) on the next MSM stream; ticket b collects MSM b.
int msm_fixed_launch_batch(Device* d, const void* const* sc, int nb, const MsmFixedBase& fb, size_t off, size_t n,
                           hipStream_t producer, MsmTicket* t) {
  if (nb < 1 || nb > MSM_MAX_BATCH) return fail(H2G_ERR_ARG, "msm: bad batch size");
  RCCHK(msm_ring_init(d));
  int rings[MSM_MAX_BATCH];
  int got = 0;
  for (int k = 0; k < MSM_RING && got < nb; k++) {
    const int r = (d->next_ring + k) % MSM_RING;
    if (!d->ring_busy[r]) rings[got++] = r;
  }
  if (got < nb) return fail(H2G_ERR_STATE, "msm: too many outstanding asynchronous MSMs");
  d->next_ring = (rings[nb - 1] + 1) % MSM_RING;
  const int slot = d->next_slot;
  d->next_slot = (slot + 1) % MSM_STREAMS;
  hipStream_t ms = d->mstream[slot];
  // order after the producer's work (the scalars)
  HIPCHK(hipEventRecord(d->ring_ev[rings[0]], producer));
  HIPCHK(hipStreamWaitEvent(ms, d->ring_ev[rings[0]], 0));
  MsmPhaseEvents* pe = nullptr;
  if (g_profile && n > 0) {
    MsmPhaseEvents ev;
    for (auto& e : ev.ev) HIPCHK(hipEventCreate(&e));
    RCCHK(prof_entries_slot(&ev));
    ev.msms = nb;
    g_msm_prof.push_back(ev);
    pe = &g_msm_prof.back();
  }
  G1xyzz* host = reinterpret_cast<G1xyzz*>(d->h_ring);
  if (n == 0) {
    for (int b = 0; b < nb; b++) std::memset(host + rings[b], 0, sizeof(G1xyzz));  // identity (ZZ = 0)
  } else {
    MsmScalarList list;
    for (int b = 0; b < nb; b++) list.p[b] = reinterpret_cast<const Fr*>(sc[b]);
    if (nb == 1) HIPCHK(msm_run_fixed(list.p[0], fb, off, n, &d->mws[slot], nullptr, ms, pe));
    else HIPCHK(msm_run_fixed_batch(list, nb, fb, off, n, &d->mws[slot], ms, pe));
    const G1xyzz* win = reinterpret_cast<const G1xyzz*>(d->mws[slot].windows);
    for (int b = 0; b < nb; b++)
      HIPCHK(hipMemcpyAsync(host + rings[b], win + b, sizeof(G1xyzz), hipMemcpyDeviceToHost, ms));
  }
  for (int b = 0; b < nb; b++) {
    HIPCHK(hipEventRecord(d->ring_ev[rings[b]], ms));
    d->ring_busy[rings[b]] = true;
    t[b].slot = slot;
    t[b].ring = rings[b];
    t[b].c = fb.c;
    t[b].done = d->ring_ev[rings[b]];
  }
  return H2G_OK;
}

int msm_fixed_launch(Device* d, const void* sc, const MsmFixedBase& fb, size_t off, size_t n, hipStream_t producer,
                     MsmTicket* t) {
  return msm_fixed_launch_batch(d, &sc, 1, fb, off, n, producer, t);
}

int msm_collect(Device* d, MsmTicket* t, uint64_t* out) {
  if (t->ring < 0) return fail(H2G_ERR_STATE, "msm: collect without launch");
  HIPCHK(hipEventSynchronize(t->done));
  const G1xyzz* host = reinterpret_cast<const G1xyzz*>(d->h_ring) + t->ring;
  const G1Affine r = msm_windows_host_finish(host, 1, t->c);
  std::memcpy(out, &r, 64);
  d->ring_busy[t->ring] = false;
  t->ring = -1;
  return H2G_OK;
}

// the same, left in XYZZ form (the caller converts a batch with one inversion)
int msm_collect_xyzz(Device* d, MsmTicket* t, G1xyzz* out) {
  if (t->ring < 0) return fail(H2G_ERR_STATE, "msm: collect without launch");
  HIPCHK(hipEventSynchronize(t->done));
  *out = reinterpret_cast<const G1xyzz*>(d->h_ring)[t->ring];  // one window (fixed-base tickets)
  d->ring_busy[t->ring] = false;
  t->ring = -1;
  return H2G_OK;
}

int msm_fence(Device* d, hipStream_t consumer) {
  if (!d->h_ring) return H2G_OK;
  for (int i = 0; i < MSM_STREAMS; i++) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventRecord(e, d->mstream[i]));
    HIPCHK(hipStreamWaitEvent(consumer, e, 0));
    HIPCHK(hipEventDestroy(e));
  }
  return H2G_OK;
}

// MSM against a descriptor's bases [off, off + n): fixed-base tables when present
int msm_desc_impl(Device* d, const void* sc, const Descriptor& ds, size_t off, size_t n, uint64_t* out, int* is_id,
                  hipStream_t st) {
  if (ds.fb.table) return msm_fixed_host_impl(d, sc, ds.fb, off, n, out, is_id, st);
  return msm_host_impl(d, sc, (const char*)ds.d + off * 64, n, 0, out, is_id, st);
}

int ntt_dev_impl_batch(Device* d, const Fr* const* src, uint64_t n_in, Fr* const* dst, int count, uint64_t out_len,
                       int L, const Fr& omega, int in_dist, const Fr& iz1, const Fr& iz2, int has_scale,
                       const Fr& scale, int out_dist, const Fr& oz1, const Fr& oz2, hipStream_t st) {
  if (count < 1 || count > NTT_MAX_BATCH) return fail(H2G_ERR_ARG, "ntt: batch size");
  NttArgs a;
  // a scale goes into the first pass's twiddle table (tables per omega and scale): the
  // last pass then multiplies only for an output coset distribution
  int rc = get_tables(d, omega, L, st, &a.tab, has_scale && L > NTT_SMALL_MAX_LOG ? scale : Fr::one());
  if (rc) return rc;
  const size_t N = (size_t)1 << L;
  // the transform stream's NTTs run beside the prover stream's: each has its own work buffer
  DevBuf& wb = d->xstream != nullptr && st == d->xstream ? d->xwork : d->work;
  if (L > NTT_SMALL_MAX_LOG) {
    hipError_t e = wb.ensure((size_t)count * N * sizeof(Fr));
    if (e != hipSuccess) return hip_fail(e, "ntt work buffer");
  }
  a.src = src[0];
  a.n_in = n_in;
  a.work = reinterpret_cast<Fr*>(wb.p);
  a.dst = dst[0];
  a.count = count;
  for (int b = 0; b < count; b++) {
    a.srcs[b] = src[b];
    a.dsts[b] = dst[b];
  }
  a.out_len = out_len;
  a.in_distribute = in_dist;
  a.in_z1 = iz1;
  a.in_z2 = iz2;
  a.has_scale = has_scale;
  a.scale = scale;
  a.out_distribute = out_dist;
  a.out_z1 = oz1;
  a.out_z2 = oz2;
  HIPCHK(ntt_run(a, st));
  return H2G_OK;
}

int ntt_dev_impl(Device* d, const Fr* src, uint64_t n_in, Fr* dst, uint64_t out_len, int L, const Fr& omega,
                 int in_dist, const Fr& iz1, const Fr& iz2, int has_scale, const Fr& scale, int out_dist,
                 const Fr& oz1, const Fr& oz2, hipStream_t st) {
  return ntt_dev_impl_batch(d, &src, n_in, &dst, 1, out_len, L, omega, in_dist, iz1, iz2, has_scale, scale, out_dist,
                            oz1, oz2, st);
}

Domain* get_dom(uint64_t h) {
  auto it = g_dom.find(h);
  return it == g_dom.end() ? nullptr : it->second.get();
}


int domain_init(Domain* dm, uint32_t j, uint32_t k) {   // EvaluationDomain::new (domain.rs:38-144)
  if (j < 2 || k > FR_S) return fail(H2G_ERR_ARG, "domain: bad j/k");
  dm->j = j;
  dm->k = k;
  const uint64_t n = 1ull << k;
  const uint64_t qdeg = j - 1;
  uint32_t ek = k;
  while ((1ull << ek) < n * qdeg) ek++;
  if (ek > FR_S) return fail(H2G_ERR_ARG, "domain: extended_k > S");
  dm->ek = ek;
  Fr eo = root_of_unity();
  for (uint32_t i = ek; i < FR_S; i++) eo = sqr(eo);
  Fr o = eo;
  for (uint32_t i = k; i < ek; i++) o = sqr(o);
  dm->ext_omega = eo;
  dm->omega = o;
  dm->g_coset = zeta();
  dm->g_coset_inv = sqr(dm->g_coset);
  const uint64_t tlen = 1ull << (ek - k);
  const Fr orig = pow_u64(dm->g_coset, n), step = pow_u64(eo, n);
  Fr c = orig;
  dm->t_evals.resize(tlen);
  for (uint64_t i = 0; i < tlen; i++) {
    dm->t_evals[i] = inv(c - Fr::one());
    c = c * step;
  }
  dm->ifft_div = inv(from_u64<FrParams>(n));
  dm->ext_ifft_div = inv(from_u64<FrParams>(1ull << ek));
  dm->bary = inv(from_u64<FrParams>(n));
  dm->ext_omega_inv = inv(eo);
  dm->omega_inv = inv(o);
  HIPCHK(hipMalloc(&dm->d_t, tlen * sizeof(Fr)));
  HIPCHK(hipMemcpy(dm->d_t, dm->t_evals.data(), tlen * sizeof(Fr), hipMemcpyHostToDevice));
  return H2G_OK;
}

void domain_release(Domain* dm) {
  if (dm->d_t) (void)hipFree(dm->d_t);
  dm->d_t = nullptr;
}

// lagrange_to_coeff (domain.rs:216-226): iFFT, * 1/n
int lagrange_to_coeff(Device* d, const Domain& dm, const Fr* src, Fr* dst, hipStream_t st) {
  return lagrange_to_coeff_batch(d, dm, &src, &dst, 1, st);
}
int lagrange_to_coeff_batch(Device* d, const Domain& dm, const Fr* const* src, Fr* const* dst, int count,
                            hipStream_t st) {
  const Fr one = Fr::one();
  const uint64_t n = 1ull << dm.k;
  for (int b0 = 0; b0 < count; b0 += NTT_MAX_BATCH)
    RCCHK(ntt_dev_impl_batch(d, src + b0, n, dst + b0, std::min(NTT_MAX_BATCH, count - b0), n, (int)dm.k,
                             dm.omega_inv, 0, one, one, 1, dm.ifft_div, 0, one, one, st));
  return H2G_OK;
}

// coeff_to_extended (domain.rs:230-244): distribute zeta powers, zero-pad, FFT over the extended domain
int coeff_to_extended(Device* d, const Domain& dm, const Fr* src, Fr* dst, hipStream_t st) {
  return coeff_to_extended_batch(d, dm, &src, &dst, 1, st);
}
int coeff_to_extended_batch(Device* d, const Domain& dm, const Fr* const* src, Fr* const* dst, int count,
                            hipStream_t st) {
  const Fr one = Fr::one();
  const uint64_t n = 1ull << dm.k, ext = 1ull << dm.ek;
  for (int b0 = 0; b0 < count; b0 += NTT_MAX_BATCH)
    RCCHK(ntt_dev_impl_batch(d, src + b0, n, dst + b0, std::min(NTT_MAX_BATCH, count - b0), ext, (int)dm.ek,
                             dm.ext_omega, 1, dm.g_coset, dm.g_coset_inv, 0, one, 0, one, one, st));
  return H2G_OK;
}

// extended_to_coeff (domain.rs:271-293): inverse FFT, * 1/2^ek, undistribute, truncate to n (j - 1)
int extended_to_coeff(Device* d, const Domain& dm, const Fr* src, Fr* dst, hipStream_t st) {
  const Fr one = Fr::one();
  const uint64_t ext = 1ull << dm.ek;
  const uint64_t out_len = (1ull << dm.k) * (dm.j - 1);
  return ntt_dev_impl(d, src, ext, dst, out_len, (int)dm.ek, dm.ext_omega_inv, 0, one, one, 1, dm.ext_ifft_div, 1,
                      dm.g_coset_inv, dm.g_coset, st);
}

Fr fr_delta() {
  const uint64_t v[4] = {0x9a0c322befd78855ULL, 0x46e82d14249b563cULL, 0x5983a663e0b0b7a7ULL, 0x22ab452baaa111adULL};
  return fr_from_limbs(v);
}

}  // namespace rt
}  // namespace h2g

#define NEED_DEV()                                                            \
  std::lock_guard<std::recursive_mutex> _lk(g_mu);                            \
  Device* d = cur();                                                          \
  if (!d) return fail(H2G_ERR_STATE, "h2g_init has not been called");         \
  HIPCHK(hipSetDevice(d->id));

extern "C" {

int h2g_abi_version(void) { return 1; }
const char* h2g_last_error(void) { return g_err.c_str(); }

// A/B: k idle streams created ahead of the device stream shift every stream's hardware
// queue by k.  C3 k = 22: 72.5-73.1 ms at 0, 72.8-73.7 at 1, 75.4-76.9 at 2, 76.2-77.1 at 3
// (keccak-style within 0.5 ms; profiles/r06/xs/ab_queue_shift.log)
#ifndef H2G_QUEUE_SHIFT
#define H2G_QUEUE_SHIFT 0
#endif
#ifndef H2G_EAGER_STREAMS  // A/B builds: 0 = the MSM streams created by the first asynchronous MSM
#define H2G_EAGER_STREAMS 1
#endif
int h2g_init(const int* devices, int ndev) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!g_devs.empty()) return H2G_OK;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) return fail(H2G_ERR_DEVICE, "no HIP device available");
  std::vector<int> ids;
  if (!devices || ndev <= 0) ids.push_back(0);
  else ids.assign(devices, devices + ndev);
  for (int id : ids) {
    if (id < 0 || id >= count) return fail(H2G_ERR_ARG, "device index out of range");
    auto dev = std::make_unique<Device>();
    dev->id = id;
    HIPCHK(hipSetDevice(id));
    // Streams in a fixed order: the device stream, then the two MSM streams.  With
    // GPU_MAX_HW_QUEUES = 4 each takes the next hardware queue, and the order matters: C3
    // k = 22 ran 73.8 ms with the MSM streams on the second and third queue, 77.1 ms when an
    // (idle) stream created before them pushed them to the third and fourth
    // (profiles/r06/xs/ab_eager.log).  The prover's transform stream comes later, from the
    // first single-GPU proof with lookups (prove_impl), so that multi-GPU runs leave the
    // fourth queue to the communicators' streams (an emulated C3 N = 8 replay lost 1 ms
    // with it taken: profiles/r06/emulation_final/).
    for (int q = 0; q < H2G_QUEUE_SHIFT; q++) {  // A/B: idle streams ahead of the device stream
      hipStream_t idle = nullptr;
      HIPCHK(hipStreamCreateWithFlags(&idle, hipStreamNonBlocking));
    }
    HIPCHK(hipStreamCreateWithFlags(&dev->stream, hipStreamNonBlocking));
    if (H2G_EAGER_STREAMS) RCCHK(msm_ring_init(dev.get()));
    HIPCHK(ntt_init_attributes());
    g_devs.push_back(std::move(dev));
  }
  g_cur = 0;
  return H2G_OK;
}

int h2g_shutdown(void) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  for (auto& kv : g_desc) {
    if (kv.second.d) (void)hipFree(kv.second.d);
  }
  g_desc.clear();
  for (auto& kv : g_dom) {
    if (kv.second->d_t) (void)hipFree(kv.second->d_t);
  }
  g_dom.clear();
  for (auto& dev : g_devs) {
    (void)hipSetDevice(dev->id);
    (void)hipStreamSynchronize(dev->stream);
    if (dev->xstream) (void)hipStreamSynchronize(dev->xstream);
    msm_free(&dev->msm);
    for (int i = 0; i < MSM_STREAMS; i++)
      if (dev->mstream[i]) {
        (void)hipStreamSynchronize(dev->mstream[i]);
        (void)hipStreamDestroy(dev->mstream[i]);
      }
    for (int i = 0; i < MSM_STREAMS; i++) msm_free(&dev->mws[i]);
    for (int i = 0; i < MSM_RING; i++)
      if (dev->ring_ev[i]) (void)hipEventDestroy(dev->ring_ev[i]);
    if (dev->h_ring) (void)hipHostFree(dev->h_ring);
    dev->a.release();
    dev->b.release();
    dev->c.release();
    dev->work.release();
    dev->out.release();
    for (auto& kv : dev->ntt_tables) ntt_free_tables(&kv.second);
    if (dev->xstream) (void)hipStreamDestroy(dev->xstream);
    if (dev->xev_in) (void)hipEventDestroy(dev->xev_in);
    if (dev->xev_done) (void)hipEventDestroy(dev->xev_done);
    dev->xwork.release();
    if (dev->h_windows) (void)hipHostFree(dev->h_windows);
    (void)hipStreamDestroy(dev->stream);
  }
  g_devs.clear();
  return H2G_OK;
}

int h2g_device_count(int* out) {
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
  *out = c;
  return H2G_OK;
}

int h2g_device_mem_info(uint64_t* free_bytes, uint64_t* total_bytes) {
  NEED_DEV();
  if (!free_bytes || !total_bytes) return fail(H2G_ERR_ARG, "device_mem_info: null output");
  size_t f = 0, t = 0;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemGetInfo(&f, &t));
  *free_bytes = f;
  *total_bytes = t;
  return H2G_OK;
}

int h2g_set_device(int index) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (index < 0 || index >= (int)g_devs.size()) return fail(H2G_ERR_ARG, "device index");
  g_cur = index;
  return H2G_OK;
}

// ---------------------------------------------------------------- MSM
int h2g_msm(const uint64_t* coeffs, const uint64_t* bases, size_t n, uint64_t out[8], int* is_id) {
  NEED_DEV();
  if (n && (!coeffs || !bases)) return fail(H2G_ERR_ARG, "msm: null input");
  HIPCHK(d->a.ensure(n * 32 + 32));
  HIPCHK(d->b.ensure(n * 64 + 64));
  HIPCHK(d->out.ensure(64));
  HIPCHK(hipMemcpyAsync(d->a.p, coeffs, n * 32, hipMemcpyHostToDevice, d->stream));
  HIPCHK(hipMemcpyAsync(d->b.p, bases, n * 64, hipMemcpyHostToDevice, d->stream));
  return msm_host_impl(d, d->a.p, d->b.p, n, 0, out, is_id, d->stream);
}

static int make_desc(const uint64_t* data, size_t n, size_t elem_bytes, bool is_base, uint64_t* handle) {
  NEED_DEV();
  if (!handle || (n && !data)) return fail(H2G_ERR_ARG, "descriptor: null argument");
  Descriptor ds;
  ds.device = g_cur;
  ds.n = n;
  ds.is_base = is_base;
  HIPCHK(hipMalloc(&ds.d, n * elem_bytes + 64));
  HIPCHK(hipMemcpyAsync(ds.d, data, n * elem_bytes, hipMemcpyHostToDevice, d->stream));
  if (is_base && n >= 2) {
    // resident bases: precompute the fixed-base windows; the table's window 0 is the bases
    HIPCHK(msm_fixed_base_build((const G1Affine*)ds.d, n, 0, &ds.fb, d->stream));
    HIPCHK(hipStreamSynchronize(d->stream));
    (void)hipFree(ds.d);
    ds.d = ds.fb.table;
  }
  HIPCHK(hipStreamSynchronize(d->stream));
  *handle = g_next_handle++;
  g_desc[*handle] = ds;
  return H2G_OK;
}

int h2g_msm_coeffs_descriptor(const uint64_t* coeffs, size_t n, uint64_t* handle) {
  return make_desc(coeffs, n, 32, false, handle);
}
int h2g_msm_base_descriptor(const uint64_t* bases, size_t n, uint64_t* handle) {
  return make_desc(bases, n, 64, true, handle);
}
int h2g_msm_base_descriptor_dev(const void* d_bases, size_t n, int window_bits, uint64_t* handle) {
  NEED_DEV();
  if (!handle || !d_bases || n < 2) return fail(H2G_ERR_ARG, "descriptor: bad argument");
  Descriptor ds;
  ds.device = g_cur;
  ds.n = n;
  ds.is_base = true;
  HIPCHK(msm_fixed_base_build((const G1Affine*)d_bases, n, window_bits, &ds.fb, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  ds.d = ds.fb.table;
  *handle = g_next_handle++;
  g_desc[*handle] = ds;
  return H2G_OK;
}

int h2g_msm_with_cached_base_dev(const void* d_scalars, size_t n, uint64_t base, size_t off, uint64_t out[8],
                                 int* is_id, void* stream) {
  NEED_DEV();
  auto it = g_desc.find(base);
  if (it == g_desc.end() || !it->second.is_base) return fail(H2G_ERR_HANDLE, "unknown base descriptor");
  if (off + n > it->second.n) return fail(H2G_ERR_ARG, "msm: bases.len() < size");
  if (n && !d_scalars) return fail(H2G_ERR_ARG, "msm: null scalars");
  return msm_desc_impl(d, d_scalars, it->second, off, n, out, is_id, pick_stream(d, stream));
}

int h2g_msm_descriptor_free(uint64_t handle) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  auto it = g_desc.find(handle);
  if (it == g_desc.end()) return fail(H2G_ERR_HANDLE, "unknown descriptor");
  if (it->second.d) (void)hipFree(it->second.d);
  g_desc.erase(it);
  return H2G_OK;
}
int h2g_descriptor_device_ptr(uint64_t handle, void** d_ptr, size_t* n) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  auto it = g_desc.find(handle);
  if (it == g_desc.end()) return fail(H2G_ERR_HANDLE, "unknown descriptor");
  if (d_ptr) *d_ptr = it->second.d;
  if (n) *n = it->second.n;
  return H2G_OK;
}

int h2g_msm_with_cached_scalars(uint64_t coeffs, const uint64_t* bases, size_t n, uint64_t out[8], int* is_id) {
  NEED_DEV();
  auto it = g_desc.find(coeffs);
  if (it == g_desc.end() || it->second.is_base) return fail(H2G_ERR_HANDLE, "unknown coeffs descriptor");
  if (it->second.n != n) return fail(H2G_ERR_ARG, "msm: coeffs.len() != bases.len()");
  HIPCHK(d->b.ensure(n * 64 + 64));
  HIPCHK(d->out.ensure(64));
  HIPCHK(hipMemcpyAsync(d->b.p, bases, n * 64, hipMemcpyHostToDevice, d->stream));
  return msm_host_impl(d, it->second.d, d->b.p, n, 0, out, is_id, d->stream);
}

int h2g_msm_with_cached_base(const uint64_t* coeffs, size_t n, uint64_t base, size_t off, uint64_t out[8],
                             int* is_id) {
  NEED_DEV();
  auto it = g_desc.find(base);
  if (it == g_desc.end() || !it->second.is_base) return fail(H2G_ERR_HANDLE, "unknown base descriptor");
  if (off + n > it->second.n) return fail(H2G_ERR_ARG, "msm: bases.len() < size");
  HIPCHK(d->a.ensure(n * 32 + 32));
  HIPCHK(d->out.ensure(64));
  HIPCHK(hipMemcpyAsync(d->a.p, coeffs, n * 32, hipMemcpyHostToDevice, d->stream));
  return msm_desc_impl(d, d->a.p, it->second, off, n, out, is_id, d->stream);
}

int h2g_msm_with_cached_inputs(uint64_t coeffs, uint64_t base, size_t off, uint64_t out[8], int* is_id) {
  NEED_DEV();
  auto ic = g_desc.find(coeffs);
  auto ib = g_desc.find(base);
  if (ic == g_desc.end() || ic->second.is_base) return fail(H2G_ERR_HANDLE, "unknown coeffs descriptor");
  if (ib == g_desc.end() || !ib->second.is_base) return fail(H2G_ERR_HANDLE, "unknown base descriptor");
  const size_t n = ic->second.n;
  if (off + n > ib->second.n) return fail(H2G_ERR_ARG, "msm: bases.len() < size");
  return msm_desc_impl(d, ic->second.d, ib->second, off, n, out, is_id, d->stream);
}

int h2g_msm_dev(const void* sc, const void* bs, size_t n, void* out, void* stream) {
  return h2g_msm_dev_cfg(sc, bs, n, 0, out, stream);
}

int h2g_msm_dev_cfg(const void* sc, const void* bs, size_t n, int c, void* out, void* stream) {
  NEED_DEV();
  if (!out || (n && (!sc || !bs))) return fail(H2G_ERR_ARG, "msm_dev: null pointer");
  if (c < 0 || c > 24) return fail(H2G_ERR_ARG, "msm_dev: window_bits out of range");
  return msm_dev_impl(d, sc, bs, n, c, out, pick_stream(d, stream));
}

int h2g_msm_dev_host(const void* sc, const void* bs, size_t n, int c, uint64_t out[8], int* is_id, void* stream) {
  NEED_DEV();
  if (!out || (n && (!sc || !bs))) return fail(H2G_ERR_ARG, "msm_dev_host: null pointer");
  if (c < 0 || c > 24) return fail(H2G_ERR_ARG, "msm_dev_host: window_bits out of range");
  return msm_host_impl(d, sc, bs, n, c, out, is_id, pick_stream(d, stream));
}

int h2g_srs_setup_dev(const uint64_t s[4], size_t n, void* d_out, void* stream) {
  NEED_DEV();
  if (!s || (n && !d_out)) return fail(H2G_ERR_ARG, "srs: null pointer");
  HIPCHK(srs_setup(fr_from_limbs(s), n, reinterpret_cast<G1Affine*>(d_out), pick_stream(d, stream)));
  return H2G_OK;
}

// ---------------------------------------------------------------- FFT
int h2g_fft_dev(void* a, uint32_t log_n, const uint64_t omega[4], void* stream) {
  NEED_DEV();
  if (!a || !omega || log_n > FR_S) return fail(H2G_ERR_ARG, "fft: bad argument");
  const Fr w = fr_from_limbs(omega);
  const Fr one = Fr::one();
  const uint64_t N = 1ull << log_n;
  return ntt_dev_impl(d, (const Fr*)a, N, (Fr*)a, N, (int)log_n, w, 0, one, one, 0, one, 0, one, one,
                      pick_stream(d, stream));
}

int h2g_fft(uint64_t* a, uint32_t log_n, const uint64_t omega[4]) {
  NEED_DEV();
  if (!a || !omega || log_n > FR_S) return fail(H2G_ERR_ARG, "fft: bad argument");
  const size_t bytes = ((size_t)1 << log_n) * 32;
  HIPCHK(d->a.ensure(bytes));
  HIPCHK(hipMemcpyAsync(d->a.p, a, bytes, hipMemcpyHostToDevice, d->stream));
  int rc = h2g_fft_dev(d->a.p, log_n, omega, nullptr);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(a, d->a.p, bytes, hipMemcpyDeviceToHost, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  return H2G_OK;
}

// ---------------------------------------------------------------- EvaluationDomain
int h2g_domain_create(uint32_t j, uint32_t k, uint64_t* handle) {
  NEED_DEV();
  if (!handle) return fail(H2G_ERR_ARG, "domain: null handle");
  auto dm = std::make_unique<Domain>();
  RCCHK(domain_init(dm.get(), j, k));
  *handle = g_next_handle++;
  g_dom[*handle] = std::move(dm);
  return H2G_OK;
}

int h2g_domain_free(uint64_t handle) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  auto it = g_dom.find(handle);
  if (it == g_dom.end()) return fail(H2G_ERR_HANDLE, "unknown domain");
  if (it->second->d_t) (void)hipFree(it->second->d_t);
  g_dom.erase(it);
  return H2G_OK;
}

int h2g_domain_info(uint64_t handle, uint32_t* k, uint32_t* ek, uint64_t consts[36]) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  Domain* dm = get_dom(handle);
  if (!dm) return fail(H2G_ERR_HANDLE, "unknown domain");
  if (k) *k = dm->k;
  if (ek) *ek = dm->ek;
  if (consts) {
    const Fr c[9] = {dm->omega, dm->omega_inv, dm->ext_omega, dm->ext_omega_inv, dm->g_coset,
                     dm->g_coset_inv, dm->ifft_div, dm->ext_ifft_div, dm->bary};
    for (int i = 0; i < 9; i++) fr_to_limbs(c[i], consts + 4 * i);
  }
  return H2G_OK;
}

int h2g_lagrange_to_coeff_dev(uint64_t dom, void* a, void* stream) {
  NEED_DEV();
  Domain* dm = get_dom(dom);
  if (!dm) return fail(H2G_ERR_HANDLE, "unknown domain");
  if (!a) return fail(H2G_ERR_ARG, "null");
  return lagrange_to_coeff(d, *dm, (const Fr*)a, (Fr*)a, pick_stream(d, stream));
}

int h2g_coeff_to_extended_dev(uint64_t dom, const void* a, void* out, void* stream) {
  NEED_DEV();
  Domain* dm = get_dom(dom);
  if (!dm) return fail(H2G_ERR_HANDLE, "unknown domain");
  if (!a || !out) return fail(H2G_ERR_ARG, "null");
  if (a == out) return fail(H2G_ERR_ARG, "coeff_to_extended: in and out must differ");
  return coeff_to_extended(d, *dm, (const Fr*)a, (Fr*)out, pick_stream(d, stream));
}

int h2g_extended_to_coeff_dev(uint64_t dom, const void* a, void* out, void* stream) {
  NEED_DEV();
  Domain* dm = get_dom(dom);
  if (!dm) return fail(H2G_ERR_HANDLE, "unknown domain");
  if (!a || !out) return fail(H2G_ERR_ARG, "null");
  return extended_to_coeff(d, *dm, (const Fr*)a, (Fr*)out, pick_stream(d, stream));
}

int h2g_divide_by_vanishing_poly_dev(uint64_t dom, void* a, void* stream) {
  NEED_DEV();
  Domain* dm = get_dom(dom);
  if (!dm) return fail(H2G_ERR_HANDLE, "unknown domain");
  if (!a) return fail(H2G_ERR_ARG, "null");
  HIPCHK(poly_mul_cyclic((Fr*)a, 1ull << dm->ek, dm->d_t, dm->t_evals.size(), pick_stream(d, stream)));
  return H2G_OK;
}

// host-pointer domain wrappers
static int host_roundtrip(size_t in_elems, const uint64_t* in, size_t out_elems, uint64_t* out,
                          int (*fn)(uint64_t, const void*, void*, void*), uint64_t dom) {
  NEED_DEV();
  HIPCHK(d->b.ensure(in_elems * 32 + 32));
  HIPCHK(d->c.ensure(out_elems * 32 + 32));
  HIPCHK(hipMemcpyAsync(d->b.p, in, in_elems * 32, hipMemcpyHostToDevice, d->stream));
  int rc = fn(dom, d->b.p, d->c.p, nullptr);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(out, d->c.p, out_elems * 32, hipMemcpyDeviceToHost, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  return H2G_OK;
}

int h2g_lagrange_to_coeff(uint64_t dom, uint64_t* a) {
  NEED_DEV();
  Domain* dm = get_dom(dom);
  if (!dm) return fail(H2G_ERR_HANDLE, "unknown domain");
  const size_t n = 1ull << dm->k;
  HIPCHK(d->b.ensure(n * 32));
  HIPCHK(hipMemcpyAsync(d->b.p, a, n * 32, hipMemcpyHostToDevice, d->stream));
  int rc = h2g_lagrange_to_coeff_dev(dom, d->b.p, nullptr);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(a, d->b.p, n * 32, hipMemcpyDeviceToHost, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  return H2G_OK;
}

int h2g_coeff_to_extended(uint64_t dom, const uint64_t* a, uint64_t* out) {
  Domain* dm;
  {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    dm = get_dom(dom);
    if (!dm) return fail(H2G_ERR_HANDLE, "unknown domain");
  }
  return host_roundtrip(1ull << dm->k, a, 1ull << dm->ek, out, h2g_coeff_to_extended_dev, dom);
}

int h2g_extended_to_coeff(uint64_t dom, const uint64_t* a, uint64_t* out) {
  Domain* dm;
  {
    std::lock_guard<std::recursive_mutex> lk(g_mu);
    dm = get_dom(dom);
    if (!dm) return fail(H2G_ERR_HANDLE, "unknown domain");
  }
  return host_roundtrip(1ull << dm->ek, a, (1ull << dm->k) * (dm->j - 1), out, h2g_extended_to_coeff_dev, dom);
}

int h2g_divide_by_vanishing_poly(uint64_t dom, uint64_t* a) {
  NEED_DEV();
  Domain* dm = get_dom(dom);
  if (!dm) return fail(H2G_ERR_HANDLE, "unknown domain");
  const size_t n = 1ull << dm->ek;
  HIPCHK(d->b.ensure(n * 32));
  HIPCHK(hipMemcpyAsync(d->b.p, a, n * 32, hipMemcpyHostToDevice, d->stream));
  int rc = h2g_divide_by_vanishing_poly_dev(dom, d->b.p, nullptr);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(a, d->b.p, n * 32, hipMemcpyDeviceToHost, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  return H2G_OK;
}

// ---------------------------------------------------------------- poly ops
int h2g_fr_op_dev(int op, const void* a, const void* b, const uint64_t c[4], void* out, size_t n, void* stream) {
  NEED_DEV();
  if (op < 0 || op > 6) return fail(H2G_ERR_ARG, "fr_op: unknown op");
  if (n && (!a || !out || ((op <= 2 || op == 6) && !b) || (op >= 3 && !c)))
    return fail(H2G_ERR_ARG, "fr_op: null pointer");
  hipStream_t st = pick_stream(d, stream);
  const Fr cv = op >= 3 ? fr_from_limbs(c) : Fr::zero();
  HIPCHK(poly_binop(op, (const Fr*)a, (const Fr*)b, cv, (Fr*)out, n, st));
  return H2G_OK;
}

int h2g_fr_op(int op, const uint64_t* a, const uint64_t* b, const uint64_t c[4], uint64_t* out, size_t n) {
  NEED_DEV();
  HIPCHK(d->a.ensure(n * 32 + 32));
  HIPCHK(d->b.ensure(n * 32 + 32));
  HIPCHK(d->c.ensure(n * 32 + 32));
  HIPCHK(hipMemcpyAsync(d->a.p, a, n * 32, hipMemcpyHostToDevice, d->stream));
  if (b) HIPCHK(hipMemcpyAsync(d->b.p, b, n * 32, hipMemcpyHostToDevice, d->stream));
  int rc = h2g_fr_op_dev(op, d->a.p, b ? d->b.p : nullptr, c, d->c.p, n, nullptr);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(out, d->c.p, n * 32, hipMemcpyDeviceToHost, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  return H2G_OK;
}

int h2g_fr_batch_invert_dev(void* a, size_t n, void* stream) {
  NEED_DEV();
  if (n && !a) return fail(H2G_ERR_ARG, "null");
  HIPCHK(d->work.ensure(n * 32 + 32));
  HIPCHK(poly_batch_invert((Fr*)a, n, (Fr*)d->work.p, pick_stream(d, stream)));
  return H2G_OK;
}

int h2g_fr_batch_invert(uint64_t* a, size_t n) {
  NEED_DEV();
  HIPCHK(d->a.ensure(n * 32 + 32));
  HIPCHK(hipMemcpyAsync(d->a.p, a, n * 32, hipMemcpyHostToDevice, d->stream));
  int rc = h2g_fr_batch_invert_dev(d->a.p, n, nullptr);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(a, d->a.p, n * 32, hipMemcpyDeviceToHost, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  return H2G_OK;
}

int h2g_fr_prefix_product_dev(const void* a, void* out, size_t n, void* stream) {
  NEED_DEV();
  if (n && (!a || !out)) return fail(H2G_ERR_ARG, "null");
  const size_t sl = poly_prefix_scratch_len(n);
  HIPCHK(d->work.ensure(sl * 32 + 32));
  HIPCHK(poly_prefix_product((const Fr*)a, (Fr*)out, n, (Fr*)d->work.p, sl, pick_stream(d, stream)));
  return H2G_OK;
}

int h2g_fr_prefix_product(const uint64_t* a, uint64_t* out, size_t n) {
  NEED_DEV();
  HIPCHK(d->a.ensure(n * 32 + 32));
  HIPCHK(d->c.ensure(n * 32 + 32));
  HIPCHK(hipMemcpyAsync(d->a.p, a, n * 32, hipMemcpyHostToDevice, d->stream));
  int rc = h2g_fr_prefix_product_dev(d->a.p, d->c.p, n, nullptr);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(out, d->c.p, n * 32, hipMemcpyDeviceToHost, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  return H2G_OK;
}

// exclusive prefix sum of u32 counts (the lookup argument's compactions and radix sort)
int h2g_u32_exclusive_scan_dev(const void* in, void* out, size_t n, void* stream) {
  NEED_DEV();
  if (n && (!in || !out)) return fail(H2G_ERR_ARG, "null");
  if (n >= 0xffffffffull) return fail(H2G_ERR_ARG, "scan: length >= 2^32");
  HIPCHK(d->work.ensure(scan_u32_scratch_bytes(n) + 256));
  HIPCHK(exclusive_scan_u32((const uint32_t*)in, (uint32_t*)out, n, d->work.p, pick_stream(d, stream)));
  return H2G_OK;
}

// ---------------------------------------------------------------- memory / events
int h2g_dev_alloc(size_t bytes, void** p) {
  NEED_DEV();
  HIPCHK(hipMalloc(p, bytes ? bytes : 16));
  return H2G_OK;
}
int h2g_dev_free(void* p) {
  NEED_DEV();
  HIPCHK(hipFree(p));
  return H2G_OK;
}
int h2g_memcpy_htod(void* dst, const void* src, size_t bytes) {
  NEED_DEV();
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return H2G_OK;
}
int h2g_memcpy_dtoh(void* dst, const void* src, size_t bytes) {
  NEED_DEV();
  HIPCHK(hipStreamSynchronize(d->stream));
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return H2G_OK;
}
int h2g_memcpy_dtod(void* dst, const void* src, size_t bytes) {
  NEED_DEV();
  if (bytes && (!dst || !src)) return fail(H2G_ERR_ARG, "memcpy_dtod: null pointer");
  // on the library stream and waited for: a device-to-device hipMemcpy may return before
  // the copy is done, and the prover's non-blocking streams would not order after it
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  return H2G_OK;
}
int h2g_synchronize(void) {
  NEED_DEV();
  HIPCHK(hipStreamSynchronize(d->stream));
  HIPCHK(hipDeviceSynchronize());
  return H2G_OK;
}
int h2g_event_create(void** ev) {
  NEED_DEV();
  hipEvent_t e;
  HIPCHK(hipEventCreate(&e));
  *ev = e;
  return H2G_OK;
}
int h2g_event_destroy(void* ev) {
  NEED_DEV();
  HIPCHK(hipEventDestroy((hipEvent_t)ev));
  return H2G_OK;
}
int h2g_event_record(void* ev, void* stream) {
  NEED_DEV();
  HIPCHK(hipEventRecord((hipEvent_t)ev, pick_stream(d, stream)));
  return H2G_OK;
}
int h2g_event_elapsed_ms(void* a, void* b, float* ms) {
  NEED_DEV();
  HIPCHK(hipEventSynchronize((hipEvent_t)b));
  HIPCHK(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b));
  return H2G_OK;
}

// ---------------------------------------------------------------- profiling
int h2g_profile_enable(int on) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  g_profile = on != 0;
  return H2G_OK;
}

int h2g_profile_msm_entries(uint64_t* total, int* uncounted) {
  NEED_DEV();
  if (!total) return fail(H2G_ERR_ARG, "profile_msm_entries: null total");
  uint64_t t = 0;
  int un = 0;
  for (auto& pe : g_msm_prof) {
    HIPCHK(hipEventSynchronize(pe.ev[MSM_NPHASES]));
    if (pe.entries) t += *pe.entries;
    else un++;
  }
  *total = t;
  if (uncounted) *uncounted = un;
  return H2G_OK;
}

int h2g_profile_msm_collect(float* ms, int max_phases, int* n_phases, int* calls) {
  NEED_DEV();
  const int np = MSM_NPHASES < max_phases ? MSM_NPHASES : max_phases;
  for (int i = 0; i < np; i++) ms[i] = 0.f;
  for (auto& pe : g_msm_prof) {
    HIPCHK(hipEventSynchronize(pe.ev[MSM_NPHASES]));
    for (int i = 0; i < np; i++) {
      float t = 0.f;
      HIPCHK(hipEventElapsedTime(&t, pe.ev[i], pe.ev[i + 1]));
      ms[i] += t;
    }
  }
  if (calls) {
    int c = 0;
    for (auto& pe : g_msm_prof) c += pe.msms;
    *calls = c;
  }
  if (n_phases) *n_phases = np;
  // ms[NPHASES], ms[NPHASES + 1] (when asked for): the union of the accumulate intervals and
  // of the whole-MSM intervals over every recorded MSM -- the busy time of overlapping MSMs
  // (two MSM streams), so that work / union is the aggregate rate, not the per-launch one
  if (max_phases >= MSM_NPHASES + 2 && !g_msm_prof.empty()) {
    const hipEvent_t ref = g_msm_prof.front().ev[0];
    auto union_ms = [&](int a, int b) -> float {
      std::vector<std::pair<float, float>> iv;
      for (auto& pe : g_msm_prof) {
        float s = 0.f, e = 0.f;
        if (hipEventElapsedTime(&s, ref, pe.ev[a]) != hipSuccess) return -1.f;
        if (hipEventElapsedTime(&e, ref, pe.ev[b]) != hipSuccess) return -1.f;
        iv.emplace_back(s, e);
      }
      std::sort(iv.begin(), iv.end());
      float tot = 0.f, cs = iv[0].first, ce = iv[0].second;
      for (size_t i = 1; i < iv.size(); i++) {
        if (iv[i].first > ce) {
          tot += ce - cs;
          cs = iv[i].first;
          ce = iv[i].second;
        } else if (iv[i].second > ce) {
          ce = iv[i].second;
        }
      }
      return tot + (ce - cs);
    };
    ms[MSM_NPHASES] = union_ms(3, 4);
    ms[MSM_NPHASES + 1] = union_ms(0, MSM_NPHASES);
  }
  for (auto& pe : g_msm_prof)
    for (auto& e : pe.ev) (void)hipEventDestroy(e);
  g_msm_prof.clear();
  return H2G_OK;
}

// ---------------------------------------------------------------- host point helper
int h2g_g1_add_affine(const uint64_t a[8], const uint64_t b[8], uint64_t out[8]) {
  G1Affine pa, pb;
  std::memcpy(&pa, a, 64);
  std::memcpy(&pb, b, 64);
  const G1xyzz s = xyzz_madd(G1xyzz::from_affine(pa), pb);
  const G1Affine r = xyzz_to_affine(s);
  std::memcpy(out, &r, 64);
  return H2G_OK;
}

}  // extern "C"
