// msm.h -- Pippenger MSM over BN254 G1 (see msm.hip).
#pragma once
#include "bn254.h"

namespace h2g {

struct MsmConfig {
  int c = 0;         // window bits (0: choose from n)
  int item_len = 0;  // entries per accumulation chunk (0: choose)
};

// Device workspace, grown on demand and reused across calls.
struct MsmWorkspace {
  size_t cap[10] = {};  // byte capacity of each buffer below (grown on demand, never shrunk)
  int last_c = 0, last_W = 0;    // window config of the most recent msm_run
  void* ent = nullptr;           // u64 [n*W] coarse-binned entries (key << 32 | value)
  void* vals_out = nullptr;      // u32 [n*W] values (table index | sign << 31) in bucket order
  void* item_bucket = nullptr;   // big-bucket work items
  void* partials = nullptr;      // G1xyzz [2 * chunks] boundary slots
  void* buckets = nullptr;       // G1xyzz [W*NB]
  void* segs = nullptr;          // G1xyzz: reduction levels (2 ping-pong arrays + block sums)
  void* windows = nullptr;       // G1xyzz [W]
  void* result = nullptr;        // counters: [0] items, [1] multi-item buckets
  void* item_off = nullptr;      // uint4 multi-item big buckets (bucket, first item, items)
  void* total_items = nullptr;   // G1xyzz partial sums of big-bucket items
  void* sort_tmp = nullptr;  // partition counts / offsets, per-key offsets; zero-initialised
  size_t sort_tmp_bytes = 0;
  size_t sort_kcap = 0;  // per-key array's capacity (buckets of all sets)
};

int msm_choose_c(size_t n);
int msm_windows_for(int c);

// Optional per-phase HIP events (profiling).  Phases: digits, sort, bucket_bounds,
// accumulate, bucket_fixup, reduce -> 7 events, recorded on the MSM's stream.
static constexpr int MSM_NPHASES = 6;
struct MsmPhaseEvents {
  hipEvent_t ev[MSM_NPHASES + 1];
  int msms = 1;  // MSMs the timed pipeline served (a batch counts each)
  uint32_t* entries = nullptr;  // pinned: receives the sorted-entry (nonzero digit) count
};

// Scalar vectors of a batch of MSMs (kernel argument by value).
static constexpr int MSM_MAX_BATCH = 64;
struct MsmScalarList {
  const Fr* p[MSM_MAX_BATCH];
};

// sum_i scalars[i] * bases[i]; scalars Montgomery Fr, bases affine Montgomery Fq
// (halo2curves layout).  Asynchronous on `st`.  If d_out != nullptr the affine
// result is written there by one device lane; otherwise the W window sums are
// left in ws->windows (G1xyzz[ws->last_W]) for msm_windows_host_finish.
hipError_t msm_run(const Fr* d_scalars, const G1Affine* d_bases, size_t n, MsmWorkspace* ws,
                   const MsmConfig& cfg, G1Affine* d_out, hipStream_t st, MsmPhaseEvents* prof = nullptr);
G1Affine msm_windows_host_finish(const G1xyzz* h_windows, int W, int c);
void msm_free(MsmWorkspace* ws);

// Fixed-base mode for resident bases (SRS, base descriptors): windows are
// pre-multiplied, table[w * n + i] = [2^(c w)] bases[i], so all W windows share one
// set of 2^(c-1) buckets (one reduction instead of W; larger c affordable).
// W * n * 64 B of HBM per table (e.g. 3.5 GB for n = 2^22, c = 20).
struct MsmFixedBase {
  G1Affine* table = nullptr;
  size_t n = 0;
  int c = 0, W = 0;
};
int msm_choose_c_fixed(size_t n);
hipError_t msm_fixed_base_build(const G1Affine* d_bases, size_t n, int c, MsmFixedBase* fb, hipStream_t st);
void msm_fixed_base_free(MsmFixedBase* fb);
// inclusive prefix sums of n affine points: out[i] = in[0] + ... + in[i] (setup; scratch
// allocated and freed inside)
hipError_t msm_prefix_points(const G1Affine* in, size_t n, G1Affine* out, hipStream_t st);
// sum_{i < n} scalars[i] * bases[off + i]; leaves ws->windows[0] (ws->last_W = 1)
hipError_t msm_run_fixed(const Fr* d_scalars, const MsmFixedBase& fb, size_t off, size_t n, MsmWorkspace* ws,
                         G1Affine* d_out, hipStream_t st, MsmPhaseEvents* prof = nullptr);
// nbatch MSMs sum_i list.p[b][i] * bases[off + i] (b < nbatch <= MSM_MAX_BATCH) as one
// pipeline -- one digits launch, one sort, one accumulation, one reduction with a bucket
// set per MSM -- so the latency-bound reduction is paid once.  Leaves MSM b's sum in
// ws->windows[b] (ws->last_W = nbatch).  nbatch * W * n must stay below 2^31.
hipError_t msm_run_fixed_batch(const MsmScalarList& list, int nbatch, const MsmFixedBase& fb, size_t off, size_t n,
                               MsmWorkspace* ws, hipStream_t st, MsmPhaseEvents* prof = nullptr);

}  // namespace h2g
