// msm.h -- Pippenger MSM over BN254 G1 (see msm.hip).
#pragma once
#include "bn254.h"

namespace h2g {

struct MsmConfig {
  int c = 0;          // window bits (0: choose from n)
  int item_len = 0;   // max points per accumulation work item (0: choose)
};

// Device workspace, grown on demand and reused across calls.
struct MsmWorkspace {
  size_t cap_n = 0;
  int cap_c = 0;
  void* keys_in = nullptr;     // u32 [n*W]
  void* keys_out = nullptr;    // u32 [n*W]
  void* vals_in = nullptr;     // u32 [n*W]
  void* vals_out = nullptr;    // u32 [n*W]
  void* bucket_start = nullptr;  // u32 [W*NB]
  void* bucket_end = nullptr;    // u32 [W*NB]
  void* item_off = nullptr;      // u32 [W*NB + 1]
  void* item_bucket = nullptr;   // u32 [max items]
  void* partials = nullptr;      // G1xyzz [max items]
  void* buckets = nullptr;       // G1xyzz [W*NB]
  void* segs = nullptr;          // G1xyzz [W*SEGS]
  void* windows = nullptr;       // G1xyzz [W]
  void* result = nullptr;        // G1Affine + flag
  void* total_items = nullptr;   // u32
  void* sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  void* scan_tmp = nullptr;
  size_t scan_tmp_bytes = 0;
};

int msm_choose_c(size_t n);

// Optional per-phase HIP events (profiling).  Phases: digits, sort, bucket_bounds,
// accumulate, bucket_sum, reduce -> 7 events, recorded on the MSM's stream.
static constexpr int MSM_NPHASES = 6;
struct MsmPhaseEvents {
  hipEvent_t ev[MSM_NPHASES + 1];
};

// result (device, G1Affine) = sum_i scalars[i] * bases[i]; scalars Montgomery Fr,
// bases affine Montgomery Fq (halo2curves layout).  Asynchronous on `st`.
hipError_t msm_run(const Fr* d_scalars, const G1Affine* d_bases, size_t n, MsmWorkspace* ws,
                   const MsmConfig& cfg, G1Affine* d_out, hipStream_t st, MsmPhaseEvents* prof = nullptr);
void msm_free(MsmWorkspace* ws);

}  // namespace h2g
