// radix.h -- LSD radix sort of (u64 key, u32 value) pairs and stream compaction (radix.hip):
// the sorts and selections of permute_expression_pair (lookup/prover.rs:410-494) without a
// library sort.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "prover_kernels.h"

namespace h2g {

// exclusive scan of len u32 (len < 2^32, in == out allowed); scratch >= scan_u32_scratch_bytes(len)
size_t scan_u32_scratch_bytes(size_t len);
hipError_t exclusive_scan_u32(const uint32_t* in, uint32_t* out, size_t len, void* scratch, hipStream_t st);

// Stable sort of n (keys[i], vals[i]) by key bits [lo_bit, hi_bit), 8 bits per pass,
// ping-ponging between (keys, vals) and (keys_alt, vals_alt): *in_alt says which pair holds
// the result (an odd number of passes ends in the alt buffers).  scratch >=
// radix_sort_scratch_bytes(n).
size_t radix_sort_scratch_bytes(size_t n);
hipError_t radix_sort_pairs(uint64_t* keys, uint32_t* vals, uint64_t* keys_alt, uint32_t* vals_alt, size_t n,
                            int lo_bit, int hi_bit, void* scratch, hipStream_t st, bool* in_alt);

// the full sort's building blocks: out[i] = i; key[i] = 64-bit limb `limb` of canon[idx[i]]
hipError_t iota_u32(uint32_t* out, size_t n, hipStream_t st);
hipError_t canon_limb_keys(const CanonKey* canon, const uint32_t* idx, size_t n, int limb, uint64_t* key,
                           hipStream_t st);

// out[j] = in[i] (compact_canon) / i (compact_index) for the j-th i < n with flags[i] != 0,
// in order; *d_count = their number.  scratch >= compact_scratch_bytes(n).
size_t compact_scratch_bytes(size_t n);
hipError_t compact_canon(const CanonKey* in, const uint8_t* flags, size_t n, CanonKey* out, uint32_t* d_count,
                         void* scratch, hipStream_t st);
hipError_t compact_index(const uint8_t* flags, size_t n, uint32_t* out, uint32_t* d_count, void* scratch,
                         hipStream_t st);

}  // namespace h2g
