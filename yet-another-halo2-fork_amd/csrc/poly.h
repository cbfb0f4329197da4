// poly.h -- elementwise and scan kernels over Fr vectors (see poly.hip).
#pragma once
#include "bn254.h"

namespace h2g {

enum PolyOp : int {
  POLY_ADD = 0,        // out = a + b            (poly.rs:200-212 Add)
  POLY_SUB = 1,        // out = a - b            (poly.rs:214-226 Sub)
  POLY_MUL = 2,        // out = a * b            (evaluation.rs products)
  POLY_SCALE = 3,      // out = a * c            (poly.rs:244-266 Mul<F>)
  POLY_SUB_CONST = 4,  // out = a - c            (poly.rs:268-276 Sub<F>)
  POLY_ADD_CONST = 5,  // out = a + c
  POLY_AXPY = 6,       // out = a * c + b        (shplonk / vanishing folds)
};

hipError_t poly_binop(int op, const Fr* a, const Fr* b, const Fr& c, Fr* out, size_t n, hipStream_t st);
// a[i] *= t[i mod t_len]   (domain.rs:297-316); t_len must be a power of two
hipError_t poly_mul_cyclic(Fr* a, size_t n, const Fr* t, size_t t_len, hipStream_t st);
// ff BatchInvert semantics (zeros stay zero), in place; scratch >= n Fr
hipError_t poly_batch_invert(Fr* a, size_t n, Fr* scratch, hipStream_t st);
// count independent batch inversions of n elements (a[i] in place, scratch[i] >= n Fr),
// POLY_INV_MAX_BATCH arrays per launch
static constexpr int POLY_INV_MAX_BATCH = 16;
hipError_t poly_batch_invert_multi(Fr* const* a, Fr* const* scratch, int count, size_t n, hipStream_t st);
// out[i] = prod_{j<=i} a[j]; scratch >= 2 * ceil(n / 2^?) Fr (see poly.hip)
hipError_t poly_prefix_product(const Fr* a, Fr* out, size_t n, Fr* scratch, size_t scratch_len, hipStream_t st);
size_t poly_prefix_scratch_len(size_t n);
// count independent prefix products (out[i] may alias a[i]); scratch >= min(count, 16) *
// poly_prefix_scratch_len(n) Fr
hipError_t poly_prefix_product_multi(const Fr* const* a, Fr* const* out, int count, size_t n, Fr* scratch,
                                     size_t scratch_len, hipStream_t st);

}  // namespace h2g
