// srs.h -- device SRS generation (see srs.hip).
#pragma once
#include "bn254.h"

namespace h2g {
hipError_t srs_setup(const Fr& s, size_t n, G1Affine* d_out, hipStream_t st);
}
