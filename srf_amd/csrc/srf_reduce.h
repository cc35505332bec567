// Host-side launcher of the deterministic column-sum (reduce.hip).
#pragma once
#include <algorithm>

#include "srf_common.h"

namespace srf {
constexpr int kColsumMaxSlices = 64;
// scratch must hold colsum_scratch_floats(rows, cols) floats.
size_t colsum_scratch_floats(int rows, int cols);
int colsum(const float* in, int rows, int cols, float* out, float* scratch, hipStream_t st);
}  // namespace srf
