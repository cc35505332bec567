// Host-side launcher of the deterministic column-sum (reduce.hip).
#pragma once
#include <algorithm>

#include "srf_common.h"

namespace srf {
constexpr int kColsumMaxSlices = 64;
// scratch must hold colsum_scratch_floats(rows, cols) floats.
size_t colsum_scratch_floats(int rows, int cols);
// Optional scatter of the column sums: columns [start_k, start_k + width_k) go to
// dst[k][0 .. width_k) (start_k = sum of the earlier widths), e.g. a packed
// (d_beta | d_gamma) partial straight into two parameter gradients.
struct ColSplit {
  float* dst[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  int width[6] = {0, 0, 0, 0, 0, 0};
};
// out (may be null when split is given) receives all cols sums.
int colsum(const float* in, int rows, int cols, float* out, float* scratch, hipStream_t st,
           const ColSplit& split = ColSplit{});
}  // namespace srf
