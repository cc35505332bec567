// Deterministic column sums shared by the backward passes:
// out[c] = sum_r in[r][c] over a [rows][cols] slab of per-block partials.
// Up to 4096 rows (or >= 128 column blocks): colsum_one, one launch.
// Stage 1: blocks of 4 row-lanes x 64 columns stream a slice of rows (coalesced
// along columns) into part[slice][cols]; stage 2: one thread per column adds the
// slices in order.  Fixed order => bitwise reproducible.
#include "srf_common.h"
#include "srf_reduce.h"

namespace {
using srf::ColSplit;

__global__ __launch_bounds__(256) void colsum_stage1(const float* __restrict__ in, int rows, int cols,
                                                     int rows_per_slice, float* __restrict__ part) {
  __shared__ float sh[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_slice, r1 = min(rows, r0 + rows_per_slice);
  float s = 0.f;
  if (c < cols) {
#pragma unroll 8
    for (int r = r0 + rg; r < r1; r += 4) s += in[(size_t)r * cols + c];
  }
  sh[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && c < cols) {
    const int l = threadIdx.x & 63;
    part[(size_t)blockIdx.y * cols + c] = sh[0][l] + sh[1][l] + sh[2][l] + sh[3][l];
  }
}

__global__ void colsum_stage2(const float* __restrict__ part, int slices, int cols, float* __restrict__ out,
                              ColSplit split) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
#pragma unroll 8
  for (int k = 0; k < slices; ++k) s += part[(size_t)k * cols + c];
  if (out) out[c] = s;
  int start = 0;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    if (split.dst[k] && c >= start && c < start + split.width[k]) split.dst[k][c - start] = s;
    start += split.width[k];
  }
}

// One launch for moderate row counts: a 1024-thread block per CW columns, 1024/CW row
// lanes each summing rows r = lane (mod 1024/CW) in order, then the lane sums in
// order.  CW = 64 when there are enough column blocks; CW = 16 for narrow slabs (four
// times the row lanes, so a few blocks still keep many loads in flight).
template <int CW>
__global__ __launch_bounds__(1024) void colsum_one(const float* __restrict__ in, int rows, int cols,
                                                   float* __restrict__ out, ColSplit split) {
  constexpr int RG = 1024 / CW;
  __shared__ float sh[RG][CW];
  const int l = threadIdx.x % CW, rg = threadIdx.x / CW;
  const int c = blockIdx.x * CW + l;
  float s = 0.f;
  if (c < cols) {
#pragma unroll 8
    for (int r = rg; r < rows; r += RG) s += in[(size_t)r * cols + c];
  }
  sh[rg][l] = s;
  __syncthreads();
  if (rg != 0 || c >= cols) return;
  float t = 0.f;
#pragma unroll 16
  for (int k = 0; k < RG; ++k) t += sh[k][l];
  if (out) out[c] = t;
  int start = 0;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    if (split.dst[k] && c >= start && c < start + split.width[k]) split.dst[k][c - start] = t;
    start += split.width[k];
  }
}

}  // namespace

namespace srf {

size_t colsum_scratch_floats(int rows, int cols) { return (size_t)kColsumMaxSlices * cols; (void)rows; }

int colsum(const float* in, int rows, int cols, float* out, float* scratch, hipStream_t st, const ColSplit& split) {
  if (rows <= 128) {   // few partial rows: one pass, one thread per column
    hipLaunchKernelGGL(colsum_stage2, dim3((cols + 255) / 256), dim3(256), 0, st, in, rows, cols, out, split);
    SRF_LAUNCH_CHECK("colsum_stage2");
    return SRF_OK;
  }
  const int cblocks = (cols + 63) / 64;
  if ((size_t)rows * 64 <= 256 * 1024 || cblocks >= 128) {
    // up to 16K rows per 16 lanes (<= 1K adds per thread) or enough column blocks to fill the
    // chip: one launch instead of two
    if (cblocks < 64)
      hipLaunchKernelGGL(colsum_one<16>, dim3((cols + 15) / 16), dim3(1024), 0, st, in, rows, cols, out, split);
    else
      hipLaunchKernelGGL(colsum_one<64>, dim3(cblocks), dim3(1024), 0, st, in, rows, cols, out, split);
    SRF_LAUNCH_CHECK("colsum_one");
    return SRF_OK;
  }
  int slices = std::max(1, std::min(kColsumMaxSlices, (1024 + cblocks - 1) / cblocks));
  slices = std::min(slices, std::max(1, rows / 16));
  const int rps = (rows + slices - 1) / slices;
  slices = (rows + rps - 1) / rps;
  hipLaunchKernelGGL(colsum_stage1, dim3(cblocks, slices), dim3(256), 0, st, in, rows, cols, rps, scratch);
  SRF_LAUNCH_CHECK("colsum_stage1");
  hipLaunchKernelGGL(colsum_stage2, dim3((cols + 255) / 256), dim3(256), 0, st, scratch, slices, cols, out, split);
  SRF_LAUNCH_CHECK("colsum_stage2");
  return SRF_OK;
}

}  // namespace srf
