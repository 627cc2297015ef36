// Device side of the periodic fault-tolerance strategies:
// remapping (strategy.cpp:35-137) and genetic (strategy.cpp:139-288).
//
// The reference runs both on the host over cpu_data()/cpu_diff(), which in GPU
// mode flips every FC blob's head to the CPU and back (SyncedMemory, a9).  Here
// the fault statistics are reduced on the device and the neuron moves are
// gathers with device index vectors; only the per-neuron counts (a few KB) and
// the permutation vectors cross PCIe.  Everything is integer counting or a
// copy, so results are bit-exact by construction.
#include "rram_common.hpp"

namespace rram {
namespace {

// Flag of one cell as remapping sees it: failed (e < 0, strictly — GetFailFlagMat,
// strategy.cpp:41, Appendix A Q7) and stuck at zero (v == 0).
__global__ void __launch_bounds__(256)
    k_stuck_zero_counts(const float* __restrict__ e, const float* __restrict__ v, int rows, int cols,
                        unsigned* __restrict__ row_counts, unsigned* __restrict__ col_counts) {
  __shared__ unsigned wsum[4];
  for (int r = blockIdx.x; r < rows; r += gridDim.x) {
    const float* er = e + (int64_t)r * cols;
    const float* vr = v + (int64_t)r * cols;
    unsigned cnt = 0;
    for (int c = threadIdx.x; c < cols; c += 256) {
      if (er[c] < 0.0f && vr[c] == 0.0f) {
        ++cnt;
        // flags are sparse (fault rate), so the column atomics are rare
        if (col_counts) atomicAdd(col_counts + c, 1u);
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0 && row_counts) row_counts[r] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
}

// dst[to[j] * len + c] = src[from[j] * len + c]; one block per moved row,
// 16-B accesses when the rows are 16-B aligned.
__global__ void __launch_bounds__(256)
    k_permute_rows(const float* __restrict__ src, float* __restrict__ dst, int64_t len,
                   const int* __restrict__ to, const int* __restrict__ from, int n, int vec) {
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const float* s = src + (int64_t)from[j] * len;
    float* d = dst + (int64_t)to[j] * len;
    if (vec) {
      const int64_t n4 = len >> 2;
      for (int64_t i = threadIdx.x; i < n4; i += 256)
        reinterpret_cast<float4*>(d)[i] = reinterpret_cast<const float4*>(s)[i];
    } else {
      for (int64_t i = threadIdx.x; i < len; i += 256) d[i] = s[i];
    }
  }
}

// dst[k * cols + to[j]] = src[k * cols + from[j]] for every row k.
__global__ void __launch_bounds__(256)
    k_permute_cols(const float* __restrict__ src, float* __restrict__ dst, int rows, int cols,
                   const int* __restrict__ to, const int* __restrict__ from, int n) {
  const int64_t total = (int64_t)rows * n;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int k = static_cast<int>(idx / n);
    const int j = static_cast<int>(idx - (int64_t)k * n);
    dst[(int64_t)k * cols + to[j]] = src[(int64_t)k * cols + from[j]];
  }
}

__global__ void __launch_bounds__(256)
    k_permute_elems(const float* __restrict__ src, float* __restrict__ dst, const int* __restrict__ to,
                    const int* __restrict__ from, int n) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x)
    dst[to[j]] = src[from[j]];
}

}  // namespace
}  // namespace rram

using namespace rram;

extern "C" {

int rram_stuck_zero_counts(const float* endurance, const float* values, int rows, int cols,
                           unsigned* row_counts, unsigned* col_counts, rram_stream_t s) {
  RRAM_REQUIRE(rows >= 0 && cols >= 0, "stuck_zero_counts: negative size");
  if (rows == 0 || cols == 0) return RRAM_OK;
  RRAM_REQUIRE(endurance && values, "stuck_zero_counts: NULL");
  const int grid = rows < 4096 ? rows : 4096;
  hipLaunchKernelGGL(k_stuck_zero_counts, dim3(grid), dim3(kThreads), 0, as_stream(s), endurance, values, rows,
                     cols, row_counts, col_counts);
  return launch_status("stuck_zero_counts");
}

int rram_permute_rows(const float* src, float* dst, int64_t row_len, const int* to, const int* from, int n,
                      rram_stream_t s) {
  RRAM_REQUIRE(row_len >= 0 && n >= 0, "permute_rows: negative size");
  if (row_len == 0 || n == 0) return RRAM_OK;
  RRAM_REQUIRE(src && dst && to && from && src != dst, "permute_rows: NULL or in place");
  const int vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) == 0 &&
                  (row_len & 3) == 0;
  const int grid = n < 8192 ? n : 8192;
  hipLaunchKernelGGL(k_permute_rows, dim3(grid), dim3(kThreads), 0, as_stream(s), src, dst, row_len, to, from, n,
                     vec);
  return launch_status("permute_rows");
}

int rram_permute_cols(const float* src, float* dst, int rows, int cols, const int* to, const int* from, int n,
                      rram_stream_t s) {
  RRAM_REQUIRE(rows >= 0 && cols >= 0 && n >= 0, "permute_cols: negative size");
  if (rows == 0 || n == 0) return RRAM_OK;
  RRAM_REQUIRE(src && dst && to && from && src != dst, "permute_cols: NULL or in place");
  hipLaunchKernelGGL(k_permute_cols, dim3(stream_blocks((int64_t)rows * n)), dim3(kThreads), 0, as_stream(s), src,
                     dst, rows, cols, to, from, n);
  return launch_status("permute_cols");
}

int rram_permute_elems(const float* src, float* dst, const int* to, const int* from, int n, rram_stream_t s) {
  RRAM_REQUIRE(n >= 0, "permute_elems: negative size");
  if (n == 0) return RRAM_OK;
  RRAM_REQUIRE(src && dst && to && from && src != dst, "permute_elems: NULL or in place");
  hipLaunchKernelGGL(k_permute_elems, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(s), src, dst, to, from,
                     n);
  return launch_status("permute_elems");
}

}  // extern "C"
