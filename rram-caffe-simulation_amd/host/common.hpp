// Runtime context for the host side (replaces the reference's Caffe singleton,
// include/caffe/common.hpp:109-176): one stream, one seed, one reusable device
// workspace, the phase enum and Caffe-style CHECK macros.  Errors are thrown
// as caffe::Error; the C-ABI layer (capi.cpp) turns them into status codes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "rram_kernels.h"

namespace caffe {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define CAFFE_CHECK(cond, msg)                                                      \
  do {                                                                              \
    if (!(cond)) {                                                                  \
      std::ostringstream o_;                                                        \
      o_ << __FILE__ << ":" << __LINE__ << " Check failed: " #cond ": " << msg;      \
      throw ::caffe::Error(o_.str());                                               \
    }                                                                               \
  } while (0)

// Kernel status -> exception (Caffe's CUDA_CHECK/CHECK abort; we raise).
#define RRAM_CALL(expr)                                                              \
  do {                                                                               \
    int rc_ = (expr);                                                                \
    if (rc_ != RRAM_OK) {                                                            \
      std::ostringstream o_;                                                         \
      o_ << #expr << " -> " << rc_ << ": " << rram_last_error();                     \
      throw ::caffe::Error(o_.str());                                                \
    }                                                                                \
  } while (0)

#define HIP_CALL(expr)                                                               \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess) throw ::caffe::Error(std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

enum Phase { TRAIN = 0, TEST = 1 };

class Caffe {
 public:
  static Caffe& Get();
  static rram_stream_t stream() { return Get().stream_; }
  static hipStream_t hip_stream() { return reinterpret_cast<hipStream_t>(Get().stream_); }
  static void set_stream(rram_stream_t s) { Get().stream_ = s; }
  static uint64_t seed() { return Get().seed_; }
  static void set_random_seed(uint64_t s) { Get().seed_ = s; }
  // Shared device workspace (split-K partials, conv backward col buffer).
  // Grows monotonically; never shrinks while a net is alive.
  static void* workspace(size_t bytes);
  static size_t workspace_size() { return Get().ws_bytes_; }
  // Bumped whenever a device scratch buffer of the host side (this
  // workspace, a weight pack, an octet companion) is freed: captured graphs
  // hold raw pointers into them and are re-captured when it moves (with the
  // kernel library's rram_scratch_generation).
  static std::atomic<uint64_t>& scratch_gen();
  static void synchronize();
  // Nonzero while a Solver::Step call runs, a fresh value per call: the
  // flipped convolution kernels one iteration's fused update writes
  // (SyncedMemory::wflip) are read by the next iteration's backward only
  // within the call that wrote them -- no caller code runs between the two
  // but the gradient-sync hooks, which write diffs only.
  static uint64_t step_epoch() { return Get().epoch_; }
  static void set_step_epoch(uint64_t e) { Get().epoch_ = e; }

 private:
  Caffe() = default;
  rram_stream_t stream_ = nullptr;
  uint64_t seed_ = 1701;
  uint64_t epoch_ = 0;
  void* ws_ = nullptr;
  size_t ws_bytes_ = 0;
};

// the working stream is inside a hipGraph capture (relaxed mode: the query is allowed)
inline bool stream_capturing() {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  HIP_CALL(hipStreamIsCapturing(Caffe::hip_stream(), &st));
  return st == hipStreamCaptureStatusActive;
}

}  // namespace caffe
