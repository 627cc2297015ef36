// Multi-GPU in the C++ host: the reference's P2PSync (include/caffe/parallel.hpp,
// src/caffe/parallel.cpp:201-437; entry tools/caffe.cpp:247-249
// `P2PSync<float> sync(solver, NULL, param); sync.Run(gpus)`) rebuilt for one
// process per GPU over RCCL (xGMI), instead of one thread per GPU with a
// peer-to-peer tree.
//
//   Comm           one RCCL communicator (ncclCommInitRank from a unique id the
//                  caller distributes: a file, MPI, torch's store ...)
//   P2PSync<Dtype> the solver hooks: on_start broadcasts the flat parameter
//                  buffer from rank 0 (parallel.cpp:286-322), on_gradients_ready
//                  sum-all-reduces the flat gradient buffer and scales it by
//                  1/N (parallel.cpp:324-380, :377) -- optionally as per-layer
//                  buckets started from the backward hook on a collective
//                  stream while earlier layers are still in backward.
//
// Every learnable param is aliased into the solver's flat data / diff buffers
// (the GPUParams layout, parallel.cpp:25-115), so one collective covers all
// gradients.  The fault state is replicated with identical seeds on every rank,
// so each rank's Fail() equals the reference's root Fail + broadcast.
#pragma once

#include <memory>
#include <utility>
#include <vector>

#include "solver.hpp"

typedef struct ncclComm* ncclComm_t;

namespace caffe {

class Comm {
 public:
  // id: NCCL_UNIQUE_ID_BYTES (128) bytes from unique_id() on one rank
  Comm(const unsigned char* id, int rank, int world);
  ~Comm();
  static void unique_id(unsigned char* out);  // 128 bytes
  int rank() const { return rank_; }
  int world() const { return world_; }
  ncclComm_t comm() const { return comm_; }
  // in-place sum all-reduce of n floats on stream s (asynchronous)
  void allreduce_f32(float* buf, int64_t n, hipStream_t s);
  void broadcast_f32(float* buf, int64_t n, int root, hipStream_t s);
  // in-place all-reduce of n host doubles (op 0 sum, 1 max); synchronous
  void allreduce_host_f64(double* vals, int n, int op);
  void barrier();

 private:
  ncclComm_t comm_ = nullptr;
  int rank_ = 0, world_ = 1;
  double* dscratch_ = nullptr;
  int dscratch_n_ = 0;
};

// per-layer gradient buckets in backward order (the Python plan_buckets):
// ranges[i] = the [begin, end) flat ranges of layer i's learnable params;
// returns {layer, (begin, end)}: after that layer's Backward the suffix
// [begin, end) is final.  Empty when a layer's ranges are not contiguous.
std::vector<std::pair<int, std::pair<int64_t, int64_t>>> plan_buckets(
    const std::vector<std::vector<std::pair<int64_t, int64_t>>>& ranges, int64_t bucket_elems);

template <typename Dtype>
class P2PSync {
 public:
  // overlap: bucketed all-reduce from the per-layer backward hook (needs
  // iter_size 1; nets whose gradients fit one bucket keep the single
  // all-reduce).  The solver must outlive this object; the destructor
  // detaches the hooks.
  P2PSync(Solver<Dtype>* solver, std::shared_ptr<Comm> comm, double bucket_mb, bool overlap);
  ~P2PSync();
  void on_start();             // broadcast the parameters from rank 0
  void on_gradients_ready();   // all-reduce + 1/N
  void on_layer_backward(int layer);
  long long allreduce_calls() const { return allreduce_calls_; }
  long long bucket_calls() const { return bucket_calls_; }
  int buckets() const { return static_cast<int>(plan_.size()); }
  int64_t params() const { return n_; }

 private:
  Solver<Dtype>* solver_;
  std::shared_ptr<Comm> comm_;
  Dtype* data_ = nullptr;
  Dtype* diff_ = nullptr;
  int64_t n_ = 0;
  bool overlap_ = false;
  std::vector<std::pair<int, std::pair<int64_t, int64_t>>> plan_;
  int64_t reduced_lo_ = 0;   // the gradients at [reduced_lo_, n_) are in flight / done
  bool pending_ = false;
  hipStream_t cstream_ = nullptr;   // collective stream (overlap)
  hipEvent_t ev_bwd_ = nullptr, ev_done_ = nullptr;
  long long allreduce_calls_ = 0, bucket_calls_ = 0;
};

}  // namespace caffe
