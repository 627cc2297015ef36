// P2PSync over RCCL (parallel.hpp).  Reference: src/caffe/parallel.cpp:201-437
// (P2PSync ctor / on_start / on_gradients_ready / Run), tools/caffe.cpp:247-249.
#include "parallel.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>

namespace caffe {

#define NCCL_CALL(expr)                                                                         \
  do {                                                                                          \
    ncclResult_t r_ = (expr);                                                                   \
    if (r_ != ncclSuccess) throw ::caffe::Error(std::string(#expr ": ") + ncclGetErrorString(r_)); \
  } while (0)

static_assert(NCCL_UNIQUE_ID_BYTES == 128, "rram_caffe.h documents 128-byte communicator ids");

void Comm::unique_id(unsigned char* out) {
  ncclUniqueId id;
  NCCL_CALL(ncclGetUniqueId(&id));
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
}

Comm::Comm(const unsigned char* id, int rank, int world) : rank_(rank), world_(world) {
  CAFFE_CHECK(world >= 1 && rank >= 0 && rank < world, "Comm: rank " << rank << " outside world " << world);
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
  NCCL_CALL(ncclCommInitRank(&comm_, world, uid, rank));
}

Comm::~Comm() {
  if (dscratch_) (void)hipFree(dscratch_);
  if (comm_) (void)ncclCommDestroy(comm_);
}

void Comm::allreduce_f32(float* buf, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  NCCL_CALL(ncclAllReduce(buf, buf, static_cast<size_t>(n), ncclFloat32, ncclSum, comm_, s));
}

void Comm::broadcast_f32(float* buf, int64_t n, int root, hipStream_t s) {
  if (n <= 0) return;
  NCCL_CALL(ncclBroadcast(buf, buf, static_cast<size_t>(n), ncclFloat32, root, comm_, s));
}

void Comm::allreduce_host_f64(double* vals, int n, int op) {
  CAFFE_CHECK(n >= 0 && (op == 0 || op == 1), "Comm: bad all-reduce request");
  if (n == 0) return;
  hipStream_t s = Caffe::hip_stream();
  if (n > dscratch_n_) {
    if (dscratch_) {
      HIP_CALL(hipStreamSynchronize(s));
      HIP_CALL(hipFree(dscratch_));
      dscratch_ = nullptr;
    }
    HIP_CALL(hipMalloc(&dscratch_, n * sizeof(double)));
    dscratch_n_ = n;
  }
  HIP_CALL(hipMemcpyAsync(dscratch_, vals, n * sizeof(double), hipMemcpyHostToDevice, s));
  NCCL_CALL(ncclAllReduce(dscratch_, dscratch_, static_cast<size_t>(n), ncclFloat64, op == 0 ? ncclSum : ncclMax,
                          comm_, s));
  HIP_CALL(hipMemcpyAsync(vals, dscratch_, n * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_CALL(hipStreamSynchronize(s));
}

void Comm::barrier() {
  double x = 0.0;
  allreduce_host_f64(&x, 1, 0);
}

std::vector<std::pair<int, std::pair<int64_t, int64_t>>> plan_buckets(
    const std::vector<std::vector<std::pair<int64_t, int64_t>>>& ranges, int64_t bucket_elems) {
  std::vector<std::pair<int, std::pair<int64_t, int64_t>>> plan;
  // the suffix property needs the layers' ranges to tile the buffer in layer order
  int64_t next = 0;
  for (const auto& rs : ranges)
    for (const auto& r : rs) {
      if (r.first != next) return {};
      next = r.second;
    }
  int64_t hi = -1, lo = -1;
  for (int i = static_cast<int>(ranges.size()) - 1; i >= 0; --i) {
    const auto& rs = ranges[i];
    if (rs.empty()) continue;
    int64_t b = rs.front().first, e = rs.front().second;
    for (const auto& r : rs) {
      b = std::min(b, r.first);
      e = std::max(e, r.second);
    }
    if (hi < 0) hi = e;
    lo = lo < 0 ? b : std::min(lo, b);
    if (hi - lo >= bucket_elems && i > 0) {
      plan.push_back({i, {lo, hi}});
      hi = lo;
      lo = -1;
    }
  }
  return plan;
}

template <typename Dtype>
P2PSync<Dtype>::P2PSync(Solver<Dtype>* solver, std::shared_ptr<Comm> comm, double bucket_mb, bool overlap)
    : solver_(solver), comm_(std::move(comm)) {
  static_assert(sizeof(Dtype) == 4, "float gradients");
  CAFFE_CHECK(solver_ && comm_, "P2PSync: NULL solver / communicator");
  Net<Dtype>* net = solver_->net().get();
  n_ = net->flat_param_count();
  data_ = solver_->flat_data();
  diff_ = solver_->flat_diff();
  const auto& lp = net->learnable_params();
  // the solver's flat buffers (GPUParams): every learnable param must live in
  // them at its offset, as Net::alias_flat_params left it
  bool aliased = data_ != nullptr && n_ > 0;
  int64_t off = 0;
  for (auto* p : lp) {
    if (!aliased) break;
    aliased = p->gpu_data() == data_ + off && p->gpu_diff() == diff_ + off;
    off += p->count();
  }
  CAFFE_CHECK(aliased || n_ == 0,
              "P2PSync: the solver's params are not aliased into its flat buffers (flat_params: false, or re-aliased)");
  reduced_lo_ = n_;
  const int iter_size = static_cast<int>(solver_->param().integer("iter_size", 1));
  overlap_ = overlap && comm_->world() > 1 && iter_size == 1 && n_ > 0;
  if (overlap_) {
    std::vector<std::vector<std::pair<int64_t, int64_t>>> ranges(net->layers().size());
    for (size_t i = 0; i < net->layers().size(); ++i)
      for (auto& b : net->layers()[i]->blobs()) {
        const Dtype* d = b->gpu_data();
        if (d >= data_ && d < data_ + n_) ranges[i].push_back({d - data_, d - data_ + b->count()});
      }
    const int64_t elems = static_cast<int64_t>(bucket_mb * (1 << 20)) / static_cast<int64_t>(sizeof(Dtype));
    plan_ = plan_buckets(ranges, std::max<int64_t>(1, elems));
    overlap_ = !plan_.empty();
  }
  if (overlap_) {
    HIP_CALL(hipStreamCreateWithFlags(&cstream_, hipStreamNonBlocking));
    HIP_CALL(hipEventCreateWithFlags(&ev_bwd_, hipEventDisableTiming));
    HIP_CALL(hipEventCreateWithFlags(&ev_done_, hipEventDisableTiming));
    net->on_backward_layer = [this](int i) { on_layer_backward(i); };
  }
  solver_->on_gradients_ready = [this] { on_gradients_ready(); };
  on_start();
}

template <typename Dtype>
P2PSync<Dtype>::~P2PSync() {
  solver_->on_gradients_ready = nullptr;
  if (overlap_) solver_->net()->on_backward_layer = nullptr;
  if (cstream_) {
    (void)hipStreamSynchronize(cstream_);
    (void)hipStreamDestroy(cstream_);
  }
  if (ev_bwd_) (void)hipEventDestroy(ev_bwd_);
  if (ev_done_) (void)hipEventDestroy(ev_done_);
}

// parallel.cpp:286-322: the root's parameters reach every solver before the
// first iteration (here a broadcast of the flat data buffer from rank 0)
template <typename Dtype>
void P2PSync<Dtype>::on_start() {
  if (comm_->world() > 1) comm_->broadcast_f32(reinterpret_cast<float*>(data_), n_, 0, Caffe::hip_stream());
  HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
}

template <typename Dtype>
void P2PSync<Dtype>::on_layer_backward(int layer) {
  for (const auto& b : plan_) {
    if (b.first != layer) continue;
    // the gradients of layers >= `layer` are final: reduce them on the
    // collective stream while backward continues on the working stream
    HIP_CALL(hipEventRecord(ev_bwd_, Caffe::hip_stream()));
    HIP_CALL(hipStreamWaitEvent(cstream_, ev_bwd_, 0));
    comm_->allreduce_f32(reinterpret_cast<float*>(diff_) + b.second.first, b.second.second - b.second.first, cstream_);
    reduced_lo_ = b.second.first;
    pending_ = true;
    ++bucket_calls_;
  }
}

// parallel.cpp:324-380: sum the gradients of every solver, scale by 1/N (:377)
template <typename Dtype>
void P2PSync<Dtype>::on_gradients_ready() {
  hipStream_t s = Caffe::hip_stream();
  float* g = reinterpret_cast<float*>(diff_);
  if (overlap_) {
    HIP_CALL(hipEventRecord(ev_bwd_, s));
    HIP_CALL(hipStreamWaitEvent(cstream_, ev_bwd_, 0));
    if (reduced_lo_ > 0) {
      comm_->allreduce_f32(g, reduced_lo_, cstream_);
      ++bucket_calls_;
    }
    HIP_CALL(hipEventRecord(ev_done_, cstream_));
    HIP_CALL(hipStreamWaitEvent(s, ev_done_, 0));   // the update waits for the collective stream
    reduced_lo_ = n_;
    pending_ = false;
  } else {
    comm_->allreduce_f32(g, n_, s);   // world 1 included: the collective path N > 1 takes
  }
  if (comm_->world() > 1) RRAM_CALL(rram_scal(n_, 1.0f / static_cast<float>(comm_->world()), g, Caffe::stream()));
  ++allreduce_calls_;
}

template class P2PSync<float>;

}  // namespace caffe
