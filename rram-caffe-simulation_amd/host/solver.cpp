#include "solver.hpp"

#include "hdf5.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <set>
#include <sstream>

namespace caffe {

GraphStream::~GraphStream() {
  if (own_) {
    (void)hipStreamSynchronize(own_);
    (void)hipStreamDestroy(own_);
  }
  if (ev_in_) (void)hipEventDestroy(ev_in_);
  if (ev_out_) (void)hipEventDestroy(ev_out_);
}

void GraphStream::enter() {
  if (Caffe::hip_stream() != nullptr) return;
  if (!own_) {
    HIP_CALL(hipStreamCreateWithFlags(&own_, hipStreamNonBlocking));
    HIP_CALL(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming));
    HIP_CALL(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
  }
  HIP_CALL(hipEventRecord(ev_in_, nullptr));
  HIP_CALL(hipStreamWaitEvent(own_, ev_in_, 0));
  Caffe::set_stream(reinterpret_cast<rram_stream_t>(own_));
  active_ = true;
}

void GraphStream::leave() {
  if (!active_) return;
  active_ = false;
  Caffe::set_stream(nullptr);
  // no throw from a destructor path: a failed record / wait surfaces at the
  // caller's next synchronisation
  if (hipEventRecord(ev_out_, own_) == hipSuccess) (void)hipStreamWaitEvent(nullptr, ev_out_, 0);
}

// ============================================================ FailureMaker
template <typename Dtype>
FailureMaker<Dtype>::~FailureMaker() {
  if (d_counts_) (void)hipFree(d_counts_);
}

template <typename Dtype>
std::shared_ptr<FailureMaker<Dtype>> FailureMaker<Dtype>::CreateMaker(const Msg& param,
                                                                      std::shared_ptr<Net<Dtype>> net) {
  const std::string type = param.str("type", "gaussian");
  if (type == "gaussian") return std::make_shared<GaussianFailureMaker<Dtype>>(param, net);
  CAFFE_CHECK(type != "uniform", "failure_pattern type 'uniform' is declared in caffe.proto but not implemented "
                                 "by the reference either (Appendix A Q13)");
  return nullptr;
}

template <typename Dtype>
std::vector<Blob<Dtype>*> FailureMaker<Dtype>::fail_iterations() {
  std::vector<Blob<Dtype>*> v;
  for (auto& b : fail_iterations_) v.push_back(b.get());
  return v;
}

template <typename Dtype>
std::vector<unsigned long long> FailureMaker<Dtype>::broken_counts() {
  std::vector<unsigned long long> h(fail_iterations_.size(), 0);
  if (d_counts_ && !h.empty()) {
    HIP_CALL(hipMemcpyAsync(h.data(), d_counts_, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                            Caffe::hip_stream()));
    HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
  }
  return h;
}

// failure_maker.cpp:5-52
template <typename Dtype>
GaussianFailureMaker<Dtype>::GaussianFailureMaker(const Msg& param, std::shared_ptr<Net<Dtype>> net)
    : FailureMaker<Dtype>(param) {
  this->net_ = net;
  long long neg = 10, zero = 20, pos = 10;  // defaults (failure_maker.cpp:17-21)
  if (const Msg* fp = param.sub("failure_prob")) {
    neg = fp->integer("neg", 10);
    zero = fp->integer("zero", 20);
    pos = fp->integer("pos", 10);
    CAFFE_CHECK(neg >= 0, "Probability for failure to -1 must be greater or equal than 0");
    CAFFE_CHECK(zero >= 0, "Probability for failure to 0 must be greater or equal than 0");
    CAFFE_CHECK(pos >= 0, "Probability for failure to 1 must be greater or equal than 0");
  }
  const long long sum = neg + zero + pos;
  CAFFE_CHECK(sum > 0, "failure_prob entries sum to 0");
  const uint64_t thr_neg = ((uint64_t)neg * (1ull << 32) + sum - 1) / sum;
  const uint64_t thr_zero = ((uint64_t)(neg + zero) * (1ull << 32) + sum - 1) / sum;
  const float mean = static_cast<float>(param.num("mean", 10000));  // caffe.proto:255 defaults
  const float std = static_cast<float>(param.num("std", 100));
  decrement = static_cast<float>(param.num("rram_decrement", 100.0));
  const auto& fps = net->failure_learnable_params();
  for (size_t i = 0; i < fps.size(); ++i) {
    auto b = std::make_unique<Blob<Dtype>>(fps[i]->shape());
    RRAM_CALL(rram_fault_init(b->mutable_gpu_data(), b->mutable_gpu_diff(), b->count(), mean, std, thr_neg,
                              thr_zero, Caffe::seed(), 0u, static_cast<uint32_t>(i), Caffe::stream()));
    this->fail_iterations_.push_back(std::move(b));
  }
  if (!fps.empty()) {
    HIP_CALL(hipMalloc(&this->d_counts_, fps.size() * sizeof(unsigned long long)));
    HIP_CALL(hipMemsetAsync(this->d_counts_, 0, fps.size() * sizeof(unsigned long long), Caffe::hip_stream()));
  }
}

// failure_maker.cu:44-58 — all blobs in batched launches of <= RRAM_MAX_SEGS
template <typename Dtype>
void GaussianFailureMaker<Dtype>::Fail_gpu(int /*iter*/) {
  const auto& fps = this->net_->failure_learnable_params();
  const size_t n = fps.size();
  if (!n) return;
  HIP_CALL(hipMemsetAsync(this->d_counts_, 0, n * sizeof(unsigned long long), Caffe::hip_stream()));
  std::vector<rram_fail_seg> segs(n);
  for (size_t i = 0; i < n; ++i) {
    auto& fi = this->fail_iterations_[i];
    segs[i] = rram_fail_seg{fps[i]->gpu_diff(), fps[i]->mutable_gpu_data(), fi->mutable_gpu_data(), fi->gpu_diff(),
                            fps[i]->count()};
  }
  for (size_t s = 0; s < n; s += RRAM_MAX_SEGS) {
    const int k = static_cast<int>(std::min<size_t>(RRAM_MAX_SEGS, n - s));
    RRAM_CALL(rram_fail_apply_batched(segs.data() + s, k, decrement, epsilon, this->d_counts_ + s, Caffe::stream()));
  }
}

// ============================================================ strategies
template <typename Dtype>
std::shared_ptr<FailureStrategy<Dtype>> FailureStrategy<Dtype>::CreateStrategy(
    const Msg& param, std::shared_ptr<FailureMaker<Dtype>> fm, std::shared_ptr<Net<Dtype>> net,
    const Solver<Dtype>* s) {
  const std::string type = param.str("type");
  if (type == "threshold") {
    auto p = std::make_shared<ThresholdFailureStrategy<Dtype>>(param, fm, net, s);
    p->reference_lr_index = param.boolean("rram_reference_lr_index", false);
    return p;
  }
  if (type == "remapping") {
    auto p = std::make_shared<RemappingFailureStrategy<Dtype>>(param, fm, net, s);
    p->reference_compat = param.boolean("rram_reference_compat", false);
    return p;
  }
  if (type == "genetic") {
    auto p = std::make_shared<GeneticFailureStrategy<Dtype>>(param, fm, net, s);
    p->reference_compat = param.boolean("rram_reference_compat", false);
    return p;
  }
  throw Error("No strategy named `" + type + "` exists.");
}

template <typename Dtype>
float ThresholdFailureStrategy<Dtype>::threshold_for(int i) const {
  const auto& lr = this->net_->params_lr();
  const int idx = reference_lr_index ? i : this->net_->failure_learnable_param_ids()[i];
  CAFFE_CHECK(idx < (int)lr.size(), "params_lr index out of range");
  // strategy.cpp:13-14: rate = params_lr * lr (fp32), threshold = threshold_ * rate
  const float rate = static_cast<float>(lr[idx]) * static_cast<float>(this->solver_->GetLearningRate());
  return threshold() * rate;
}

// strategy.cpp:7-33, on the device (no D2H/H2D round trip)
template <typename Dtype>
void ThresholdFailureStrategy<Dtype>::Apply() {
  const auto& fps = this->net_->failure_learnable_params();
  for (size_t i = 0; i < fps.size(); ++i)
    RRAM_CALL(rram_threshold_strategy(fps[i]->mutable_gpu_diff(), fps[i]->count(), threshold_for((int)i), nullptr,
                                      Caffe::stream()));
}

// ================================================================ Solver
static Msg load_net_param(const Msg& sp, const Msg* net_param) {
  if (net_param) return *net_param;
  if (const Msg* np = sp.sub("net_param")) return *np;
  if (const Msg* np = sp.sub("train_net_param")) return *np;
  std::string f = sp.str("net", sp.str("train_net", ""));
  CAFFE_CHECK(!f.empty(), "solver: no net given (net / net_param / train_net)");
  return parse_prototxt_file(f);
}

template <typename Dtype>
Solver<Dtype>::Solver(const Msg& sp, const Msg* net_param, const Msg& options) : param_(sp), options_(options) {
  if (sp.has("random_seed") && sp.integer("random_seed") >= 0)
    Caffe::set_random_seed(static_cast<uint64_t>(sp.integer("random_seed")));
  fused_update_ = options.boolean("fused_update", false);
  flip_cache_ = options.boolean("conv_flip_cache", true);
  const Msg np = load_net_param(sp, net_param);
  net_ = std::make_shared<Net<Dtype>>(np, TRAIN, options);
  // solver.cpp:132-148: fault maker and strategies on the root solver
  if (const Msg* fp = sp.sub("failure_pattern")) InitFailurePattern(*fp);
  for (auto* st : sp.subs("failure_strategy")) {
    auto p = FailureStrategy<Dtype>::CreateStrategy(*st, fmaker_, net_, this);
    strategys_.push_back(p);
  }
  // test nets (solver.cpp:155-230): test_net_param / test_net, else the train net in TEST phase
  std::vector<Msg> tnp;
  for (auto* t : sp.subs("test_net_param")) tnp.push_back(*t);
  for (auto& f : sp.strs("test_net")) tnp.push_back(parse_prototxt_file(f));
  if (tnp.empty() && sp.count("test_iter") > 0) tnp.push_back(np);
  for (auto& t : tnp) {
    test_nets_.push_back(std::make_shared<Net<Dtype>>(t, TEST, options));
    test_nets_.back()->ShareTrainedLayersWith(net_.get());
  }
  for (auto* p : net_->learnable_params()) {
    history_.push_back(std::make_unique<Blob<Dtype>>(p->shape()));
    HIP_CALL(hipMemsetAsync(history_.back()->mutable_gpu_data(), 0, p->count() * sizeof(Dtype), Caffe::hip_stream()));
    temp_.push_back(std::make_unique<Blob<Dtype>>(p->shape()));
  }
  CAFFE_CHECK(param_.str("type", "SGD") == "SGD" && param_.str("solver_type", "SGD") == "SGD",
              "only the SGD solver is part of this build (SURVEY.md §2.1)");
  const int64_t nflat = net_->flat_param_count();
  if (nflat > 0 && options.boolean("flat_params", true)) {
    HIP_CALL(hipMalloc(&flat_, 2 * nflat * sizeof(Dtype)));
    net_->alias_flat_params(static_cast<Dtype*>(flat_), static_cast<Dtype*>(flat_) + nflat);
  }
}

template <typename Dtype>
Solver<Dtype>::~Solver() {
  drop_graphs();
  if (flat_) {
    (void)hipStreamSynchronize(Caffe::hip_stream());
    (void)hipFree(flat_);
  }
}

// solver.cpp:14-23
template <typename Dtype>
void Solver<Dtype>::InitFailurePattern(const Msg& fp) {
  if (fp.str("type", "gaussian") == "none") return;
  fmaker_ = FailureMaker<Dtype>::CreateMaker(fp, net_);
}

// sgd_solver.cpp GetLearningRate
template <typename Dtype>
Dtype Solver<Dtype>::GetLearningRate() const {
  // sgd_solver.cpp:27-63.  base_lr / gamma / power are `optional float` in
  // caffe.proto, so they are rounded to fp32 first; the fp32 sub-expressions
  // (1 + gamma*iter, 1 - iter/max_iter) stay fp32 and pow/exp run in double
  // (the C library ::pow the unqualified calls bind to), as in the reference.
  const std::string policy = param_.str("lr_policy", "fixed");
  const float base = static_cast<float>(param_.num("base_lr", 0.01));
  const float gamma = static_cast<float>(param_.num("gamma", 0.0));
  const float power = static_cast<float>(param_.num("power", 0.0));
  const int it = iter_;
  if (policy == "fixed") return (Dtype)base;
  if (policy == "step") {
    const int step = it / (int)param_.integer("stepsize", 1);
    return (Dtype)((double)base * std::pow((double)gamma, (double)step));
  }
  if (policy == "exp") return (Dtype)((double)base * std::pow((double)gamma, (double)it));
  if (policy == "inv") {
    const float b = 1.0f + gamma * static_cast<float>(it);
    return (Dtype)((double)base * std::pow((double)b, (double)-power));
  }
  if (policy == "multistep") {
    auto sv = param_.nums("stepvalue");
    int step = 0;
    while (step < (int)sv.size() && it >= sv[step]) ++step;
    return (Dtype)((double)base * std::pow((double)gamma, (double)step));
  }
  if (policy == "poly") {
    const float b = 1.0f - static_cast<float>(it) / static_cast<float>(param_.integer("max_iter", 1));
    return (Dtype)((double)base * std::pow((double)b, (double)power));
  }
  if (policy == "sigmoid") {
    const float x = -gamma * (static_cast<float>(it) - static_cast<float>(param_.integer("stepsize", 1)));
    return (Dtype)((double)base * (1.0 / (1.0 + std::exp((double)x))));
  }
  throw Error("Unknown learning rate policy: " + policy);
}

template <typename Dtype>
void Solver<Dtype>::ClipGradients() {
  const double clip = param_.num("clip_gradients", -1.0);
  if (clip < 0) return;
  const auto& ps = net_->learnable_params();
  double sumsq = 0;
  Dtype* dtmp = nullptr;
  HIP_CALL(hipMallocAsync(reinterpret_cast<void**>(&dtmp), sizeof(Dtype), Caffe::hip_stream()));
  for (auto* p : ps) {
    Dtype h = 0;
    RRAM_CALL(rram_dot(p->count(), p->gpu_diff(), p->gpu_diff(), dtmp, Caffe::stream()));
    HIP_CALL(hipMemcpyAsync(&h, dtmp, sizeof(Dtype), hipMemcpyDeviceToHost, Caffe::hip_stream()));
    HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
    sumsq += h;
  }
  HIP_CALL(hipFreeAsync(dtmp, Caffe::hip_stream()));
  const double l2 = std::sqrt(sumsq);
  if (l2 > clip)
    for (auto* p : ps) RRAM_CALL(rram_scal(p->count(), (Dtype)(clip / l2), p->mutable_gpu_diff(), Caffe::stream()));
}

// sgd_solver.cpp:148-214
template <typename Dtype>
void Solver<Dtype>::Regularize(int id) {
  auto* p = net_->learnable_params()[id];
  const Dtype decay = (Dtype)param_.num("weight_decay", 0.0) * net_->params_weight_decay()[id];
  if (decay == Dtype(0)) return;
  const std::string rt = param_.str("regularization_type", "L2");
  if (rt == "L2") {
    RRAM_CALL(rram_axpy(p->count(), decay, p->gpu_data(), p->mutable_gpu_diff(), Caffe::stream()));
  } else if (rt == "L1") {
    RRAM_CALL(rram_sign(p->count(), p->gpu_data(), temp_[id]->mutable_gpu_data(), Caffe::stream()));
    RRAM_CALL(rram_axpy(p->count(), decay, temp_[id]->gpu_data(), p->mutable_gpu_diff(), Caffe::stream()));
  } else {
    throw Error("Unknown regularization type: " + rt);
  }
}

// sgd_solver.cpp:216-247 (GPU branch: SGDUpdate kernel)
template <typename Dtype>
void Solver<Dtype>::ComputeUpdateValue(int id, Dtype rate) {
  auto* p = net_->learnable_params()[id];
  const Dtype local = rate * net_->params_lr()[id];
  RRAM_CALL(rram_sgd_update(p->mutable_gpu_diff(), history_[id]->mutable_gpu_data(), p->count(),
                            (Dtype)param_.num("momentum", 0.0), local, Caffe::stream()));
}

// sgd_solver.cpp:101-116 (Normalize for iter_size > 1 folded into a scale)
template <typename Dtype>
void Solver<Dtype>::ComputeUpdate() {
  const Dtype rate = GetLearningRate();
  ClipGradients();
  const int iter_size = (int)param_.integer("iter_size", 1);
  const auto& ps = net_->learnable_params();
  for (int i = 0; i < (int)ps.size(); ++i) {
    if (iter_size > 1) RRAM_CALL(rram_scal(ps[i]->count(), Dtype(1) / iter_size, ps[i]->mutable_gpu_diff(), Caffe::stream()));
    Regularize(i);
    ComputeUpdateValue(i, rate);
  }
}

// solver.cpp:25-33
template <typename Dtype>
void Solver<Dtype>::ApplyStrategy() {
  if (!fmaker_) return;
  for (auto& s : strategys_) s->Apply();
}

template <typename Dtype>
void Solver<Dtype>::ApplyUpdate() {
  net_->Update();
}

// Regularize(L2) + SGDUpdate + threshold + Update + Fail in
// one HBM pass per blob.  Same arithmetic sequence as the separate kernels.
template <typename Dtype>
void Solver<Dtype>::FusedTail() {
  const Dtype rate = GetLearningRate();
  const auto& ps = net_->learnable_params();
  const auto& fids = net_->failure_learnable_param_ids();
  const Dtype mom = (Dtype)param_.num("momentum", 0.0);
  const Dtype wd = (Dtype)param_.num("weight_decay", 0.0);
  // only reached when every configured strategy is a ThresholdFailureStrategy
  // and there is at most one (Step's can_fuse); anything else runs unfused
  ThresholdFailureStrategy<Dtype>* thr =
      strategys_.empty() ? nullptr : dynamic_cast<ThresholdFailureStrategy<Dtype>*>(strategys_[0].get());
  auto* gm = dynamic_cast<GaussianFailureMaker<Dtype>*>(fmaker_.get());
  std::vector<Blob<Dtype>*> fi = fmaker_ ? fmaker_->fail_iterations() : std::vector<Blob<Dtype>*>();
  // (cleared with the parameter diffs at the iteration's start, Step)
  unsigned long long* counts = fmaker_ ? fmaker_->device_counts() : nullptr;
  // one launch for all blobs (rram_fused_update_fail_batched; a net with more
  // learnable blobs than one launch takes goes one launch per RRAM_MAX_SEGS)
  // The flipped kernels of the convolutions whose stride-1 data gradient
  // reads them (Layer::flip_geometry) come out of the same pass, for the next
  // iteration's backward within this Step call (Caffe::step_epoch); not while
  // a graph is captured.  They replace a flip launch per layer per iteration.
  const uint64_t epoch = Caffe::step_epoch();
  struct Flip {
    SyncedMemory* m;
    int g, ci, co, t;
  };
  std::vector<Flip> flips;
  if (flip_cache_ && epoch != 0 && !stream_capturing())
    for (const auto& l : net_->layers()) {
      Flip f{};
      if (!l->blobs().empty() && l->flip_geometry(&f.g, &f.ci, &f.co, &f.t)) {
        f.m = l->blobs()[0]->data().get();
        flips.push_back(f);
      }
    }
  std::vector<SyncedMemory*> flipped;
  std::vector<rram_update_seg> segs;
  for (int i = 0; i < (int)ps.size(); ++i) {
    int f = -1;
    for (int k = 0; k < (int)fids.size(); ++k)
      if (fids[k] == i) f = k;
    const bool faulty = gm && f >= 0;
    rram_update_seg sg{};
    sg.w = ps[i]->mutable_gpu_data();
    sg.g = ps[i]->mutable_gpu_diff();
    sg.h = history_[i]->mutable_gpu_data();
    sg.endurance = faulty ? fi[f]->mutable_gpu_data() : nullptr;
    sg.values = faulty ? fi[f]->gpu_diff() : nullptr;
    sg.n = ps[i]->count();
    sg.decay = wd * net_->params_weight_decay()[i];
    sg.local_rate = rate * net_->params_lr()[i];
    sg.apply_thr = (faulty && thr) ? 1 : 0;
    sg.thr = (faulty && thr) ? thr->threshold_for(f) : 0.0f;
    sg.broken_count = (faulty && counts) ? counts + f : nullptr;
    for (const Flip& fl : flips)
      if (fl.m == ps[i]->data().get() && (int64_t)fl.g * fl.ci * fl.co * fl.t == sg.n) {
        sg.w_flip = static_cast<float*>(fl.m->wflip(static_cast<size_t>(sg.n) * sizeof(Dtype)));
        sg.flip_groups = fl.g;
        sg.flip_cin = fl.ci;
        sg.flip_cout = fl.co;
        sg.flip_taps = fl.t;
        flipped.push_back(fl.m);
        break;
      }
    segs.push_back(sg);
  }
  for (size_t b = 0; b < segs.size(); b += RRAM_MAX_SEGS)
    RRAM_CALL(rram_fused_update_fail_batched(segs.data() + b, (int)std::min<size_t>(RRAM_MAX_SEGS, segs.size() - b), mom,
                                             gm ? gm->decrement : 100.0f, gm ? gm->epsilon : 1e-20f, Caffe::stream()));
  for (SyncedMemory* m : flipped) m->set_wflip_valid(epoch);
}

template <typename Dtype>
void Solver<Dtype>::drop_graphs() {
  for (int k = 0; k < 2; ++k) {
    if (gx_[k]) (void)hipGraphExecDestroy(gx_[k]);
    if (gg_[k]) (void)hipGraphDestroy(gg_[k]);
    gx_[k] = nullptr;
    gg_[k] = nullptr;
  }
  graph_warm_ = false;
  graph_ptrs_.clear();
}

template <typename Dtype>
void Solver<Dtype>::set_graph(bool on) {
  if (on)
    for (const auto& l : net_->layers()) {
      const std::string t = l->type();
      CAFFE_CHECK(t != "Dropout" && t != "HDF5Data",
                  "Solver graph replay: " << l->name() << " (" << t << ") changes per iteration on the host");
    }
  else
    drop_graphs();
  graph_ = on;
}

// the device pointers a captured iteration depends on
template <typename Dtype>
std::vector<const void*> Solver<Dtype>::graph_key() const {
  std::vector<const void*> k;
  for (const auto& b : net_->blobs()) {
    k.push_back(b->data()->gpu_data());
    k.push_back(b->diff()->gpu_data());
  }
  for (auto* p : net_->learnable_params()) {
    k.push_back(p->data()->gpu_data());
    k.push_back(p->diff()->gpu_data());
  }
  for (const auto& h : history_) k.push_back(h->data()->gpu_data());
  if (fmaker_) {
    for (auto* b : fmaker_->fail_iterations()) {
      k.push_back(b->data()->gpu_data());
      k.push_back(b->diff()->gpu_data());
    }
    k.push_back(fmaker_->device_counts());
  }
  k.push_back(Caffe::hip_stream());
  // the scratch the captured launches read and write (workspace, packs,
  // split-K partials, gather tables): eager work between replays may have
  // reallocated it (a larger test batch, another net on this thread)
  k.push_back(reinterpret_cast<const void*>(static_cast<uintptr_t>(Caffe::scratch_gen().load())));
  k.push_back(reinterpret_cast<const void*>(static_cast<uintptr_t>(rram_scratch_generation())));
  return k;
}

// graph k (0: clear + forward + backward, 1: the fused tail): captured from
// body() on first use, then launched
template <typename Dtype>
template <typename F>
void Solver<Dtype>::capture_launch(int k, F&& body) {
  hipStream_t st = Caffe::hip_stream();
  if (!gx_[k]) {
    HIP_CALL(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
    try {
      body();
    } catch (...) {
      hipGraph_t g = nullptr;
      (void)hipStreamEndCapture(st, &g);
      if (g) (void)hipGraphDestroy(g);
      throw;
    }
    HIP_CALL(hipStreamEndCapture(st, &gg_[k]));
    HIP_CALL(hipGraphInstantiate(&gx_[k], gg_[k], nullptr, nullptr, 0));
  }
  HIP_CALL(hipGraphLaunch(gx_[k], st));
}

// solver.cpp:237-325 (fork order: ComputeUpdate -> ApplyStrategy -> ApplyUpdate -> Fail)
template <typename Dtype>
void Solver<Dtype>::Step(int iters) {
  // a fresh Caffe::step_epoch for this call (the flipped-kernel companions
  // written by its updates are read only within it), 0 again on the way out
  struct EpochScope {
    EpochScope() {
      static std::atomic<uint64_t> next{0};
      Caffe::set_step_epoch(++next);
    }
    ~EpochScope() { Caffe::set_step_epoch(0); }
  } epoch_scope;
  const int stop = iter_ + iters;
  const int display = (int)param_.integer("display", 0);
  const int test_interval = (int)param_.integer("test_interval", 0);
  const int average_loss = (int)param_.integer("average_loss", 1);
  const int iter_size = (int)param_.integer("iter_size", 1);
  // The fused tail folds Regularize(L2) + SGDUpdate + threshold + Update +
  // Fail into one pass; remapping / genetic strategies (and more than one
  // strategy) need the reference order ComputeUpdate -> ApplyStrategy ->
  // ApplyUpdate -> Fail (solver.cpp:300-305), so they disable fusion.
  bool fusable_strategies = strategys_.size() <= 1;
  for (auto& st : strategys_)
    fusable_strategies = fusable_strategies && dynamic_cast<ThresholdFailureStrategy<Dtype>*>(st.get()) != nullptr;
  const bool can_fuse = fused_update_ && fusable_strategies && param_.num("clip_gradients", -1.0) < 0 &&
                        iter_size == 1 && param_.str("regularization_type", "L2") == "L2";
  // the fused tail's Fail counters are cleared with the parameter diffs (one launch)
  unsigned long long* fail_counts = can_fuse && fmaker_ ? fmaker_->device_counts() : nullptr;
  const int64_t n_fail_counts = fail_counts ? static_cast<int64_t>(fmaker_->fail_iterations().size()) : 0;
  while (iter_ < stop) {
    const bool test_now =
        test_interval && iter_ % test_interval == 0 && (iter_ > 0 || param_.boolean("test_initialization", true));
    const bool disp = display && iter_ % display == 0;
    // (a learning rate that moves every iteration, e.g. lr_policy "inv",
    // keeps the eager path: a graph is only worth its capture when replayed)
    const Dtype rate_now = graph_ ? GetLearningRate() : Dtype(0);
    const bool rate_stable = rate_now == graph_prev_rate_;
    graph_prev_rate_ = rate_now;
    if (graph_ && rate_stable && can_fuse && !test_now && !disp && average_loss <= 1 && !net_->on_backward_layer &&
        !net_->timing_on()) {
      // the first such iteration runs eager (workspaces and scratch buffers
      // get allocated on the section's stream), the next one captures
      const Dtype rate = rate_now;
      bool warm = graph_warm_;
      net_->set_iter((uint64_t)iter_);
      {
        GraphStreamScope sc(gstream_);
        // a new rate recaptures now; a key changed since the capture -- or
        // since the eager warm-up iteration -- means freed / reallocated
        // scratch: this iteration then runs eager again (rebuilding tables,
        // growing buffers outside any capture) and the next one captures
        const bool moved = warm && graph_key() != graph_ptrs_;
        if (gx_[0] && (rate != graph_rate_ || moved)) drop_graphs();
        if (moved) warm = false;
        auto fb = [&] {
          net_->ClearParamDiffs(fail_counts, n_fail_counts);
          net_->Forward(false);
          net_->Backward();
        };
        if (warm)
          capture_launch(0, fb);
        else
          fb();
      }
      if (on_gradients_ready) on_gradients_ready();  // on the caller's stream, after the section
      {
        GraphStreamScope sc(gstream_);
        if (warm) {
          capture_launch(1, [&] { FusedTail(); });
          graph_rate_ = rate;
          // a replayed update rewrote the weights without FusedTail's host
          // side: no flipped kernel written before it is current
          for (auto* p : net_->learnable_params()) p->data()->drop_wflip();
        } else {
          FusedTail();
        }
        graph_ptrs_ = graph_key();  // the scratch this iteration ran (or was captured) with
      }
      graph_warm_ = true;
      ++iter_;
      const long long snap = param_.integer("snapshot", 0);
      if (snap && iter_ % snap == 0) Snapshot();
      continue;
    }
    net_->ClearParamDiffs(fail_counts, n_fail_counts);
    if (test_now) TestAll();
    net_->set_iter((uint64_t)iter_);
    Dtype loss = 0;
    for (int i = 0; i < iter_size; ++i) {
      loss += net_->Forward(disp || average_loss > 1);
      net_->Backward();
    }
    loss /= iter_size;
    if (disp || average_loss > 1) {
      if ((int)losses_.size() < average_loss) {
        losses_.push_back(loss);
        smoothed_loss_ = (smoothed_loss_ * (losses_.size() - 1) + loss) / losses_.size();
      } else {
        const int idx = iter_ % average_loss;
        smoothed_loss_ += (loss - losses_[idx]) / average_loss;
        losses_[idx] = loss;
      }
    }
    if (disp) {
      std::ostringstream o;
      o << "Iteration " << iter_ << ", loss = " << smoothed_loss_;
      emit(o.str());
    }
    if (on_gradients_ready) on_gradients_ready();
    if (can_fuse) {
      FusedTail();
    } else {
      ComputeUpdate();
      ApplyStrategy();
      ApplyUpdate();
      Fail(iter_);
    }
    ++iter_;
    const long long snap = param_.integer("snapshot", 0);  // solver.cpp:312-318
    if (snap && iter_ % snap == 0) Snapshot();
  }
}

template <typename Dtype>
void Solver<Dtype>::Solve(const char* resume_file) {
  if (resume_file) {
    emit(std::string("Restoring previous solver status from ") + resume_file);
    Restore(resume_file);
  }
  const int max_iter = (int)param_.integer("max_iter", 0);
  Step(max_iter - iter_);
  // solver.cpp:345-350 (only with a snapshot_prefix: the reference would write
  // "_iter_N.caffemodel" into the working directory without one)
  const long long snap = param_.integer("snapshot", 0);
  if (param_.has("snapshot_prefix") && param_.boolean("snapshot_after_train", true) && (!snap || iter_ % snap != 0))
    Snapshot();
  if (param_.integer("display", 0) && max_iter % std::max<long long>(1, param_.integer("display", 1)) == 0) {
    std::ostringstream o;
    o << "Iteration " << iter_ << ", loss = " << smoothed_loss_;
    emit(o.str());
  }
  const int ti = (int)param_.integer("test_interval", 0);
  if (ti && iter_ % ti == 0) TestAll();
  emit("Optimization Done.");
}

// solver.cpp:461-495 + sgd_solver.cpp:249-305: weights then solver state, as
// binary proto (.caffemodel / .solverstate) or HDF5 (.caffemodel.h5 /
// .solverstate.h5); the fault maps go to <prefix>_iter_N.faultstate either way
template <typename Dtype>
std::string Solver<Dtype>::Snapshot() {
  const std::string fmt = param_.str("snapshot_format", "BINARYPROTO");
  CAFFE_CHECK(fmt == "BINARYPROTO" || fmt == "HDF5", "Unsupported snapshot format " << fmt);
  const bool diff = param_.boolean("snapshot_diff", false);
  std::string state;
  if (fmt == "HDF5") {
    const std::string model = SnapshotFilename(".caffemodel.h5");
    emit("Snapshotting to HDF5 file " + model);
    net_->ToHDF5(model, diff);
    state = SnapshotFilename(".solverstate.h5");
    emit("Snapshotting solver state to HDF5 file " + state);
    h5::Handle f = h5::create_file(state);
    h5::save_int(f.id(), "iter", iter_);
    h5::save_string(f.id(), "learned_net", model);
    h5::save_int(f.id(), "current_step", current_step_);
    h5::Handle hg = h5::create_group(f.id(), "history");
    for (size_t i = 0; i < history_.size(); ++i) {
      const BlobProtoData p = BlobToProto(history_[i].get(), false);
      h5::save_floats(hg.id(), std::to_string(i),
                      std::vector<int64_t>(history_[i]->shape().begin(), history_[i]->shape().end()), p.data.data());
    }
  } else {
    const std::string model = SnapshotFilename(".caffemodel");
    emit("Snapshotting to binary proto file " + model);
    WriteFileBytes(model, SerializeNetParameter(net_->ToProto(diff)));
    SolverStateData st;
    st.iter = iter_;
    st.learned_net = model;
    st.current_step = current_step_;
    for (auto& h : history_) st.history.push_back(BlobToProto(h.get(), false));
    state = SnapshotFilename(".solverstate");
    emit("Snapshotting solver state to binary proto file " + state);
    WriteFileBytes(state, SerializeSolverState(st));
  }
  if (fmaker_) {
    std::vector<BlobProtoData> fs;
    for (auto* b : fmaker_->fail_iterations()) fs.push_back(BlobToProto(b, true));  // data = e, diff = v
    WriteFileBytes(SnapshotFilename(".faultstate"), SerializeBlobProtoVector(fs));
  }
  return state;
}

static bool ends_with(const std::string& s, const std::string& suf) {
  return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

// solver.cpp:520-530 + sgd_solver.cpp:307-351
template <typename Dtype>
void Solver<Dtype>::Restore(const std::string& state_file) {
  std::string fault_file;
  if (ends_with(state_file, ".h5")) {
    h5::Handle f = h5::open_file(state_file);
    iter_ = h5::load_int(f.id(), "iter");
    if (h5::dataset_exists(f.id(), "learned_net")) net_->CopyTrainedLayersFrom(h5::load_string(f.id(), "learned_net"));
    current_step_ = h5::load_int(f.id(), "current_step");
    h5::Handle hg = h5::open_group(f.id(), "history");
    CAFFE_CHECK(h5::num_links(hg.id()) == (int)history_.size(), "Incorrect length of history blobs.");
    for (size_t i = 0; i < history_.size(); ++i) {
      std::vector<int64_t> dims;
      BlobProtoData p;
      p.data = h5::load_floats(hg.id(), std::to_string(i), &dims);
      CAFFE_CHECK((int64_t)p.data.size() == history_[i]->count(), "history blob " << i << ": size mismatch");
      BlobFromProto(history_[i].get(), p);
    }
    if (ends_with(state_file, ".solverstate.h5"))
      fault_file = state_file.substr(0, state_file.size() - 15) + ".faultstate";
  } else {
    const SolverStateData st = ParseSolverState(ReadFileBytes(state_file));
    iter_ = st.iter;
    if (!st.learned_net.empty()) net_->CopyTrainedLayersFrom(st.learned_net);
    current_step_ = st.current_step;
    CAFFE_CHECK(st.history.size() == history_.size(), "Incorrect length of history blobs.");
    for (size_t i = 0; i < history_.size(); ++i) {
      CAFFE_CHECK(ShapeEquals(history_[i]->shape(), st.history[i]), "history blob " << i << ": shape mismatch");
      BlobFromProto(history_[i].get(), st.history[i]);
    }
    if (ends_with(state_file, ".solverstate"))
      fault_file = state_file.substr(0, state_file.size() - 12) + ".faultstate";
  }
  if (fmaker_ && !fault_file.empty()) {
    std::ifstream probe(fault_file, std::ios::binary);
    if (probe.good()) {
      const auto fs = ParseBlobProtoVector(ReadFileBytes(fault_file));
      auto fi = fmaker_->fail_iterations();
      CAFFE_CHECK(fs.size() == fi.size(), "fault state: " << fs.size() << " blobs, net has " << fi.size());
      for (size_t i = 0; i < fi.size(); ++i) {
        CAFFE_CHECK(ShapeEquals(fi[i]->shape(), fs[i]) && !fs[i].diff.empty(), "fault state blob " << i << ": mismatch");
        BlobFromProto(fi[i], fs[i]);
      }
      emit("Restored fault state from " + fault_file);
    }
  }
}

template <typename Dtype>
std::vector<std::vector<Dtype>> Solver<Dtype>::TestAll() {
  std::vector<std::vector<Dtype>> r;
  for (int i = 0; i < (int)test_nets_.size(); ++i) r.push_back(Test(i));
  return r;
}

// solver.cpp:385-458: mean over test_iter of every output element
template <typename Dtype>
std::vector<Dtype> Solver<Dtype>::Test(int id) {
  CAFFE_CHECK(id >= 0 && id < (int)test_nets_.size(), "test net index out of range");
  auto tn = test_nets_[id];
  auto ti = param_.nums("test_iter");
  const int iters = ti.empty() ? 1 : (int)ti[std::min<size_t>(id, ti.size() - 1)];
  std::vector<Dtype> score;
  Dtype loss = 0;
  for (int it = 0; it < iters; ++it) {
    loss += tn->Forward(true);
    int k = 0;
    for (auto* b : tn->output_blobs()) {
      std::vector<Dtype> h(b->count());
      HIP_CALL(hipMemcpyAsync(h.data(), b->gpu_data(), b->count() * sizeof(Dtype), hipMemcpyDeviceToHost,
                              Caffe::hip_stream()));
      HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
      for (Dtype v : h) {
        if (it == 0) score.push_back(v);
        else score[k] += v;
        ++k;
      }
    }
  }
  for (auto& s : score) s /= iters;
  std::ostringstream o;
  o << "Iteration " << iter_ << ", Testing net (#" << id << ")";
  emit(o.str());
  int k = 0;
  for (size_t j = 0; j < tn->output_blobs().size(); ++j) {
    const int bid = tn->output_blob_indices()[j];
    const float lw = tn->blob_loss_weights()[bid];
    for (int64_t e = 0; e < tn->output_blobs()[j]->count(); ++e, ++k) {
      std::ostringstream l;
      l << "    Test net output #" << k << ": " << tn->blob_names()[bid] << " = " << score[k];
      if (lw) l << " (* " << lw << " = " << lw * score[k] << " loss)";
      emit(l.str());
    }
  }
  return score;
}

// ============================================================ MonteCarlo
template <typename Dtype>
MonteCarlo<Dtype>::MonteCarlo(std::shared_ptr<Net<Dtype>> net, const std::vector<rram_inject_cfg>& cfgs,
                              uint64_t seed, int max_maps)
    : net_(net), seed_(seed), max_maps_(max_maps) {
  params_ = net_->failure_learnable_params();
  CAFFE_CHECK(!params_.empty(), "MonteCarlo: the net has no faultable (InnerProduct) parameters");
  CAFFE_CHECK(cfgs.size() == 1 || cfgs.size() == params_.size(),
              "MonteCarlo: give one inject config or one per faultable blob (" << params_.size() << ")");
  cfgs_ = cfgs;
  if (cfgs_.size() == 1) cfgs_.resize(params_.size(), cfgs[0]);
  for (auto* p : params_) {
    Dtype* c = nullptr;
    HIP_CALL(hipMalloc(reinterpret_cast<void**>(&c), p->count() * sizeof(Dtype)));
    HIP_CALL(hipMemcpyAsync(c, p->gpu_data(), p->count() * sizeof(Dtype), hipMemcpyDeviceToDevice, Caffe::hip_stream()));
    clean_.push_back(c);
  }
  for (auto* b : net_->output_blobs())
    if (b->count() == 1) outs_.push_back(b);
  const size_t no = std::max<size_t>(outs_.size(), 1);
  HIP_CALL(hipMalloc(reinterpret_cast<void**>(&d_sums_), no * sizeof(Dtype)));
  HIP_CALL(hipMalloc(reinterpret_cast<void**>(&d_per_map_), std::max(1, max_maps_) * no * sizeof(Dtype)));
  HIP_CALL(hipMalloc(reinterpret_cast<void**>(&d_broken_), params_.size() * sizeof(unsigned long long)));
  const auto& fl = net_->failure_learnable_layer_ids();
  first_fault_layer_ = *std::min_element(fl.begin(), fl.end());
  // RRAM_MC_OVERLAP=1 runs each map's injection on a side stream under the
  // layers before the first faultable one, released after the second
  // convolution (the persistent conv1 kernel holds every CU; conv2, the
  // dominant kernel, keeps the chip to itself) on a 256-block grid.  Off by
  // default: the injection shares the CUs with norm2 / pool2 / conv3 and
  // stretches from 89 to ~310 us, conv3 from 0.303 to 0.375 ms, and the live
  // bench measured serial 0.2-1.1 % ahead (profiles/r05_ab_mc_overlap.txt;
  // with per-layer events the overlap had led by 1.2 %).  The graph replay
  // (set_graph) is serial either way.
  {
    const char* e = getenv("RRAM_MC_OVERLAP");
    overlap_ = e && atoi(e) == 1 && first_fault_layer_ > 0;
  }
#ifndef RRAM_MC_RELEASE_AFTER_CONV
#define RRAM_MC_RELEASE_AFTER_CONV 2
#endif
  release_after_ = -1;  // no such convolution: the injection starts with the prefix
  for (int i = 0, n = 0; RRAM_MC_RELEASE_AFTER_CONV && i < first_fault_layer_ - 1; ++i)
    if (std::string(net_->layers()[i]->type()) == "Convolution" && ++n == RRAM_MC_RELEASE_AFTER_CONV) {
      release_after_ = i;
      break;
    }
  // between maps only the injection rewrites weights: the convolutions keep
  // their packed weights (Net::set_weight_pack_cache) unless a faultable blob
  // is theirs (the conv-fault extension), which every map's mutable access
  // invalidates, or a caller was handed the weights' pointer (SyncedMemory::expose)
  net_->set_weight_pack_cache(true);
  if (overlap_) {
    HIP_CALL(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
    HIP_CALL(hipEventCreateWithFlags(&ev_free_, hipEventDisableTiming));
    HIP_CALL(hipEventCreateWithFlags(&ev_injected_, hipEventDisableTiming));
  }
  Reset();
}

template <typename Dtype>
MonteCarlo<Dtype>::~MonteCarlo() {
  try {
    RestoreClean();
    net_->set_weight_pack_cache(false);
    Caffe::synchronize();
  } catch (...) {
  }
  drop_graph();
  if (d_state_) (void)hipFree(d_state_);
  for (auto* c : clean_) (void)hipFree(c);
  if (side_) {
    (void)hipStreamSynchronize(side_);
    (void)hipStreamDestroy(side_);
    (void)hipEventDestroy(ev_free_);
    (void)hipEventDestroy(ev_injected_);
  }
  (void)hipFree(d_sums_);
  (void)hipFree(d_per_map_);
  (void)hipFree(d_broken_);
}

template <typename Dtype>
void MonteCarlo<Dtype>::Reset() {
  maps_run_ = 0;
  if (d_state_) HIP_CALL(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_state_ + 1), 0, 1, Caffe::hip_stream()));
  HIP_CALL(hipMemsetAsync(d_sums_, 0, std::max<size_t>(outs_.size(), 1) * sizeof(Dtype), Caffe::hip_stream()));
  HIP_CALL(hipMemsetAsync(d_broken_, 0, params_.size() * sizeof(unsigned long long), Caffe::hip_stream()));
}

template <typename Dtype>
void MonteCarlo<Dtype>::RestoreClean() {
  for (size_t i = 0; i < params_.size(); ++i)
    HIP_CALL(hipMemcpyAsync(params_[i]->mutable_gpu_data(), clean_[i], params_[i]->count() * sizeof(Dtype),
                            hipMemcpyDeviceToDevice, Caffe::hip_stream()));
}

template <typename Dtype>
void MonteCarlo<Dtype>::set_reuse_prefix(bool on) {
  if (on) {
    const auto& L = net_->layers();
    const auto& tops = net_->top_vecs();
    // compare the memory, not the Blob: Split, single-input Concat and
    // single-top Slice tops share their bottom's SyncedMemory (ShareData)
    std::set<const SyncedMemory*> prefix_mem;
    for (int i = 0; i < first_fault_layer_; ++i) {
      CAFFE_CHECK(std::string(L[i]->type()) != "HDF5Data",
                  "MonteCarlo prefix reuse: layer " << net_->layer_names()[i] << " (HDF5Data) advances between forwards");
      for (auto* b : tops[i]) prefix_mem.insert(b->data().get());
    }
    for (size_t i = first_fault_layer_; i < L.size(); ++i) {
      // Split / Concat / Slice tops that share a prefix blob's memory are
      // views of it, not writes (they write only into memory of their own)
      const std::string t = L[i]->type();
      if (t == "Split" || t == "Concat" || t == "Slice") continue;
      for (auto* b : tops[i])
        CAFFE_CHECK(!prefix_mem.count(b->data().get()), "MonteCarlo prefix reuse: layer " << net_->layer_names()[i]
                                                << " writes a blob of the layers before the first faultable one");
    }
  }
  reuse_prefix_ = on;
  prefix_done_ = false;  // (re-)enabling recomputes the prefix on the next map
}

template <typename Dtype>
void MonteCarlo<Dtype>::drop_graph() {
  if (gexec_) (void)hipGraphExecDestroy(gexec_);
  if (graph_g_) (void)hipGraphDestroy(graph_g_);
  gexec_ = nullptr;
  graph_g_ = nullptr;
  graph_warm_ = false;
  graph_ptrs_.clear();
}

template <typename Dtype>
void MonteCarlo<Dtype>::set_graph(bool on) {
  if (on) {
    for (const auto& l : net_->layers())
      CAFFE_CHECK(std::string(l->type()) != "HDF5Data",
                  "MonteCarlo graph replay: " << l->name() << " (HDF5Data) advances between forwards");
    if (!d_state_) {
      HIP_CALL(hipMalloc(reinterpret_cast<void**>(&d_state_), 2 * sizeof(uint32_t)));
      HIP_CALL(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_state_), 0, 1, Caffe::hip_stream()));
      HIP_CALL(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_state_ + 1), maps_run_, 1, Caffe::hip_stream()));
    }
  } else {
    drop_graph();
  }
  graph_ = on;
}

// the device pointers a captured map depends on: every blob's and
// parameter's data and diff (a reshape or a set_gpu_data moves them), the
// clean copies and the statistics buffers
template <typename Dtype>
std::vector<const void*> MonteCarlo<Dtype>::graph_key() const {
  std::vector<const void*> k;
  for (const auto& b : net_->blobs()) k.push_back(b->data()->gpu_data());
  for (auto* p : net_->learnable_params()) {
    k.push_back(p->data()->gpu_data());
    k.push_back(static_cast<const void*>(p));
  }
  for (auto* c : clean_) k.push_back(c);
  k.push_back(d_sums_);
  k.push_back(d_per_map_);
  k.push_back(d_broken_);
  k.push_back(Caffe::hip_stream());
  // the scratch the captured launches read and write (workspace, packs,
  // split-K partials, gather tables): eager work between replays may have
  // reallocated it (a larger test batch, another net on this thread)
  k.push_back(reinterpret_cast<const void*>(static_cast<uintptr_t>(Caffe::scratch_gen().load())));
  k.push_back(reinterpret_cast<const void*>(static_cast<uintptr_t>(rram_scratch_generation())));
  return k;
}

// One map on the working stream: injection (map id m, or from d_state_[0]),
// the whole forward, the statistics (row maps_run_, or d_state_[1], which
// then advances together with the map id).
template <typename Dtype>
void MonteCarlo<Dtype>::map_body(bool dev_state, uint32_t m) {
  std::vector<rram_inject_seg> segs(params_.size());
  for (size_t i = 0; i < params_.size(); ++i)
    segs[i] = rram_inject_seg{clean_[i], params_[i]->mutable_gpu_data(), params_[i]->count(), (uint32_t)i, 0, cfgs_[i]};
  for (size_t s = 0; s < segs.size(); s += RRAM_MAX_SEGS) {
    const int k = static_cast<int>(std::min<size_t>(RRAM_MAX_SEGS, segs.size() - s));
    if (dev_state)
      RRAM_CALL(rram_inject_rng_batched_dev(segs.data() + s, k, seed_, d_state_, d_broken_ + s, Caffe::stream()));
    else
      RRAM_CALL(rram_inject_rng_batched(segs.data() + s, k, seed_, m, d_broken_ + s, Caffe::stream()));
  }
  net_->Forward(false);
  const size_t no = outs_.size();
  if (no == 0 && dev_state) {  // still advance the map id and the row
    rram_mc_outputs mo{};
    RRAM_CALL(rram_mc_accumulate_dev(&mo, d_sums_, nullptr, 1, 0, reinterpret_cast<int*>(d_state_ + 1), d_state_, 1,
                                     Caffe::stream()));
  }
  for (size_t k0 = 0; k0 < no; k0 += RRAM_MC_MAX_OUTPUTS) {
    rram_mc_outputs mo{};
    mo.n = static_cast<int>(std::min<size_t>(RRAM_MC_MAX_OUTPUTS, no - k0));
    for (int k = 0; k < mo.n; ++k) mo.p[k] = outs_[k0 + k]->gpu_data();
    if (dev_state)
      RRAM_CALL(rram_mc_accumulate_dev(&mo, d_sums_ + k0, d_per_map_ + k0, static_cast<int64_t>(no), max_maps_,
                                       reinterpret_cast<int*>(d_state_ + 1), d_state_,
                                       k0 + RRAM_MC_MAX_OUTPUTS >= no ? 1 : 0, Caffe::stream()));
    else
      RRAM_CALL(rram_mc_accumulate(&mo, d_sums_ + k0,
                                   maps_run_ < max_maps_ ? d_per_map_ + (size_t)maps_run_ * no + k0 : nullptr,
                                   Caffe::stream()));
  }
}

template <typename Dtype>
void MonteCarlo<Dtype>::Run(uint32_t map_begin, uint32_t map_count) {
  if (graph_ && !reuse_prefix_ && !timing_ && !net_->timing_on() && map_count > 0) {
    GraphStreamScope sc(gstream_);
    hipStream_t st = Caffe::hip_stream();
    HIP_CALL(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_state_), static_cast<int>(map_begin), 1, st));
    // the scratch moved since the capture -- or since the eager warm-up map
    // (a capture now would rebuild freed tables inside it): eager again
    if ((gexec_ || graph_warm_) && graph_key() != graph_ptrs_) drop_graph();
    for (uint32_t m = map_begin; m < map_begin + map_count; ++m) {
      if (!gexec_) {
        if (!graph_warm_) {
          // eager first (every workspace and pack buffer gets allocated), on
          // the device-state path the graph will replay
          map_body(true, m);
          graph_warm_ = true;
          graph_ptrs_ = graph_key();
          ++maps_run_;
          continue;
        }
        // every cache the forward keeps across calls (octet companions,
        // packed weights) is dropped, so the captured map recomputes what it
        // reads and stays exact whatever the host-side cache state is later
        for (const auto& b : net_->blobs()) (void)b->mutable_gpu_data();
        for (auto* p : net_->learnable_params()) (void)p->mutable_gpu_data();
        HIP_CALL(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
        try {
          map_body(true, m);
        } catch (...) {
          hipGraph_t g = nullptr;
          (void)hipStreamEndCapture(st, &g);
          if (g) (void)hipGraphDestroy(g);
          throw;
        }
        HIP_CALL(hipStreamEndCapture(st, &graph_g_));
        HIP_CALL(hipGraphInstantiate(&gexec_, graph_g_, nullptr, nullptr, 0));
        graph_ptrs_ = graph_key();
      }
      HIP_CALL(hipGraphLaunch(gexec_, st));
      ++maps_run_;
    }
    return;
  }
  if (d_state_)  // keep the device-side row in step with the eager maps
    HIP_CALL(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_state_ + 1), maps_run_ + static_cast<int>(map_count),
                               1, Caffe::hip_stream()));
  std::vector<rram_inject_seg> segs(params_.size());
  for (size_t i = 0; i < params_.size(); ++i)
    segs[i] = rram_inject_seg{clean_[i], params_[i]->mutable_gpu_data(), params_[i]->count(), (uint32_t)i, 0, cfgs_[i]};
  const size_t no = outs_.size();
  const int L = static_cast<int>(net_->layers().size());
  // overlapped, the injection gets a 256-block grid (it shares the CUs);
  // serial, the default 2048
#ifndef RRAM_MC_OVERLAP_GRID
#define RRAM_MC_OVERLAP_GRID 256
#endif
  const int prev_grid = rram_set_inject_grid(overlap_ && !reuse_prefix_ ? RRAM_MC_OVERLAP_GRID : 0);
  // the statistics folded into the layers that store each scalar output
  // (Layer::set_top_accumulator): no rram_mc_accumulate launch per map when
  // every output's producer takes it (all or none)
  std::vector<Layer<Dtype>*> acc_layers;
  struct ClearAcc {  // the layers never keep pointers into this driver past Run (exceptions included)
    std::vector<Layer<Dtype>*>& v;
    ~ClearAcc() {
      for (auto* a : v) a->set_top_accumulator(nullptr, nullptr);
    }
  } clear_acc{acc_layers};
  {
    const auto& L = net_->layers();
    const auto& tops = net_->top_vecs();
    for (size_t k = 0; k < no; ++k) {
      Layer<Dtype>* prod = nullptr;
      int prod_l = -1;
      for (size_t l = 0; l < L.size(); ++l)
        if (!tops[l].empty() && tops[l][0] == outs_[k]) {
          prod = L[l].get();
          prod_l = static_cast<int>(l);
        }
      // a producer inside the reused prefix runs on the first map only: its
      // constant output is then accumulated by rram_mc_accumulate every map
      const bool in_prefix = reuse_prefix_ && prod_l < first_fault_layer_;
      if (!prod || in_prefix || !prod->set_top_accumulator(d_sums_ + k, nullptr)) {
        for (auto* a : acc_layers) a->set_top_accumulator(nullptr, nullptr);
        acc_layers.clear();
        break;
      }
      acc_layers.push_back(prod);
    }
  }
  for (uint32_t m = map_begin; m < map_begin + map_count; ++m) {
    for (size_t k = 0; k < acc_layers.size(); ++k)
      acc_layers[k]->set_top_accumulator(d_sums_ + k, maps_run_ < max_maps_ ? d_per_map_ + (size_t)maps_run_ * no + k
                                                                            : nullptr);
    if (m != map_begin)
      for (auto* p : params_) (void)p->mutable_gpu_data();
    hipStream_t is = Caffe::hip_stream();
    const bool skip_prefix = reuse_prefix_ && prefix_done_ && first_fault_layer_ > 0;
    const bool overlap = overlap_ && !skip_prefix;
    if (overlap) {
      // released after the second convolution (see the constructor)
      if (release_after_ >= 0) net_->ForwardFromTo(0, release_after_, false);
      HIP_CALL(hipEventRecord(ev_free_, Caffe::hip_stream()));  // previous map's forward is done with the weights
      HIP_CALL(hipStreamWaitEvent(side_, ev_free_, 0));
      is = side_;
    }
    if (timing_) timer_.start(0, is);
    for (size_t s = 0; s < segs.size(); s += RRAM_MAX_SEGS) {
      const int k = static_cast<int>(std::min<size_t>(RRAM_MAX_SEGS, segs.size() - s));
      RRAM_CALL(rram_inject_rng_batched(segs.data() + s, k, seed_, m, d_broken_ + s, is));
    }
    if (timing_) timer_.stop(0, is);
    if (overlap) {
      HIP_CALL(hipEventRecord(ev_injected_, side_));
      net_->ForwardFromTo(release_after_ + 1, first_fault_layer_ - 1, false);  // the rest of the prefix runs under the injection
      HIP_CALL(hipStreamWaitEvent(Caffe::hip_stream(), ev_injected_, 0));
      net_->ForwardFromTo(first_fault_layer_, L - 1, false);
    } else if (skip_prefix) {
      net_->ForwardFromTo(first_fault_layer_, L - 1, false);  // the prefix's blobs hold the first map's bits
    } else {
      net_->Forward(false);
    }
    if (reuse_prefix_) prefix_done_ = true;
    for (size_t k0 = 0; acc_layers.empty() && k0 < no; k0 += RRAM_MC_MAX_OUTPUTS) {
      rram_mc_outputs mo{};
      mo.n = static_cast<int>(std::min<size_t>(RRAM_MC_MAX_OUTPUTS, no - k0));
      for (int k = 0; k < mo.n; ++k) mo.p[k] = outs_[k0 + k]->gpu_data();
      RRAM_CALL(rram_mc_accumulate(&mo, d_sums_ + k0,
                                   maps_run_ < max_maps_ ? d_per_map_ + (size_t)maps_run_ * no + k0 : nullptr,
                                   Caffe::stream()));
    }
    ++maps_run_;
  }
  rram_set_inject_grid(prev_grid);
}

template <typename Dtype>
void MonteCarlo<Dtype>::Stats(std::vector<double>& outputs, std::vector<unsigned long long>& broken,
                              std::vector<float>& per_map) const {
  const size_t no = outs_.size();
  std::vector<Dtype> s(no);
  broken.assign(params_.size(), 0);
  const int pm = std::min(maps_run_, max_maps_);
  per_map.assign((size_t)pm * no, 0.f);
  if (no) HIP_CALL(hipMemcpyAsync(s.data(), d_sums_, no * sizeof(Dtype), hipMemcpyDeviceToHost, Caffe::hip_stream()));
  HIP_CALL(hipMemcpyAsync(broken.data(), d_broken_, broken.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                          Caffe::hip_stream()));
  if (pm && no)
    HIP_CALL(hipMemcpyAsync(per_map.data(), d_per_map_, per_map.size() * sizeof(float), hipMemcpyDeviceToHost,
                            Caffe::hip_stream()));
  HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
  outputs.assign(s.begin(), s.end());
}

template class FailureMaker<float>;
template class GaussianFailureMaker<float>;
template class FailureStrategy<float>;
template class ThresholdFailureStrategy<float>;
template class Solver<float>;
template class MonteCarlo<float>;

}  // namespace caffe
