// Fault model, fault-tolerance strategies, SGD solver and the Monte-Carlo
// fault-map driver.
//
//   FailureMaker / GaussianFailureMaker  — include/caffe/failure_maker.hpp:11-96,
//       src/caffe/failure_maker.cpp, failure_maker.cu
//   FailureStrategy / ThresholdFailureStrategy — include/caffe/strategy.hpp:34-82,
//       src/caffe/strategy.cpp:7-33 (a3)
//   Solver / SGDSolver — src/caffe/solver.cpp (fork hooks :14-40, :132-148,
//       Step order :237-325, Test :385-458), src/caffe/solvers/sgd_solver.cpp (a4, a11)
//   MonteCarlo — the reference's one-map-per-run fault-injected Test
//        generalised to many maps per launch sequence.
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "net.hpp"

namespace caffe {

// hipStreamBeginCapture refuses the legacy NULL stream (e.g. torch's default
// stream).  On it, a graph section (eager warm-up, capture, launches) runs on
// a private non-blocking stream instead, ordered after the caller's earlier
// work and before its later work by two events, with Caffe's stream switched
// for the section so every launch and stream-keyed scratch buffer of the
// section sees one stream.  On any other stream it does nothing.
class GraphStream {
 public:
  GraphStream() = default;
  GraphStream(const GraphStream&) = delete;
  GraphStream& operator=(const GraphStream&) = delete;
  ~GraphStream();
  void enter();
  void leave();

 private:
  hipStream_t own_ = nullptr;
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;
  bool active_ = false;
};
struct GraphStreamScope {
  explicit GraphStreamScope(GraphStream& g) : g_(g) { g_.enter(); }
  ~GraphStreamScope() { g_.leave(); }
  GraphStream& g_;
};

template <typename Dtype>
class Solver;

template <typename Dtype>
class FailureMaker {
 public:
  explicit FailureMaker(const Msg& param) : param_(param) {}
  virtual ~FailureMaker();
  // failure_maker.hpp:23-30: nullptr unless type == "gaussian"
  static std::shared_ptr<FailureMaker<Dtype>> CreateMaker(const Msg& param, std::shared_ptr<Net<Dtype>> net);
  // failure_maker.hpp:32-58 without the per-iteration D2H count (Appendix A Q5):
  // the broken count accumulates on the device, read it with broken_counts().
  void Fail(int iter) { Fail_gpu(iter); }
  virtual void Fail_gpu(int iter) = 0;
  std::vector<Blob<Dtype>*> fail_iterations();
  std::vector<unsigned long long> broken_counts();  // per failure param, after the last Fail()
  unsigned long long* device_counts() { return d_counts_; }
  const Msg& param() const { return param_; }

 protected:
  Msg param_;
  std::shared_ptr<Net<Dtype>> net_;
  // endurance in data, stuck value in diff (reference layout, failure_maker.cpp:30-36)
  std::vector<std::unique_ptr<Blob<Dtype>>> fail_iterations_;
  unsigned long long* d_counts_ = nullptr;
};

template <typename Dtype>
class GaussianFailureMaker : public FailureMaker<Dtype> {
 public:
  GaussianFailureMaker(const Msg& param, std::shared_ptr<Net<Dtype>> net);
  void Fail_gpu(int iter) override;
  float decrement = 100.0f;  // "batch size FIXME" constant (failure_maker.cpp:73)
  float epsilon = 1e-20f;    // failure_maker.cpp:56
};

template <typename Dtype>
class FailureStrategy {
 public:
  FailureStrategy(const Msg& param, std::shared_ptr<FailureMaker<Dtype>> fm, std::shared_ptr<Net<Dtype>> net,
                  const Solver<Dtype>* solver)
      : param_(param), fmaker_(fm), net_(net), solver_(solver) {}
  virtual ~FailureStrategy() = default;
  // strategy.hpp:34-50; unknown type -> Error (Appendix A Q10: fail cleanly)
  static std::shared_ptr<FailureStrategy<Dtype>> CreateStrategy(const Msg& param, std::shared_ptr<FailureMaker<Dtype>> fm,
                                                                std::shared_ptr<Net<Dtype>> net, const Solver<Dtype>* s);
  virtual void Apply() = 0;
  virtual const char* type() const = 0;

 protected:
  Msg param_;
  std::shared_ptr<FailureMaker<Dtype>> fmaker_;
  std::shared_ptr<Net<Dtype>> net_;
  const Solver<Dtype>* solver_;
};

template <typename Dtype>
class ThresholdFailureStrategy : public FailureStrategy<Dtype> {
 public:
  using FailureStrategy<Dtype>::FailureStrategy;
  void Apply() override;
  const char* type() const override { return "threshold"; }
  float threshold() const { return static_cast<float>(this->param_.num("threshold", 0.001)); }
  // per failure param: threshold * lr * lr_mult (strategy.cpp:12-14)
  float threshold_for(int failure_param_index) const;
  // Appendix A Q6: the reference indexes params_lr() with the failure-param
  // index; true reproduces that quirk, false (default) uses the param's own lr_mult.
  bool reference_lr_index = false;
};

// glibc rand()/random() (TYPE_3 additive feedback generator of srandom_r /
// random_r): the reference's genetic strategy draws with unseeded rand()
// (strategy.cpp:170-175, Appendix A Q9), i.e. this generator at seed 1.
class GlibcRand {
 public:
  explicit GlibcRand(uint32_t seed = 1);
  int operator()();  // in [0, RAND_MAX = 2^31 - 1]

 private:
  uint32_t r_[34];
  int i_ = 0;  // ring position of r[k - 34]
};

// strategy.hpp:84-142 / strategy.cpp:35-137.  Every `period` iterations after
// `start`, the FC neurons are re-ordered so that the neurons the pretrained
// prune order ranks most prunable land on the physical neurons with the most
// stuck-at-zero cells.  Counts on the device, sort on the host (std::sort with
// the reference comparator, so ties resolve identically), moves as gathers.
// rram_reference_compat: true reproduces Appendix A Q8 (bias rows copied from
// the weight array, strategy.cpp:118-119).
template <typename Dtype>
class RemappingFailureStrategy : public FailureStrategy<Dtype> {
 public:
  RemappingFailureStrategy(const Msg& param, std::shared_ptr<FailureMaker<Dtype>> fm, std::shared_ptr<Net<Dtype>> net,
                           const Solver<Dtype>* solver);
  void Apply() override;
  const char* type() const override { return "remapping"; }
  // orders[i-1] for FC pair (i-1, i): neuron indices of FC layer i-1 sorted
  // by (#flagged cells in its input row + #flagged cells in its output column)
  std::vector<std::vector<int>> SortFCNeurons();
  const std::vector<std::vector<int>>& prune_orders() const { return prune_orders_; }
  bool reference_compat = false;

 private:
  int period_ = 100, start_ = 0, times_ = 0;
  std::vector<std::vector<int>> prune_orders_;
};

// strategy.hpp:144-183 / strategy.cpp:139-288.  Random pairwise neuron swaps
// accepted when they move failed cells onto weights the prune net marks as
// prunable.  The decisions only read the fault state and the prune masks, so
// they run on host copies; the accepted swaps compose into one permutation
// per FC blob, applied on the device in one gather per array.
// rram_reference_compat: true reproduces Q9's flat prune_input[n1]/[n2] swap
// (strategy.cpp:265-267); rram_rand_seed (default 1 = glibc's unseeded rand).
template <typename Dtype>
class GeneticFailureStrategy : public FailureStrategy<Dtype> {
 public:
  GeneticFailureStrategy(const Msg& param, std::shared_ptr<FailureMaker<Dtype>> fm, std::shared_ptr<Net<Dtype>> net,
                         const Solver<Dtype>* solver);
  void Apply() override;
  const char* type() const override { return "genetic"; }
  int CalculateOverallDist();
  int last_before() const { return before_; }
  int last_after() const { return after_; }
  int last_accepted() const { return accepted_; }
  bool reference_compat = false;

 private:
  void FetchEndurance();
  int switch_time_ = 100, period_ = 100, start_ = 0, times_ = 0;
  int before_ = 0, after_ = 0, accepted_ = 0;
  GlibcRand rand_;
  std::vector<std::vector<float>> prune_;  // prune net failure params (host, mutated by swaps)
  std::vector<std::vector<float>> endur_;     // endurance of every failure param (host copy per Apply)
};

template <typename Dtype>
class Solver {
 public:
  // solver_param: SolverParameter text; net_param (optional) overrides `net:`;
  // options: net options (data_shape, num_classes, fault_layers, fuse_relu)
  // plus `fused_update` (true: one fused HBM pass per blob for the training tail).
  Solver(const Msg& solver_param, const Msg* net_param, const Msg& options);
  virtual ~Solver();

  void Step(int iters);
  // solver.cpp:328-370; resume_file: a .solverstate to Restore() first
  void Solve(const char* resume_file = nullptr);
  // solver.cpp:461-518 (BINARYPROTO): <prefix>_iter_N.caffemodel and
  // .solverstate, plus <prefix>_iter_N.faultstate with the fault maps
  // (Appendix A Q11: the reference redraws them on resume).  Returns the
  // .solverstate path.
  std::string Snapshot();
  // sgd_solver.cpp:309-326; the fault maps come back too when the matching
  // .faultstate file exists
  void Restore(const std::string& state_file);
  const Msg& net_options() const { return options_; }
  void emit_log(const std::string& s) const {
    if (log) log(s);
  }
  // returns the mean of every output element of test net `id` over test_iter
  std::vector<Dtype> Test(int id = 0);
  std::vector<std::vector<Dtype>> TestAll();

  std::shared_ptr<Net<Dtype>> net() { return net_; }
  const std::vector<std::shared_ptr<Net<Dtype>>>& test_nets() const { return test_nets_; }
  int iter() const { return iter_; }
  const Msg& param() const { return param_; }
  Dtype GetLearningRate() const;
  std::shared_ptr<FailureMaker<Dtype>> failure_maker() { return fmaker_; }
  const std::vector<std::shared_ptr<FailureStrategy<Dtype>>>& strategies() const { return strategys_; }
  Dtype smoothed_loss() const { return smoothed_loss_; }
  // SGDSolver::history() (sgd_solver.hpp:29): momentum history, one blob per learnable param
  const std::vector<std::unique_ptr<Blob<Dtype>>>& history() const { return history_; }
  // Solver::Callback::on_gradients_ready (solver.hpp:80-91): the data-parallel
  // hook (RCCL all-reduce of the flat gradient buffer).
  std::function<void()> on_gradients_ready;
  std::function<void(const std::string&)> log;
  // hipGraph replay of the training iteration (opt-in; launch-bound small
  // nets, no reference counterpart): [ClearParamDiffs + Forward + Backward]
  // and the fused update tail are each captured once, after one eager
  // iteration, and replayed; on_gradients_ready (the data-parallel RCCL
  // all-reduce) runs between the two launches, outside any graph.
  // Iterations that display, test, snapshot or average the loss run eager,
  // as does everything when the fused tail is off or a per-layer backward
  // hook is set; a changed learning rate or moved buffers recapture.  Nets
  // with per-iteration host state (Dropout, HDF5Data) are refused.
  // Bit-identical to the eager iterations.
  void set_graph(bool on);
  bool graph_active() const { return gx_[0] != nullptr; }
  // the flat learnable data / diff buffers every param is aliased into
  // (nullptr when the `flat_params: false` option turned them off)
  Dtype* flat_data() const { return static_cast<Dtype*>(flat_); }
  Dtype* flat_diff() const { return flat_ ? static_cast<Dtype*>(flat_) + net_->flat_param_count() : nullptr; }

 protected:
  bool graph_ = false, graph_warm_ = false;
  hipGraph_t gg_[2] = {nullptr, nullptr};
  hipGraphExec_t gx_[2] = {nullptr, nullptr};
  GraphStream gstream_;
  Dtype graph_rate_ = 0, graph_prev_rate_ = -1;
  std::vector<const void*> graph_ptrs_;
  std::vector<const void*> graph_key() const;
  void drop_graphs();
  template <typename F>
  void capture_launch(int k, F&& body);
  void InitFailurePattern(const Msg& failure_param);
  void ComputeUpdate();
  void ApplyStrategy();
  void ApplyUpdate();
  void FusedTail();
  void Fail(int iter) {
    if (fmaker_) fmaker_->Fail(iter);
  }
  void ClipGradients();
  void Regularize(int param_id);
  void ComputeUpdateValue(int param_id, Dtype rate);
  void emit(const std::string& s) {
    if (log) log(s);
  }

  std::string SnapshotFilename(const std::string& ext) const {
    return param_.str("snapshot_prefix") + "_iter_" + std::to_string(iter_) + ext;
  }

  Msg param_;
  Msg options_;
  // flat learnable data / diff buffers the params are aliased into
  // (ClearParamDiffs becomes one memset; the data-parallel all-reduce re-aliases)
  void* flat_ = nullptr;
  std::shared_ptr<Net<Dtype>> net_;
  std::vector<std::shared_ptr<Net<Dtype>>> test_nets_;
  std::vector<std::unique_ptr<Blob<Dtype>>> history_, temp_;
  std::shared_ptr<FailureMaker<Dtype>> fmaker_;
  std::vector<std::shared_ptr<FailureStrategy<Dtype>>> strategys_;
  int iter_ = 0, current_step_ = 0;
  Dtype smoothed_loss_ = 0;
  std::vector<Dtype> losses_;
  bool fused_update_ = false;
  bool flip_cache_ = true;  // option conv_flip_cache: FusedTail writes the flipped kernels (rram_update_seg.w_flip)
};

// Monte-Carlo fault-map inference (north_star).
// For every map m: inject(clean IP weights -> net weights) with the counter
// RNG keyed by (seed, m, blob), forward the TEST net, accumulate its outputs
// (accuracy, loss) and the per-blob broken-cell counts on the device.
template <typename Dtype>
class MonteCarlo {
 public:
  MonteCarlo(std::shared_ptr<Net<Dtype>> net, const std::vector<rram_inject_cfg>& cfgs, uint64_t seed,
             int max_maps);
  ~MonteCarlo();
  void Run(uint32_t map_begin, uint32_t map_count);
  void Reset();
  // sums over the maps run so far: outputs[n_outputs] (each output's mean over
  // its elements), broken[n_fault_blobs], per_map[maps_run][n_outputs]
  void Stats(std::vector<double>& outputs, std::vector<unsigned long long>& broken,
             std::vector<float>& per_map) const;
  int maps_run() const { return maps_run_; }
  int num_outputs() const { return static_cast<int>(outs_.size()); }
  void RestoreClean();
  // hipEvent timing of the injection launches (key 0)
  void set_timing(bool on) { timing_ = on; }
  // Prefix reuse (opt-in; a different workload from the reference's, which
  // runs every map's whole forward): under reference semantics only the
  // InnerProduct blobs are faulted, so the layers before the first faultable
  // one compute the same bits for every map of a fixed input batch.  On, the
  // next map runs them once and the following maps start at the first
  // faultable layer.  Refused when a source layer advances between forwards
  // (HDF5Data) or a later layer writes a prefix blob in place; the caller
  // re-enables it after changing the input batch or a prefix weight.
  void set_reuse_prefix(bool on);
  // hipGraph replay (opt-in; for launch-bound small nets): one map (injection
  // + forward + statistics) is captured once and replayed per map, the map
  // id and the per-map row advancing in device memory (rram_inject_rng_batched_dev,
  // rram_mc_accumulate_dev).  Bit-identical to the eager maps.  Falls back to
  // the eager path while timing, injection overlap or prefix reuse is on, and
  // refuses nets whose source layers advance between forwards (HDF5Data).
  void set_graph(bool on);
  bool graph_active() const { return gexec_ != nullptr; }
  EventTimer& timer() { return timer_; }
  int64_t fault_weights() const {
    int64_t n = 0;
    for (auto* p : params_) n += p->count();
    return n;
  }

 private:
  bool timing_ = false;
  bool reuse_prefix_ = false, prefix_done_ = false;
  EventTimer timer_;
  std::shared_ptr<Net<Dtype>> net_;
  std::vector<rram_inject_cfg> cfgs_;
  uint64_t seed_;
  int max_maps_;
  int maps_run_ = 0;
  std::vector<Blob<Dtype>*> params_;
  std::vector<Dtype*> clean_;
  std::vector<Blob<Dtype>*> outs_;
  // injection overlap: map m's injection runs on side_ while the layers
  // before the first faultable one run on the working stream; the faultable
  // layers wait for it (ev_injected_), the next injection waits for the
  // previous map's forward (ev_free_)
  bool overlap_ = true;
  int first_fault_layer_ = 0;
  int release_after_ = -1;  // overlapped maps: the prefix layer after which the injection starts
  hipStream_t side_ = nullptr;
  hipEvent_t ev_free_ = nullptr, ev_injected_ = nullptr;
  Dtype* d_sums_ = nullptr;       // [n_outputs]
  Dtype* d_per_map_ = nullptr;    // [max_maps][n_outputs]
  unsigned long long* d_broken_ = nullptr;
  // graph replay: d_state_ = {map id, per-map row} on the device
  bool graph_ = false, graph_warm_ = false;
  uint32_t* d_state_ = nullptr;
  hipGraph_t graph_g_ = nullptr;
  hipGraphExec_t gexec_ = nullptr;
  GraphStream gstream_;
  std::vector<const void*> graph_ptrs_;  // the device pointers the graph was captured with
  void map_body(bool dev_state, uint32_t m);  // one map's launches on the working stream
  std::vector<const void*> graph_key() const;
  void drop_graph();
};

}  // namespace caffe
