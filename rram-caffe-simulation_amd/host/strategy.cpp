// Remapping and genetic fault-tolerance strategies:
// include/caffe/strategy.hpp:84-183, src/caffe/strategy.cpp:35-288.
#include <algorithm>
#include <fstream>
#include <numeric>
#include <sstream>

#include "solver.hpp"

namespace caffe {

// ================================================================ GlibcRand
// srandom_r: r[0] = seed (0 -> 1), r[i] = 16807 r[i-1] mod (2^31 - 1) for
// i < 31, r[31..33] = r[0..2]; then r[i] = r[i-31] + r[i-3] (mod 2^32) and the
// k-th output is r[k + 344] >> 1 (the first 310 words are discarded).
GlibcRand::GlibcRand(uint32_t seed) {
  int64_t r[34];
  r[0] = seed == 0 ? 1 : static_cast<int32_t>(seed);
  for (int i = 1; i < 31; ++i) {
    r[i] = (16807LL * r[i - 1]) % 2147483647LL;
    if (r[i] < 0) r[i] += 2147483647LL;
  }
  for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
  for (int i = 0; i < 34; ++i) r_[i] = static_cast<uint32_t>(r[i]);
  i_ = 0;  // r_[i_] holds r[k - 34] for the next index k (k = 34 now)
  for (int k = 34; k < 344; ++k) (void)(*this)();
}

int GlibcRand::operator()() {
  // r[k] = r[k-31] + r[k-3]; the ring holds r[k-34 .. k-1] starting at i_
  const uint32_t v = r_[(i_ + 3) % 34] + r_[(i_ + 31) % 34];
  r_[i_] = v;
  i_ = (i_ + 1) % 34;
  return static_cast<int>(v >> 1);
}

namespace {

// device int vector for the gathers; freed on the stream after use
struct DevInts {
  int* p = nullptr;
  explicit DevInts(const std::vector<int>& h) {
    HIP_CALL(hipMallocAsync(reinterpret_cast<void**>(&p), std::max<size_t>(h.size(), 1) * sizeof(int),
                            Caffe::hip_stream()));
    HIP_CALL(hipMemcpyAsync(p, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice, Caffe::hip_stream()));
  }
  ~DevInts() { (void)hipFreeAsync(p, Caffe::hip_stream()); }
};
struct DevFloats {
  float* p = nullptr;
  explicit DevFloats(int64_t n) {
    HIP_CALL(hipMallocAsync(reinterpret_cast<void**>(&p), std::max<int64_t>(n, 1) * sizeof(float), Caffe::hip_stream()));
  }
  ~DevFloats() { (void)hipFreeAsync(p, Caffe::hip_stream()); }
};

void d2d(float* dst, const float* src, int64_t n) {
  HIP_CALL(hipMemcpyAsync(dst, src, n * sizeof(float), hipMemcpyDeviceToDevice, Caffe::hip_stream()));
}

template <typename Dtype>
std::vector<Blob<Dtype>*> fail_blobs(const std::shared_ptr<FailureMaker<Dtype>>& fm, const char* who) {
  CAFFE_CHECK(fm != nullptr && dynamic_cast<GaussianFailureMaker<Dtype>*>(fm.get()) != nullptr,
              who << " failure strategy needs a gaussian failure_pattern");
  return fm->fail_iterations();
}

// new rows/cols of a [rows x cols] blob (data and diff): row r <- old row rp[r],
// column c <- old column cp[c]; identity vectors are skipped
template <typename Dtype>
void permute_blob(Blob<Dtype>* b, const std::vector<int>* rp, const std::vector<int>* cp) {
  const int rows = b->shape(0), cols = b->count() / std::max(rows, 1);
  DevFloats tmp(b->count());
  auto is_id = [](const std::vector<int>* v) {
    if (!v) return true;
    for (size_t i = 0; i < v->size(); ++i)
      if ((*v)[i] != (int)i) return false;
    return true;
  };
  for (int which = 0; which < 2; ++which) {
    Dtype* arr = which == 0 ? b->mutable_gpu_data() : b->mutable_gpu_diff();
    if (!is_id(rp)) {
      std::vector<int> to(rp->size());
      std::iota(to.begin(), to.end(), 0);
      DevInts dto(to), dfrom(*rp);
      d2d(tmp.p, arr, b->count());
      RRAM_CALL(rram_permute_rows(tmp.p, arr, cols, dto.p, dfrom.p, (int)to.size(), Caffe::stream()));
    }
    if (!is_id(cp)) {
      std::vector<int> to(cp->size());
      std::iota(to.begin(), to.end(), 0);
      DevInts dto(to), dfrom(*cp);
      d2d(tmp.p, arr, b->count());
      RRAM_CALL(rram_permute_cols(tmp.p, arr, rows, cols, dto.p, dfrom.p, (int)to.size(), Caffe::stream()));
    }
  }
}

}  // namespace

// ======================================================= remapping strategy
// strategy.hpp:87-124
template <typename Dtype>
RemappingFailureStrategy<Dtype>::RemappingFailureStrategy(const Msg& param, std::shared_ptr<FailureMaker<Dtype>> fm,
                                                          std::shared_ptr<Net<Dtype>> net, const Solver<Dtype>* s)
    : FailureStrategy<Dtype>(param, fm, net, s) {
  period_ = (int)param.integer("period", 100);
  start_ = (int)param.integer("start", 0);
  CAFFE_CHECK(period_ > 0, "`period` must be postive!");
  CAFFE_CHECK(start_ >= 0, "`start` must be non-negative!");
  CAFFE_CHECK(param.has("prune_order_file"), "remapping failure strategy must have a prune order file.");
  const std::string path = param.str("prune_order_file");
  std::ifstream fs(path);
  CAFFE_CHECK(fs.is_open(), "cannot open prune order file " << path);
  const auto& fps = net->failure_learnable_params();
  const auto& fc = net->fc_params_ids_;
  for (size_t i = 1; i < fc.size(); ++i) {
    const int n = fps[fc[i]]->shape(1);
    std::vector<int> order;
    for (int j = 0; j < n; ++j) {
      int v;
      CAFFE_CHECK(static_cast<bool>(fs >> v), "prune order file not correct");
      order.push_back(v);
    }
    prune_orders_.push_back(order);
  }
}

// strategy.cpp:48-86
template <typename Dtype>
std::vector<std::vector<int>> RemappingFailureStrategy<Dtype>::SortFCNeurons() {
  const auto& fps = this->net_->failure_learnable_params();
  const auto& fc = this->net_->fc_params_ids_;
  auto fi = fail_blobs(this->fmaker_, "remapping");
  const size_t size = fc.size();
  std::vector<std::vector<unsigned>> rc(size), cc(size);
  for (size_t i = 0; i < size; ++i) {
    Blob<Dtype>* f = fi[fc[i]];
    const int rows = f->shape(0), cols = f->shape(1);
    std::vector<unsigned> zero(cols, 0u);
    unsigned* d = nullptr;
    HIP_CALL(hipMallocAsync(reinterpret_cast<void**>(&d), (size_t)(rows + cols) * sizeof(unsigned), Caffe::hip_stream()));
    HIP_CALL(hipMemsetAsync(d + rows, 0, (size_t)cols * sizeof(unsigned), Caffe::hip_stream()));
    RRAM_CALL(rram_stuck_zero_counts(f->gpu_data(), f->gpu_diff(), rows, cols, d, d + rows, Caffe::stream()));
    rc[i].resize(rows);
    cc[i].resize(cols);
    HIP_CALL(hipMemcpyAsync(rc[i].data(), d, rows * sizeof(unsigned), hipMemcpyDeviceToHost, Caffe::hip_stream()));
    HIP_CALL(hipMemcpyAsync(cc[i].data(), d + rows, cols * sizeof(unsigned), hipMemcpyDeviceToHost, Caffe::hip_stream()));
    HIP_CALL(hipFreeAsync(d, Caffe::hip_stream()));
  }
  HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
  std::vector<std::vector<int>> orders;
  for (size_t i = 1; i < size; ++i) {
    const int n_in = fps[fc[i - 1]]->shape(0);
    CAFFE_CHECK(fps[fc[i]]->shape(1) == n_in, "FC layers " << i - 1 << " and " << i << " are not adjacent ("
                                                         << n_in << " outputs feed " << fps[fc[i]]->shape(1) << " inputs)");
    std::vector<int> zero_nums(n_in);
    for (int j = 0; j < n_in; ++j) zero_nums[j] = static_cast<int>(rc[i - 1][j] + cc[i][j]);
    std::vector<int> idx(zero_nums.size());
    std::iota(idx.begin(), idx.end(), 0);
    // the reference's unstable sort and comparator, so ties resolve the same way
    std::sort(idx.begin(), idx.end(), [&zero_nums](size_t i1, size_t i2) { return zero_nums[i1] < zero_nums[i2]; });
    orders.push_back(idx);
  }
  return orders;
}

// strategy.cpp:88-137
template <typename Dtype>
void RemappingFailureStrategy<Dtype>::Apply() {
  ++times_;
  if (times_ < start_ || (times_ - start_) % period_ != 0) return;
  const auto& fps = this->net_->failure_learnable_params();
  const auto& fc = this->net_->fc_params_ids_;
  const auto orders = SortFCNeurons();
  for (size_t i = 1; i < fc.size(); ++i) {
    const std::vector<int>& order = orders[i - 1];
    const std::vector<int>& prune = prune_orders_[i - 1];
    CAFFE_CHECK(order.size() == prune.size(), "prune order length " << prune.size() << " != " << order.size());
    Blob<Dtype>* win = fps[fc[i - 1]];
    CAFFE_CHECK(fc[i - 1] + 1 < (int)fps.size() && fps[fc[i - 1] + 1]->count() == win->shape(0),
                "remapping needs a bias after FC weight blob " << fc[i - 1]);
    Blob<Dtype>* bin = fps[fc[i - 1] + 1];
    Blob<Dtype>* wout = fps[fc[i]];
    const int dim = win->shape(1);
    DevInts dto(order), dfrom(prune);
    const int n = (int)order.size();
    {  // input weights (rows) and biases
      DevFloats tw(win->count()), tb(bin->count());
      for (int which = 0; which < 2; ++which) {
        Dtype* w = which == 0 ? win->mutable_gpu_data() : win->mutable_gpu_diff();
        Dtype* b = which == 0 ? bin->mutable_gpu_data() : bin->mutable_gpu_diff();
        d2d(tw.p, w, win->count());
        d2d(tb.p, b, bin->count());
        RRAM_CALL(rram_permute_rows(tw.p, w, dim, dto.p, dfrom.p, n, Caffe::stream()));
        // Q8: the reference reads the bias from the weight array (strategy.cpp:118-119)
        RRAM_CALL(rram_permute_elems(reference_compat ? tw.p : tb.p, b, dto.p, dfrom.p, n, Caffe::stream()));
      }
    }
    {  // output weights (columns)
      DevFloats tw(wout->count());
      for (int which = 0; which < 2; ++which) {
        Dtype* w = which == 0 ? wout->mutable_gpu_data() : wout->mutable_gpu_diff();
        d2d(tw.p, w, wout->count());
        RRAM_CALL(rram_permute_cols(tw.p, w, wout->shape(0), wout->shape(1), dto.p, dfrom.p, n, Caffe::stream()));
      }
    }
  }
  HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
}

// ========================================================= genetic strategy
// strategy.hpp:147-165
template <typename Dtype>
GeneticFailureStrategy<Dtype>::GeneticFailureStrategy(const Msg& param, std::shared_ptr<FailureMaker<Dtype>> fm,
                                                      std::shared_ptr<Net<Dtype>> net, const Solver<Dtype>* s)
    : FailureStrategy<Dtype>(param, fm, net, s), rand_(static_cast<uint32_t>(param.integer("rram_rand_seed", 1))) {
  switch_time_ = (int)param.integer("switch_time", 100);
  CAFFE_CHECK(switch_time_ > 0, "`switch_time_` must be postive!");
  period_ = (int)param.integer("period", 100);
  start_ = (int)param.integer("start", 0);
  CAFFE_CHECK(period_ > 0, "`period` must be postive!");
  CAFFE_CHECK(start_ >= 0, "`start` must be non-negative!");
  CAFFE_CHECK(param.has("prune_net_file"), "genetic failure strategy must have a prune net file.");
  CAFFE_CHECK(param.has("prune_model_file"), "genetic failure strategy must have a prune model file.");
  // the prune net (TEST phase) only lends its failure-param values: host copies
  Net<Dtype> prune(parse_prototxt_file(param.str("prune_net_file")), TEST, s ? s->net_options() : Msg());
  prune.CopyTrainedLayersFrom(param.str("prune_model_file"));
  const auto& pp = prune.failure_learnable_params();
  CAFFE_CHECK(pp.size() == net->failure_learnable_params().size(),
              "prune net has " << pp.size() << " failure params, the trained net " << net->failure_learnable_params().size());
  for (size_t i = 0; i < pp.size(); ++i) {
    CAFFE_CHECK(pp[i]->shape() == net->failure_learnable_params()[i]->shape(), "prune net param " << i << " shape mismatch");
    prune_.push_back(BlobToProto(pp[i], false).data);
  }
}

template <typename Dtype>
void GeneticFailureStrategy<Dtype>::FetchEndurance() {
  auto fi = fail_blobs(this->fmaker_, "genetic");
  endur_.resize(fi.size());
  for (size_t i = 0; i < fi.size(); ++i) {
    endur_[i].resize(fi[i]->count());
    HIP_CALL(hipMemcpyAsync(endur_[i].data(), fi[i]->gpu_data(), endur_[i].size() * sizeof(float), hipMemcpyDeviceToHost,
                            Caffe::hip_stream()));
  }
  HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
}

// strategy.cpp:139-156
template <typename Dtype>
int GeneticFailureStrategy<Dtype>::CalculateOverallDist() {
  const float eps = 1e-20f;
  int dist = 0;
  for (size_t i = 0; i < endur_.size(); ++i)
    for (size_t j = 0; j < endur_[i].size(); ++j)
      if (prune_[i][j] < eps && endur_[i][j] < 0) dist += 1;
  return dist;
}

// strategy.cpp:158-288
template <typename Dtype>
void GeneticFailureStrategy<Dtype>::Apply() {
  ++times_;
  if (times_ < start_ || (times_ - start_) % period_ != 0) return;
  const float eps = 1e-20f;
  const auto& fps = this->net_->failure_learnable_params();
  const auto& fc = this->net_->fc_params_ids_;
  const int size = (int)fc.size();
  CAFFE_CHECK(size >= 2, "genetic strategy needs at least two InnerProduct layers");
  FetchEndurance();
  before_ = CalculateOverallDist();
  // accepted swaps compose into row permutations (input side: weights, biases)
  // and column permutations (output side) per failure param
  std::vector<std::vector<int>> rowp(fps.size()), colp(fps.size());
  accepted_ = 0;
  for (int i = 0; i < switch_time_;) {
    const int layer_index = rand_() % (size - 1) + 1;
    const int a = fc[layer_index - 1], b = fc[layer_index];
    const int layer_dim = fps[a]->shape(0), input_layer_dim = fps[a]->shape(1);
    const int n1 = rand_() % layer_dim;
    const int n2 = rand_() % layer_dim;
    if (n1 == n2) continue;
    ++i;
    const int output_layer_dim = fps[b]->shape(0);
    const float* fin = endur_[a].data();
    const float* fout = endur_[b].data();
    float* pin = prune_[a].data();
    float* pout = prune_[b].data();
    int before = 0, after = 0;
    for (int j = 0; j < input_layer_dim; ++j) {
      const int64_t r1 = (int64_t)n1 * input_layer_dim + j, r2 = (int64_t)n2 * input_layer_dim + j;
      if (pin[r1] < eps && fin[r1] < 0) before += 1;
      if (pin[r2] < eps && fin[r1] < 0) after += 1;
      if (pin[r2] < eps && fin[r2] < 0) before += 1;
      if (pin[r1] < eps && fin[r2] < 0) after += 1;
    }
    for (int j = 0; j < output_layer_dim; ++j) {
      const int64_t c1 = (int64_t)j * layer_dim + n1, c2 = (int64_t)j * layer_dim + n2;
      if (pout[c1] < eps && fout[c1] < 0) before += 1;
      if (pout[c2] < eps && fout[c1] < 0) after += 1;
      if (pout[c2] < eps && fout[c2] < 0) before += 1;
      if (pout[c1] < eps && fout[c2] < 0) after += 1;
    }
    if (after < before) {
      ++accepted_;
      auto& rp = rowp[a];
      if (rp.empty()) {
        rp.resize(layer_dim);
        std::iota(rp.begin(), rp.end(), 0);
      }
      std::swap(rp[n1], rp[n2]);
      auto& cp = colp[b];
      if (cp.empty()) {
        cp.resize(fps[b]->shape(1));
        std::iota(cp.begin(), cp.end(), 0);
      }
      std::swap(cp[n1], cp[n2]);
      // prune input rows
      std::swap_ranges(pin + (int64_t)n1 * input_layer_dim, pin + (int64_t)(n1 + 1) * input_layer_dim,
                       pin + (int64_t)n2 * input_layer_dim);
      if (reference_compat) {
        std::swap(pin[n1], pin[n2]);  // Q9: flat elements of the weight array
      } else if (a + 1 < (int)prune_.size() && (int)prune_[a + 1].size() == layer_dim) {
        std::swap(prune_[a + 1][n1], prune_[a + 1][n2]);  // the prune bias, as intended
      }
      for (int k = 0; k < output_layer_dim; ++k)
        std::swap(pout[(int64_t)k * layer_dim + n1], pout[(int64_t)k * layer_dim + n2]);
    }
  }
  after_ = CalculateOverallDist();
  if (this->solver_) {
    std::ostringstream o;
    o << "dist: before: " << before_ << " after: " << after_;
    this->solver_->emit_log(o.str());
  }
  for (size_t p = 0; p < fps.size(); ++p) {
    const bool rows = !rowp[p].empty(), cols = !colp[p].empty();
    if (!rows && !cols) continue;
    permute_blob(fps[p], rows ? &rowp[p] : nullptr, cols ? &colp[p] : nullptr);
    // the bias follows its neuron's row (strategy.cpp:250-255)
    if (rows && p + 1 < fps.size() && fps[p + 1]->count() == fps[p]->shape(0) && fps[p + 1]->num_axes() == 1)
      permute_blob(fps[p + 1], &rowp[p], nullptr);
  }
  HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
}

template class RemappingFailureStrategy<float>;
template class GeneticFailureStrategy<float>;

}  // namespace caffe
