// Layer implementations (device-only) + registry + fillers.
#include "layers.hpp"

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <fstream>

#include "hdf5.hpp"

namespace caffe {

// ---------------------------------------------------------------- base
template <typename Dtype>
Dtype Layer<Dtype>::Forward(const std::vector<Blob<Dtype>*>& bottom,
                            const std::vector<Blob<Dtype>*>& top) {
  Reshape(bottom, top);
  Forward_gpu(bottom, top);
  return Dtype(0);  // loss is read from the loss tops by Net (no per-layer sync)
}

template <typename Dtype>
void Layer<Dtype>::CheckBlobCounts(const std::vector<Blob<Dtype>*>& bottom,
                                   const std::vector<Blob<Dtype>*>& top) {
  const std::string nm = name() + " (" + type() + ")";
  if (ExactNumBottomBlobs() >= 0)
    CAFFE_CHECK((int)bottom.size() == ExactNumBottomBlobs(), nm << " takes " << ExactNumBottomBlobs() << " bottom blob(s)");
  if (MinBottomBlobs() >= 0)
    CAFFE_CHECK((int)bottom.size() >= MinBottomBlobs(), nm << " takes at least " << MinBottomBlobs() << " bottom blob(s)");
  if (ExactNumTopBlobs() >= 0)
    CAFFE_CHECK((int)top.size() == ExactNumTopBlobs(), nm << " produces " << ExactNumTopBlobs() << " top blob(s)");
  if (MinTopBlobs() >= 0)
    CAFFE_CHECK((int)top.size() >= MinTopBlobs(), nm << " produces at least " << MinTopBlobs() << " top blob(s)");
  if (EqualNumBottomTopBlobs())
    CAFFE_CHECK(bottom.size() == top.size(), nm << " needs equal bottom and top counts");
}

template <typename Dtype>
void Layer<Dtype>::SetLossWeights(const std::vector<Blob<Dtype>*>& top) {
  auto lw = layer_param_.nums("loss_weight");
  loss_.assign(top.size(), Dtype(0));
  if (!lw.empty()) {
    CAFFE_CHECK(lw.size() == top.size(), name() << ": loss_weight must be given for every top");
    for (size_t i = 0; i < top.size(); ++i) loss_[i] = static_cast<Dtype>(lw[i]);
  } else if (IsLoss() && !top.empty()) {
    loss_[0] = Dtype(1);
  }
}

template <typename Dtype>
std::map<std::string, typename LayerRegistry<Dtype>::Creator>& LayerRegistry<Dtype>::Registry() {
  static std::map<std::string, Creator> r;
  return r;
}
template <typename Dtype>
std::shared_ptr<Layer<Dtype>> LayerRegistry<Dtype>::CreateLayer(const Msg& param) {
  const std::string t = param.str("type");
  auto& r = Registry();
  auto it = r.find(t);
  CAFFE_CHECK(it != r.end(), "Unknown layer type: " << t << " (layer " << param.str("name") << ")");
  return it->second(param);
}
template <typename Dtype>
std::vector<std::string> LayerRegistry<Dtype>::LayerTypeList() {
  std::vector<std::string> v;
  for (auto& kv : Registry()) v.push_back(kv.first);
  return v;
}

template class Layer<float>;
template class LayerRegistry<float>;

// --------------------------------------------------------------- fillers
static uint32_t hash32(const std::string& s) {
  uint32_t h = 2166136261u;
  for (unsigned char c : s) h = (h ^ c) * 16777619u;
  return h;
}

void FillBlob(Blob<float>* blob, const Msg& f, uint64_t seed, uint32_t sid) {
  const std::string type = f.str("type", "constant");
  const int64_t n = blob->count();
  float* d = blob->mutable_gpu_data();
  const rram_stream_t s = Caffe::stream();
  auto fan = [&](bool in) -> double {
    if (blob->num_axes() < 2) return (double)n;
    return in ? (double)n / blob->shape(0) : (double)n / blob->shape(1);
  };
  auto norm_n = [&]() -> double {
    const std::string vn = f.str("variance_norm", "FAN_IN");
    if (vn == "FAN_OUT") return fan(false);
    if (vn == "AVERAGE") return (fan(true) + fan(false)) / 2.0;
    return fan(true);
  };
  if (type == "constant") {
    RRAM_CALL(rram_set(n, static_cast<float>(f.num("value", 0.0)), d, s));
  } else if (type == "gaussian") {
    RRAM_CALL(rram_fill_gaussian(d, n, static_cast<float>(f.num("mean", 0.0)),
                                 static_cast<float>(f.num("std", 1.0)), seed, sid, s));
    CAFFE_CHECK(f.integer("sparse", -1) < 0, "gaussian filler: sparse is not supported");
  } else if (type == "uniform") {
    RRAM_CALL(rram_fill_uniform(d, n, static_cast<float>(f.num("min", 0.0)),
                                static_cast<float>(f.num("max", 1.0)), seed, sid, s));
  } else if (type == "xavier") {  // filler.hpp XavierFiller: U(-sqrt(3/n), sqrt(3/n))
    const float sc = static_cast<float>(std::sqrt(3.0 / norm_n()));
    RRAM_CALL(rram_fill_uniform(d, n, -sc, sc, seed, sid, s));
  } else if (type == "msra") {  // MSRAFiller: N(0, sqrt(2/n))
    RRAM_CALL(rram_fill_gaussian(d, n, 0.0f, static_cast<float>(std::sqrt(2.0 / norm_n())), seed, sid, s));
  } else {
    throw Error("Unknown filler type: " + type);
  }
}

static std::vector<int> ints_of(const Msg& m, const std::string& k) {
  std::vector<int> r;
  for (double v : m.nums(k)) r.push_back(static_cast<int>(v));
  return r;
}

// Caffe's kernel/stride/pad parsing (base_conv_layer.cpp:19-110, 2-D case)
static void hw_param(const Msg& p, const std::string& base, int def, int& h, int& w) {
  if (p.has(base + "_h") || p.has(base + "_w")) {
    h = static_cast<int>(p.integer(base + "_h", def));
    w = static_cast<int>(p.integer(base + "_w", def));
    return;
  }
  const std::string key = base == "kernel" ? "kernel_size" : base;
  auto v = ints_of(p, key);
  if (v.empty()) {
    h = w = def;
  } else if (v.size() == 1) {
    h = w = v[0];
  } else {
    h = v[0];
    w = v[1];
  }
}

// ★ ------------------------------------------------------- Convolution
template <typename Dtype>
void ConvolutionLayer<Dtype>::LayerSetUp(const std::vector<Blob<Dtype>*>& bottom,
                                         const std::vector<Blob<Dtype>*>& top) {
  const Msg& cp = this->layer_param_.sub_or_empty("convolution_param");
  CAFFE_CHECK(bottom[0]->num_axes() == 4, "Convolution: only 2-D (4-axis) inputs are supported");
  int kh, kw, sh, sw, ph, pw, dh, dw;
  hw_param(cp, "kernel", 0, kh, kw);
  hw_param(cp, "stride", 1, sh, sw);
  hw_param(cp, "pad", 0, ph, pw);
  hw_param(cp, "dilation", 1, dh, dw);
  CAFFE_CHECK(kh > 0 && kw > 0, "Convolution: kernel size must be given and > 0");
  desc_ = rram_conv_desc{0, bottom[0]->shape(1), 0, 0, (int)cp.integer("num_output", 0), kh, kw, ph, pw,
                         sh, sw, dh, dw, (int)cp.integer("group", 1), 0, 0};
  CAFFE_CHECK(desc_.num_output > 0, "Convolution: num_output must be > 0");
  CAFFE_CHECK(desc_.channels % desc_.group == 0 && desc_.num_output % desc_.group == 0,
              "Convolution: channels/num_output must be divisible by group");
  bias_term_ = cp.boolean("bias_term", true);
  this->blobs_.clear();
  this->blobs_.push_back(std::make_shared<Blob<Dtype>>(
      std::vector<int>{desc_.num_output, desc_.channels / desc_.group, kh, kw}));
  const uint64_t seed = Caffe::seed() ^ (uint64_t)hash32(this->name()) << 20;
  FillBlob(this->blobs_[0].get(), cp.sub_or_empty("weight_filler"), seed, 0);
  if (bias_term_) {
    this->blobs_.push_back(std::make_shared<Blob<Dtype>>(std::vector<int>{desc_.num_output}));
    FillBlob(this->blobs_[1].get(), cp.sub_or_empty("bias_filler"), seed, 1);
  }
  this->param_propagate_down_.assign(this->blobs_.size(), true);
}

template <typename Dtype>
void ConvolutionLayer<Dtype>::Reshape(const std::vector<Blob<Dtype>*>& bottom,
                                      const std::vector<Blob<Dtype>*>& top) {
  CAFFE_CHECK(bottom[0]->shape(1) == desc_.channels, this->name() << ": input channels changed");
  desc_.num = bottom[0]->shape(0);
  desc_.height = bottom[0]->shape(2);
  desc_.width = bottom[0]->shape(3);
  RRAM_CALL(rram_conv_out_shape(&desc_));
  top[0]->Reshape({desc_.num, desc_.num_output, desc_.out_h, desc_.out_w});
  const int eng = rram_get_f32_engine();
  if (desc_.num != oct_key_[0] || desc_.height != oct_key_[1] || desc_.width != oct_key_[2] || eng != oct_key_[3]) {
    want_in_oct_ = rram_conv_input_octets(&desc_) == 1;
    oct_key_[0] = desc_.num;
    oct_key_[1] = desc_.height;
    oct_key_[2] = desc_.width;
    oct_key_[3] = eng;
  }
  // ask the producer of the input for its octet companion
  if (want_in_oct_) bottom[0]->data()->wants_octets = true;
  flip_ok_ = this->phase_ == TRAIN && rram_conv2d_flip_applies(&desc_) == 1;
}

template <typename Dtype>
bool ConvolutionLayer<Dtype>::flip_geometry(int* g, int* cin_g, int* cout_g, int* taps) const {
  if (!flip_ok_) return false;
  *g = desc_.group;
  *cin_g = desc_.channels / desc_.group;
  *cout_g = desc_.num_output / desc_.group;
  *taps = desc_.kernel_h * desc_.kernel_w;
  return true;
}

// the octet companion a producer writes next to top (nullptr: not wanted).
// RRAM_OCTETS selects the producers: 0 none (every convolution packs its
// input), 1 (default) all, 2 the fused LRN + max pool only.  Measured on
// MI355X (AlexNet b256, per-layer hipEvents): round 2 (profiles/
// r02_ab_octets.txt) the epilogue companions lost (conv3's epilogue +40 us /
// conv4 -35, conv4's +40 / conv5 -32); round 3, with conv5 at two workgroups
// per CU and per-image conv2 tiles, all producers win by 8 us per map
// (conv3 +30, conv4 +3, conv5 -41: 112.7-113.3k vs 112.1-113.1k images/s,
// profiles/r03_ab_octets.txt).
enum OctetProducer { kOctConv = 1, kOctPool = 2 };
bool octets_enabled(int producer) {
  static const int mode = [] {
    const char* e = std::getenv("RRAM_OCTETS");
    return e ? std::atoi(e) : 1;
  }();
  return mode == 1 || (mode == 2 && producer == kOctPool);
}
template <typename Dtype>
void* octets_for(Blob<Dtype>* top, int producer) {
  SyncedMemory* m = top->data().get();
  if (!octets_enabled(producer) || !m->wants_octets || top->num_axes() != 4 || top->shape(1) % 8 != 0)
    return nullptr;
  return m->octets(static_cast<size_t>(top->count()) * 6);
}
template <typename Dtype>
void mark_octets(Blob<Dtype>* top) {
  const int shp[4] = {top->shape(0), top->shape(1), top->shape(2), top->shape(3)};
  top->data()->set_octets_valid(shp);
}

template <typename Dtype>
void ConvolutionLayer<Dtype>::Forward_gpu(const std::vector<Blob<Dtype>*>& bottom,
                                          const std::vector<Blob<Dtype>*>& top) {
  CAFFE_CHECK(bottom[0] != top[0], this->name() << ": in-place convolution is not allowed");
  const int shp[4] = {desc_.num, desc_.channels, desc_.height, desc_.width};
  const void* xo = nullptr;
  if (want_in_oct_) {
    // the input's companion: written by its producer, else packed here into
    // the blob's own companion so the other consumers of the same blob (the
    // inception branches) reuse it instead of each packing a scratch copy
    SyncedMemory* xm = bottom[0]->data().get();
    xo = xm->valid_octets(shp);
    CAFFE_CHECK(xo != nullptr || !xm->fp32_stale,
                this->name() << ": input companion invalid while its producer skipped the fp32 output");
    if (xo == nullptr) {
      void* buf = xm->octets(static_cast<size_t>(bottom[0]->count()) * 6);
      RRAM_CALL(rram_pack_octets(bottom[0]->gpu_data(), buf, shp[0], shp[1], shp[2], shp[3], Caffe::stream()));
      xm->set_octets_valid(shp);
      xo = buf;
    }
  }
  // without a companion the kernel reads the fp32 bottom: it must have been
  // written (a pooled-output fold decided at the producer's forward against
  // an engine / plan that no longer holds would leave it stale)
  CAFFE_CHECK(xo != nullptr || !bottom[0]->data()->fp32_stale,
              this->name() << ": fp32 input unwritten (its producer wrote only the octet companion)");
  const float* bias = bias_term_ ? this->blobs_[1]->gpu_data() : nullptr;
  const size_t wpb = cache_wpack ? rram_conv_weight_pack_bytes(&desc_) : 0;
  if (concat_top_ != nullptr) {
    // TEST-phase Concat fold: straight into the Concat top's channel slice
    // (replaces concat_layer.cu's copy of this bottom); top[0] stays unwritten
    const int64_t hw = (int64_t)desc_.out_h * desc_.out_w;
    CAFFE_CHECK(concat_top_->num_axes() == 4 && concat_top_->shape(0) == desc_.num &&
                    concat_top_->count(2) == hw && concat_off_ + desc_.num_output <= concat_top_->shape(1),
                this->name() << ": folded Concat top " << concat_top_->shape_string() << " does not fit");
    float* yc = concat_top_->mutable_gpu_data() + concat_off_ * hw;
    void* wp = nullptr;
    int wvalid = 0;
    uint64_t key = 0;
    SyncedMemory* wm = this->blobs_[0]->data().get();
    if (wpb > 0) {
      const int* f = reinterpret_cast<const int*>(&desc_);
      key = 1469598103934665603ull;
      for (size_t i = 0; i < sizeof(rram_conv_desc) / sizeof(int); ++i) key = (key ^ (uint32_t)f[i]) * 1099511628211ull;
      key = (key ^ (uint64_t)rram_get_f32_engine()) * 1099511628211ull;
      (void)this->blobs_[0]->gpu_data();
      wp = wm->wpack(wpb);
      wvalid = wm->wpack_valid(key) ? 1 : 0;
    }
    RRAM_CALL(rram_conv2d_fwd_strided(&desc_, bottom[0]->gpu_data(), xo, this->blobs_[0]->gpu_data(), wp, wvalid,
                                      bias, yc, (int64_t)concat_top_->shape(1) * hw, fused_relu ? 1 : 0,
                                      Caffe::stream()));
    if (wpb > 0) wm->set_wpack_valid(key);
    return;
  }
  float* y = top[0]->mutable_gpu_data();  // invalidates top's companion
  void* yo = octets_for(top[0], kOctConv);
  // convolution-output fold: the only reader takes the companion, so the
  // fp32 top is not written (materialised on demand by Net::materialize_blob)
  const bool skip_y = yo != nullptr && octet_reader_ != nullptr && octet_reader_->input_octets_now(top[0]) &&
                      rram_conv_output_octets_only(&desc_) == 1;
  if (skip_y) y = nullptr;
  if (wpb > 0) {
    // the pack is valid for this layer's shape and engine until the weights'
    // next mutable access (the MC driver's injection, a solver update, ...)
    SyncedMemory* wm = this->blobs_[0]->data().get();
    // key: every field of the descriptor (the pack layout follows the tile
    // plan, which depends on kernel / stride / pad / dilation and the output
    // shape) plus the engine, so two convolutions sharing one weight blob
    // never read each other's pack
    const int* f = reinterpret_cast<const int*>(&desc_);
    uint64_t key = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(rram_conv_desc) / sizeof(int); ++i) key = (key ^ (uint32_t)f[i]) * 1099511628211ull;
    key = (key ^ (uint64_t)rram_get_f32_engine()) * 1099511628211ull;
    const float* w = this->blobs_[0]->gpu_data();
    void* wp = wm->wpack(wpb);
    RRAM_CALL(rram_conv2d_fwd_cached(&desc_, bottom[0]->gpu_data(), xo, w, wp, wm->wpack_valid(key) ? 1 : 0, bias, y,
                                     yo, fused_relu ? 1 : 0, Caffe::stream()));
    wm->set_wpack_valid(key);
  } else {
    RRAM_CALL(rram_conv2d_fwd_octets(&desc_, bottom[0]->gpu_data(), xo, this->blobs_[0]->gpu_data(), bias, y, yo,
                                     fused_relu ? 1 : 0, Caffe::stream()));
  }
  if (yo) mark_octets(top[0]);
  top[0]->data()->fp32_stale = skip_y;
}

template <typename Dtype>
void ConvolutionLayer<Dtype>::Backward_gpu(const std::vector<Blob<Dtype>*>& top,
                                           const std::vector<bool>& pd,
                                           const std::vector<Blob<Dtype>*>& bottom) {
  const bool dw = this->param_propagate_down(0);
  const bool db = bias_term_ && this->param_propagate_down(1);
  const bool dx = pd.size() > 0 && pd[0];
  if (!dw && !db && !dx) return;
  const size_t need = rram_conv2d_bwd_workspace(&desc_, 1);
  // chunk up to 256 images per col buffer (bounded at 1 GiB), plus the
  // weight-gradient split-K partials (64 before round 4: CIFAR conv2 at b100
  // then ran two im2col + weight-GEMM + split-K passes instead of one)
  int imgs = std::max(1, std::min(desc_.num, (int)std::min<size_t>(256, (1ull << 30) / std::max<size_t>(need, 1))));
  void* ws = Caffe::workspace(rram_conv2d_bwd_workspace(&desc_, imgs) + 256);
  // the flipped kernel the last fused update of this Solver::Step call wrote
  // next to the weights (Solver::FusedTail), unless a graph is being captured
  // (a replay must not depend on the host-side companion state)
  const float* wf = nullptr;
  SyncedMemory& wm = *this->blobs_[0]->data();
  if (dx && flip_ok_ && wm.wflip_valid(Caffe::step_epoch()) && !stream_capturing())
    wf = static_cast<const float*>(wm.wflip(0));
  RRAM_CALL(rram_conv2d_bwd_ex(&desc_, bottom[0]->gpu_data(), this->blobs_[0]->gpu_data(), wf,
                               top[0]->gpu_diff(), dw ? this->blobs_[0]->mutable_gpu_diff() : nullptr,
                               db ? this->blobs_[1]->mutable_gpu_diff() : nullptr,
                               dx ? bottom[0]->mutable_gpu_diff() : nullptr, ws, Caffe::workspace_size(),
                               Caffe::stream()));
}

// ★ ------------------------------------------------------ InnerProduct
template <typename Dtype>
void InnerProductLayer<Dtype>::LayerSetUp(const std::vector<Blob<Dtype>*>& bottom,
                                          const std::vector<Blob<Dtype>*>& top) {
  const Msg& ip = this->layer_param_.sub_or_empty("inner_product_param");
  N_ = static_cast<int>(ip.integer("num_output", 0));
  CAFFE_CHECK(N_ > 0, this->name() << ": num_output must be > 0");
  bias_term_ = ip.boolean("bias_term", true);
  transpose_ = ip.boolean("transpose", false);
  axis_ = static_cast<int>(ip.integer("axis", 1));
  if (axis_ < 0) axis_ += bottom[0]->num_axes();
  K_ = static_cast<int>(bottom[0]->count(axis_));
  this->blobs_.clear();
  this->blobs_.push_back(std::make_shared<Blob<Dtype>>(
      transpose_ ? std::vector<int>{K_, N_} : std::vector<int>{N_, K_}));
  const uint64_t seed = Caffe::seed() ^ (uint64_t)hash32(this->name()) << 20;
  FillBlob(this->blobs_[0].get(), ip.sub_or_empty("weight_filler"), seed, 0);
  if (bias_term_) {
    this->blobs_.push_back(std::make_shared<Blob<Dtype>>(std::vector<int>{N_}));
    FillBlob(this->blobs_[1].get(), ip.sub_or_empty("bias_filler"), seed, 1);
  }
  this->param_propagate_down_.assign(this->blobs_.size(), true);
}

template <typename Dtype>
void InnerProductLayer<Dtype>::Reshape(const std::vector<Blob<Dtype>*>& bottom,
                                       const std::vector<Blob<Dtype>*>& top) {
  CAFFE_CHECK(bottom[0]->count(axis_) == K_, this->name() << ": input size incompatible with weights");
  M_ = static_cast<int>(bottom[0]->count(0, axis_));
  std::vector<int> s(bottom[0]->shape().begin(), bottom[0]->shape().begin() + axis_);
  s.push_back(N_);
  top[0]->Reshape(s);
  // TEST phase on the bf16x6 engine: ask the producer of the input for its
  // packed-row form (an InnerProduct producer writes it from its split-K
  // reduce: fc6 -> fc7), key = (M, K, rows per tile)
  in_rows_key_ = 0;
  int bmc = 0;
  const size_t rb = (this->phase_ == TEST && !transpose_)
                        ? rram_ip_rows_pack_bytes(M_, N_, K_, ws_request(), &bmc)
                        : 0;
#ifndef RRAM_IP_ROWS  // A/B builds: 0 = every InnerProduct packs its own input
#define RRAM_IP_ROWS 1
#endif
  if (RRAM_IP_ROWS && rb > 0 && bmc > 0 && bmc < 4096) {
    in_rows_key_ = (static_cast<uint64_t>(M_) << 40) | (static_cast<uint64_t>(K_) << 12) | static_cast<uint64_t>(bmc);
    bottom[0]->data()->wants_rows = in_rows_key_;
    bottom[0]->data()->wants_rows_bytes = rb;
  }
}

template <typename Dtype>
void InnerProductLayer<Dtype>::Forward_gpu(const std::vector<Blob<Dtype>*>& bottom,
                                           const std::vector<Blob<Dtype>*>& top) {
  void* ws = Caffe::workspace(ws_request());
  // the packed-row companions (TEST, Reshape): read the input's when its
  // producer wrote it, write the output's when the consumer asked
  const void* xr = in_rows_key_ ? bottom[0]->data()->valid_rows(in_rows_key_) : nullptr;
  SyncedMemory& ym = *top[0]->data();
  const uint64_t ykey = (this->phase_ == TEST && !transpose_) ? ym.wants_rows : 0;
  if (xr != nullptr || ykey != 0) {
    float* y = top[0]->mutable_gpu_data();  // (drops the old companion; written again below)
    void* yr = ykey ? ym.rows(ym.wants_rows_bytes) : nullptr;
    int written = 0;
    RRAM_CALL(rram_ip_fwd_rows(bottom[0]->gpu_data(), xr, this->blobs_[0]->gpu_data(),
                               bias_term_ ? this->blobs_[1]->gpu_data() : nullptr, y, yr,
                               static_cast<int>(ykey & 0xFFF), M_, N_, K_, fused_relu ? 1 : 0, ws,
                               Caffe::workspace_size(), &written, Caffe::stream()));
    if (written) ym.set_rows_valid(ykey);
    return;
  }
  RRAM_CALL(rram_ip_fwd(bottom[0]->gpu_data(), this->blobs_[0]->gpu_data(),
                        bias_term_ ? this->blobs_[1]->gpu_data() : nullptr,
                        top[0]->mutable_gpu_data(), M_, N_, K_, transpose_ ? 1 : 0,
                        fused_relu ? 1 : 0, ws, Caffe::workspace_size(), Caffe::stream()));
}

template <typename Dtype>
void InnerProductLayer<Dtype>::Backward_gpu(const std::vector<Blob<Dtype>*>& top,
                                            const std::vector<bool>& pd,
                                            const std::vector<Blob<Dtype>*>& bottom) {
  RRAM_CALL(rram_ip_bwd(bottom[0]->gpu_data(), this->blobs_[0]->gpu_data(), top[0]->gpu_diff(),
                        this->param_propagate_down(0) ? this->blobs_[0]->mutable_gpu_diff() : nullptr,
                        (bias_term_ && this->param_propagate_down(1)) ? this->blobs_[1]->mutable_gpu_diff() : nullptr,
                        (pd.size() && pd[0]) ? bottom[0]->mutable_gpu_diff() : nullptr, M_, N_, K_,
                        transpose_ ? 1 : 0, Caffe::stream()));
}

// ------------------------------------------------------------------ ReLU
template <typename Dtype>
void ReLULayer<Dtype>::Forward_gpu(const std::vector<Blob<Dtype>*>& bottom,
                                   const std::vector<Blob<Dtype>*>& top) {
  if (folded) return;  // applied in the producer's epilogue / output store
  RRAM_CALL(rram_relu_fwd(bottom[0]->gpu_data(), top[0]->mutable_gpu_data(), bottom[0]->count(),
                          negative_slope(), Caffe::stream()));
}
template <typename Dtype>
void ReLULayer<Dtype>::Backward_gpu(const std::vector<Blob<Dtype>*>& top, const std::vector<bool>& pd,
                                    const std::vector<Blob<Dtype>*>& bottom) {
  if (!pd.size() || !pd[0] || bwd_folded) return;  // bwd_folded: applied by the consumer's backward
  // in-place: bottom data is the ReLU output; x > 0 <=> y > 0 for slope 0 (relu_layer.cu:35-44)
  RRAM_CALL(rram_relu_bwd(bottom[0]->gpu_data(), top[0]->gpu_diff(), bottom[0]->mutable_gpu_diff(),
                          bottom[0]->count(), negative_slope(), Caffe::stream()));
}

// ----------------------------------------------------------------- Split
template <typename Dtype>
void SplitLayer<Dtype>::Reshape(const std::vector<Blob<Dtype>*>& bottom,
                                const std::vector<Blob<Dtype>*>& top) {
  for (auto* t : top) {
    t->ReshapeLike(*bottom[0]);
    t->ShareData(*bottom[0]);
  }
}
template <typename Dtype>
void SplitLayer<Dtype>::Backward_gpu(const std::vector<Blob<Dtype>*>& top, const std::vector<bool>& pd,
                                     const std::vector<Blob<Dtype>*>& bottom) {
  if (!pd.size() || !pd[0]) return;
  const int64_t n = bottom[0]->count();
  if (top.size() == 1) {
    HIP_CALL(hipMemcpyAsync(bottom[0]->mutable_gpu_diff(), top[0]->gpu_diff(), n * sizeof(Dtype),
                            hipMemcpyDeviceToDevice, Caffe::hip_stream()));
    return;
  }
  RRAM_CALL(rram_add(n, top[0]->gpu_diff(), top[1]->gpu_diff(), bottom[0]->mutable_gpu_diff(), Caffe::stream()));
  for (size_t i = 2; i < top.size(); ++i)
    RRAM_CALL(rram_axpy(n, 1.0f, top[i]->gpu_diff(), bottom[0]->mutable_gpu_diff(), Caffe::stream()));
}

// --------------------------------------------------------------- Pooling
template <typename Dtype>
class PoolingLayer : public Layer<Dtype> {
 public:
  explicit PoolingLayer(const Msg& p) : Layer<Dtype>(p) {}
  const char* type() const override { return "Pooling"; }
  int ExactNumBottomBlobs() const override { return 1; }
  int MinTopBlobs() const override { return 1; }
  void LayerSetUp(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    const Msg& pp = this->layer_param_.sub_or_empty("pooling_param");
    const std::string pool = pp.str("pool", "MAX");
    CAFFE_CHECK(pool == "MAX" || pool == "AVE", this->name() << ": pool " << pool << " not supported");
    method_ = pool == "MAX" ? RRAM_POOL_MAX : RRAM_POOL_AVE;
    // pooling_layer.hpp:29-33: MAX may publish its argmax as a second top
    CAFFE_CHECK(top.size() == 1 || (top.size() == 2 && method_ == RRAM_POOL_MAX),
                this->name() << ": Pooling produces 1 top (2 for MAX: output and mask)");
    top_mask_ = top.size() > 1;
    global_ = pp.boolean("global_pooling", false);
    hw_param(pp, "kernel", 0, kh_, kw_);
    hw_param(pp, "stride", 1, sh_, sw_);
    hw_param(pp, "pad", 0, ph_, pw_);
    if (!global_) CAFFE_CHECK(kh_ > 0 && kw_ > 0, this->name() << ": kernel size required");
    (void)bottom;
  }
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    C_ = bottom[0]->shape(1);
    H_ = bottom[0]->shape(2);
    W_ = bottom[0]->shape(3);
    if (global_) {
      kh_ = H_;
      kw_ = W_;
    }
    // pooling_layer.cpp:90-104
    PH_ = (int)std::ceil((float)(H_ + 2 * ph_ - kh_) / sh_) + 1;
    PW_ = (int)std::ceil((float)(W_ + 2 * pw_ - kw_) / sw_) + 1;
    if (ph_ || pw_) {
      if ((PH_ - 1) * sh_ >= H_ + ph_) --PH_;
      if ((PW_ - 1) * sw_ >= W_ + pw_) --PW_;
    }
    top[0]->Reshape({bottom[0]->shape(0), C_, PH_, PW_});
    if (top.size() > 1) top[1]->ReshapeLike(*top[0]);
    if (method_ == RRAM_POOL_MAX) mask_.Reshape(top[0]->shape());
  }

  bool fuse_lrn_before(Blob<Dtype>* lrn_bottom, int size, float alpha, float beta, float k) override {
    if (this->phase_ != TEST || method_ != RRAM_POOL_MAX || global_ || top_mask_ || kh_ != kw_ || (kh_ != 2 && kh_ != 3) ||
        ph_ >= kh_ || pw_ >= kw_ || (size != 3 && size != 5))
      return false;
    lrn_src_ = lrn_bottom;
    if (lrn_bottom == nullptr) octet_reader_ = nullptr;  // a plain pool writes its top
    lrn_size_ = size;
    lrn_alpha_ = alpha;
    lrn_beta_ = beta;
    lrn_k_ = k;
    return true;
  }
  bool set_octet_reader(Layer<Dtype>* reader) override {
    if (reader != nullptr && lrn_src_ == nullptr) return false;
    octet_reader_ = reader;
    return true;
  }
  bool fuse_relu_before_bwd(float slope) override {
    if (this->phase_ != TRAIN) return false;
    relu_bwd_ = true;
    relu_bwd_slope_ = slope;
    return true;
  }
  bool fuse_relu_after(float slope) override {
    if (lrn_src_ != nullptr) return false;  // the LRN + pool kernel has no ReLU store
    relu_ = true;
    relu_slope_ = slope;
    return true;
  }

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    if (lrn_src_ != nullptr) {  // LRN folded into this pool (Net::Net, TEST phase)
      float* y = top[0]->mutable_gpu_data();
      void* yo = octets_for(top[0], kOctPool);
      // pooled-output fold: the only reader takes the companion, so the fp32
      // top is not written (materialised on demand by Net::materialize_blob)
      const bool skip_y = yo != nullptr && octet_reader_ != nullptr && octet_reader_->input_octets_now(top[0]);
      RRAM_CALL(rram_lrn_maxpool_fwd_octets(lrn_src_->gpu_data(), skip_y ? nullptr : y, yo, bottom[0]->shape(0), C_,
                                            H_, W_, PH_, PW_, kh_, sh_, sw_, ph_, pw_, lrn_size_, lrn_alpha_,
                                            lrn_beta_, lrn_k_, Caffe::stream()));
      if (yo) mark_octets(top[0]);
      top[0]->data()->fp32_stale = skip_y;
      return;
    }
    const bool top_mask = top.size() > 1;
    int* mask = (method_ == RRAM_POOL_MAX && (this->phase_ == TRAIN || top_mask))
                    ? reinterpret_cast<int*>(mask_.mutable_gpu_data()) : nullptr;
    if (relu_)  // the in-place ReLU that follows (Net::Net fold), in the same store
      RRAM_CALL(rram_pool_relu_fwd(bottom[0]->gpu_data(), top[0]->mutable_gpu_data(), mask, bottom[0]->shape(0), C_,
                                   H_, W_, PH_, PW_, kh_, kw_, sh_, sw_, ph_, pw_, method_, relu_slope_,
                                   Caffe::stream()));
    else
      RRAM_CALL(rram_pool_fwd(bottom[0]->gpu_data(), top[0]->mutable_gpu_data(), mask, bottom[0]->shape(0), C_, H_,
                              W_, PH_, PW_, kh_, kw_, sh_, sw_, ph_, pw_, method_, Caffe::stream()));
    // the top mask holds the argmax index as a float (pooling_layer.cu:30-34)
    if (top_mask) RRAM_CALL(rram_i32_to_f32(mask, top[1]->mutable_gpu_data(), top[1]->count(), Caffe::stream()));
  }
  void Backward_gpu(const std::vector<Blob<Dtype>*>& top, const std::vector<bool>& pd,
                    const std::vector<Blob<Dtype>*>& bottom) override {
    if (!pd.size() || !pd[0]) return;
    CAFFE_CHECK(method_ != RRAM_POOL_MAX || this->phase_ == TRAIN, "MAX pool backward needs TRAIN phase");
    // relu_bwd_: the in-place ReLU before this pool (Net::Net fold); its output is our bottom data
    RRAM_CALL(rram_pool_relu_bwd(top[0]->gpu_diff(),
                                 method_ == RRAM_POOL_MAX ? reinterpret_cast<const int*>(mask_.gpu_data()) : nullptr,
                                 bottom[0]->mutable_gpu_diff(), bottom[0]->shape(0), C_, H_, W_, PH_, PW_, kh_, kw_,
                                 sh_, sw_, ph_, pw_, method_, relu_bwd_ ? bottom[0]->gpu_data() : nullptr,
                                 relu_bwd_slope_, Caffe::stream()));
  }
  int method_ = RRAM_POOL_MAX, kh_ = 0, kw_ = 0, sh_ = 1, sw_ = 1, ph_ = 0, pw_ = 0;
  int C_ = 0, H_ = 0, W_ = 0, PH_ = 0, PW_ = 0;
  bool global_ = false, top_mask_ = false, relu_ = false, relu_bwd_ = false;
  float relu_slope_ = 0.0f, relu_bwd_slope_ = 0.0f;
  Blob<Dtype> mask_;
  Blob<Dtype>* lrn_src_ = nullptr;  // bottom of a folded LRN (nullptr: unfused)
  Layer<Dtype>* octet_reader_ = nullptr;  // pooled-output fold: the top's only reader
  int lrn_size_ = 5;
  float lrn_alpha_ = 1, lrn_beta_ = 0.75f, lrn_k_ = 1;
};

// -------------------------------------------------------------------- LRN
template <typename Dtype>
class LRNLayer : public Layer<Dtype> {
 public:
  explicit LRNLayer(const Msg& p) : Layer<Dtype>(p) {}
  const char* type() const override { return "LRN"; }
  int ExactNumBottomBlobs() const override { return 1; }
  int ExactNumTopBlobs() const override { return 1; }
  void LayerSetUp(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>&) override {
    const Msg& lp = this->layer_param_.sub_or_empty("lrn_param");
    size_ = (int)lp.integer("local_size", 5);
    alpha_ = (float)lp.num("alpha", 1.0);
    beta_ = (float)lp.num("beta", 0.75);
    k_ = (float)lp.num("k", 1.0);
    const std::string region = lp.str("norm_region", "ACROSS_CHANNELS");
    CAFFE_CHECK(region == "ACROSS_CHANNELS" || region == "WITHIN_CHANNEL",
                this->name() << ": unknown norm_region " << region);
    within_ = region == "WITHIN_CHANNEL";
    CAFFE_CHECK(size_ % 2 == 1, "LRN only supports odd values for local_size");
  }
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    top[0]->ReshapeLike(*bottom[0]);
    if (this->phase_ == TRAIN) scale_.ReshapeLike(*bottom[0]);
  }
  bool lrn_params(int& size, float& alpha, float& beta, float& k) const override {
    if (within_) return false;
    size = size_;
    alpha = alpha_;
    beta = beta_;
    k = k_;
    return true;
  }

  bool fuse_relu_before_bwd(float slope) override {
    if (this->phase_ != TRAIN || !within_) return false;
    relu_bwd_ = true;
    relu_bwd_slope_ = slope;
    return true;
  }

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    CAFFE_CHECK(bottom[0] != top[0], "LRN cannot run in place");
    if (this->folded_into_next) return;  // computed by the following MAX pool
    auto& b = *bottom[0];
    float* sc = this->phase_ == TRAIN ? scale_.mutable_gpu_data() : nullptr;
    if (within_)
      RRAM_CALL(rram_lrn_within_fwd(b.gpu_data(), top[0]->mutable_gpu_data(), sc, b.shape(0), b.shape(1),
                                    b.shape(2), b.shape(3), size_, alpha_, beta_, Caffe::stream()));
    else
      RRAM_CALL(rram_lrn_fwd(b.gpu_data(), top[0]->mutable_gpu_data(), sc, b.shape(0), b.shape(1), b.shape(2),
                             b.shape(3), size_, alpha_, beta_, k_, Caffe::stream()));
  }
  void Backward_gpu(const std::vector<Blob<Dtype>*>& top, const std::vector<bool>& pd,
                    const std::vector<Blob<Dtype>*>& bottom) override {
    if (!pd.size() || !pd[0]) return;
    auto& b = *bottom[0];
    if (within_ && relu_bwd_)  // the in-place ReLU before this LRN (Net::Net fold); its output is our bottom
      RRAM_CALL(rram_lrn_within_relu_bwd(b.gpu_data(), scale_.gpu_data(), top[0]->gpu_diff(), b.mutable_gpu_diff(),
                                         b.shape(0), b.shape(1), b.shape(2), b.shape(3), size_, alpha_, beta_,
                                         relu_bwd_slope_, Caffe::stream()));
    else if (within_)
      RRAM_CALL(rram_lrn_within_bwd(b.gpu_data(), scale_.gpu_data(), top[0]->gpu_diff(), b.mutable_gpu_diff(),
                                    b.shape(0), b.shape(1), b.shape(2), b.shape(3), size_, alpha_, beta_,
                                    Caffe::stream()));
    else
      RRAM_CALL(rram_lrn_bwd(b.gpu_data(), top[0]->gpu_data(), scale_.gpu_data(), top[0]->gpu_diff(),
                             b.mutable_gpu_diff(), b.shape(0), b.shape(1), b.shape(2), b.shape(3), size_,
                             alpha_, beta_, Caffe::stream()));
  }
  int size_ = 5;
  float alpha_ = 1, beta_ = 0.75f, k_ = 1;
  bool within_ = false, relu_bwd_ = false;
  float relu_bwd_slope_ = 0.0f;
  Blob<Dtype> scale_;
};

// ---------------------------------------------------------------- Dropout
template <typename Dtype>
class DropoutLayer : public Layer<Dtype> {
 public:
  explicit DropoutLayer(const Msg& p) : Layer<Dtype>(p) {}
  const char* type() const override { return "Dropout"; }
  int ExactNumBottomBlobs() const override { return 1; }
  int ExactNumTopBlobs() const override { return 1; }
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    ratio_ = (float)this->layer_param_.sub_or_empty("dropout_param").num("dropout_ratio", 0.5);
    top[0]->ReshapeLike(*bottom[0]);
    if (this->phase_ == TRAIN) mask_.ReshapeLike(*bottom[0]);
  }

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    const int64_t n = bottom[0]->count();
    if (this->phase_ == TRAIN) {
      RRAM_CALL(rram_dropout_fwd(bottom[0]->gpu_data(), top[0]->mutable_gpu_data(),
                                 reinterpret_cast<unsigned*>(mask_.mutable_gpu_data()), n, ratio_,
                                 Caffe::seed(), this->layer_id, this->iter, Caffe::stream()));
    } else if (bottom[0] != top[0]) {
      HIP_CALL(hipMemcpyAsync(top[0]->mutable_gpu_data(), bottom[0]->gpu_data(), n * sizeof(Dtype),
                              hipMemcpyDeviceToDevice, Caffe::hip_stream()));
    }
  }
  void Backward_gpu(const std::vector<Blob<Dtype>*>& top, const std::vector<bool>& pd,
                    const std::vector<Blob<Dtype>*>& bottom) override {
    if (!pd.size() || !pd[0]) return;
    const int64_t n = bottom[0]->count();
    if (this->phase_ == TRAIN) {
      RRAM_CALL(rram_dropout_bwd(top[0]->gpu_diff(), reinterpret_cast<const unsigned*>(mask_.gpu_data()),
                                 bottom[0]->mutable_gpu_diff(), n, ratio_, Caffe::stream()));
    } else if (bottom[0] != top[0]) {
      HIP_CALL(hipMemcpyAsync(bottom[0]->mutable_gpu_diff(), top[0]->gpu_diff(), n * sizeof(Dtype),
                              hipMemcpyDeviceToDevice, Caffe::hip_stream()));
    }
  }
  float ratio_ = 0.5f;
  Blob<Dtype> mask_;
};

static void softmax_dims(const Blob<float>& b, int axis, int& outer, int& C, int& inner) {
  if (axis < 0) axis += b.num_axes();
  outer = (int)b.count(0, axis);
  C = b.shape(axis);
  inner = (int)b.count(axis + 1);
}

// ---------------------------------------------------------------- Softmax
template <typename Dtype>
class SoftmaxLayer : public Layer<Dtype> {
 public:
  explicit SoftmaxLayer(const Msg& p) : Layer<Dtype>(p) {}
  const char* type() const override { return "Softmax"; }
  int ExactNumBottomBlobs() const override { return 1; }
  int ExactNumTopBlobs() const override { return 1; }
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    top[0]->ReshapeLike(*bottom[0]);
  }

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    int o, c, i;
    softmax_dims(*bottom[0], (int)this->layer_param_.sub_or_empty("softmax_param").integer("axis", 1), o, c, i);
    RRAM_CALL(rram_softmax_fwd(bottom[0]->gpu_data(), top[0]->mutable_gpu_data(), o, c, i, Caffe::stream()));
  }
  void Backward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<bool>& pd,
                    const std::vector<Blob<Dtype>*>&) override {
    CAFFE_CHECK(!pd.size() || !pd[0], "Softmax backward is not part of this build (use SoftmaxWithLoss)");
  }
};

// -------------------------------------------------------- SoftmaxWithLoss
template <typename Dtype>
class SoftmaxWithLossLayer : public Layer<Dtype> {
 public:
  explicit SoftmaxWithLossLayer(const Msg& p) : Layer<Dtype>(p) {}
  const char* type() const override { return "SoftmaxWithLoss"; }
  int ExactNumBottomBlobs() const override { return 2; }
  int MinTopBlobs() const override { return 1; }
  bool IsLoss() const override { return true; }
  bool AutoTopBlobs() const override { return true; }
  void LayerSetUp(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>&) override {
    const Msg& lp = this->layer_param_.sub_or_empty("loss_param");
    ignore_ = lp.has("ignore_label") ? (int)lp.integer("ignore_label") : -1;
    const std::string norm = lp.str("normalization", lp.has("normalize") ? (lp.boolean("normalize") ? "VALID" : "BATCH_SIZE") : "VALID");
    CAFFE_CHECK(norm == "VALID" || (norm == "BATCH_SIZE" && ignore_ < 0) || (norm == "FULL" && ignore_ < 0),
                this->name() << ": loss normalization " << norm << " not supported");
    axis_ = (int)this->layer_param_.sub_or_empty("softmax_param").integer("axis", 1);
  }
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    prob_.ReshapeLike(*bottom[0]);
    top[0]->Reshape({});
    if (top.size() > 1) top[1]->ReshapeLike(*bottom[0]);
  }
  bool set_top_accumulator(float* sum, float* row) override {
    if (this->phase_ == TRAIN && sum) return false;  // the TRAIN head (loss + dx in one launch) has no fold
    acc_sum_ = sum;
    acc_row_ = sum ? row : nullptr;
    return true;
  }

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    int o, c, i;
    softmax_dims(*bottom[0], axis_, o, c, i);
    // (a one-block fused softmax + loss measured slower on the CIFAR-10 quick MC head: latency-bound)
    RRAM_CALL(rram_softmax_fwd(bottom[0]->gpu_data(), prob_.mutable_gpu_data(), o, c, i, Caffe::stream()));
    // TRAIN, small head: the bottom gradient in the same launch as the loss
    // (Backward then has nothing left to do; writing it when no backward
    // follows is harmless: nothing else writes this diff)
    dx_in_fwd_ = this->phase_ == TRAIN && (int64_t)o * c * i <= 65536;
    if (dx_in_fwd_)
      RRAM_CALL(rram_softmax_loss_fwd_bwd(prob_.gpu_data(), bottom[1]->gpu_data(), top[0]->mutable_gpu_data(),
                                          bottom[0]->mutable_gpu_diff(), o, c, i, ignore_, this->loss(0),
                                          Caffe::stream()));
    else
      RRAM_CALL(rram_softmax_loss_fwd_acc(prob_.gpu_data(), bottom[1]->gpu_data(), top[0]->mutable_gpu_data(), o,
                                          c, i, ignore_, acc_sum_, acc_row_, Caffe::stream()));
    if (top.size() > 1)
      HIP_CALL(hipMemcpyAsync(top[1]->mutable_gpu_data(), prob_.gpu_data(), prob_.count() * sizeof(Dtype),
                              hipMemcpyDeviceToDevice, Caffe::hip_stream()));
  }
  void Backward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<bool>& pd,
                    const std::vector<Blob<Dtype>*>& bottom) override {
    CAFFE_CHECK(pd.size() < 2 || !pd[1], this->name() << " cannot backpropagate to label inputs");
    if (!pd.size() || !pd[0] || dx_in_fwd_) return;
    int o, c, i;
    softmax_dims(*bottom[0], axis_, o, c, i);
    RRAM_CALL(rram_softmax_loss_bwd(prob_.gpu_data(), bottom[1]->gpu_data(), bottom[0]->mutable_gpu_diff(),
                                    o, c, i, ignore_, this->loss(0), Caffe::stream()));
  }
  Blob<Dtype> prob_;
  int ignore_ = -1, axis_ = 1;
  bool dx_in_fwd_ = false;
  float *acc_sum_ = nullptr, *acc_row_ = nullptr;  // set_top_accumulator (TEST)
};

// --------------------------------------------------------------- Accuracy
template <typename Dtype>
class AccuracyLayer : public Layer<Dtype> {
 public:
  explicit AccuracyLayer(const Msg& p) : Layer<Dtype>(p) {}
  const char* type() const override { return "Accuracy"; }
  int ExactNumBottomBlobs() const override { return 2; }
  int ExactNumTopBlobs() const override { return 1; }
  void LayerSetUp(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>&) override {
    const Msg& ap = this->layer_param_.sub_or_empty("accuracy_param");
    top_k_ = (int)ap.integer("top_k", 1);
    axis_ = (int)ap.integer("axis", 1);
    ignore_ = ap.has("ignore_label") ? (int)ap.integer("ignore_label") : -1;
  }
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    int o, c, i;
    softmax_dims(*bottom[0], axis_, o, c, i);
    CAFFE_CHECK(top_k_ <= c, "top_k must be less than or equal to the number of classes");
    CAFFE_CHECK((int64_t)o * i == bottom[1]->count(), "number of labels must match number of predictions");
    top[0]->Reshape({});
    counts_.Reshape({2});
  }
  bool AllowForceBackward(int) const override { return false; }
  bool set_top_accumulator(float* sum, float* row) override {
    acc_sum_ = sum;
    acc_row_ = sum ? row : nullptr;
    return true;
  }

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    int o, c, i;
    softmax_dims(*bottom[0], axis_, o, c, i);
    float* cnt = counts_.mutable_gpu_data();
    RRAM_CALL(rram_accuracy_acc(bottom[0]->gpu_data(), bottom[1]->gpu_data(), cnt, cnt + 1,
                                top[0]->mutable_gpu_data(), o, c, i, top_k_, ignore_, acc_sum_, acc_row_,
                                Caffe::stream()));
  }
  void Backward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<bool>&,
                    const std::vector<Blob<Dtype>*>&) override {}
  int top_k_ = 1, axis_ = 1, ignore_ = -1;
  Blob<Dtype> counts_;
  float *acc_sum_ = nullptr, *acc_row_ = nullptr;  // set_top_accumulator
};

// ----------------------------------------------------------------- Concat
// concat_layer.cpp:9-67 / .cu:22-66: any axis; bottom i occupies the slot
// [off, off + shape_i(axis)) of every [outer] row of the top
static int canon_axis(int axis, int num_axes) { return axis < 0 ? axis + num_axes : axis; }

template <typename Dtype>
class ConcatLayer : public Layer<Dtype> {
 public:
  explicit ConcatLayer(const Msg& p) : Layer<Dtype>(p) {}
  const char* type() const override { return "Concat"; }
  int MinBottomBlobs() const override { return 1; }
  int ExactNumTopBlobs() const override { return 1; }
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    const Msg& cp = this->layer_param_.sub_or_empty("concat_param");
    // concat_dim is the V1 spelling of axis (concat_layer.cpp:16-21)
    axis_ = canon_axis((int)cp.integer("axis", cp.integer("concat_dim", 1)), bottom[0]->num_axes());
    CAFFE_CHECK(axis_ >= 0 && axis_ < bottom[0]->num_axes(), this->name() << ": concat axis out of range");
    std::vector<int> s = bottom[0]->shape();
    int along = 0;
    for (auto* b : bottom) {
      CAFFE_CHECK(b->num_axes() == (int)s.size(), this->name() << ": all inputs must have the same #axes");
      for (int a = 0; a < (int)s.size(); ++a)
        if (a != axis_)
          CAFFE_CHECK(b->shape(a) == s[a], this->name() << ": all inputs must have the same shape, except at concat_axis");
      along += b->shape(axis_);
    }
    s[axis_] = along;
    top[0]->Reshape(s);
    if (bottom.size() == 1) top[0]->ShareData(*bottom[0]), top[0]->ShareDiff(*bottom[0]);
  }

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    if (bottom.size() == 1) return;
    const int inner = (int)top[0]->count(axis_ + 1), outer = (int)top[0]->count(0, axis_);
    const int dci = top[0]->shape(axis_) * inner;
    int off = 0;
    for (size_t i = 0; i < bottom.size(); ++i) {
      const int sci = bottom[i]->shape(axis_) * inner;
      // a folded bottom's producer already wrote its slice (Net: TEST-phase Concat fold)
      if (!(i < skip_.size() && skip_[i]))
        RRAM_CALL(rram_concat_copy(bottom[i]->gpu_data(), top[0]->mutable_gpu_data(), outer, sci, dci, off, 0,
                                   Caffe::stream()));
      off += sci;
    }
  }
 public:
  void skip_concat_bottom(int i, bool skip) override {
    if ((int)skip_.size() <= i) skip_.resize(i + 1, false);
    skip_[i] = skip;
  }
  int axis() const { return axis_; }

 protected:
  std::vector<bool> skip_;
  void Backward_gpu(const std::vector<Blob<Dtype>*>& top, const std::vector<bool>& pd,
                    const std::vector<Blob<Dtype>*>& bottom) override {
    if (bottom.size() == 1) return;
    const int inner = (int)top[0]->count(axis_ + 1), outer = (int)top[0]->count(0, axis_);
    const int dci = top[0]->shape(axis_) * inner;
    int off = 0;
    for (size_t i = 0; i < bottom.size(); ++i) {
      const int sci = bottom[i]->shape(axis_) * inner;
      if (i < pd.size() && pd[i])
        RRAM_CALL(rram_concat_copy(bottom[i]->mutable_gpu_diff(), const_cast<float*>(top[0]->gpu_diff()), outer,
                                   sci, dci, off, 1, Caffe::stream()));
      off += sci;
    }
  }
  int axis_ = 1;
};

// ------------------------------------------------------------------ Slice
// slice_layer.cpp:9-94 / .cu:22-66: the inverse of Concat (slice_point list or
// an even split; slice_dim is the V1 spelling of axis)
template <typename Dtype>
class SliceLayer : public Layer<Dtype> {
 public:
  explicit SliceLayer(const Msg& p) : Layer<Dtype>(p) {}
  const char* type() const override { return "Slice"; }
  int ExactNumBottomBlobs() const override { return 1; }
  int MinTopBlobs() const override { return 1; }
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    const Msg& sp = this->layer_param_.sub_or_empty("slice_param");
    axis_ = canon_axis((int)sp.integer("axis", sp.integer("slice_dim", 1)), bottom[0]->num_axes());
    CAFFE_CHECK(axis_ >= 0 && axis_ < bottom[0]->num_axes(), this->name() << ": slice axis out of range");
    const int along = bottom[0]->shape(axis_);
    const auto pts = ints_of(sp, "slice_point");
    sizes_.clear();
    if (!pts.empty()) {
      CAFFE_CHECK(pts.size() == top.size() - 1, this->name() << ": need one slice_point fewer than tops");
      int prev = 0;
      for (int p : pts) {
        CAFFE_CHECK(p > prev, this->name() << ": slice points must be increasing");
        sizes_.push_back(p - prev);
        prev = p;
      }
      CAFFE_CHECK(along > prev, this->name() << ": last slice point beyond the axis");
      sizes_.push_back(along - prev);
    } else {
      CAFFE_CHECK(along % (int)top.size() == 0, this->name() << ": number of top blobs (" << top.size()
                                                             << ") should evenly divide input slice axis (" << along << ")");
      sizes_.assign(top.size(), along / (int)top.size());
    }
    std::vector<int> s = bottom[0]->shape();
    for (size_t i = 0; i < top.size(); ++i) {
      s[axis_] = sizes_[i];
      top[i]->Reshape(s);
    }
    if (top.size() == 1) top[0]->ShareData(*bottom[0]), top[0]->ShareDiff(*bottom[0]);
  }

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    if (top.size() == 1) return;
    const int inner = (int)bottom[0]->count(axis_ + 1), outer = (int)bottom[0]->count(0, axis_);
    const int dci = bottom[0]->shape(axis_) * inner;
    int off = 0;
    for (size_t i = 0; i < top.size(); ++i) {
      const int sci = sizes_[i] * inner;
      RRAM_CALL(rram_concat_copy(top[i]->mutable_gpu_data(), const_cast<float*>(bottom[0]->gpu_data()), outer, sci,
                                 dci, off, 1, Caffe::stream()));
      off += sci;
    }
  }
  void Backward_gpu(const std::vector<Blob<Dtype>*>& top, const std::vector<bool>& pd,
                    const std::vector<Blob<Dtype>*>& bottom) override {
    if (top.size() == 1 || !pd.size() || !pd[0]) return;
    const int inner = (int)bottom[0]->count(axis_ + 1), outer = (int)bottom[0]->count(0, axis_);
    const int dci = bottom[0]->shape(axis_) * inner;
    int off = 0;
    for (size_t i = 0; i < top.size(); ++i) {
      const int sci = sizes_[i] * inner;
      RRAM_CALL(rram_concat_copy(top[i]->gpu_diff(), bottom[0]->mutable_gpu_diff(), outer, sci, dci, off, 0,
                                 Caffe::stream()));
      off += sci;
    }
  }
  int axis_ = 1;
  std::vector<int> sizes_;
};

// ---------------------------------------------------------- EuclideanLoss
// euclidean_loss_layer.cpp:9-20, .cu:9-38: loss = ||a - b||^2 / (2 num);
// d/da = +loss_weight / num * (a - b), d/db = -loss_weight / num * (a - b)
template <typename Dtype>
class EuclideanLossLayer : public Layer<Dtype> {
 public:
  explicit EuclideanLossLayer(const Msg& p) : Layer<Dtype>(p) {}
  const char* type() const override { return "EuclideanLoss"; }
  int ExactNumBottomBlobs() const override { return 2; }
  int ExactNumTopBlobs() const override { return 1; }
  bool IsLoss() const override { return true; }
  bool AutoTopBlobs() const override { return true; }
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    CAFFE_CHECK(bottom[0]->shape(0) == bottom[1]->shape(0),
                "The data and label should have the same first dimension.");  // loss_layer.cpp:22-24
    CAFFE_CHECK(bottom[0]->count(1) == bottom[1]->count(1), "Inputs must have the same dimension.");
    top[0]->Reshape({});
    diff_.ReshapeLike(*bottom[0]);
  }

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    RRAM_CALL(rram_euclidean_loss_fwd(bottom[0]->gpu_data(), bottom[1]->gpu_data(), diff_.mutable_gpu_data(),
                                      top[0]->mutable_gpu_data(), bottom[0]->count(), bottom[0]->shape(0),
                                      Caffe::stream()));
  }
  void Backward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<bool>& pd,
                    const std::vector<Blob<Dtype>*>& bottom) override {
    for (int i = 0; i < 2; ++i) {
      if ((int)pd.size() <= i || !pd[i]) continue;
      // the top diff of a loss layer is its loss weight (net.cpp:BackwardFromTo seeds it)
      const Dtype alpha = (i == 0 ? Dtype(1) : Dtype(-1)) * this->loss(0) / bottom[i]->shape(0);
      RRAM_CALL(rram_euclidean_loss_bwd(diff_.gpu_data(), bottom[i]->mutable_gpu_diff(), bottom[i]->count(), alpha,
                                        Caffe::stream()));
    }
  }
  Blob<Dtype> diff_;
};

// ----------------------------------------------------- data-like layers
static std::vector<int> shape_of(const Msg& s) { return ints_of(s, "dim"); }

template <typename Dtype>
class InputLayer : public Layer<Dtype> {
 public:
  explicit InputLayer(const Msg& p) : Layer<Dtype>(p) {}
  const char* type() const override { return "Input"; }
  int ExactNumBottomBlobs() const override { return 0; }
  void LayerSetUp(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>& top) override {
    auto shapes = this->layer_param_.sub_or_empty("input_param").subs("shape");
    CAFFE_CHECK(shapes.size() == 1 || shapes.size() == top.size(),
                this->name() << ": give one input shape or one per top");
    for (size_t i = 0; i < top.size(); ++i) top[i]->Reshape(shape_of(*shapes[shapes.size() == 1 ? 0 : i]));
  }
  void Reshape(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>&) override {}

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>&) override {}
  void Backward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<bool>&,
                    const std::vector<Blob<Dtype>*>&) override {}
};

template <typename Dtype>
class DummyDataLayer : public Layer<Dtype> {
 public:
  explicit DummyDataLayer(const Msg& p) : Layer<Dtype>(p) {}
  const char* type() const override { return "DummyData"; }
  int ExactNumBottomBlobs() const override { return 0; }
  void LayerSetUp(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>& top) override {
    const Msg& dp = this->layer_param_.sub_or_empty("dummy_data_param");
    auto shapes = dp.subs("shape");
    auto fillers = dp.subs("data_filler");
    for (size_t i = 0; i < top.size(); ++i) {
      if (!shapes.empty()) {
        top[i]->Reshape(shape_of(*shapes[shapes.size() == 1 ? 0 : i]));
      } else {
        auto g = [&](const char* k) { auto v = dp.nums(k); return v.empty() ? 1 : (int)v[v.size() == 1 ? 0 : i]; };
        top[i]->Reshape({g("num"), g("channels"), g("height"), g("width")});
      }
      static const Msg zero;
      const Msg& f = fillers.empty() ? zero : *fillers[fillers.size() == 1 ? 0 : i];
      FillBlob(top[i], f, Caffe::seed() ^ 0xD0D0ull, (uint32_t)(this->layer_id * 16 + i));
    }
  }
  void Reshape(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>&) override {}

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>&) override {}
  void Backward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<bool>&,
                    const std::vector<Blob<Dtype>*>&) override {}
};

// Data / ImageData / MemoryData / WindowData: the configs' LMDB /
// LevelDB / image sources are out of scope, so these tops are
// synthetic tensors of the shape the source would produce:
// integer pixels U{0..255}, minus 128 when the layer subtracts a mean, times
// transform_param.scale; labels U{0..num_classes-1}.  The per-image shape
// comes from the net option `data_shape` (set via rram_net_create).
template <typename Dtype>
class SyntheticDataLayer : public Layer<Dtype> {
 public:
  explicit SyntheticDataLayer(const Msg& p) : Layer<Dtype>(p) {}
  const char* type() const override { return "Data"; }
  int ExactNumBottomBlobs() const override { return 0; }
  void LayerSetUp(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>& top) override {
    const Msg& p = this->layer_param_;
    const Msg* dp = nullptr;
    for (const char* k : {"data_param", "image_data_param", "memory_data_param", "window_data_param"})
      if (p.sub(k)) dp = p.sub(k);
    const int batch = dp ? (int)dp->integer("batch_size", 1) : 1;
    const Msg& tp = p.sub_or_empty("transform_param");
    std::vector<int> img = ints_of(p, "rram_data_shape");
    CAFFE_CHECK(img.size() == 3, this->name() << ": synthetic data needs a C,H,W data_shape option");
    if (tp.has("crop_size")) img[1] = img[2] = (int)tp.integer("crop_size");
    std::vector<int> s{batch};
    s.insert(s.end(), img.begin(), img.end());
    top[0]->Reshape(s);
    const float scale = (float)tp.num("scale", 1.0);
    const bool mean = tp.has("mean_file") || tp.has("mean_value");
    const uint64_t seed = Caffe::seed() ^ 0xDA7Aull ^ ((uint64_t)p.integer("rram_data_seed", 0) * 0x9E3779B97F4A7C15ull);
    RRAM_CALL(rram_fill_uniform_int(top[0]->mutable_gpu_data(), top[0]->count(), 256, mean ? -128.0f : 0.0f,
                                    seed, this->layer_id * 16, Caffe::stream()));
    if (scale != 1.0f) RRAM_CALL(rram_scal(top[0]->count(), scale, top[0]->mutable_gpu_data(), Caffe::stream()));
    if (top.size() > 1) {
      top[1]->Reshape({batch});
      const int classes = (int)p.integer("rram_num_classes", 10);
      RRAM_CALL(rram_fill_uniform_int(top[1]->mutable_gpu_data(), batch, classes, 0.0f, seed,
                                      this->layer_id * 16 + 1, Caffe::stream()));
    }
  }
  void Reshape(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>&) override {}

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>&) override {}
  void Backward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<bool>&,
                    const std::vector<Blob<Dtype>*>&) override {}
};

// HDF5Data (hdf5_data_layer.cpp:20-122, .cu:17-46): every top is the dataset
// of the same name in the .h5 files the `source` list names, read through
// libhdf5 (host/hdf5.cpp) and kept resident on the device; a Forward copies
// batch_size rows, cycling the files in list order (shuffle is not part of
// this build).  Under data-parallel training rank r of N takes only the rows
// whose running index is r mod N (Caffe 1.0's HDF5DataLayer::Skip), so N
// ranks x batch B see exactly the rows one process x batch N*B sees.
template <typename Dtype>
class HDF5DataLayer : public Layer<Dtype> {
 public:
  explicit HDF5DataLayer(const Msg& p) : Layer<Dtype>(p) {}
  ~HDF5DataLayer() override {
    for (float* d : dev_) (void)hipFree(d);
  }
  const char* type() const override { return "HDF5Data"; }
  int ExactNumBottomBlobs() const override { return 0; }
  int MinTopBlobs() const override { return 1; }
  void LayerSetUp(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>& top) override {
    const Msg& hp = this->layer_param_.sub_or_empty("hdf5_data_param");
    batch_ = (int)hp.integer("batch_size", 0);
    CAFFE_CHECK(batch_ > 0, this->name() << ": hdf5_data_param.batch_size must be > 0");
    CAFFE_CHECK(!hp.boolean("shuffle", false), this->name() << ": hdf5_data_param.shuffle is not supported");
    const std::string source = hp.str("source", "");
    std::ifstream list(source);
    CAFFE_CHECK(list.good(), "Failed to open source file " << source);
    std::vector<std::string> files;
    for (std::string line; std::getline(list, line);) {
      const size_t a = line.find_first_not_of(" \t\r"), b = line.find_last_not_of(" \t\r");
      if (a != std::string::npos) files.push_back(line.substr(a, b - a + 1));
    }
    CAFFE_CHECK(!files.empty(), "No HDF5 files listed in " << source);
    const auto tops = this->layer_param_.strs("top");
    std::vector<std::vector<float>> host(top.size());
    rows_ = 0;
    for (const auto& f : files) {
      h5::Handle fh = h5::open_file(f);
      int64_t frows = -1;
      for (size_t j = 0; j < top.size(); ++j) {
        std::vector<int64_t> dims;
        std::vector<float> v = h5::load_floats(fh.id(), tops[j], &dims);
        CAFFE_CHECK(!dims.empty(), f << ": dataset " << tops[j] << " has no axes");
        if (frows < 0) frows = dims[0];
        CAFFE_CHECK(dims[0] == frows, f << ": datasets must have the same number of rows");  // hdf5_data_layer.cpp:57-60
        std::vector<int> shape(dims.begin(), dims.end());
        shape[0] = batch_;
        if (shapes_.size() <= j) shapes_.push_back(shape);
        CAFFE_CHECK(shapes_[j] == shape, f << ": dataset " << tops[j] << " row shape differs between files");
        host[j].insert(host[j].end(), v.begin(), v.end());
      }
      rows_ += frows;
    }
    CAFFE_CHECK(rows_ > 0, this->name() << ": the HDF5 files hold no rows");
    for (size_t j = 0; j < top.size(); ++j) {
      float* d = nullptr;
      HIP_CALL(hipMalloc(&d, host[j].size() * sizeof(float)));
      HIP_CALL(hipMemcpy(d, host[j].data(), host[j].size() * sizeof(float), hipMemcpyHostToDevice));
      dev_.push_back(d);
      row_elems_.push_back((int64_t)(host[j].size() / rows_));
      top[j]->Reshape(shapes_[j]);
    }
    rank_ = (int)this->layer_param_.integer("rram_solver_rank", 0);
    world_ = std::max(1, (int)this->layer_param_.integer("rram_solver_count", 1));
    if (this->phase_ == TEST) rank_ = 0, world_ = 1;  // Skip() never skips in TEST
  }
  void Reshape(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>&) override {}

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>& top) override {
    for (int i = 0; i < batch_; ++i) {
      while (offset_++ % world_ != rank_) row_ = (row_ + 1) % rows_;
      for (size_t j = 0; j < top.size(); ++j)
        HIP_CALL(hipMemcpyAsync(top[j]->mutable_gpu_data() + i * row_elems_[j], dev_[j] + row_ * row_elems_[j],
                                row_elems_[j] * sizeof(float), hipMemcpyDeviceToDevice, Caffe::hip_stream()));
      row_ = (row_ + 1) % rows_;
    }
  }
  void Backward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<bool>&,
                    const std::vector<Blob<Dtype>*>&) override {}
  int batch_ = 0, rank_ = 0, world_ = 1;
  int64_t rows_ = 0, row_ = 0, offset_ = 0;
  std::vector<std::vector<int>> shapes_;
  std::vector<int64_t> row_elems_;
  std::vector<float*> dev_;
};

REGISTER_LAYER_CLASS(Convolution);
REGISTER_LAYER_CLASS(InnerProduct);
REGISTER_LAYER_CLASS(ReLU);
REGISTER_LAYER_CLASS(Split);
REGISTER_LAYER_CLASS(Pooling);
REGISTER_LAYER_CLASS(LRN);
REGISTER_LAYER_CLASS(Dropout);
REGISTER_LAYER_CLASS(Softmax);
REGISTER_LAYER_CLASS(SoftmaxWithLoss);
REGISTER_LAYER_CLASS(Accuracy);
REGISTER_LAYER_CLASS(Concat);
REGISTER_LAYER_CLASS(Input);
REGISTER_LAYER_CLASS(DummyData);
REGISTER_LAYER_CLASS(Slice);
REGISTER_LAYER_CLASS(EuclideanLoss);
REGISTER_LAYER_CLASS(HDF5Data);
static ::caffe::LayerRegisterer<float> g_data_aliases[] = {
    {"Data", [](const Msg& p) -> std::shared_ptr<Layer<float>> { return std::make_shared<SyntheticDataLayer<float>>(p); }},
    {"ImageData", [](const Msg& p) -> std::shared_ptr<Layer<float>> { return std::make_shared<SyntheticDataLayer<float>>(p); }},
    {"MemoryData", [](const Msg& p) -> std::shared_ptr<Layer<float>> { return std::make_shared<SyntheticDataLayer<float>>(p); }},
    {"WindowData", [](const Msg& p) -> std::shared_ptr<Layer<float>> { return std::make_shared<SyntheticDataLayer<float>>(p); }},
};

template class ConvolutionLayer<float>;
template class InnerProductLayer<float>;
template class ReLULayer<float>;
template class SplitLayer<float>;

}  // namespace caffe
