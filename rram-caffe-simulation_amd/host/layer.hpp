// Layer<Dtype> plugin API (include/caffe/layer.hpp:33-445) and the layer
// registry (layer_factory.hpp:127-135).  Public non-virtual SetUp / Forward /
// Backward; protected virtual LayerSetUp / Reshape / Forward_gpu /
// Backward_gpu.  This build is device-only: Forward_cpu/Backward_cpu are not
// part of the product (the CPU restatement lives in oracle/ as a checker).
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "blob.hpp"
#include "proto.hpp"

namespace caffe {

template <typename Dtype>
class Net;

template <typename Dtype>
class Layer {
 public:
  explicit Layer(const Msg& param) : layer_param_(param) {
    phase_ = param.str("phase", "TRAIN") == "TEST" ? TEST : TRAIN;
  }
  virtual ~Layer() = default;

  void SetUp(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) {
    CheckBlobCounts(bottom, top);
    LayerSetUp(bottom, top);
    Reshape(bottom, top);
    SetLossWeights(top);
  }
  virtual void LayerSetUp(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>&) {}
  virtual void Reshape(const std::vector<Blob<Dtype>*>& bottom,
                       const std::vector<Blob<Dtype>*>& top) = 0;

  // layer.hpp:451-487: Reshape -> Forward_gpu -> loss = sum(top * loss_weight)
  Dtype Forward(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top);
  void Backward(const std::vector<Blob<Dtype>*>& top, const std::vector<bool>& propagate_down,
                const std::vector<Blob<Dtype>*>& bottom) {
    Backward_gpu(top, propagate_down, bottom);
  }

  std::vector<std::shared_ptr<Blob<Dtype>>>& blobs() { return blobs_; }
  const Msg& layer_param() const { return layer_param_; }
  std::string name() const { return layer_param_.str("name"); }
  virtual const char* type() const = 0;
  virtual int ExactNumBottomBlobs() const { return -1; }
  virtual int MinBottomBlobs() const { return -1; }
  virtual int ExactNumTopBlobs() const { return -1; }
  virtual int MinTopBlobs() const { return -1; }
  virtual bool EqualNumBottomTopBlobs() const { return false; }
  virtual bool AllowForceBackward(int) const { return true; }
  virtual bool IsLoss() const { return false; }
  // layer.hpp:282-288 / loss_layer.hpp:40: loss layers get an anonymous top
  // when the prototxt names none (Net allocates it, net.cpp:123-135)
  virtual bool AutoTopBlobs() const { return false; }

  Dtype loss(int top_index) const {
    return top_index < (int)loss_.size() ? loss_[top_index] : Dtype(0);
  }
  void set_loss(int top_index, Dtype v) {
    if ((int)loss_.size() <= top_index) loss_.resize(top_index + 1, Dtype(0));
    loss_[top_index] = v;
  }
  bool param_propagate_down(int i) const {
    return i < (int)param_propagate_down_.size() ? param_propagate_down_[i] : false;
  }
  void set_param_propagate_down(int i, bool v) {
    if ((int)param_propagate_down_.size() <= i) param_propagate_down_.resize(i + 1, true);
    param_propagate_down_[i] = v;
  }
  Phase phase() const { return phase_; }
  void set_phase(Phase p) { phase_ = p; }
  // per-layer id used to decorrelate RNG streams (dropout, fillers)
  uint32_t layer_id = 0;
  uint64_t iter = 0;

  // TEST-phase fusion (Net::Net): an ACROSS_CHANNELS LRN whose top only feeds
  // a MAX pool hands its work to the pool (rram_lrn_maxpool_fwd); the LRN's
  // Forward then only reshapes.  lrn_params() reports an LRN's parameters,
  // fuse_lrn_before() asks the consumer to take them over.
  virtual bool lrn_params(int& /*size*/, float& /*alpha*/, float& /*beta*/, float& /*k*/) const {
    return false;
  }
  virtual bool fuse_lrn_before(Blob<Dtype>* /*lrn_bottom*/, int /*size*/, float /*alpha*/,
                               float /*beta*/, float /*k*/) {
    return false;
  }
  bool folded_into_next = false;
  // TEST-phase pooled-output fold (Net::Net): a folded LRN + MAX pool whose
  // top's only reader is a Convolution that reads the top's octet companion
  // writes only the companion; set_octet_reader() names that reader (nullptr
  // undoes it), input_octets_now() is the reader's check, per forward, that it
  // will read the companion of an input shaped like `bottom` (engine and plan
  // as they stand then)
  virtual bool set_octet_reader(Layer* /*reader*/) { return false; }
  // a convolution whose data gradient reads its kernel flipped: the geometry
  // of blobs()[0] for rram_update_seg.w_flip (ConvolutionLayer)
  virtual bool flip_geometry(int* /*g*/, int* /*cin_g*/, int* /*cout_g*/, int* /*taps*/) const { return false; }
  virtual bool input_octets_now(const Blob<Dtype>* /*bottom*/) const { return false; }
  // ReLU fold into a Pooling producer (Net::Net, any phase): an in-place ReLU
  // right after a layer that accepts it is applied in that layer's output
  // store (rram_pool_relu_fwd); the ReLU's Backward still runs.
  virtual bool fuse_relu_after(float /*slope*/) { return false; }
  // the mirror in backward (TRAIN): a layer right after an in-place ReLU that
  // applies the ReLU's backward factor to the bottom diff it writes
  // (rram_pool_relu_bwd); the ReLU's Backward then does nothing
  virtual bool fuse_relu_before_bwd(float /*slope*/) { return false; }
  // MonteCarlo statistics folded into the producer of a scalar output
  // (Accuracy, SoftmaxWithLoss in TEST): while set, Forward also does
  // *sum += top, *row = top (row nullable) in the kernel that stores the top,
  // so the MC driver launches no accumulate kernel.  sum == nullptr clears it;
  // false: the layer cannot (the driver then accumulates itself).
  virtual bool set_top_accumulator(float* /*sum*/, float* /*row*/) { return false; }
  // TEST-phase Concat fold (Net::Net): a producer whose top only feeds a
  // channel Concat writes its output straight into the Concat top at a
  // channel offset (write_into_concat: true when it can), and the Concat then
  // skips that bottom's copy (skip_concat_bottom).  The producer's own top is
  // then never materialised (like a folded LRN's) until Net::materialize_blob
  // undoes the fold (the C-ABI does for every blob it hands out).
  virtual bool write_into_concat(Blob<Dtype>* /*concat_top*/, int /*channel_offset*/) { return false; }
  virtual void skip_concat_bottom(int /*bottom_index*/, bool /*skip*/) {}

 protected:
  virtual void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom,
                           const std::vector<Blob<Dtype>*>& top) = 0;
  virtual void Backward_gpu(const std::vector<Blob<Dtype>*>& top,
                            const std::vector<bool>& propagate_down,
                            const std::vector<Blob<Dtype>*>& bottom) = 0;
  void CheckBlobCounts(const std::vector<Blob<Dtype>*>& bottom,
                       const std::vector<Blob<Dtype>*>& top);
  void SetLossWeights(const std::vector<Blob<Dtype>*>& top);

  Msg layer_param_;
  Phase phase_;
  std::vector<std::shared_ptr<Blob<Dtype>>> blobs_;
  std::vector<bool> param_propagate_down_;
  std::vector<Dtype> loss_;
};

// ------------------------------------------------------------ registry
template <typename Dtype>
class LayerRegistry {
 public:
  using Creator = std::function<std::shared_ptr<Layer<Dtype>>(const Msg&)>;
  static std::map<std::string, Creator>& Registry();
  static void AddCreator(const std::string& type, Creator c) { Registry()[type] = std::move(c); }
  static std::shared_ptr<Layer<Dtype>> CreateLayer(const Msg& param);
  static std::vector<std::string> LayerTypeList();
};

template <typename Dtype>
struct LayerRegisterer {
  LayerRegisterer(const std::string& type, typename LayerRegistry<Dtype>::Creator c) {
    LayerRegistry<Dtype>::AddCreator(type, std::move(c));
  }
};

#define REGISTER_LAYER_CLASS(type)                                                  \
  static ::caffe::LayerRegisterer<float> g_creator_f_##type(                        \
      #type, [](const ::caffe::Msg& p) -> std::shared_ptr<::caffe::Layer<float>> {  \
        return std::make_shared<type##Layer<float>>(p);                             \
      })

// Fill a parameter blob from a FillerParameter message (filler.hpp):
// constant / gaussian / uniform / xavier / msra, seeded counter RNG.
void FillBlob(Blob<float>* blob, const Msg& filler, uint64_t seed, uint32_t stream_id);

}  // namespace caffe
