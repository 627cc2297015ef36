// Concrete layers.  ★ = on the fault-simulation hot path:
// Convolution (a5/a6), InnerProduct (a7).  The rest are the minimal support
// layers the configs need, each a thin call into
// librram_kernels.so.
#pragma once

#include "layer.hpp"

namespace caffe {

// ★ Convolution (conv_layer.cpp:7-73, base_conv_layer.cpp:11-254): implicit
// GEMM forward on fp32 MFMA over the whole batch; optional fused ReLU when
// the net folds a following in-place ReLU into this layer.
template <typename Dtype>
class ConvolutionLayer : public Layer<Dtype> {
 public:
  explicit ConvolutionLayer(const Msg& p) : Layer<Dtype>(p) {}
  void LayerSetUp(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override;
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override;
  const char* type() const override { return "Convolution"; }
  int ExactNumBottomBlobs() const override { return 1; }
  int ExactNumTopBlobs() const override { return 1; }
  bool fused_relu = false;
  // keep the bf16x6 engine's packed weights next to the weight blob
  // (SyncedMemory::wpack, rram_conv2d_fwd_cached) while the weights are
  // unchanged; set by Net::set_weight_pack_cache for the Monte-Carlo driver
  bool cache_wpack = false;
  const rram_conv_desc& desc() const { return desc_; }
  bool input_octets_now(const Blob<Dtype>* bottom) const override {
    if (bottom->num_axes() != 4) return false;
    rram_conv_desc d = desc_;
    d.num = bottom->shape(0);
    d.height = bottom->shape(2);
    d.width = bottom->shape(3);
    return bottom->shape(1) == d.channels && rram_conv_input_octets(&d) == 1;
  }
  bool write_into_concat(Blob<Dtype>* concat_top, int channel_offset) override {
    concat_top_ = concat_top;
    concat_off_ = channel_offset;
    return true;
  }
  // TEST-phase convolution-output fold (Net::Net): the top's only reader is
  // a convolution taking its octet companion; each forward that both sides
  // confirm (rram_conv_output_octets_only, the reader's input_octets_now)
  // writes only the companion (the pooled-output fold's convolution form)
  // (TRAIN phase) the stride-1 data gradient runs as a forward convolution
  // with the flipped kernel (rram_conv2d_flip_applies): its geometry, for
  // the solver's fused update to write that kernel (rram_update_seg.w_flip)
  bool flip_geometry(int* g, int* cin_g, int* cout_g, int* taps) const override;
  bool set_octet_reader(Layer<Dtype>* reader) override {
    if (reader != nullptr && (this->phase_ != TEST || concat_top_ != nullptr)) return false;
    octet_reader_ = reader;
    return true;
  }

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override;
  void Backward_gpu(const std::vector<Blob<Dtype>*>& top, const std::vector<bool>& pd,
                    const std::vector<Blob<Dtype>*>& bottom) override;
  rram_conv_desc desc_{};
  bool bias_term_ = true;
  // the forward reads its input's channel-octet companion (cached per input shape / engine)
  bool want_in_oct_ = false;
  int oct_key_[4] = {-1, -1, -1, -1};
  Blob<Dtype>* concat_top_ = nullptr;  // write_into_concat: the output goes to this top at channel concat_off_
  int concat_off_ = 0;
  Layer<Dtype>* octet_reader_ = nullptr;  // convolution-output fold: the top's only reader
  bool flip_ok_ = false;
};

// ★ InnerProduct (inner_product_layer.cpp:9-141, .cu:9-75).
template <typename Dtype>
class InnerProductLayer : public Layer<Dtype> {
 public:
  explicit InnerProductLayer(const Msg& p) : Layer<Dtype>(p) {}
  void LayerSetUp(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override;
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override;
  const char* type() const override { return "InnerProduct"; }
  int ExactNumBottomBlobs() const override { return 1; }
  int ExactNumTopBlobs() const override { return 1; }
  bool fused_relu = false;
  int M() const { return M_; }
  int N() const { return N_; }
  int K() const { return K_; }

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override;
  void Backward_gpu(const std::vector<Blob<Dtype>*>& top, const std::vector<bool>& pd,
                    const std::vector<Blob<Dtype>*>& bottom) override;
  int M_ = 0, N_ = 0, K_ = 0, axis_ = 1;
  bool bias_term_ = true, transpose_ = false;
  // split-K partials need up to 16 x M x N floats (<= 256 MB)
  size_t ws_request() const { return std::min<size_t>((size_t)16 * M_ * N_ * sizeof(float), 256ull << 20); }
  uint64_t in_rows_key_ = 0;  // the packed-row companion this layer reads (Reshape; 0: none)
};

template <typename Dtype>
class ReLULayer : public Layer<Dtype> {
 public:
  explicit ReLULayer(const Msg& p) : Layer<Dtype>(p) {}
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override {
    top[0]->ReshapeLike(*bottom[0]);
  }
  const char* type() const override { return "ReLU"; }
  float negative_slope() const {
    return static_cast<float>(this->layer_param_.sub_or_empty("relu_param").num("negative_slope", 0.0));
  }
  // set by Net when the producing Conv/IP layer applies the ReLU in its epilogue
  bool folded = false;
  // set by Net when the consuming layer applies the ReLU's backward factor
  bool bwd_folded = false;

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override;
  void Backward_gpu(const std::vector<Blob<Dtype>*>& top, const std::vector<bool>& pd,
                    const std::vector<Blob<Dtype>*>& bottom) override;
};

template <typename Dtype>
class SplitLayer : public Layer<Dtype> {
 public:
  explicit SplitLayer(const Msg& p) : Layer<Dtype>(p) {}
  void Reshape(const std::vector<Blob<Dtype>*>& bottom, const std::vector<Blob<Dtype>*>& top) override;
  const char* type() const override { return "Split"; }

 protected:
  void Forward_gpu(const std::vector<Blob<Dtype>*>&, const std::vector<Blob<Dtype>*>&) override {}
  void Backward_gpu(const std::vector<Blob<Dtype>*>& top, const std::vector<bool>& pd,
                    const std::vector<Blob<Dtype>*>& bottom) override;
};

}  // namespace caffe
