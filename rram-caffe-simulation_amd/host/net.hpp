// Net<Dtype>: the layer DAG (src/caffe/net.cpp, include/caffe/net.hpp).
// Keeps the reference's fault-parameter registry: failure_learnable_params()
// holds the weights and biases of every InnerProduct layer and fc_params_ids_
// the 2-D ones (net.cpp:482-493, net.hpp:181-186).
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "io.hpp"
#include "layers.hpp"
#include "timer.hpp"

namespace caffe {

template <typename Dtype>
void BlobFromProto(Blob<Dtype>* b, const BlobProtoData& p);  // shape-checked by the caller
template <typename Dtype>
BlobProtoData BlobToProto(Blob<Dtype>* b, bool write_diff);

template <typename Dtype>
class Net {
 public:
  // options: data_shape ("C,H,W" for synthetic Data layers), num_classes,
  // fault_layers ("InnerProduct" = reference; "InnerProduct,Convolution" = extension),
  // fuse_relu (true).
  Net(const Msg& param, Phase phase, const Msg& options = Msg());

  Dtype Forward(bool compute_loss = true);
  Dtype ForwardFromTo(int start, int end, bool compute_loss = true);
  void Backward();
  Dtype ForwardBackward() {
    Dtype l = Forward(true);
    Backward();
    return l;
  }
  void Update();
  // also (nullable): n_also counters cleared in the same launch (the solver's Fail counters)
  void ClearParamDiffs(unsigned long long* also = nullptr, int64_t n_also = 0);
  void ShareTrainedLayersWith(const Net* other);
  // .caffemodel weights (net.cpp:765-880, binary proto only; io.hpp)
  void CopyTrainedLayersFrom(const NetProtoData& param);
  // binary proto, or HDF5 when the name ends in ".h5" (net.cpp:803-860)
  void CopyTrainedLayersFrom(const std::string& path);
  void CopyTrainedLayersFromHDF5(const std::string& path);
  NetProtoData ToProto(bool write_diff = false) const;
  // net.cpp:862-932: group "data" (and "diff") / layer name / dataset "<param index>"
  void ToHDF5(const std::string& path, bool write_diff = false) const;

  const std::string& name() const { return name_; }
  Phase phase() const { return phase_; }
  const std::vector<std::shared_ptr<Layer<Dtype>>>& layers() const { return layers_; }
  const std::vector<std::vector<Blob<Dtype>*>>& top_vecs() const { return top_vecs_; }
  const std::vector<std::string>& layer_names() const { return layer_names_; }
  const std::vector<std::shared_ptr<Blob<Dtype>>>& blobs() const { return blobs_; }
  const std::vector<std::string>& blob_names() const { return blob_names_; }
  const std::vector<Blob<Dtype>*>& learnable_params() const { return learnable_params_; }
  const std::vector<float>& params_lr() const { return params_lr_; }
  const std::vector<float>& params_weight_decay() const { return params_weight_decay_; }
  const std::vector<Blob<Dtype>*>& failure_learnable_params() const { return failure_learnable_params_; }
  const std::vector<int>& failure_learnable_layer_ids() const { return failure_learnable_layer_ids_; }
  // index into learnable_params() of each failure param (fixes Appendix A Q6)
  const std::vector<int>& failure_learnable_param_ids() const { return failure_learnable_param_ids_; }
  std::vector<int> fc_params_ids_;
  const std::vector<Blob<Dtype>*>& output_blobs() const { return net_output_blobs_; }
  const std::vector<int>& output_blob_indices() const { return net_output_blob_indices_; }
  const std::vector<float>& blob_loss_weights() const { return blob_loss_weights_; }
  std::shared_ptr<Blob<Dtype>> blob_by_name(const std::string& n) const;
  std::shared_ptr<Layer<Dtype>> layer_by_name(const std::string& n) const;
  bool has_blob(const std::string& n) const { return blob_names_index_.count(n) > 0; }

  // Flat learnable-parameter buffers (parallel.cpp:25-115 GPUParams): copies
  // the current values into `data` / zeroes `diff` and aliases every learnable
  // param into them, so one all-reduce covers all gradients.
  int64_t flat_param_count() const;
  void alias_flat_params(Dtype* data, Dtype* diff);

  // Called after layer i's Backward (in backward order, every layer index),
  // so a data-parallel driver can start reducing the gradients that are final
  // while earlier layers still run backward.
  std::function<void(int)> on_backward_layer;

  void set_iter(uint64_t it) {
    for (auto& l : layers_) l->iter = it;
  }

  // per-layer forward timing with hipEvents (`caffe time`, tools/caffe.cpp:334-421):
  // 0 off, 1 every layer, 2 only layers that own parameters (conv / IP)
  void set_timing(int mode) { timing_ = mode; }
  bool timing_on() const { return timing_ != 0; }
  // events around layer i only (mode 3): one kernel's live timing at the
  // least event overhead
  void set_timing_layer(int i) {
    timing_ = 3;
    timed_layer_ = i;
  }
  // convolution layers keep their packed weights between forwards while the
  // weights are unchanged (ConvolutionLayer::cache_wpack); off drops every pack
  void set_weight_pack_cache(bool on);
  // Undo a TEST-phase fold that leaves blob b unwritten (a caller asked for it
  // through the C-ABI, so it must hold its layer's output as in the
  // reference).  A folded Concat bottom gets its current values back from the
  // Concat top's slice; a folded LRN's top is computed now from its bottom.
  // Later forwards write b again (the producer stores it, the consumer reads it).
  void materialize_blob(const Blob<Dtype>* b);
  EventTimer& timer() { return timer_; }

 private:
  struct ConcatFold {
    int writer, concat, bottom;  // producing Convolution, Concat layer, bottom index
    int offset;                  // channel offset of the slice
  };
  std::vector<ConcatFold> concat_folds_;
  struct LrnFold {
    int lrn, pool, size;  // the folded LRN, the MAX pool computing it, its parameters
    float alpha, beta, k;
  };
  std::vector<LrnFold> lrn_folds_;
  std::vector<int> oct_y_folds_;  // pooled- / convolution-output folds: the producing layers
  int timing_ = 0;
  int timed_layer_ = -1;
  EventTimer timer_;
  Dtype* flat_diff_ = nullptr;  // set by alias_flat_params
  void AppendParam(int layer_id, int param_id, const Msg& layer_param);

  std::string name_;
  Phase phase_;
  std::vector<std::shared_ptr<Layer<Dtype>>> layers_;
  std::vector<std::string> layer_names_;
  std::map<std::string, int> layer_names_index_;
  std::vector<std::shared_ptr<Blob<Dtype>>> blobs_;
  std::vector<std::string> blob_names_;
  std::map<std::string, int> blob_names_index_;
  std::vector<std::vector<Blob<Dtype>*>> bottom_vecs_, top_vecs_;
  std::vector<std::vector<int>> bottom_id_vecs_, top_id_vecs_;
  std::vector<std::vector<bool>> bottom_need_backward_;
  std::vector<bool> layer_need_backward_;
  std::vector<bool> blob_need_backward_;
  bool blob_need_backward_flag(int id) const { return blob_need_backward_[id]; }
  std::vector<std::shared_ptr<Blob<Dtype>>> params_;
  std::vector<Blob<Dtype>*> learnable_params_;
  std::vector<float> params_lr_, params_weight_decay_;
  std::vector<int> param_owners_;
  std::vector<std::vector<int>> param_id_vecs_;  // per layer: net param id of each of its blobs
  std::map<std::string, int> param_names_index_;
  std::vector<Blob<Dtype>*> failure_learnable_params_;
  std::vector<int> failure_learnable_layer_ids_, failure_learnable_param_ids_;
  std::vector<Blob<Dtype>*> net_output_blobs_;
  std::vector<int> net_output_blob_indices_;
  std::vector<float> blob_loss_weights_;
  std::vector<std::string> fault_layer_types_;
};

// Phase/rule filtering (net.cpp FilterNet + StateMeetsRule, phase only) and
// split insertion for blobs consumed more than once (insert_splits.cpp).
Msg FilterNet(const Msg& param, Phase phase);
Msg InsertSplits(const Msg& param);
// Structural description after input conversion, phase filtering and split
// insertion: one line per layer "name\ttype\tbottoms\ttops" (comma-joined).
// Pure host logic (no device), used by the CPU tests.
std::string DescribeNet(const Msg& param, Phase phase);

}  // namespace caffe
