// SyncedMemory + Blob: the reference's lazy host/device mirror
// (include/caffe/syncedmem.hpp:45-83, src/caffe/syncedmem.cpp:25-153;
// include/caffe/blob.hpp:209-274).  Device-resident by default: a host mirror
// is only materialised when cpu_data() is asked for, so the fault path never
// ping-pongs.  set_gpu_data() borrows external memory,
// which is how parameters are aliased into one flat buffer for data-parallel
// gradient all-reduce (parallel.cpp:25-115).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "common.hpp"

namespace caffe {

class SyncedMemory {
 public:
  enum SyncedHead { UNINITIALIZED, HEAD_AT_CPU, HEAD_AT_GPU, SYNCED };
  explicit SyncedMemory(size_t size = 0) : size_(size) {}
  ~SyncedMemory();
  SyncedMemory(const SyncedMemory&) = delete;
  SyncedMemory& operator=(const SyncedMemory&) = delete;

  const void* cpu_data();
  const void* gpu_data();
  void* mutable_cpu_data();
  void* mutable_gpu_data();
  void set_cpu_data(void* data);   // borrow host memory
  void set_gpu_data(void* data);   // borrow device memory
  SyncedHead head() const { return head_; }
  size_t size() const { return size_; }

  // Channel-octet companion (rram_conv2d_fwd_octets): a device buffer with the
  // pre-split bf16x3 form of this memory's NCHW contents.  It is valid only
  // while the data is unchanged since a producer wrote both (every mutable_* /
  // set_* access invalidates it), only for the shape it was written for, and
  // never once the C-ABI handed the data pointer out (expose(): the caller may
  // write a new batch through it with no mutable access, e.g. into an Input
  // blob, so a companion packed from the old batch must not be read).
  void* octets(size_t bytes);  // the buffer, grown to `bytes`
  const void* valid_octets(const int (&shape)[4]) const;
  void set_octets_valid(const int (&shape)[4]);
  bool wants_octets = false;  // a consumer would read the companion
  // the producer wrote only the companion (TEST-phase pooled-output fold,
  // Net::Net): the fp32 contents are stale until Net::materialize_blob
  bool fp32_stale = false;

  // Packed-weight companion (rram_conv2d_fwd_cached): the bf16x6 engine's
  // pre-split form of these weights, valid for one key (the layer's shape and
  // engine) until the next mutable_* / set_* access, like the octet companion.
  void* wpack(size_t bytes);  // the buffer, grown to `bytes`
  bool wpack_valid(uint64_t key) const { return wp_valid_ && !exposed_ && wp_key_ == key; }
  // the C-ABI handed this memory's device pointer to a caller, who may write
  // through it at any time without a mutable access: no pack or octet
  // companion is trusted after
  void expose() { exposed_ = true; }
  bool exposed() const { return exposed_; }
  void set_wpack_valid(uint64_t key) {
    wp_key_ = key;
    wp_valid_ = wp_ptr_ != nullptr;
  }
  void drop_wpack() { wp_valid_ = false; }

  // Flipped-kernel companion (rram_update_seg.w_flip): these convolution
  // weights transposed per group and rotated 180 degrees, written by the
  // solver's fused update next to the weights, read by the stride-1 data
  // gradient (rram_conv2d_bwd_ex).  Valid for the Solver::Step call that
  // wrote it (Caffe::step_epoch) until the next mutable_* / set_* access.
  void* wflip(size_t bytes);  // the buffer, grown to `bytes`
  bool wflip_valid(uint64_t epoch) const { return wf_valid_ && epoch != 0 && wf_epoch_ == epoch; }
  void set_wflip_valid(uint64_t epoch) {
    wf_epoch_ = epoch;
    wf_valid_ = wf_ptr_ != nullptr && epoch != 0;
  }
  void drop_wflip() { wf_valid_ = false; }

  // Packed-rows companion (rram_ip_fwd_rows): an InnerProduct input in the
  // bf16x6 engine's packed-row form, written by the producing InnerProduct's
  // split-K reduce for one key (the consumer's rows per tile and shape), valid
  // until the next mutable_* / set_* access, like the octet companion.
  // wants_rows: the key a consumer asked for at Reshape (0: none).
  void* rows(size_t bytes);  // the buffer, grown to `bytes`
  const void* valid_rows(uint64_t key) const { return rw_valid_ && !exposed_ && rw_key_ == key ? rw_ptr_ : nullptr; }
  void set_rows_valid(uint64_t key) {
    rw_key_ = key;
    rw_valid_ = rw_ptr_ != nullptr;
  }
  uint64_t wants_rows = 0;
  size_t wants_rows_bytes = 0;

 private:
  void to_cpu();
  void to_gpu();
  void* cpu_ptr_ = nullptr;
  void* gpu_ptr_ = nullptr;
  size_t size_;
  SyncedHead head_ = UNINITIALIZED;
  bool own_cpu_ = false, own_gpu_ = false;
  void* oct_ptr_ = nullptr;
  size_t oct_bytes_ = 0;
  bool oct_valid_ = false;
  int oct_shape_[4] = {0, 0, 0, 0};
  void* wp_ptr_ = nullptr;
  size_t wp_bytes_ = 0;
  bool wp_valid_ = false;
  uint64_t wp_key_ = 0;
  void* rw_ptr_ = nullptr;
  size_t rw_bytes_ = 0;
  bool rw_valid_ = false;
  uint64_t rw_key_ = 0;
  void* wf_ptr_ = nullptr;
  size_t wf_bytes_ = 0;
  bool wf_valid_ = false;
  uint64_t wf_epoch_ = 0;
  bool exposed_ = false;
};

template <typename Dtype>
class Blob {
 public:
  Blob() = default;
  explicit Blob(const std::vector<int>& shape) { Reshape(shape); }
  void Reshape(const std::vector<int>& shape);
  void ReshapeLike(const Blob& o) { Reshape(o.shape()); }
  const std::vector<int>& shape() const { return shape_; }
  int shape(int i) const { return shape_[i < 0 ? i + (int)shape_.size() : i]; }
  int num_axes() const { return static_cast<int>(shape_.size()); }
  int64_t count() const { return count_; }
  int64_t count(int start, int end = -1) const;
  std::string shape_string() const;

  const Dtype* cpu_data() const { return static_cast<const Dtype*>(data_->cpu_data()); }
  const Dtype* gpu_data() const { return static_cast<const Dtype*>(data_->gpu_data()); }
  const Dtype* cpu_diff() const { return static_cast<const Dtype*>(diff_->cpu_data()); }
  const Dtype* gpu_diff() const { return static_cast<const Dtype*>(diff_->gpu_data()); }
  Dtype* mutable_cpu_data() { return static_cast<Dtype*>(data_->mutable_cpu_data()); }
  Dtype* mutable_gpu_data() { return static_cast<Dtype*>(data_->mutable_gpu_data()); }
  Dtype* mutable_cpu_diff() { return static_cast<Dtype*>(diff_->mutable_cpu_data()); }
  Dtype* mutable_gpu_diff() { return static_cast<Dtype*>(diff_->mutable_gpu_data()); }
  void set_gpu_data(Dtype* p) { data_->set_gpu_data(p); }
  void set_gpu_diff(Dtype* p) { diff_->set_gpu_data(p); }

  // data -= diff (blob.cpp:156-179, caffe_gpu_axpy(-1))
  void Update();
  void ShareData(const Blob& o) { data_ = o.data_; }
  void ShareDiff(const Blob& o) { diff_ = o.diff_; }
  const std::shared_ptr<SyncedMemory>& data() const { return data_; }
  const std::shared_ptr<SyncedMemory>& diff() const { return diff_; }

 private:
  std::vector<int> shape_;
  int64_t count_ = 0, capacity_ = 0;
  std::shared_ptr<SyncedMemory> data_, diff_;
};

}  // namespace caffe
