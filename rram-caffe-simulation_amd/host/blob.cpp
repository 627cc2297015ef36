#include "blob.hpp"

#include <atomic>
#include <cstdlib>
#include <cstring>

namespace caffe {

Caffe& Caffe::Get() {
  static thread_local Caffe inst;  // one context per thread (common.cpp:13-20)
  return inst;
}

std::atomic<uint64_t>& Caffe::scratch_gen() {
  static std::atomic<uint64_t> g{0};
  return g;
}

void* Caffe::workspace(size_t bytes) {
  Caffe& c = Get();
  if (bytes > c.ws_bytes_) {
    if (c.ws_) {
      HIP_CALL(hipStreamSynchronize(hip_stream()));
      HIP_CALL(hipFree(c.ws_));
      scratch_gen().fetch_add(1);
    }
    c.ws_ = nullptr;
    HIP_CALL(hipMalloc(&c.ws_, bytes));
    c.ws_bytes_ = bytes;
  }
  return c.ws_;
}

void Caffe::synchronize() { HIP_CALL(hipStreamSynchronize(hip_stream())); }

SyncedMemory::~SyncedMemory() {
  if (own_cpu_ && cpu_ptr_) std::free(cpu_ptr_);
  if (own_gpu_ && gpu_ptr_) (void)hipFree(gpu_ptr_);
  if (oct_ptr_) (void)hipFree(oct_ptr_);
  if (wp_ptr_) (void)hipFree(wp_ptr_);
  if (wf_ptr_) (void)hipFree(wf_ptr_);
  if (rw_ptr_) (void)hipFree(rw_ptr_);
}

void* SyncedMemory::rows(size_t bytes) {
  if (bytes > rw_bytes_) {
    if (rw_ptr_) {
      HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
      HIP_CALL(hipFree(rw_ptr_));
      Caffe::scratch_gen().fetch_add(1);
    }
    rw_ptr_ = nullptr;
    HIP_CALL(hipMalloc(&rw_ptr_, bytes));
    rw_bytes_ = bytes;
    rw_valid_ = false;
  }
  return rw_ptr_;
}

void* SyncedMemory::wflip(size_t bytes) {
  if (bytes > wf_bytes_) {
    if (wf_ptr_) {
      HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
      HIP_CALL(hipFree(wf_ptr_));
      Caffe::scratch_gen().fetch_add(1);
    }
    wf_ptr_ = nullptr;
    HIP_CALL(hipMalloc(&wf_ptr_, bytes));
    wf_bytes_ = bytes;
    wf_valid_ = false;
  }
  return wf_ptr_;
}

void* SyncedMemory::wpack(size_t bytes) {
  if (bytes > wp_bytes_) {
    if (wp_ptr_) {
      HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
      HIP_CALL(hipFree(wp_ptr_));
      Caffe::scratch_gen().fetch_add(1);
    }
    wp_ptr_ = nullptr;
    HIP_CALL(hipMalloc(&wp_ptr_, bytes));
    wp_bytes_ = bytes;
    wp_valid_ = false;
  }
  return wp_ptr_;
}

void* SyncedMemory::octets(size_t bytes) {
  if (bytes > oct_bytes_) {
    if (oct_ptr_) {
      HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
      HIP_CALL(hipFree(oct_ptr_));
      Caffe::scratch_gen().fetch_add(1);
    }
    oct_ptr_ = nullptr;
    HIP_CALL(hipMalloc(&oct_ptr_, bytes));
    oct_bytes_ = bytes;
    oct_valid_ = false;
  }
  return oct_ptr_;
}
const void* SyncedMemory::valid_octets(const int (&shape)[4]) const {
  if (!oct_valid_ || exposed_) return nullptr;
  for (int i = 0; i < 4; ++i)
    if (shape[i] != oct_shape_[i]) return nullptr;
  return oct_ptr_;
}
void SyncedMemory::set_octets_valid(const int (&shape)[4]) {
  for (int i = 0; i < 4; ++i) oct_shape_[i] = shape[i];
  oct_valid_ = oct_ptr_ != nullptr;
}

void SyncedMemory::to_cpu() {
  switch (head_) {
    case UNINITIALIZED:
      cpu_ptr_ = std::calloc(1, size_ ? size_ : 1);
      own_cpu_ = true;
      head_ = HEAD_AT_CPU;
      break;
    case HEAD_AT_GPU:
      if (!cpu_ptr_) {
        cpu_ptr_ = std::malloc(size_ ? size_ : 1);
        own_cpu_ = true;
      }
      HIP_CALL(hipMemcpyAsync(cpu_ptr_, gpu_ptr_, size_, hipMemcpyDeviceToHost, Caffe::hip_stream()));
      HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
      head_ = SYNCED;
      break;
    case HEAD_AT_CPU:
    case SYNCED:
      break;
  }
}

void SyncedMemory::to_gpu() {
  switch (head_) {
    case UNINITIALIZED:
      HIP_CALL(hipMalloc(&gpu_ptr_, size_ ? size_ : 4));
      HIP_CALL(hipMemsetAsync(gpu_ptr_, 0, size_, Caffe::hip_stream()));
      own_gpu_ = true;
      head_ = HEAD_AT_GPU;
      break;
    case HEAD_AT_CPU:
      if (!gpu_ptr_) {
        HIP_CALL(hipMalloc(&gpu_ptr_, size_ ? size_ : 4));
        own_gpu_ = true;
      }
      HIP_CALL(hipMemcpyAsync(gpu_ptr_, cpu_ptr_, size_, hipMemcpyHostToDevice, Caffe::hip_stream()));
      HIP_CALL(hipStreamSynchronize(Caffe::hip_stream()));
      head_ = SYNCED;
      break;
    case HEAD_AT_GPU:
    case SYNCED:
      break;
  }
}

const void* SyncedMemory::cpu_data() {
  CAFFE_CHECK(!fp32_stale, "host read of a blob whose producer wrote only its octet companion "
                           "(Net::materialize_blob first)");
  to_cpu();
  return cpu_ptr_;
}
const void* SyncedMemory::gpu_data() {
  to_gpu();
  return gpu_ptr_;
}
void* SyncedMemory::mutable_cpu_data() {
  oct_valid_ = false;
  wp_valid_ = false;
  wf_valid_ = false;
  rw_valid_ = false;
  fp32_stale = false;
  to_cpu();
  head_ = HEAD_AT_CPU;
  return cpu_ptr_;
}
void* SyncedMemory::mutable_gpu_data() {
  oct_valid_ = false;
  wp_valid_ = false;
  wf_valid_ = false;
  rw_valid_ = false;
  fp32_stale = false;
  to_gpu();
  head_ = HEAD_AT_GPU;
  return gpu_ptr_;
}
void SyncedMemory::set_cpu_data(void* data) {
  CAFFE_CHECK(data, "set_cpu_data(NULL)");
  oct_valid_ = false;
  wp_valid_ = false;
  wf_valid_ = false;
  rw_valid_ = false;
  fp32_stale = false;
  if (own_cpu_ && cpu_ptr_) std::free(cpu_ptr_);
  cpu_ptr_ = data;
  own_cpu_ = false;
  head_ = HEAD_AT_CPU;
}
void SyncedMemory::set_gpu_data(void* data) {
  CAFFE_CHECK(data, "set_gpu_data(NULL)");
  oct_valid_ = false;
  wp_valid_ = false;
  wf_valid_ = false;
  rw_valid_ = false;
  fp32_stale = false;
  if (own_gpu_ && gpu_ptr_) (void)hipFree(gpu_ptr_);
  gpu_ptr_ = data;
  own_gpu_ = false;
  head_ = HEAD_AT_GPU;
}

template <typename Dtype>
void Blob<Dtype>::Reshape(const std::vector<int>& shape) {
  int64_t c = 1;
  for (int d : shape) {
    CAFFE_CHECK(d >= 0, "negative blob dimension");
    c *= d;
  }
  shape_ = shape;
  count_ = c;
  if (count_ > capacity_ || !data_) {
    capacity_ = count_;
    data_ = std::make_shared<SyncedMemory>(capacity_ * sizeof(Dtype));
    diff_ = std::make_shared<SyncedMemory>(capacity_ * sizeof(Dtype));
  }
}

template <typename Dtype>
int64_t Blob<Dtype>::count(int start, int end) const {
  if (end < 0) end = num_axes();
  int64_t c = 1;
  for (int i = start; i < end; ++i) c *= shape_[i];
  return c;
}

template <typename Dtype>
std::string Blob<Dtype>::shape_string() const {
  std::ostringstream o;
  for (int d : shape_) o << d << " ";
  o << "(" << count_ << ")";
  return o.str();
}

template <typename Dtype>
void Blob<Dtype>::Update() {
  RRAM_CALL(rram_axpy(count_, Dtype(-1), gpu_diff(), mutable_gpu_data(), Caffe::stream()));
}

template class Blob<float>;

}  // namespace caffe
