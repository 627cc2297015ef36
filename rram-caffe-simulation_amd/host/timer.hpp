// hipEvent timers on the working stream (benchmark.cpp:30-95 Timer, used by
// `caffe time`, tools/caffe.cpp:334-421).  Events are recorded around each
// timed region without synchronising; collect() waits once and sums.
#pragma once

#include <map>
#include <string>
#include <utility>
#include <vector>

#include "common.hpp"

namespace caffe {

class EventTimer {
 public:
  ~EventTimer() { clear(); }
  // stream: where the timed work runs (nullptr = the working stream)
  void start(int key, hipStream_t stream = nullptr) {
    hipEvent_t a = take(), b = take();
    HIP_CALL(hipEventRecord(a, stream ? stream : Caffe::hip_stream()));
    open_[key] = pending_.size();
    pending_.push_back({key, {a, b}});
  }
  void stop(int key, hipStream_t stream = nullptr) {
    auto it = open_.find(key);
    CAFFE_CHECK(it != open_.end(), "EventTimer::stop without start");
    HIP_CALL(hipEventRecord(pending_[it->second].second.second, stream ? stream : Caffe::hip_stream()));
    open_.erase(it);
  }
  // waits for all recorded intervals; adds them to totals() / counts()
  void collect() {
    for (auto& p : pending_) {
      HIP_CALL(hipEventSynchronize(p.second.second));
      float ms = 0.f;
      HIP_CALL(hipEventElapsedTime(&ms, p.second.first, p.second.second));
      totals_[p.first] += ms;
      counts_[p.first] += 1;
      free_.push_back(p.second.first);
      free_.push_back(p.second.second);
    }
    pending_.clear();
  }
  void clear() {
    for (auto& p : pending_) {
      free_.push_back(p.second.first);
      free_.push_back(p.second.second);
    }
    for (hipEvent_t e : free_) (void)hipEventDestroy(e);
    free_.clear();
    pending_.clear();
    open_.clear();
    totals_.clear();
    counts_.clear();
  }
  const std::map<int, double>& totals() const { return totals_; }
  const std::map<int, long>& counts() const { return counts_; }

 private:
  // events are pooled (no create/destroy per interval) and skip the
  // system-scope release fence: they only order work on this device
  hipEvent_t take() {
    if (!free_.empty()) {
      hipEvent_t e = free_.back();
      free_.pop_back();
      return e;
    }
    hipEvent_t e;
    HIP_CALL(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    return e;
  }
  std::vector<hipEvent_t> free_;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending_;
  std::map<int, size_t> open_;
  std::map<int, double> totals_;
  std::map<int, long> counts_;
};

}  // namespace caffe
