// Native data-loading runtime: partitioned samplers + a multi-threaded,
// pinned-memory batch assembler.
//
// Replaces torch-dataset's Dataset(url, {partition, partitions}) +
// sampledBatcher{samplerKind, batchSize, processor} worker threads
// (examples/cifar10.lua:41-92, examples/mnist.lua:26-40, examples/Data.lua:10-61).
//
//  * PartitionSampler: node `partition` of `partitions` sees a contiguous
//    1/partitions slice of the dataset; kinds:
//      linear        - in order (test sets)
//      permutation   - a fresh shuffle of the slice every epoch (mnist.lua:31-40)
//      label-uniform - draw a class uniformly, then a sample of that class
//                      (cifar10.lua:53-71)
//      uniform       - i.i.d. uniform over the slice
//    Deterministic given (seed, partition): xoshiro256** streams.
//  * BatchAssembler: `threads` workers gather uint8 samples into `depth`
//    pinned host slots (hipHostMalloc) in sequence order, so the H2D copy of
//    slot k overlaps the gather of slot k+1..k+depth-1 and GPU compute.
//    Normalisation/cast happens on the GPU (metrics.hip gather_normalize), so
//    only uint8 crosses PCIe (4x less than fp32).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

#include "dl_common.h"

namespace dl {

struct Xoshiro256 {
  uint64_t s[4];
  static uint64_t splitmix(uint64_t& x) {
    uint64_t z = (x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  explicit Xoshiro256(uint64_t seed = 0) {
    uint64_t x = seed;
    for (auto& v : s) v = splitmix(x);
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
    s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }  // bias negligible for dataset sizes
};

enum SamplerKind : int { kLinear = 0, kPermutation = 1, kLabelUniform = 2, kUniform = 3 };

class PartitionSampler {
 public:
  // labels may be empty unless kind == kLabelUniform. partition is 0-based.
  PartitionSampler(int64_t n, std::vector<int64_t> labels, int num_classes, int partition, int partitions, int kind,
                   uint64_t seed)
      : kind_(kind), rng_(seed * 0x100000001b3ull + (uint64_t)partition) {
    if (partitions < 1 || partition < 0 || partition >= partitions) throw std::runtime_error("bad partition");
    lo_ = n * partition / partitions;
    hi_ = n * (partition + 1) / partitions;
    if (kind == kLabelUniform) {
      if ((int64_t)labels.size() != n) throw std::runtime_error("label-uniform sampler needs labels");
      by_class_.assign(num_classes, {});
      for (int64_t i = lo_; i < hi_; ++i) {
        int64_t c = labels[i];
        if (c < 0 || c >= num_classes) throw std::runtime_error("label out of range");
        by_class_[c].push_back(i);
      }
      for (auto& v : by_class_)
        if (!v.empty()) nonempty_.push_back(&v - &by_class_[0]);
      if (nonempty_.empty()) throw std::runtime_error("empty partition");
    }
    reset_epoch();
  }

  int64_t size() const { return hi_ - lo_; }
  int64_t num_batches(int64_t batch) const { return (size() + batch - 1) / batch; }

  void reset_epoch() {
    pos_ = 0;
    if (kind_ == kPermutation) {
      perm_.resize(size());
      for (int64_t i = 0; i < size(); ++i) perm_[i] = lo_ + i;
      for (int64_t i = size() - 1; i > 0; --i) std::swap(perm_[i], perm_[rng_.below(i + 1)]);
    }
  }

  // Fills `out[0:batch]`; returns the number of valid entries (the last batch
  // of a linear/permutation epoch may be short; its tail repeats the last index).
  int64_t next_batch(int64_t* out, int64_t batch) {
    int64_t valid = batch;
    for (int64_t b = 0; b < batch; ++b) {
      int64_t v;
      switch (kind_) {
        case kLinear:
        case kPermutation: {
          if (pos_ >= size()) {  // epoch wrap
            if (b > 0) { valid = std::min(valid, b); v = out[b - 1]; break; }
            reset_epoch();
          }
          v = kind_ == kLinear ? lo_ + pos_ : perm_[pos_];
          ++pos_;
          break;
        }
        case kLabelUniform: {
          const auto& cls = by_class_[nonempty_[rng_.below(nonempty_.size())]];
          v = cls[rng_.below(cls.size())];
          break;
        }
        default:
          v = lo_ + (int64_t)rng_.below(size());
      }
      out[b] = v;
    }
    return valid;
  }

 private:
  int kind_;
  int64_t lo_ = 0, hi_ = 0, pos_ = 0;
  Xoshiro256 rng_;
  std::vector<int64_t> perm_;
  std::vector<std::vector<int64_t>> by_class_;
  std::vector<int64_t> nonempty_;
};

class BatchAssembler {
 public:
  // images: host uint8 [n, sample_bytes], labels: host int64 [n] (both must
  // stay alive), sampler owned by the assembler.
  BatchAssembler(uintptr_t images, uintptr_t labels, int64_t n, int64_t sample_bytes, PartitionSampler* sampler,
                 int64_t batch, int threads, int depth)
      : img_((const uint8_t*)images), lab_((const int64_t*)labels), n_(n), sb_(sample_bytes), sampler_(sampler),
        batch_(batch), depth_(depth) {
    if (depth < 1 || threads < 1) throw std::runtime_error("depth/threads must be >= 1");
    slots_.resize(depth);
    for (auto& s : slots_) {
      // pinned (DMA-able) host slots when a HIP device exists; plain memory otherwise (CPU tests)
      if (hipHostMalloc((void**)&s.images, batch * sample_bytes, hipHostMallocDefault) != hipSuccess ||
          hipHostMalloc((void**)&s.labels, batch * sizeof(int64_t), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        pinned_ = false;
        s.images = (uint8_t*)std::malloc(batch * sample_bytes);
        s.labels = (int64_t*)std::malloc(batch * sizeof(int64_t));
        if (!s.images || !s.labels) throw std::runtime_error("BatchAssembler: out of host memory");
      }
      s.indices.resize(batch);
    }
    for (int t = 0; t < threads; ++t) workers_.emplace_back([this] { work(); });
  }

  ~BatchAssembler() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& w : workers_) w.join();
    for (auto& s : slots_) {
      if (pinned_) {
        (void)hipHostFree(s.images);
        (void)hipHostFree(s.labels);
      } else {
        std::free(s.images);
        std::free(s.labels);
      }
    }
    delete sampler_;
  }

  // Blocks until the next batch in sequence order is ready; returns its slot.
  int next() {
    std::unique_lock<std::mutex> lk(mu_);
    const int64_t seq = consume_seq_++;
    const int slot = (int)(seq % depth_);
    cv_.wait(lk, [&] { return slots_[slot].ready_seq == seq || stop_; });
    if (stop_) throw std::runtime_error("assembler stopped");
    slots_[slot].in_use = true;
    return slot;
  }

  void release(int slot) {
    {
      std::lock_guard<std::mutex> g(mu_);
      slots_[slot].in_use = false;
      slots_[slot].ready_seq = -1;
    }
    cv_.notify_all();
  }

  uintptr_t slot_images(int s) const { return (uintptr_t)slots_[s].images; }
  uintptr_t slot_labels(int s) const { return (uintptr_t)slots_[s].labels; }
  int64_t slot_valid(int s) const { return slots_[s].valid; }
  int64_t num_batches() const { return sampler_->num_batches(batch_); }
  void reset_epoch() {
    std::lock_guard<std::mutex> g(mu_);
    sampler_->reset_epoch();
  }

 private:
  struct Slot {
    uint8_t* images = nullptr;
    int64_t* labels = nullptr;
    std::vector<int64_t> indices;
    int64_t valid = 0;
    int64_t ready_seq = -1;
    bool in_use = false;
    bool filling = false;
  };

  void work() {
    for (;;) {
      int slot;
      int64_t seq;
      {
        std::unique_lock<std::mutex> lk(mu_);
        // the next sequence number may be produced once its slot is free
        cv_.wait(lk, [&] {
          if (stop_) return true;
          const Slot& s = slots_[produce_seq_ % depth_];
          return produce_seq_ < consume_seq_ + depth_ && !s.in_use && !s.filling && s.ready_seq < 0;
        });
        if (stop_) return;
        seq = produce_seq_++;
        slot = (int)(seq % depth_);
        Slot& s = slots_[slot];
        s.filling = true;
        s.valid = sampler_->next_batch(s.indices.data(), batch_);  // sequence-ordered draw
      }
      Slot& s = slots_[slot];
      for (int64_t b = 0; b < batch_; ++b) {
        const int64_t i = s.indices[b];
        std::memcpy(s.images + b * sb_, img_ + i * sb_, sb_);
        s.labels[b] = lab_ ? lab_[i] : 0;
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        s.filling = false;
        s.ready_seq = seq;
      }
      cv_.notify_all();
    }
  }

  const uint8_t* img_;
  const int64_t* lab_;
  int64_t n_, sb_;
  PartitionSampler* sampler_;
  int64_t batch_;
  int depth_;
  std::vector<Slot> slots_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_;
  int64_t produce_seq_ = 0, consume_seq_ = 0;
  bool stop_ = false;
  bool pinned_ = true;
};

}  // namespace dl
