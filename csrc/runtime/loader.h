// Native data-loading runtime: partitioned samplers.
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
//  The dataset partition itself lives in HBM (data/__init__.py): a step
//  uploads only indices (or nothing: DeviceLoader), and the gather +
//  normalisation is a GPU kernel (metrics.hip gather_normalize, prep_step_gather).
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


}  // namespace dl
