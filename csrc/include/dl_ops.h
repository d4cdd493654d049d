// Host-side launcher declarations for every HIP kernel in csrc/kernels.
// All take raw device pointers (uintptr_t) and a HIP stream handle so that the
// Python layer can enqueue them on torch streams (and inside hipGraph capture).
#pragma once
#include <stdint.h>

namespace dl {

// flat_ops.hip -------------------------------------------------------------
void sgd_update(uintptr_t p, uintptr_t g, uintptr_t mom, uintptr_t p16, uintptr_t slot, float lr, float momentum,
                float wd, int64_t n, uintptr_t stream);
void scale_by_count(uintptr_t x, uintptr_t slot, int64_t n, uintptr_t stream);
void elastic_step(uintptr_t p, uintptr_t c, uintptr_t pending, uintptr_t out, uintptr_t p16, float alpha, int64_t n,
                  uintptr_t stream);
void add_inplace(uintptr_t y, uintptr_t x, int64_t n, uintptr_t stream);
void fill_f32(uintptr_t x, float v, int64_t n, int64_t slot_index, float slot_value, uintptr_t stream);
void cast_f32_bf16(uintptr_t x, uintptr_t y, int64_t n, uintptr_t stream);
void multi_copy(uintptr_t segs, int nseg, int64_t max_bytes, uintptr_t stream);

// metrics.hip ---------------------------------------------------------------
void confusion_update(uintptr_t pred, int pred_is_bf16, uintptr_t target, uintptr_t mat, int B, int C,
                      uintptr_t stream);
void gather_normalize(uintptr_t images, uintptr_t idx, uintptr_t out, int B, int HW, int Cs, int Cd, float m0,
                      float m1, float m2, float s0, float s1, float s2, uintptr_t stream);

}  // namespace dl
