// Test/diagnostic support (NOT part of the product library): built into the
// separate extension torch_distlearn_amd._C_testing by csrc/build.py.
//
// Emulate the CU footprint of a concurrently running RCCL
// collective on one GPU.
//
// RCCL's gfx950 all-reduce workgroup (rcclGenericKernel in librccl's code
// object: 256 threads, 261-280 arch VGPRs + 17-32 AGPRs, 19,744 B LDS) shares
// a CU only with compute workgroups that fit beside it.  On a multi-GPU run
// the bucketed all-reduce overlaps the backward convolutions; this kernel
// reproduces that footprint (same workgroup size, register and LDS budget)
// so the effect of R occupied CUs on the training step can be measured on a
// one-GPU box (scripts/emulate_rccl.py).  Each workgroup spins on the 100 MHz
// constant clock for `us` microseconds and exits: every wave reaches the end.
#include <pybind11/pybind11.h>

#include "dl_common.h"

namespace dl {

__global__ void __launch_bounds__(256) occupy_kernel(int us, float* __restrict__ sink) {
  __shared__ float lds[19744 / 4];
  // claim the register budget of an RCCL wave: arch VGPRs up to v255, 32 AGPRs
  asm volatile("" ::: "v255", "a31");
  lds[threadIdx.x] = (float)threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long ticks = (unsigned long long)us * 100ull;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (threadIdx.x == 0 && sink) sink[blockIdx.x] = lds[(blockIdx.x + 1) & 255];
}

// Control: one wave, no LDS, few registers -- fits beside any workgroup, so
// whatever it costs the step is the price of a second active queue, not of
// occupied CU resources.
__global__ void __launch_bounds__(64) occupy_light_kernel(int us, float* __restrict__ sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long ticks = (unsigned long long)us * 100ull;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0 && sink) sink[blockIdx.x] = 1.f;
}

void occupy_cus(int blocks, int us, uintptr_t sink, uintptr_t stream) {
  if (blocks == 0) return;
  if (us > 2000000) throw std::runtime_error("occupy_cus: at most 2 s");
  if (blocks < 0)  // light control variant
    occupy_light_kernel<<<-blocks, 64, 0, as_stream(stream)>>>(us, (float*)sink);
  else
    occupy_kernel<<<blocks, 256, 0, as_stream(stream)>>>(us, (float*)sink);
  DL_HIP_CHECK(hipGetLastError());
}

// Price of the per-K-step synchronisation of the conv kernels: `n` rounds of
// (mode 0) s_barrier, (1) lgkmcnt(0) + s_barrier, (2) one ds_read_b128 of the
// ring + lgkmcnt(0) + s_barrier, in `blocks` workgroups of `threads` holding
// `lds` bytes of dynamic LDS (128 KiB = the wgrad's one workgroup per CU).
__global__ void barrier_loop_kernel(int n, int mode, float* __restrict__ sink) {
  extern __shared__ float dyn[];
  float acc = 0.f;
  for (int i = 0; i < n; ++i) {
    if (mode == 2) {
      acc += dyn[(threadIdx.x * 4 + i * 64) & 1023];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else if (mode == 1) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
  }
  if (threadIdx.x == 0 && sink) sink[blockIdx.x] = acc;
}

void barrier_loop(int blocks, int threads, int n, int mode, int lds, uintptr_t sink, uintptr_t stream) {
  if (threads % 64 || threads > 1024 || lds < 4096 || lds > 160 * 1024 || n < 0 || n > 1000000)
    throw std::runtime_error("barrier_loop: bad launch");
  static bool attr = false;
  if (!attr) {
    DL_HIP_CHECK(hipFuncSetAttribute((const void*)barrier_loop_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024));
    attr = true;
  }
  barrier_loop_kernel<<<blocks, threads, lds, as_stream(stream)>>>(n, mode, (float*)sink);
  DL_HIP_CHECK(hipGetLastError());
}

// Fill every CU's LDS with a bit pattern (all 160 KiB of dynamic LDS, one
// workgroup per CU x `rounds`): a kernel that reads LDS it never wrote in its
// own launch then sees the pattern instead of whatever an earlier kernel left.
__global__ void __launch_bounds__(256) lds_poison_kernel(unsigned pattern) {
  extern __shared__ unsigned dynp[];
  for (int i = threadIdx.x; i < 160 * 1024 / 4; i += 256) dynp[i] = pattern;
  __syncthreads();
}

void lds_poison(int blocks, unsigned pattern, uintptr_t stream) {
  static bool attr = false;
  if (!attr) {
    DL_HIP_CHECK(hipFuncSetAttribute((const void*)lds_poison_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024));
    attr = true;
  }
  if (blocks < 1 || blocks > 65536) throw std::runtime_error("lds_poison: bad grid");
  lds_poison_kernel<<<blocks, 256, 160 * 1024, as_stream(stream)>>>(pattern);
  DL_HIP_CHECK(hipGetLastError());
}

}  // namespace dl

PYBIND11_MODULE(_C_testing, m) {
  m.def("lds_poison", &dl::lds_poison);
  m.def("barrier_loop", &dl::barrier_loop);
  m.doc() = "distlearn test/diagnostic kernels (not part of the product library)";
  m.def("occupy_cus", &dl::occupy_cus);
}
