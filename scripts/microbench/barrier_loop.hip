// Calibration: cost of an LDS-heavy workgroup's skeleton (barrier loop) on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int LDS_BYTES>
__global__ void __launch_bounds__(256) skel(int iters, int* out) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  int acc = threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    acc += smem[(threadIdx.x * 16 + i * 64) % LDS_BYTES];
  }
  if (acc == 123456) out[0] = acc;
}
template <int LDS>
float run(int grid, int iters, int* out) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) skel<LDS><<<grid, 256>>>(iters, out);
  hipEventRecord(a);
  for (int r = 0; r < 20; ++r) skel<LDS><<<grid, 256>>>(iters, out);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); return ms * 1000 / 20;
}
int main() {
  int* out; hipMalloc(&out, 4);
  for (int iters : {1, 25, 100}) {
    printf("iters %3d: lds16K grid256 %7.2f us | lds96K grid256 %7.2f us | lds96K grid1024 %7.2f us\n", iters,
           run<16384>(256, iters, out), run<98304>(256, iters, out), run<98304>(1024, iters, out));
  }
  return 0;
}
