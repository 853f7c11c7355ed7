// Microbenchmark: cost of a workgroup barrier (1024 threads) and the shader clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(1024) void bar_kernel(uint64_t *out, int iters, int mode) {
  __shared__ uint32_t x[1024];
  x[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const uint64_t w0 = wall_clock64();
  const uint64_t c0 = clock64();
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    if (mode == 0) {
      __syncthreads();
    } else if (mode == 1) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      acc += x[(threadIdx.x + i) & 1023];
      __syncthreads();
      x[(threadIdx.x * 7 + i) & 1023] = acc;
    }
  }
  const uint64_t w1 = wall_clock64();
  const uint64_t c1 = clock64();
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = w1 - w0;
    out[1] = c1 - c0;
    out[2] = acc;
  }
}

int main() {
  uint64_t *d, h[3];
  hipMalloc(&d, 64);
  for (int threads : {1024, 256, 64}) {
    for (int mode = 0; mode < 3; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(bar_kernel, dim3(26), dim3(threads), 0, 0, d, 1000, mode);
        hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
      }
      printf("threads %4d mode %d: %.1f ns/barrier, %.1f clk/barrier, clock %.2f GHz\n", threads,
             mode, h[0] * 10.0 / 1000, h[1] / 1000.0, h[1] / (h[0] * 10.0));
    }
  }
  return 0;
}
