// Microbenchmark: back-to-back launch cost of an (almost) empty kernel vs grid
// size, block size and static LDS.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int LDS_BYTES>
__global__ __launch_bounds__(256) void empty_kernel(int *out, int flag) {
  __shared__ int buf[LDS_BYTES / 4 > 0 ? LDS_BYTES / 4 : 1];
  if (flag == 12345) {  // never true: keeps the LDS allocation alive
    buf[threadIdx.x] = threadIdx.x;
    __syncthreads();
    out[blockIdx.x] = buf[(threadIdx.x + 1) & 255];
  }
}

template <int LDS>
float time_it(int blocks, int threads, int *d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 20; ++i) empty_kernel<LDS><<<blocks, threads>>>(d, 0);
  hipEventRecord(e0);
  const int n = 200;
  for (int i = 0; i < n; ++i) empty_kernel<LDS><<<blocks, threads>>>(d, 0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / n;
}

int main() {
  int *d;
  (void)hipMalloc(&d, 1 << 20);
  for (int blocks : {256, 512, 1024, 2496, 4096, 8192}) {
    printf("blocks %5d x256: lds0 %.2f us  lds17K %.2f us  lds64K %.2f us | x64 lds0 %.2f us\n", blocks,
           time_it<0>(blocks, 256, d), time_it<17 * 1024>(blocks, 256, d),
           time_it<64 * 1024>(blocks, 256, d), time_it<0>(blocks, 64, d));
  }
  return 0;
}
