// MFMA throughput calibration: every wave issues N x 16 v_mfma_f32_16x16x32_bf16 on
// 16 independent accumulators (operands in registers).  Sweeps workgroup size /
// count; reports TFLOP/s.  One JSON object on stdout.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void mfma_kernel(int n, float *sink) {
  const int lane = threadIdx.x & 63;
  bf16x8 a = bf16x8{short(lane), 1, 2, 3, 4, 5, 6, 7};
  bf16x8 b = bf16x8{7, 6, 5, 4, 3, 2, 1, short(lane)};
  f32x4 acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < n; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 1.2345f) sink[0] = s;
}

int main() {
  float *sink;
  CK(hipMalloc(&sink, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("{\"runs\": [");
  bool first = true;
  const int n = 256;  // 4096 MFMAs per wave
  for (int threads : {64, 256, 512}) {
    for (int waves_total : {256, 1024, 2048}) {
      const int grid = waves_total / (threads / 64);
      mfma_kernel<<<grid, threads>>>(n, sink);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int r = 0; r < 10; ++r) mfma_kernel<<<grid, threads>>>(n, sink);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 100.0;  // per launch
      const double flops = 2.0 * 16 * 16 * 32 * 16.0 * n * waves_total;
      printf("%s{\"threads\": %d, \"waves\": %d, \"us\": %.2f, \"TFLOP/s\": %.0f}", first ? "" : ", ",
             threads, waves_total, us, flops / us / 1e6);
      first = false;
    }
  }
  printf("]}\n");
  return 0;
}
