// LDS-DMA lane-pattern microbenchmark for the weight-gradient GEMM's operand
// stream (gemm.hip, COL operands: dW = dY^T X over the batch).  Every workgroup
// (256 threads, 48 KiB ring of 3 k groups, 3 per CU) streams a 64-column panel of
// a [4096 x 400] bf16 matrix over a 512-row K slice into LDS, 8 pieces of 1 KiB per
// 64-row group, like gemm_tile; nothing is computed.  Lane patterns of a piece
// (8 rows x 128 B either way):
//   col  : gemm.hip's COL mapping (lanes 2q, 2q+1 one row: a 4-lane quad spans 2 rows)
//   row  : lane = 8 row + chunk (a quad spans 64 contiguous bytes of one row)
//   vgpr : the row pattern through VGPRs (global_load_dwordx4 + ds_write_b128)
// Reports us per launch and GB/s per CU.  One JSON object on stdout.
#include <hip/hip_runtime.h>

#include <cstdint>
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

constexpr int KG = 64, NBUF = 3, COLS = 400, ROWS = 4096, KSLICE = 4096;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int PAT>
__global__ __launch_bounds__(256) void stream_kernel(const uint16_t *__restrict__ m, int panels,
                                                     uint32_t *sink) {
  __shared__ __attribute__((aligned(16))) uint16_t ring[NBUF][8 * 512];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // grids of several copies re-read the same slices: slice wraps at ROWS / KSLICE
  const int panel = blockIdx.x % panels, slice = (blockIdx.x / panels) % (ROWS / KSLICE);
  const int c0 = panel * 64;
  const int64_t r0 = static_cast<int64_t>(slice) * KSLICE;
  int roff[2], coff[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int t = wave + 4 * u;
    if (PAT == 0) {  // gemm.hip COL
      coff[u] = (lane >> 4) * 16 + (lane & 1) * 8;
      roff[u] = t * 8 + ((lane & 15) >> 1);
    } else {
      coff[u] = (lane & 7) * 8;
      roff[u] = t * 8 + (lane >> 3);
    }
    if (c0 + coff[u] >= COLS) coff[u] = 0;  // keep inside the matrix (timing only)
  }
  constexpr int NG = KSLICE / KG;
  uint4 v[2];
  auto issue = [&](int kg) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint16_t *src = m + (r0 + kg * KG + roff[u]) * COLS + c0 + coff[u];
      if (PAT == 2)
        v[u] = *reinterpret_cast<const uint4 *>(src);
      else
        __builtin_amdgcn_global_load_lds(src, &ring[kg % NBUF][(wave + 4 * u) * 512], 16, 0, 0);
    }
  };
  uint32_t x = 0;
  if (PAT == 2) {
    for (int kg = 0; kg < NG; ++kg) {
      issue(kg);
#pragma unroll
      for (int u = 0; u < 2; ++u)
        *reinterpret_cast<uint4 *>(&ring[kg % NBUF][(wave + 4 * u) * 512 + lane * 8]) = v[u];
      __syncthreads();
      x ^= ring[kg % NBUF][tid * 4];
    }
  } else {
    for (int kg = 0; kg < NBUF - 1; ++kg) issue(kg);
    for (int kg = 0; kg < NG; ++kg) {
      if (kg + 1 < NG) wait_vmcnt<2>(); else wait_vmcnt<0>();
      asm volatile("s_barrier" ::: "memory");
      if (kg + NBUF - 1 < NG) issue(kg + NBUF - 1);
      x ^= ring[kg % NBUF][tid * 4];
    }
  }
  if (x == 0x9e3779b9u) sink[0] = x;
}

template <int PAT>
static float run(const uint16_t *m, int grid, int panels, uint32_t *sink) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) stream_kernel<PAT><<<grid, 256>>>(m, panels, sink);
  CK(hipDeviceSynchronize());
  const int it = 50;
  CK(hipEventRecord(e0));
  for (int i = 0; i < it; ++i) stream_kernel<PAT><<<grid, 256>>>(m, panels, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / it;
}

int main() {
  uint16_t *m;
  uint32_t *sink;
  CK(hipMalloc(&m, static_cast<size_t>(ROWS) * COLS * 2));
  CK(hipMemset(m, 1, static_cast<size_t>(ROWS) * COLS * 2));
  CK(hipMalloc(&sink, 64));
  const int panels = 7, slices = ROWS / KSLICE;
  const char *names[3] = {"col", "row", "vgpr"};
  printf("{\"what\": \"64-col panels of a [4096 x 400] bf16 matrix, all 4096 rows per workgroup, 8 x 1 KiB "
         "pieces per 64-row group\", \"runs\": [");
  bool first = true;
  (void)slices;
  for (int grid : {56, 256, 512, 768}) {  // workgroups, each streaming a whole 4096-row panel
    for (int pat = 0; pat < 3; ++pat) {
      const float us = pat == 0 ? run<0>(m, grid, panels, sink)
                                : pat == 1 ? run<1>(m, grid, panels, sink) : run<2>(m, grid, panels, sink);
      const double bytes = static_cast<double>(grid) * KSLICE * 128;
      const int busy = grid < 256 ? grid : 256;
      printf("%s{\"pattern\": \"%s\", \"grid\": %d, \"us\": %.2f, \"GB/s\": %.0f, \"per_cu_GB/s\": %.1f}",
             first ? "" : ", ", names[pat], grid, us, bytes / us / 1e3, bytes / us / 1e3 / busy);
      first = false;
    }
  }
  printf("]}\n");
  return 0;
}
