// L2 broadcast-read ceiling for the fused tower's access shape (tower.hip): every
// workgroup streams the SAME weight image (L2 / MALL resident) in 1 KiB blocks,
// wave w reading tiles w, w + 8, ... with PF k steps of NT blocks in flight.
// Sweeps the grid (CUs busy), threads per workgroup, PF and a per-workgroup
// rotation of the starting step, and reports per-CU and aggregate GB/s, so the
// tower's bound (per-CU fill rate vs the XCD L2's aggregate rate) is measured,
// not guessed.  One JSON object on stdout.  Build: hipcc --offload-arch=gfx950 -O3.
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

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// image: tiles x ksteps blocks of 1 KiB; each wave owns tiles wave + nw * i
template <int PF, int NT>
__global__ void bcast_kernel(const char *__restrict__ img, int tiles, int ksteps, int reps, int rotate,
                             uint32_t *__restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int bytes = tiles * ksteps * 1024;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(img), 0, bytes, 0x00020000);
  int voff[NT];
  int nreal = 0;
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const int t = wave + nw * i;
    voff[i] = (t < tiles ? t : 0) * ksteps * 1024 + lane * 16;
    nreal += t < tiles;
  }
  const int rot = rotate ? static_cast<int>(blockIdx.x % static_cast<unsigned>(ksteps)) : 0;
  uint32_t x = 0;
  for (int r = 0; r < reps; ++r) {
    u32x4 w[PF][NT];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int s = (p + rot) % ksteps;
#pragma unroll
      for (int i = 0; i < NT; ++i)
        w[p][i] = i < nreal ? __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff[i], s * 1024, 0) : u32x4{0, 0, 0, 0};
    }
    for (int s0 = 0; s0 < ksteps; s0 += PF) {
#pragma unroll
      for (int p = 0; p < PF; ++p) {
#pragma unroll
        for (int i = 0; i < NT; ++i) x ^= w[p][i].x ^ w[p][i].y ^ w[p][i].z ^ w[p][i].w;
        const int sn = s0 + p + PF;
        if (sn < ksteps) {
          const int s = (sn + rot) % ksteps;
#pragma unroll
          for (int i = 0; i < NT; ++i)
            w[p][i] = i < nreal ? __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff[i], s * 1024, 0) : u32x4{0, 0, 0, 0};
        }
      }
    }
  }
  if (x == 0x9e3779b9u) sink[0] = x;
}

template <int PF, int NT>
static float run(const char *img, int tiles, int ksteps, int reps, int rotate, int grid, int threads,
                 uint32_t *sink) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i)
    bcast_kernel<PF, NT><<<grid, threads>>>(img, tiles, ksteps, reps, rotate, sink);
  CK(hipDeviceSynchronize());
  const int it = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < it; ++i)
    bcast_kernel<PF, NT><<<grid, threads>>>(img, tiles, ksteps, reps, rotate, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1000.f / it;
}

int main() {
  // one 400 x 432 layer image: 25 tiles x 14 k steps of 1 KiB (350 KiB)
  const int tiles = 25, ksteps = 14, reps = 6;
  char *img;
  uint32_t *sink;
  CK(hipMalloc(&img, tiles * ksteps * 1024));
  CK(hipMemset(img, 1, tiles * ksteps * 1024));
  CK(hipMalloc(&sink, 64));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("{\"what\": \"every workgroup streams the same %d-KiB image %d times (tower access shape)\", "
         "\"cus\": %d, \"runs\": [", tiles * ksteps, reps, cus);
  bool first = true;
  const int grids[] = {32, 64, 128, 256, 512};
  for (int threads : {512, 256}) {
    for (int rotate : {1, 0}) {
      for (int pf : {4, 8}) {
        for (int g : grids) {
          const int nw = threads / 64;
          float us;
          if (nw == 8)
            us = pf == 4 ? run<4, 4>(img, tiles, ksteps, reps, rotate, g, threads, sink)
                         : run<8, 4>(img, tiles, ksteps, reps, rotate, g, threads, sink);
          else
            us = pf == 4 ? run<4, 7>(img, tiles, ksteps, reps, rotate, g, threads, sink)
                         : run<8, 7>(img, tiles, ksteps, reps, rotate, g, threads, sink);
          const double bytes = static_cast<double>(g) * tiles * ksteps * 1024 * reps;
          const int busy = g < cus ? g : cus;
          printf("%s{\"threads\": %d, \"rotate\": %d, \"pf\": %d, \"grid\": %d, \"us\": %.2f, "
                 "\"agg_GB/s\": %.0f, \"per_cu_GB/s\": %.1f}",
                 first ? "" : ", ", threads, rotate, pf, g, us, bytes / us / 1e3, bytes / us / 1e3 / busy);
          first = false;
        }
      }
    }
  }
  printf("]}\n");
  return 0;
}
