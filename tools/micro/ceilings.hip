// Step-0 memory ceilings of one MI355X (SURVEY.md §7 step 0, §8(d) "attainable"):
//   * stream copy / stream read (16 B per lane, grid-stride), GB/s;
//   * random row gather: ids (uint32, uniform) -> rows of P = 32 / 64 / 128 B read
//     by P/16 lanes with one 16-B load each (the bank's access shape), from a
//     table of 64 MB (the C2 bank: Infinity-Cache resident) and 6 GB (HBM);
//       - bandwidth form: 16 M lookups per launch,
//       - C2 form: 4096 x 26 = 106,496 lookups per launch (one step's gather),
//         the latency-bound shape the interaction kernel runs at.
// Output: one JSON object on stdout.  Every timing is the average over back-to-back
// launches bracketed by HIP events.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ __launch_bounds__(256) void copy_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst,
                                                   int64_t n) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += gridDim.x * 256ll) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void read_kernel(const uint4 *__restrict__ src, int64_t n,
                                                   uint32_t *__restrict__ sink) {
  uint32_t x = 0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += gridDim.x * 256ll) {
    const uint4 v = src[i];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x9e3779b9u) sink[0] = x;  // keeps the loads alive
}

__global__ __launch_bounds__(256) void ids_kernel(uint32_t *ids, int64_t n, uint32_t rows, uint32_t seed) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= n) return;
  uint64_t z = (static_cast<uint64_t>(i) + seed) * 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z ^= z >> 31;
  ids[i] = static_cast<uint32_t>(z % rows);
}

// one worker of LPR lanes per lookup, W lookups in flight per worker
template <int LPR, int W>
__global__ __launch_bounds__(256) void gather_kernel(const uint4 *__restrict__ table, const uint32_t *__restrict__ ids,
                                                     int64_t n, uint32_t *__restrict__ sink) {
  constexpr int WPB = 256 / LPR;
  const int l = threadIdx.x % LPR;
  const int64_t w0 = (blockIdx.x * static_cast<int64_t>(WPB) + threadIdx.x / LPR) * W;
  uint32_t id[W];
#pragma unroll
  for (int k = 0; k < W; ++k) id[k] = w0 + k < n ? ids[w0 + k] : 0xffffffffu;
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < W; ++k) {
    if (id[k] != 0xffffffffu) {
      const uint4 v = table[static_cast<int64_t>(id[k]) * LPR + l];
      x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (x == 0x9e3779b9u) sink[0] = x;
}

__global__ void empty_kernel(uint32_t *sink, int flag) {
  if (flag == 12345) sink[0] = 1;
}

template <typename F>
static double time_us(F &&launch, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) launch();
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1e3 / reps;
}

template <int LPR>
static double gather_us(const uint4 *table, const uint32_t *ids, int64_t n, uint32_t *sink, int reps) {
  constexpr int W = 4;
  constexpr int WPB = 256 / LPR;
  const int64_t blocks = (n + WPB * W - 1) / (WPB * W);
  return time_us([&] { gather_kernel<LPR, W><<<dim3(static_cast<unsigned>(blocks)), 256>>>(table, ids, n, sink); },
                 reps);
}

int main(int argc, char **argv) {
  const bool quick = argc > 1 && std::string(argv[1]) == "--quick";
  uint32_t *sink;
  CK(hipMalloc(&sink, 64));
  std::string js = "{";
  char buf[512];

  // --- stream copy / read over 2 GiB ---
  {
    const int64_t bytes = int64_t(2) << 30;
    uint4 *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 0, bytes));
    const int64_t n = bytes / 16;
    const unsigned grid = 256 * 8;
    const double tc = time_us([&] { copy_kernel<<<grid, 256>>>(a, b, n); }, 20);
    const double tr = time_us([&] { read_kernel<<<grid, 256>>>(a, n, sink); }, 20);
    snprintf(buf, sizeof buf,
             "\"stream_copy\": {\"bytes_moved\": %lld, \"us\": %.1f, \"GB/s\": %.0f}, "
             "\"stream_read\": {\"bytes\": %lld, \"us\": %.1f, \"GB/s\": %.0f}, ",
             (long long)(2 * bytes), tc, 2.0 * bytes / tc * 1e-3, (long long)bytes, tr, bytes / tr * 1e-3);
    js += buf;
    CK(hipFree(a));
    CK(hipFree(b));
  }

  // --- dependent launch floor ---
  {
    const double te = time_us([&] { empty_kernel<<<256, 256>>>(sink, 0); }, 200);
    snprintf(buf, sizeof buf, "\"empty_launch_us\": %.2f, ", te);
    js += buf;
  }

  // --- random row gathers ---
  js += "\"gather\": [";
  const int64_t big_n = int64_t(16) << 20;   // lookups, bandwidth form
  const int64_t c2_n = int64_t(4096) * 26;   // lookups, one C2 step
  uint32_t *ids;
  CK(hipMalloc(&ids, big_n * 4));
  bool first = true;
  std::vector<int64_t> tables = {int64_t(64) << 20};
  if (!quick) tables.push_back(int64_t(6) << 30);
  for (int64_t tbytes : tables) {
    uint4 *table;
    CK(hipMalloc(&table, tbytes));
    CK(hipMemset(table, 3, tbytes));
    for (int pitch : {32, 64, 128}) {
      const uint32_t rows = static_cast<uint32_t>(tbytes / pitch);
      ids_kernel<<<dim3(static_cast<unsigned>((big_n + 255) / 256)), 256>>>(ids, big_n, rows, 17u + pitch);
      CK(hipDeviceSynchronize());
      double tb = 0, tc2 = 0;
      switch (pitch) {
        case 32: tb = gather_us<2>(table, ids, big_n, sink, 10); tc2 = gather_us<2>(table, ids, c2_n, sink, 200); break;
        case 64: tb = gather_us<4>(table, ids, big_n, sink, 10); tc2 = gather_us<4>(table, ids, c2_n, sink, 200); break;
        default: tb = gather_us<8>(table, ids, big_n, sink, 10); tc2 = gather_us<8>(table, ids, c2_n, sink, 200); break;
      }
      snprintf(buf, sizeof buf,
               "%s{\"table_bytes\": %lld, \"row_bytes\": %d, \"lookups\": %lld, \"us\": %.1f, "
               "\"row_GB/s\": %.0f, \"c2_lookups\": %lld, \"c2_us\": %.2f, \"c2_row_GB/s\": %.0f}",
               first ? "" : ", ", (long long)tbytes, pitch, (long long)big_n, tb, big_n * double(pitch) / tb * 1e-3,
               (long long)c2_n, tc2, c2_n * double(pitch) / tc2 * 1e-3);
      js += buf;
      first = false;
    }
    CK(hipFree(table));
  }
  js += "]}";
  printf("%s\n", js.c_str());
  return 0;
}
