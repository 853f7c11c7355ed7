// Batch feed: copy a packed batch record from pinned host memory into its device
// slot with a kernel on the caller's stream (pytorchrec_amd/loader.py).
//
// hipMemcpyAsync hands a pinned H2D copy to a DMA engine; a HIP graph launched
// behind it on the same stream then waits on the host for that engine
// (measured: 0.19-0.33 ms/step instead of 0.13).  Here the compute queue reads
// the host record directly over PCIe (the pinned allocation is device-visible
// at the same address), so the copy is one more kernel in stream order and the
// host never blocks.  16-B loads, several in flight per lane.
#include <algorithm>

#include "common.h"

namespace mrec {

__global__ __launch_bounds__(256) void batch_stage_kernel(const uint4 *__restrict__ src,
                                                          uint4 *__restrict__ dst, int64_t n16) {
  constexpr int U = 4;  // independent 16-B loads per lane per trip
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) dst[i + u * stride] = v[u];
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

// the record at the device cursor (state[0]) of a pinned epoch buffer; the last
// workgroup to finish (ticket state[1]) advances the cursor, so a HIP graph that
// contains this launch stages the NEXT record on every replay
__global__ __launch_bounds__(256) void batch_stage_cursor_kernel(const char *__restrict__ base,
                                                                 int64_t record_bytes,
                                                                 int64_t n_records,
                                                                 uint4 *__restrict__ dst,
                                                                 unsigned long long *state) {
  __shared__ long long s_rec;
  if (threadIdx.x == 0)
    s_rec = static_cast<long long>(__hip_atomic_load(state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  __syncthreads();
  const long long rec = s_rec;
  if (rec >= 0 && rec < n_records) {
    const uint4 *src = reinterpret_cast<const uint4 *>(base + rec * record_bytes);
    const int64_t n16 = record_bytes / 16;
    constexpr int U = 4;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
    int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = src[i + u * stride];
#pragma unroll
      for (int u = 0; u < U; ++u) dst[i + u * stride] = v[u];
    }
    for (; i < n16; i += stride) dst[i] = src[i];
  }
  __syncthreads();  // every thread of this workgroup has read the cursor (s_rec)
  if (threadIdx.x == 0) {
    const unsigned long long t =
        __hip_atomic_fetch_add(state + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {  // the last arriver: every workgroup read the cursor already
      __hip_atomic_store(state + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(state, static_cast<unsigned long long>(rec + 1), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace mrec

using namespace mrec;

extern "C" {

mrec_status mrec_batch_stage(void *dst, const void *host_src, int64_t bytes, mrec_stream stream) {
  MREC_CHECK_ARG(bytes >= 0, "bytes < 0");
  MREC_CHECK_ARG(bytes == 0 || (dst != nullptr && host_src != nullptr), "NULL pointer");
  MREC_CHECK_ARG(bytes % 16 == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(host_src) & 15) == 0,
                 "dst / host_src must be 16-B aligned and bytes a multiple of 16");
  if (bytes == 0) return MREC_OK;
  // the record must be pinned, device-visible host memory: translate it (and
  // refuse anything else rather than let the kernel fault on an unmapped page)
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, host_src) != hipSuccess || attr.type != hipMemoryTypeHost ||
      attr.devicePointer == nullptr) {
    (void)hipGetLastError();
    set_error("mrec_batch_stage: host_src is not pinned (hipHostMalloc) host memory");
    return MREC_EINVAL;
  }
  host_src = attr.devicePointer;
  const int64_t n16 = bytes / 16;
  const int64_t blocks = std::min<int64_t>((n16 + 1023) / 1024, 1024);
  batch_stage_kernel<<<dim3(static_cast<unsigned>(std::max<int64_t>(blocks, 1))), 256, 0,
                       static_cast<hipStream_t>(stream)>>>(
      static_cast<const uint4 *>(host_src), static_cast<uint4 *>(dst), n16);
  return launch_status("mrec_batch_stage");
}

mrec_status mrec_batch_stage_cursor(void *dst, const void *host_base, int64_t record_bytes,
                                    int64_t n_records, uint64_t *d_state, mrec_stream stream) {
  MREC_CHECK_ARG(record_bytes > 0 && n_records >= 0, "bad record size / count");
  MREC_CHECK_ARG(dst && host_base && d_state, "NULL pointer");
  MREC_CHECK_ARG(record_bytes % 16 == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(host_base) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(d_state) & 7) == 0,
                 "dst / host_base must be 16-B aligned, record_bytes a multiple of 16");
  // the whole epoch buffer must be pinned, device-visible host memory
  hipPointerAttribute_t attr;
  const char *last = static_cast<const char *>(host_base) +
                     (n_records > 0 ? n_records * record_bytes - 1 : 0);
  if (hipPointerGetAttributes(&attr, host_base) != hipSuccess || attr.type != hipMemoryTypeHost ||
      attr.devicePointer == nullptr) {
    (void)hipGetLastError();
    set_error("mrec_batch_stage_cursor: host_base is not pinned (hipHostMalloc) host memory");
    return MREC_EINVAL;
  }
  const char *dev_base = static_cast<const char *>(attr.devicePointer);
  hipPointerAttribute_t attr2;
  if (hipPointerGetAttributes(&attr2, last) != hipSuccess || attr2.type != hipMemoryTypeHost ||
      static_cast<const char *>(attr2.devicePointer) != dev_base + (last - static_cast<const char *>(host_base))) {
    (void)hipGetLastError();
    set_error("mrec_batch_stage_cursor: the epoch buffer is not one pinned allocation");
    return MREC_EINVAL;
  }
  const int64_t n16 = record_bytes / 16;
  const int64_t blocks = std::max<int64_t>(std::min<int64_t>((n16 + 1023) / 1024, 1024), 1);
  batch_stage_cursor_kernel<<<dim3(static_cast<unsigned>(blocks)), 256, 0,
                              static_cast<hipStream_t>(stream)>>>(
      dev_base, record_bytes, n_records, static_cast<uint4 *>(dst),
      reinterpret_cast<unsigned long long *>(d_state));
  return launch_status("mrec_batch_stage_cursor");
}

}  // extern "C"
