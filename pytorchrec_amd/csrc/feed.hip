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

}  // extern "C"
