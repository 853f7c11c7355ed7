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
#include <cstdlib>

#include "feed_common.h"

namespace mrec {

__global__ __launch_bounds__(256) void batch_stage_kernel(const feed_u32x4 *__restrict__ src,
                                                          feed_u32x4 *__restrict__ dst, int64_t n16,
                                                          int64_t w16) {
  constexpr int U = 4;  // independent 16-B loads per lane per trip
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  for (; i < n16; i += U * stride) {  // (as feed_copy_body_u: U loads on every trip)
    feed_u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = i + u * stride;
      v[u] = src[p < n16 ? p : n16 - 1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = i + u * stride;
      if (p < w16)
        feed_widen(dst, p, v[u]);
      else if (p < n16)
        dst[p + w16] = v[u];
    }
  }
}

__global__ __launch_bounds__(256) void batch_stage_cursor_kernel(FeedCopy fc) {
  __shared__ long long s_rec;
  feed_copy_body<256>(fc, blockIdx.x, &s_rec);
}

mrec_status build_feed_copy(const mrec_feed_job *job, int threads, FeedCopy *out) {
  *out = FeedCopy{};
  MREC_CHECK_ARG(job != nullptr, "NULL feed job");
  const mrec_feed_job &j = *job;
  MREC_CHECK_ARG(j.record_bytes > 0 && j.n_records >= 0, "bad record size / count");
  MREC_CHECK_ARG(j.dst && j.host_base && j.d_state, "NULL pointer");
  MREC_CHECK_ARG(j.record_bytes % 16 == 0 && (reinterpret_cast<uintptr_t>(j.dst) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(j.host_base) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(j.d_state) & 7) == 0,
                 "dst / host_base must be 16-B aligned, record_bytes a multiple of 16");
  // the whole epoch buffer must be ONE pinned, device-visible host allocation
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, j.host_base) != hipSuccess || attr.type != hipMemoryTypeHost ||
      attr.devicePointer == nullptr) {
    (void)hipGetLastError();
    set_error("feed job: host_base is not pinned (hipHostMalloc) host memory");
    return MREC_EINVAL;
  }
  const char *dev_base = static_cast<const char *>(attr.devicePointer);
  if (j.n_records > 0) {
    const char *last = static_cast<const char *>(j.host_base) + j.n_records * j.record_bytes - 1;
    hipPointerAttribute_t attr2;
    if (hipPointerGetAttributes(&attr2, last) != hipSuccess || attr2.type != hipMemoryTypeHost ||
        static_cast<const char *>(attr2.devicePointer) !=
            dev_base + (last - static_cast<const char *>(j.host_base))) {
      (void)hipGetLastError();
      set_error("feed job: the epoch buffer is not one pinned allocation");
      return MREC_EINVAL;
    }
  }
  MREC_CHECK_ARG(j.widen_bytes >= 0 && j.widen_bytes % 16 == 0 && j.widen_bytes <= j.record_bytes,
                 "feed job: widen_bytes must be a multiple of 16 within the record");
  out->w16 = j.widen_bytes / 16;
  out->src = dev_base;
  out->record_bytes = j.record_bytes;
  out->n_records = j.n_records;
  out->dst = static_cast<uint4 *>(j.dst);
  out->state = reinterpret_cast<unsigned long long *>(j.d_state);
  const int64_t n16 = j.record_bytes / 16;
  // 32 loads in flight per lane (MREC_FEED_UNROLL=4|16|32): fewer copying workgroups
  static const int unroll = [] {
    const char *e = std::getenv("MREC_FEED_UNROLL");
    const int u = e ? std::atoi(e) : 32;
    return u == 4 || u == 16 ? u : 32;
  }();
  out->unroll = unroll;
  out->blocks = static_cast<int>(std::max<int64_t>(
      std::min<int64_t>((n16 + unroll * threads - 1) / (unroll * threads), 1024), 1));
  return MREC_OK;
}

}  // namespace mrec

using namespace mrec;

extern "C" {

mrec_status mrec_batch_stage(void *dst, const void *host_src, int64_t bytes, mrec_stream stream) {
  return mrec_batch_stage_ex(dst, host_src, bytes, 0, stream);
}

mrec_status mrec_batch_stage_ex(void *dst, const void *host_src, int64_t bytes, int64_t widen_bytes,
                                mrec_stream stream) {
  MREC_CHECK_ARG(bytes >= 0, "bytes < 0");
  MREC_CHECK_ARG(widen_bytes >= 0 && widen_bytes % 16 == 0 && widen_bytes <= bytes,
                 "widen_bytes must be a multiple of 16 within bytes");
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
      static_cast<const feed_u32x4 *>(host_src), static_cast<feed_u32x4 *>(dst), n16,
      widen_bytes / 16);
  return launch_status("mrec_batch_stage");
}

mrec_status mrec_batch_stage_cursor(void *dst, const void *host_base, int64_t record_bytes,
                                    int64_t n_records, uint64_t *d_state, mrec_stream stream) {
  const mrec_feed_job job{dst, host_base, record_bytes, n_records, d_state, 0};
  return mrec_batch_stage_job(&job, stream);
}

mrec_status mrec_batch_stage_job(const mrec_feed_job *job, mrec_stream stream) {
  FeedCopy fc;
  if (mrec_status st = build_feed_copy(job, 256, &fc); st != MREC_OK) return st;
  batch_stage_cursor_kernel<<<dim3(static_cast<unsigned>(fc.blocks)), 256, 0,
                              static_cast<hipStream_t>(stream)>>>(fc);
  return launch_status("mrec_batch_stage_job");
}

}  // extern "C"
