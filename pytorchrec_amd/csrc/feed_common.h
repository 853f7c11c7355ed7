// The batch feed's copy of one pinned host record into its device slot, as a body
// any launch can run in some of its workgroups (feed.hip's own kernels; the tower's
// weight-gradient launch, tower_dw.hip, where the PCIe reads overlap the L2-bound
// MFMA work instead of taking their own ~15 us on the step's critical path).
//
// The record index is a device cursor (state[0]); the workgroups that copy it count
// themselves on a ticket (state[1]) and the last one advances the cursor, so a HIP
// graph holding the launch stages the next record on every replay.
#pragma once
#include "common.h"

namespace mrec {

struct FeedCopy {
  const char *src;            // device address of the pinned epoch buffer
  int64_t record_bytes;
  int64_t n_records;
  uint4 *dst;                 // the device slot
  unsigned long long *state;  // [0] cursor, [1] ticket
  int blocks;                 // workgroups of the launch that copy (0: none)
  int unroll;                 // 16-B loads in flight per lane: 4, 16 or 32 (fewer copying
                              // workgroups, so fewer CUs with host loads in flight)
  int64_t w16;                // the record's first w16 16-B pieces are uint16 -> int32 (ABI 29)
};

typedef unsigned int feed_u32x4 __attribute__((ext_vector_type(4)));

// host piece p < w16 of a record: 8 uint16 values written as 8 zero-extended int32
// (device pieces 2p, 2p + 1); later pieces land w16 pieces further on
__device__ __forceinline__ void feed_widen(feed_u32x4 *dst, int64_t p, feed_u32x4 v) {
  dst[2 * p] = feed_u32x4{v.x & 0xffffu, v.x >> 16, v.y & 0xffffu, v.y >> 16};
  dst[2 * p + 1] = feed_u32x4{v.z & 0xffffu, v.z >> 16, v.w & 0xffffu, v.w >> 16};
}

// run by workgroup `b` of the `fc.blocks` copying ones (THREADS threads each)
template <int THREADS, int U = 4>
__device__ __forceinline__ void feed_copy_body_u(const FeedCopy &fc, int b, long long *s_rec) {
  if (threadIdx.x == 0)
    *s_rec = static_cast<long long>(
        __hip_atomic_load(fc.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  __syncthreads();
  const long long rec = *s_rec;
  if (rec >= 0 && rec < fc.n_records) {
    // the clang vector type, not HIP's uint4 struct: an array of the struct stayed a
    // stack object (ScratchSize 528 B/lane at U = 32, every value through scratch);
    // the vector array is promoted to registers (U loads in flight, no scratch)
    typedef feed_u32x4 u32x4;
    const u32x4 *src = reinterpret_cast<const u32x4 *>(fc.src + rec * fc.record_bytes);
    u32x4 *dst = reinterpret_cast<u32x4 *>(fc.dst);
    const int64_t w16 = fc.w16;
    const int64_t n16 = fc.record_bytes / 16;
    const int64_t stride = static_cast<int64_t>(fc.blocks) * THREADS;
    int64_t i = static_cast<int64_t>(b) * THREADS + threadIdx.x;
    // U loads in flight on every trip, the last one included (clamped addresses,
    // predicated stores): with the workgroup count rounded up, a remainder loop of
    // single loads took most pieces one PCIe round trip at a time
    for (; i < n16; i += U * stride) {
      u32x4 v[U];
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
  __syncthreads();  // every thread of this workgroup has read the cursor
  if (threadIdx.x == 0) {
    const unsigned long long t =
        __hip_atomic_fetch_add(fc.state + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == static_cast<unsigned long long>(fc.blocks) - 1) {  // every workgroup read it
      __hip_atomic_store(fc.state + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(fc.state, static_cast<unsigned long long>(rec + 1), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int THREADS>
__device__ __forceinline__ void feed_copy_body(const FeedCopy &fc, int b, long long *s_rec) {
  if (fc.unroll == 32)  // uniform
    feed_copy_body_u<THREADS, 32>(fc, b, s_rec);
  else if (fc.unroll == 16)
    feed_copy_body_u<THREADS, 16>(fc, b, s_rec);
  else
    feed_copy_body_u<THREADS, 4>(fc, b, s_rec);
}

// host (feed.hip): validate a mrec_feed_job and fill *out (blocks: the copying
// workgroups of THREADS threads)
mrec_status build_feed_copy(const mrec_feed_job *job, int threads, FeedCopy *out);

}  // namespace mrec
