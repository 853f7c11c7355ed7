// Embedding backward: deterministic sorted-segment scatter-add with a fused
// row-sparse update.
//
// plan  : one 1024-thread workgroup per table groups the lookups by row.
//         Batches <= 4096: an LDS hash table and packed atomics (three barriers)
//         give every row a segment, unordered.  Batches <= 8192: a stable LDS
//         radix sort.  Outputs: the lookups grouped by row (perm), the segment
//         starts / lengths and the rows.  Depends only on the ids, so it can
//         overlap the MLP forward on a side stream.
// apply : one LPR-lane worker per unique row sums the per-lookup gradients of
//         its segment in fp32, ascending sample order (bitwise reproducible and
//         independent of the plan's layout), and
//         updates the row once (SGD, or accumulates a dense grad).  Segments
//         longer than SHORT_SEG (hot Zipf rows) are summed by the whole workgroup
//         with a fixed-order LDS tree so one hot row cannot serialise a worker.
#include <algorithm>

#include "common.h"
#include "emb_apply.h"
#include "emb_plan.h"
#include "optim_common.h"
#include "gemm_common.h"

namespace mrec {

#ifndef MREC_APPLY_EXP
#define MREC_APPLY_EXP 0  // microbenchmark variants (tools/bench_apply.py, tools/gpu_apply_exp.sh); 0 = product
#endif

constexpr int kMaxPlanKeys = 8192;

// ---------------------------------------------------------------------------
// plan: stable LSD radix sort of the table's ids in LDS
// ---------------------------------------------------------------------------
// Element i (= sample b, ascending) sits in "round" r = i / 1024, lane t = i % 1024,
// so a wave's 64 lanes hold 64 consecutive elements and the (round, wave) groups
// are in element order.  Each 4-bit pass ranks an element inside its wave with
// 4 ballots (lanes with the same digit), writes per-(digit, group) counts in
// digit-major order, and one block scan of that array gives every element's
// destination: digit base + earlier groups with that digit + rank in wave.
// Stability makes equal ids keep ascending b, so segments come out in the
// reference's accumulation order.  Invalid ids (out of range, padding) get the
// key `rows`, one past every valid id, and therefore sort last.
constexpr int kRadixBits = 4;
constexpr int kDigits = 1 << kRadixBits;
constexpr int kMaxRounds = kMaxPlanKeys / kPlanThreads;  // 8
constexpr int kMaxGroups = kMaxRounds * (kPlanThreads / 64);  // 128

__device__ __forceinline__ uint64_t digit_peers(uint32_t d) {
  uint64_t m = ~0ull;
#pragma unroll
  for (int k = 0; k < kRadixBits; ++k) {
    const uint64_t bk = __ballot((d >> k) & 1u);
    m &= ((d >> k) & 1u) ? bk : ~bk;
  }
  return m;
}

// block-wide exclusive scan of n <= 2*kPlanThreads uint32 values in place
__device__ void block_exclusive_scan(uint32_t *a, int n, uint32_t *wtot, uint32_t *total) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int i0 = 2 * tid;
  const uint32_t v0 = i0 < n ? a[i0] : 0u;
  const uint32_t v1 = i0 + 1 < n ? a[i0 + 1] : 0u;
  uint32_t incl = v0 + v1;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_up(incl, off);
    if (lane >= off) incl += t;
  }
  if (lane == 63) wtot[wid] = incl;
  __syncthreads();
  if (wid == 0) {
    uint32_t w = lane < kPlanThreads / 64 ? wtot[lane] : 0u;
    uint32_t wi = w;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t t = __shfl_up(wi, off);
      if (lane >= off) wi += t;
    }
    if (lane < kPlanThreads / 64) wtot[lane] = wi - w;
    if (lane == kPlanThreads / 64 - 1 && total) *total = wi;
  }
  __syncthreads();
  const uint32_t ex = wtot[wid] + incl - v0 - v1;
  if (i0 < n) a[i0] = ex;
  if (i0 + 1 < n) a[i0 + 1] = ex + v0;
  __syncthreads();
}


// Stable LSD radix sort of N = rounds * 1024 LDS keys (payload = element index),
// then segment detection; writes perm / seg / uniq / hdr[0..1] of table t.
// Keys >= rows are invalid and sort last.  Must be called by all 1024 threads.
__device__ void sort_and_segment(uint32_t *keyA, uint32_t *keyB, uint16_t *payA, uint16_t *payB,
                                 int rounds, uint32_t rows, uint32_t *hist, uint32_t *wtot,
                                 const TableWs &t, uint32_t *s_total, int32_t *s_nvalid) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int N = rounds * kPlanThreads;
  const int G = rounds * (kPlanThreads / 64);
  if (tid == 0) *s_nvalid = 0;
  const int bits = 32 - __clz(rows);  // covers every key value 0..rows
  const int passes = (bits + kRadixBits - 1) / kRadixBits;
  uint32_t *kin = keyA, *kout = keyB;
  uint16_t *pin = payA, *pout = payB;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  __syncthreads();
  for (int p = 0; p < passes; ++p) {
    const int sh = p * kRadixBits;
    for (int i = tid; i < kDigits * G; i += kPlanThreads) hist[i] = 0u;
    __syncthreads();
    for (int r = 0; r < rounds; ++r) {
      const uint32_t d = (kin[r * kPlanThreads + tid] >> sh) & (kDigits - 1);
      const uint64_t m = digit_peers(d);
      if ((m & lt) == 0) hist[d * G + r * (kPlanThreads / 64) + wid] = __popcll(m);
    }
    __syncthreads();
    block_exclusive_scan(hist, kDigits * G, wtot, nullptr);
    for (int r = 0; r < rounds; ++r) {
      const int i = r * kPlanThreads + tid;
      const uint32_t key = kin[i];
      const uint32_t d = (key >> sh) & (kDigits - 1);
      const uint64_t m = digit_peers(d);
      const uint32_t dst = hist[d * G + r * (kPlanThreads / 64) + wid] + __popcll(m & lt);
      kout[dst] = key;
      pout[dst] = pin[i];
    }
    __syncthreads();
    uint32_t *tk = kin; kin = kout; kout = tk;
    uint16_t *tp = pin; pin = pout; pout = tp;
    if (p < 4) PLAN_STAMP(5 + p);
  }
  // segments: head flags over the sorted valid prefix, block scan of per-thread counts
  const int chunk = (N + kPlanThreads - 1) / kPlanThreads;
  const int lo = tid * chunk;
  const int hi = min(lo + chunk, N);
  uint32_t cnt = 0;
  for (int i = lo; i < hi; ++i) {
    const uint32_t k = kin[i];
    if (k < rows && (i == 0 || kin[i - 1] != k)) ++cnt;
  }
  hist[tid] = cnt;
  __syncthreads();
  block_exclusive_scan(hist, kPlanThreads, wtot, s_total);
  PLAN_STAMP(9);
  uint32_t u = hist[tid];
  for (int i = lo; i < hi; ++i) {
    const uint32_t k = kin[i];
    if (k >= rows) break;
    t.perm[i] = pin[i];
    if (i == 0 || kin[i - 1] != k) {
      t.seg[u] = i;
      t.uniq[u] = static_cast<int32_t>(k);
      ++u;
    }
    if (i + 1 == N || kin[i + 1] >= rows) *s_nvalid = i + 1;  // the one last valid element
  }
  __syncthreads();
  if (tid == 0) {
    const int nu = static_cast<int>(*s_total);
    t.hdr[0] = nu;
    t.hdr[1] = *s_nvalid;
    t.seg[nu] = *s_nvalid;
  }
}

__global__ __launch_bounds__(kPlanThreads) void plan_kernel(BankArgs bank, IdsArgs ids, int64_t B,
                                                            int rounds, void *ws,
                                                            int32_t *__restrict__ oob,
                                                            uint64_t *__restrict__ d_step) {
  __shared__ uint32_t keyA[kMaxPlanKeys], keyB[kMaxPlanKeys];
  __shared__ uint16_t payA[kMaxPlanKeys], payB[kMaxPlanKeys];
  __shared__ uint32_t hist[kDigits * kMaxGroups];
  __shared__ uint32_t wtot[kPlanThreads / 64];
  __shared__ uint32_t s_total;
  __shared__ int32_t s_nvalid;
  const int f = blockIdx.x;
  const int tid = threadIdx.x;
  const uint32_t rows = static_cast<uint32_t>(bank.rows[f]);
  const int N = rounds * kPlanThreads;
  for (int i = tid; i < N; i += kPlanThreads) {
    uint32_t key = rows;  // invalid / padding
    if (i < B) {
      const int64_t id = load_id(ids, f, i);
      if (id >= 0 && id < static_cast<int64_t>(rows)) {
        key = static_cast<uint32_t>(id);
      } else if (oob && !(ids.pad_negative && id < 0)) {
        *oob = 1;
      }
    }
    keyA[i] = key;
    payA[i] = static_cast<uint16_t>(i);
  }
  const TableWs t = table_ws(ws, f, B);
  sort_and_segment(keyA, keyB, payA, payB, rounds, rows, hist, wtot, t, &s_total, &s_nvalid);
  if (tid == 0) {
    t.hdr[2] = 0;
    t.hdr[3] = ws_layout_tag(kLayoutSorted, B);
    if (d_step && f == 0) *d_step += 1;
  }
}

// ---------------------------------------------------------------------------
// hash plan kernel (body in emb_plan.h, shared with the GEMM launch that runs it
// beside a backward GEMM: gemm.hip)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kPlanThreads) void plan_hash_kernel(BankArgs bank, IdsArgs ids,
                                                                 int64_t B, void *ws,
                                                                 int32_t *__restrict__ oob,
                                                                 uint64_t *__restrict__ d_step) {
  __shared__ __attribute__((aligned(16))) uint32_t smem[2 * kHashSlots + 2];
  plan_hash_body<kPlanThreads, kHashSlots>(bank, ids, B, ws, oob, d_step, blockIdx.x / kPlanBuckets,
                                           blockIdx.x % kPlanBuckets, smem);
}

// diagnostics (mrec_diag_plan_hash_variant): the plan body at other workgroup sizes /
// slot counts than the production launches use (the 512-thread body)
template <int THREADS, int SLOTS, int MAXB>
__global__ __launch_bounds__(THREADS) void plan_hash_variant_kernel(BankArgs bank, IdsArgs ids,
                                                                    int64_t B, void *ws,
                                                                    int32_t *__restrict__ oob) {
  __shared__ __attribute__((aligned(16))) uint32_t smem[2 * SLOTS + 2];
  plan_hash_body<THREADS, SLOTS, MAXB>(bank, ids, B, ws, oob, nullptr, blockIdx.x / kPlanBuckets,
                                       blockIdx.x % kPlanBuckets, smem);
}

// ---------------------------------------------------------------------------
// apply (helpers in emb_apply.h)
// ---------------------------------------------------------------------------
// deferred split-K reductions ride in trailing workgroups (CoReduce, gemm_common.h)
// hot segments (> short_seg lookups) of a (table, bucket) are spread over kHotPer
// workgroups of their own (segment k by workgroup k % kHotPer), so a bucket's hot
// rows are summed in parallel instead of one after another by its segment block
#ifndef MREC_HOT_PER
#define MREC_HOT_PER 4
#endif
constexpr int kHotPer = MREC_HOT_PER;
// One hot segment (> kShortSeg lookups) summed by the whole workgroup, in a
// fixed order independent of how the plan listed it: the samples go into an LDS
// bitmap of the batch (<= kHashMaxEntries), worker w sums the w-th, (w + WPB)-th
// ... smallest samples (rank -> sample by a binary search over per-word popcount
// prefixes), then a fixed shuffle tree inside each wave and the 4 wave partials
// in order.  ~2.6 KiB of LDS, so the apply launch keeps full occupancy.
template <typename T, int LPR>
struct HotSeg {
  static constexpr int EPL = Vec<T>::EPL;
  static constexpr int WPB = 256 / LPR;
  static constexpr int kHotChunk = 1024;  // ranks expanded per pass (a multiple of WPB)
  uint32_t bits[kHashMaxEntries / 32];
  uint32_t pre[kHashMaxEntries / 32];
  int32_t srt[kHotChunk];
  float red[4][LPR * EPL];
  uint32_t wsum[4];

  // samples: perm[0, sn); v: the row's values for the FM term (nullptr: take v
  // from x0, the sorted layout's rule)
  template <bool ROW_V, int MODE = -1>
  __device__ __forceinline__ void run(const BankArgs &bank, const ApplyArgs &a, int f, int64_t row,
                                      const int32_t *perm, int sn, int64_t B, const float *v,
                                      int worker, int e0, bool v_lane, bool w_lane, bool live) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int D = bank.dim;
    const int nwords = static_cast<int>((B + 31) / 32);  // <= 256: one per thread
    if (tid < nwords) bits[tid] = 0u;
    __syncthreads();
    for (int i = tid; i < sn; i += 256) {
      const int b = perm[i];
      atomicOr(&bits[b >> 5], 1u << (b & 31));
    }
    __syncthreads();
    const uint32_t c = tid < nwords ? __popc(bits[tid]) : 0u;
    uint32_t incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t x = __shfl_up(incl, off);
      if (lane >= off) incl += x;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    if (tid < nwords) {
      uint32_t p = incl - c;
      for (int k2 = 0; k2 < wid; ++k2) p += wsum[k2];
      pre[tid] = p;
    }
    __syncthreads();
    float acc[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) acc[j] = 0.f;
    // ranks -> samples, kHotChunk ranks at a time: thread t expands its bitmap word
    // into srt[rank - c0]; worker w then takes ranks w, w + WPB, ... (ascending, as
    // always), KB of them per round with every gradient load issued first
#ifndef MREC_HOT_KB
#define MREC_HOT_KB 2
#endif
    constexpr int KB = MREC_HOT_KB;
#pragma unroll 1
    for (int c0 = 0; c0 < sn; c0 += kHotChunk) {
      if (tid < nwords) {
        uint32_t wb = bits[tid];
        int r = static_cast<int>(pre[tid]);
        while (wb && r < c0 + kHotChunk) {
          if (r >= c0) srt[r - c0] = tid * 32 + __ffs(wb) - 1;
          wb &= wb - 1;
          ++r;
        }
      }
      __syncthreads();
      const int c1 = min(sn, c0 + kHotChunk);
#if MREC_APPLY_EXP == 17  // (diagnostic: no hot-segment gradient loads)
      if (live && sn < 0) {
#else
      if (live) {
#endif
#pragma unroll 1
        for (int i0 = c0 + worker; i0 < c1; i0 += WPB * KB) {
          int bs[KB];
#pragma unroll
          for (int u = 0; u < KB; ++u) {
            const int i = i0 + u * WPB;
            bs[u] = i < c1 ? srt[i - c0] : -1;
          }
          float g[KB][EPL];
#pragma unroll
          for (int u = 0; u < KB; ++u) {
            const int b = bs[u] < 0 ? bs[0] : bs[u];  // (a repeat of a valid one; not added)
            if constexpr (ROW_V)
              lookup_grad_v<EPL>(a, b, f, D, e0, v_lane, w_lane, v, g[u]);
            else
              lookup_grad<EPL>(a, b, f, D, e0, v_lane, w_lane, g[u]);
          }
#pragma unroll
          for (int u = 0; u < KB; ++u)
            if (bs[u] >= 0)
#pragma unroll
              for (int j = 0; j < EPL; ++j) acc[j] += g[u][j];
        }
      }
      __syncthreads();  // srt is rewritten by the next chunk
    }
#pragma unroll
    for (int off = LPR; off < 64; off <<= 1)
#pragma unroll
      for (int j = 0; j < EPL; ++j) acc[j] += __shfl_xor(acc[j], off);
    if (lane < LPR)
#pragma unroll
      for (int j = 0; j < EPL; ++j) red[wid][e0 + j] = acc[j];
    __syncthreads();
    if (tid < LPR) {  // worker 0, all its lanes (the row update may reduce across them)
#pragma unroll
      for (int j = 0; j < EPL; ++j) acc[j] = ((red[0][e0 + j] + red[1][e0 + j]) + red[2][e0 + j]) + red[3][e0 + j];
      const int64_t grow = bank.row_offset[f] + row;
      uint4 raw = make_uint4(0u, 0u, 0u, 0u);
      if (live) raw = *reinterpret_cast<const uint4 *>(row_ptr_g<T, MODE>(bank, a, grow, e0));
      row_update<T, LPR, MODE>(bank, a, grow, e0, v_lane, w_lane, live, acc, raw);
    }
    __syncthreads();
  }
};

// ---------------------------------------------------------------------------
// apply, hash layout (emb_plan.h).  Grid (1-D):
//   * F * kPlanBuckets segment blocks, first (dispatched first): block (f, r)
//     updates the repeated rows of its bucket, one LPR-lane worker per segment of
//     <= short_seg lookups (the lookups' sample indices are ranked inside the
//     worker by shuffles, their gradients loaded kSegBatch at a time and summed in
//     ascending sample order -- the order of a sequential scatter-add), then the
//     bucket's hot segments with the whole workgroup (HotSeg);
//   * ceil(B * F / WPB) sample-major blocks for the rows hit once: worker q takes
//     lookup (b, f) = (q / F, q % F), so a wave reads one 64-B stretch of lut and
//     consecutive slices of the dx rows (coalesced);
//   * the co-launched split-K reductions.
// The FM term of a lookup's gradient, dfm_b (fm_sum_b - v), takes v from the row
// it updates (the forward gathered the same bits): the gathered rows are not
// re-read from x0.  Row offsets come from the plan's copy in the workspace.
// ---------------------------------------------------------------------------
#ifndef MREC_APPLY_WAVES
#define MREC_APPLY_WAVES 6  // waves per SIMD: every sample-major block of C2 resident at once
#endif
#ifndef MREC_SEG_BATCH
#define MREC_SEG_BATCH 1
#endif
constexpr int kSegBatch = MREC_SEG_BATCH;  // gradient loads in flight per segment step

template <typename T, int LPR, int MODE>
__device__ __forceinline__ void apply_segment(const BankArgs &bank, const ApplyArgs &a,
                                              const BucketWs &t, int f, int64_t toff_f,
                                              const int4 d, int l, int e0, bool v_lane,
                                              bool w_lane, bool live) {
  constexpr int EPL = Vec<T>::EPL;
  constexpr int PER = (kShortSeg + LPR - 1) / LPR;  // samples held per lane
  const int D = bank.dim;
  const int n = d.y;
  const int64_t grow = toff_f + d.x;
  uint4 raw = make_uint4(0u, 0u, 0u, 0u);
  if (live) raw = *reinterpret_cast<const uint4 *>(row_ptr_g<T, MODE>(bank, a, grow, e0));
  float v[EPL];
#pragma unroll
  for (int j = 0; j < EPL; ++j) v[j] = 0.f;
  if (a.dfm && v_lane) {
    uint4 vr = MODE == MREC_BWD_DENSE_GRAD
                   ? *reinterpret_cast<const uint4 *>(reinterpret_cast<const T *>(bank.data) +
                                                      grow * static_cast<int64_t>(bank.row_stride) + e0)
                   : raw;
    if (MODE < 0 && bank.adam.kind)  // the row as the forward read it: as of step t - 1
      vr = adam_current<T>(bank, grow, e0, EPL, vr, *bank.adam.d_t - 1);
    Vec<T>::to_f32(vr, v);
  }
  float acc[EPL];
#pragma unroll
  for (int j = 0; j < EPL; ++j) acc[j] = 0.f;
  if (n == 2) {  // both lookups in the descriptor: ascending b, loads in flight together
    if (live) {
      float g0[EPL], g1[EPL];
      lookup_grad_v<EPL>(a, min(d.z, d.w), f, D, e0, v_lane, w_lane, v, g0);
      lookup_grad_v<EPL>(a, max(d.z, d.w), f, D, e0, v_lane, w_lane, v, g1);
#pragma unroll
      for (int j = 0; j < EPL; ++j) acc[j] = (acc[j] + g0[j]) + g1[j];
    }
  } else {
    // the worker's lanes hold the n (<= short_seg) samples, PER each; step k takes
    // the k-th smallest (the samples of a segment are distinct) by an in-worker min
    int p[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) p[i] = l + i * LPR < n ? t.perm[d.z + l + i * LPR] : INT_MAX;
    int last = -1;
#if MREC_APPLY_EXP == 16  // (diagnostic: no segment gradient loop)
    if (n < 0)
#endif
#pragma unroll 1
    for (int k0 = 0; k0 < n; k0 += kSegBatch) {
      int sb[kSegBatch];
#pragma unroll
      for (int k = 0; k < kSegBatch; ++k) {
        int m = INT_MAX;
#pragma unroll
        for (int i = 0; i < PER; ++i) m = (p[i] > last && p[i] < m) ? p[i] : m;
#pragma unroll
        for (int off = 1; off < LPR; off <<= 1) m = min(m, __shfl_xor(m, off));
        sb[k] = m;
        if (m != INT_MAX) last = m;
      }
      float g[kSegBatch][EPL];
#pragma unroll
      for (int k = 0; k < kSegBatch; ++k) {
#pragma unroll
        for (int j = 0; j < EPL; ++j) g[k][j] = 0.f;
        if (live && sb[k] != INT_MAX) lookup_grad_v<EPL>(a, sb[k], f, D, e0, v_lane, w_lane, v, g[k]);
      }
#pragma unroll
      for (int k = 0; k < kSegBatch; ++k)
        if (sb[k] != INT_MAX)
#pragma unroll
          for (int j = 0; j < EPL; ++j) acc[j] += g[k][j];
    }
  }
  row_update<T, LPR, MODE>(bank, a, grow, e0, v_lane, w_lane, live, acc, raw);
}

template <typename T, int LPR, int MODE, bool KC>
__global__ __launch_bounds__(256, MREC_APPLY_WAVES) void apply_hash_kernel(BankArgs bank, int64_t B,
                                                                           const void *ws, ApplyArgs a,
                                                                           int seg_blocks, int sm_blocks,
                                                                           CoReduce co, KClock kc) {
#ifdef MREC_KC_CAT  // (diagnostic: clock shards per block kind: co-reduce, segments, hot, singles)
  const int cb_ = co.start[co.n], bb_ = static_cast<int>(blockIdx.x) - cb_;
  KcScope<KC> kc_scope(kc, bb_ < 0 ? 0 : bb_ < seg_blocks ? 1 : bb_ < seg_blocks * (1 + kHotPer) ? 2 : 3);
#else
  KcScope<KC> kc_scope(kc);
#endif
  // the co-launched reductions take the leading workgroups: independent of the
  // embedding update, they start first instead of trailing it
#if MREC_APPLY_EXP == 13  // (diagnostic: reductions trailing the apply blocks)
  const int co_blocks = 0;
  if (static_cast<int>(blockIdx.x) >= seg_blocks * (1 + kHotPer) + sm_blocks) {
    co_reduce(co, blockIdx.x - seg_blocks * (1 + kHotPer) - sm_blocks);
    return;
  }
#else
  const int co_blocks0 = co.start[co.n];
  if (static_cast<int>(blockIdx.x) < co_blocks0) {  // uniform
#if MREC_APPLY_EXP != 12
    co_reduce(co, blockIdx.x);
#endif
    return;
  }
  // the data-parallel dense SGD tiles (independent of the embedding update)
  if (static_cast<int>(blockIdx.x) < co_blocks0 + a.sgd_blocks) {  // uniform
    sgd_tile(*a.sgd, static_cast<int>(blockIdx.x) - co_blocks0);
    return;
  }
  const int co_blocks = co_blocks0 + a.sgd_blocks;
#endif
  if (a.d_step) a.seed += *a.d_step * 0x9e3779b97f4a7c15ull;
  constexpr int EPL = Vec<T>::EPL;
  constexpr int WPB = 256 / LPR;
  const int worker = threadIdx.x / LPR;
  const int l = threadIdx.x % LPR;
  const int e0 = l * EPL;
  const int D = bank.dim;
  const int F = bank.n_tables;
  const bool v_lane = e0 + EPL <= D;
  const bool w_lane = bank.has_w && e0 == D;
  const bool live = v_lane || w_lane;
  const int blk = blockIdx.x - co_blocks;
  const int64_t *__restrict__ toff = table_offsets(ws, F, B);

  if (blk < seg_blocks) {  // uniform: the repeated rows of one (table, bucket)
#if MREC_APPLY_EXP == 8 || MREC_APPLY_EXP == 14
    return;
#endif
    const int f = blk / kPlanBuckets, r = blk - f * kPlanBuckets;
    const BucketWs t = bucket_ws(ws, f, r, B);
    // the first pass's descriptor is loaded beside the header (unconditionally, from
    // a clamped slot; used only when the header says it is a segment): one memory
    // round trip less on the block's chain (header -> descriptor -> gradients -> row)
    const int64_t scap = seg_cap(B);
    const int4 dpre = t.desc[worker < scap ? worker : 0];
    const int nseg = t.hdr[0];
    asm volatile("" ::"v"(dpre.x), "v"(dpre.y), "v"(dpre.z), "v"(dpre.w));  // (not sunk below)
    const int64_t toff_f = bank.row_offset[f];
    const int sshort = short_seg(LPR);
    for (int s0 = 0; s0 < nseg; s0 += WPB) {  // uniform
      const int s = s0 + worker;
      if (s < nseg) {
        const int4 d = s0 == 0 ? dpre : t.desc[s];
        if (d.y <= sshort)
          apply_segment<T, LPR, MODE>(bank, a, t, f, toff_f, d, l, e0, v_lane, w_lane, live);
      }
    }
    return;
  }
  if (blk < seg_blocks * (1 + kHotPer)) {  // uniform: hot segments k = h, h + kHotPer, ...
#if MREC_APPLY_EXP == 10 || MREC_APPLY_EXP == 14
    return;
#endif
    const int q = blk - seg_blocks;
    const int fr = q / kHotPer, h = q - fr * kHotPer;
    const int f = fr / kPlanBuckets, r = fr - f * kPlanBuckets;
    const BucketWs t = bucket_ws(ws, f, r, B);
    const int nl = t.hdr[2];
    if (h >= nl) return;  // uniform
    const int64_t toff_f = bank.row_offset[f];
    __shared__ HotSeg<T, LPR> hot;
    for (int k = h; k < nl; k += kHotPer) {
      const int4 d = t.desc[t.longl[k]];
      float v[EPL];
#pragma unroll
      for (int j = 0; j < EPL; ++j) v[j] = 0.f;
      if (a.dfm && v_lane) {
        uint4 vr = *reinterpret_cast<const uint4 *>(
            reinterpret_cast<const T *>(bank.data) +
            (toff_f + d.x) * static_cast<int64_t>(bank.row_stride) + e0);
        if (MODE < 0 && bank.adam.kind)  // the row as the forward read it
          vr = adam_current<T>(bank, toff_f + d.x, e0, EPL, vr, *bank.adam.d_t - 1);
        Vec<T>::to_f32(vr, v);
      }
      hot.template run<true, MODE>(bank, a, f, d.x, t.perm + d.z, d.y, B, v, worker, e0, v_lane,
                                   w_lane, live);
    }
    return;
  }

  // a row hit once: one lookup, one update
#if MREC_APPLY_EXP == 15
  return;
#endif
  const int64_t q = static_cast<int64_t>(blk - seg_blocks * (1 + kHotPer)) * WPB + worker;
  if (q >= B * F) return;  // whole workers
  const bool rowwise = MODE < 0 && a.mode == MREC_BWD_ROWWISE_ADAGRAD;
  if (!live && !rowwise) return;
  const int64_t b = q / F;
  const int f = static_cast<int>(q - b * F);
  const int code = lookup_table(ws, F, B)[q];
  // this lookup's gradient inputs depend on (b, f) only: issued beside the lut load,
  // not behind the branch on its verdict (one memory round trip less per row)
  float gdx[EPL], fs[EPL];
  float dfm_c = 0.f;
#pragma unroll
  for (int j = 0; j < EPL; ++j) gdx[j] = fs[j] = 0.f;
  const bool pre = live && !a.g_occ && !a.g_rec;
  if (pre) {
    if (v_lane) {
      const int64_t col = static_cast<int64_t>(f) * D + e0;
      if (a.dx) {
        if (a.dx_bf16)
          load_bf16xN<EPL>(static_cast<const uint16_t *>(a.dx) + b * a.dx_ld + col, gdx);
        else
          load_f32xN<EPL>(static_cast<const float *>(a.dx) + b * a.dx_ld + col, gdx);
      }
      if (a.dfm) {
        dfm_c = a.dfm[b];
        load_f32xN<EPL>(a.fm_sum + b * D + e0, fs);
      }
    } else if (w_lane && a.dw) {
      gdx[0] = a.dw[b];
    }
  }
  if (code < 0) return;  // whole workers
  const int64_t grow = toff[f] + code;
  uint4 raw = make_uint4(0u, 0u, 0u, 0u);
  if (live) raw = *reinterpret_cast<const uint4 *>(row_ptr_g<T, MODE>(bank, a, grow, e0));
  float v[EPL];
  if (a.dfm && v_lane) {
    uint4 vr = MODE == MREC_BWD_DENSE_GRAD
                   ? *reinterpret_cast<const uint4 *>(reinterpret_cast<const T *>(bank.data) +
                                                      grow * static_cast<int64_t>(bank.row_stride) + e0)
                   : raw;
    if (MODE < 0 && bank.adam.kind)  // the row as the forward read it: as of step t - 1
      vr = adam_current<T>(bank, grow, e0, EPL, vr, *bank.adam.d_t - 1);
    Vec<T>::to_f32(vr, v);
  }
  float acc[EPL];
#pragma unroll
  for (int j = 0; j < EPL; ++j) acc[j] = 0.f;
  if (pre) {  // = add_lookup_grad_v on the pre-loaded inputs (same operations)
    if (v_lane && a.dfm) {
#pragma unroll
      for (int j = 0; j < EPL; ++j) gdx[j] = fmaf(dfm_c, fs[j] - v[j], gdx[j]);
    }
#pragma unroll
    for (int j = 0; j < EPL; ++j) acc[j] += gdx[j];
  } else if (live) {
    add_lookup_grad_v<EPL>(a, b, f, D, e0, v_lane, w_lane, v, acc);
  }
#if MREC_APPLY_EXP == 9
  if (acc[0] == 12345.f) *(float *)a.grad = acc[1];
  return;
#endif
  row_update<T, LPR, MODE>(bank, a, grow, e0, v_lane, w_lane, live, acc, raw);
}

// ---------------------------------------------------------------------------
// apply, sorted layout (batches up to MREC_BWD_MAX_BATCH): one LPR-lane worker
// per segment (= unique row) sums its lookups in ascending sample order;
// segments longer than kShortSeg are summed by the whole workgroup.  Grid:
// F * seg_blocks segment blocks (table f = blk / seg_blocks), then the
// co-launched reductions.
// ---------------------------------------------------------------------------
template <typename T, int LPR>
__global__ __launch_bounds__(256, 6) void apply_kernel(BankArgs bank, int64_t B, const void *ws,
                                                       ApplyArgs a, int seg_blocks,
                                                       int apply_blocks, CoReduce co) {
  if (static_cast<int>(blockIdx.x) >= apply_blocks) {  // uniform: a co-launched reduction
    co_reduce(co, blockIdx.x - apply_blocks);
    return;
  }
  if (a.d_step) a.seed += *a.d_step * 0x9e3779b97f4a7c15ull;
  constexpr int EPL = Vec<T>::EPL;
  constexpr int WPB = 256 / LPR;
  __shared__ int32_t long_list[WPB];
  __shared__ int32_t n_long;
  __shared__ HotSeg<T, LPR> hot;
  const int worker = threadIdx.x / LPR;
  const int l = threadIdx.x % LPR;
  const int e0 = l * EPL;
  const int D = bank.dim;
  const bool v_lane = e0 + EPL <= D;
  const bool w_lane = bank.has_w && e0 == D;
  const bool live = v_lane || w_lane;
  const int blk = blockIdx.x;
  const int f = blk / seg_blocks;
  const TableWs t = table_ws(ws, f, B);
  const int ublk = (blk - f * seg_blocks) * WPB;
  const int u = ublk + worker;
  // the segment is loaded together with the header (one latency)
  int row = 0, s0 = 0, n = 0;
  if (u < B) {
    row = t.uniq[u];
    s0 = t.seg[u];
    n = t.seg[u + 1] - s0;
  }
  const int nu = t.hdr[0];
  if (ublk >= nu) return;  // uniform per block
  if (threadIdx.x == 0) n_long = 0;
  __syncthreads();

  bool mine = u < nu;
  if (mine && n > kShortSeg) {
    if (l == 0) long_list[atomicAdd(&n_long, 1)] = u;
    mine = false;
  }
  if (mine) {  // all the worker's lanes (the row update may reduce across them)
    // the row's old contents are fetched first, in parallel with the gradients
    uint4 raw = make_uint4(0u, 0u, 0u, 0u);
    if (live) raw = *reinterpret_cast<const uint4 *>(row_ptr<T>(bank, a, f, row, e0));
    float acc[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) acc[j] = 0.f;
    if (live)
      for (int j = 0; j < n; ++j) add_lookup_grad<EPL>(a, t.perm[s0 + j], f, D, e0, v_lane, w_lane, acc);
    row_update<T, LPR, -1>(bank, a, bank.row_offset[f] + row, e0, v_lane, w_lane, live, acc, raw);
  }
  __syncthreads();
  const int nl = n_long;
  for (int k = 0; k < nl; ++k) {
    // each hot segment is summed independently, so the (atomic) list order does
    // not change any result; the sorted layout's perm is already ascending, the
    // bitmap pass keeps it so
    const int uu = long_list[k];
    const int lrow = t.uniq[uu];
    const int ls0 = t.seg[uu];
    const int sn = t.seg[uu + 1] - ls0;
    hot.template run<false>(bank, a, f, lrow, t.perm + ls0, sn, B, nullptr, worker, e0, v_lane,
                            w_lane, live);
  }
}

// MREC_BWD_ADAM: every row behind the current step t runs its missed zero-gradient
// steps (opt_row_update with g = 0 brings it to t); one LPR-lane worker per row
template <typename T, int LPR>
__global__ __launch_bounds__(256) void optim_flush_kernel(BankArgs bank, int64_t total_rows,
                                                          ApplyArgs a) {
  constexpr int EPL = Vec<T>::EPL;
  constexpr int WPB = 256 / LPR;
  const int worker = threadIdx.x / LPR, l = threadIdx.x % LPR, e0 = l * EPL;
  const int D = bank.dim;
  const bool v_lane = e0 + EPL <= D, w_lane = bank.has_w && e0 == D;
  const bool live = v_lane || w_lane;
  const int64_t t = *a.opt.d_t;
  float acc[EPL];
#pragma unroll
  for (int j = 0; j < EPL; ++j) acc[j] = 0.f;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * WPB + worker; r < total_rows;
       r += static_cast<int64_t>(gridDim.x) * WPB) {
    if (a.opt.row_step[r] >= t) continue;  // whole workers
    uint4 raw = make_uint4(0u, 0u, 0u, 0u);
    if (live) raw = *reinterpret_cast<const uint4 *>(row_ptr_g<T>(bank, a, r, e0));
    opt_row_update<T, LPR>(bank, a, r, e0, v_lane, w_lane, live, acc, raw);
  }
}

mrec_status build_plan_job(const mrec_plan_job *plan, PlanJob *out) {
  int eb, lpr;
  mrec_status st = make_bank_args(plan->bank, &out->bank, &eb, &lpr);
  if (st != MREC_OK) return st;
  if ((st = make_ids_args(plan->ids, out->bank.n_tables, &out->ids)) != MREC_OK) return st;
  MREC_CHECK_ARG(plan->batch >= 1 && hash_layout(plan->batch, out->ids.pad_negative != 0),
                 "plan batch must be in [1, MREC_BWD_HASH_MAX_BATCH] (padded exchange views: "
                 "[1, MREC_BWD_MAX_BATCH])");
  MREC_CHECK_ARG(plan->workspace != nullptr, "plan workspace is NULL");
  if (plan->ws_bytes < static_cast<size_t>(hash_ws_bytes(out->bank.n_tables, plan->batch))) {
    set_error("plan workspace too small");
    return MREC_ENOSPC;
  }
  for (int f = 0; f < out->bank.n_tables; ++f)
    MREC_CHECK_ARG(out->bank.rows[f] < (int64_t(1) << 31), "rows per table must be < 2^31");
  ws_layout_record(plan->workspace, kLayoutHash, plan->batch, out->bank.n_tables,
                   out->ids.pad_negative != 0);
  out->B = plan->batch;
  out->ws = plan->workspace;
  out->oob = plan->d_oob_flag;
  out->d_step = plan->d_step;
  return MREC_OK;
}

}  // namespace mrec

using namespace mrec;

extern "C" {

#ifdef MREC_PLAN_PROF
void mrec_plan_prof_read(uint64_t *out16) { hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_plan_prof), 128); }
#endif

int64_t mrec_emb_optim_state_ld(int32_t dim, int32_t has_w) {
  return (static_cast<int64_t>(dim) + (has_w ? 1 : 0) + 3) / 4 * 4;
}

mrec_status mrec_emb_optim_flush(const mrec_table_bank *bank, mrec_bwd_mode mode, float lr,
                                 mrec_stream stream) {
  BankArgs ba;
  int eb, lpr;
  mrec_status st = make_bank_args(bank, &ba, &eb, &lpr);
  if (st != MREC_OK) return st;
  if (mode != MREC_BWD_ADAM) return MREC_OK;
  ApplyArgs a{};
  a.mode = mode;
  a.lr = lr;
  if ((st = make_opt_args(bank, mode, &a.opt)) != MREC_OK) return st;
  int64_t total = 0;
  for (int f = 0; f < ba.n_tables; ++f) total = std::max(total, ba.row_offset[f] + ba.rows[f]);
  if (total == 0) return MREC_OK;
  const int wpb = 256 / lpr;
  const int64_t want = (total + wpb - 1) / wpb;
  const dim3 grid(static_cast<unsigned>(std::min<int64_t>(want, 8192)));
  hipStream_t s = static_cast<hipStream_t>(stream);
#define MREC_FK(T, L) optim_flush_kernel<T, L><<<grid, 256, 0, s>>>(ba, total, a)
  if (bank->dtype == MREC_BF16) {
    switch (lpr) {
      case 1: MREC_FK(uint16_t, 1); break;
      case 2: MREC_FK(uint16_t, 2); break;
      case 4: MREC_FK(uint16_t, 4); break;
      case 8: MREC_FK(uint16_t, 8); break;
      default: MREC_FK(uint16_t, 16); break;
    }
  } else {
    switch (lpr) {
      case 1: MREC_FK(float, 1); break;
      case 2: MREC_FK(float, 2); break;
      case 4: MREC_FK(float, 4); break;
      case 8: MREC_FK(float, 8); break;
      default: MREC_FK(float, 16); break;
    }
  }
#undef MREC_FK
  return launch_status("mrec_emb_optim_flush");
}

size_t mrec_emb_bwd_workspace_size(int32_t n_tables, int64_t batch) {
  if (n_tables <= 0 || batch < 0) return 0;
  // the larger of the two layouts (which one a call takes depends on whether its
  // ids are a padded exchange view, not known here)
  const int64_t sorted = int64_t(n_tables) * table_ws_bytes(batch);
  const int64_t hashed = hash_ws_bytes(n_tables, batch);
  return static_cast<size_t>(sorted > hashed ? sorted : hashed);
}

mrec_status mrec_emb_bwd_plan(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                              void *workspace, size_t ws_bytes, int32_t *d_oob_flag,
                              uint64_t *d_step, mrec_stream stream) {
  BankArgs ba;
  IdsArgs ia;
  int eb, lpr;
  mrec_status st = make_bank_args(bank, &ba, &eb, &lpr);
  if (st != MREC_OK) return st;
  if ((st = make_ids_args(ids, ba.n_tables, &ia)) != MREC_OK) return st;
  MREC_CHECK_ARG(batch >= 0 && batch <= kMaxPlanKeys, "batch must be in [0, MREC_BWD_MAX_BATCH]");
  MREC_CHECK_ARG(workspace != nullptr, "workspace is NULL");
  if (ws_bytes < mrec_emb_bwd_workspace_size(ba.n_tables, batch)) {
    set_error("mrec_emb_bwd_plan: workspace too small");
    return MREC_ENOSPC;
  }
  for (int f = 0; f < ba.n_tables; ++f)
    MREC_CHECK_ARG(ba.rows[f] < (int64_t(1) << 31), "rows per table must be < 2^31");
  const int rounds = static_cast<int>((batch + kPlanThreads - 1) / kPlanThreads);
  const bool hash = batch >= 1 && hash_layout(batch, ia.pad_negative != 0);
  ws_layout_record(workspace, hash ? kLayoutHash : kLayoutSorted, batch, ba.n_tables,
                   ia.pad_negative != 0);
  if (hash) {
    plan_hash_kernel<<<dim3(ba.n_tables * kPlanBuckets), kPlanThreads, 0,
                       static_cast<hipStream_t>(stream)>>>(
        ba, ia, batch, workspace, d_oob_flag, d_step);
    return launch_status("mrec_emb_bwd_plan");
  }
  plan_kernel<<<dim3(ba.n_tables), kPlanThreads, 0, static_cast<hipStream_t>(stream)>>>(
      ba, ia, batch, rounds < 1 ? 1 : rounds, workspace, d_oob_flag, d_step);
  return launch_status("mrec_emb_bwd_plan");
}

// diagnostics (not in mrec.h): the hash plan of mrec_emb_bwd_plan run by the plan body
// instantiated for `threads` threads and `slots` LDS slots (variants: 1024 / 8192 --
// the production instantiation --, 512 / 8192, 256 / 8192, 512 / 4096 for batches <=
// 4096).  The workspace it leaves drives mrec_emb_bwd_apply like the standalone plan's.
mrec_status mrec_diag_plan_hash_variant(const mrec_table_bank *bank, const mrec_ids *ids,
                                        int64_t batch, void *workspace, size_t ws_bytes,
                                        int32_t threads, int32_t slots, int32_t *d_oob_flag,
                                        mrec_stream stream) {
  BankArgs ba;
  IdsArgs ia;
  int eb, lpr;
  mrec_status st = make_bank_args(bank, &ba, &eb, &lpr);
  if (st != MREC_OK) return st;
  if ((st = make_ids_args(ids, ba.n_tables, &ia)) != MREC_OK) return st;
  MREC_CHECK_ARG(batch >= 1 && hash_layout(batch, ia.pad_negative != 0),
                 "the batch must take the hash layout");
  MREC_CHECK_ARG(workspace && ws_bytes >= static_cast<size_t>(mrec_emb_bwd_workspace_size(ba.n_tables, batch)),
                 "workspace too small");
  const dim3 grid(ba.n_tables * kPlanBuckets);
  hipStream_t s = static_cast<hipStream_t>(stream);
  ws_layout_record(workspace, kLayoutHash, batch, ba.n_tables, ia.pad_negative != 0);
  if (threads == 1024 && slots == 8192)
    plan_hash_variant_kernel<1024, 8192, kHashMaxEntries><<<grid, 1024, 0, s>>>(ba, ia, batch, workspace, d_oob_flag);
  else if (threads == 512 && slots == 8192)
    plan_hash_variant_kernel<512, 8192, kHashMaxEntries><<<grid, 512, 0, s>>>(ba, ia, batch, workspace, d_oob_flag);
  else if (threads == 256 && slots == 8192)
    plan_hash_variant_kernel<256, 8192, kHashMaxEntries><<<grid, 256, 0, s>>>(ba, ia, batch, workspace, d_oob_flag);
  else if (threads == 512 && slots == 4096 && batch <= 4096)
    plan_hash_variant_kernel<512, 4096, 4096><<<grid, 512, 0, s>>>(ba, ia, batch, workspace, d_oob_flag);
  else
    MREC_CHECK_ARG(false, "no such plan variant");
  return launch_status("mrec_diag_plan_hash_variant");
}

}  // extern "C"

struct GivenWire {  // mrec_emb_bwd_apply_wire: given gradients as wire records
  const void *wire;
  int bf16;
  int pitch;  // elements per record
  const int32_t *pref;
  int64_t cap_rows;
};
struct RecOut {  // mrec_emb_bwd_apply_rec: DENSE_GRAD sums into wire records
  void *wire;
  int rec_dw;
  const int32_t *pref;
  int cap;
  int64_t cap_rows;
};

static mrec_status apply_impl(const mrec_table_bank *bank, int64_t batch, const void *workspace,
                              size_t ws_bytes, const void *dx, mrec_dtype dx_dtype, int64_t dx_ld,
                              const float *dfm, const float *fm_sum, const void *x0,
                              mrec_dtype x0_dtype, int64_t x0_ld, const float *dw,
                              const float *g_occ, int64_t g_ld, int64_t chunk,
                              int64_t chunk_stride, mrec_bwd_mode mode, float lr, uint64_t seed,
                              const uint64_t *d_step, void *grad, int32_t n_reduce,
                              const mrec_gemm_call *reduce, mrec_stream stream,
                              const GivenWire *gw = nullptr, const RecOut *ro = nullptr,
                              const void *sgd_table = nullptr, int32_t sgd_blocks = 0);

extern "C" {

mrec_status mrec_emb_bwd_apply(const mrec_table_bank *bank, int64_t batch, const void *workspace,
                               size_t ws_bytes, const void *dx, mrec_dtype dx_dtype, int64_t dx_ld,
                               const float *dfm, const float *fm_sum, const void *x0,
                               mrec_dtype x0_dtype, int64_t x0_ld, const float *dw,
                               mrec_bwd_mode mode, float lr, uint64_t seed,
                               const uint64_t *d_step, void *grad, mrec_stream stream) {
  return apply_impl(bank, batch, workspace, ws_bytes, dx, dx_dtype, dx_ld, dfm, fm_sum, x0,
                    x0_dtype, x0_ld, dw, nullptr, 0, 0, 0, mode, lr, seed, d_step, grad, 0,
                    nullptr, stream);
}

mrec_status mrec_emb_bwd_apply_ex(const mrec_table_bank *bank, int64_t batch,
                                  const void *workspace, size_t ws_bytes, const void *dx,
                                  mrec_dtype dx_dtype, int64_t dx_ld, const float *dfm,
                                  const float *fm_sum, const void *x0, mrec_dtype x0_dtype,
                                  int64_t x0_ld, const float *dw, mrec_bwd_mode mode, float lr,
                                  uint64_t seed, const uint64_t *d_step, void *grad,
                                  int32_t n_reduce, const mrec_gemm_call *reduce,
                                  mrec_stream stream) {
  return apply_impl(bank, batch, workspace, ws_bytes, dx, dx_dtype, dx_ld, dfm, fm_sum, x0,
                    x0_dtype, x0_ld, dw, nullptr, 0, 0, 0, mode, lr, seed, d_step, grad, n_reduce,
                    reduce, stream);
}

mrec_status mrec_emb_bwd_apply_given(const mrec_table_bank *bank, int64_t batch,
                                     const void *workspace, size_t ws_bytes, const void *dx,
                                     mrec_dtype dx_dtype, int64_t dx_ld, const float *dfm,
                                     const float *fm_sum, const void *x0, mrec_dtype x0_dtype,
                                     int64_t x0_ld, const float *dw, const float *g_occ,
                                     int64_t g_ld, int64_t chunk, int64_t chunk_stride,
                                     mrec_bwd_mode mode, float lr, uint64_t seed,
                                     const uint64_t *d_step, void *grad, int32_t n_reduce,
                                     const mrec_gemm_call *reduce, mrec_stream stream) {
  return apply_impl(bank, batch, workspace, ws_bytes, dx, dx_dtype, dx_ld, dfm, fm_sum, x0,
                    x0_dtype, x0_ld, dw, g_occ, g_ld, chunk, chunk_stride, mode, lr, seed, d_step,
                    grad, n_reduce, reduce, stream);
}

mrec_status mrec_emb_bwd_apply_rec(const mrec_table_bank *bank, int64_t batch,
                                   const void *workspace, size_t ws_bytes, const void *dx,
                                   mrec_dtype dx_dtype, int64_t dx_ld, const float *dfm,
                                   const float *fm_sum, const void *x0, mrec_dtype x0_dtype,
                                   int64_t x0_ld, const float *dw, const mrec_grad_records *out,
                                   int32_t n_reduce, const mrec_gemm_call *reduce,
                                   mrec_stream stream) {
  MREC_CHECK_ARG(out != nullptr, "out is NULL");
  MREC_CHECK_ARG(out->rec_bytes > 0 && out->rec_bytes % 4 == 0, "bad record bytes");
  const RecOut ro{out->wire, out->rec_bytes / 4, out->pref, out->cap, out->cap_rows};
  return apply_impl(bank, batch, workspace, ws_bytes, dx, dx_dtype, dx_ld, dfm, fm_sum, x0,
                    x0_dtype, x0_ld, dw, nullptr, 0, 0, 0, MREC_BWD_DENSE_GRAD, 0.f, 0, nullptr,
                    nullptr, n_reduce, reduce, stream, nullptr, &ro);
}

mrec_status mrec_emb_bwd_apply_wire(const mrec_table_bank *bank, int64_t batch,
                                    const void *workspace, size_t ws_bytes, const void *wire,
                                    int32_t rec_bytes, mrec_dtype wire_dtype, const int32_t *pref,
                                    int32_t cap_rows, int64_t chunk, int64_t chunk_stride,
                                    mrec_bwd_mode mode, float lr, uint64_t seed,
                                    const uint64_t *d_step, void *grad, int32_t n_reduce,
                                    const mrec_gemm_call *reduce, mrec_stream stream) {
  MREC_CHECK_ARG(wire_dtype == MREC_BF16 || wire_dtype == MREC_F32, "wire dtype must be BF16/F32");
  const int es = wire_dtype == MREC_BF16 ? 2 : 4;
  MREC_CHECK_ARG(rec_bytes > 0 && rec_bytes % es == 0 && rec_bytes % 4 == 0, "bad record bytes");
  const GivenWire gw{wire, wire_dtype == MREC_BF16 ? 1 : 0, rec_bytes / es, pref, cap_rows};
  return apply_impl(bank, batch, workspace, ws_bytes, nullptr, MREC_F32, 0, nullptr, nullptr,
                    nullptr, MREC_F32, 0, nullptr, nullptr, 0, chunk, chunk_stride, mode, lr, seed,
                    d_step, grad, n_reduce, reduce, stream, &gw);
}

mrec_status mrec_emb_bwd_apply_wire_sgd(const mrec_table_bank *bank, int64_t batch,
                                        const void *workspace, size_t ws_bytes, const void *wire,
                                        int32_t rec_bytes, mrec_dtype wire_dtype,
                                        const int32_t *pref, int32_t cap_rows, int64_t chunk,
                                        int64_t chunk_stride, mrec_bwd_mode mode, float lr,
                                        uint64_t seed, const uint64_t *d_step, void *grad,
                                        int32_t n_reduce, const mrec_gemm_call *reduce,
                                        const void *sgd_table, int32_t sgd_blocks,
                                        mrec_stream stream) {
  MREC_CHECK_ARG(wire_dtype == MREC_BF16 || wire_dtype == MREC_F32, "wire dtype must be BF16/F32");
  const int es = wire_dtype == MREC_BF16 ? 2 : 4;
  MREC_CHECK_ARG(rec_bytes > 0 && rec_bytes % es == 0 && rec_bytes % 4 == 0, "bad record bytes");
  MREC_CHECK_ARG(sgd_table == nullptr || (reinterpret_cast<uintptr_t>(sgd_table) & 15) == 0,
                 "sgd table not 16-B aligned");
  const GivenWire gw{wire, wire_dtype == MREC_BF16 ? 1 : 0, rec_bytes / es, pref, cap_rows};
  return apply_impl(bank, batch, workspace, ws_bytes, nullptr, MREC_F32, 0, nullptr, nullptr,
                    nullptr, MREC_F32, 0, nullptr, nullptr, 0, chunk, chunk_stride, mode, lr, seed,
                    d_step, grad, n_reduce, reduce, stream, &gw, nullptr, sgd_table, sgd_blocks);
}

}  // extern "C"

static mrec_status apply_impl(const mrec_table_bank *bank, int64_t batch, const void *workspace,
                              size_t ws_bytes, const void *dx, mrec_dtype dx_dtype, int64_t dx_ld,
                              const float *dfm, const float *fm_sum, const void *x0,
                              mrec_dtype x0_dtype, int64_t x0_ld, const float *dw,
                              const float *g_occ, int64_t g_ld, int64_t chunk,
                              int64_t chunk_stride, mrec_bwd_mode mode, float lr, uint64_t seed,
                              const uint64_t *d_step, void *grad, int32_t n_reduce,
                              const mrec_gemm_call *reduce, mrec_stream stream,
                              const GivenWire *gw, const RecOut *ro, const void *sgd_table,
                              int32_t sgd_blocks) {
  BankArgs ba;
  int eb, lpr;
  mrec_status st = make_bank_args(bank, &ba, &eb, &lpr);
  if (st != MREC_OK) return st;
  MREC_CHECK_ARG(batch >= 0 && batch <= kMaxPlanKeys, "batch must be in [0, MREC_BWD_MAX_BATCH]");
  MREC_CHECK_ARG(workspace != nullptr, "workspace is NULL");
  if (ws_bytes < mrec_emb_bwd_workspace_size(ba.n_tables, batch)) {
    set_error("mrec_emb_bwd_apply: workspace too small");
    return MREC_ENOSPC;
  }
  MREC_CHECK_ARG(mode >= MREC_BWD_DENSE_GRAD && mode <= MREC_BWD_ADAM, "bad mode");
  // the layout this apply reads (hash: batch <= 4096, or an exchange view's given
  // gradients up to 8192 entries) must be the one the workspace's plan wrote
  const bool hash = hash_layout(batch, g_occ != nullptr || gw != nullptr);
  if ((st = ws_layout_check(workspace, hash ? kLayoutHash : kLayoutSorted, batch, ba.n_tables,
                            gw ? "mrec_emb_bwd_apply_wire"
                               : ro ? "mrec_emb_bwd_apply_rec"
                                    : g_occ ? "mrec_emb_bwd_apply_given" : "mrec_emb_bwd_apply")) !=
      MREC_OK)
    return st;
  MREC_CHECK_ARG(mode != MREC_BWD_DENSE_GRAD || grad != nullptr || ro != nullptr,
                 "DENSE_GRAD needs grad");
  if (ro) {
    MREC_CHECK_ARG(mode == MREC_BWD_DENSE_GRAD && grad == nullptr, "records take DENSE_GRAD sums");
    MREC_CHECK_ARG(hash_layout(batch, false), "record output needs the hash layout (batch <= 4096)");
    MREC_CHECK_ARG(ro->wire && ro->pref && ro->cap >= 1 && ro->cap_rows >= 1 &&
                       (reinterpret_cast<uintptr_t>(ro->wire) & 3) == 0,
                   "records: NULL wire / pref, bad cap");
    MREC_CHECK_ARG(ro->rec_dw * 4 >= (ba.dim + (ba.has_w ? 1 : 0)) * eb, "record narrower than a row");
    grad = bank->data;  // (the raw loads of the old sums read the rows: never used)
  }
  OptArgs opt{};
  if ((st = make_opt_args(bank, mode, &opt)) != MREC_OK) return st;
  const int F = ba.n_tables, D = ba.dim;
  if (dx) {
    MREC_CHECK_ARG(dx_dtype == MREC_F32 || dx_dtype == MREC_BF16, "dx dtype must be F32/BF16");
    const int xb = dx_dtype == MREC_F32 ? 4 : 2;
    MREC_CHECK_ARG(dx_ld >= static_cast<int64_t>(F) * D, "dx_ld < F*dim");
    MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(dx) & 15) == 0 && (dx_ld * xb) % 16 == 0,
                   "dx must be 16B aligned with 16B-multiple rows");
  }
  if (dfm) {
    MREC_CHECK_ARG(fm_sum != nullptr && x0 != nullptr, "dfm needs fm_sum and x0");
    MREC_CHECK_ARG(x0_dtype == MREC_F32 || x0_dtype == MREC_BF16, "x0 dtype must be F32/BF16");
    const int xb = x0_dtype == MREC_F32 ? 4 : 2;
    MREC_CHECK_ARG(x0_ld >= static_cast<int64_t>(F) * D, "x0_ld < F*dim");
    MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(x0) & 15) == 0 && (x0_ld * xb) % 16 == 0 &&
                       (reinterpret_cast<uintptr_t>(fm_sum) & 15) == 0,
                   "x0/fm_sum must be 16B aligned with 16B-multiple rows");
  }
  MREC_CHECK_ARG(dw == nullptr || ba.has_w, "dw given but bank has no w column");
  if (gw) {
    MREC_CHECK_ARG(!dx && !dfm && !dw && !g_occ, "wire gradients exclude dx / dfm / dw / g_occ");
    MREC_CHECK_ARG(gw->wire && gw->pref && gw->cap_rows >= 1, "NULL wire / pref");
    MREC_CHECK_ARG(gw->pitch >= D + (ba.has_w ? 1 : 0) && (gw->pitch * (gw->bf16 ? 2 : 4)) % 4 == 0 &&
                       (reinterpret_cast<uintptr_t>(gw->wire) & 3) == 0,
                   "records: pitch >= dim + has_w elements, 4-B aligned");
    MREC_CHECK_ARG(chunk >= 1 && chunk_stride >= F * chunk, "bad chunk");
  }
  if (g_occ) {
    MREC_CHECK_ARG(!dx && !dfm && !dw, "g_occ excludes dx / dfm / dw");
    MREC_CHECK_ARG(g_ld >= D + (ba.has_w ? 1 : 0) && g_ld % 4 == 0 &&
                       (reinterpret_cast<uintptr_t>(g_occ) & 15) == 0,
                   "g_occ rows must be 16B aligned, g_ld >= dim + has_w, g_ld % 4 == 0");
    MREC_CHECK_ARG(chunk >= 0 && (chunk == 0 || chunk_stride >= F * chunk), "bad chunk");
  }
  ApplyArgs a{};
  a.dx = dx;
  a.dx_ld = dx_ld;
  a.dx_bf16 = dx_dtype == MREC_BF16;
  a.dfm = dfm;
  a.fm_sum = fm_sum;
  a.x0 = x0;
  a.x0_ld = x0_ld;
  a.x0_bf16 = x0_dtype == MREC_BF16;
  a.dw = dw;
  a.mode = mode;
  a.lr = lr;
  a.seed = seed;
  a.d_step = d_step;
  a.grad = grad;
  a.g_occ = g_occ;
  a.g_ld = g_ld;
  a.chunk = chunk;
  a.chunk_stride = chunk_stride;
  a.g_rec = gw ? gw->wire : nullptr;
  a.g_rec_bf16 = gw ? gw->bf16 : 0;
  a.g_rec_pitch = gw ? gw->pitch : 0;
  a.g_pref = gw ? gw->pref : nullptr;
  a.g_cap_rows = gw ? gw->cap_rows : 0;
  a.g_F = F;
  a.opt = opt;
  a.o_rec = ro ? static_cast<uint32_t *>(ro->wire) : nullptr;
  a.o_rec_dw = ro ? ro->rec_dw : 0;
  a.o_pref = ro ? ro->pref : nullptr;
  a.o_F = F;
  a.o_cap = ro ? ro->cap : 1;
  a.o_cap_rows = ro ? ro->cap_rows : 0;
  MREC_CHECK_ARG(sgd_blocks >= 0 && (sgd_blocks == 0 || sgd_table != nullptr),
                 "sgd_blocks > 0 needs the table");
  a.sgd = static_cast<const SgdArgs *>(sgd_table);
  a.sgd_blocks = sgd_blocks;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int wpb = 256 / lpr;
  // hash layout (batch <= kHashMaxKeys or an exchange view, see mrec_emb_bwd_plan):
  // sample-major blocks + one hot-segment block per (table, bucket); sorted
  // layout: one block per WPB segments of each table
  const int seg_blocks = hash ? (batch > 0 ? F * kPlanBuckets : 0)
                              : static_cast<int>((batch + wpb - 1) / wpb);
  const int64_t sm_blocks = hash ? (batch * F + wpb - 1) / wpb : 0;
  const int apply_blocks =
      static_cast<int>(hash ? seg_blocks * (1 + kHotPer) + sm_blocks
                           : static_cast<int64_t>(seg_blocks) * F);
  CoReduce co = {};
  int co_blocks = 0;
  if (mrec_status st = build_co_reduce(n_reduce, reduce, &co, &co_blocks); st != MREC_OK)
    return st;
  co_blocks += sgd_blocks;  // (the SGD tiles follow the reductions, hash layout only)
  MREC_CHECK_ARG(sgd_blocks == 0 || hash, "SGD tiles ride in the hash-layout apply only");
  if (apply_blocks + co_blocks == 0) return MREC_OK;  // (batch 0 still runs the reductions)
  const dim3 grid(static_cast<unsigned>(apply_blocks + co_blocks));
  const KClock kc = hash ? kclock_take() : KClock{nullptr, 0};
#define MREC_AKM(T, L, M)                                                                         \
  do {                                                                                            \
    if (kc.buf)                                                                                   \
      apply_hash_kernel<T, L, M, true><<<grid, 256, 0, s>>>(ba, batch, workspace, a, seg_blocks,  \
                                                            static_cast<int>(sm_blocks), co, kc); \
    else                                                                                          \
      apply_hash_kernel<T, L, M, false><<<grid, 256, 0, s>>>(ba, batch, workspace, a, seg_blocks, \
                                                             static_cast<int>(sm_blocks), co, kc); \
  } while (0)
#define MREC_AK(T, L)                                                                            \
  do {                                                                                           \
    if (hash) {                                                                                  \
      if (mode == MREC_BWD_SGD) MREC_AKM(T, L, MREC_BWD_SGD);                                    \
      else if (mode == MREC_BWD_SGD_SR) MREC_AKM(T, L, MREC_BWD_SGD_SR);                         \
      else if (mode == MREC_BWD_DENSE_GRAD) MREC_AKM(T, L, MREC_BWD_DENSE_GRAD);                 \
      else MREC_AKM(T, L, -1); /* fused optimizers */                                            \
    } else                                                                                       \
      apply_kernel<T, L><<<grid, 256, 0, s>>>(ba, batch, workspace, a, seg_blocks, apply_blocks, \
                                              co);                                               \
  } while (0)
  if (bank->dtype == MREC_BF16) {
    switch (lpr) {
      case 1: MREC_AK(uint16_t, 1); break;
      case 2: MREC_AK(uint16_t, 2); break;
      case 4: MREC_AK(uint16_t, 4); break;
      case 8: MREC_AK(uint16_t, 8); break;
      default: MREC_AK(uint16_t, 16); break;
    }
  } else {
    switch (lpr) {
      case 1: MREC_AK(float, 1); break;
      case 2: MREC_AK(float, 2); break;
      case 4: MREC_AK(float, 4); break;
      case 8: MREC_AK(float, 8); break;
      default: MREC_AK(float, 16); break;
    }
  }
#undef MREC_AK
#undef MREC_AKM
  return launch_status("mrec_emb_bwd_apply");
}
