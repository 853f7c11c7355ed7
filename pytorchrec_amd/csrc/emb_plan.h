// Embedding-backward plan: per-table workspace layout and the hash plan body.
// Included by emb_bwd.hip (the standalone plan kernel and apply) and by gemm.hip
// (the plan run by spare workgroups of a backward GEMM launch).
#pragma once
#include "common.h"

namespace mrec {

constexpr int kPlanThreads = 1024;

struct TableWs {  // per-table workspace view of the sorted layout
  int32_t *hdr;   // [4] = {n segments, n lookups in segments, 0, layout}
  int32_t *perm;  // [Bp]   sample index of position i
  int32_t *seg;   // [Bp+1] segment starts
  int32_t *uniq;  // [Bp]   local row id of segment u
};
// layout 0 (sorted plan, batches up to MREC_BWD_MAX_BATCH): segments in
//   ascending row order, each segment's lookups in ascending sample order in
//   perm, segment u = [seg[u], seg[u + 1]).
// layout 1 (hash plan, batch <= MREC_BWD_HASH_MAX_BATCH or a padded exchange view):
//   per (table, bucket) descriptors of the rows hit more than once, and the
//   sample-major lookup table lut[b][f] (below, BucketWs / lookup_table).
// (kLayoutSorted / kLayoutHash: common.h)

__host__ __device__ inline int64_t pad4(int64_t x) { return (x + 3) & ~int64_t(3); }

__host__ __device__ inline int64_t table_ws_bytes(int64_t batch) {
  const int64_t bp = pad4(batch);
  int64_t bytes = 16 + 4 * (bp + (bp + 4) + bp);
  return (bytes + 255) & ~int64_t(255);
}

__host__ __device__ inline TableWs table_ws(const void *ws, int f, int64_t batch) {
  char *base = static_cast<char *>(const_cast<void *>(ws)) + f * table_ws_bytes(batch);
  const int64_t bp = pad4(batch);
  TableWs t;
  t.hdr = reinterpret_cast<int32_t *>(base);
  t.perm = reinterpret_cast<int32_t *>(base + 16);
  t.seg = t.perm + bp;
  t.uniq = t.seg + bp + 4;
  return t;
}

#ifdef MREC_PLAN_PROF
__device__ uint64_t g_plan_prof[16];
#define PLAN_STAMP(k)                                              \
  do {                                                             \
    __syncthreads();                                               \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_plan_prof[k] = wall_clock64(); \
  } while (0)
#else
#define PLAN_STAMP(k) \
  do {                \
  } while (0)
#endif

// ---------------------------------------------------------------------------
// hash plan (batch <= 4096; padded exchange views <= 8192 entries).
//
// Work split: table f's rows are cut into kPlanBuckets buckets by a hash of the
// row id, and one workgroup plans each (table, bucket): it loads all of the
// table's ids (L2 hits after the first), keeps the ones of its bucket and groups
// them in an LDS hash table.  Buckets partition the rows, so no row's lookups
// are split over workgroups and no cross-workgroup merge is needed; a table's
// plan runs on 8 CUs instead of 1 (C2: 208 workgroups beside the interaction; 8
// buckets over 4: interaction + apply 21.2 -> 19.4 us, step 0.0937 -> 0.0917 ms,
// same-box A/B -- the apply's segment blocks are per (table, bucket) too).
// A workgroup barrier costs ~135 ns at 1024 threads (tools/micro/barrier.hip);
// the body needs three:
//   1. insert: each id of the bucket goes into the hash table (linear probing;
//      tables of <= SLOTS rows index the slots directly), counting its lookups;
//   2. claim: every lookup takes a ticket on its slot; a row hit once writes its
//      row into the sample-major lookup table lut[b][f], the lookups of a
//      repeated row write -1 there and ticket 0 allocates the row's segment
//      (wave-aggregated packed LDS atomic: {segment, perm start}) and publishes
//      the start in the slot;
//   3. place: lookup i of a repeated row goes into the segment descriptor (two
//      lookups) or to perm[start + ticket].
// Segments longer than short_seg (hot rows) are also listed in the bucket's long
// list, which apply sums with a whole workgroup.  The order of a segment's
// lookups follows the atomics; apply sorts them back into ascending sample
// order, so the arithmetic does not depend on the schedule.
// ---------------------------------------------------------------------------
constexpr int kHashMaxKeys = 4096;     // dense batches up to this use the hash plan
constexpr int kHashMaxEntries = 8192;  // padded exchange views (ids.pad_negative) up to this:
                                       // their valid ids are ~1/2 of the entries (cap = 2x share)
constexpr int kHashSlots = 8192;       // per workgroup: any bucket fits at load factor <= 1/2
#ifndef MREC_PLAN_BUCKETS_LOG2
#define MREC_PLAN_BUCKETS_LOG2 3
#endif
constexpr int kPlanBuckets = 1 << MREC_PLAN_BUCKETS_LOG2;  // workgroups per table
#ifndef MREC_SHORT_SEG
#define MREC_SHORT_SEG 16
#endif
constexpr int kShortSeg = MREC_SHORT_SEG;  // longer segments: the bucket's long list
constexpr uint32_t kEmpty = 0xffffffffu;

// segments up to this many lookups are summed by one wave of the apply (one
// lookup per LPR-lane worker), longer ones by a whole workgroup
__host__ __device__ inline int short_seg(int lpr) {
  return 64 / lpr < kShortSeg ? 64 / lpr : kShortSeg;
}

// hash layout for `batch` entries (the same rule in plan and apply)
__host__ __device__ inline bool hash_layout(int64_t batch, bool padded) {
  return batch <= kHashMaxKeys || (padded && batch <= kHashMaxEntries);
}

__host__ __device__ inline uint32_t plan_bucket(uint32_t key) {
  return (key * 0x85ebca77u) >> (32 - MREC_PLAN_BUCKETS_LOG2);  // the top bits
}

// hash-layout workspace: F x kPlanBuckets bucket regions, then lut[B][F]
struct BucketWs {
  int32_t *hdr;    // [4] = {segments, perm entries, long segments, layout}
  int4 *desc;      // [seg_cap] segment u = {row, n, b0 | perm start, b1}
  int32_t *perm;   // [B] lookups of segments with n > 2
  int32_t *longl;  // [B / kShortSeg + 4] segment ids of the long segments
};

__host__ __device__ inline int64_t seg_cap(int64_t batch) { return batch / 2 + 4; }

__host__ __device__ inline int64_t bucket_ws_bytes(int64_t batch) {
  const int64_t bp = pad4(batch);
  const int64_t bytes = 16 + 16 * seg_cap(batch) + 4 * bp + 4 * (bp / kShortSeg + 4);
  return (bytes + 255) & ~int64_t(255);
}

__host__ __device__ inline int64_t hash_ws_bytes(int n_tables, int64_t batch) {
  const int64_t lut = (4 * pad4(batch) * n_tables + 255) & ~int64_t(255);
  const int64_t offs = (8 * int64_t(n_tables) + 255) & ~int64_t(255);
  return int64_t(n_tables) * kPlanBuckets * bucket_ws_bytes(batch) + lut + offs;
}

__host__ __device__ inline BucketWs bucket_ws(const void *ws, int f, int r, int64_t batch) {
  char *base = static_cast<char *>(const_cast<void *>(ws)) +
               (int64_t(f) * kPlanBuckets + r) * bucket_ws_bytes(batch);
  BucketWs t;
  t.hdr = reinterpret_cast<int32_t *>(base);
  t.desc = reinterpret_cast<int4 *>(base + 16);
  t.perm = reinterpret_cast<int32_t *>(t.desc + seg_cap(batch));
  t.longl = t.perm + pad4(batch);
  return t;
}

// lut[b * F + f]: row (>= 0) of a row hit once, -1 otherwise (a repeated row's
// lookup, an invalid id)
__host__ __device__ inline int32_t *lookup_table(const void *ws, int n_tables, int64_t batch) {
  return reinterpret_cast<int32_t *>(static_cast<char *>(const_cast<void *>(ws)) +
                                     int64_t(n_tables) * kPlanBuckets * bucket_ws_bytes(batch));
}

// the bank's table row offsets, copied by the plan: the apply indexes them per
// lane from memory (a per-lane index into the kernel-argument array would be
// lowered to a select chain over all of it in scalar registers)
__host__ __device__ inline int64_t *table_offsets(const void *ws, int n_tables, int64_t batch) {
  return reinterpret_cast<int64_t *>(
      reinterpret_cast<char *>(lookup_table(ws, n_tables, batch)) +
      ((4 * pad4(batch) * n_tables + 255) & ~int64_t(255)));
}

// smem: 2 * SLOTS + 2 words.  Called by all THREADS threads of the workgroup that
// plans (table f, bucket r).
template <int THREADS, int SLOTS, int MAXB = kHashMaxEntries>
__device__ __forceinline__ void plan_hash_body(const BankArgs &bank, const IdsArgs &ids, int64_t B,
                                               void *ws, int32_t *__restrict__ oob,
                                               uint64_t *__restrict__ d_step, int f, int r,
                                               uint32_t *smem) {
  // every entry in [0, B) is one thread's k-th round: B <= MAXB (host-checked) and
  // MAXB a multiple of THREADS; SLOTS >= MAXB bounds the linear probing (a bucket
  // holds at most B distinct keys, so an empty slot always exists)
  static_assert(THREADS % 64 == 0 && MAXB % THREADS == 0, "whole waves, whole rounds");
  static_assert(SLOTS >= MAXB, "the probe loop needs a free slot for every distinct key");
  constexpr int kRounds = MAXB / THREADS;
  uint32_t *hkey = smem;          // [SLOTS] row id; after the claim: (segment << 16) | start
  uint32_t *hcnt = smem + SLOTS;  // [SLOTS] (tickets << 16) | lookups
  uint32_t &s_tot = smem[2 * SLOTS];       // (segments << 16) | perm entries
  uint32_t &s_long = smem[2 * SLOTS + 1];  // long segments
  const int tid = threadIdx.x, lane = tid & 63;
  const int F = bank.n_tables;
  const uint32_t rows = static_cast<uint32_t>(bank.rows[f]);
  const bool direct = rows <= static_cast<uint32_t>(SLOTS);
  const BucketWs t = bucket_ws(ws, f, r, B);
  int32_t *__restrict__ lut = lookup_table(ws, F, B);
  PLAN_STAMP(0);
  // ids of this thread's lookups, loads issued before anything waits on them
  int64_t id[kRounds];
  load_ids_batch<kRounds>(ids, f, tid, THREADS, B, -1, id);
  static_assert(SLOTS % (4 * THREADS) == 0, "16-B LDS init");
  for (int i = 4 * tid; i < SLOTS; i += 4 * THREADS) {
    *reinterpret_cast<uint4 *>(hkey + i) = make_uint4(kEmpty, kEmpty, kEmpty, kEmpty);
    *reinterpret_cast<uint4 *>(hcnt + i) = make_uint4(0u, 0u, 0u, 0u);
  }
  if (tid == 0) {
    s_tot = 0u;
    s_long = 0u;
  }
  __syncthreads();
  PLAN_STAMP(1);
  // 1. insert (this bucket's valid ids); invalid ids are bucket 0's
  uint32_t slot[kRounds];
#pragma unroll
  for (int k = 0; k < kRounds; ++k) {
    const int i = k * THREADS + tid;
    slot[k] = kEmpty;
    if (i < B) {
      if (id[k] >= 0 && id[k] < static_cast<int64_t>(rows)) {
        const uint32_t key = static_cast<uint32_t>(id[k]);
        if (plan_bucket(key) == static_cast<uint32_t>(r)) {
          uint32_t h = key;
          if (!direct) {
            h = static_cast<uint32_t>((static_cast<uint64_t>(key * 2654435761u) * SLOTS) >> 32);
            for (;;) {
              const uint32_t old = atomicCAS(&hkey[h], kEmpty, key);
              if (old == kEmpty || old == key) break;
              h = h + 1 == SLOTS ? 0u : h + 1;
            }
          }
          atomicAdd(&hcnt[h], 1u);
          slot[k] = h;
        }
      } else if (r == 0) {
        lut[static_cast<int64_t>(i) * F + f] = -1;
        if (oob && !(ids.pad_negative && id[k] < 0)) *oob = 1;
      }
    }
  }
  __syncthreads();
  PLAN_STAMP(2);
  // 2. claim
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t ticket[kRounds], count[kRounds];
#pragma unroll
  for (int k = 0; k < kRounds; ++k) {
    ticket[k] = 0;
    count[k] = 0;
  }
#pragma unroll
  for (int k = 0; k < kRounds; ++k) {
    if (k * THREADS >= B) break;  // uniform
    const int i = k * THREADS + tid;
    uint32_t cnt = 0;
    if (slot[k] != kEmpty) {
      const uint32_t old = atomicAdd(&hcnt[slot[k]], 1u << 16);
      ticket[k] = old >> 16;
      cnt = old & 0xffffu;
      count[k] = cnt;
      const uint32_t row = direct ? slot[k] : hkey[slot[k]];
      if (cnt == 1) lut[static_cast<int64_t>(i) * F + f] = static_cast<int32_t>(row);
      else if (ticket[k] != 0) lut[static_cast<int64_t>(i) * F + f] = -1;
    }
    const bool claim = cnt > 1 && ticket[k] == 0;
    const uint64_t mc = __ballot(claim);
    if (mc == 0) continue;  // uniform
    const uint32_t need = (claim && cnt > 2) ? cnt : 0u;  // perm entries
    uint32_t incl = need;  // inclusive scan of the perm entries claimed
    if (__ballot(need != 0u) != 0ull) {  // uniform: only rows hit >= 3 times take perm
#pragma unroll                              // entries (most claims are pairs: no scan)
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(incl, off);
        if (lane >= off) incl += v;
      }
    }
    const int last = 63 - __clzll(mc);
    uint32_t base = 0;
    if (lane == last) base = atomicAdd(&s_tot, (static_cast<uint32_t>(__popcll(mc)) << 16) | incl);
    base = __shfl(base, last);
    if (claim) {
      const uint32_t u = (base >> 16) + __popcll(mc & lt);
      const uint32_t start = (base & 0xffffu) + incl - need;
      const uint32_t row = direct ? slot[k] : hkey[slot[k]];
      int32_t *d = reinterpret_cast<int32_t *>(t.desc + u);
      d[0] = static_cast<int32_t>(row);
      d[1] = static_cast<int32_t>(cnt);
      if (cnt > 2) d[2] = static_cast<int32_t>(start);
      hkey[slot[k]] = (u << 16) | start;  // only the claimer reads this slot's key
      lut[static_cast<int64_t>(i) * F + f] = -1;
      if (cnt > static_cast<uint32_t>(short_seg(bank.lpr)))
        t.longl[atomicAdd(&s_long, 1u)] = static_cast<int32_t>(u);
    }
  }
  __syncthreads();
  PLAN_STAMP(3);
  // 3. place
#pragma unroll
  for (int k = 0; k < kRounds; ++k) {
    const int i = k * THREADS + tid;
    if (i < B && count[k] > 1) {
      const uint32_t us = hkey[slot[k]];
      if (count[k] == 2)
        reinterpret_cast<int32_t *>(t.desc + (us >> 16))[2 + ticket[k]] = i;
      else
        t.perm[(us & 0xffffu) + ticket[k]] = i;
    }
  }
  if (tid == 0) {
    t.hdr[0] = static_cast<int32_t>(s_tot >> 16);
    t.hdr[1] = static_cast<int32_t>(s_tot & 0xffffu);
    t.hdr[2] = static_cast<int32_t>(s_long);
    t.hdr[3] = ws_layout_tag(kLayoutHash, B);
    if (r == 0) table_offsets(ws, F, B)[f] = bank.row_offset[f];
    if (d_step && f == 0 && r == 0) *d_step += 1;
  }
  PLAN_STAMP(4);
}

struct PlanJob {  // an embedding-backward hash plan run by spare workgroups of another launch
  BankArgs bank;
  IdsArgs ids;
  int64_t B;
  void *ws;
  int32_t *oob;
  uint64_t *d_step;
};

// host: validate a mrec_plan_job and fill its kernel arguments (emb_bwd.hip)
mrec_status build_plan_job(const mrec_plan_job *plan, PlanJob *out);

}  // namespace mrec
