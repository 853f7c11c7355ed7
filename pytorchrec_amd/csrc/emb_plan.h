// Embedding-backward plan: per-table workspace layout and the hash plan body.
// Included by emb_bwd.hip (the standalone plan kernel and apply) and by gemm.hip
// (the plan run by spare workgroups of a backward GEMM launch).
#pragma once
#include "common.h"

namespace mrec {

constexpr int kPlanThreads = 1024;

struct TableWs {  // per-table workspace view
  int32_t *hdr;   // [4] = {n segments, n lookups in segments, 0, layout}
  int4 *desc;     // [Bp/2+4] hash layout: segment u = {row, n, b0 | start, b1}
  int32_t *perm;  // [Bp]   sample index of position i
  int32_t *seg;   // [Bp+1] sorted layout: segment starts
  int32_t *uniq;  // [Bp]   sorted layout: local row id of segment u
  int32_t *lut;   // [Bp]   hash layout: row of lookup b if no other lookup hits it, else -1
};
// layout 0 (sorted plan): segments in ascending row order, each segment's
//   lookups in ascending sample order in perm, segment u = [seg[u], seg[u + 1]).
// layout 1 (hash plan): only rows hit more than once get a segment (<= B/2 of
//   them), in arbitrary order; a row hit once is listed in lut[b] of its lookup
//   and updated sample-major by apply.  Segment u is desc[u] = {row, n, b0, b1}
//   when n == 2 (both lookups in the descriptor) and {row, n, start, -} with the
//   lookups in perm[start, start + n) otherwise.  The order of a segment's
//   lookups is arbitrary -- apply restores ascending sample order itself, so
//   the arithmetic is identical to layout 0.
constexpr int kLayoutSorted = 0;
constexpr int kLayoutHash = 1;

__host__ __device__ inline int64_t pad4(int64_t x) { return (x + 3) & ~int64_t(3); }

__host__ __device__ inline int64_t table_ws_bytes(int64_t batch) {
  const int64_t bp = pad4(batch);
  int64_t bytes = 16 + 16 * (bp / 2 + 4) + 4 * (bp + (bp + 4) + bp + bp);
  return (bytes + 255) & ~int64_t(255);
}

__host__ __device__ inline TableWs table_ws(const void *ws, int f, int64_t batch) {
  char *base = static_cast<char *>(const_cast<void *>(ws)) + f * table_ws_bytes(batch);
  const int64_t bp = pad4(batch);
  TableWs t;
  t.hdr = reinterpret_cast<int32_t *>(base);
  t.desc = reinterpret_cast<int4 *>(base + 16);
  t.perm = reinterpret_cast<int32_t *>(t.desc + bp / 2 + 4);
  t.seg = t.perm + bp;
  t.uniq = t.seg + bp + 4;
  t.lut = t.uniq + bp;
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
// hash plan (batch <= 4096).  A workgroup barrier costs ~135 ns at 1024 threads
// (tools/micro/barrier.hip) and every 4-bit radix pass needs six, so the sorted
// plan spends most of its time in barriers.  The hash plan needs three:
//   1. insert: each valid id goes into an LDS hash table (linear probing),
//      counting its lookups (low 16 bits of the slot word);
//   2. claim: a row hit once is written to lut[i] of its lookup; otherwise every
//      lookup takes a ticket on its slot (high 16 bits) and ticket 0 allocates
//      the row's segment -- a wave-aggregated packed atomic hands out
//      {segment index, start} -- and publishes the start in the slot;
//   3. place: lookup i of a repeated row goes to perm[start + ticket].
// Segment order and the order inside a segment follow the atomics, so the
// workspace layout is not deterministic; apply sorts every segment's lookups
// back into ascending sample order, so the updates are.
// ---------------------------------------------------------------------------
constexpr int kHashMaxKeys = 4096;     // dense batches up to this use the hash plan
constexpr int kHashMaxEntries = 8192;  // padded exchange views (ids.pad_negative) up to this:
                                       // their valid ids are ~1/2 of the entries (cap = 2x share)
constexpr int kHashSlots = 8192;  // load factor <= 1/2 (standalone 1024-thread kernel)
constexpr int kHashSlotsSmall = 6016;  // 47 KiB: the plan inside a GEMM launch (<= 48 KiB LDS)
constexpr uint32_t kEmpty = 0xffffffffu;

// hash layout for `batch` entries (the same rule in plan and apply)
__host__ __device__ inline bool hash_layout(int64_t batch, bool padded) {
  return batch <= kHashMaxKeys || (padded && batch <= kHashMaxEntries);
}

template <int THREADS, int SLOTS, int MAXB = kHashMaxEntries>
__device__ __forceinline__ void plan_hash_body(const BankArgs &bank, const IdsArgs &ids, int64_t B,
                                               void *ws, int32_t *__restrict__ oob,
                                               uint64_t *__restrict__ d_step, int f,
                                               uint32_t *smem) {
  constexpr int kRounds = MAXB / THREADS;
  uint32_t *hkey = smem;          // [SLOTS] row id; after the claim: (segment << 16) | start
  uint32_t *hcnt = smem + SLOTS;  // [SLOTS] (tickets << 16) | lookups
  uint32_t &s_tot = smem[2 * SLOTS];  // (segments << 16) | lookups placed
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t rows = static_cast<uint32_t>(bank.rows[f]);
  const bool direct = rows <= static_cast<uint32_t>(SLOTS);
  const TableWs t = table_ws(ws, f, B);
  PLAN_STAMP(0);
  // ids of this thread's lookups, loads issued before anything waits on them
  int64_t id[kRounds];
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int i = r * THREADS + tid;
    id[r] = i < B ? load_id(ids, f, i) : -1;
  }
  for (int i = tid; i < SLOTS; i += THREADS) {
    hkey[i] = kEmpty;
    hcnt[i] = 0u;
  }
  if (tid == 0) s_tot = 0u;
  __syncthreads();
  PLAN_STAMP(1);
  // 1. insert
  uint32_t slot[kRounds];
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int i = r * THREADS + tid;
    slot[r] = kEmpty;
    if (i < B) {
      if (id[r] >= 0 && id[r] < static_cast<int64_t>(rows)) {
        const uint32_t key = static_cast<uint32_t>(id[r]);
        uint32_t h = key;  // tables of <= SLOTS rows index the slots directly
        if (!direct) {
          h = static_cast<uint32_t>((static_cast<uint64_t>(key * 2654435761u) * SLOTS) >> 32);
          for (;;) {
            const uint32_t old = atomicCAS(&hkey[h], kEmpty, key);
            if (old == kEmpty || old == key) break;
            h = h + 1 == SLOTS ? 0u : h + 1;
          }
        }
        atomicAdd(&hcnt[h], 1u);
        slot[r] = h;
      } else if (oob && !(ids.pad_negative && id[r] < 0)) {
        *oob = 1;
      }
    }
  }
  __syncthreads();
  PLAN_STAMP(2);
  // 2. claim
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t ticket[kRounds], count[kRounds];
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    ticket[r] = 0;
    count[r] = 0;
  }
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    if (r * THREADS >= B) break;  // uniform
    uint32_t cnt = 0;
    if (slot[r] != kEmpty) {
      const uint32_t old = atomicAdd(&hcnt[slot[r]], 1u << 16);
      ticket[r] = old >> 16;
      cnt = old & 0xffffu;
      count[r] = cnt;
    }
    {
      const int i = r * THREADS + tid;
      if (i < B)
        t.lut[i] = cnt == 1 ? static_cast<int32_t>(direct ? slot[r] : hkey[slot[r]]) : -1;
    }
    const bool claim = cnt > 1 && ticket[r] == 0;
    const uint64_t mc = __ballot(claim);
    if (mc == 0) continue;  // uniform
    uint32_t incl = claim ? cnt : 0u;  // inclusive scan of the claimed lengths
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t v = __shfl_up(incl, off);
      if (lane >= off) incl += v;
    }
    const int last = 63 - __clzll(mc);
    uint32_t base = 0;
    if (lane == last) base = atomicAdd(&s_tot, (static_cast<uint32_t>(__popcll(mc)) << 16) | incl);
    base = __shfl(base, last);
    if (claim) {
      const uint32_t u = (base >> 16) + __popcll(mc & lt);
      const uint32_t start = (base & 0xffffu) + incl - cnt;
      int32_t *d = reinterpret_cast<int32_t *>(t.desc + u);
      d[0] = static_cast<int32_t>(direct ? slot[r] : hkey[slot[r]]);
      d[1] = static_cast<int32_t>(cnt);
      if (cnt > 2) d[2] = static_cast<int32_t>(start);
      hkey[slot[r]] = (u << 16) | start;  // only the claimer reads this slot's key
    }
  }
  __syncthreads();
  PLAN_STAMP(3);
  // 3. place
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int i = r * THREADS + tid;
    if (i < B && count[r] > 1) {
      const uint32_t us = hkey[slot[r]];
      if (count[r] == 2)
        reinterpret_cast<int32_t *>(t.desc + (us >> 16))[2 + ticket[r]] = i;
      else
        t.perm[(us & 0xffffu) + ticket[r]] = i;
    }
  }
  if (tid == 0) {
    t.hdr[0] = static_cast<int32_t>(s_tot >> 16);
    t.hdr[1] = static_cast<int32_t>(s_tot & 0xffffu);
    t.hdr[2] = 0;
    t.hdr[3] = kLayoutHash;
    if (d_step && f == 0) *d_step += 1;
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
