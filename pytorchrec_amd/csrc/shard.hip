// Row-sharded embedding tables: the id -> owner exchange around the hot path.
// (The compact exchange of ABI 19 -- bucketize_dedup, gather_wire, wire_move -- is
// described at its kernels below.)
//
// bucketize   (sender, fwd) : stable counting sort of each table's ids by owner
//                             rank (id % W) into fixed-capacity send slots, and the
//                             slot of every lookup (where its row will come back);
// gather      (owner,  fwd) : rows of the received local ids -> send buffer;
// lookup_grad (sender, bwd) : per-lookup gradient rows written to the slot the row
//                             came from, ready for the reverse all-to-all.
// The owner's update reuses the hash plan over the padded exchange view (run inside
// the interaction launch, mrec_interact_fwd_ex) and mrec_emb_bwd_apply_given.  All
// three kernels are HBM/latency bound byte moves.
#include <algorithm>

#include "common.h"
#include "emb_plan.h"

namespace mrec {

constexpr int kBT = 1024;          // bucketize threads (one workgroup per table)
constexpr int kBWaves = kBT / 64;  // 16
constexpr int kBHist = 2048;       // (W + 1) * groups

struct RowsArg {
  int64_t v[MREC_MAX_TABLES];
};

// wave lanes holding the same owner value d (nbits-bit values)
__device__ __forceinline__ uint64_t same_value_lanes(uint32_t d, int nbits) {
  uint64_t m = ~0ull;
  for (int k = 0; k < nbits; ++k) {
    const uint64_t bk = __ballot((d >> k) & 1u);
    m &= ((d >> k) & 1u) ? bk : ~bk;
  }
  return m;
}

// exclusive scan of n <= 2 * kBT values in place (1024-thread block)
__device__ void scan_2048(uint32_t *a, int n, uint32_t *wtot) {
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
    const uint32_t w = lane < kBWaves ? wtot[lane] : 0u;
    uint32_t wi = w;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t t = __shfl_up(wi, off);
      if (lane >= off) wi += t;
    }
    if (lane < kBWaves) wtot[lane] = wi - w;
  }
  __syncthreads();
  const uint32_t ex = wtot[wid] + incl - v0 - v1;
  if (i0 < n) a[i0] = ex;
  if (i0 + 1 < n) a[i0 + 1] = ex + v0;
  __syncthreads();
}

// Element i of the table (sample b = i, ascending) sits in round r = i / 1024,
// wave w, so (round, wave) groups are in sample order; per-(owner, group) counts
// in owner-major order + one scan give each element its stable slot.
__global__ __launch_bounds__(kBT) void bucketize_kernel(IdsArgs ids, RowsArg rows, int64_t B,
                                                        int W, int cap, int F,
                                                        int32_t *__restrict__ send_ids,
                                                        int32_t *__restrict__ pos,
                                                        int32_t *__restrict__ overflow,
                                                        int32_t *__restrict__ oob) {
  __shared__ uint32_t hist[kBHist];
  __shared__ uint32_t wtot[kBWaves];
  const int f = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t rows_f = rows.v[f];
  const int rounds = static_cast<int>((B + kBT - 1) / kBT);
  const int G = rounds * kBWaves;
  const int nh = (W + 1) * G;
  const int nbits = 32 - __clz(static_cast<uint32_t>(W));  // values 0..W
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  // every round's id is loaded before the first is used (one memory latency, not
  // one per round); ids < rows < 2^31, so owner / local row use 32-bit division
  constexpr int kPre = 8;
  int64_t pre[kPre];
  load_ids_batch<kPre>(ids, f, tid, kBT, B, -1, pre);
  auto id_of = [&](int r, int64_t i) -> int64_t {
    if (i >= B) return -1;
    if (r < kPre) {
#pragma unroll
      for (int k = 0; k < kPre; ++k)
        if (k == r) return pre[k];
    }
    return load_id(ids, f, i);
  };
  for (int i = tid; i < nh; i += kBT) hist[i] = 0u;
  __syncthreads();
  for (int r = 0; r < rounds; ++r) {
    const int64_t i = static_cast<int64_t>(r) * kBT + tid;
    uint32_t d = static_cast<uint32_t>(W);
    const int64_t id = id_of(r, i);
    if (id >= 0 && id < rows_f) d = static_cast<uint32_t>(id) % static_cast<uint32_t>(W);
    const uint64_t m = same_value_lanes(d, nbits);
    if ((m & lt) == 0) hist[d * G + r * kBWaves + wid] = __popcll(m);
  }
  __syncthreads();
  scan_2048(hist, nh, wtot);
  for (int r = 0; r < rounds; ++r) {
    const int64_t i = static_cast<int64_t>(r) * kBT + tid;
    uint32_t d = static_cast<uint32_t>(W);
    const int64_t id = id_of(r, i);
    if (id >= 0 && id < rows_f) d = static_cast<uint32_t>(id) % static_cast<uint32_t>(W);
    const uint64_t m = same_value_lanes(d, nbits);
    if (i >= B) continue;
    if (d == static_cast<uint32_t>(W)) {
      if (oob) *oob = 1;
      pos[f * B + i] = -1;
      continue;
    }
    const uint32_t slot = hist[d * G + r * kBWaves + wid] + __popcll(m & lt) - hist[d * G];
    if (slot >= static_cast<uint32_t>(cap)) {
      if (overflow) atomicOr(overflow, 1);  // bit 0: a table's `cap` slots
      pos[f * B + i] = -1;
      continue;
    }
    const int64_t s = (static_cast<int64_t>(d) * F + f) * cap + slot;
    send_ids[s] = static_cast<int32_t>(static_cast<uint32_t>(id) / static_cast<uint32_t>(W));
    pos[f * B + i] = static_cast<int32_t>(s);
  }
  // padding slots of every owner part
  for (int d = 0; d < W; ++d) {
    const uint32_t cnt = min(static_cast<uint32_t>(cap), hist[(d + 1) * G] - hist[d * G]);
    int32_t *part = send_ids + (static_cast<int64_t>(d) * F + f) * cap;
    for (int s = static_cast<int>(cnt) + tid; s < cap; s += kBT) part[s] = -1;
  }
}

// ---------------------------------------------------------------------------
// Compact (deduplicated) exchange, ABI 19.
//
// bucketize_dedup: as bucketize, but only the FIRST lookup of each distinct id
// (ascending sample order) takes a slot -- the distinct ids of a table are found in
// an LDS hash table (linear probing; the smallest sample index of each id kept by
// an LDS atomic min) -- and every later lookup of that id gets the same pos.  Each
// owner part of send_ids is [n_tables][cap] slots followed by the n_tables counts
// (the header every wire kernel reads).
// ---------------------------------------------------------------------------

// (kEmpty: emb_plan.h)

__device__ __forceinline__ uint32_t id_hash(uint32_t x, uint32_t mask) {
  return (x * 2654435761u) & mask;
}

// Batches past one workgroup's hash (8192 samples) are cut into C chunks of cb
// samples (grid y): chunk c of the batch is its own "sub-sender", part d * C + c of
// send_ids (owner d's C parts contiguous, so the equal-split all-to-all still moves
// W parts of C * P); an id repeated across chunks takes a slot in each.
// Quarters (ABI 28, mrec_shard_bucketize_dedup_q): H = 2^lgH workgroups per (table,
// chunk), workgroup h taking the ids whose dedup_quarter is h, so each inserts and
// ranks ~1/H of the table's distinct ids (the id loads, the LDS hash and the ranks
// were one workgroup's serial chain: 3.3 + 0.6 + 3.4 + 2.2 + 2.1 us at C2's shape).
// A part's slots are then quarter-major (quarter 0's distinct ids in first-lookup
// order, then quarter 1's, ...): each workgroup publishes its per-owner counts and
// waits for its H - 1 siblings (one agent-scope ticket, bounded spin; the siblings
// are adjacent workgroups, dispatched together) to place its ids after the lower
// quarters'.  The slot order changes no arithmetic (one entry per distinct id and
// owner); cpu_bucketize_dedup restates the same order.
__host__ __device__ inline uint32_t dedup_quarter(uint32_t key, int lgH) {
  return lgH ? (key * 0x9e3779b1u) >> (32 - lgH) : 0u;
}
constexpr int kDedupMaxW = 128;  // (W + 1) * groups <= 2048 keeps W below this anyway

template <bool KC>
__global__ __launch_bounds__(kBT) void bucketize_dedup_kernel(IdsArgs ids, RowsArg rows, int64_t Btot,
                                                              int W, int cap, int F, int hs,
                                                              int32_t *__restrict__ send_ids,
                                                              int32_t *__restrict__ pos,
                                                              int32_t *__restrict__ overflow,
                                                              int32_t *__restrict__ oob, int C,
                                                              int64_t cb, int lgH,
                                                              int32_t *__restrict__ qcnt,
                                                              unsigned long long *__restrict__ arrive,
                                                              int spin_bound, KClock kc) {
  KcScope<KC> kc_scope(kc);  // (clocked instantiation: bench.py in-step times)
  __shared__ uint32_t hist[kBHist];
  __shared__ uint32_t wtot[kBWaves];
  __shared__ uint32_t s_base[kDedupMaxW], s_tot[kDedupMaxW];
  __shared__ int s_ok;
  extern __shared__ uint32_t hash_lds[];  // keys [hs] | (first << 16 | slot) [hs]
  uint32_t *keys = hash_lds;
  uint32_t *fs = hash_lds + hs;
  const uint32_t hmask = static_cast<uint32_t>(hs - 1);
  const int H = 1 << lgH;
  const int f = blockIdx.x >> lgH;
  const int qh = blockIdx.x & (H - 1);
  const int c = blockIdx.y;
  const int64_t s0 = static_cast<int64_t>(c) * cb;
  const int64_t B = min(cb, Btot - s0);  // this chunk's samples
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t rows_f = rows.v[f];
  const int rounds = static_cast<int>((B + kBT - 1) / kBT);  // <= 8 (B <= 8192)
  const int G = rounds * kBWaves;
  const int nh = (W + 1) * G;
  const int nbits = 32 - __clz(static_cast<uint32_t>(W));
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t P = static_cast<int64_t>(F) * cap + F;  // int32 per owner part
  constexpr int kR = 8;
  int64_t idv[kR];
  load_ids_batch<kR>(ids, f, s0 + tid, kBT, s0 + B, -2, idv);
#ifndef MREC_BKT_EXP
#define MREC_BKT_EXP 0
#endif
#if MREC_BKT_EXP  // (diagnostics: phases skipped; the message left empty: no slot, no count)
  auto diag_exit = [&](bool keep) {
    if (keep) *oob = 7;
    for (int r = 0; r < kR; ++r) {
      const int64_t i = static_cast<int64_t>(r) * kBT + tid;
      if (i < B) pos[f * Btot + s0 + i] = -1;
    }
    for (int d = 0; d < W; ++d) {
      const int64_t pd = (static_cast<int64_t>(d) * C + c) * P;
      for (int s = tid; s < cap; s += kBT) send_ids[pd + static_cast<int64_t>(f) * cap + s] = -1;
      if (tid == 0) send_ids[pd + static_cast<int64_t>(F) * cap + f] = 0;
    }
  };
#endif
#if MREC_BKT_EXP == 1  // (diagnostic: the id loads only)
  diag_exit(idv[0] == -12345 && idv[kR - 1] == -12345);
  return;
#endif
  for (int i = tid; i < nh; i += kBT) hist[i] = 0u;
  for (int i = tid; i < hs; i += kBT) {
    keys[i] = kEmpty;
    fs[i] = kEmpty;
  }
  __syncthreads();
#if MREC_BKT_EXP == 2  // (diagnostic: + the LDS init)
  diag_exit(idv[0] == -12345 && idv[kR - 1] == -12345 && keys[tid] == 5u);
  return;
#endif
  // 1. distinct ids: insert, keep the first sample index of each
  uint32_t hpos[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    hpos[r] = kEmpty;
    const int64_t id = idv[r];
    if (id >= 0 && id < rows_f && dedup_quarter(static_cast<uint32_t>(id), lgH) == static_cast<uint32_t>(qh)) {
      const uint32_t key = static_cast<uint32_t>(id);
      uint32_t h = id_hash(key, hmask);
      while (true) {
        const uint32_t prev = atomicCAS(&keys[h], kEmpty, key);
        if (prev == kEmpty || prev == key) break;
        h = (h + 1) & hmask;
      }
      hpos[r] = h;
      atomicMin(&fs[h], (static_cast<uint32_t>(r * kBT + tid) << 16) | 0xffffu);
    }
  }
  __syncthreads();
#if MREC_BKT_EXP == 3  // (diagnostic: + the inserts)
  diag_exit(hpos[0] == 12345u);
  return;
#endif
  // 2. stable per-owner ranks of the first lookups (owner W = no slot)
  uint32_t dv[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    if (r >= rounds) continue;
    uint32_t d = static_cast<uint32_t>(W);
    const uint32_t i = static_cast<uint32_t>(r * kBT + tid);
    if (hpos[r] != kEmpty && (fs[hpos[r]] >> 16) == i)
      d = static_cast<uint32_t>(idv[r]) % static_cast<uint32_t>(W);
    dv[r] = d;
    const uint64_t m = same_value_lanes(d, nbits);
    if ((m & lt) == 0) hist[d * G + r * kBWaves + wid] = __popcll(m);
  }
  __syncthreads();
  scan_2048(hist, nh, wtot);
#if MREC_BKT_EXP == 4  // (diagnostic: + the ranks and the scan)
  diag_exit(hist[tid] == 12345u);
  return;
#endif
  // this quarter's slot base per owner (after the lower quarters') and the totals
  if (H == 1) {
    if (tid < W) {
      s_base[tid] = 0u;
      s_tot[tid] = hist[(tid + 1) * G] - hist[tid * G];
    }
  } else {
    const int64_t q0 = (static_cast<int64_t>(c) * F + f) * H;
    if (tid < W)
      __hip_atomic_store(qcnt + (q0 + qh) * W + tid,
                         static_cast<int32_t>(hist[(tid + 1) * G] - hist[tid * G]),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the counts are agent-scope atomic (write-through) stores, drained before the
    // ticket and read back by agent-scope atomic loads: no release / acquire fence
    // (MI355X L1 invalidation ~1.7 us; cdna_hip_programming.md Guideline 16 R1)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      unsigned long long *ctr = arrive + static_cast<int64_t>(c) * F + f;
      // arrivals only grow (H per call): this call's H tickets end at the next multiple
      const unsigned long long t = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long target = (t / H + 1) * H;
      int ok = 1;
      for (int spins = 0; __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target;) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > spin_bound) {
          ok = 0;
          if (overflow) atomicOr(overflow, 4);  // bit 2: a quarter's wait timed out
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: order only)
      s_ok = ok;
    }
    __syncthreads();
    if (tid < W) {
      uint32_t base = 0u, tot = 0u;
      for (int h2 = 0; h2 < H; ++h2) {
        const uint32_t v = static_cast<uint32_t>(
            __hip_atomic_load(qcnt + (q0 + h2) * W + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (h2 < qh) base += v;
        tot += v;
      }
      s_base[tid] = s_ok ? base : 0u;
      s_tot[tid] = s_ok ? tot : 0u;
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    if (r >= rounds) continue;
    const uint32_t d = dv[r];
    const uint64_t m = same_value_lanes(d, nbits);
    if (d == static_cast<uint32_t>(W)) continue;
    uint32_t slot = hist[d * G + r * kBWaves + wid] + __popcll(m & lt) - hist[d * G] + s_base[d];
    if (slot >= static_cast<uint32_t>(cap)) {
      if (overflow) atomicOr(overflow, 1);  // bit 0: a table's `cap` slots
      slot = 0xffffu;
    } else {
      send_ids[(static_cast<int64_t>(d) * C + c) * P + static_cast<int64_t>(f) * cap + slot] =
          static_cast<int32_t>(static_cast<uint32_t>(idv[r]) / static_cast<uint32_t>(W));
    }
    fs[hpos[r]] = (static_cast<uint32_t>(r * kBT + tid) << 16) | slot;
  }
  __syncthreads();
  // 3. every lookup: the slot of its id
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int64_t i = static_cast<int64_t>(r) * kBT + tid;
    if (r >= rounds || i >= B) continue;
    const int64_t id = idv[r];
    if (hpos[r] == kEmpty) {
      const bool valid = id >= 0 && id < rows_f;
      if (valid) continue;  // another quarter's id: its workgroup writes the slot
      if (qh == 0) {        // an invalid id: quarter 0 alone flags it
        if (oob && id != -2) *oob = 1;
        pos[f * Btot + s0 + i] = -1;
      }
      continue;
    }
    const uint32_t slot = fs[hpos[r]] & 0xffffu;
    const uint32_t d = static_cast<uint32_t>(id) % static_cast<uint32_t>(W);
    pos[f * Btot + s0 + i] =
        slot == 0xffffu ? -1
                        : static_cast<int32_t>(((static_cast<int64_t>(d) * C + c) * F + f) * cap + slot);
  }
  // 4. counts header and padding slots of every owner part (the last quarter: every
  // quarter's slots lie below the total)
  if (qh == H - 1) {
    for (int d = 0; d < W; ++d) {
      const uint32_t cnt = min(static_cast<uint32_t>(cap), s_tot[d]);
      const int64_t pd = (static_cast<int64_t>(d) * C + c) * P;
      int32_t *part = send_ids + pd + static_cast<int64_t>(f) * cap;
      for (int s = static_cast<int>(cnt) + tid; s < cap; s += kBT) part[s] = -1;
      if (tid == 0) send_ids[pd + static_cast<int64_t>(F) * cap + f] = static_cast<int32_t>(cnt);
    }
  }
}

// ---------------------------------------------------------------------------
// wire records: round4((dim + has_w) * elem bytes) bytes per distinct row (bf16,
// dim 16 + w: 36 B, against 64 B per slot), part p of a wire buffer holds cap_rows
// records; table f's entries of part p start at prefix_p(f) = sum_{g<f} count_p(g)
// (the counts of the header of `hdr`, W parts of n_tables*cap + n_tables int32).
// The kernels below walk one part's records as a FLAT element space (record x
// dword): a workgroup takes kWireElems consecutive elements, so lanes touch
// consecutive dwords of the wire (coalesced) and every workgroup has the same
// amount of work whatever the per-table counts; an element's table comes from a
// binary search of the part's count prefix, kept in LDS.
// ---------------------------------------------------------------------------

constexpr int kWireThreads = 1024;
#ifndef MREC_WIRE_PER
#define MREC_WIRE_PER 2
#endif
constexpr int kWirePer = MREC_WIRE_PER;  // elements per thread
constexpr int kWireElems = kWireThreads * kWirePer;

struct WireArgs {
  const int32_t *hdr;  // W parts of F*cap + F (counts at F*cap + f)
  int W, F, cap, cap_rows;
  int32_t *pref;  // gather: [W][F] per-part table prefixes written here (NULL: not)
  int rec_dw;          // dwords per record
  int32_t *overflow;
};

// exclusive prefix of part p's per-table counts into pre[0..F]; returns the part's
// record total, clipped to cap_rows (and flags the overflow)
__device__ __forceinline__ int wire_prefix(const WireArgs &w, int p, int *pre) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int32_t *h = w.hdr + static_cast<int64_t>(p) * (static_cast<int64_t>(w.F) * w.cap + w.F) +
                       static_cast<int64_t>(w.F) * w.cap;
    int s = lane < w.F ? h[lane] : 0;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int t = __shfl_up(s, off);
      if (lane >= off) s += t;
    }
    if (lane < w.F) pre[lane + 1] = s;
    if (lane == 0) pre[0] = 0;
  }
  __syncthreads();
  int tot = pre[w.F];
  if (tot > w.cap_rows) {
    if (w.overflow && threadIdx.x == 0) atomicOr(w.overflow, 2);  // bit 1: `cap_rows` records
    tot = w.cap_rows;
  }
  return tot;
}

// the table holding record r (< the part's total): the largest f with pre[f] <= r
__device__ __forceinline__ int wire_table(const int *pre, int F, int r) {
  int lo = 0, hi = F;  // pre[lo] <= r < pre[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (pre[mid] <= r)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// owner: local bank rows of part p's received ids -> wire records (grid: chunks x W,
// flattened: blockIdx.x = p * chunks + chunk after `plan_blocks` leading workgroups
// that run the owner's backward hash plan over the same received ids, PLAN).  ADAM:
// a lazily updated Adam bank's rows go out as of the current step (adam_current on
// the 16-B chunk holding the dword, as mrec_shard_gather does for the slot rows).
template <bool PLAN, typename T = uint16_t, bool ADAM = false, bool KC = false>
__global__ __launch_bounds__(kWireThreads) void gather_wire_kernel(BankArgs bank, WireArgs w,
                                                                   const int32_t *__restrict__ recv,
                                                                   uint32_t *__restrict__ wire,
                                                                   int chunks, PlanJob plan,
                                                                   int plan_blocks, KClock kc) {
  KcScope<KC> kc_scope(kc);
  if constexpr (PLAN) {
    if (static_cast<int>(blockIdx.x) < plan_blocks) {  // uniform: (table, bucket) plans
      __shared__ __attribute__((aligned(16))) uint32_t smem[2 * kHashSlots + 2];
      plan_hash_body<kWireThreads, kHashSlots>(plan.bank, plan.ids, plan.B, plan.ws, plan.oob,
                                               plan.d_step, blockIdx.x / kPlanBuckets,
                                               blockIdx.x % kPlanBuckets, smem);
      return;
    }
  }
  __shared__ int pre[MREC_MAX_TABLES + 1];
  __shared__ int64_t roff[MREC_MAX_TABLES], nrows[MREC_MAX_TABLES];
  const int gb = static_cast<int>(blockIdx.x) - (PLAN ? plan_blocks : 0);
  const int p = gb / chunks, cx = gb - p * chunks;
  if (threadIdx.x < w.F) {
    roff[threadIdx.x] = bank.row_offset[threadIdx.x];
    nrows[threadIdx.x] = bank.rows[threadIdx.x];
  }
  const int tot = wire_prefix(w, p, pre);  // (its barrier covers roff / nrows too)
  if (w.pref && cx == 0 && threadIdx.x < w.F) w.pref[p * w.F + threadIdx.x] = pre[threadIdx.x];
  // element indices fit 32 bits (checked on the host): 32-bit divisions, not 64-bit
  const uint32_t n = static_cast<uint32_t>(tot) * static_cast<uint32_t>(w.rec_dw);
  const uint32_t e0 = static_cast<uint32_t>(cx) * kWireElems + threadIdx.x;
  if (e0 - threadIdx.x >= n) return;
  const uint32_t rdw = static_cast<uint32_t>(w.rec_dw);
  const int32_t *ids = recv + static_cast<int64_t>(p) * (static_cast<int64_t>(w.F) * w.cap + w.F);
  const uint32_t *data = reinterpret_cast<const uint32_t *>(bank.data);
  const int row_dw = bank.lpr * 4;
  // every id load first, unconditionally (element 0 past n) and pinned by an empty
  // use: under `if (e < n)` each load waited on its own (one round trip per element)
  int64_t src[kWirePer];
  int32_t idv[kWirePer];
  int fr[kWirePer], kr[kWirePer];
#pragma unroll
  for (int it = 0; it < kWirePer; ++it) {
    const uint32_t e = e0 + it * kWireThreads;
    const uint32_t ec = e < n ? e : 0u;
    const int r = static_cast<int>(ec / rdw);
    kr[it] = static_cast<int>(ec - r * rdw);
    fr[it] = wire_table(pre, w.F, r);
    idv[it] = ids[static_cast<int64_t>(fr[it]) * w.cap + (r - pre[fr[it]])];
  }
#pragma unroll
  for (int it = 0; it < kWirePer; ++it) asm volatile("" ::"v"(idv[it]));
#pragma unroll
  for (int it = 0; it < kWirePer; ++it) {
    const int64_t id = idv[it];
    const int f = fr[it];
    src[it] = (e0 + it * kWireThreads < n && id >= 0 && id < nrows[f])
                  ? (roff[f] + id) * row_dw + kr[it]
                  : -1;
  }
  uint32_t v[kWirePer];
  if constexpr (!ADAM) {  // the row dwords the same way
#pragma unroll
    for (int it = 0; it < kWirePer; ++it) v[it] = data[src[it] >= 0 ? src[it] : 0];
#pragma unroll
    for (int it = 0; it < kWirePer; ++it) asm volatile("" ::"v"(v[it]));
  }
#pragma unroll
  for (int it = 0; it < kWirePer; ++it) {
    if constexpr (ADAM) {
      constexpr int EPL = Vec<T>::EPL;
      v[it] = 0u;
      if (src[it] >= 0) {
        const int64_t grow = src[it] / row_dw;
        const int k = static_cast<int>(src[it] - grow * row_dw), c = k >> 2;
        uint4 raw = reinterpret_cast<const uint4 *>(bank.data)[grow * bank.lpr + c];
        raw = adam_current<T>(bank, grow, c * EPL, live_elems(bank, c * EPL, EPL), raw,
                              *bank.adam.d_t);
        const uint32_t q[4] = {raw.x, raw.y, raw.z, raw.w};
        v[it] = q[k & 3];
      }
    } else {
      v[it] = src[it] >= 0 ? v[it] : 0u;
    }
  }
  uint32_t *dst = wire + static_cast<int64_t>(p) * w.cap_rows * w.rec_dw;
#pragma unroll
  for (int it = 0; it < kWirePer; ++it) {
    const uint32_t e = e0 + it * kWireThreads;
    if (e < n) dst[e] = v[it];
  }
}

// wire records <-> slot rows [(p * F + f) * cap + j] of `slots` (row pitch slot_dw
// dwords).  unpack (elements = record x max(slot_dw, zero_dw)): the record into
// the slot row (dwords past the record zeroed; with to_f32 the bf16 record is
// widened to fp32: dwords of fp32 = 2 x record elements), and zero the first
// zero_dw dwords of the same row of `zero` when given; pack (elements = record x
// rec_dw): the slot row's first rec_dw dwords into the record.  Grid: chunks x W.
template <bool UNPACK, bool TO_F32, bool KC = false>
__global__ __launch_bounds__(kWireThreads) void wire_move_kernel(WireArgs w,
                                                                 uint32_t *__restrict__ wire,
                                                                 uint32_t *__restrict__ slots,
                                                                 int slot_dw,
                                                                 uint32_t *__restrict__ zero,
                                                                 int zero_dw, KClock kc) {
  KcScope<KC> kc_scope(kc);
  __shared__ int pre[MREC_MAX_TABLES + 1];
  const int p = blockIdx.y;
  const int tot = wire_prefix(w, p, pre);
  // unpack: the part's table prefixes for the sender's gradient records (ABI 26)
  if (UNPACK && w.pref && blockIdx.x == 0 && threadIdx.x < w.F)
    w.pref[p * w.F + threadIdx.x] = pre[threadIdx.x];
  const int epr = UNPACK ? max(slot_dw, zero ? zero_dw : 0) : w.rec_dw;
  // element indices fit 32 bits (checked on the host): 32-bit divisions, not 64-bit
  const uint32_t n = static_cast<uint32_t>(tot) * static_cast<uint32_t>(epr);
  const uint32_t e0 = blockIdx.x * kWireElems + threadIdx.x;
  if (e0 - threadIdx.x >= n) return;
  const uint32_t uepr = static_cast<uint32_t>(epr);
  uint32_t *rec0 = wire + static_cast<int64_t>(p) * w.cap_rows * w.rec_dw;
  int64_t srow[kWirePer];
  int kk[kWirePer], rr[kWirePer];
#pragma unroll
  for (int it = 0; it < kWirePer; ++it) {
    const uint32_t e = e0 + it * kWireThreads;
    srow[it] = -1;
    kk[it] = 0;
    rr[it] = 0;
    if (e < n) {
      const uint32_t r = e / uepr;
      const int f = wire_table(pre, w.F, static_cast<int>(r));
      srow[it] = (static_cast<int64_t>(p) * w.F + f) * w.cap + (static_cast<int>(r) - pre[f]);
      kk[it] = static_cast<int>(e - r * uepr);
      rr[it] = static_cast<int>(r);
    }
  }
  if constexpr (UNPACK) {
    uint32_t v[kWirePer];
#pragma unroll
    for (int it = 0; it < kWirePer; ++it) {
      const int k = kk[it];
      const int src = TO_F32 ? (k >> 1) : k;
      v[it] = (srow[it] >= 0 && src < w.rec_dw && (!TO_F32 || k < 2 * w.rec_dw))
                  ? rec0[static_cast<int64_t>(rr[it]) * w.rec_dw + src]
                  : 0u;
    }
#pragma unroll
    for (int it = 0; it < kWirePer; ++it) {
      if (srow[it] < 0) continue;
      const int k = kk[it];
      uint32_t x = v[it];
      if constexpr (TO_F32) x = (k & 1) ? (x & 0xffff0000u) : (x << 16);  // bf16 pair -> fp32
      if (k < slot_dw) slots[srow[it] * slot_dw + k] = x;
      if (zero && k < zero_dw) zero[srow[it] * zero_dw + k] = 0u;
    }
  } else {
    uint32_t v[kWirePer];
#pragma unroll
    for (int it = 0; it < kWirePer; ++it)
      v[it] = srow[it] >= 0 ? slots[srow[it] * slot_dw + kk[it]] : 0u;
#pragma unroll
    for (int it = 0; it < kWirePer; ++it)
      if (srow[it] >= 0) rec0[static_cast<int64_t>(rr[it]) * w.rec_dw + kk[it]] = v[it];
  }
}

static dim3 wire_grid(const WireArgs &w, int elems_per_record) {
  const int64_t chunks = (static_cast<int64_t>(w.cap_rows) * elems_per_record + kWireElems - 1) /
                         kWireElems;
  return dim3(static_cast<unsigned>(chunks), static_cast<unsigned>(w.W));
}

template <int LPR, typename T = uint16_t, bool ADAM = false>
__global__ __launch_bounds__(256) void shard_gather_kernel(BankArgs bank, const int32_t *__restrict__ recv,
                                                           int64_t n, int cap,
                                                           uint4 *__restrict__ out) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const int64_t j = t / LPR;
  const int l = static_cast<int>(t % LPR);
  if (j >= n) return;
  const int f = static_cast<int>((j / cap) % bank.n_tables);
  const int64_t id = recv[j];
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (id >= 0 && id < bank.rows[f]) {
    v = reinterpret_cast<const uint4 *>(bank.data)[(bank.row_offset[f] + id) * LPR + l];
    if constexpr (ADAM) {  // a lazily updated Adam bank: the row as of the last step
      constexpr int EPL = Vec<T>::EPL;
      v = adam_current<T>(bank, bank.row_offset[f] + id, l * EPL, live_elems(bank, l * EPL, EPL), v,
                          *bank.adam.d_t);
    }
  }
  out[j * LPR + l] = v;
}

struct LookupGradArgs {
  const int32_t *pos;
  const void *dx;
  int64_t dx_ld;
  int dx_bf16;
  const float *dfm;
  const float *fm_sum;
  const void *x0;
  int64_t x0_ld;
  int x0_bf16;
  const float *dw;
  float *g;
  int64_t g_ld;
  int64_t B;
  int F, D, has_w, chunks;
};

__device__ __forceinline__ float ld_elem(const void *p, int bf16, int64_t i) {
  return bf16 ? bf16_to_f32(static_cast<const uint16_t *>(p)[i]) : static_cast<const float *>(p)[i];
}

// 4 consecutive elements (4-aligned, 8/16-B aligned rows) as floats
__device__ __forceinline__ void ld4(const void *p, int bf16, int64_t i, float *v) {
  if (bf16) {
    const uint2 r = *reinterpret_cast<const uint2 *>(static_cast<const uint16_t *>(p) + i);
    v[0] = __uint_as_float(r.x << 16);
    v[1] = __uint_as_float(r.x & 0xffff0000u);
    v[2] = __uint_as_float(r.y << 16);
    v[3] = __uint_as_float(r.y & 0xffff0000u);
  } else {
    const float4 r = *reinterpret_cast<const float4 *>(static_cast<const float *>(p) + i);
    v[0] = r.x;
    v[1] = r.y;
    v[2] = r.z;
    v[3] = r.w;
  }
}

// one wave per sample; lane -> (table f, 4-float chunk c) items, so the sample's
// dx / x0 row segments are read contiguously and every 16-B gradient chunk lands
// in the row of the slot its lookup's row came from
__global__ __launch_bounds__(256) void lookup_grad_kernel(LookupGradArgs a) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= a.B) return;
  const float dfm = a.dfm ? a.dfm[b] : 0.f;
  const float dw = (a.dw && a.has_w) ? a.dw[b] : 0.f;
  const int items = a.F * a.chunks;
  for (int it = lane; it < items; it += 64) {
    const int f = it / a.chunks;
    const int c = it - f * a.chunks;
    const int32_t p = a.pos[static_cast<int64_t>(f) * a.B + b];
    if (p < 0) continue;
    float g[4] = {0.f, 0.f, 0.f, 0.f};
    const int e0 = c * 4;
    if (e0 < a.D) {  // D % 4 == 0: the chunk is all embedding elements
      const int64_t col = static_cast<int64_t>(f) * a.D + e0;
      if (a.dx) ld4(a.dx, a.dx_bf16, b * a.dx_ld + col, g);
      if (a.dfm) {
        float x[4];
        ld4(a.x0, a.x0_bf16, b * a.x0_ld + col, x);
        const float4 s = *reinterpret_cast<const float4 *>(a.fm_sum + b * a.D + e0);
        g[0] = fmaf(dfm, s.x - x[0], g[0]);
        g[1] = fmaf(dfm, s.y - x[1], g[1]);
        g[2] = fmaf(dfm, s.z - x[2], g[2]);
        g[3] = fmaf(dfm, s.w - x[3], g[3]);
      }
    } else if (e0 == a.D) {
      g[0] = dw;
    }
    *reinterpret_cast<float4 *>(a.g + static_cast<int64_t>(p) * a.g_ld + e0) =
        make_float4(g[0], g[1], g[2], g[3]);
  }
}

}  // namespace mrec

using namespace mrec;

extern "C" {

mrec_status mrec_shard_bucketize(const mrec_ids *ids, int32_t n_tables, const int64_t *rows,
                                 int64_t batch, int32_t world, int32_t cap, int32_t *send_ids,
                                 int32_t *pos, int32_t *d_overflow, int32_t *d_oob_flag,
                                 mrec_stream stream) {
  MREC_CHECK_ARG(n_tables >= 1 && n_tables <= MREC_MAX_TABLES, "n_tables out of range");
  MREC_CHECK_ARG(rows != nullptr && send_ids && pos, "NULL pointer");
  MREC_CHECK_ARG(world >= 1 && cap >= 1 && batch >= 0, "bad world / cap / batch");
  IdsArgs ia;
  mrec_status st = make_ids_args(ids, n_tables, &ia);
  if (st != MREC_OK) return st;
  const int64_t groups = (batch + kBT - 1) / kBT * kBWaves;
  MREC_CHECK_ARG((world + 1) * std::max<int64_t>(groups, 1) <= kBHist,
                 "(world + 1) * ceil(batch / 64) must be <= 2048");
  RowsArg ra;
  for (int f = 0; f < MREC_MAX_TABLES; ++f) {
    ra.v[f] = f < n_tables ? rows[f] : 0;
    MREC_CHECK_ARG(ra.v[f] >= 0 && ra.v[f] < (int64_t(1) << 31), "rows per table must be < 2^31");
  }
  bucketize_kernel<<<dim3(n_tables), kBT, 0, static_cast<hipStream_t>(stream)>>>(
      ia, ra, batch, world, cap, n_tables, send_ids, pos, d_overflow, d_oob_flag);
  return launch_status("mrec_shard_bucketize");
}

mrec_status mrec_shard_gather(const mrec_table_bank *local, const int32_t *recv_ids,
                              int32_t world, int32_t cap, void *rows_out, mrec_stream stream) {
  BankArgs ba;
  int eb, lpr;
  mrec_status st = make_bank_args(local, &ba, &eb, &lpr);
  if (st != MREC_OK) return st;
  MREC_CHECK_ARG(recv_ids && rows_out, "NULL pointer");
  MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(rows_out) & 15) == 0, "rows_out not 16B aligned");
  MREC_CHECK_ARG(world >= 1 && cap >= 1, "bad world / cap");
  const int64_t n = static_cast<int64_t>(world) * ba.n_tables * cap;
  const int64_t threads = n * lpr;
  const dim3 grid(static_cast<unsigned>((threads + 255) / 256));
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint4 *out = static_cast<uint4 *>(rows_out);
#define MREC_SGK(T, A)                                                                           \
  switch (lpr) {                                                                                 \
    case 1: shard_gather_kernel<1, T, A><<<grid, 256, 0, s>>>(ba, recv_ids, n, cap, out); break;  \
    case 2: shard_gather_kernel<2, T, A><<<grid, 256, 0, s>>>(ba, recv_ids, n, cap, out); break;  \
    case 4: shard_gather_kernel<4, T, A><<<grid, 256, 0, s>>>(ba, recv_ids, n, cap, out); break;  \
    case 8: shard_gather_kernel<8, T, A><<<grid, 256, 0, s>>>(ba, recv_ids, n, cap, out); break;  \
    default: shard_gather_kernel<16, T, A><<<grid, 256, 0, s>>>(ba, recv_ids, n, cap, out); break; \
  }
  if (!ba.adam.kind) {
    MREC_SGK(uint16_t, false)  // (T only matters to the Adam catch-up)
  } else if (local->dtype == MREC_BF16) {
    MREC_SGK(uint16_t, true)
  } else {
    MREC_SGK(float, true)
  }
#undef MREC_SGK
  return launch_status("mrec_shard_gather");
}

mrec_status mrec_shard_lookup_grad(int64_t batch, int32_t n_tables, int32_t dim, int32_t has_w,
                                   const int32_t *pos, const void *dx, mrec_dtype dx_dtype,
                                   int64_t dx_ld, const float *dfm, const float *fm_sum,
                                   const void *x0, mrec_dtype x0_dtype, int64_t x0_ld,
                                   const float *dw, float *g_out, int64_t g_ld,
                                   mrec_stream stream) {
  MREC_CHECK_ARG(batch >= 0 && n_tables >= 1 && dim >= 1 && dim % 4 == 0, "bad shape");
  MREC_CHECK_ARG(pos && g_out, "NULL pointer");
  MREC_CHECK_ARG(!dx || (reinterpret_cast<uintptr_t>(dx) & 15) == 0, "dx not 16B aligned");
  MREC_CHECK_ARG(!dfm || ((reinterpret_cast<uintptr_t>(x0) & 15) == 0 &&
                          (reinterpret_cast<uintptr_t>(fm_sum) & 15) == 0),
                 "x0 / fm_sum not 16B aligned");
  MREC_CHECK_ARG(g_ld % 4 == 0 && g_ld >= dim + (has_w ? 1 : 0) &&
                     (reinterpret_cast<uintptr_t>(g_out) & 15) == 0,
                 "g_out rows must be 16B aligned with g_ld % 4 == 0 and >= dim + has_w");
  MREC_CHECK_ARG(!dx || dx_ld >= static_cast<int64_t>(n_tables) * dim, "dx_ld too small");
  MREC_CHECK_ARG(!dfm || (fm_sum && x0 && x0_ld >= static_cast<int64_t>(n_tables) * dim),
                 "dfm needs fm_sum and x0 (x0_ld >= F*dim)");
  MREC_CHECK_ARG(!dw || has_w, "dw needs has_w");
  if (batch == 0) return MREC_OK;
  LookupGradArgs a;
  a.pos = pos;
  a.dx = dx;
  a.dx_ld = dx_ld;
  a.dx_bf16 = dx_dtype == MREC_BF16;
  a.dfm = dfm;
  a.fm_sum = fm_sum;
  a.x0 = x0;
  a.x0_ld = x0_ld;
  a.x0_bf16 = x0_dtype == MREC_BF16;
  a.dw = dw;
  a.g = g_out;
  a.g_ld = g_ld;
  a.B = batch;
  a.F = n_tables;
  a.D = dim;
  a.has_w = has_w ? 1 : 0;
  a.chunks = (dim + a.has_w + 3) / 4;
  lookup_grad_kernel<<<dim3(static_cast<unsigned>((batch + 3) / 4)), 256, 0,
                       static_cast<hipStream_t>(stream)>>>(a);
  return launch_status("mrec_shard_lookup_grad");
}


// ---- compact exchange (ABI 19) ----------------------------------------------

static mrec_status bucketize_dedup_launch(const mrec_ids *ids, int32_t n_tables,
                                          const int64_t *rows, int64_t batch, int32_t world,
                                          int32_t cap, int64_t chunk_batch, int32_t quarters,
                                          void *scratch, int32_t *send_ids, int32_t *pos,
                                          int32_t *d_overflow, int32_t *d_oob_flag,
                                          mrec_stream stream);

static int64_t dedup_chunks(int64_t batch, int64_t chunk_batch) {
  return batch > 0 ? (batch + chunk_batch - 1) / chunk_batch : 1;
}

size_t mrec_shard_dedup_scratch_bytes(int32_t n_tables, int64_t chunks, int32_t world,
                                      int32_t quarters) {
  if (n_tables < 1 || chunks < 1 || world < 1 || quarters < 1) return 0;
  const int64_t arrive = (chunks * n_tables * 8 + 255) / 256 * 256;
  return static_cast<size_t>(arrive + chunks * n_tables * quarters * world * 4);
}

mrec_status mrec_shard_bucketize_dedup_q(const mrec_ids *ids, int32_t n_tables,
                                         const int64_t *rows, int64_t batch, int32_t world,
                                         int32_t cap, int64_t chunk_batch, int32_t quarters,
                                         void *scratch, size_t scratch_bytes, int32_t *send_ids,
                                         int32_t *pos, int32_t *d_overflow, int32_t *d_oob_flag,
                                         mrec_stream stream) {
  MREC_CHECK_ARG(quarters >= 1 && quarters <= 16 && (quarters & (quarters - 1)) == 0,
                 "quarters must be a power of two in [1, 16]");
  MREC_CHECK_ARG(world <= kDedupMaxW, "world too large for the dedup bucketize");
  const int64_t C = dedup_chunks(batch, std::max<int64_t>(chunk_batch, 1));
  if (quarters > 1) {
    MREC_CHECK_ARG(scratch != nullptr && (reinterpret_cast<uintptr_t>(scratch) & 7) == 0 &&
                       scratch_bytes >= mrec_shard_dedup_scratch_bytes(n_tables, C, world, quarters),
                   "quarters > 1 need mrec_shard_dedup_scratch_bytes of zeroed scratch");
  }
  return bucketize_dedup_launch(ids, n_tables, rows, batch, world, cap, chunk_batch, quarters,
                                scratch, send_ids, pos, d_overflow, d_oob_flag, stream);
}

mrec_status mrec_shard_bucketize_dedup_ex(const mrec_ids *ids, int32_t n_tables,
                                          const int64_t *rows, int64_t batch, int32_t world,
                                          int32_t cap, int64_t chunk_batch, int32_t *send_ids,
                                          int32_t *pos, int32_t *d_overflow, int32_t *d_oob_flag,
                                          mrec_stream stream) {
  return bucketize_dedup_launch(ids, n_tables, rows, batch, world, cap, chunk_batch, 1, nullptr,
                                send_ids, pos, d_overflow, d_oob_flag, stream);
}

static mrec_status bucketize_dedup_launch(const mrec_ids *ids, int32_t n_tables,
                                          const int64_t *rows, int64_t batch, int32_t world,
                                          int32_t cap, int64_t chunk_batch, int32_t quarters,
                                          void *scratch, int32_t *send_ids, int32_t *pos,
                                          int32_t *d_overflow, int32_t *d_oob_flag,
                                          mrec_stream stream) {
  MREC_CHECK_ARG(n_tables >= 1 && n_tables <= MREC_MAX_TABLES, "n_tables out of range");
  MREC_CHECK_ARG(rows != nullptr && send_ids && pos, "NULL pointer");
  MREC_CHECK_ARG(world >= 1 && cap >= 1 && cap < 65535 && batch >= 0,
                 "bad world / cap / batch (cap < 65535)");
  MREC_CHECK_ARG(chunk_batch >= 1 && chunk_batch <= 8192, "chunk_batch must be in [1, 8192]");
  const int64_t C = batch > 0 ? (batch + chunk_batch - 1) / chunk_batch : 1;
  MREC_CHECK_ARG(C <= 65535 && batch * n_tables < (int64_t(1) << 31) &&
                     int64_t(world) * C * n_tables * cap < (int64_t(1) << 31),
                 "batch / chunks too large for int32 slots");
  IdsArgs ia;
  mrec_status st = make_ids_args(ids, n_tables, &ia);
  if (st != MREC_OK) return st;
  const int64_t cb = std::min<int64_t>(chunk_batch, std::max<int64_t>(batch, 1));
  const int64_t groups = (cb + kBT - 1) / kBT * kBWaves;
  MREC_CHECK_ARG((world + 1) * std::max<int64_t>(groups, 1) <= kBHist,
                 "(world + 1) * ceil(chunk_batch / 64) must be <= 2048");
  RowsArg ra;
  for (int f = 0; f < MREC_MAX_TABLES; ++f) {
    ra.v[f] = f < n_tables ? rows[f] : 0;
    MREC_CHECK_ARG(ra.v[f] >= 0 && ra.v[f] < (int64_t(1) << 31), "rows per table must be < 2^31");
  }
  int hs = 1024;
  while (hs < 2 * cb) hs *= 2;  // load factor <= 1/2
  const size_t lds = static_cast<size_t>(hs) * 8;
  static int attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(bucketize_dedup_kernel<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 16384 * 8);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(bucketize_dedup_kernel<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 16384 * 8);
    (void)hipGetLastError();
    return 1;
  }();
  (void)attr;
  const KClock kc = kclock_take();
  int lgH = 0;
  while ((1 << lgH) < quarters) ++lgH;
  unsigned long long *arrive = static_cast<unsigned long long *>(scratch);
  int32_t *qcnt = scratch ? reinterpret_cast<int32_t *>(static_cast<char *>(scratch) +
                                                        (C * n_tables * 8 + 255) / 256 * 256)
                          : nullptr;
  const int spin_bound = 1 << 22;  // ~0.1 s of sleeps: then the overflow word's bit 2
  const dim3 grid(static_cast<unsigned>(n_tables) << lgH, static_cast<unsigned>(C));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (kc.buf)
    bucketize_dedup_kernel<true><<<grid, kBT, lds, s>>>(ia, ra, batch, world, cap, n_tables, hs,
                                                        send_ids, pos, d_overflow, d_oob_flag,
                                                        static_cast<int>(C), cb, lgH, qcnt, arrive,
                                                        spin_bound, kc);
  else
    bucketize_dedup_kernel<false><<<grid, kBT, lds, s>>>(ia, ra, batch, world, cap, n_tables, hs,
                                                         send_ids, pos, d_overflow, d_oob_flag,
                                                         static_cast<int>(C), cb, lgH, qcnt, arrive,
                                                         spin_bound, kc);
  return launch_status("mrec_shard_bucketize_dedup");
}

mrec_status mrec_shard_bucketize_dedup(const mrec_ids *ids, int32_t n_tables, const int64_t *rows,
                                       int64_t batch, int32_t world, int32_t cap,
                                       int32_t *send_ids, int32_t *pos, int32_t *d_overflow,
                                       int32_t *d_oob_flag, mrec_stream stream) {
  MREC_CHECK_ARG(batch >= 0 && batch <= 8192, "batch must be <= 8192 (mrec_shard_bucketize_dedup_ex "
                                              "takes larger batches in chunks)");
  return mrec_shard_bucketize_dedup_ex(ids, n_tables, rows, batch, world, cap,
                                       std::max<int64_t>(batch, 1), send_ids, pos, d_overflow,
                                       d_oob_flag, stream);
}

int32_t mrec_shard_wire_bytes(int32_t dim, int32_t has_w, mrec_dtype dtype) {
  const int es = dtype == MREC_BF16 ? 2 : 4;
  return ((dim + (has_w ? 1 : 0)) * es + 3) / 4 * 4;
}

static mrec_status wire_args(const int32_t *hdr, int32_t world, int32_t n_tables, int32_t cap,
                             int32_t cap_rows, int32_t rec_bytes, int32_t *d_overflow,
                             WireArgs *w) {
  MREC_CHECK_ARG(hdr != nullptr, "NULL header ids");
  MREC_CHECK_ARG(world >= 1 && n_tables >= 1 && n_tables <= MREC_MAX_TABLES && cap >= 1 &&
                     cap_rows >= 1, "bad world / tables / cap");
  MREC_CHECK_ARG(rec_bytes % 4 == 0 && rec_bytes >= 4 && rec_bytes <= 72,
                 "record bytes must be a multiple of 4 in [4, 72]");
  // the wire kernels index a part's elements (records x <= 64 dwords) in 32 bits
  MREC_CHECK_ARG(static_cast<int64_t>(cap_rows) * 64 < (int64_t(1) << 31), "cap_rows too large");
  w->hdr = hdr;
  w->W = world;
  w->F = n_tables;
  w->cap = cap;
  w->cap_rows = cap_rows;
  w->rec_dw = rec_bytes / 4;
  w->overflow = d_overflow;
  w->pref = nullptr;
  return MREC_OK;
}

mrec_status mrec_shard_gather_wire(const mrec_table_bank *local, const int32_t *recv_ids,
                                   int32_t world, int32_t cap, int32_t cap_rows, void *wire,
                                   int32_t *d_overflow, const mrec_plan_job *plan,
                                   mrec_stream stream) {
  return mrec_shard_gather_wire_ex(local, recv_ids, world, cap, cap_rows, wire, nullptr, d_overflow,
                                   plan, stream);
}

mrec_status mrec_shard_gather_wire_ex(const mrec_table_bank *local, const int32_t *recv_ids,
                                      int32_t world, int32_t cap, int32_t cap_rows, void *wire,
                                      int32_t *pref, int32_t *d_overflow,
                                      const mrec_plan_job *plan, mrec_stream stream) {
  BankArgs ba;
  int eb, lpr;
  mrec_status st = make_bank_args(local, &ba, &eb, &lpr);
  if (st != MREC_OK) return st;
  MREC_CHECK_ARG(recv_ids && wire, "NULL pointer");
  MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(wire) & 3) == 0, "wire not 4-B aligned");
  const int rec = mrec_shard_wire_bytes(ba.dim, ba.has_w, local->dtype);
  MREC_CHECK_ARG(rec <= ba.row_stride * eb, "record wider than the bank row");
  WireArgs w;
  st = wire_args(recv_ids, world, ba.n_tables, cap, cap_rows, rec, d_overflow, &w);
  if (st != MREC_OK) return st;
  w.pref = pref;
  const dim3 g = wire_grid(w, w.rec_dw);
  const int chunks = static_cast<int>(g.x);
  PlanJob job{};
  int pb = 0;
  if (plan) {
    if ((st = build_plan_job(plan, &job)) != MREC_OK) return st;
    pb = job.bank.n_tables * kPlanBuckets;
  }
  const dim3 gf(static_cast<unsigned>(pb + chunks * world));
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint32_t *wd = static_cast<uint32_t *>(wire);
  const KClock kc = kclock_take();
#define MREC_GW(P, T, A)                                                                          \
  do {                                                                                            \
    if (kc.buf)                                                                                   \
      gather_wire_kernel<P, T, A, true><<<gf, kWireThreads, 0, s>>>(ba, w, recv_ids, wd, chunks,  \
                                                                    job, pb, kc);                 \
    else                                                                                          \
      gather_wire_kernel<P, T, A, false><<<gf, kWireThreads, 0, s>>>(ba, w, recv_ids, wd, chunks, \
                                                                     job, pb, kc);                \
  } while (0)
  if (!ba.adam.kind) {
    if (plan)
      MREC_GW(true, uint16_t, false);
    else
      MREC_GW(false, uint16_t, false);
  } else if (local->dtype == MREC_BF16) {  // a lazily updated Adam bank
    if (plan)
      MREC_GW(true, uint16_t, true);
    else
      MREC_GW(false, uint16_t, true);
  } else {
    if (plan)
      MREC_GW(true, float, true);
    else
      MREC_GW(false, float, true);
  }
#undef MREC_GW
  return launch_status("mrec_shard_gather_wire");
}

mrec_status mrec_shard_wire_unpack(const void *wire, int32_t rec_bytes, const int32_t *hdr_ids,
                                   int32_t world, int32_t n_tables, int32_t cap, int32_t cap_rows,
                                   void *slots, int64_t slot_bytes, int32_t to_f32, void *zero,
                                   int64_t zero_bytes, int32_t *d_overflow, mrec_stream stream) {
  return mrec_shard_wire_unpack_ex(wire, rec_bytes, hdr_ids, world, n_tables, cap, cap_rows, slots,
                                   slot_bytes, to_f32, zero, zero_bytes, nullptr, d_overflow,
                                   stream);
}

mrec_status mrec_shard_wire_unpack_ex(const void *wire, int32_t rec_bytes, const int32_t *hdr_ids,
                                      int32_t world, int32_t n_tables, int32_t cap,
                                      int32_t cap_rows, void *slots, int64_t slot_bytes,
                                      int32_t to_f32, void *zero, int64_t zero_bytes,
                                      int32_t *pref, int32_t *d_overflow, mrec_stream stream) {
  WireArgs w;
  mrec_status st = wire_args(hdr_ids, world, n_tables, cap, cap_rows, rec_bytes, d_overflow, &w);
  if (st != MREC_OK) return st;
  w.pref = pref;
  MREC_CHECK_ARG(wire && slots, "NULL pointer");
  MREC_CHECK_ARG(slot_bytes % 4 == 0 && zero_bytes % 4 == 0 && zero_bytes >= 0,
                 "row pitches must be multiples of 4 bytes");
  MREC_CHECK_ARG(slot_bytes >= (to_f32 ? 2 : 1) * rec_bytes, "slot rows narrower than the record");
  MREC_CHECK_ARG(slot_bytes <= 256 && zero_bytes <= 256, "slot / zero rows wider than 256 B");
  MREC_CHECK_ARG(!zero || zero_bytes > 0, "zero rows need their pitch");
  const int slot_dw = static_cast<int>(slot_bytes / 4), zero_dw = static_cast<int>(zero_bytes / 4);
  const dim3 g = wire_grid(w, std::max(slot_dw, zero ? zero_dw : 0));
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint32_t *wp = static_cast<uint32_t *>(const_cast<void *>(wire));
  const KClock kc = to_f32 ? KClock{nullptr, 0} : kclock_take();  // (the slot exchange: unclocked)
  uint32_t *sl = static_cast<uint32_t *>(slots), *zr = static_cast<uint32_t *>(zero);
  if (to_f32)
    wire_move_kernel<true, true><<<g, kWireThreads, 0, s>>>(w, wp, sl, slot_dw, zr, zero_dw, kc);
  else if (kc.buf)
    wire_move_kernel<true, false, true><<<g, kWireThreads, 0, s>>>(w, wp, sl, slot_dw, zr, zero_dw, kc);
  else
    wire_move_kernel<true, false><<<g, kWireThreads, 0, s>>>(w, wp, sl, slot_dw, zr, zero_dw, kc);
  return launch_status("mrec_shard_wire_unpack");
}

mrec_status mrec_shard_wire_pack(const void *slots, int64_t slot_bytes, int32_t rec_bytes,
                                 const int32_t *hdr_ids, int32_t world, int32_t n_tables,
                                 int32_t cap, int32_t cap_rows, void *wire, int32_t *d_overflow,
                                 mrec_stream stream) {
  WireArgs w;
  mrec_status st = wire_args(hdr_ids, world, n_tables, cap, cap_rows, rec_bytes, d_overflow, &w);
  if (st != MREC_OK) return st;
  MREC_CHECK_ARG(wire && slots, "NULL pointer");
  MREC_CHECK_ARG(slot_bytes % 4 == 0 && slot_bytes >= rec_bytes, "bad slot pitch");
  wire_move_kernel<false, false><<<wire_grid(w, w.rec_dw), kWireThreads, 0,
                                   static_cast<hipStream_t>(stream)>>>(
      w, static_cast<uint32_t *>(wire), static_cast<uint32_t *>(const_cast<void *>(slots)),
      static_cast<int>(slot_bytes / 4), nullptr, 0, KClock{nullptr, 0});
  return launch_status("mrec_shard_wire_pack");
}

}  // extern "C"
