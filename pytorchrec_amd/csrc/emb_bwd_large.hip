// Embedding backward for batches beyond one plan workgroup (> MREC_BWD_MAX_BATCH
// lookups per table, e.g. DIN's B x L history lookups): a device-wide counting
// sort by row, then one update per row.  Replaces the autograd of nn.Embedding
// (aten::embedding_dense_backward) at these sizes, with the
// same guarantees as the batched path: every row is updated ONCE with the sum of
// all its lookups' gradients, and results are bitwise reproducible.
//
// plan  (5 launches): memset counts -> count (atomic per-row histogram) ->
//       blocksum -> scan (segment starts, ascending unique-row list, long-segment
//       work list) -> place (lookup indices into their row's segment; the order
//       inside a segment follows the atomics, so it is NOT used for arithmetic).
//       Batches of <= 4M lookups take the BUCKETED plan instead (4 launches, a
//       handful of global atomics per workgroup): lookups are partitioned into NB
//       buckets by a hash of their row (so hot rows and small tables spread over
//       all buckets), then one workgroup per bucket groups its rows in an LDS hash
//       table and emits the same segment lists (see bk_hist_kernel).
// apply (3 launches): a segment of <= 16 lookups is sorted by a register network
//       and summed in ascending sample order (identical arithmetic to the batched
//       path).  A longer (hot) segment is split into chunks summed in parallel in
//       FIXED POINT: each gradient element is scaled by 2^S (S from the segment's
//       max |g| and length, so the sum cannot overflow int64) and the int64
//       partials are added with atomics — integer addition is associative, so the
//       result does not depend on the order, and it is exact up to the one
//       rounding of each term to 2^-S (relative 2^-45 of the largest term).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "emb_apply.h"
#include "gemm_common.h"

namespace mrec {

constexpr int kLgRowsPerBlock = 4096;  // scan block: 256 threads x 16 rows
constexpr int kLgChunk = 2048;         // lookups per long-segment work item
constexpr int kLgShort = 16;           // segments up to this: register sort
constexpr int kLgHuge = kLgChunk;      // longer: chunked fixed-point kernels (else one wave)
constexpr int64_t kLgMaxRows = int64_t(1) << 24;
// the workspace header's sticky error word (never cleared by a kernel; the host reads
// and clears it, mrec_emb_bwd_large_error_offset): 1 a huge-segment phase wait ran
// out, 2 a bucket's distinct rows overflowed its LDS hash
constexpr int kLgErrWord = 8;
constexpr int kLgApplyBlocks = 2048;   // grid-stride launches (device-side counts)

// workspace layout (all offsets 256-B aligned)
struct LgWs {
  int32_t *hdr;     // [16]: 0 unique rows, 1 long segments, 2 chunks, 3 huge segments,
                    // 4-6 lg_huge_kernel's queue / done counters ([0..7] zeroed per
                    // call), 8 sticky error word (kLgErrWord: host-cleared)
  int32_t *cnt;     // [R]
  int32_t *start;   // [R]
  int32_t *blk;     // [2 * nblk]: per scan block (lookups, nonzero rows)
  int32_t *uniq;    // [U] global row (ascending)
  int32_t *ustart;  // [U]
  int32_t *ulen;    // [U]
  int32_t *ulong;   // [U] long-segment index or -1
  int32_t *perm;    // [N] lookup index b (table implied by the row)
  int32_t *longs;   // [U] unique index of long segment L
  int2 *chunks;     // [C] (L, chunk)
  uint32_t *segmax; // [U] max |g| bits of long segment L (zero on entry, left zero)
  long long *acc;   // [U * stride] fixed-point sums (zero on entry, left zero)
  int32_t *bhist;   // bucketed plan: [G][NB] lookups per (chunk, bucket), then their offsets
  int32_t *btot;    // bucketed plan: [NB] lookups per bucket (zero on entry, left zero)
  int32_t *bcur;    // bucketed plan: [NB] next chunk offset inside the bucket (ditto)
  int2 *ent;        // bucketed plan: [N] (row, b) grouped by bucket
};

// bucketed plan geometry: NB buckets (a power of two, ~256 lookups each), G chunks
// of kBkChunk lookups, one 1024-thread workgroup each
constexpr int kBkThreads = 1024;
#ifndef MREC_BK_PER
#define MREC_BK_PER 4
#endif
constexpr int kBkPer = MREC_BK_PER;  // lookups per thread of the chunk kernels
constexpr int64_t kBkChunk = kBkThreads * kBkPer;
constexpr int kBkMaxNB = 8192;
constexpr int64_t kBkMaxN = int64_t(kBkMaxNB) * 256;  // <= 2M lookups
constexpr int kBkSlotBits = 11;
constexpr int kBkSlots = 1 << kBkSlotBits;  // LDS hash slots per bucket workgroup

#ifndef MREC_BK_PER_BUCKET
#define MREC_BK_PER_BUCKET 1024
#endif
constexpr int kBkPerBucket = MREC_BK_PER_BUCKET;  // lookups per bucket (power of two)

__host__ __device__ inline int bk_buckets(int64_t N) {
  int nb = 64;
  while (nb < kBkMaxNB && int64_t(nb) * kBkPerBucket < N) nb *= 2;
  return nb;
}
// chunks of the bucketed plan, 0 = the atomic plan.  The row hash spreads the R
// consecutive global rows evenly over the buckets (Fibonacci hashing), so with R
// <= NB * kBkSlots / 2 no bucket's LDS hash can fill up.  Banks past kLgMaxRows rows
// (the row-sharded owner's shard of 100M-row tables) have no atomic plan (its
// per-row arrays would be GBs) and always take the bucketed one: a bucket holds at
// most its lookups' distinct rows (~N / NB = 128-256 on average), and a bucket whose
// distinct rows do not fit its LDS hash sets the sticky error word, never silently.
__host__ __device__ inline int bk_groups(int64_t R, int64_t N) {
  if (N <= 0 || N > kBkMaxN) return 0;
  if (R <= kLgMaxRows && R > int64_t(bk_buckets(N)) * (kBkSlots / 2)) return 0;
  return static_cast<int>((N + kBkChunk - 1) / kBkChunk);
}

__host__ __device__ inline int64_t lg_align(int64_t x) { return (x + 255) & ~int64_t(255); }

// list capacities: U unique rows (the atomic plan: min(R, N) compact; the bucketed
// plan: N, bucket k's rows at its entry range), UL long-segment slots (bucketed:
// ceil(lo_k / 2049) + j for bucket k, disjoint because a long segment has > 2048
// lookups), C chunk slots (bucketed: ceil(lo_k / 2049) + ceil(lo_k / 2048) + j)
struct LgCaps {
  int64_t U, UL, C;
};
__host__ __device__ inline LgCaps lg_caps(int64_t R, int64_t N) {
  const int64_t u = R < N ? R : N;
  LgCaps c{u, u, N / kLgChunk + u + 1};
  if (bk_groups(R, N) > 0) {
    const int64_t ul = (N + kLgHuge) / (kLgHuge + 1) + 1;
    const int64_t cc = ul + (N + kLgChunk - 1) / kLgChunk + 2;
    c.U = N;
    c.UL = ul > c.UL ? ul : c.UL;
    c.C = cc > c.C ? cc : c.C;
  }
  return c;
}

__host__ __device__ inline int64_t lg_ws_bytes(int64_t R, int64_t N, int stride, LgWs *w,
                                               char *base) {
  const int64_t nblk = (R + kLgRowsPerBlock - 1) / kLgRowsPerBlock;
  const LgCaps cp = lg_caps(R, N);
  const int64_t U = cp.U, UL = cp.UL, C = cp.C;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    const int64_t at = o;
    o = lg_align(o + bytes);
    return at;
  };
  const int G = bk_groups(R, N), NB = bk_buckets(N);
  const int64_t o_hdr = take(64), o_bcnt = take(G ? 8 * NB : 0), o_segmax = take(4 * UL), o_acc = take(8 * UL * stride);
  const int64_t Ra = R <= kLgMaxRows ? R : 0;  // the atomic plan's per-row arrays
  const int64_t o_cnt = take(4 * Ra), o_start = take(4 * Ra), o_blk = take(8 * (Ra ? nblk : 0));
  const int64_t o_uniq = take(4 * U), o_ustart = take(4 * U), o_ulen = take(4 * U);
  const int64_t o_ulong = take(4 * U), o_perm = take(4 * N), o_longs = take(4 * UL);
  const int64_t o_chunks = take(8 * C);
  const int64_t o_bhist = take(G ? 4 * (int64_t(G + 1) * NB + 1) : 0);
  const int64_t o_ent = take(G ? 8 * N : 0);
  if (w) {
    w->bhist = G ? reinterpret_cast<int32_t *>(base + o_bhist) : nullptr;
    w->btot = G ? reinterpret_cast<int32_t *>(base + o_bcnt) : nullptr;
    w->bcur = G ? w->btot + NB : nullptr;
    w->ent = G ? reinterpret_cast<int2 *>(base + o_ent) : nullptr;
    w->hdr = reinterpret_cast<int32_t *>(base + o_hdr);
    w->segmax = reinterpret_cast<uint32_t *>(base + o_segmax);
    w->acc = reinterpret_cast<long long *>(base + o_acc);
    w->cnt = reinterpret_cast<int32_t *>(base + o_cnt);
    w->start = reinterpret_cast<int32_t *>(base + o_start);
    w->blk = reinterpret_cast<int32_t *>(base + o_blk);
    w->uniq = reinterpret_cast<int32_t *>(base + o_uniq);
    w->ustart = reinterpret_cast<int32_t *>(base + o_ustart);
    w->ulen = reinterpret_cast<int32_t *>(base + o_ulen);
    w->ulong = reinterpret_cast<int32_t *>(base + o_ulong);
    w->perm = reinterpret_cast<int32_t *>(base + o_perm);
    w->longs = reinterpret_cast<int32_t *>(base + o_longs);
    w->chunks = reinterpret_cast<int2 *>(base + o_chunks);
  }
  return o;
}

// bytes that must be zero before the first call (every apply leaves them zero)
__host__ inline int64_t lg_zero_bytes(int64_t R, int64_t N, int stride) {
  const int64_t UL = lg_caps(R, N).UL;
  const int64_t bcnt = bk_groups(R, N) ? lg_align(8 * bk_buckets(N)) : 0;
  return lg_align(32) + bcnt + lg_align(4 * UL) + lg_align(8 * UL * stride);
}

__device__ __forceinline__ int table_of_row(const BankArgs &bank, int64_t grow) {
  int f = 0;
  while (f + 1 < bank.n_tables && bank.row_offset[f + 1] <= grow) ++f;
  return f;
}

// ---- plan -------------------------------------------------------------------
// A wave's 64 lanes hold 64 consecutive lookups.  Equal rows in consecutive lanes
// (a DIN history's PAD tail, Zipf repeats) form a run that takes ONE atomic for
// the whole run: a hot row would otherwise serialise ~10^5 atomics on one L2
// address (measured 1.5 ms per call at C4).
struct Run {
  int32_t r;     // global row, -1 = invalid / padding
  int head;      // lane of the first lookup of this lane's run
  int len;       // run length (valid at the head)
};

__device__ __forceinline__ Run lane_run(int32_t r) {
  const int lane = threadIdx.x & 63;
  const int32_t prev = __shfl_up(r, 1);
  const bool change = lane == 0 || prev != r;
  const uint64_t changes = __ballot(change);
  const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
  Run out;
  out.r = r;
  out.head = 63 - __clzll(changes & upto);
  const uint64_t after = lane == 63 ? 0ull : (changes & ~upto);
  out.len = (after ? __ffsll(static_cast<unsigned long long>(after)) - 1 : 64) - lane;
  return out;
}

// The rows of the N lookups i_k = i0 + k * step of a thread (lookup i: table
// i / n, sample i % n; -1 for an invalid id or i >= total), every load issued
// before any is used (common.h load_ids_batch): the per-lane kernel-argument reads
// (ids.ptr[f], rows[f], row_offset[f]) first, then the ids, unconditionally from
// clamped indices.  As N calls of a one-lookup helper the compiler chained ~4
// dependent round trips per lookup (each loaded value copied out of its branch
// waits for it).
// b_out[k] = the lookup's sample (0 past `total`).
template <int N>
__device__ __forceinline__ void lookup_rows_batch(const BankArgs &bank, const IdsArgs &ids,
                                                  int64_t n, int64_t i0, int64_t step, int64_t total,
                                                  int32_t (&row)[N], int64_t (&b_out)[N],
                                                  int32_t *__restrict__ oob) {
  // (total = batch * n_tables < 2^31, checked by lg_setup: 32-bit division)
  const uint32_t un = static_cast<uint32_t>(n);
  int fk[N];
  const void *fp[N];
  int64_t nrow[N], roff[N], id[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const int64_t i = i0 + k * step;
    const uint32_t ui = static_cast<uint32_t>(i < total ? i : 0);
    fk[k] = static_cast<int>(ui / un);
    b_out[k] = static_cast<int64_t>(ui - static_cast<uint32_t>(fk[k]) * un);
  }
  __builtin_amdgcn_sched_barrier(0);  // the index math first: no register reuse waits
#pragma unroll
  for (int k = 0; k < N; ++k) {
    fp[k] = ids.ptr[fk[k]];
    nrow[k] = bank.rows[fk[k]];
    roff[k] = bank.row_offset[fk[k]];
  }
  if (ids.chunk) {  // (uniform) chunked views: the per-element path
#pragma unroll
    for (int k = 0; k < N; ++k) id[k] = load_id(ids, fk[k], b_out[k]);
  } else if (ids.is64) {
#pragma unroll
    for (int k = 0; k < N; ++k) id[k] = static_cast<const int64_t *>(fp[k])[b_out[k] * ids.stride];
  } else {
#pragma unroll
    for (int k = 0; k < N; ++k) id[k] = static_cast<const int32_t *>(fp[k])[b_out[k] * ids.stride];
  }
#pragma unroll
  for (int k = 0; k < N; ++k) {
    row[k] = -1;
    if (i0 + k * step >= total) continue;
    if (id[k] >= 0 && id[k] < nrow[k])
      row[k] = static_cast<int32_t>(roff[k] + id[k]);
    else if (oob && !(ids.pad_negative && id[k] < 0))
      *oob = 1;
  }
}

// Runs are further combined per workgroup in an LDS hash (a row's runs from
// different samples, e.g. one PAD run per history): a workgroup covers
// kLgIter * 256 consecutive lookups and pays ONE global atomic per distinct row
// it holds in LDS; a run whose row finds no LDS slot within kLgProbe probes goes
// to global memory directly.
constexpr int kLgIter = 8;
constexpr int kLgSlots = 2048;
constexpr int kLgProbe = 8;
constexpr uint32_t kLgEmpty = 0xffffffffu;

__device__ __forceinline__ int lg_slot(uint32_t *key, int32_t r) {
  uint32_t h = (static_cast<uint32_t>(r) * 2654435761u) >> 21;  // 11 bits
  for (int p = 0; p < kLgProbe; ++p) {
    const uint32_t old = atomicCAS(&key[h], kLgEmpty, static_cast<uint32_t>(r));
    if (old == kLgEmpty || old == static_cast<uint32_t>(r)) return static_cast<int>(h);
    h = (h + 1) & (kLgSlots - 1);
  }
  return -1;
}

__global__ __launch_bounds__(256) void lg_count_kernel(BankArgs bank, IdsArgs ids, int64_t n,
                                                       LgWs w, int32_t *__restrict__ oob) {
  __shared__ uint32_t key[kLgSlots];
  __shared__ int32_t val[kLgSlots];
  if (blockIdx.x == 0 && threadIdx.x < 8) w.hdr[threadIdx.x] = 0;
  for (int i = threadIdx.x; i < kLgSlots; i += 256) {
    key[i] = kLgEmpty;
    val[i] = 0;
  }
  __syncthreads();
  const int64_t total = n * bank.n_tables;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * 256 * kLgIter;
  // every id load of this thread first (one memory round trip, not kLgIter)
  int32_t rr[kLgIter];
  {
    int64_t bq[kLgIter];
    lookup_rows_batch<kLgIter>(bank, ids, n, base + threadIdx.x, 256, total, rr, bq, oob);
  }
#pragma unroll
  for (int it = 0; it < kLgIter; ++it) {
    const Run u = lane_run(rr[it]);
    if (u.r >= 0 && u.head == (threadIdx.x & 63)) {
      const int h = lg_slot(key, u.r);
      if (h >= 0)
        atomicAdd(&val[h], u.len);
      else
        atomicAdd(&w.cnt[u.r], u.len);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kLgSlots; i += 256)
    if (key[i] != kLgEmpty) atomicAdd(&w.cnt[key[i]], val[i]);
}

// block reduce of two int32 values (256 threads), result valid in thread 0
__device__ __forceinline__ int2 block_sum2(int a, int b, int2 *red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off);
    b += __shfl_xor(b, off);
  }
  if (lane == 0) red[wid] = make_int2(a, b);
  __syncthreads();
  int2 s = make_int2(0, 0);
  if (threadIdx.x == 0)
    for (int k = 0; k < 4; ++k) {
      s.x += red[k].x;
      s.y += red[k].y;
    }
  return s;
}

__global__ __launch_bounds__(256) void lg_blocksum_kernel(int64_t R, LgWs w) {
  __shared__ int2 red[4];
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kLgRowsPerBlock + threadIdx.x * 16;
  int s = 0, nz = 0;
  for (int j = 0; j < 16; ++j) {
    const int c = r0 + j < R ? w.cnt[r0 + j] : 0;
    s += c;
    nz += c > 0;
  }
  const int2 t = block_sum2(s, nz, red);
  if (threadIdx.x == 0) {
    w.blk[2 * blockIdx.x] = t.x;
    w.blk[2 * blockIdx.x + 1] = t.y;
  }
}

template <int RPT>
__global__ __launch_bounds__(256) void lg_scan_kernel(int64_t R, int nblk, LgWs w) {
  __shared__ int2 red[4];
  __shared__ int2 wex[4];
  __shared__ int2 base;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // prefix of the earlier blocks
  int ps = 0, pn = 0;
  for (int k = tid; k < static_cast<int>(blockIdx.x); k += 256) {
    ps += w.blk[2 * k];
    pn += w.blk[2 * k + 1];
  }
  const int2 p = block_sum2(ps, pn, red);
  if (tid == 0) base = p;
  __syncthreads();
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * (256 * RPT) + tid * RPT;
  int c[RPT];
  int s = 0, nz = 0;
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    c[j] = r0 + j < R ? w.cnt[r0 + j] : 0;
    s += c[j];
    nz += c[j] > 0;
  }
  // exclusive scan over threads of (s, nz)
  int is = s, in = nz;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int ts = __shfl_up(is, off), tn = __shfl_up(in, off);
    if (lane >= off) {
      is += ts;
      in += tn;
    }
  }
  if (lane == 63) wex[wid] = make_int2(is, in);
  __syncthreads();
  int es = base.x + is - s, en = base.y + in - nz;
  for (int k = 0; k < wid; ++k) {
    es += wex[k].x;
    en += wex[k].y;
  }
  // long segments and their chunks: one reservation per wave (a per-row atomic on
  // the two list counters serialised ~10^3 atomics on one address at C4)
  int nl = 0, nc = 0;
#pragma unroll
  for (int j = 0; j < RPT; ++j)
    if (c[j] > kLgHuge) {
      ++nl;
      nc += (c[j] + kLgChunk - 1) / kLgChunk;
    }
  int il = nl, ic = nc;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int tl = __shfl_up(il, off), tc = __shfl_up(ic, off);
    if (lane >= off) {
      il += tl;
      ic += tc;
    }
  }
  int bl = 0, bc = 0;
  if (lane == 63 && il > 0) {
    bl = atomicAdd(&w.hdr[1], il);
    bc = atomicAdd(&w.hdr[2], ic);
  }
  int L = __shfl(bl, 63) + il - nl;
  int cb = __shfl(bc, 63) + ic - nc;
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int64_t r = r0 + j;
    if (r >= R) break;
    w.start[r] = es;
    if (c[j] > 0) {
      w.uniq[en] = static_cast<int32_t>(r);
      w.ustart[en] = es;
      w.ulen[en] = c[j];
      int32_t myL = -1;
      if (c[j] > kLgHuge) {
        myL = L++;
        w.longs[myL] = en;
        const int nch = (c[j] + kLgChunk - 1) / kLgChunk;
        for (int k = 0; k < nch; ++k) w.chunks[cb + k] = make_int2(myL, k);
        cb += nch;
      }
      w.ulong[en] = myL;
      ++en;
    }
    es += c[j];
  }
  if (blockIdx.x == static_cast<unsigned>(nblk - 1) && tid == 255) w.hdr[0] = en;
}

// the same workgroup ranges as lg_count_kernel: runs take consecutive positions
// inside their row's LDS slot, the slot reserves its rows' positions with ONE
// global atomic, then every lookup is written to its position
__global__ __launch_bounds__(256) void lg_place_kernel(BankArgs bank, IdsArgs ids, int64_t n,
                                                       LgWs w) {
  __shared__ uint32_t key[kLgSlots];
  __shared__ int32_t val[kLgSlots];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < kLgSlots; i += 256) {
    key[i] = kLgEmpty;
    val[i] = 0;
  }
  __syncthreads();
  const int64_t total = n * bank.n_tables;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * 256 * kLgIter;
  int32_t row[kLgIter], bb[kLgIter], slot[kLgIter], off[kLgIter];
  {  // every id load first (one memory round trip)
    int64_t bq[kLgIter];
    lookup_rows_batch<kLgIter>(bank, ids, n, base + threadIdx.x, 256, total, row, bq, nullptr);
#pragma unroll
    for (int it = 0; it < kLgIter; ++it) bb[it] = static_cast<int32_t>(bq[it]);
  }
#pragma unroll
  for (int it = 0; it < kLgIter; ++it) {
    const Run u = lane_run(row[it]);
    int h = -1, k = 0;
    if (u.r >= 0 && u.head == lane) {
      h = lg_slot(key, u.r);
      if (h >= 0)
        k = atomicAdd(&val[h], u.len);  // offset inside the slot's block of positions
      else
        k = atomicSub(&w.cnt[u.r], u.len) - u.len;  // a global block of its own
    }
    h = __shfl(h, u.head);
    k = __shfl(k, u.head);
    slot[it] = h;
    off[it] = k + (lane - u.head);
  }
  __syncthreads();
  // one global reservation per slot: val becomes the slot's first position
  for (int i = threadIdx.x; i < kLgSlots; i += 256)
    if (key[i] != kLgEmpty) val[i] = atomicSub(&w.cnt[key[i]], val[i]) - val[i];
  __syncthreads();
#pragma unroll
  for (int it = 0; it < kLgIter; ++it) {
    if (row[it] < 0) continue;
    const int pos = (slot[it] >= 0 ? val[slot[it]] : 0) + off[it];
    w.perm[w.start[row[it]] + pos] = bb[it];
  }
}

// ---- bucketed plan -------------------------------------------------------------
// bucket of a row: the top bits of a multiplicative hash (rows of one table, a hot
// row's neighbours, a small table: all spread over the buckets)
__device__ __forceinline__ int bk_of(int32_t r, int lognb) {
  return static_cast<int>((static_cast<uint32_t>(r) * 2654435761u) >> (32 - lognb));
}

// chunk g: lookups [g * kBkChunk, ...) -> per-bucket counts, stored densely [g][NB]
__global__ __launch_bounds__(kBkThreads) void bk_hist_kernel(BankArgs bank, IdsArgs ids, int64_t n,
                                                             int lognb, LgWs w,
                                                             int32_t *__restrict__ oob) {
  __shared__ int32_t h[kBkMaxNB];
  const int NB = 1 << lognb;
  if (blockIdx.x == 0 && threadIdx.x < 8) w.hdr[threadIdx.x] = 0;
  for (int k = threadIdx.x; k < NB; k += kBkThreads) h[k] = 0;
  __syncthreads();
  const int64_t total = n * bank.n_tables;
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * kBkChunk + threadIdx.x;
  int32_t rr[kBkPer];
  {
    int64_t bq[kBkPer];
    lookup_rows_batch<kBkPer>(bank, ids, n, i0, kBkThreads, total, rr, bq, oob);
  }
#pragma unroll
  for (int u = 0; u < kBkPer; ++u)
    if (rr[u] >= 0) atomicAdd(&h[bk_of(rr[u], lognb)], 1);
  __syncthreads();
  int32_t *dst = w.bhist + static_cast<int64_t>(blockIdx.x) * NB;
  for (int k = threadIdx.x; k < NB; k += kBkThreads) {
    dst[k] = h[k];
    if (h[k]) atomicAdd(&w.btot[k], h[k]);  // the bucket totals (zero on entry)
  }
}

// exclusive scan of the NB bucket totals (btot) into LDS base[]; returns the sum
__device__ int bk_bucket_base(const int32_t *tot, int NB, int32_t *base, int32_t *wsum) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int KPT = kBkMaxNB / kBkThreads;  // consecutive buckets per thread
  int v[KPT], mine = 0;
#pragma unroll
  for (int q = 0; q < KPT; ++q) {
    const int k = tid * KPT + q;
    v[q] = k < NB ? tot[k] : 0;
    mine += v[q];
  }
  int incl = mine;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(incl, off);
    if (lane >= off) incl += t;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  int at = incl - mine, all = 0;
  for (int k = 0; k < kBkThreads / 64; ++k) {
    at += k < wid ? wsum[k] : 0;
    all += wsum[k];
  }
#pragma unroll
  for (int q = 0; q < KPT; ++q) {
    const int k = tid * KPT + q;
    if (k < NB) base[k] = at;
    at += v[q];
  }
  __syncthreads();
  return all;
}

// the same chunks as bk_hist_kernel: every valid lookup -> (row, b) at its
// bucket's next position (LDS cursors; the order inside a bucket is not used for
// arithmetic).  Every workgroup scans the bucket totals bk_hist_kernel summed
// (btot) itself and reserves its chunk's range in each bucket with one atomic on
// the bucket's cursor (bcur): no scan launch between the two.  Workgroup 0 also
// publishes the bucket starts in bhist's spare row G for the bucket kernels, which
// leave btot / bcur zero again.
__global__ __launch_bounds__(kBkThreads) void bk_scatter_kernel(BankArgs bank, IdsArgs ids, int64_t n,
                                                                int G, int lognb, LgWs w,
                                                                int fused) {
  __shared__ int32_t cur[kBkMaxNB];
  __shared__ int32_t wsum[kBkThreads / 64];
  const int NB = 1 << lognb;
  const int64_t total = n * bank.n_tables;
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * kBkChunk + threadIdx.x;
  // this chunk's range inside each bucket: one atomic per (chunk, bucket), issued
  // first so its round trip overlaps the id loads -- the order of the chunks inside
  // a bucket is not used for arithmetic
  constexpr int KQ = kBkMaxNB / kBkThreads;
  const int32_t *src = w.bhist + static_cast<int64_t>(blockIdx.x) * NB;
  int32_t resv[KQ];
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int k = threadIdx.x + q * kBkThreads;
    const int c = k < NB ? src[k] : 0;
    resv[q] = c ? atomicAdd(&w.bcur[k], c) : 0;
  }
  int32_t rr[kBkPer], bb[kBkPer];
  {
    int64_t bq[kBkPer];
    lookup_rows_batch<kBkPer>(bank, ids, n, i0, kBkThreads, total, rr, bq, nullptr);
#pragma unroll
    for (int u = 0; u < kBkPer; ++u) bb[u] = static_cast<int32_t>(bq[u]);
  }
  const int all = bk_bucket_base(w.btot, NB, cur, wsum);
  int32_t *pub = w.bhist + static_cast<int64_t>(G) * NB;  // spare row: bucket starts
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int k = threadIdx.x + q * kBkThreads;
    if (k >= NB) break;
    const int b0 = cur[k];
    if (blockIdx.x == 0) pub[k] = b0;
    cur[k] = b0 + resv[q];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    pub[NB] = all;
    // bucketed lists: entries with holes; the apply walks every slot (fused: only
    // the huge segments, at their long slots)
    w.hdr[0] = fused ? (all + kLgHuge) / (kLgHuge + 1) + 1 : all;
    w.hdr[2] = (all + kLgHuge) / (kLgHuge + 1) + 1 + (all + kLgChunk - 1) / kLgChunk + 2;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < kBkPer; ++u) {
    const int32_t r = rr[u];
    const int k = r >= 0 ? bk_of(r, lognb) : -1;
    const Run x = lane_run(k);  // equal buckets in consecutive lanes: one atomic
    int at = 0;
    if (x.r >= 0 && x.head == lane) at = atomicAdd(&cur[x.r], x.len);
    at = __shfl(at, x.head) + (lane - x.head);
    if (r >= 0) w.ent[at] = make_int2(r, bb[u]);
  }
}

// block-wide exclusive scan of one int per thread (256 threads); returns the total
__device__ __forceinline__ int bk_scan256(int v, int *excl, int *red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(incl, off);
    if (lane >= off) incl += t;
  }
  __syncthreads();  // red is free
  if (lane == 63) red[wid] = incl;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    base += k < wid ? red[k] : 0;
    tot += red[k];
  }
  *excl = base + incl - v;
  return tot;
}

// one workgroup per bucket: its rows in an LDS hash (kBkSlots), per-row counts ->
// segments inside the bucket's entry range [lo, hi), and the segment lists at
// slots only this bucket uses: unique rows at [lo, lo + nu) (ulen 0 marks the
// holes up to hi), huge segments (> kLgHuge lookups) at ceil(lo / 2049) + j, their
// chunks at ceil(lo / 2049) + ceil(lo / 2048) + j (x = -1 marks holes) -- no
// global atomics.
__global__ __launch_bounds__(256) void bk_group_kernel(LgWs w, int G, int lognb,
                                                       int32_t *__restrict__ err) {
  __shared__ uint32_t key[kBkSlots];
  __shared__ int32_t cnt[kBkSlots];
  __shared__ int red[4];
  constexpr int SPT = kBkSlots / 256;  // slots per thread
  const int tid = threadIdx.x, lane = tid & 63;
  const int NB = 1 << lognb;
  const int32_t *pub = w.bhist + static_cast<int64_t>(G) * NB;
  const int lo = pub[blockIdx.x], hi = pub[blockIdx.x + 1];
  if (tid == 0) {  // the scatter has used them: zero for the next call
    w.btot[blockIdx.x] = 0;
    w.bcur[blockIdx.x] = 0;
  }
  for (int k = tid; k < kBkSlots; k += 256) {
    key[k] = kLgEmpty;
    cnt[k] = 0;
  }
  __syncthreads();
  auto find = [&](int32_t r, bool insert) -> int {
    // the hash bits below the bucket's (its top lognb bits are the same for all rows)
    uint32_t hsh = ((static_cast<uint32_t>(r) * 2654435761u) << lognb) >> (32 - kBkSlotBits);
    for (int p = 0; p < kBkSlots; ++p) {
      const uint32_t k = insert ? atomicCAS(&key[hsh], kLgEmpty, static_cast<uint32_t>(r))
                                : key[hsh];
      if (k == static_cast<uint32_t>(r) || (insert && k == kLgEmpty)) return static_cast<int>(hsh);
      hsh = (hsh + 1) & (kBkSlots - 1);
    }
    return -1;
  };
  // (entries of one chunk and bucket are contiguous: a hot row comes in runs)
  for (int j0 = lo; j0 < hi; j0 += 256) {
    const int j = j0 + tid;
    const int32_t r = j < hi ? w.ent[j].x : -1;
    const Run x = lane_run(r);
    if (x.r >= 0 && x.head == lane) {
      const int s = find(x.r, true);
      if (s >= 0)
        atomicAdd(&cnt[s], x.len);
      else if (err)
        *err = 1;  // more distinct rows in one bucket than slots (excluded by bk_groups)
    }
  }
  __syncthreads();
  // per slot: segment offset, unique / long / chunk index inside the bucket
  int c[SPT], so = 0, su = 0, sl = 0, sc = 0;
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    c[q] = cnt[tid * SPT + q];
    so += c[q];
    su += c[q] > 0;
    sl += c[q] > kLgHuge;
    sc += c[q] > kLgHuge ? (c[q] + kLgChunk - 1) / kLgChunk : 0;
  }
  int eo, eu, el, ec;
  bk_scan256(so, &eo, red);
  const int nu = bk_scan256(su, &eu, red);
  bk_scan256(sl, &el, red);
  const int nc = bk_scan256(sc, &ec, red);
  const int l0 = (lo + kLgHuge) / (kLgHuge + 1);
  const int c0 = l0 + (lo + kLgChunk - 1) / kLgChunk;
  const int c1 = (hi + kLgHuge) / (kLgHuge + 1) + (hi + kLgChunk - 1) / kLgChunk;
  int u = lo + eu, L = l0 + el, cb = c0 + ec, at = lo + eo;
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    const int k = tid * SPT + q;
    if (c[q] > 0) {
      w.uniq[u] = static_cast<int32_t>(key[k]);
      w.ustart[u] = at;
      w.ulen[u] = c[q];
      int32_t myL = -1;
      if (c[q] > kLgHuge) {
        myL = L++;
        w.longs[myL] = u;
        const int nch = (c[q] + kLgChunk - 1) / kLgChunk;
        for (int t = 0; t < nch; ++t) w.chunks[cb + t] = make_int2(myL, t);
        cb += nch;
      }
      w.ulong[u] = myL;
      ++u;
    }
    cnt[k] = at;  // the slot's cursor
    at += c[q];
  }
  for (int v = lo + nu + tid; v < hi; v += 256) w.ulen[v] = 0;
  for (int v = c0 + nc + tid; v < c1; v += 256) w.chunks[v] = make_int2(-1, 0);
  if (blockIdx.x == NB - 1)  // chunk slots past the last bucket's range
    for (int v = c1 + tid; v < w.hdr[2]; v += 256) w.chunks[v] = make_int2(-1, 0);
  __syncthreads();
  for (int j0 = lo; j0 < hi; j0 += 256) {
    const int j = j0 + tid;
    const int2 e = j < hi ? w.ent[j] : make_int2(-1, 0);
    const Run x = lane_run(e.x);
    int p = 0;
    if (x.r >= 0 && x.head == lane) {
      const int s = find(x.r, false);
      p = s >= 0 ? atomicAdd(&cnt[s], x.len) : -1;
    }
    p = __shfl(p, x.head);
    if (e.x >= 0 && p >= 0) w.perm[p + (lane - x.head)] = e.y;
  }
}

// ---- apply -------------------------------------------------------------------
// pass 1 over the long segments' chunks: max |g| per segment (bits of a
// non-negative float order like the float)
template <typename T, int LPR>
__device__ __forceinline__ void lg_longmax_chunk(BankArgs bank, LgWs w, ApplyArgs a, int j) {
  constexpr int EPL = Vec<T>::EPL;
  constexpr int WPB = 256 / LPR;
  const int worker = threadIdx.x / LPR, l = threadIdx.x % LPR, e0 = l * EPL;
  const int D = bank.dim;
  const bool v_lane = e0 + EPL <= D, w_lane = bank.has_w && e0 == D;
  {
    const int2 ch = w.chunks[j];
    if (ch.x < 0) return;  // a hole (bucketed plan)
    const int u = w.longs[ch.x];
    const int f = table_of_row(bank, w.uniq[u]);
    const int s0 = w.ustart[u] + ch.y * kLgChunk;
    const int s1 = min(w.ustart[u] + w.ulen[u], s0 + kLgChunk);
    float m = 0.f;
    if (v_lane || w_lane)
      for (int i = s0 + worker; i < s1; i += WPB) {
        float g[EPL];
        lookup_grad<EPL>(a, w.perm[i], f, D, e0, v_lane, w_lane, g);
#pragma unroll
        for (int q = 0; q < EPL; ++q) m = fmaxf(m, fabsf(g[q]));
      }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    if ((threadIdx.x & 63) == 0 && m > 0.f) atomicMax(&w.segmax[ch.x], __float_as_uint(m));
  }
}

template <typename T, int LPR>
__device__ __forceinline__ void lg_longmax_body(BankArgs bank, int64_t n, LgWs w,
                                                         ApplyArgs a) {
  const int nchunks = w.hdr[2];
  for (int j = blockIdx.x; j < nchunks; j += gridDim.x) lg_longmax_chunk<T, LPR>(bank, w, a, j);
}

// fixed-point scale of long segment L: sum of len terms of |x| <= max stays < 2^62
__device__ __forceinline__ int lg_scale(float mx, int len) {
  if (!(mx > 0.f)) return 0;
  int e;
  frexpf(mx, &e);  // mx < 2^e
  int lb = 0;
  while ((1 << lb) < len) ++lb;  // len <= 2^lb
  return 61 - e - lb;            // |sum| < 2^(e + lb + S) = 2^61
}

// pass 2: fixed-point chunk sums added into the segment's int64 accumulator
// (workgroup-uniform: one chunk per call, LDS reduction with barriers)
template <typename T, int LPR>
__device__ __forceinline__ void lg_longacc_chunk(BankArgs bank, LgWs w, ApplyArgs a, int stride,
                                                 int j) {
  constexpr int EPL = Vec<T>::EPL;
  constexpr int WPB = 256 / LPR;
  __shared__ long long red[WPB][LPR * EPL];
  const int worker = threadIdx.x / LPR, l = threadIdx.x % LPR, e0 = l * EPL;
  const int D = bank.dim;
  const bool v_lane = e0 + EPL <= D, w_lane = bank.has_w && e0 == D;
  {
    const int2 ch = w.chunks[j];
    if (ch.x < 0) return;  // a hole (bucketed plan; uniform over the workgroup)
    const int u = w.longs[ch.x];
    const int f = table_of_row(bank, w.uniq[u]);
    const int s0 = w.ustart[u] + ch.y * kLgChunk;
    const int s1 = min(w.ustart[u] + w.ulen[u], s0 + kLgChunk);
    const int S = lg_scale(__uint_as_float(w.segmax[ch.x]), w.ulen[u]);
    long long acc[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) acc[q] = 0;
    if (v_lane || w_lane)
      for (int i = s0 + worker; i < s1; i += WPB) {
        float g[EPL];
        lookup_grad<EPL>(a, w.perm[i], f, D, e0, v_lane, w_lane, g);
#pragma unroll
        for (int q = 0; q < EPL; ++q) acc[q] += llrint(ldexp(static_cast<double>(g[q]), S));
      }
#pragma unroll
    for (int q = 0; q < EPL; ++q) red[worker][e0 + q] = acc[q];
    __syncthreads();
    for (int sft = WPB / 2; sft > 0; sft >>= 1) {
      if (worker < sft) {
#pragma unroll
        for (int q = 0; q < EPL; ++q) red[worker][e0 + q] += red[worker + sft][e0 + q];
      }
      __syncthreads();
    }
    if (worker == 0 && (v_lane || w_lane)) {
      long long *dst = w.acc + static_cast<int64_t>(ch.x) * stride + e0;
#pragma unroll
      for (int q = 0; q < EPL; ++q)
        atomicAdd(reinterpret_cast<unsigned long long *>(dst + q),
                  static_cast<unsigned long long>(red[0][e0 + q]));
    }
    __syncthreads();
  }
}

template <typename T, int LPR>
__device__ __forceinline__ void lg_longacc_body(BankArgs bank, int64_t n, LgWs w,
                                                         ApplyArgs a, int stride) {
  const int nchunks = w.hdr[2];
  for (int j = blockIdx.x; j < nchunks; j += gridDim.x)
    lg_longacc_chunk<T, LPR>(bank, w, a, stride, j);
}

// one update per unique row.  A wave takes 64 / LPR consecutive unique rows, one
// per worker (LPR lanes): a segment of <= 16 lookups is sorted and summed in
// ascending sample order by its worker; a segment of 17..kLgHuge lookups by the
// whole wave in fixed point (max |g| over the segment, then the int64 sum of every
// term scaled by 2^S: the arithmetic of the chunked kernels, so the same bits); a
// longer one from the chunked kernels' accumulator.
// (the unique rows [blk * WPB, (blk + 1) * WPB): wave wid takes the WPW from
// blk * WPB + wid * WPW; a.seed already advanced by the step counter)
template <typename T, int LPR>
__device__ __forceinline__ void lg_apply_block(BankArgs bank, LgWs w, ApplyArgs a, int stride,
                                               int blk) {
  constexpr int EPL = Vec<T>::EPL;
  constexpr int WPB = 256 / LPR;  // workers per workgroup
  constexpr int WPW = 64 / LPR;   // workers per wave
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wk = lane / LPR, l = lane % LPR, e0 = l * EPL;
  const int D = bank.dim;
  const bool v_lane = e0 + EPL <= D, w_lane = bank.has_w && e0 == D;
  const bool live = v_lane || w_lane;
  const int nu = w.hdr[0];
  {
    const int u0 = blk * WPB + wid * WPW;
    if (u0 >= nu) return;  // wave-uniform
    const int u = u0 + wk;
    const int len = u < nu ? w.ulen[u] : 0;  // 0: past the end, or a hole (bucketed plan)
    int64_t grow = 0;
    int f = 0, L = -1, us = 0;
    if (len > 0) {
      grow = w.uniq[u];
      f = table_of_row(bank, grow);
      L = w.ulong[u];
      us = w.ustart[u];
    }
    float acc[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) acc[q] = 0.f;
    if (len > 0 && live && L >= 0) {
      const int S = lg_scale(__uint_as_float(w.segmax[L]), len);
      long long *src = w.acc + static_cast<int64_t>(L) * stride + e0;
#pragma unroll
      for (int q = 0; q < EPL; ++q) {
        acc[q] = static_cast<float>(ldexp(static_cast<double>(src[q]), -S));
        src[q] = 0;  // left zero for the next call
      }
      if (l == 0) w.segmax[L] = 0u;
    } else if (len > 0 && live && len <= kLgShort) {
      int r[kLgShort];
#pragma unroll
      for (int j = 0; j < kLgShort; ++j) r[j] = j < len ? w.perm[us + j] : INT_MAX;
      if (len <= 4)
        bitonic_sort<4>(r);
      else if (len <= 8)
        bitonic_sort<8>(r);
      else
        bitonic_sort<16>(r);
#pragma unroll
      for (int j = 0; j < kLgShort; ++j)
        if (j < len) add_lookup_grad<EPL>(a, r[j], f, D, e0, v_lane, w_lane, acc);
    }
    // medium segments: the whole wave, one at a time (wave-uniform loop)
    uint64_t med = __ballot(l == 0 && len > kLgShort && L < 0);
    while (med) {
      const int src = __ffsll(static_cast<unsigned long long>(med)) - 1;
      med &= med - 1;
      const int mlen = __shfl(len, src), ms = __shfl(us, src), mf = __shfl(f, src);
      float m = 0.f;
      if (live) {
#pragma unroll 1
        for (int j = wk; j < mlen; j += WPW) {
          float g[EPL];
          lookup_grad<EPL>(a, w.perm[ms + j], mf, D, e0, v_lane, w_lane, g);
#pragma unroll
          for (int q = 0; q < EPL; ++q) m = fmaxf(m, fabsf(g[q]));
        }
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
      const int S = lg_scale(m, mlen);
      long long sa[EPL];
#pragma unroll
      for (int q = 0; q < EPL; ++q) sa[q] = 0;
      if (live) {
#pragma unroll 1
        for (int j = wk; j < mlen; j += WPW) {
          float g[EPL];
          lookup_grad<EPL>(a, w.perm[ms + j], mf, D, e0, v_lane, w_lane, g);
#pragma unroll
          for (int q = 0; q < EPL; ++q) sa[q] += llrint(ldexp(static_cast<double>(g[q]), S));
        }
      }
#pragma unroll
      for (int off = LPR; off < 64; off <<= 1)
#pragma unroll
        for (int q = 0; q < EPL; ++q) sa[q] += __shfl_xor(sa[q], off);
      if (wk == src / LPR)
#pragma unroll
        for (int q = 0; q < EPL; ++q) acc[q] = static_cast<float>(ldexp(static_cast<double>(sa[q]), -S));
    }
    if (len > 0) {
      uint4 raw = make_uint4(0u, 0u, 0u, 0u);
      if (live) raw = *reinterpret_cast<const uint4 *>(row_ptr_g<T>(bank, a, grow, e0));
      row_update<T, LPR, -1>(bank, a, grow, e0, v_lane, w_lane, live, acc, raw);
    }
  }
}

template <typename T, int LPR>
__device__ __forceinline__ void lg_apply_body(BankArgs bank, int64_t n, LgWs w,
                                                       ApplyArgs a, int stride) {
  constexpr int WPB = 256 / LPR;
  if (a.d_step) a.seed += *a.d_step * 0x9e3779b97f4a7c15ull;
  const int nblk = (w.hdr[0] + WPB - 1) / WPB;
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x)
    lg_apply_block<T, LPR>(bank, w, a, stride, blk);
}

template <typename T, int LPR>
__global__ __launch_bounds__(256) void lg_longmax_kernel(BankArgs bank, int64_t n, LgWs w,
                                                         ApplyArgs a) {
  lg_longmax_body<T, LPR>(bank, n, w, a);
}

template <typename T, int LPR>
__global__ __launch_bounds__(256) void lg_longacc_kernel(BankArgs bank, int64_t n, LgWs w,
                                                         ApplyArgs a, int stride) {
  lg_longacc_body<T, LPR>(bank, n, w, a, stride);
}

template <typename T, int LPR>
__global__ __launch_bounds__(256) void lg_apply_kernel(BankArgs bank, int64_t n, LgWs w,
                                                       ApplyArgs a, int stride) {
  lg_apply_body<T, LPR>(bank, n, w, a, stride);
}

// The fused path's huge segments (> kLgHuge lookups of one row): max |g|, the
// fixed-point chunk sums and the per-row update, three dependent phases in ONE
// launch.  The bucket kernel counts the huge segments in hdr[3]; with none (the
// common case: DIN's padding slots skip the PAD row) every workgroup leaves at once,
// so the step pays one empty launch instead of three.
//
// No co-residency is assumed (a grid barrier would need every workgroup resident,
// which another stream's kernels -- the batch feed, RCCL -- can break): work items
// are DEQUEUED in phase order from one counter (hdr[4]): the nc chunks of phase 0,
// the nc chunks of phase 1, then the apply blocks of phase 2.  A workgroup starting
// an item of phase p > 0 first waits until every item of phase p - 1 is done
// (hdr[4 + p] == nc).  Every such item was dequeued before it by a workgroup that is
// running and never waits while it holds it, so the wait always ends, whatever the
// number of resident workgroups.  Done counters: vmcnt(0) + barrier + release fence
// + agent add; the waiter: relaxed polls + acquire fence.  hdr[4..6] are zeroed by
// the next call's bk_hist_kernel.  The poll is still bounded (a hardware stall, or
// the test-only stall knob which adds `stall` to the target): the workgroup then sets
// the sticky error word hdr[kLgErrWord] (never cleared by a kernel; the host reads and
// clears it: mrec_emb_bwd_large_error_offset) and leaves WITHOUT touching any row --
// an update is never applied from partial sums.

__device__ __forceinline__ bool lg_wait_done(int32_t *ctr, int target, int bound) {
  for (int spins = 0; __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target;) {
    __builtin_amdgcn_s_sleep(2);
    if (++spins > bound) return false;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

template <typename T, int LPR>
__global__ __launch_bounds__(256) void lg_huge_kernel(BankArgs bank, int64_t n, LgWs w,
                                                      ApplyArgs a, int stride, int stall,
                                                      int bound) {
  constexpr int WPB = 256 / LPR;
  if (__hip_atomic_load(w.hdr + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  __shared__ int s_item, s_ok;
  if (a.d_step) a.seed += *a.d_step * 0x9e3779b97f4a7c15ull;
  const int nc = w.hdr[2];
  const int n_items = 2 * nc + (w.hdr[0] + WPB - 1) / WPB;
  int seen = 0;  // phases this workgroup has seen complete
  for (;;) {
    if (threadIdx.x == 0)
      s_item = __hip_atomic_fetch_add(w.hdr + 4, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int it = s_item;
    if (it >= n_items) break;
    const int ph = it < nc ? 0 : it < 2 * nc ? 1 : 2;
    if (ph > seen) {
      if (threadIdx.x == 0) {
        bool ok = lg_wait_done(w.hdr + 4 + ph, nc + stall, bound);
        if (!ok) __hip_atomic_store(w.hdr + kLgErrWord, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_ok = ok;
      }
      __syncthreads();
      if (!s_ok) break;  // uniform: no partial sums ever reach a row
      seen = ph;
    }
    if (ph == 0)
      lg_longmax_chunk<T, LPR>(bank, w, a, it);
    else if (ph == 1)
      lg_longacc_chunk<T, LPR>(bank, w, a, stride, it - nc);
    else
      lg_apply_block<T, LPR>(bank, w, a, stride, it - 2 * nc);
    if (ph < 2) {  // publish this item's atomics / stores, then count it done
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(w.hdr + 5 + ph, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      __syncthreads();  // s_item is rewritten by the next dequeue
    }
  }
}

// ---- fused bucketed plan + apply (mrec_emb_bwd_large_fused) ---------------------
// bk_group_kernel's grouping, then the bucket's own rows are updated right there:
// a segment of <= 16 lookups by one worker (sorted, ascending sample order), one of
// 17..kLgHuge lookups by a whole wave in fixed point (the chunked kernels'
// arithmetic: the same bits as the unfused apply); only huge segments (> kLgHuge)
// go to the lists, indexed by their long slot, for the chunked kernels that follow.
constexpr int kBkLdsPerm = 4096;  // a bucket's placed lookups stay in LDS up to this

template <typename T, int LPR>
__global__ __launch_bounds__(256) void bk_apply_kernel(BankArgs bank, LgWs w, ApplyArgs a, int G,
                                                       int lognb, CoReduce co) {
  __shared__ uint32_t key[kBkSlots];
  __shared__ int32_t cur[kBkSlots];   // counts, then placement cursors (end = start + count)
  __shared__ int32_t seg[kBkSlots];   // segment start inside the bucket
  __shared__ int32_t rowl[kBkSlots];  // short rows, then (from the top) medium rows: slots
  __shared__ int32_t lperm[kBkLdsPerm];
  __shared__ int red[4];
  __shared__ int nshort_s, nmed_s;
  constexpr int EPL = Vec<T>::EPL;
  constexpr int WPB = 256 / LPR, WPW = 64 / LPR;
  constexpr int SPT = kBkSlots / 256;
  if (a.d_step) a.seed += *a.d_step * 0x9e3779b97f4a7c15ull;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int NB = 1 << lognb;
  if (static_cast<int>(blockIdx.x) >= NB) {  // trailing workgroups: deferred MLP reductions
    co_reduce(co, blockIdx.x - NB);
    return;
  }
  const int32_t *pub = w.bhist + static_cast<int64_t>(G) * NB;
  const int lo = pub[blockIdx.x], hi = pub[blockIdx.x + 1];
  if (tid == 0) {  // the scatter has used them: zero for the next call
    w.btot[blockIdx.x] = 0;
    w.bcur[blockIdx.x] = 0;
  }
  for (int k = tid; k < kBkSlots; k += 256) {
    key[k] = kLgEmpty;
    cur[k] = 0;
  }
  __syncthreads();
  auto find = [&](int32_t r, bool insert) -> int {
    uint32_t hsh = ((static_cast<uint32_t>(r) * 2654435761u) << lognb) >> (32 - kBkSlotBits);
    for (int p = 0; p < kBkSlots; ++p) {
      const uint32_t k = insert ? atomicCAS(&key[hsh], kLgEmpty, static_cast<uint32_t>(r))
                                : key[hsh];
      if (k == static_cast<uint32_t>(r) || (insert && k == kLgEmpty)) return static_cast<int>(hsh);
      hsh = (hsh + 1) & (kBkSlots - 1);
    }
    return -1;
  };
  for (int j0 = lo; j0 < hi; j0 += 256) {
    const int j = j0 + tid;
    const int32_t r = j < hi ? w.ent[j].x : -1;
    const Run x = lane_run(r);
    if (x.r >= 0 && x.head == lane) {
      const int s = find(x.r, true);
      if (s >= 0)
        atomicAdd(&cur[s], x.len);
      else  // more distinct rows than the LDS hash (a bank past kLgMaxRows rows only)
        __hip_atomic_store(w.hdr + kLgErrWord, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  int c[SPT], so = 0, ss = 0, sm = 0, sl = 0, sc = 0;
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    c[q] = cur[tid * SPT + q];
    so += c[q];
    ss += c[q] > 0 && c[q] <= kLgShort;
    sm += c[q] > kLgShort && c[q] <= kLgHuge;
    sl += c[q] > kLgHuge;
    sc += c[q] > kLgHuge ? (c[q] + kLgChunk - 1) / kLgChunk : 0;
  }
  int eo, es, em, el, ec;
  bk_scan256(so, &eo, red);
  const int ns = bk_scan256(ss, &es, red);
  const int nm = bk_scan256(sm, &em, red);
  const int nl = bk_scan256(sl, &el, red);
  const int nc = bk_scan256(sc, &ec, red);
  if (tid == 0 && nl > 0) __hip_atomic_fetch_add(w.hdr + 3, nl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool in_lds = nl == 0 && hi - lo <= kBkLdsPerm;
  int32_t *P = in_lds ? lperm : w.perm + lo;  // the bucket's placed lookups
  const int l0 = (lo + kLgHuge) / (kLgHuge + 1), l1 = (hi + kLgHuge) / (kLgHuge + 1);
  const int c0 = l0 + (lo + kLgChunk - 1) / kLgChunk;
  const int c1 = l1 + (hi + kLgChunk - 1) / kLgChunk;
  int L = l0 + el, cb = c0 + ec, at = eo;
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    const int k = tid * SPT + q;
    if (c[q] > 0 && c[q] <= kLgShort) rowl[es++] = k;
    if (c[q] > kLgShort && c[q] <= kLgHuge) rowl[kBkSlots - 1 - em++] = k;
    if (c[q] > kLgHuge) {  // huge: the lists, at its long slot (u = L)
      w.uniq[L] = static_cast<int32_t>(key[k]);
      w.ustart[L] = lo + at;
      w.ulen[L] = c[q];
      w.ulong[L] = L;
      w.longs[L] = L;
      const int nch = (c[q] + kLgChunk - 1) / kLgChunk;
      for (int t = 0; t < nch; ++t) w.chunks[cb + t] = make_int2(L, t);
      cb += nch;
      ++L;
    }
    seg[k] = at;
    cur[k] = at;
    at += c[q];
  }
  if (tid == 0) {
    nshort_s = ns;
    nmed_s = nm;
  }
  for (int v = l0 + nl + tid; v < l1; v += 256) w.ulen[v] = 0;
  for (int v = c0 + nc + tid; v < c1; v += 256) w.chunks[v] = make_int2(-1, 0);
  if (blockIdx.x == NB - 1) {  // slots past the last bucket's ranges
    for (int v = l1 + tid; v < w.hdr[0]; v += 256) w.ulen[v] = 0;
    for (int v = c1 + tid; v < w.hdr[2]; v += 256) w.chunks[v] = make_int2(-1, 0);
  }
  __syncthreads();
  for (int j0 = lo; j0 < hi; j0 += 256) {
    const int j = j0 + tid;
    const int2 e = j < hi ? w.ent[j] : make_int2(-1, 0);
    const Run x = lane_run(e.x);
    int p = 0;
    if (x.r >= 0 && x.head == lane) {
      const int s = find(x.r, false);
      p = s >= 0 ? atomicAdd(&cur[s], x.len) : -1;
    }
    p = __shfl(p, x.head);
    if (e.x >= 0 && p >= 0) P[p + (lane - x.head)] = e.y;
  }
  __syncthreads();
  // ---- the bucket's updates
  const int wk = lane / LPR, l = lane % LPR, e0 = l * EPL;
  const int worker = tid / LPR;
  const int D = bank.dim;
  const bool v_lane = e0 + EPL <= D, w_lane = bank.has_w && e0 == D;
  const bool live = v_lane || w_lane;
  const int nsh = nshort_s, nmd = nmed_s;
  for (int r0 = 0; r0 < nsh; r0 += WPB) {  // short rows: one per worker
    const int r = r0 + worker;
    if (r >= nsh) break;
    const int k = rowl[r];
    const int len = cur[k] - seg[k];
    const int64_t grow = key[k];
    const int f = table_of_row(bank, grow);
    float acc[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) acc[q] = 0.f;
    // the row first: it does not depend on the lookups' gradients
    uint4 raw = make_uint4(0u, 0u, 0u, 0u);
    if (live) raw = *reinterpret_cast<const uint4 *>(row_ptr_g<T>(bank, a, grow, e0));
    if (live) {
      int rr[kLgShort];
#pragma unroll
      for (int j = 0; j < kLgShort; ++j) rr[j] = j < len ? P[seg[k] + j] : INT_MAX;
      if (len <= 4)
        bitonic_sort<4>(rr);
      else if (len <= 8)
        bitonic_sort<8>(rr);
      else
        bitonic_sort<16>(rr);
      // plain bf16 gradient rows (DIN's gathered-row gradient): the lookups' 16-B
      // pieces 4 at a time, issued together (clamped to the first lookup, pinned by
      // an empty use) and added in the same ascending order: the per-lookup loop
      // waited for each load in turn
      bool fast = false;
      if constexpr (EPL == 8)
        fast = v_lane && !a.g_rec && !a.g_occ && !a.dfm && a.dx && a.dx_bf16;
      if (fast) {
        const uint16_t *dxb = static_cast<const uint16_t *>(a.dx) + static_cast<int64_t>(f) * D + e0;
#pragma unroll
        for (int j0 = 0; j0 < kLgShort; j0 += 4) {
          if (j0 >= len) break;
          uint4 q4[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int b = j0 + u < len ? rr[j0 + u] : rr[0];
            q4[u] = *reinterpret_cast<const uint4 *>(dxb + static_cast<int64_t>(b) * a.dx_ld);
          }
          asm volatile("" ::"v"(q4[0].x), "v"(q4[1].x), "v"(q4[2].x), "v"(q4[3].x));
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (j0 + u < len) {
              float g[EPL];
              Vec<uint16_t>::to_f32(q4[u], g);
#pragma unroll
              for (int q = 0; q < EPL; ++q) acc[q] += g[q];
            }
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < kLgShort; ++j)
          if (j < len) add_lookup_grad<EPL>(a, rr[j], f, D, e0, v_lane, w_lane, acc);
      }
    }
    row_update<T, LPR, -1>(bank, a, grow, e0, v_lane, w_lane, live, acc, raw);
  }
  // plain bf16 gradient rows: a worker's lookups 4 at a time, their permutation
  // entries then their 16-B gradient pieces issued together (each pinned by an empty
  // use); the max and the fixed-point sums do not depend on the order (DIN's category
  // table puts all of its rows here, ~130 lookups each at C4)
  bool mfast = false;
  if constexpr (EPL == 8) mfast = v_lane && !a.g_rec && !a.g_occ && !a.dfm && a.dx && a.dx_bf16;
  for (int m = wid; m < nmd; m += 4) {  // medium rows: one per wave (wave-uniform)
    const int k = rowl[kBkSlots - 1 - m];
    const int ms = seg[k], mlen = cur[k] - seg[k];
    const int64_t grow = key[k];
    const int f = table_of_row(bank, grow);
    uint4 raw = make_uint4(0u, 0u, 0u, 0u);  // the row, for the update (issued first)
    if (live && wk == 0) raw = *reinterpret_cast<const uint4 *>(row_ptr_g<T>(bank, a, grow, e0));
    const uint16_t *dxb = mfast ? static_cast<const uint16_t *>(a.dx) + static_cast<int64_t>(f) * D + e0
                                : nullptr;
    auto grads4 = [&](int j0, uint4 (&q4)[4]) {
      int idx[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = j0 + u * WPW;
        idx[u] = P[ms + (j < mlen ? j : 0)];
      }
      asm volatile("" ::"v"(idx[0]), "v"(idx[1]), "v"(idx[2]), "v"(idx[3]));
#pragma unroll
      for (int u = 0; u < 4; ++u)
        q4[u] = *reinterpret_cast<const uint4 *>(dxb + static_cast<int64_t>(idx[u]) * a.dx_ld);
      asm volatile("" ::"v"(q4[0].x), "v"(q4[1].x), "v"(q4[2].x), "v"(q4[3].x));
    };
    float mx = 0.f;
    if (mfast) {
      for (int j0 = wk; j0 < mlen; j0 += 4 * WPW) {
        uint4 q4[4];
        grads4(j0, q4);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (j0 + u * WPW >= mlen) continue;
          float g[EPL];
          Vec<uint16_t>::to_f32(q4[u], g);
#pragma unroll
          for (int q = 0; q < EPL; ++q) mx = fmaxf(mx, fabsf(g[q]));
        }
      }
    } else if (live) {
      for (int j = wk; j < mlen; j += WPW) {
        float g[EPL];
        lookup_grad<EPL>(a, P[ms + j], f, D, e0, v_lane, w_lane, g);
#pragma unroll
        for (int q = 0; q < EPL; ++q) mx = fmaxf(mx, fabsf(g[q]));
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
    const int S = lg_scale(mx, mlen);
    long long sa[EPL];
#pragma unroll
    for (int q = 0; q < EPL; ++q) sa[q] = 0;
    if (mfast) {
      for (int j0 = wk; j0 < mlen; j0 += 4 * WPW) {
        uint4 q4[4];
        grads4(j0, q4);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (j0 + u * WPW >= mlen) continue;
          float g[EPL];
          Vec<uint16_t>::to_f32(q4[u], g);
#pragma unroll
          for (int q = 0; q < EPL; ++q) sa[q] += llrint(ldexp(static_cast<double>(g[q]), S));
        }
      }
    } else if (live) {
      for (int j = wk; j < mlen; j += WPW) {
        float g[EPL];
        lookup_grad<EPL>(a, P[ms + j], f, D, e0, v_lane, w_lane, g);
#pragma unroll
        for (int q = 0; q < EPL; ++q) sa[q] += llrint(ldexp(static_cast<double>(g[q]), S));
      }
    }
#pragma unroll
    for (int off = LPR; off < 64; off <<= 1)
#pragma unroll
      for (int q = 0; q < EPL; ++q) sa[q] += __shfl_xor(sa[q], off);
    if (wk == 0) {
      float acc[EPL];
#pragma unroll
      for (int q = 0; q < EPL; ++q) acc[q] = static_cast<float>(ldexp(static_cast<double>(sa[q]), -S));
      row_update<T, LPR, -1>(bank, a, grow, e0, v_lane, w_lane, live, acc, raw);
    }
  }
}

}  // namespace mrec

using namespace mrec;

extern "C" {

size_t mrec_emb_bwd_large_workspace_size(const mrec_table_bank *bank, int64_t batch) {
  if (!bank || batch < 0 || bank->n_tables < 1) return 0;
  int64_t R = 0;
  for (int f = 0; f < bank->n_tables; ++f) R += bank->rows[f];
  return static_cast<size_t>(lg_ws_bytes(R, batch * bank->n_tables, bank->row_stride, nullptr,
                                         nullptr));
}

size_t mrec_emb_bwd_large_zero_bytes(const mrec_table_bank *bank, int64_t batch) {
  if (!bank || batch < 0 || bank->n_tables < 1) return 0;
  int64_t R = 0;
  for (int f = 0; f < bank->n_tables; ++f) R += bank->rows[f];
  return static_cast<size_t>(lg_zero_bytes(R, batch * bank->n_tables, bank->row_stride));
}

static mrec_status lg_setup(const mrec_table_bank *bank, int64_t batch, void *ws, size_t ws_bytes,
                            BankArgs *ba, int *lpr, int64_t *R, LgWs *w) {
  int eb;
  mrec_status st = make_bank_args(bank, ba, &eb, lpr);
  if (st != MREC_OK) return st;
  MREC_CHECK_ARG(batch >= 0 && batch < (int64_t(1) << 31) / ba->n_tables,
                 "batch * n_tables must be < 2^31");
  MREC_CHECK_ARG(ws != nullptr, "workspace is NULL");
  *R = 0;
  for (int f = 0; f < ba->n_tables; ++f) *R += ba->rows[f];
  MREC_CHECK_ARG(*R < (int64_t(1) << 31), "total rows must be < 2^31");
  MREC_CHECK_ARG(*R <= kLgMaxRows || bk_groups(*R, batch * ba->n_tables) > 0,
                 "banks of more than 2^24 rows need the bucketed plan: batch * n_tables <= 2M");
  const int64_t need = lg_ws_bytes(*R, batch * ba->n_tables, ba->row_stride, w,
                                   static_cast<char *>(ws));
  if (ws_bytes < static_cast<size_t>(need)) {
    set_error("large-batch workspace too small");
    return MREC_ENOSPC;
  }
  return MREC_OK;
}

mrec_status mrec_emb_bwd_large_plan(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                                    void *workspace, size_t ws_bytes, int32_t *d_oob_flag,
                                    mrec_stream stream) {
  BankArgs ba;
  IdsArgs ia;
  int lpr;
  int64_t R;
  LgWs w;
  mrec_status st = lg_setup(bank, batch, workspace, ws_bytes, &ba, &lpr, &R, &w);
  if (st != MREC_OK) return st;
  if ((st = make_ids_args(ids, ba.n_tables, &ia)) != MREC_OK) return st;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (batch == 0) return MREC_OK;  // (apply returns early for batch 0 as well)
  const int64_t total = batch * ba.n_tables;
  const int G = bk_groups(R, total);
  // MREC_LG_ATOMIC_PLAN (diagnostics): the atomic plan's per-row arrays exist only for
  // banks up to kLgMaxRows rows (lg_ws_bytes); past that the knob is ignored
  const bool atomic_knob = std::getenv("MREC_LG_ATOMIC_PLAN") != nullptr && R <= kLgMaxRows;
  if (G > 0 && !atomic_knob) {
    const int NB = bk_buckets(total);
    int lognb = 0;
    while ((1 << lognb) < NB) ++lognb;
    bk_hist_kernel<<<dim3(G), kBkThreads, 0, s>>>(ba, ia, batch, lognb, w, d_oob_flag);
      bk_scatter_kernel<<<dim3(G), kBkThreads, 0, s>>>(ba, ia, batch, G, lognb, w, 0);
    bk_group_kernel<<<dim3(NB), 256, 0, s>>>(w, G, lognb, d_oob_flag);
    return launch_status("mrec_emb_bwd_large_plan");
  }
  MREC_CHECK_ARG(R <= kLgMaxRows, "the atomic large-batch plan needs a bank of <= 2^24 rows");
  if (hipMemsetAsync(w.cnt, 0, static_cast<size_t>(R) * 4, s) != hipSuccess)
    return launch_status("mrec_emb_bwd_large_plan (memset)");
  const int nblk = static_cast<int>((R + kLgRowsPerBlock - 1) / kLgRowsPerBlock);
  const unsigned gl = static_cast<unsigned>((total + 256 * kLgIter - 1) / (256 * kLgIter));
  lg_count_kernel<<<dim3(gl), 256, 0, s>>>(ba, ia, batch, w, d_oob_flag);
  lg_blocksum_kernel<<<dim3(nblk), 256, 0, s>>>(R, w);
  lg_scan_kernel<16><<<dim3(nblk), 256, 0, s>>>(R, nblk, w);
  lg_place_kernel<<<dim3(gl), 256, 0, s>>>(ba, ia, batch, w);
  return launch_status("mrec_emb_bwd_large_plan");
}

}  // extern "C"

// the apply arguments, checked (shared by mrec_emb_bwd_large_apply / _fused)
static mrec_status lg_apply_args(const mrec_table_bank *bank, const BankArgs &ba, const void *dx,
                                 mrec_dtype dx_dtype, int64_t dx_ld, const float *dfm,
                                 const float *fm_sum, const void *x0, mrec_dtype x0_dtype,
                                 int64_t x0_ld, const float *dw, mrec_bwd_mode mode, float lr,
                                 uint64_t seed, const uint64_t *d_step, void *grad, ApplyArgs *out) {
  MREC_CHECK_ARG(mode >= MREC_BWD_DENSE_GRAD && mode <= MREC_BWD_ADAM, "bad mode");
  OptArgs opt{};
  {
    const mrec_status so = make_opt_args(bank, mode, &opt);
    if (so != MREC_OK) return so;
  }
  MREC_CHECK_ARG(mode != MREC_BWD_DENSE_GRAD || grad != nullptr, "DENSE_GRAD needs grad");
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
  ApplyArgs a = {};
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
  a.opt = opt;
  a.grad = grad;
  *out = a;
  return MREC_OK;
}

// the chunked kernels and the per-row apply (fused: the bucket kernel first, the
// per-row apply then walks only the huge segments' slots)
template <typename T, int L>
static void lg_launch_apply(const BankArgs &ba, int64_t batch, const LgWs &w, const ApplyArgs &a,
                            int stride, int fused_nb, int G, int lognb, const CoReduce &co,
                            int co_blocks, hipStream_t s) {
  dim3 gc(kLgApplyBlocks), gu(kLgApplyBlocks);
  if (fused_nb) {
    bk_apply_kernel<T, L><<<dim3(fused_nb + co_blocks), 256, 0, s>>>(ba, w, a, G, lognb, co);
    // only huge segments are left: as many workgroups as their slots (mostly holes)
    const int64_t N = batch * ba.n_tables;
    const int64_t ul = (N + kLgHuge) / (kLgHuge + 1) + 1;
    const int64_t cc = ul + (N + kLgChunk - 1) / kLgChunk + 2;
    gc = dim3(static_cast<unsigned>(std::min<int64_t>(cc, kLgApplyBlocks)));
    gu = dim3(static_cast<unsigned>(std::min<int64_t>((ul + 256 / L - 1) / (256 / L), kLgApplyBlocks)));
    // any grid size is correct (dequeued items, no co-residency); enough to fill the
    // chip when there is work, and every workgroup leaves at once when there is none
    static const int cus = [] {
      int dev = 0, c = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
      (void)hipGetLastError();
      return std::max(1, c);
    }();
    const int64_t need = std::max<int64_t>(gc.x, gu.x);
    int stall = 0, bound = 1 << 26;  // ~seconds of 128-cycle sleeps
    if (const char *e = std::getenv("MREC_LG_HUGE_TEST_STALL")) {  // test-only: force the time-out
      stall = std::atoi(e);
      if (stall) bound = 1 << 14;
    }
    lg_huge_kernel<T, L><<<dim3(static_cast<unsigned>(std::min<int64_t>(need, 2 * cus))), 256, 0, s>>>(
        ba, batch, w, a, stride, stall, bound);
    return;
  }
  lg_longmax_kernel<T, L><<<gc, 256, 0, s>>>(ba, batch, w, a);
  lg_longacc_kernel<T, L><<<gc, 256, 0, s>>>(ba, batch, w, a, stride);
  lg_apply_kernel<T, L><<<gu, 256, 0, s>>>(ba, batch, w, a, stride);
}

static void lg_dispatch_apply(mrec_dtype dtype, int lpr, const BankArgs &ba, int64_t batch,
                              const LgWs &w, const ApplyArgs &a, int stride, int fused_nb, int G,
                              int lognb, hipStream_t s, const CoReduce &co = CoReduce{},
                              int co_blocks = 0) {
#define MREC_LG(T, L) \
  lg_launch_apply<T, L>(ba, batch, w, a, stride, fused_nb, G, lognb, co, co_blocks, s)
  if (dtype == MREC_BF16) {
    switch (lpr) {
      case 1: MREC_LG(uint16_t, 1); break;
      case 2: MREC_LG(uint16_t, 2); break;
      case 4: MREC_LG(uint16_t, 4); break;
      case 8: MREC_LG(uint16_t, 8); break;
      default: MREC_LG(uint16_t, 16); break;
    }
  } else {
    switch (lpr) {
      case 1: MREC_LG(float, 1); break;
      case 2: MREC_LG(float, 2); break;
      case 4: MREC_LG(float, 4); break;
      case 8: MREC_LG(float, 8); break;
      default: MREC_LG(float, 16); break;
    }
  }
#undef MREC_LG
}

extern "C" {

size_t mrec_emb_bwd_large_error_offset(void) { return kLgErrWord * sizeof(int32_t); }

mrec_status mrec_emb_bwd_large_apply(const mrec_table_bank *bank, int64_t batch,
                                     const void *workspace, size_t ws_bytes, const void *dx,
                                     mrec_dtype dx_dtype, int64_t dx_ld, const float *dfm,
                                     const float *fm_sum, const void *x0, mrec_dtype x0_dtype,
                                     int64_t x0_ld, const float *dw, mrec_bwd_mode mode, float lr,
                                     uint64_t seed, const uint64_t *d_step, void *grad,
                                     mrec_stream stream) {
  BankArgs ba;
  int lpr;
  int64_t R;
  LgWs w;
  mrec_status st = lg_setup(bank, batch, const_cast<void *>(workspace), ws_bytes, &ba, &lpr, &R,
                            &w);
  if (st != MREC_OK) return st;
  ApplyArgs a{};
  st = lg_apply_args(bank, ba, dx, dx_dtype, dx_ld, dfm, fm_sum, x0, x0_dtype, x0_ld, dw, mode,
                     lr, seed, d_step, grad, &a);
  if (st != MREC_OK) return st;
  if (batch == 0) return MREC_OK;
  lg_dispatch_apply(bank->dtype, lpr, ba, batch, w, a, ba.row_stride, 0, 0, 0,
                    static_cast<hipStream_t>(stream));
  return launch_status("mrec_emb_bwd_large_apply");
}

}  // extern "C"

// fused plan + apply with the apply arguments already built (own gradients, or
// given ones: the owner side of a row-sharded exchange)
static mrec_status lg_fused_impl(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                                 void *workspace, size_t ws_bytes, int32_t *d_oob_flag,
                                 const ApplyArgs &a, int32_t n_reduce,
                                 const mrec_gemm_call *reduce, mrec_stream stream) {
  BankArgs ba;
  IdsArgs ia;
  int lpr;
  int64_t R;
  LgWs w;
  mrec_status st = lg_setup(bank, batch, workspace, ws_bytes, &ba, &lpr, &R, &w);
  if (st != MREC_OK) return st;
  if ((st = make_ids_args(ids, ba.n_tables, &ia)) != MREC_OK) return st;
  CoReduce co;
  int co_blocks = 0;
  if ((st = build_co_reduce(n_reduce, reduce, &co, &co_blocks)) != MREC_OK) return st;
  const int64_t total = batch * ba.n_tables;
  const int G = batch == 0 ? 0 : bk_groups(R, total);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (G == 0 || (std::getenv("MREC_LG_ATOMIC_PLAN") && R <= kLgMaxRows)) {  // the two-call path
    if (batch > 0) {
      st = mrec_emb_bwd_large_plan(bank, ids, batch, workspace, ws_bytes, d_oob_flag, stream);
      if (st != MREC_OK) return st;
      lg_dispatch_apply(bank->dtype, lpr, ba, batch, w, a, ba.row_stride, 0, 0, 0, s);
      if ((st = launch_status("mrec_emb_bwd_large_apply")) != MREC_OK) return st;
    }
    return co.n ? mrec_gemm_multi(n_reduce, reduce, stream) : MREC_OK;
  }
  const int NB = bk_buckets(total);
  int lognb = 0;
  while ((1 << lognb) < NB) ++lognb;
  bk_hist_kernel<<<dim3(G), kBkThreads, 0, s>>>(ba, ia, batch, lognb, w, d_oob_flag);
  bk_scatter_kernel<<<dim3(G), kBkThreads, 0, s>>>(ba, ia, batch, G, lognb, w, 1);
  lg_dispatch_apply(bank->dtype, lpr, ba, batch, w, a, ba.row_stride, NB, G, lognb, s, co,
                    co_blocks);
  return launch_status("mrec_emb_bwd_large_fused");
}

extern "C" {

mrec_status mrec_emb_bwd_large_fused_ex(const mrec_table_bank *bank, const mrec_ids *ids,
                                        int64_t batch, void *workspace, size_t ws_bytes,
                                        int32_t *d_oob_flag, const void *dx, mrec_dtype dx_dtype,
                                        int64_t dx_ld, const float *dfm, const float *fm_sum,
                                        const void *x0, mrec_dtype x0_dtype, int64_t x0_ld,
                                        const float *dw, mrec_bwd_mode mode, float lr,
                                        uint64_t seed, const uint64_t *d_step, void *grad,
                                        int32_t n_reduce, const mrec_gemm_call *reduce,
                                        mrec_stream stream) {
  MREC_CHECK_ARG(bank != nullptr, "NULL bank");
  BankArgs ba;
  int es = 0, lpr = 0;
  mrec_status st = make_bank_args(bank, &ba, &es, &lpr);
  if (st != MREC_OK) return st;
  ApplyArgs a{};
  st = lg_apply_args(bank, ba, dx, dx_dtype, dx_ld, dfm, fm_sum, x0, x0_dtype, x0_ld, dw, mode,
                     lr, seed, d_step, grad, &a);
  if (st != MREC_OK) return st;
  return lg_fused_impl(bank, ids, batch, workspace, ws_bytes, d_oob_flag, a, n_reduce, reduce,
                       stream);
}

mrec_status mrec_emb_bwd_large_fused_given(const mrec_table_bank *bank, const mrec_ids *ids,
                                           int64_t batch, void *workspace, size_t ws_bytes,
                                           int32_t *d_oob_flag, const mrec_given_grads *given,
                                           mrec_bwd_mode mode, float lr, uint64_t seed,
                                           const uint64_t *d_step, void *grad, int32_t n_reduce,
                                           const mrec_gemm_call *reduce, mrec_stream stream) {
  MREC_CHECK_ARG(bank != nullptr && given != nullptr, "NULL bank / given");
  const mrec_given_grads &g = *given;
  MREC_CHECK_ARG((g.g_occ != nullptr) != (g.wire != nullptr), "exactly one of g_occ / wire");
  MREC_CHECK_ARG(g.chunk >= 1, "chunk (entries per exchange part) must be >= 1");
  BankArgs ba;
  int es = 0, lpr = 0;
  mrec_status st = make_bank_args(bank, &ba, &es, &lpr);
  if (st != MREC_OK) return st;
  ApplyArgs a{};
  st = lg_apply_args(bank, ba, nullptr, MREC_F32, 0, nullptr, nullptr, nullptr, MREC_F32, 0,
                     nullptr, mode, lr, seed, d_step, grad, &a);
  if (st != MREC_OK) return st;
  a.chunk = g.chunk;
  if (g.g_occ) {
    MREC_CHECK_ARG(g.g_ld >= ba.dim + (ba.has_w ? 1 : 0) && g.g_ld % 4 == 0 &&
                       (reinterpret_cast<uintptr_t>(g.g_occ) & 15) == 0,
                   "g_occ rows: >= dim (+w) floats, 16-B aligned");
    MREC_CHECK_ARG(g.chunk_stride >= static_cast<int64_t>(ba.n_tables) * g.chunk,
                   "chunk_stride < n_tables * chunk");
    a.g_occ = g.g_occ;
    a.g_ld = g.g_ld;
    a.chunk_stride = g.chunk_stride;
  } else {
    MREC_CHECK_ARG(g.wire_dtype == MREC_BF16 || g.wire_dtype == MREC_F32,
                   "wire dtype must be BF16/F32");
    const int wes = g.wire_dtype == MREC_BF16 ? 2 : 4;
    MREC_CHECK_ARG(g.rec_bytes > 0 && g.rec_bytes % wes == 0 && g.rec_bytes % 4 == 0 &&
                       g.rec_bytes >= (ba.dim + (ba.has_w ? 1 : 0)) * wes,
                   "bad record bytes");
    MREC_CHECK_ARG(g.pref != nullptr && g.cap_rows >= 1, "NULL pref / cap_rows < 1");
    a.g_rec = g.wire;
    a.g_rec_bf16 = g.wire_dtype == MREC_BF16;
    a.g_rec_pitch = g.rec_bytes / wes;
    a.g_pref = g.pref;
    a.g_cap_rows = g.cap_rows;
  }
  a.g_F = ba.n_tables;
  return lg_fused_impl(bank, ids, batch, workspace, ws_bytes, d_oob_flag, a, n_reduce, reduce,
                       stream);
}

mrec_status mrec_emb_bwd_large_fused(const mrec_table_bank *bank, const mrec_ids *ids,
                                     int64_t batch, void *workspace, size_t ws_bytes,
                                     int32_t *d_oob_flag, const void *dx, mrec_dtype dx_dtype,
                                     int64_t dx_ld, const float *dfm, const float *fm_sum,
                                     const void *x0, mrec_dtype x0_dtype, int64_t x0_ld,
                                     const float *dw, mrec_bwd_mode mode, float lr, uint64_t seed,
                                     const uint64_t *d_step, void *grad, mrec_stream stream) {
  return mrec_emb_bwd_large_fused_ex(bank, ids, batch, workspace, ws_bytes, d_oob_flag, dx,
                                     dx_dtype, dx_ld, dfm, fm_sum, x0, x0_dtype, x0_ld, dw, mode,
                                     lr, seed, d_step, grad, 0, nullptr, stream);
}

}  // extern "C"
