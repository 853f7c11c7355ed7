// Row-sharded embedding tables: the id -> owner exchange around the hot path.
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
#pragma unroll
  for (int r = 0; r < kPre; ++r) {
    const int64_t i = static_cast<int64_t>(r) * kBT + tid;
    pre[r] = (r < rounds && i < B) ? load_id(ids, f, i) : -1;
  }
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
      if (overflow) *overflow = 1;
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

}  // extern "C"
