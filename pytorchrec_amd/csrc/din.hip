// DIN target-attention pooling (config C4).
//
//   feat[b*L+j] = [q_b | k_bj | q_b - k_bj | q_b * k_bj]          (attention-unit input)
//   s_bj = att_out(att_mlp(feat[b*L+j]))                          (MFMA GEMMs, mrec_gemm)
//   a_bj = softmax_j over valid j (his_bj > 0 or j == 0), invalid -> 0
//   x_top[b] = [q_b | u_b],  u_b = sum_j a_bj k_bj                 (input of the top MLP)
//
// The reference has no DIN; its idioms are the masked softmax of
// scaled_dot_product_attention (SASRec.py:14-31, invalid keys -> -inf) and the
// history validity of get_valid_his_index (torchrec/model/utils.py:5-10).
// One wave per sample for the pooling (lane j = history position j, L <= 64):
// masked max / sum by wave shuffles, the weighted sum over positions through a
// per-wave LDS transpose summed in position order (deterministic).
#include "common.h"

namespace mrec {

constexpr int DIN_MAXL = 64;
constexpr int DIN_MAXE = 64;

__device__ __forceinline__ bool din_valid(const int32_t *his, int64_t ldh, int64_t b, int j) {
  return j == 0 || his[b * ldh + j] > 0;
}

// one thread per (row b*L+j, 8-element chunk of E)
__global__ __launch_bounds__(256) void din_feat_fwd_kernel(const uint16_t *__restrict__ q,
                                                           int64_t ldq,
                                                           const uint16_t *__restrict__ k,
                                                           int64_t ldk, int64_t rows, int L, int E,
                                                           uint16_t *__restrict__ feat,
                                                           int64_t ldf) {
  const int ch = E / 8;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (t >= rows * ch) return;
  const int64_t r = t / ch;
  const int c = static_cast<int>(t % ch) * 8;
  const int64_t b = r / L;
  float qv[8], kv[8];
  Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(q + b * ldq + c), qv);
  Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(k + r * ldk + c), kv);
  uint16_t *o = feat + r * ldf + c;
  *reinterpret_cast<uint4 *>(o) = *reinterpret_cast<const uint4 *>(q + b * ldq + c);
  *reinterpret_cast<uint4 *>(o + E) = *reinterpret_cast<const uint4 *>(k + r * ldk + c);
  float d[8], p[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    d[i] = qv[i] - kv[i];
    p[i] = qv[i] * kv[i];
  }
  *reinterpret_cast<uint4 *>(o + 2 * E) =
      make_uint4(pack_bf16x2(d[0], d[1]), pack_bf16x2(d[2], d[3]), pack_bf16x2(d[4], d[5]),
                 pack_bf16x2(d[6], d[7]));
  *reinterpret_cast<uint4 *>(o + 3 * E) =
      make_uint4(pack_bf16x2(p[0], p[1]), pack_bf16x2(p[2], p[3]), pack_bf16x2(p[4], p[5]),
                 pack_bf16x2(p[6], p[7]));
}

// 4 samples per 256-thread workgroup, one wave each
__global__ __launch_bounds__(256) void din_pool_fwd_kernel(
    const float *__restrict__ s, int64_t lds, const int32_t *__restrict__ his, int64_t ldh,
    const uint16_t *__restrict__ q, int64_t ldq, const uint16_t *__restrict__ k, int64_t ldk,
    int64_t B, int L, int E, float *__restrict__ a_out, uint16_t *__restrict__ top, int64_t ldt) {
  __shared__ float tr[4][DIN_MAXL][DIN_MAXE + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 4 + w;
  if (b >= B) return;  // uniform per wave; no block-wide barrier below
  const bool on = lane < L;
  const bool val = on && din_valid(his, ldh, b, lane);
  const float sj = val ? s[(b * L + lane) * lds] : -INFINITY;
  float m = sj;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  const float e = val ? __expf(sj - m) : 0.f;
  float sum = e;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
  const float a = e / sum;
  if (on) a_out[b * L + lane] = a;
  if (on) {
    const uint16_t *kr = k + (b * L + lane) * ldk;
    for (int c = 0; c < E; c += 8) {
      float kv[8];
      Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(kr + c), kv);
#pragma unroll
      for (int i = 0; i < 8; ++i) tr[w][lane][c + i] = a * kv[i];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes, then its reads
  if (lane < E) {
    float u = 0.f;
    for (int j = 0; j < L; ++j) u += tr[w][j][lane];  // position order
    top[b * ldt + E + lane] = f32_to_bf16_rne(u);
    top[b * ldt + lane] = q[b * ldq + lane];
  }
  for (int c = 2 * E + lane; c < ldt; c += 64) top[b * ldt + c] = 0;  // zero pad columns
}

// pooling backward: du = dtop[:, E:2E]; g_j = du . k_j;
//   ds_j = a_j (g_j - sum_i a_i g_i);  dk_j = a_j du  (fp32, written, not added)
__global__ __launch_bounds__(256) void din_pool_bwd_kernel(
    const uint16_t *__restrict__ dtop, int64_t lddt, const float *__restrict__ a_in,
    const uint16_t *__restrict__ k, int64_t ldk, int64_t B, int L, int E, float *__restrict__ ds,
    float *__restrict__ dk, int64_t lddk) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 4 + w;
  if (b >= B) return;
  const bool on = lane < L;
  const float a = on ? a_in[b * L + lane] : 0.f;
  float g = 0.f;
  if (on) {
    const uint16_t *kr = k + (b * L + lane) * ldk;
    const uint16_t *du = dtop + b * lddt + E;
    float *dkr = dk + (b * L + lane) * lddk;
    for (int c = 0; c < E; c += 8) {
      float kv[8], dv[8];
      Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(kr + c), kv);
      Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(du + c), dv);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        g = fmaf(dv[i], kv[i], g);
        dkr[c + i] = a * dv[i];
      }
    }
  }
  float ag = a * g;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ag += __shfl_xor(ag, off);
  if (on) ds[b * L + lane] = a * (g - ag);
}

// attention-unit input backward (+ the pooling's dk, + the direct q gradient):
//   dk_j += df_k - df_(q-k) + df_(q*k) * q
//   dq    = dtop[:, :E] + sum_j (df_q + df_(q-k) + df_(q*k) * k_j)      (position order)
// ROWS: the final dq / dk go to one bf16 gradient of the gathered rows
// [target rows (B) | history rows (B L)] (row stride ld_rows) instead of fp32 dq
// and dk in place -- the gather's input gradient as autograd wants it (bf16),
// without slice-backward zero fills, copies and an add of the two pieces
template <bool ROWS>
__global__ __launch_bounds__(256) void din_feat_bwd_kernel(
    const uint16_t *__restrict__ df, int64_t lddf, const uint16_t *__restrict__ dtop,
    int64_t lddt, const uint16_t *__restrict__ q, int64_t ldq, const uint16_t *__restrict__ k,
    int64_t ldk, int64_t B, int L, int E, float *__restrict__ dk, int64_t lddk,
    float *__restrict__ dq, int64_t lddq, uint16_t *__restrict__ drows, int64_t ld_rows) {
  __shared__ float tr[4][DIN_MAXL][DIN_MAXE + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 4 + w;
  if (b >= B) return;
  // lane task t = (history position j, 8-column chunk c): consecutive lanes take
  // consecutive chunks of a row, so the df / k reads and the dk read-modify-write
  // are 16-B accesses along rows (one lane per whole row made every dk access a
  // scalar 4-B one, 67 us per C4 step)
  const int nc = E / 8;
  const bool vec = (reinterpret_cast<uintptr_t>(dk) & 15) == 0 && (lddk & 3) == 0;
  for (int t = lane; t < L * nc; t += 64) {
    const int j = t / nc, c = (t - j * nc) * 8;
    const int64_t r = b * L + j;
    const uint16_t *d = df + r * lddf;
    float f0[8], f1[8], f2[8], f3[8], kv[8], qv[8];
    Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(d + c), f0);
    Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(d + E + c), f1);
    Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(d + 2 * E + c), f2);
    Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(d + 3 * E + c), f3);
    Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(k + r * ldk + c), kv);
    Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(q + b * ldq + c), qv);
    float *dkr = dk + r * lddk + c;
    float o[8];
    if (vec) {
      const float4 a0 = *reinterpret_cast<const float4 *>(dkr);
      const float4 a1 = *reinterpret_cast<const float4 *>(dkr + 4);
      o[0] = a0.x; o[1] = a0.y; o[2] = a0.z; o[3] = a0.w;
      o[4] = a1.x; o[5] = a1.y; o[6] = a1.z; o[7] = a1.w;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = dkr[i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      o[i] += f1[i] - f2[i] + f3[i] * qv[i];
      tr[w][j][c + i] = f0[i] + f2[i] + f3[i] * kv[i];
    }
    if constexpr (ROWS) {
      *reinterpret_cast<uint4 *>(drows + (B + r) * ld_rows + c) =
          make_uint4(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]), pack_bf16x2(o[4], o[5]),
                     pack_bf16x2(o[6], o[7]));
    } else if (vec) {
      *reinterpret_cast<float4 *>(dkr) = make_float4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<float4 *>(dkr + 4) = make_float4(o[4], o[5], o[6], o[7]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) dkr[i] = o[i];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes, then its reads
  if (lane < E) {
    float v = bf16_to_f32(dtop[b * lddt + lane]);
    for (int j = 0; j < L; ++j) v += tr[w][j][lane];
    if constexpr (ROWS)
      drows[b * ld_rows + lane] = f32_to_bf16_rne(v);
    else
      dq[b * lddq + lane] = v;
  }
}

// DIN lookup ids, one thread per (sample, slot 0..L): out[b] = target id, out[B + b L
// + j] = history id if position j is valid (his > 0 or j == 0), else -1 (a padded
// slot: zero row forward, skipped by the backward), for the item and category tables.
// Only a PAD history position (his == 0, j > 0) becomes a padding slot.  Every other
// id that is negative or does not fit int32 -- the targets, position 0, a negative
// his anywhere, the category of a non-PAD position, a negative category anywhere --
// becomes INT32_MAX, a row no table has (the host checks category_num < 2^31 - 1),
// so the gather's range check raises IndexError for it as nn.Embedding does over
// the whole [B, L] tensors: never a silent zero row or a wrapped row.  (Not
// detected: a category id >= its table's rows at a PAD position.)
template <typename I>
__device__ __forceinline__ int32_t din_narrow_id(I v) {
  return (v < 0 || v >= static_cast<I>(INT32_MAX)) ? INT32_MAX : static_cast<int32_t>(v);
}

template <typename I>
__global__ __launch_bounds__(256) void din_ids_kernel(const I *__restrict__ iid,
                                                      const I *__restrict__ cid,
                                                      const I *__restrict__ his, int64_t ldh,
                                                      const I *__restrict__ hcat, int64_t ldc,
                                                      int64_t B, int L, int32_t *__restrict__ out_i,
                                                      int32_t *__restrict__ out_c) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (t >= B * (L + 1)) return;
  const int64_t b = t / (L + 1);
  const int j = static_cast<int>(t - b * (L + 1));
  if (j == L) {
    out_i[b] = din_narrow_id(iid[b]);
    out_c[b] = din_narrow_id(cid[b]);
    return;
  }
  const I h = his[b * ldh + j];
  const I c = hcat[b * ldc + j];
  const bool pad = j > 0 && h == 0;  // masked (h < 0 is an error wherever it sits)
  out_i[B + b * L + j] = pad ? -1 : din_narrow_id(h);
  out_c[B + b * L + j] = (pad && c >= 0) ? -1 : din_narrow_id(c);
}

// mrec_din_gather: the lookup ids of din_ids_kernel built in the gather itself (one
// launch instead of two): worker (i, f) over the N = B (L + 1) lookup positions and
// the two tables; its lane 0 also writes the id for the embedding backward.  A
// padding slot (-1) gathers a zero row; an invalid id (INT32_MAX) sets the OOB flag.
template <typename I, typename T, typename O, int LPR>
__global__ __launch_bounds__(256) void din_gather_kernel(BankArgs bank, const I *__restrict__ iid,
                                                         const I *__restrict__ cid,
                                                         const I *__restrict__ his, int64_t ldh,
                                                         const I *__restrict__ hcat, int64_t ldc,
                                                         int64_t B, int L, int32_t *__restrict__ out_i,
                                                         int32_t *__restrict__ out_c,
                                                         O *__restrict__ out, int64_t out_ld,
                                                         int32_t *__restrict__ oob) {
  constexpr int EPL = Vec<T>::EPL;
  constexpr int WPB = 256 / LPR;
  const int64_t g = static_cast<int64_t>(blockIdx.x) * WPB + threadIdx.x / LPR;
  const int l = threadIdx.x % LPR;
  const int64_t N = B * (L + 1);
  if (g >= 2 * N) return;
  const int64_t i = g >> 1;
  const int f = static_cast<int>(g & 1);
  // Every id source is loaded before any is used, from clamped indices (a target
  // lookup reads his[0] / hcat[0], a history one iid[0] / cid[0], and drops them), and
  // the two tables' bounds come from the kernel arguments by constant index: as
  // written before, his -> hcat -> rows[f] -> row_offset[f] -> row ran as ~5 dependent
  // round trips (a loaded value copied out of a branch waits for its load).
  const bool tgt = i < B;
  int64_t bb = 0;
  int j = 0;
  if (!tgt) {
    const int64_t r = i - B;
    if (N < (int64_t(1) << 31)) {  // (uniform) 32-bit division
      const uint32_t q = static_cast<uint32_t>(r) / static_cast<uint32_t>(L);
      bb = q;
      j = static_cast<int>(static_cast<uint32_t>(r) - q * static_cast<uint32_t>(L));
    } else {
      bb = r / L;
      j = static_cast<int>(r - bb * L);
    }
  }
  const I tv = (f ? cid : iid)[tgt ? i : 0];
  const I h = his[bb * ldh + j];
  const I c = hcat[bb * ldc + j];
  // (an empty use of all three: the compiler would otherwise sink each load into the
  // branch that consumes it, one round trip after the other)
  asm volatile("" ::"v"(tv), "v"(h), "v"(c));
  int32_t id;
  if (tgt) {
    id = din_narrow_id(tv);
  } else {
    const bool pad = j > 0 && h == 0;  // masked (h < 0 is an error wherever it sits)
    id = f == 0 ? (pad ? -1 : din_narrow_id(h)) : ((pad && c >= 0) ? -1 : din_narrow_id(c));
  }
  if (l == 0) (f ? out_c : out_i)[i] = id;
  const int64_t nrow = f ? bank.rows[1] : bank.rows[0];
  const int64_t roff = f ? bank.row_offset[1] : bank.row_offset[0];
  const bool ok = id >= 0 && id < nrow;
  uint4 raw = *reinterpret_cast<const uint4 *>(reinterpret_cast<const T *>(bank.data) +
                                               (ok ? roff + id : 0) *
                                                   static_cast<int64_t>(bank.row_stride) +
                                               l * EPL);
  if (!ok) {
    raw = make_uint4(0, 0, 0, 0);
    if (l == 0 && oob && id >= 0) *oob = 1;
  }
  const int D = bank.dim;
  const int e0 = l * EPL;
  if (e0 + EPL > D) return;
  O *dst = out + i * out_ld + static_cast<int64_t>(f) * D + e0;
  if constexpr (sizeof(O) == sizeof(T)) {
    *reinterpret_cast<uint4 *>(dst) = raw;  // bit copy
  } else {
    float v[EPL];
    Vec<T>::to_f32(raw, v);
    if constexpr (sizeof(O) == 4) {
#pragma unroll
      for (int q = 0; q < EPL; q += 4)
        *reinterpret_cast<float4 *>(dst + q) = make_float4(v[q], v[q + 1], v[q + 2], v[q + 3]);
    } else {
      *reinterpret_cast<uint2 *>(dst) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    }
  }
}

template <typename I, typename T, typename O>
static void din_gather_launch(int lpr, const BankArgs &ba, const void *iid, const void *cid,
                              const void *his, int64_t ldh, const void *hcat, int64_t ldc,
                              int64_t B, int L, int32_t *oi, int32_t *oc, void *out,
                              int64_t out_ld, int32_t *oob, hipStream_t s) {
  const int64_t work = 2 * B * (L + 1);
  const int wpb = 256 / lpr;
  const dim3 grid(static_cast<unsigned>((work + wpb - 1) / wpb));
  const I *a = static_cast<const I *>(iid), *c = static_cast<const I *>(cid);
  const I *h = static_cast<const I *>(his), *hc = static_cast<const I *>(hcat);
  O *o = static_cast<O *>(out);
#define MREC_DG(LP) \
  din_gather_kernel<I, T, O, LP><<<grid, 256, 0, s>>>(ba, a, c, h, ldh, hc, ldc, B, L, oi, oc, o, out_ld, oob)
  switch (lpr) {
    case 1: MREC_DG(1); break;
    case 2: MREC_DG(2); break;
    case 4: MREC_DG(4); break;
    case 8: MREC_DG(8); break;
    default: MREC_DG(16); break;
  }
#undef MREC_DG
}

template <typename I>
static void din_gather_dispatch(mrec_dtype bank_dt, mrec_dtype out_dt, int lpr, const BankArgs &ba,
                                const void *iid, const void *cid, const void *his, int64_t ldh,
                                const void *hcat, int64_t ldc, int64_t B, int L, int32_t *oi,
                                int32_t *oc, void *out, int64_t out_ld, int32_t *oob, hipStream_t s) {
  if (bank_dt == MREC_BF16) {
    if (out_dt == MREC_BF16)
      din_gather_launch<I, uint16_t, uint16_t>(lpr, ba, iid, cid, his, ldh, hcat, ldc, B, L, oi, oc, out, out_ld, oob, s);
    else
      din_gather_launch<I, uint16_t, float>(lpr, ba, iid, cid, his, ldh, hcat, ldc, B, L, oi, oc, out, out_ld, oob, s);
  } else {
    if (out_dt == MREC_BF16)
      din_gather_launch<I, float, uint16_t>(lpr, ba, iid, cid, his, ldh, hcat, ldc, B, L, oi, oc, out, out_ld, oob, s);
    else
      din_gather_launch<I, float, float>(lpr, ba, iid, cid, his, ldh, hcat, ldc, B, L, oi, oc, out, out_ld, oob, s);
  }
}

static bool a16(const void *p, int64_t ld) {
  return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 8 == 0;
}

}  // namespace mrec

using namespace mrec;

extern "C" {

mrec_status mrec_din_lookup_ids(const void *iid, const void *cid, const void *his, int64_t ld_his,
                                const void *hcat, int64_t ld_hcat, int32_t ids_dtype,
                                int64_t batch, int32_t L, int32_t *out_item, int32_t *out_cate,
                                mrec_stream stream) {
  MREC_CHECK_ARG(iid && cid && his && hcat && out_item && out_cate, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0 && L >= 1 && ld_his >= L && ld_hcat >= L, "bad shape / strides");
  MREC_CHECK_ARG(ids_dtype == MREC_I32 || ids_dtype == MREC_I64, "ids must be int32 or int64");
  if (batch == 0) return MREC_OK;
  const int64_t n = batch * (L + 1);
  const dim3 g(static_cast<unsigned>((n + 255) / 256));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (ids_dtype == MREC_I32)
    din_ids_kernel<int32_t><<<g, 256, 0, s>>>(
        static_cast<const int32_t *>(iid), static_cast<const int32_t *>(cid),
        static_cast<const int32_t *>(his), ld_his, static_cast<const int32_t *>(hcat), ld_hcat,
        batch, L, out_item, out_cate);
  else
    din_ids_kernel<int64_t><<<g, 256, 0, s>>>(
        static_cast<const int64_t *>(iid), static_cast<const int64_t *>(cid),
        static_cast<const int64_t *>(his), ld_his, static_cast<const int64_t *>(hcat), ld_hcat,
        batch, L, out_item, out_cate);
  return launch_status("mrec_din_lookup_ids");
}

mrec_status mrec_din_gather(const mrec_table_bank *bank, const void *iid, const void *cid,
                            const void *his, int64_t ld_his, const void *hcat, int64_t ld_hcat,
                            int32_t ids_dtype, int64_t batch, int32_t L, int32_t *out_item,
                            int32_t *out_cate, void *out, mrec_dtype out_dtype, int64_t out_ld,
                            int32_t *d_oob_flag, mrec_stream stream) {
  BankArgs ba;
  int eb, lpr;
  mrec_status st = make_bank_args(bank, &ba, &eb, &lpr);
  if (st != MREC_OK) return st;
  MREC_CHECK_ARG(ba.n_tables == 2, "the DIN bank has two tables (item, category)");
  MREC_CHECK_ARG(!ba.adam.kind, "a lazily updated Adam bank reads rows through mrec_emb_gather_fwd");
  MREC_CHECK_ARG(iid && cid && his && hcat && out_item && out_cate && out, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0 && L >= 1 && ld_his >= L && ld_hcat >= L, "bad shape / strides");
  MREC_CHECK_ARG(ids_dtype == MREC_I32 || ids_dtype == MREC_I64, "ids must be int32 or int64");
  MREC_CHECK_ARG(out_dtype == MREC_F32 || out_dtype == MREC_BF16, "out dtype must be F32/BF16");
  const int ob = out_dtype == MREC_F32 ? 4 : 2;
  MREC_CHECK_ARG(out_ld >= 2 * ba.dim, "out_ld < 2 * dim");
  MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0 && (out_ld * ob) % 16 == 0 &&
                     (ba.dim * ob) % 16 == 0,
                 "out must be 16B aligned with 16B-multiple rows");
  MREC_CHECK_ARG(ba.rows[0] < INT32_MAX && ba.rows[1] < INT32_MAX,
                 "DIN padded lookups need tables of fewer than 2^31 - 1 rows");
  if (batch == 0) return MREC_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (ids_dtype == MREC_I32)
    din_gather_dispatch<int32_t>(bank->dtype, out_dtype, lpr, ba, iid, cid, his, ld_his, hcat,
                                 ld_hcat, batch, L, out_item, out_cate, out, out_ld, d_oob_flag, s);
  else
    din_gather_dispatch<int64_t>(bank->dtype, out_dtype, lpr, ba, iid, cid, his, ld_his, hcat,
                                 ld_hcat, batch, L, out_item, out_cate, out, out_ld, d_oob_flag, s);
  return launch_status("mrec_din_gather");
}

mrec_status mrec_din_feat_fwd(const void *q, int64_t ldq, const void *k, int64_t ldk,
                              int64_t batch, int32_t L, int32_t E, void *feat, int64_t ldf,
                              mrec_stream stream) {
  MREC_CHECK_ARG(q && k && feat, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0 && L >= 1 && L <= DIN_MAXL && E >= 8 && E <= DIN_MAXE && E % 8 == 0,
                 "need 1 <= L <= 64, 8 <= E <= 64, E % 8 == 0");
  MREC_CHECK_ARG(a16(q, ldq) && a16(k, ldk) && a16(feat, ldf) && ldf >= 4 * E,
                 "rows must be 16-byte aligned, ldf >= 4E");
  const int64_t rows = batch * L;
  if (rows == 0) return MREC_OK;
  const int64_t threads = rows * (E / 8);
  din_feat_fwd_kernel<<<dim3(static_cast<unsigned>((threads + 255) / 256)), 256, 0,
                        static_cast<hipStream_t>(stream)>>>(
      static_cast<const uint16_t *>(q), ldq, static_cast<const uint16_t *>(k), ldk, rows, L, E,
      static_cast<uint16_t *>(feat), ldf);
  return launch_status("mrec_din_feat_fwd");
}

mrec_status mrec_din_pool_fwd(const float *s, int64_t ld_s, const int32_t *his, int64_t ld_his,
                              const void *q,
                              int64_t ldq, const void *k, int64_t ldk, int64_t batch, int32_t L,
                              int32_t E, float *a, void *top, int64_t ldt, mrec_stream stream) {
  MREC_CHECK_ARG(s && his && q && k && a && top, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0 && L >= 1 && L <= DIN_MAXL && E >= 8 && E <= DIN_MAXE && E % 8 == 0,
                 "need 1 <= L <= 64, 8 <= E <= 64, E % 8 == 0");
  MREC_CHECK_ARG(a16(k, ldk) && ldt >= 2 * E && ld_his >= L && ld_s >= 1, "bad strides");
  if (batch == 0) return MREC_OK;
  din_pool_fwd_kernel<<<dim3(static_cast<unsigned>((batch + 3) / 4)), 256, 0,
                        static_cast<hipStream_t>(stream)>>>(
      s, ld_s, his, ld_his, static_cast<const uint16_t *>(q), ldq, static_cast<const uint16_t *>(k), ldk,
      batch, L, E, a, static_cast<uint16_t *>(top), ldt);
  return launch_status("mrec_din_pool_fwd");
}

mrec_status mrec_din_pool_bwd(const void *dtop, int64_t lddt, const float *a, const void *k,
                              int64_t ldk, int64_t batch, int32_t L, int32_t E, float *ds,
                              float *dk, int64_t lddk, mrec_stream stream) {
  MREC_CHECK_ARG(dtop && a && k && ds && dk, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0 && L >= 1 && L <= DIN_MAXL && E >= 8 && E <= DIN_MAXE && E % 8 == 0,
                 "need 1 <= L <= 64, 8 <= E <= 64, E % 8 == 0");
  MREC_CHECK_ARG(a16(dtop, lddt) && a16(k, ldk) && lddt >= 2 * E && lddk >= E, "bad strides");
  if (batch == 0) return MREC_OK;
  din_pool_bwd_kernel<<<dim3(static_cast<unsigned>((batch + 3) / 4)), 256, 0,
                        static_cast<hipStream_t>(stream)>>>(
      static_cast<const uint16_t *>(dtop), lddt, a, static_cast<const uint16_t *>(k), ldk, batch,
      L, E, ds, dk, lddk);
  return launch_status("mrec_din_pool_bwd");
}

mrec_status mrec_din_feat_bwd(const void *dfeat, int64_t lddf, const void *dtop, int64_t lddt,
                              const void *q, int64_t ldq, const void *k, int64_t ldk,
                              int64_t batch, int32_t L, int32_t E, float *dk, int64_t lddk,
                              float *dq, int64_t lddq, mrec_stream stream) {
  MREC_CHECK_ARG(dfeat && dtop && q && k && dk && dq, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0 && L >= 1 && L <= DIN_MAXL && E >= 8 && E <= DIN_MAXE && E % 8 == 0,
                 "need 1 <= L <= 64, 8 <= E <= 64, E % 8 == 0");
  MREC_CHECK_ARG(a16(dfeat, lddf) && a16(q, ldq) && a16(k, ldk) && lddf >= 4 * E && lddk >= E &&
                     lddq >= E,
                 "bad strides");
  if (batch == 0) return MREC_OK;
  din_feat_bwd_kernel<false><<<dim3(static_cast<unsigned>((batch + 3) / 4)), 256, 0,
                               static_cast<hipStream_t>(stream)>>>(
      static_cast<const uint16_t *>(dfeat), lddf, static_cast<const uint16_t *>(dtop), lddt,
      static_cast<const uint16_t *>(q), ldq, static_cast<const uint16_t *>(k), ldk, batch, L, E, dk,
      lddk, dq, lddq, nullptr, 0);
  return launch_status("mrec_din_feat_bwd");
}

mrec_status mrec_din_feat_bwd_rows(const void *dfeat, int64_t lddf, const void *dtop, int64_t lddt,
                                   const void *q, int64_t ldq, const void *k, int64_t ldk,
                                   int64_t batch, int32_t L, int32_t E, const float *dk,
                                   int64_t lddk, void *d_rows, int64_t ld_rows, mrec_stream stream) {
  MREC_CHECK_ARG(dfeat && dtop && q && k && dk && d_rows, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0 && L >= 1 && L <= DIN_MAXL && E >= 8 && E <= DIN_MAXE && E % 8 == 0,
                 "need 1 <= L <= 64, 8 <= E <= 64, E % 8 == 0");
  MREC_CHECK_ARG(a16(dfeat, lddf) && a16(q, ldq) && a16(k, ldk) && a16(d_rows, ld_rows) &&
                     lddf >= 4 * E && lddk >= E && ld_rows >= E,
                 "bad strides");
  if (batch == 0) return MREC_OK;
  din_feat_bwd_kernel<true><<<dim3(static_cast<unsigned>((batch + 3) / 4)), 256, 0,
                              static_cast<hipStream_t>(stream)>>>(
      static_cast<const uint16_t *>(dfeat), lddf, static_cast<const uint16_t *>(dtop), lddt,
      static_cast<const uint16_t *>(q), ldq, static_cast<const uint16_t *>(k), ldk, batch, L, E,
      const_cast<float *>(dk), lddk, nullptr, 0, static_cast<uint16_t *>(d_rows), ld_rows);
  return launch_status("mrec_din_feat_bwd_rows");
}

}  // extern "C"
