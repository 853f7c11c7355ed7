// Forward kernels: multi-table gather, fused gather + FM + first-order + deep
// input builder, standalone FM2.
//
// Row access: a table row is 16..256 bytes (a power of two), read by a "worker"
// of LPR = row_bytes/16 consecutive lanes with one 16-byte load each, so one
// wave-instruction reads 64/LPR whole rows, each as one contiguous request.
#include "common.h"
#include "emb_plan.h"

namespace mrec {

// ---------------------------------------------------------------------------
// plain gather: worker per (b, f) lookup
// ---------------------------------------------------------------------------
// ADAM: the bank trains with the lazy fused Adam (stale rows are caught up on
// read); a template flag so the common instantiation carries none of that code
template <typename T, typename O, int LPR, bool ADAM = false>
__global__ __launch_bounds__(256) void gather_kernel(BankArgs bank, IdsArgs ids, int64_t B,
                                                     O *__restrict__ out, int64_t out_ld,
                                                     float *__restrict__ w_out,
                                                     int32_t *__restrict__ oob) {
  constexpr int EPL = Vec<T>::EPL;
  constexpr int WPB = 256 / LPR;
  const int F = bank.n_tables;
  const int64_t g = static_cast<int64_t>(blockIdx.x) * WPB + threadIdx.x / LPR;
  const int l = threadIdx.x % LPR;
  if (g >= B * F) return;
  const int64_t b = g / F;
  const int f = static_cast<int>(g - b * F);
  const int64_t id = load_id(ids, f, b);
  const bool ok = id >= 0 && id < bank.rows[f];
  uint4 raw = make_uint4(0, 0, 0, 0);
  if (ok) {
    const T *row = reinterpret_cast<const T *>(bank.data) +
                   (bank.row_offset[f] + id) * static_cast<int64_t>(bank.row_stride);
    raw = *reinterpret_cast<const uint4 *>(row + l * EPL);
    if constexpr (ADAM)  // a lazily updated Adam bank: the row as of the last step
      raw = adam_current<T>(bank, bank.row_offset[f] + id, l * EPL, live_elems(bank, l * EPL, EPL),
                            raw, *bank.adam.d_t);
  } else if (l == 0 && oob && !(ids.pad_negative && id < 0)) {
    *oob = 1;  // (a negative id of a padded view is a zero row, skipped by the backward)
  }
  const int D = bank.dim;
  const int e0 = l * EPL;
  if (e0 + EPL <= D) {
    O *dst = out + b * out_ld + static_cast<int64_t>(f) * D + e0;
    if constexpr (sizeof(O) == sizeof(T)) {
      *reinterpret_cast<uint4 *>(dst) = raw;  // bit copy
    } else {
      float v[EPL];
      Vec<T>::to_f32(raw, v);
      if constexpr (sizeof(O) == 4) {  // widen bf16 -> f32 (exact)
#pragma unroll
        for (int j = 0; j < EPL; j += 4)
          *reinterpret_cast<float4 *>(dst + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
      } else {  // narrow f32 -> bf16 (RNE)
        *reinterpret_cast<uint2 *>(dst) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      }
    }
  } else if (w_out && bank.has_w && e0 == D) {
    float v[EPL];
    Vec<T>::to_f32(raw, v);
    w_out[b * F + f] = v[0];
  }
}

// ---------------------------------------------------------------------------
// fused interaction: one wave per sample
// ---------------------------------------------------------------------------
struct InteractArgs {
  const float *dense;
  int n_dense;
  int64_t dense_ld;
  const float *dense_w;
  const float *bias;
  int flags;
  void *x0v;
  int64_t x0_ld;
  int x0_cols;
  float *logit;
  float *fm_sum;
  int32_t *oob;
  // REC (mrec_interact_fwd_rec): rows from the compact exchange's wire records
  const uint32_t *rec_wire;  // [parts][cap_rows] records of rec_dw dwords
  const int32_t *rec_hdr;    // the ids message they answer: parts x (F * cap + F), counts last
  int rec_dw, rec_cap, rec_cap_rows, rec_parts;
  int32_t *rec_pref;         // out (nullable): [parts][F] table prefixes
  int32_t *rec_overflow;     // nullable: bit 1 = a part holds more than cap_rows records
};

#ifdef MREC_INTERACT_PROF
// diagnostics: per-sample wall-clock stamps (100 MHz) of the last launch: start,
// ids landed, rows landed, x0 / sums issued, logit issued (mrec_interact_prof_read)
__device__ uint64_t g_interact_prof[8192][5];
#define IA_STAMP(k, dep)                                                        \
  do {                                                                          \
    if (lane == 0 && b < 8192) {                                                \
      asm volatile("" ::"v"(dep));                                              \
      g_interact_prof[b][k] = __builtin_amdgcn_s_memrealtime();                 \
    }                                                                           \
  } while (0)
#else
#define IA_STAMP(k, dep) \
  do {                   \
  } while (0)
#endif

// sample b, by the wave whose lane this is.  REC: the bank is the sender's slot rows
// [(p * F + f) * cap + j] (ids = those slots), which are NOT filled yet: each row comes
// from its wire record p * cap_rows + pref[p][f] + j (s_pref: the parts' table
// prefixes in LDS) by dword loads (records are 4-B aligned), and is also written into
// its slot row -- the bytes mrec_shard_wire_unpack_ex would have written there (the
// record, zeros past it), which the sender's backward reads -- so the unpack launch
// is gone.  Lookups of one slot store the same bytes.
template <typename T, int LPR, bool X0_BF16, bool ADAM, bool REC = false>
__device__ __forceinline__ void interact_sample(const BankArgs &bank, const IdsArgs &ids,
                                                const InteractArgs &ia, int64_t b, int lane,
                                                const int32_t *s_pref = nullptr) {
  constexpr int EPL = Vec<T>::EPL;
  constexpr int WPW = 64 / LPR;                             // rows per wave-instruction
  constexpr int MAXIT = (MREC_MAX_TABLES + WPW - 1) / WPW;  // field iterations
  const float *__restrict__ dense = ia.dense;
  const int n_dense = ia.n_dense;
  const int64_t dense_ld = ia.dense_ld;
  const float *__restrict__ dense_w = ia.dense_w;
  const float *__restrict__ bias = ia.bias;
  const int flags = ia.flags;
  void *__restrict__ x0v = ia.x0v;
  const int64_t x0_ld = ia.x0_ld;
  const int x0_cols = ia.x0_cols;
  float *__restrict__ logit = ia.logit;
  float *__restrict__ fm_sum = ia.fm_sum;
  int32_t *__restrict__ oob = ia.oob;
  const int worker = lane / LPR;
  const int l = lane % LPR;
  const int e0 = l * EPL;
  const int F = bank.n_tables;
  const int D = bank.dim;
  const bool v_lane = e0 + EPL <= D;
  const bool w_lane = bank.has_w && e0 == D;

  // the dense features and their first-order weights depend on b only: loaded
  // first, so their latency hides under the id -> row chain (n_dense <= 64)
  const bool dense64 = n_dense <= 64;
  float dv = 0.f, dwv = 0.f;
  if (dense64 && lane < n_dense) {
    dv = dense[b * dense_ld + lane];
    if (dense_w) dwv = dense_w[lane];
  }
  // phase 1: issue every row load of this sample before consuming any
  IA_STAMP(0, 0);
#ifdef MREC_INTERACT_PROF
  {
    const int64_t id0 = load_id(ids, worker < F ? worker : 0, b);
    IA_STAMP(1, static_cast<int>(id0));
  }
#endif
  // The lane's field metadata (kernel-argument arrays indexed per lane: vector loads),
  // then its ids, then its rows, each group issued unconditionally (a clamped field /
  // row, masked afterwards): under `if (valid)` every loaded value was copied out of
  // its branch and the copy waited for it, which chained ~5 round trips per field.
  uint4 raw[MAXIT];
  const void *fptr[MAXIT];
  int64_t frows[MAXIT], foff[MAXIT], idv[MAXIT];
  bool okv[MAXIT];
  // (iterations past the last field load table F - 1's id again: no branch per
  // iteration, whose join would wait for the load)
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) {
    const int fc = min(it * WPW + worker, F - 1);
    fptr[it] = ids.ptr[fc];
    frows[it] = bank.rows[fc];
    foff[it] = bank.row_offset[fc];
  }
  if (ids.chunk) {  // (uniform) chunked views: the per-element path
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) idv[it] = load_id(ids, min(it * WPW + worker, F - 1), b);
  } else if (ids.is64) {
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) idv[it] = static_cast<const int64_t *>(fptr[it])[b * ids.stride];
  } else {
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) idv[it] = static_cast<const int32_t *>(fptr[it])[b * ids.stride];
  }
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) {
    raw[it] = make_uint4(0, 0, 0, 0);
    okv[it] = false;
    if (it * WPW >= F) continue;  // uniform
    okv[it] = it * WPW + worker < F && idv[it] >= 0 && idv[it] < frows[it];
    if constexpr (REC) {
      // slot s of table fc -> its record; dwords 4 l .. 4 l + 3 of the row (past the
      // record: zeros), every load from a clamped index, masked below
      const int fc = min(it * WPW + worker, F - 1);
      const uint32_t sl = okv[it] ? static_cast<uint32_t>(idv[it]) : 0u;
      const uint32_t fcap = static_cast<uint32_t>(F) * static_cast<uint32_t>(ia.rec_cap);
      const uint32_t pp = sl / fcap;
      const int32_t j = static_cast<int32_t>(sl - (pp * F + fc) * static_cast<uint32_t>(ia.rec_cap));
      const int32_t r = s_pref[pp * F + fc] + j;
      okv[it] = okv[it] && j >= 0 && j < ia.rec_cap && r < ia.rec_cap_rows;
      const uint32_t *src = ia.rec_wire + (static_cast<int64_t>(pp) * ia.rec_cap_rows + (okv[it] ? r : 0)) *
                                              ia.rec_dw;
      uint32_t w4[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) w4[k] = src[min(4 * l + k, ia.rec_dw - 1)];
#pragma unroll
      for (int k = 0; k < 4; ++k) w4[k] = 4 * l + k < ia.rec_dw ? w4[k] : 0u;
      raw[it] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    } else {
      const int64_t grow = okv[it] ? foff[it] + idv[it] : 0;
      raw[it] = *reinterpret_cast<const uint4 *>(reinterpret_cast<const T *>(bank.data) +
                                                 grow * static_cast<int64_t>(bank.row_stride) + e0);
    }
  }
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) {
    if (it * WPW >= F) continue;  // uniform
    const int f = it * WPW + worker;
    if (!okv[it]) {
      raw[it] = make_uint4(0, 0, 0, 0);
      if (f < F && l == 0 && oob) *oob = 1;
    } else if constexpr (ADAM) {  // a lazily updated Adam bank: the row as of the last step
      raw[it] = adam_current<T>(bank, foff[it] + idv[it], e0, live_elems(bank, e0, EPL), raw[it],
                                *bank.adam.d_t);
    }
  }
  if constexpr (REC) {  // the slot rows the backward reads (the unpack's bytes)
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      if (it * WPW >= F) continue;  // uniform
      if (okv[it])
        *reinterpret_cast<uint4 *>(reinterpret_cast<T *>(bank.data) +
                                   idv[it] * static_cast<int64_t>(bank.row_stride) + e0) = raw[it];
    }
  }

  IA_STAMP(2, raw[0].x ^ raw[MAXIT - 1].x);
  // phase 2: per-lane sums over this lane's fields + deep-input write
  float s[EPL], q[EPL];
#pragma unroll
  for (int j = 0; j < EPL; ++j) s[j] = q[j] = 0.f;
  float wsum = 0.f;
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) {
    const int f = it * WPW + worker;
    if (it * WPW >= F || f >= F) continue;
    float v[EPL];
    Vec<T>::to_f32(raw[it], v);
    if (v_lane) {
#pragma unroll
      for (int j = 0; j < EPL; ++j) {
        s[j] += v[j];
        q[j] = fmaf(v[j], v[j], q[j]);
      }
      if (x0v) {
        const int64_t o = b * x0_ld + static_cast<int64_t>(f) * D + e0;
        if constexpr (X0_BF16) {
          uint16_t *dst = static_cast<uint16_t *>(x0v) + o;
          if constexpr (sizeof(T) == 2) {
            *reinterpret_cast<uint4 *>(dst) = raw[it];
          } else {
            *reinterpret_cast<uint2 *>(dst) =
                make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
          }
        } else {
          float *dst = static_cast<float *>(x0v) + o;
#pragma unroll
          for (int j = 0; j < EPL; j += 4)
            *reinterpret_cast<float4 *>(dst + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
        }
      }
    } else if (w_lane) {
      wsum += v[0];
    }
  }

  // reduce over workers (lanes with equal l): sum_d S_d^2 - sum_{f,d} v_fd^2, so
  // each lane folds its squares first and the workers reduce EPL + 2 values
  float qt = 0.f;
#pragma unroll
  for (int j = 0; j < EPL; ++j) qt += q[j];
  float fm = 0.f;
  if constexpr (LPR == 4) {  // DPP rows + permlane swaps (common.h), no LDS traffic
#pragma unroll
    for (int j = 0; j < EPL; ++j) s[j] = sum_mod4_lanes(s[j]);
    qt = sum_mod4_lanes(qt);
    wsum = sum_mod4_lanes(wsum);
    if (v_lane) {
#pragma unroll
      for (int j = 0; j < EPL; ++j) fm = fmaf(s[j], s[j], fm);
      fm -= qt;
    }
    fm = sum_quad(fm);
    wsum = sum_quad(wsum);
  } else {
#pragma unroll
    for (int off = LPR; off < 64; off <<= 1) {
#pragma unroll
      for (int j = 0; j < EPL; ++j) s[j] += __shfl_xor(s[j], off);
      qt += __shfl_xor(qt, off);
      wsum += __shfl_xor(wsum, off);
    }
    if (v_lane) {
#pragma unroll
      for (int j = 0; j < EPL; ++j) fm = fmaf(s[j], s[j], fm);
      fm -= qt;
    }
#pragma unroll
    for (int off = 1; off < LPR; off <<= 1) {
      fm += __shfl_xor(fm, off);
      wsum += __shfl_xor(wsum, off);
    }
  }
  if (fm_sum && worker == 0 && v_lane) {
    float *dst = fm_sum + b * D + e0;
#pragma unroll
    for (int j = 0; j < EPL; j += 4)
      *reinterpret_cast<float4 *>(dst + j) = make_float4(s[j], s[j + 1], s[j + 2], s[j + 3]);
  }

  IA_STAMP(3, __float_as_int(fm));
  // dense features: first-order dot + copy into x0, zero the pad columns
  float ds = 0.f;
  if (dense64)
    ds = dv * dwv;
  else if (dense_w)
    for (int j = lane; j < n_dense; j += 64) ds = fmaf(dense[b * dense_ld + j], dense_w[j], ds);
  ds = sum_wave(ds);
  if (x0v) {
    const int base = F * D;
    for (int c = base + lane; c < x0_cols; c += 64) {
      const int j = c - base;
      const float x = j < n_dense ? (dense64 && j == lane ? dv : dense[b * dense_ld + j]) : 0.f;
      if constexpr (X0_BF16)
        static_cast<uint16_t *>(x0v)[b * x0_ld + c] = f32_to_bf16_rne(x);
      else
        static_cast<float *>(x0v)[b * x0_ld + c] = x;
    }
  }
  if (lane == 0 && logit) {
    float y = (bias ? bias[0] : 0.f) + ds;
    if (flags & MREC_INTERACT_FM2) y += 0.5f * fm;
    if (flags & MREC_INTERACT_FIRST_ORDER) y += wsum;
    logit[b] = y;
  }
  IA_STAMP(4, __float_as_int(ds));
}

template <typename T, int LPR, bool X0_BF16, bool ADAM>
__global__ __launch_bounds__(256) void interact_kernel(BankArgs bank, IdsArgs ids, int64_t B,
                                                       InteractArgs ia) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  interact_sample<T, LPR, X0_BF16, ADAM>(bank, ids, ia, b, threadIdx.x & 63);
}

// the interaction (16 samples per 1024-thread workgroup) with the embedding-
// backward hash plan in the leading workgroups: a HIP graph runs the step's
// kernels one after another, so the plan would otherwise cost a kernel of its own
template <typename T, int LPR, bool X0_BF16, bool ADAM, bool KC>
__global__ __launch_bounds__(1024) void interact_plan_kernel(BankArgs bank, IdsArgs ids, int64_t B,
                                                             InteractArgs ia, PlanJob plan,
                                                             int plan_blocks, KClock kc) {
  __shared__ __attribute__((aligned(16))) uint32_t smem[2 * kHashSlots + 2];
  KcScope<KC> kc_scope(kc);
  if (static_cast<int>(blockIdx.x) < plan_blocks) {  // uniform: (table, bucket) plans
    plan_hash_body<1024, kHashSlots>(plan.bank, plan.ids, plan.B, plan.ws, plan.oob, plan.d_step,
                                     blockIdx.x / kPlanBuckets, blockIdx.x % kPlanBuckets, smem);
    return;
  }
  const int64_t b = static_cast<int64_t>(blockIdx.x - plan_blocks) * 16 + (threadIdx.x >> 6);
  if (b >= B) return;
  interact_sample<T, LPR, X0_BF16, ADAM>(bank, ids, ia, b, threadIdx.x & 63);
}

// the same launch over the compact exchange's wire records (interact_sample REC):
// every sample workgroup first builds the parts' table prefixes in LDS (the running
// sums of the counts the ids message carries, as the unpack did); the first one also
// writes them out for the sender's gradient records (mrec_emb_bwd_apply_rec)
template <typename T, int LPR, bool X0_BF16, bool KC>
__global__ __launch_bounds__(1024) void interact_rec_kernel(BankArgs bank, IdsArgs ids, int64_t B,
                                                            InteractArgs ia, PlanJob plan,
                                                            int plan_blocks, KClock kc) {
  __shared__ __attribute__((aligned(16))) uint32_t smem[2 * kHashSlots + 2];
  KcScope<KC> kc_scope(kc);
  if (static_cast<int>(blockIdx.x) < plan_blocks) {  // uniform: (table, bucket) plans
    plan_hash_body<1024, kHashSlots>(plan.bank, plan.ids, plan.B, plan.ws, plan.oob, plan.d_step,
                                     blockIdx.x / kPlanBuckets, blockIdx.x % kPlanBuckets, smem);
    return;
  }
  const int F = bank.n_tables;
  int32_t *s_pref = reinterpret_cast<int32_t *>(smem);  // [parts][F] (host: parts * F <= 8192)
  {
    // one wave per part (lane = table, F <= 64): the counts by one load per lane, the
    // exclusive prefix by a shuffle scan (a per-thread array of 64 counts cost 64
    // VGPRs: 6 instead of 8 waves per SIMD, half the workgroups resident)
    const int lane = threadIdx.x & 63;
    const bool first = static_cast<int>(blockIdx.x) == plan_blocks;
    for (int p = threadIdx.x >> 6; p < ia.rec_parts; p += 16) {
      const int32_t *h = ia.rec_hdr + static_cast<int64_t>(p) * (static_cast<int64_t>(F) * ia.rec_cap + F) +
                         static_cast<int64_t>(F) * ia.rec_cap;
      const int32_t c = lane < F ? h[lane] : 0;
      int32_t incl = c;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int32_t t = __shfl_up(incl, off);
        if (lane >= off) incl += t;
      }
      if (lane < F) {
        s_pref[p * F + lane] = incl - c;
        if (first && ia.rec_pref) ia.rec_pref[p * F + lane] = incl - c;
      }
      if (first && lane == 63 && incl > ia.rec_cap_rows && ia.rec_overflow)
        atomicOr(ia.rec_overflow, 2);
    }
  }
  __syncthreads();
  const int64_t b = static_cast<int64_t>(blockIdx.x - plan_blocks) * 16 + (threadIdx.x >> 6);
  if (b >= B) return;
  interact_sample<T, LPR, X0_BF16, false, true>(bank, ids, ia, b, threadIdx.x & 63, s_pref);
}

// ---------------------------------------------------------------------------
// standalone FM2 on [B, F, D] fp32: one wave per sample, lanes over d
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fm2_fwd_kernel(const float *__restrict__ v, int64_t B,
                                                      int F, int D, float *__restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float *vb = v + b * F * D;
  float acc = 0.f;
  for (int d = lane; d < D; d += 64) {
    float s = 0.f, q = 0.f;
    for (int f = 0; f < F; ++f) {
      const float x = vb[f * D + d];
      s += x;
      q = fmaf(x, x, q);
    }
    acc += s * s - q;
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) acc += __shfl_xor(acc, off);
  if (lane == 0) y[b] = 0.5f * acc;
}

__global__ __launch_bounds__(256) void fm2_bwd_kernel(const float *__restrict__ v,
                                                      const float *__restrict__ dy, int64_t B,
                                                      int F, int D, float *__restrict__ dv) {
  const int lane = threadIdx.x & 63;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float *vb = v + b * F * D;
  float *gb = dv + b * F * D;
  const float g = dy[b];
  for (int d = lane; d < D; d += 64) {
    float s = 0.f;
    for (int f = 0; f < F; ++f) s += vb[f * D + d];
    for (int f = 0; f < F; ++f) gb[f * D + d] = g * (s - vb[f * D + d]);
  }
}

// ---------------------------------------------------------------------------
// dispatch helpers
// ---------------------------------------------------------------------------
template <typename T, typename O>
static void launch_gather(int lpr, const BankArgs &ba, const IdsArgs &ia, int64_t B, void *out,
                          int64_t out_ld, float *w_out, int32_t *oob, hipStream_t s) {
  const int64_t work = B * ba.n_tables;
  const int wpb = 256 / lpr;
  const dim3 grid(static_cast<unsigned>((work + wpb - 1) / wpb));
  O *o = static_cast<O *>(out);
#define MREC_GK(A)                                                                                \
  switch (lpr) {                                                                                  \
    case 1: gather_kernel<T, O, 1, A><<<grid, 256, 0, s>>>(ba, ia, B, o, out_ld, w_out, oob); break; \
    case 2: gather_kernel<T, O, 2, A><<<grid, 256, 0, s>>>(ba, ia, B, o, out_ld, w_out, oob); break; \
    case 4: gather_kernel<T, O, 4, A><<<grid, 256, 0, s>>>(ba, ia, B, o, out_ld, w_out, oob); break; \
    case 8: gather_kernel<T, O, 8, A><<<grid, 256, 0, s>>>(ba, ia, B, o, out_ld, w_out, oob); break; \
    default: gather_kernel<T, O, 16, A><<<grid, 256, 0, s>>>(ba, ia, B, o, out_ld, w_out, oob); break; \
  }
  if (ba.adam.kind) {
    MREC_GK(true)
  } else {
    MREC_GK(false)
  }
#undef MREC_GK
}

template <typename T, bool XB>
static void launch_interact(int lpr, const BankArgs &ba, const IdsArgs &ids, int64_t B,
                            const InteractArgs &ia, const PlanJob *plan, hipStream_t s) {
  const int pb = plan ? plan->bank.n_tables * kPlanBuckets : 0;
  const dim3 grid(static_cast<unsigned>((B + 3) / 4));
  const dim3 grid_p(static_cast<unsigned>(pb + (B + 15) / 16));
  const KClock kc = plan ? kclock_take() : KClock{nullptr, 0};  // (the fused step's launch)
#define MREC_IKA(L, A)                                                                      \
  do {                                                                                      \
    if (plan && kc.buf)                                                                     \
      interact_plan_kernel<T, L, XB, A, true><<<grid_p, 1024, 0, s>>>(ba, ids, B, ia, *plan, \
                                                                      pb, kc);              \
    else if (plan)                                                                          \
      interact_plan_kernel<T, L, XB, A, false><<<grid_p, 1024, 0, s>>>(ba, ids, B, ia,      \
                                                                       *plan, pb, kc);      \
    else                                                                                    \
      interact_kernel<T, L, XB, A><<<grid, 256, 0, s>>>(ba, ids, B, ia);                    \
  } while (0)
#define MREC_IK(L)              \
  do {                          \
    if (ba.adam.kind)           \
      MREC_IKA(L, true);        \
    else                        \
      MREC_IKA(L, false);       \
  } while (0)
  switch (lpr) {
    case 1: MREC_IK(1); break;
    case 2: MREC_IK(2); break;
    case 4: MREC_IK(4); break;
    case 8: MREC_IK(8); break;
    default: MREC_IK(16); break;
  }
#undef MREC_IK
#undef MREC_IKA
}

}  // namespace mrec

using namespace mrec;

extern "C" {

mrec_status mrec_emb_gather_fwd(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                                void *out, mrec_dtype out_dtype, int64_t out_ld, float *w_out,
                                int32_t *d_oob_flag, mrec_stream stream) {
  BankArgs ba;
  IdsArgs ia;
  int eb, lpr;
  mrec_status st = make_bank_args(bank, &ba, &eb, &lpr);
  if (st != MREC_OK) return st;
  if ((st = make_ids_args(ids, ba.n_tables, &ia)) != MREC_OK) return st;
  MREC_CHECK_ARG(batch >= 0, "batch < 0");
  MREC_CHECK_ARG(out != nullptr, "out is NULL");
  MREC_CHECK_ARG(out_dtype == MREC_F32 || out_dtype == MREC_BF16, "out dtype must be F32/BF16");
  const int ob = out_dtype == MREC_F32 ? 4 : 2;
  MREC_CHECK_ARG(out_ld >= static_cast<int64_t>(ba.n_tables) * ba.dim, "out_ld < n_tables*dim");
  MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0 && (out_ld * ob) % 16 == 0 &&
                     (ba.dim * ob) % 16 == 0,
                 "out must be 16B aligned with 16B-multiple rows");
  MREC_CHECK_ARG(w_out == nullptr || ba.has_w, "w_out requested but bank has no w column");
  if (batch == 0) return MREC_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (bank->dtype == MREC_BF16) {
    if (out_dtype == MREC_BF16)
      launch_gather<uint16_t, uint16_t>(lpr, ba, ia, batch, out, out_ld, w_out, d_oob_flag, s);
    else
      launch_gather<uint16_t, float>(lpr, ba, ia, batch, out, out_ld, w_out, d_oob_flag, s);
  } else {
    if (out_dtype == MREC_BF16)
      launch_gather<float, uint16_t>(lpr, ba, ia, batch, out, out_ld, w_out, d_oob_flag, s);
    else
      launch_gather<float, float>(lpr, ba, ia, batch, out, out_ld, w_out, d_oob_flag, s);
  }
  return launch_status("mrec_emb_gather_fwd");
}

mrec_status mrec_interact_fwd(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                              const float *dense, int32_t n_dense, int64_t dense_ld,
                              const float *dense_w, const float *bias, int32_t flags, void *x0,
                              mrec_dtype x0_dtype, int64_t x0_ld, int32_t x0_cols, float *logit,
                              float *fm_sum, int32_t *d_oob_flag, mrec_stream stream) {
  return mrec_interact_fwd_ex(bank, ids, batch, dense, n_dense, dense_ld, dense_w, bias, flags, x0,
                              x0_dtype, x0_ld, x0_cols, logit, fm_sum, d_oob_flag, nullptr, stream);
}

mrec_status mrec_interact_fwd_ex(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                                 const float *dense, int32_t n_dense, int64_t dense_ld,
                                 const float *dense_w, const float *bias, int32_t flags, void *x0,
                                 mrec_dtype x0_dtype, int64_t x0_ld, int32_t x0_cols, float *logit,
                                 float *fm_sum, int32_t *d_oob_flag, const mrec_plan_job *plan,
                                 mrec_stream stream) {
  return mrec_interact_fwd_rec(bank, ids, batch, dense, n_dense, dense_ld, dense_w, bias, flags,
                               x0, x0_dtype, x0_ld, x0_cols, logit, fm_sum, d_oob_flag, plan,
                               nullptr, stream);
}

mrec_status mrec_interact_fwd_rec(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                                  const float *dense, int32_t n_dense, int64_t dense_ld,
                                  const float *dense_w, const float *bias, int32_t flags, void *x0,
                                  mrec_dtype x0_dtype, int64_t x0_ld, int32_t x0_cols, float *logit,
                                  float *fm_sum, int32_t *d_oob_flag, const mrec_plan_job *plan,
                                  const mrec_wire_rows *rec, mrec_stream stream) {
  BankArgs ba;
  IdsArgs ia;
  int eb, lpr;
  mrec_status st = make_bank_args(bank, &ba, &eb, &lpr);
  if (st != MREC_OK) return st;
  if ((st = make_ids_args(ids, ba.n_tables, &ia)) != MREC_OK) return st;
  MREC_CHECK_ARG(batch >= 0, "batch < 0");
  MREC_CHECK_ARG(n_dense >= 0, "n_dense < 0");
  MREC_CHECK_ARG(n_dense == 0 || (dense != nullptr && dense_ld >= n_dense),
                 "dense NULL or dense_ld < n_dense");
  MREC_CHECK_ARG(!(flags & MREC_INTERACT_FIRST_ORDER) || ba.has_w,
                 "FIRST_ORDER requested but bank has no w column");
  if (x0) {
    MREC_CHECK_ARG(x0_dtype == MREC_F32 || x0_dtype == MREC_BF16, "x0 dtype must be F32/BF16");
    const int xb = x0_dtype == MREC_F32 ? 4 : 2;
    MREC_CHECK_ARG(x0_cols >= ba.n_tables * ba.dim + n_dense && x0_ld >= x0_cols,
                   "x0_cols < F*dim + n_dense or x0_ld < x0_cols");
    MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(x0) & 15) == 0 && (x0_ld * xb) % 16 == 0 &&
                       (ba.dim * xb) % 16 == 0,
                   "x0 must be 16B aligned with 16B-multiple rows");
  }
  MREC_CHECK_ARG(fm_sum == nullptr || (reinterpret_cast<uintptr_t>(fm_sum) & 15) == 0,
                 "fm_sum not 16B aligned");
  PlanJob pj;
  if (plan) {
    if ((st = build_plan_job(plan, &pj)) != MREC_OK) return st;
  }
  if (batch == 0) return MREC_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool xb16 = x0 && x0_dtype == MREC_BF16;
  InteractArgs args{};
  args.dense = dense;
  args.n_dense = n_dense;
  args.dense_ld = dense_ld;
  args.dense_w = dense_w;
  args.bias = bias;
  args.flags = flags;
  args.x0v = x0;
  args.x0_ld = x0_ld;
  args.x0_cols = x0_cols;
  args.logit = logit;
  args.fm_sum = fm_sum;
  args.oob = d_oob_flag;
  const PlanJob *pp = plan ? &pj : nullptr;
  if (rec) {
    MREC_CHECK_ARG(bank->dtype == MREC_BF16 && lpr == 4 && !ba.adam.kind,
                   "records: bf16 slot rows of 64 B, no Adam catch-up (else unpack them)");
    MREC_CHECK_ARG(rec->wire && rec->hdr, "records: NULL wire / hdr");
    MREC_CHECK_ARG(rec->rec_bytes >= 4 && rec->rec_bytes % 4 == 0 &&
                       rec->rec_bytes <= ba.row_stride * eb &&
                       (reinterpret_cast<uintptr_t>(rec->wire) & 3) == 0,
                   "records: 4-B multiple no wider than a slot row, 4-B aligned wire");
    MREC_CHECK_ARG(rec->parts >= 1 && rec->cap >= 1 && rec->cap_rows >= 1 &&
                       static_cast<int64_t>(rec->parts) * ba.n_tables <= 8192 &&
                       rec->parts <= 1024,
                   "records: parts in [1, 1024], parts * n_tables <= 8192, cap / cap_rows >= 1");
    for (int f = 0; f < ba.n_tables; ++f)
      MREC_CHECK_ARG(ba.row_offset[f] == 0 &&
                         ba.rows[f] == static_cast<int64_t>(rec->parts) * ba.n_tables * rec->cap,
                     "records: the bank must be the slot rows (every table = all parts x tables x cap)");
    args.rec_wire = static_cast<const uint32_t *>(rec->wire);
    args.rec_hdr = rec->hdr;
    args.rec_dw = rec->rec_bytes / 4;
    args.rec_cap = rec->cap;
    args.rec_cap_rows = rec->cap_rows;
    args.rec_parts = rec->parts;
    args.rec_pref = rec->pref;
    args.rec_overflow = rec->d_overflow;
    const int pb = pp ? pp->bank.n_tables * kPlanBuckets : 0;
    const dim3 grid(static_cast<unsigned>(pb + (batch + 15) / 16));
    const KClock kc = kclock_take();
    PlanJob none{};
    const PlanJob &job = pp ? *pp : none;
#define MREC_IRK(XB)                                                                          \
  do {                                                                                        \
    if (kc.buf)                                                                               \
      interact_rec_kernel<uint16_t, 4, XB, true><<<grid, 1024, 0, s>>>(ba, ia, batch, args,   \
                                                                      job, pb, kc);           \
    else                                                                                      \
      interact_rec_kernel<uint16_t, 4, XB, false><<<grid, 1024, 0, s>>>(ba, ia, batch, args,  \
                                                                       job, pb, kc);          \
  } while (0)
    if (xb16)
      MREC_IRK(true);
    else
      MREC_IRK(false);
#undef MREC_IRK
    return launch_status("mrec_interact_fwd_rec");
  }
  if (bank->dtype == MREC_BF16) {
    if (xb16)
      launch_interact<uint16_t, true>(lpr, ba, ia, batch, args, pp, s);
    else
      launch_interact<uint16_t, false>(lpr, ba, ia, batch, args, pp, s);
  } else {
    if (xb16)
      launch_interact<float, true>(lpr, ba, ia, batch, args, pp, s);
    else
      launch_interact<float, false>(lpr, ba, ia, batch, args, pp, s);
  }
  return launch_status("mrec_interact_fwd");
}

mrec_status mrec_fm2_fwd(const float *v, int64_t batch, int32_t fields, int32_t dim, float *y,
                         mrec_stream stream) {
  MREC_CHECK_ARG(v != nullptr && y != nullptr, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0 && fields >= 1 && dim >= 1, "bad shape");
  if (batch == 0) return MREC_OK;
  fm2_fwd_kernel<<<dim3(static_cast<unsigned>((batch + 3) / 4)), 256, 0,
                   static_cast<hipStream_t>(stream)>>>(v, batch, fields, dim, y);
  return launch_status("mrec_fm2_fwd");
}

mrec_status mrec_fm2_bwd(const float *v, const float *dy, int64_t batch, int32_t fields,
                         int32_t dim, float *dv, mrec_stream stream) {
  MREC_CHECK_ARG(v != nullptr && dy != nullptr && dv != nullptr, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0 && fields >= 1 && dim >= 1, "bad shape");
  if (batch == 0) return MREC_OK;
  fm2_bwd_kernel<<<dim3(static_cast<unsigned>((batch + 3) / 4)), 256, 0,
                   static_cast<hipStream_t>(stream)>>>(v, dy, batch, fields, dim, dv);
  return launch_status("mrec_fm2_bwd");
}

}  // extern "C"

#ifdef MREC_INTERACT_PROF
extern "C" void mrec_interact_prof_read(uint64_t *out, int n) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(mrec::g_interact_prof), sizeof(uint64_t) * 5 * n);
}
#endif
