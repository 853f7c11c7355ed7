// Embedding backward: deterministic sorted-segment scatter-add with a fused
// row-sparse update.
//
// plan  : one 1024-thread workgroup per table sorts its (id, sample) keys with
//         an LDS bitonic network (<= 16384 keys, 128 KiB of LDS), then emits the
//         permutation, the unique rows and their segment starts.  Depends only on
//         the ids, so it can overlap the MLP forward on a side stream.
// apply : one LPR-lane worker per unique row sums the per-lookup gradients of
//         its segment in fp32, ascending sample order (bitwise reproducible), and
//         updates the row once (SGD, or accumulates a dense grad).  Segments
//         longer than SHORT_SEG (hot Zipf rows) are summed by the whole workgroup
//         with a fixed-order LDS tree so one hot row cannot serialise a worker.
#include "common.h"

namespace mrec {

constexpr int kPlanThreads = 1024;
constexpr int kMaxPlanKeys = 16384;
constexpr int kShortSeg = 16;

struct TableWs {  // per-table workspace view
  int32_t *hdr;   // [4] = {n_unique, n_valid, 0, 0}
  int32_t *perm;  // [Bp]   sample index of sorted position i
  int32_t *seg;   // [Bp+1] segment starts
  int32_t *uniq;  // [Bp]   local row id of segment u
};

__host__ __device__ inline int64_t pad4(int64_t x) { return (x + 3) & ~int64_t(3); }

__host__ __device__ inline int64_t table_ws_bytes(int64_t batch) {
  const int64_t bp = pad4(batch);
  int64_t bytes = 4 * (4 + bp + (bp + 4) + bp);
  return (bytes + 255) & ~int64_t(255);
}

__host__ __device__ inline TableWs table_ws(const void *ws, int f, int64_t batch) {
  char *base = static_cast<char *>(const_cast<void *>(ws)) + f * table_ws_bytes(batch);
  const int64_t bp = pad4(batch);
  TableWs t;
  t.hdr = reinterpret_cast<int32_t *>(base);
  t.perm = t.hdr + 4;
  t.seg = t.perm + bp;
  t.uniq = t.seg + bp + 4;
  return t;
}

// ---------------------------------------------------------------------------
// plan
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kPlanThreads) void plan_kernel(BankArgs bank, IdsArgs ids, int64_t B,
                                                            int NP, void *ws,
                                                            int32_t *__restrict__ oob) {
  __shared__ uint64_t keys[kMaxPlanKeys];
  __shared__ int32_t wsum[kPlanThreads / 64 + 1];
  __shared__ int32_t s_nvalid;
  const int f = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t rows = bank.rows[f];
  if (tid == 0) s_nvalid = 0;
  for (int i = tid; i < NP; i += kPlanThreads) {
    uint64_t key = ~0ull;
    if (i < B) {
      const int64_t id = load_id(ids, f, i);
      if (id >= 0 && id < rows) {
        key = (static_cast<uint64_t>(id) << 32) | static_cast<uint32_t>(i);
      } else {
        key = (0xffffffffull << 32) | static_cast<uint32_t>(i);
        if (oob) *oob = 1;
      }
    }
    keys[i] = key;
  }
  __syncthreads();
  // bitonic network, ascending; every thread owns NP/2/threads comparators
  for (int k = 2; k <= NP; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int p = tid; p < (NP >> 1); p += kPlanThreads) {
        const int i = 2 * j * (p / j) + (p % j);
        const int ix = i + j;
        const uint64_t a = keys[i], c = keys[ix];
        const bool up = (i & k) == 0;
        if ((a > c) == up) {
          keys[i] = c;
          keys[ix] = a;
        }
      }
      __syncthreads();
    }
  }
  // segment heads: contiguous chunk per thread, block exclusive scan of counts
  const int chunk = (NP + kPlanThreads - 1) / kPlanThreads;
  const int lo = tid * chunk;
  const int hi = min(lo + chunk, NP);
  int cnt = 0;
  for (int i = lo; i < hi; ++i) {
    const uint32_t id = static_cast<uint32_t>(keys[i] >> 32);
    const bool valid = id != 0xffffffffu;
    if (valid && (i == 0 || static_cast<uint32_t>(keys[i - 1] >> 32) != id)) ++cnt;
    if (valid && (i + 1 == NP || static_cast<uint32_t>(keys[i + 1] >> 32) == 0xffffffffu))
      s_nvalid = i + 1;  // exactly one writer: the last valid position
  }
  const int lane = tid & 63, wid = tid >> 6;
  int incl = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(incl, off);
    if (lane >= off) incl += t;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int w = 0; w < kPlanThreads / 64; ++w) {
      const int t = wsum[w];
      wsum[w] = run;
      run += t;
    }
    wsum[kPlanThreads / 64] = run;
  }
  __syncthreads();
  int u = wsum[wid] + incl - cnt;  // exclusive prefix
  TableWs t = table_ws(ws, f, B);
  const int nvalid = s_nvalid;
  for (int i = lo; i < hi; ++i) {
    const uint64_t key = keys[i];
    const uint32_t id = static_cast<uint32_t>(key >> 32);
    if (id == 0xffffffffu) break;
    t.perm[i] = static_cast<int32_t>(key & 0xffffffffu);
    if (i == 0 || static_cast<uint32_t>(keys[i - 1] >> 32) != id) {
      t.seg[u] = i;
      t.uniq[u] = static_cast<int32_t>(id);
      ++u;
    }
  }
  if (tid == 0) {
    const int nu = wsum[kPlanThreads / 64];
    t.hdr[0] = nu;
    t.hdr[1] = nvalid;
    t.seg[nu] = nvalid;
  }
}

// ---------------------------------------------------------------------------
// apply
// ---------------------------------------------------------------------------
struct ApplyArgs {
  const void *dx;
  int64_t dx_ld;
  int dx_bf16;
  const float *dfm;
  const float *fm_sum;
  const void *x0;
  int64_t x0_ld;
  int x0_bf16;
  const float *dw;
  int mode;
  float lr;
  uint64_t seed;
  void *grad;
};

template <int EPL>
__device__ __forceinline__ void load_f32xN(const float *p, float *v) {
#pragma unroll
  for (int j = 0; j < EPL; j += 4) {
    const float4 x = *reinterpret_cast<const float4 *>(p + j);
    v[j] = x.x;
    v[j + 1] = x.y;
    v[j + 2] = x.z;
    v[j + 3] = x.w;
  }
}

template <int EPL>
__device__ __forceinline__ void load_bf16xN(const uint16_t *p, float *v) {
  if constexpr (EPL == 8) {
    Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(p), v);
  } else {
    const uint2 r = *reinterpret_cast<const uint2 *>(p);
    v[0] = __uint_as_float(r.x << 16);
    v[1] = __uint_as_float(r.x & 0xffff0000u);
    v[2] = __uint_as_float(r.y << 16);
    v[3] = __uint_as_float(r.y & 0xffff0000u);
  }
}

// gradient of lookup (b, f) for this lane's EPL elements, added into acc
template <int EPL>
__device__ __forceinline__ void add_lookup_grad(const ApplyArgs &a, int64_t b, int f, int D,
                                                int e0, bool v_lane, bool w_lane, float *acc) {
  if (v_lane) {
    const int64_t col = static_cast<int64_t>(f) * D + e0;
    float g[EPL];
    if (a.dx) {
      if (a.dx_bf16)
        load_bf16xN<EPL>(static_cast<const uint16_t *>(a.dx) + b * a.dx_ld + col, g);
      else
        load_f32xN<EPL>(static_cast<const float *>(a.dx) + b * a.dx_ld + col, g);
#pragma unroll
      for (int j = 0; j < EPL; ++j) acc[j] += g[j];
    }
    if (a.dfm) {
      const float c = a.dfm[b];
      float s[EPL], v[EPL];
      load_f32xN<EPL>(a.fm_sum + b * D + e0, s);
      if (a.x0_bf16)
        load_bf16xN<EPL>(static_cast<const uint16_t *>(a.x0) + b * a.x0_ld + col, v);
      else
        load_f32xN<EPL>(static_cast<const float *>(a.x0) + b * a.x0_ld + col, v);
#pragma unroll
      for (int j = 0; j < EPL; ++j) acc[j] = fmaf(c, s[j] - v[j], acc[j]);
    }
  } else if (w_lane && a.dw) {
    acc[0] += a.dw[b];
  }
}

template <typename T>
__device__ __forceinline__ void apply_row(const BankArgs &bank, const ApplyArgs &a, int f,
                                          int64_t row, int e0, bool v_lane, const float *acc) {
  constexpr int EPL = Vec<T>::EPL;
  const int64_t grow = bank.row_offset[f] + row;
  const int64_t off = grow * static_cast<int64_t>(bank.row_stride) + e0;
  T *p = reinterpret_cast<T *>(a.mode == MREC_BWD_DENSE_GRAD ? static_cast<char *>(a.grad)
                                                              : bank.data) +
         off;
  const uint4 raw = *reinterpret_cast<const uint4 *>(p);
  float old[EPL];
  Vec<T>::to_f32(raw, old);
  const int live = v_lane ? EPL : 1;  // w lane: only element D is live
  float nv[EPL];
#pragma unroll
  for (int j = 0; j < EPL; ++j)
    nv[j] = (a.mode == MREC_BWD_DENSE_GRAD) ? old[j] + acc[j] : fmaf(-a.lr, acc[j], old[j]);
  uint4 out;
  if constexpr (sizeof(T) == 4) {
    const uint32_t o[4] = {raw.x, raw.y, raw.z, raw.w};
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = j < live ? __float_as_uint(nv[j]) : o[j];
    out = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    const uint32_t o[4] = {raw.x, raw.y, raw.z, raw.w};
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint16_t h[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int j = 2 * k + q;
        if (j < live) {
          h[q] = (a.mode == MREC_BWD_SGD_SR)
                     ? f32_to_bf16_sr(nv[j], hash3(a.seed, grow, static_cast<uint32_t>(e0 + j)))
                     : f32_to_bf16_rne(nv[j]);
        } else {
          h[q] = static_cast<uint16_t>(q ? (o[k] >> 16) : (o[k] & 0xffffu));
        }
      }
      w[k] = static_cast<uint32_t>(h[0]) | (static_cast<uint32_t>(h[1]) << 16);
    }
    out = make_uint4(w[0], w[1], w[2], w[3]);
  }
  *reinterpret_cast<uint4 *>(p) = out;
}

template <typename T, int LPR>
__global__ __launch_bounds__(256) void apply_kernel(BankArgs bank, int64_t B, const void *ws,
                                                    ApplyArgs a) {
  constexpr int EPL = Vec<T>::EPL;
  constexpr int WPB = 256 / LPR;
  __shared__ int32_t long_list[WPB];
  __shared__ int32_t n_long;
  __shared__ float red[WPB][LPR * EPL + 1];
  const int f = blockIdx.y;
  const TableWs t = table_ws(ws, f, B);
  const int nu = t.hdr[0];
  const int ublk = blockIdx.x * WPB;
  if (ublk >= nu) return;  // uniform per block
  const int worker = threadIdx.x / LPR;
  const int l = threadIdx.x % LPR;
  const int e0 = l * EPL;
  const int D = bank.dim;
  const bool v_lane = e0 + EPL <= D;
  const bool w_lane = bank.has_w && e0 == D;
  const bool live = v_lane || w_lane;
  if (threadIdx.x == 0) n_long = 0;
  __syncthreads();

  const int u = ublk + worker;
  bool mine = u < nu;
  int start = 0, end = 0;
  if (mine) {
    start = t.seg[u];
    end = t.seg[u + 1];
    if (end - start > kShortSeg) {
      if (l == 0) long_list[atomicAdd(&n_long, 1)] = u;
      mine = false;
    }
  }
  if (mine && live) {
    float acc[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) acc[j] = 0.f;
    for (int i = start; i < end; i += 4) {
      int bb[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) bb[k] = (i + k < end) ? t.perm[i + k] : -1;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (bb[k] >= 0) add_lookup_grad<EPL>(a, bb[k], f, D, e0, v_lane, w_lane, acc);
    }
    apply_row<T>(bank, a, f, t.uniq[u], e0, v_lane, acc);
  }
  __syncthreads();
  const int nl = n_long;
  for (int k = 0; k < nl; ++k) {
    // each hot segment is summed independently, so the (atomic) list order
    // does not change any result
    const int uu = long_list[k];
    const int s0 = t.seg[uu], s1 = t.seg[uu + 1];
    float acc[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) acc[j] = 0.f;
    if (live)
      for (int i = s0 + worker; i < s1; i += WPB)
        add_lookup_grad<EPL>(a, t.perm[i], f, D, e0, v_lane, w_lane, acc);
#pragma unroll
    for (int j = 0; j < EPL; ++j) red[worker][e0 + j] = acc[j];
    __syncthreads();
    for (int sft = WPB / 2; sft > 0; sft >>= 1) {
      if (worker < sft) {
#pragma unroll
        for (int j = 0; j < EPL; ++j) red[worker][e0 + j] += red[worker + sft][e0 + j];
      }
      __syncthreads();
    }
    if (worker == 0 && live) {
#pragma unroll
      for (int j = 0; j < EPL; ++j) acc[j] = red[0][e0 + j];
      apply_row<T>(bank, a, f, t.uniq[uu], e0, v_lane, acc);
    }
    __syncthreads();
  }
}

}  // namespace mrec

using namespace mrec;

extern "C" {

size_t mrec_emb_bwd_workspace_size(int32_t n_tables, int64_t batch) {
  if (n_tables <= 0 || batch < 0) return 0;
  return static_cast<size_t>(n_tables) * static_cast<size_t>(table_ws_bytes(batch));
}

mrec_status mrec_emb_bwd_plan(const mrec_table_bank *bank, const mrec_ids *ids, int64_t batch,
                              void *workspace, size_t ws_bytes, int32_t *d_oob_flag,
                              mrec_stream stream) {
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
  int np = 1;
  while (np < batch) np <<= 1;
  if (np < 2) np = 2;
  plan_kernel<<<dim3(ba.n_tables), kPlanThreads, 0, static_cast<hipStream_t>(stream)>>>(
      ba, ia, batch, np, workspace, d_oob_flag);
  return launch_status("mrec_emb_bwd_plan");
}

mrec_status mrec_emb_bwd_apply(const mrec_table_bank *bank, int64_t batch, const void *workspace,
                               size_t ws_bytes, const void *dx, mrec_dtype dx_dtype, int64_t dx_ld,
                               const float *dfm, const float *fm_sum, const void *x0,
                               mrec_dtype x0_dtype, int64_t x0_ld, const float *dw,
                               mrec_bwd_mode mode, float lr, uint64_t seed, void *grad,
                               mrec_stream stream) {
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
  MREC_CHECK_ARG(mode == MREC_BWD_DENSE_GRAD || mode == MREC_BWD_SGD || mode == MREC_BWD_SGD_SR,
                 "bad mode");
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
  if (batch == 0) return MREC_OK;
  ApplyArgs a;
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
  a.grad = grad;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int wpb = 256 / lpr;
  const dim3 grid(static_cast<unsigned>((batch + wpb - 1) / wpb), static_cast<unsigned>(F));
#define MREC_AK(T, L) apply_kernel<T, L><<<grid, 256, 0, s>>>(ba, batch, workspace, a)
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
  return launch_status("mrec_emb_bwd_apply");
}

}  // extern "C"
