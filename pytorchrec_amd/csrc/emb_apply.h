// Embedding-backward apply helpers: the per-lookup gradient, the row update
// (SGD with RNE / stochastic rounding, or dense-gradient accumulation) and the
// register sort network.  Shared by the batched apply (emb_bwd.hip) and the
// large-batch path (emb_bwd_large.hip).
#pragma once
#include "common.h"

namespace mrec {

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
  const uint64_t *d_step;
  void *grad;
  // per-lookup gradient rows given directly (owner side of a sharded table):
  // lookup b of table f -> g_occ[idx * g_ld + e], idx = chunked(b) + f * chunk
  const float *g_occ;
  int64_t g_ld;
  int64_t chunk;
  int64_t chunk_stride;
  // or read straight from the received wire records (ABI 23, owner side of the
  // compact exchange): entry j of part p, table f -> record p * cap_rows +
  // pref[p * F + f] + j (p = b / chunk, j = b % chunk), pitch g_rec_pitch elements
  const void *g_rec;
  int g_rec_bf16;
  int g_rec_pitch;
  const int32_t *g_pref;
  int64_t g_cap_rows;
  int g_F;
  OptArgs opt;
  // DENSE_GRAD straight into wire records (ABI 26, sender side of the compact
  // exchange, mrec_emb_bwd_apply_rec): slot row s = (p * F + f) * cap + j -> record
  // p * cap_rows + o_pref[p * F + f] + j (o_rec_dw dwords); no wire pack launch
  uint32_t *o_rec;
  int o_rec_dw;
  const int32_t *o_pref;
  int o_F, o_cap;
  int64_t o_cap_rows;
  // data-parallel dense SGD tiles riding in this launch (ABI 28,
  // mrec_emb_bwd_apply_wire_sgd): a device-resident SgdArgs (optim_common.h)
  const struct SgdArgs *sgd;
  int sgd_blocks;
};

// a given gradient from a wire record (4-B aligned rows: records are not 16-B).
// An entry past its part's cap_rows records had its record clipped by the sender
// (the overflow flag is set): zero gradient -- never another entry's record.
template <int EPL>
__device__ __forceinline__ void wire_grad(const ApplyArgs &a, int64_t b, int f, int D, int e0,
                                          bool v_lane, bool w_lane, float *g) {
  const int64_t p = b / a.chunk, j = b - p * a.chunk;
  const int64_t in_part = a.g_pref[p * a.g_F + f] + j;
  if (in_part >= a.g_cap_rows) return;  // g stays zero (lookup_grad zeroed it)
  const int64_t rec = p * a.g_cap_rows + in_part;
  if (a.g_rec_bf16) {
    const uint16_t *go = static_cast<const uint16_t *>(a.g_rec) + rec * a.g_rec_pitch;
    if (v_lane) {
      const uint32_t *q = reinterpret_cast<const uint32_t *>(go + e0);
#pragma unroll
      for (int i = 0; i < EPL / 2; ++i) {
        const uint32_t x = q[i];
        g[2 * i] = __uint_as_float(x << 16);
        g[2 * i + 1] = __uint_as_float(x & 0xffff0000u);
      }
    } else if (w_lane) {
      g[0] = __uint_as_float(static_cast<uint32_t>(go[D]) << 16);
    }
  } else {
    const float *go = static_cast<const float *>(a.g_rec) + rec * a.g_rec_pitch;
    if (v_lane) {
#pragma unroll
      for (int i = 0; i < EPL; ++i) g[i] = go[e0 + i];
    } else if (w_lane) {
      g[0] = go[D];
    }
  }
}

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

// gradient of lookup (b, f) for this lane's EPL elements (w lane: g[0])
template <int EPL>
__device__ __forceinline__ void lookup_grad(const ApplyArgs &a, int64_t b, int f, int D, int e0,
                                            bool v_lane, bool w_lane, float *g) {
#pragma unroll
  for (int j = 0; j < EPL; ++j) g[j] = 0.f;
  if (a.g_rec) {
    wire_grad<EPL>(a, b, f, D, e0, v_lane, w_lane, g);
    return;
  }
  if (a.g_occ) {
    const int64_t idx = a.chunk ? (b / a.chunk) * a.chunk_stride + f * a.chunk + b % a.chunk : b;
    const float *go = a.g_occ + idx * a.g_ld;
    if (v_lane)
      load_f32xN<EPL>(go + e0, g);
    else if (w_lane)
      g[0] = go[D];
    return;
  }
  if (v_lane) {
    // the same arithmetic as mrec_shard_lookup_grad, so sharded and unsharded
    // updates agree
    const int64_t col = static_cast<int64_t>(f) * D + e0;
    if (a.dx) {
      if (a.dx_bf16)
        load_bf16xN<EPL>(static_cast<const uint16_t *>(a.dx) + b * a.dx_ld + col, g);
      else
        load_f32xN<EPL>(static_cast<const float *>(a.dx) + b * a.dx_ld + col, g);
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
      for (int j = 0; j < EPL; ++j) g[j] = fmaf(c, s[j] - v[j], g[j]);
    }
  } else if (w_lane && a.dw) {
    g[0] = a.dw[b];
  }
}

// gradient of lookup (b, f) with the row's current values v (this lane's EPL
// elements, bank dtype widened) for the FM term: the hash-layout apply reads the
// row it updates anyway, so the gathered rows are not re-read from x0
template <int EPL>
__device__ __forceinline__ void lookup_grad_v(const ApplyArgs &a, int64_t b, int f, int D, int e0,
                                              bool v_lane, bool w_lane, const float *v, float *g) {
#pragma unroll
  for (int j = 0; j < EPL; ++j) g[j] = 0.f;
  if (a.g_rec) {
    wire_grad<EPL>(a, b, f, D, e0, v_lane, w_lane, g);
    return;
  }
  if (a.g_occ) {
    const int64_t idx = a.chunk ? (b / a.chunk) * a.chunk_stride + f * a.chunk + b % a.chunk : b;
    const float *go = a.g_occ + idx * a.g_ld;
    if (v_lane)
      load_f32xN<EPL>(go + e0, g);
    else if (w_lane)
      g[0] = go[D];
    return;
  }
  if (v_lane) {
    const int64_t col = static_cast<int64_t>(f) * D + e0;
    if (a.dx) {
      if (a.dx_bf16)
        load_bf16xN<EPL>(static_cast<const uint16_t *>(a.dx) + b * a.dx_ld + col, g);
      else
        load_f32xN<EPL>(static_cast<const float *>(a.dx) + b * a.dx_ld + col, g);
    }
    if (a.dfm) {
      const float c = a.dfm[b];
      float s[EPL];
      load_f32xN<EPL>(a.fm_sum + b * D + e0, s);
#pragma unroll
      for (int j = 0; j < EPL; ++j) g[j] = fmaf(c, s[j] - v[j], g[j]);
    }
  } else if (w_lane && a.dw) {
    g[0] = a.dw[b];
  }
}

template <int EPL>
__device__ __forceinline__ void add_lookup_grad_v(const ApplyArgs &a, int64_t b, int f, int D,
                                                  int e0, bool v_lane, bool w_lane, const float *v,
                                                  float *acc) {
  float g[EPL];
  lookup_grad_v<EPL>(a, b, f, D, e0, v_lane, w_lane, v, g);
#pragma unroll
  for (int j = 0; j < EPL; ++j) acc[j] += g[j];
}

// per-lookup gradient first, then one add into the segment sum
template <int EPL>
__device__ __forceinline__ void add_lookup_grad(const ApplyArgs &a, int64_t b, int f, int D,
                                                int e0, bool v_lane, bool w_lane, float *acc) {
  float g[EPL];
  lookup_grad<EPL>(a, b, f, D, e0, v_lane, w_lane, g);
#pragma unroll
  for (int j = 0; j < EPL; ++j) acc[j] += g[j];
}

// element e0 of global row `grow` (table offset already added): the bank, or the
// dense gradient buffer in DENSE_GRAD mode
// (MODE >= 0: the update mode fixed at compile time, else a.mode)
template <typename T, int MODE = -1>
__device__ __forceinline__ T *row_ptr_g(const BankArgs &bank, const ApplyArgs &a, int64_t grow,
                                        int e0) {
  const int mode = MODE >= 0 ? MODE : a.mode;
  const int64_t off = grow * static_cast<int64_t>(bank.row_stride) + e0;
  return reinterpret_cast<T *>(mode == MREC_BWD_DENSE_GRAD ? static_cast<char *>(a.grad)
                                                            : bank.data) +
         off;
}

template <typename T>
__device__ __forceinline__ T *row_ptr(const BankArgs &bank, const ApplyArgs &a, int f,
                                      int64_t row, int e0) {
  return row_ptr_g<T>(bank, a, bank.row_offset[f] + row, e0);
}

// DENSE_GRAD into a wire record (a.o_rec): the sums the slot row would hold after
// the zeroed buffer's `0 + acc`, rounded to the table dtype as there; the record's
// dwords only (a w lane: its one dword, element D and the zero pad beside it).  An
// entry past its part's cap_rows records is dropped (the unpack flagged it).
template <typename T>
__device__ __forceinline__ void rec_out(const ApplyArgs &a, int64_t grow, int e0, bool v_lane,
                                        const float *acc) {
  constexpr int EPL = Vec<T>::EPL;
  const int64_t fc = static_cast<int64_t>(a.o_F) * a.o_cap;
  const int64_t p = grow / fc, rem = grow - p * fc;
  const int f = static_cast<int>(rem / a.o_cap);
  const int64_t j = rem - static_cast<int64_t>(f) * a.o_cap;
  const int64_t in_part = a.o_pref[p * a.o_F + f] + j;
  if (in_part >= a.o_cap_rows) return;
  uint32_t *dst = a.o_rec + (p * a.o_cap_rows + in_part) * a.o_rec_dw +
                  e0 * static_cast<int>(sizeof(T)) / 4;
  if constexpr (sizeof(T) == 4) {
    if (v_lane) {
#pragma unroll
      for (int k = 0; k < EPL; ++k) dst[k] = __float_as_uint(0.f + acc[k]);
    } else {
      dst[0] = __float_as_uint(0.f + acc[0]);
    }
  } else {
    if (v_lane) {
#pragma unroll
      for (int k = 0; k < EPL / 2; ++k)
        dst[k] = static_cast<uint32_t>(f32_to_bf16_rne(0.f + acc[2 * k])) |
                 (static_cast<uint32_t>(f32_to_bf16_rne(0.f + acc[2 * k + 1])) << 16);
    } else {
      dst[0] = static_cast<uint32_t>(f32_to_bf16_rne(0.f + acc[0]));
    }
  }
}

// new value of this lane's 16 bytes of global row `grow` from its old contents `raw`
template <typename T, int MODE = -1>
__device__ __forceinline__ void apply_row_raw_g(const BankArgs &bank, const ApplyArgs &a,
                                                int64_t grow, int e0, bool v_lane,
                                                const float *acc, const uint4 raw) {
  constexpr int EPL = Vec<T>::EPL;
  if constexpr (MODE == MREC_BWD_DENSE_GRAD) {
    if (a.o_rec) {  // uniform
      rec_out<T>(a, grow, e0, v_lane, acc);
      return;
    }
  }
  const int mode = MODE >= 0 ? MODE : a.mode;
  T *p = row_ptr_g<T, MODE>(bank, a, grow, e0);
  float old[EPL];
  Vec<T>::to_f32(raw, old);
  const int live = v_lane ? EPL : 1;  // w lane: only element D is live
  float nv[EPL];
#pragma unroll
  for (int j = 0; j < EPL; ++j)
    nv[j] = (mode == MREC_BWD_DENSE_GRAD) ? old[j] + acc[j] : fmaf(-a.lr, acc[j], old[j]);
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
          h[q] = (mode == MREC_BWD_SGD_SR)
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

template <typename T>
__device__ __forceinline__ void apply_row_raw(const BankArgs &bank, const ApplyArgs &a, int f,
                                              int64_t row, int e0, bool v_lane, const float *acc,
                                              const uint4 raw) {
  apply_row_raw_g<T>(bank, a, bank.row_offset[f] + row, e0, v_lane, acc, raw);
}

template <typename T>
__device__ __forceinline__ void apply_row(const BankArgs &bank, const ApplyArgs &a, int f,
                                          int64_t row, int e0, bool v_lane, const float *acc) {
  const uint4 raw = *reinterpret_cast<const uint4 *>(row_ptr<T>(bank, a, f, row, e0));
  apply_row_raw<T>(bank, a, f, row, e0, v_lane, acc, raw);
}

// Fused-optimizer update of this lane's 16 bytes of global row `grow` with the
// row's summed gradient `acc` (modes ADAGRAD / ROWWISE_ADAGRAD / ADAM).  Called by
// ALL LPR lanes of the row's worker (row-wise Adagrad sums g^2 across them);
// lanes without a live element (`live` false) only take part in that sum.
template <typename T, int LPR>
__device__ __forceinline__ void opt_row_update(const BankArgs &bank, const ApplyArgs &a,
                                               int64_t grow, int e0, bool v_lane, bool w_lane,
                                               bool live, const float *acc, const uint4 raw) {
  constexpr int EPL = Vec<T>::EPL;
  const OptArgs &o = a.opt;
  const int n = v_lane ? EPL : (w_lane ? 1 : 0);
  float g[EPL];
#pragma unroll
  for (int j = 0; j < EPL; ++j) g[j] = acc[j] * o.gscale;
  acc = g;
  float sq = 0.f;
  if (a.mode == MREC_BWD_ROWWISE_ADAGRAD) {
    if (v_lane)
#pragma unroll
      for (int j = 0; j < EPL; ++j) sq = fmaf(acc[j], acc[j], sq);
#pragma unroll
    for (int off = 1; off < LPR; off <<= 1) sq += __shfl_xor(sq, off);
  }
  if (!live) return;
  float p[EPL];
  Vec<T>::to_f32(raw, p);
  if (a.mode == MREC_BWD_ROWWISE_ADAGRAD) {
    float *st = o.s0 + grow * 2 + (v_lane ? 0 : 1);
    const float G = *st + (v_lane ? sq / static_cast<float>(bank.dim) : acc[0] * acc[0]);
    if (e0 == 0 || w_lane) *st = G;
    const float den = sqrtf(G) + o.eps;
#pragma unroll
    for (int j = 0; j < EPL; ++j)
      if (j < n) p[j] = p[j] - a.lr * (acc[j] / den);
  } else if (a.mode == MREC_BWD_ADAGRAD) {
    float *st = o.s0 + grow * o.ld + e0;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      if (j < n) {
        const float sum = fmaf(acc[j], acc[j], st[j]);
        st[j] = sum;
        p[j] = p[j] - a.lr * (acc[j] / (sqrtf(sum) + o.eps));
      }
    }
  } else {  // MREC_BWD_ADAM
    const int64_t t = *o.d_t;
    const int64_t t0 = o.row_step[grow];
    float *mp = o.s0 + grow * o.ld + e0;
    float *vp = o.s1 + grow * o.ld + e0;
    float m[EPL], v[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      m[j] = j < n ? mp[j] : 0.f;
      v[j] = j < n ? vp[j] : 0.f;
    }
    double b1p = pow(o.beta1, static_cast<double>(t0 + 1));
    double b2p = pow(o.beta2, static_cast<double>(t0 + 1));
    for (int64_t st = t0 + 1; st < t; ++st) {  // the zero-gradient steps this row missed
      const AdamStep sc = adam_scalars(o, a.lr, b1p, b2p);
#pragma unroll
      for (int j = 0; j < EPL; ++j)
        if (j < n) adam_elem(o, sc, a.lr, 0.f, p[j], m[j], v[j]);
      b1p *= o.beta1;
      b2p *= o.beta2;
    }
    const AdamStep sc = adam_scalars(o, a.lr, b1p, b2p);
#pragma unroll
    for (int j = 0; j < EPL; ++j)
      if (j < n) adam_elem(o, sc, a.lr, acc[j], p[j], m[j], v[j]);
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      if (j < n) {
        mp[j] = m[j];
        vp[j] = v[j];
      }
    }
    if (e0 == 0) o.row_step[grow] = static_cast<int32_t>(t);
  }
  // pack: live elements rounded once (RNE), the rest keep their bits
  T *dst = reinterpret_cast<T *>(bank.data) + grow * static_cast<int64_t>(bank.row_stride) + e0;
  const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
  uint32_t o4[4];
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o4[j] = j < n ? __float_as_uint(p[j]) : w[j];
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t lo = 2 * k < n ? f32_to_bf16_rne(p[2 * k]) : (w[k] & 0xffffu);
      const uint32_t hi = 2 * k + 1 < n ? f32_to_bf16_rne(p[2 * k + 1]) : (w[k] >> 16);
      o4[k] = lo | (hi << 16);
    }
  }
  *reinterpret_cast<uint4 *>(dst) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
}

// The row update of every apply path: fixed modes by template (MODE >= 0), else
// the runtime mode; all LPR lanes of the worker call it.
template <typename T, int LPR, int MODE>
__device__ __forceinline__ void row_update(const BankArgs &bank, const ApplyArgs &a, int64_t grow,
                                           int e0, bool v_lane, bool w_lane, bool live,
                                           const float *acc, const uint4 raw) {
  if (MODE >= 0 || a.mode <= MREC_BWD_SGD_SR) {
    if (live) apply_row_raw_g<T, MODE>(bank, a, grow, e0, v_lane, acc, raw);
  } else {
    opt_row_update<T, LPR>(bank, a, grow, e0, v_lane, w_lane, live, acc, raw);
  }
}

__device__ __forceinline__ void cswap(int &a, int &b) {
  const int lo = min(a, b), hi = max(a, b);
  a = lo;
  b = hi;
}

// ascending bitonic network on r[0, N) (compile-time indices: stays in VGPRs)
template <int N>
__device__ __forceinline__ void bitonic_sort(int *r) {
#pragma unroll
  for (int k = 2; k <= N; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int l = i ^ j;
        if (l > i) {
          if ((i & k) == 0)
            cswap(r[i], r[l]);
          else
            cswap(r[l], r[i]);
        }
      }
}

}  // namespace mrec
