// Shared helpers for libmrec (gfx950 only).  Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "mrec.h"

namespace mrec {

// ---------------------------------------------------------------------------
// status / error reporting (thread-local last error, no exceptions cross ABI)
// ---------------------------------------------------------------------------
void set_error(const std::string &msg);

#define MREC_CHECK_ARG(cond, msg)                                                          \
  do {                                                                                     \
    if (!(cond)) {                                                                         \
      ::mrec::set_error(std::string(__func__) + ": " + (msg));                             \
      return MREC_EINVAL;                                                                  \
    }                                                                                      \
  } while (0)

mrec_status launch_status(const char *what);  // hipGetLastError -> status

// ---------------------------------------------------------------------------
// Embedding-backward workspace layout tags (ABI 28).  A plan decides the layout
// (sorted or hash) from its batch and whether its ids are a padded exchange view;
// an apply decides it from its batch and whether the gradients are given.  The two
// can disagree (a padded plan of 4096 < B <= 8192 entries followed by a plain
// apply), and the apply would then read the workspace in the wrong layout.  So
// every plan records {layout, batch, tables} per workspace address on the host when
// it is issued (and stamps the same tag into the device headers, ws_layout_tag),
// and every apply entry checks its own expectation against the record before it
// launches: a mismatch, or a workspace no plan was issued for, is MREC_EINVAL.
// Host-only (no device read, no sync): graph capture records the plan first too.
// ---------------------------------------------------------------------------
constexpr int kLayoutSorted = 0;  // emb_plan.h describes both layouts
constexpr int kLayoutHash = 1;
__host__ __device__ inline int32_t ws_layout_tag(int layout, int64_t batch) {
  return static_cast<int32_t>((batch << 2) | layout);
}
void ws_layout_record(const void *ws, int layout, int64_t batch, int n_tables, bool padded);
mrec_status ws_layout_check(const void *ws, int layout, int64_t batch, int n_tables,
                            const char *who);

// ---------------------------------------------------------------------------
// Kernel clock (measurement only, mrec_kernel_clock; layout in mrec.h).
// The clocked kernels are a separate instantiation (template flag KC), launched
// only while the clock is on: KcScope<false> is empty, so the production kernels
// compile exactly as they would without it; KcScope<true> reads the clock on entry
// (a uniform value, kept in scalar registers) and writes both stamps on every
// return path of the wave, after the wave's own stores are acknowledged, into the
// wave's own shard line (waves sharing an address serialise their atomics: 64
// shards per slot cost the 16-wave interaction workgroups ~15 us).
// ---------------------------------------------------------------------------
struct KClock {
  unsigned long long *buf;
  int slot;
};
KClock kclock_take();  // host: the next slot when the clock is on, else {NULL, 0}

template <bool ON>
struct KcScope {
  __device__ explicit KcScope(const KClock &) {}
  __device__ KcScope(const KClock &, int) {}
};
template <>
struct KcScope<true> {
  KClock kc;
  unsigned long long t0;
  int cat = -1;  // (diagnostic builds: a block category owns shards [cat * 1024, + 1024))
  __device__ explicit KcScope(const KClock &k) : kc(k), t0(__builtin_amdgcn_s_memrealtime()) {}
  __device__ KcScope(const KClock &k, int c) : kc(k), t0(__builtin_amdgcn_s_memrealtime()), cat(c) {}
  __device__ ~KcScope() {
    if ((threadIdx.x & 63) == 0) {
#ifndef MREC_KC_NOWAIT  // (diagnostic: stamp at the last issue, not the last acknowledgement)
      __builtin_amdgcn_s_waitcnt(0);
#endif
      const unsigned wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
      const unsigned shard = cat < 0 ? wave % MREC_KCLOCK_SHARDS : cat * 1024 + (wave & 1023);
      unsigned long long *p =
          kc.buf + (static_cast<int64_t>(kc.slot) * MREC_KCLOCK_SHARDS + shard) * MREC_KCLOCK_SHARD_U64;
      atomicMin(p, t0);
      atomicMax(p + 1, static_cast<unsigned long long>(__builtin_amdgcn_s_memrealtime()));
    }
  }
};

// ---------------------------------------------------------------------------
// kernel argument blocks (passed by value; <= 4 KiB kernarg segment)
// ---------------------------------------------------------------------------
// fused optimizer of the update (mrec_optim); kind = the apply's mode
struct OptArgs {
  int kind;  // the optimizer's mrec_bwd_mode (0: none)
  double beta1, beta2;
  float eps, wd, gscale, lr;
  int flags;
  float *s0, *s1;
  int32_t *row_step;
  const int64_t *d_t;
  int64_t ld;
};

struct BankArgs {
  char *data;
  int64_t row_offset[MREC_MAX_TABLES];
  int64_t rows[MREC_MAX_TABLES];
  int32_t n_tables;
  int32_t dim;
  int32_t row_stride;  // elements
  int32_t has_w;
  int32_t lpr;  // lanes per row: row bytes / 16
  OptArgs adam;  // a fused Adam's state (kind MREC_BWD_ADAM) for reads of current rows
};

struct IdsArgs {
  const void *ptr[MREC_MAX_TABLES];
  int64_t stride;
  int64_t chunk;         // 0: element b at b * stride
  int64_t chunk_stride;  // else at (b / chunk) * chunk_stride + b % chunk
  int32_t is64;
  int32_t pad_negative;
};

mrec_status make_bank_args(const mrec_table_bank *bank, BankArgs *out, int *elem_bytes,
                           int *lanes_per_row);
mrec_status make_ids_args(const mrec_ids *ids, int n_tables, IdsArgs *out);
// the fused optimizer of a mode >= MREC_BWD_ADAGRAD from bank->optim (checked)
mrec_status make_opt_args(const mrec_table_bank *bank, int mode, OptArgs *out);

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// cross-lane sums without the LDS crossbar: DPP row rotations inside a 16-lane row
// and the gfx950 permlane swaps across rows / halves (ds_bpermute, which
// __shfl_xor lowers to, costs an LDS transfer per value: the interaction's 68
// per wave took ~3 us of an 8 us launch, tools/bench_interact.py)
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float swap16_sum(float v) {  // + the paired row (rows 0<->1, 2<->3)
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap32_sum(float v) {  // + the other half of the wave
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// sum over the 16 lanes of the wave with this lane's index mod 4 (every lane gets it)
__device__ __forceinline__ float sum_mod4_lanes(float v) {
  v += dpp_f32<0x124>(v);  // row_ror:4
  v += dpp_f32<0x128>(v);  // row_ror:8
  return swap32_sum(swap16_sum(v));
}
// sum over this lane's quad (lanes 4q .. 4q + 3)
__device__ __forceinline__ float sum_quad(float v) {
  v += dpp_f32<0xb1>(v);  // quad_perm [1, 0, 3, 2]
  return v + dpp_f32<0x4e>(v);  // quad_perm [2, 3, 0, 1]
}
// sum over all 64 lanes
__device__ __forceinline__ float sum_wave(float v) { return sum_mod4_lanes(sum_quad(v)); }
// max over all 64 lanes (every lane gets it; order-free, so equal to any other order)
__device__ __forceinline__ float max_wave(float v) {
  v = fmaxf(v, dpp_f32<0xb1>(v));   // quad_perm [1, 0, 3, 2]
  v = fmaxf(v, dpp_f32<0x4e>(v));   // quad_perm [2, 3, 0, 1]
  v = fmaxf(v, dpp_f32<0x124>(v));  // row_ror:4
  v = fmaxf(v, dpp_f32<0x128>(v));  // row_ror:8
  const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r16[0]), __uint_as_float(r16[1]));
  const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r32[0]), __uint_as_float(r32[1]));
}

__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(static_cast<uint32_t>(h) << 16);
}

// round-to-nearest-even with v_cvt_pk_bf16_f32 (the kernels' f32 mode: RNE,
// denormals kept; NaN stays NaN).  The integer form -- (u + 0x7fff + lsb) >> 16 with
// a NaN test -- gives the same bits on every non-NaN input and cost ~5 VALU ops per
// value: the DIN attention backward's ~70 conversions per lane and sample were
// ~14 us of C4's step (r05).
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{lo, hi}), bf16x2_t));
}
__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  return static_cast<uint16_t>(pack_bf16x2(f, 0.f));
}

// stochastic rounding with 16 random bits (unbiased: E[result] = f)
__device__ __forceinline__ uint16_t f32_to_bf16_sr(float f, uint32_t rnd) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);
  return static_cast<uint16_t>((u + (rnd & 0xffffu)) >> 16);
}

__device__ __forceinline__ uint32_t hash3(uint64_t seed, uint64_t row, uint32_t col) {
  uint32_t x = static_cast<uint32_t>(seed) ^ static_cast<uint32_t>(seed >> 32) * 0x27d4eb2fu;
  x ^= static_cast<uint32_t>(row) * 0x9e3779b1u;
  x ^= static_cast<uint32_t>(row >> 32) * 0x85ebca77u;
  x ^= col * 0xc2b2ae3du;
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ int64_t load_id(const IdsArgs &ids, int f, int64_t b) {
  const int64_t off = ids.chunk ? (b / ids.chunk) * ids.chunk_stride + b % ids.chunk : b * ids.stride;
  if (ids.is64) return static_cast<const int64_t *>(ids.ptr[f])[off];
  return static_cast<int64_t>(static_cast<const int32_t *>(ids.ptr[f])[off]);
}

// ids of table f at samples i_k = base + k * step (k < N); `fill` for i_k >= limit.
// Every load is issued before any is used: unconditional loads from clamped indices
// (sample 0 past `limit`), masked afterwards.  A load inside `i < B ? load_id(..) : -1`
// has its value copied out of the branch, and that copy waits for it: the compiler
// serialised such loops into one memory round trip per id (r05: the hash plan's 8
// rounds per thread were ~8 us of its 9).  The layout branches (is64, chunk) are
// uniform and taken once, outside the loads.
template <int N>
__device__ __forceinline__ void load_ids_batch(const IdsArgs &ids, int f, int64_t base, int64_t step,
                                               int64_t limit, int64_t fill, int64_t (&out)[N]) {
  if (limit <= 0) {
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = fill;
    return;
  }
  if (ids.chunk) {  // chunked sender views: the per-element path
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const int64_t i = base + k * step;
      out[k] = i < limit ? load_id(ids, f, i) : fill;
    }
    return;
  }
  if (ids.is64) {
    const int64_t *p = static_cast<const int64_t *>(ids.ptr[f]);
    int64_t v[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const int64_t i = base + k * step;
      v[k] = p[(i < limit ? i : 0) * ids.stride];
    }
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = base + k * step < limit ? v[k] : fill;
  } else {
    const int32_t *p = static_cast<const int32_t *>(ids.ptr[f]);
    int32_t v[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const int64_t i = base + k * step;
      v[k] = p[(i < limit ? i : 0) * ids.stride];
    }
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = base + k * step < limit ? static_cast<int64_t>(v[k]) : fill;
  }
}

// 16 bytes of a row as floats: EPL = 8 (bf16) or 4 (f32)
template <typename T>
struct Vec;
template <>
struct Vec<uint16_t> {
  static constexpr int EPL = 8;
  __device__ __forceinline__ static void to_f32(const uint4 &r, float *v) {
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
};
template <>
struct Vec<float> {
  static constexpr int EPL = 4;
  __device__ __forceinline__ static void to_f32(const uint4 &r, float *v) {
    v[0] = __uint_as_float(r.x);
    v[1] = __uint_as_float(r.y);
    v[2] = __uint_as_float(r.z);
    v[3] = __uint_as_float(r.w);
  }
};


// Per-step scalars of Adam / AdamW at step s (b1p = beta1^s, b2p = beta2^s, in
// double like the host-side scalars of the dense optimizers).
struct AdamStep {
  float b1, omb1, b2, omb2;  // beta1, 1 - beta1, beta2, 1 - beta2 (rounded from double)
  float step;                // lr / bc1 (Adam) or lr sqrt(bc2) / bc1 (AdamW)
  float rbc2;                // 1 / sqrt(bc2) (Adam)
};
__device__ __forceinline__ AdamStep adam_scalars(const OptArgs &o, float lr, double b1p,
                                                 double b2p) {
  AdamStep a;
  a.b1 = static_cast<float>(o.beta1);
  a.omb1 = static_cast<float>(1.0 - o.beta1);
  a.b2 = static_cast<float>(o.beta2);
  a.omb2 = static_cast<float>(1.0 - o.beta2);
  const bool bc = !(o.flags & MREC_OPT_NO_BIAS_CORRECTION);
  const double bc1 = bc ? 1.0 - b1p : 1.0;
  const double bc2 = bc ? 1.0 - b2p : 1.0;
  if (o.flags & MREC_OPT_DECOUPLED_WD) {
    a.step = static_cast<float>(bc ? lr * sqrt(bc2) / bc1 : lr);
    a.rbc2 = 1.f;
  } else {
    a.step = static_cast<float>(lr / bc1);
    a.rbc2 = static_cast<float>(1.0 / sqrt(bc2));
  }
  return a;
}

// One Adam / AdamW step of one element, in the operation order of the reference
// (optim/AdamW.py:46-59) / torch.optim.Adam.
__device__ __forceinline__ void adam_elem(const OptArgs &o, const AdamStep &s, float lr, float g,
                                          float &p, float &m, float &v) {
  const bool decoupled = o.flags & MREC_OPT_DECOUPLED_WD;
  if (!decoupled && o.wd != 0.f) g = fmaf(o.wd, p, g);
  m = fmaf(s.b1, m, s.omb1 * g);
  v = fmaf(s.b2, v, s.omb2 * g * g);
  if (decoupled) {
    p = p - s.step * (m / (sqrtf(v) + o.eps));
    if (o.wd > 0.f) p = p - (lr * o.wd) * p;
  } else {
    const float denom = sqrtf(v) * s.rbc2 + o.eps;
    p = p - s.step * (m / denom);
  }
}


// A row of a bank trained by the fused (lazy, dense-compatible) Adam is stored as of
// its last update, row_step[grow]; dense Adam would have moved it on every step
// since (momentum).  Readers that need its value as of step `t_now` (the forward
// gathers: t_now = completed steps; the apply's FM term: t_now = t - 1) run the
// missed zero-gradient steps on this lane's 16 bytes in registers, without writing
// (the update of the row does the same steps and writes).  Bank dtype in and out.
template <typename T>
__device__ __forceinline__ uint4 adam_current(const BankArgs &bank, int64_t grow, int e0, int n,
                                              uint4 raw, int64_t t_now) {
  constexpr int EPL = Vec<T>::EPL;
  const OptArgs &o = bank.adam;
  if (o.kind != MREC_BWD_ADAM || n == 0) return raw;
  const int64_t t0 = o.row_step[grow];
  if (t0 >= t_now) return raw;
  float p[EPL], m[EPL], v[EPL];
  Vec<T>::to_f32(raw, p);
  const float *mp = o.s0 + grow * o.ld + e0;
  const float *vp = o.s1 + grow * o.ld + e0;
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    m[j] = j < n ? mp[j] : 0.f;
    v[j] = j < n ? vp[j] : 0.f;
  }
  double b1p = pow(o.beta1, static_cast<double>(t0 + 1));
  double b2p = pow(o.beta2, static_cast<double>(t0 + 1));
  for (int64_t st = t0 + 1; st <= t_now; ++st) {
    const AdamStep sc = adam_scalars(o, o.lr, b1p, b2p);
#pragma unroll
    for (int j = 0; j < EPL; ++j)
      if (j < n) adam_elem(o, sc, o.lr, 0.f, p[j], m[j], v[j]);
    b1p *= o.beta1;
    b2p *= o.beta2;
  }
  const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
  uint32_t r[4];
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = j < n ? __float_as_uint(p[j]) : w[j];
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t lo = 2 * k < n ? f32_to_bf16_rne(p[2 * k]) : (w[k] & 0xffffu);
      const uint32_t hi = 2 * k + 1 < n ? f32_to_bf16_rne(p[2 * k + 1]) : (w[k] >> 16);
      r[k] = lo | (hi << 16);
    }
  }
  return make_uint4(r[0], r[1], r[2], r[3]);
}

// elements of a lane's 16 bytes that are live (vector or first-order weight)
__device__ __forceinline__ int live_elems(const BankArgs &bank, int e0, int epl) {
  if (e0 + epl <= bank.dim) return epl;
  return (bank.has_w && e0 == bank.dim) ? 1 : 0;
}

}  // namespace mrec
