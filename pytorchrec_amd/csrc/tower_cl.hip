// Cluster tower: the fused MLP tower + CTR head + BCE of mrec_tower_fwd_bwd with
// every 64-row block shared by a CLUSTER of 4 workgroups.
//
// Why: the 16-row kernel (tower.hip) has every workgroup stream EVERY layer's
// weight images (2 MB per step at the C2 shape) from L2, once per 16 rows: ~0.5 GB
// of L2 -> CU traffic for 0.5 M parameters, and the tower is bound by the per-CU L2
// read rate (~70 GB/s per CU for lines every CU reads).  Here workgroup c of a
// cluster owns one quarter of every layer's output columns (16-column tiles
// [c T / 4, (c + 1) T / 4)) for the cluster's 64 rows, so it streams a quarter of
// the weights, each fragment feeding 4 row tiles (4x the MFMA work per L2 byte).
// Between layers the 4 workgroups swap their column slices through a small global
// exchange buffer:
//   producer: 16-B sc1 stores of its slice -> every storing wave s_waitcnt
//             vmcnt(0) -> workgroup barrier -> one lane adds 1 to the cluster's
//             counter (agent-scope atomic);
//   consumer: one lane polls the counter with sc1 loads (MI355X_MICROARCH.md
//             "Workgroup dispatch ... inter-workgroup visibility", first row of the
//             measured hand-off table) -> barrier -> sc1 loads of the peers' slices.
// The layer's first weight fragments are already in flight while it waits.  Only
// the activations (a quarter each way) and 64 fp32 partial logits cross
// workgroups; the k-fragment images for mrec_tower_dw, dx0, the head partials,
// z, dz and the loss leave exactly as from the 16-row kernel (same layouts, same
// per-16-row head / loss partials).
//
// Per workgroup (512 threads = 8 waves): wave w owns output tile t0 + w of the
// slice (<= 8 tiles = 128 columns) for all 4 row tiles: per k step ONE 1 KiB
// weight fragment (buffer load, fragment order, tower_common.h) and 4 activation
// fragments from LDS, 4 v_mfma_f32_16x16x32_bf16.
//
// LDS: IN [64][s_in] (the layer input: x0, then the assembled h_l / dh_l rows),
// OWN[l] [64][s_own] (this workgroup's slice of h_{l+1}: the ReLU masks of the
// backward, overwritten in place by the gradient it masks), small parameters.
//
// Residency: a spinning workgroup waits for its 3 peers, so the launch needs all
// of its workgroups resident at once: the host uses it only when the grid (4 per
// 64 rows) fits one workgroup per CU (B <= 4096 on 256 CUs).  A poll that never
// completes gives up after ~2^22 tries and sets the workspace's error word (no
// hang; the results are then wrong and the host reports it).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "tower_common.h"

namespace mrec {

constexpr int CL_WG = 4;          // workgroups per cluster
constexpr int CL_ROWS = 64;       // rows per cluster: 4 row tiles of 16
constexpr int CL_THREADS = 512;   // 8 waves, one output tile each
constexpr int CL_WAVES = CL_THREADS / 64;
constexpr int CL_MAXL = 4;
constexpr int CL_MAXT = 8;        // tiles per slice (width <= 512 -> 32 tiles / 4)
constexpr int CL_LDX = 512;       // exchange buffer row stride (elements)
constexpr unsigned CL_SPIN_MAX = 1u << 22;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kSc1 = 16;  // buffer-instruction cache policy: sc1 (L1 bypass / write-through)

struct ClArgs {
  int64_t B;
  int L;
  int width[CL_MAXL + 1];
  const uint16_t *x0;
  int64_t ld_x0;
  const uint16_t *wf[CL_MAXL];
  const uint16_t *wb[CL_MAXL];
  int wf_bytes[CL_MAXL], wb_bytes[CL_MAXL];
  const float *bias[CL_MAXL];
  const float *head_w, *head_b, *base, *xs;
  int64_t ld_xs;
  int ns;
  const float *ws, *b2, *y;
  uint16_t *h_out[CL_MAXL];
  int64_t ld_h[CL_MAXL];
  uint16_t *dh_out[CL_MAXL];
  int64_t ld_dh[CL_MAXL];
  uint16_t *dx0;
  int64_t ld_dx0;
  float *z, *dz, *part;
  int64_t ldp;
  float *loss_part;
  unsigned *ticket;
  float *loss;
  float invB;
  int kfrag, nsteps;
  uint16_t *x0_img;
  int mode;
  const float *dz_in;
  int store_mode;
  int rotate;
  unsigned long long *stamps;  // diagnostics: [grid][32] wall-clock stamps (NULL: off)
  int force_sc1;  // MREC_TOWER_CL_SC1=1: the placement-independent hand-off everywhere
  int diag;  // timing experiments only (MREC_TOWER_CL_DIAG): 1 no polls, 2 no weight loads,
             // 4 no peer gathers -- wrong results
  // cluster workspace
  unsigned *err;
  unsigned *epoch;   // launch counter: hand-off flags are epoch * 64 + hand-offs done
  unsigned *gticket; // workgroups finished (the last one advances the epoch)
  unsigned *flags;   // [nclus][4] hand-off flags (one 16-B granule per cluster)
  unsigned *xcc;     // [nclus][4] (epoch + 1) << 4 | XCD of each member
  float *zx;         // [nclus][4][64] partial logits
  uint16_t *xb[2]; // exchange buffers [B][CL_LDX] bf16 (ping-pong by hand-off parity)
  int nclus;
  // LDS plan (bytes)
  int off_in, s_in;
  int off_own[CL_MAXL], s_own;
  int off_f;   // floats: z[64] | dz[64] | loss[64] | part scratch
  int off_p;   // floats: bias slices [L][128] | head_w slice [128] | y[64] | base[64] | b0
  int lds_bytes;
};

__host__ __device__ __forceinline__ int cl_t0(int T, int c) { return (c * T) / CL_WG; }

__device__ __forceinline__ int cl_rot(int s, int rot, int ksteps) {
  if (s >= ksteps) return 0;  // padded step: its weights read as zeros
  const int r = s + rot;
  return r >= ksteps ? r - ksteps : r;
}

// ---------------------------------------------------------------------------
// hand-off
// ---------------------------------------------------------------------------

// Hand-off state of a workgroup.  Members of a cluster that all sit on one XCD
// ("local": checked at run time from HW_REG_XCC_ID, placement only decides speed)
// hand off through that XCD's L2: plain stores (the lines stay in L2), plain flag
// stores, sc1 loads (L1 bypassed, served by the shared L2).  Otherwise sc1 stores of
// data and flags (written through to memory) and sc1 loads: the placement-independent
// form of MI355X_MICROARCH.md's hand-off table (row 1).
struct ClSync {
  unsigned *flags;  // the cluster's 4 flags (16-B aligned)
  unsigned base;    // epoch * 64
  int c;
  int local;
};

__device__ __forceinline__ unsigned cl_xcc_id() {
  return static_cast<unsigned>(__builtin_amdgcn_s_getreg((3 << 11) | 20)) & 15u;  // HW_REG_XCC_ID
}

// producer: after every wave drained its stores, one lane publishes hand-off h
__device__ __forceinline__ void cl_signal(const ClSync &sy, unsigned h) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned v = sy.base + h + 1;
    if (sy.local)
      *reinterpret_cast<volatile unsigned *>(sy.flags + sy.c) = v;
    else
      __hip_atomic_store(sy.flags + sy.c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// consumer: one lane polls the cluster's 4 flags (one 16-B sc1 load) until every
// member published hand-off h; the others wait at the barrier
__device__ __forceinline__ void cl_wait(const ClArgs &a, const ClSync &sy, unsigned h) {
  if (threadIdx.x == 0) {
    const unsigned target = sy.base + h + 1;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(sy.flags, 0, 16, 0x00020000);
    unsigned n = 0;
    while (true) {
      const u32x4 f = __builtin_amdgcn_raw_buffer_load_b128(rs, 0, 0, kSc1);
      if (min(min(f[0], f[1]), min(f[2], f[3])) >= target) break;
      __builtin_amdgcn_s_sleep(1);
      if (++n == CL_SPIN_MAX) {
        __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

// The peers' column slices of hand-off buffer `xb` (rows of this cluster) -> IN,
// tiles [0, T) except the own [t0, t1); then the pad columns [16 T, 32 ceil(T / 2))
// of IN are zeroed (read by the last k step, never written by a slice).
__device__ __forceinline__ void cl_gather_peers(const ClArgs &a, const uint16_t *xb, char *in,
                                                int T, int t0, int t1, int64_t row0) {
  const int nch = 2 * (T - (t1 - t0));  // 16-B chunks per row from the peers
  const int rows = static_cast<int>(min<int64_t>(CL_ROWS, a.B - row0));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t *>(xb + row0 * CL_LDX), 0, rows * CL_LDX * 2, 0x00020000);
  constexpr int MAXQ = (CL_ROWS * 2 * 32) / CL_THREADS;  // <= 64 chunks per row
  // every load is issued unconditionally (an invalid one at an offset past the
  // descriptor's range reads zeros) and consumed after the last: as branches, each
  // load was followed by its own wait, one round trip per chunk
  u32x4 v[MAXQ];
#pragma unroll
  for (int q = 0; q < MAXQ; ++q) {
    const int i = threadIdx.x + q * CL_THREADS;
    const int r = i / nch, k = i - r * nch;
    const int ch = k < 2 * t0 ? k : k + 2 * (t1 - t0);
    const int off = (i < CL_ROWS * nch && r < rows) ? (r * CL_LDX + ch * 8) * 2 : 0x40000000;
    v[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kSc1);
  }
  const int s_in = a.s_in;
#pragma unroll
  for (int q = 0; q < MAXQ; ++q) {
    const int i = threadIdx.x + q * CL_THREADS;
    if (i < CL_ROWS * nch) {
      const int r = i / nch, k = i - r * nch;
      const int ch = k < 2 * t0 ? k : k + 2 * (t1 - t0);
      *reinterpret_cast<u32x4 *>(in + r * s_in + ch * 16) = v[q];
    }
  }
  const int zc = 2 * (tw_ceil(T, 2) * 2 - T);  // 16-B chunks of pad per row (0 or 2)
  if (zc) {
    for (int i = threadIdx.x; i < CL_ROWS * zc; i += CL_THREADS) {
      const int r = i / zc, k = i - r * zc;
      *reinterpret_cast<u32x4 *>(in + r * s_in + (2 * T + k) * 16) = u32x4{0u, 0u, 0u, 0u};
    }
  }
}

// own slice OWN (nt tiles) -> IN columns [16 t0, 16 (t0 + nt)) and, when xb, the
// exchange buffer (sc1 stores, rows < B)
__device__ __forceinline__ void cl_publish(const ClArgs &a, const char *own, char *in, uint16_t *xb,
                                           int t0, int nt, int64_t row0, int local) {
  const int nch = 2 * nt;
  const int rows = static_cast<int>(min<int64_t>(CL_ROWS, a.B - row0));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      xb ? xb + row0 * CL_LDX : const_cast<uint16_t *>(a.x0), 0, xb ? rows * CL_LDX * 2 : 0,
      0x00020000);
  for (int i = threadIdx.x; i < CL_ROWS * nch; i += CL_THREADS) {
    const int r = i / nch, k = i - r * nch;
    const u32x4 v = *reinterpret_cast<const u32x4 *>(own + r * a.s_own + k * 16);
    *reinterpret_cast<u32x4 *>(in + r * a.s_in + (2 * t0 + k) * 16) = v;
    if (xb && r < rows) {
      if (local)
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (r * CL_LDX + (2 * t0 + k) * 8) * 2, 0, 0);
      else
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (r * CL_LDX + (2 * t0 + k) * 8) * 2, 0, kSc1);
    }
  }
}

// ---------------------------------------------------------------------------
// outputs of a slice (64 rows x nt tiles from tile t0) in the launch's layouts
// ---------------------------------------------------------------------------

__device__ __forceinline__ void cl_store_rows(const ClArgs &a, const char *blk, int s_blk, int t0,
                                              int nt, int width, uint16_t *dst, int64_t ld,
                                              int64_t row0) {
  if (!dst || a.store_mode == 2) return;
  const int lim = tw_ceil(width, 8) - 2 * t0;  // chunks inside round8(width)
  const int nch = min(2 * nt, lim);
  if (nch <= 0) return;
  const int rows = static_cast<int>(min<int64_t>(CL_ROWS, a.B - row0));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      dst + row0 * ld, 0, static_cast<int>(rows * ld * 2), 0x00020000);
  for (int i = threadIdx.x; i < CL_ROWS * nch; i += CL_THREADS) {
    const int r = i / nch, k = i - r * nch;
    if (r < rows) {
      const u32x4 v = *reinterpret_cast<const u32x4 *>(blk + r * s_blk + k * 16);
      const int off = static_cast<int>((r * ld + (2 * t0 + k) * 8) * 2);
      if (a.store_mode == 1)
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, kSc1);
      else
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
    }
  }
}

// k-fragment image (tower_common.h kfrag_idx) of the slice: per 16-row quarter and
// tile, 32 lanes x 16 B = the quarter's contiguous 512-B half of the 1 KiB block,
// built with two ds_read_b64_tr_b16 per lane (rows 32 B apart mod 256: conflict
// free).  Every lane runs the reads (EXEC all ones); rows >= B are zeros.
__device__ __forceinline__ void cl_store_kfrag(const ClArgs &a, const char *blk, int s_blk, int t0,
                                               int nt, int width, uint16_t *img, int64_t row0) {
  if (!img || a.store_mode == 2) return;
  const int bytes = static_cast<int>(kfrag_elems(a.B, width) * 2);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(img, 0, bytes, 0x00020000);
  const int per_q = nt * 32;
  const int n = 4 * per_q;
  const int i16 = threadIdx.x & 15;
  typedef short v4s_t __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;
  for (int base = 0; base < n; base += CL_THREADS) {
    const int idx = base + static_cast<int>(threadIdx.x);
    const bool on = idx < n;
    const int q = on ? idx / per_q : 0;
    const int rem = on ? idx - q * per_q : 0;
    const int t = rem >> 5, gl = (rem >> 4) & 1;
    const char *p = blk + (16 * q + 8 * gl + (i16 >> 2)) * s_blk + (t * 16 + 4 * (i16 & 3)) * 2;
    const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t *)(p));
    const v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t *)(p + 4 * s_blk));
    if (!on) continue;
    const int64_t r0 = row0 + 16 * q;
    const int st = static_cast<int>(r0 >> 5), h = static_cast<int>((r0 >> 4) & 1);
    if (st >= a.nsteps) continue;  // a quarter wholly past the batch's last k step
    uint32_t w[4] = {static_cast<uint16_t>(lo[0]) | (uint32_t(static_cast<uint16_t>(lo[1])) << 16),
                     static_cast<uint16_t>(lo[2]) | (uint32_t(static_cast<uint16_t>(lo[3])) << 16),
                     static_cast<uint16_t>(hi[0]) | (uint32_t(static_cast<uint16_t>(hi[1])) << 16),
                     static_cast<uint16_t>(hi[2]) | (uint32_t(static_cast<uint16_t>(hi[3])) << 16)};
    const int64_t rlim = a.B - r0 - 8 * gl;
    if (rlim < 8) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e >= rlim) w[e >> 1] &= (e & 1) ? 0x0000ffffu : 0xffff0000u;
    }
    const int off = (((t0 + t) * a.nsteps + st) * 64 + i16 + 16 * (2 * h + gl)) * 16;
    if (a.store_mode == 1)
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{w[0], w[1], w[2], w[3]}, rs, off, 0, kSc1);
    else
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{w[0], w[1], w[2], w[3]}, rs, off, 0, 0);
  }
}

__device__ __forceinline__ void cl_out(const ClArgs &a, const char *blk, int t0, int nt, int width,
                                       uint16_t *dst, int64_t ld, int64_t row0) {
  if (a.kfrag)
    cl_store_kfrag(a, blk, a.s_own, t0, nt, width, dst, row0);
  else
    cl_store_rows(a, blk, a.s_own, t0, nt, width, dst, ld, row0);
}

// ---------------------------------------------------------------------------
// one layer: the wave's weight fragments are issued right after the previous
// hand-off was signalled (all k steps at once: they load while the workgroup waits
// for its peers), then the peers' slices, then the MFMA k loop
// ---------------------------------------------------------------------------

constexpr int CL_KS = 16;  // k steps of a layer input (widths <= 512)

struct ClWait {  // what to do before the k loop
  unsigned long long *stamp_poll;  // LDS slots stamped after the poll / the gather (or NULL)
  unsigned long long *stamp_in;
  ClSync sy;
  int hand;         // < 0: nothing to wait for (layer 0: x0 is already in IN)
  const uint16_t *xb;
  int T, t0, t1;
  int64_t row0;
};

__device__ __forceinline__ void cl_do_wait(const ClArgs &a, const ClWait &w, char *in) {
  if (w.hand < 0) return;
  if (!(a.diag & 1)) cl_wait(a, w.sy, static_cast<unsigned>(w.hand));
  if (w.stamp_poll && threadIdx.x == 0) *w.stamp_poll = wall_clock64();
  if (!(a.diag & 4)) cl_gather_peers(a, w.xb, in, w.T, w.t0, w.t1, w.row0);
  __syncthreads();
  if (w.stamp_in && threadIdx.x == 0) *w.stamp_in = wall_clock64();
}

// the wave's fragments of output tile `tile` for every k step (rot: the first step)
__device__ __forceinline__ void cl_issue(bf16x8 (&wfr)[CL_KS], const uint16_t *img, int img_bytes,
                                         int ksteps, int tile, int rot, bool act, int diag = 0) {
  if (!act || (diag & 2)) return;
  const int lane = threadIdx.x & 63;
  const int voff = (tile * ksteps * 512 + lane * 8) * 2;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(img), 0, img_bytes, 0x00020000);
#pragma unroll
  for (int s = 0; s < CL_KS; ++s)
    if (s < ksteps)
      wfr[s] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, cl_rot(s, rot, ksteps) * 1024, 0));
}

__device__ __forceinline__ int cl_rot_of(const ClArgs &a, int cluster, int ksteps) {
  return a.rotate ? cluster % ksteps : 0;
}

// The k loop of one wave's tile over all 4 row tiles: the activation fragments of
// step s + 1 are read from LDS while step s's MFMAs run (register double buffer)
template <int KS>
__device__ __forceinline__ void cl_kloop(f32x4 (&acc)[4], const bf16x8 (&wfr)[CL_KS],
                                         const char *brow, int s_in, int rot) {
  const int s16 = 16 * s_in;
  bf16x8 b[2][4];
  {
    const int kk = cl_rot(0, rot, KS) * 64;
#pragma unroll
    for (int r = 0; r < 4; ++r) b[0][r] = *reinterpret_cast<const bf16x8 *>(brow + r * s16 + kk);
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int cur = s & 1;
    if (s + 1 < KS) {
      const int kk = cl_rot(s + 1, rot, KS) * 64;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        b[cur ^ 1][r] = *reinterpret_cast<const bf16x8 *>(brow + r * s16 + kk);
    }
    // fence: the next step's 4 LDS reads stay ahead of this step's 4 MFMAs (the
    // scheduler otherwise sinks each read to just before its MFMA: 2 in flight)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[s], b[cur][r], acc[r], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// One layer of the slice: out tile t0 + wave (if the slice has it) over all 64
// rows, from the fragments in wfr (cl_issue: fwd image = tiles over out features,
// bwd image = tiles over in features; `ksteps` = k steps of the input width).
// Epilogue into `out` ([64][s_own], local columns): FWD relu(acc + bias) (columns
// >= width_out -> 0); BWD acc * [mask > 0] (mask may alias out: same element, same
// lane), columns >= width_out -> 0.
template <bool BWD>
__device__ __forceinline__ void cl_layer(const ClArgs &a, const bf16x8 (&wfr)[CL_KS], int ksteps,
                                         int width_out, int t0, int nt, char *in, char *out,
                                         const float *bias, const char *mask, const ClWait &w,
                                         int cluster) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const bool act = wave < nt;
  const int t = t0 + wave;
  cl_do_wait(a, w, in);
  if (!act) return;
  f32x4 acc[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int rot = cl_rot_of(a, cluster, ksteps);
  const char *brow = in + r16 * a.s_in + g * 16;
  switch (ksteps) {  // compile-time k steps: one straight-line, branch-free k loop
#define CL_KCASE(K) \
    case K: cl_kloop<K>(acc, wfr, brow, a.s_in, rot); break;
    CL_KCASE(1) CL_KCASE(2) CL_KCASE(3) CL_KCASE(4) CL_KCASE(5) CL_KCASE(6) CL_KCASE(7)
    CL_KCASE(8) CL_KCASE(9) CL_KCASE(10) CL_KCASE(11) CL_KCASE(12) CL_KCASE(13) CL_KCASE(14)
    CL_KCASE(15) CL_KCASE(16)
#undef CL_KCASE
    default: break;
  }
  const int cl0 = 16 * wave + 4 * g;  // local column of acc[r][0]
  const int c0 = 16 * t + 4 * g;      // its global column
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = 16 * r + r16;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = c0 + i;
      float x = acc[r][i];
      if constexpr (!BWD)
        x = c < width_out ? fmaxf(x + bias[cl0 + i], 0.f) : 0.f;
      else
        x = c < width_out ? x : 0.f;
      v[i] = x;
    }
    if (BWD && mask) {
      const uint2 mk = *reinterpret_cast<const uint2 *>(mask + m * a.s_own + cl0 * 2);
      if (!bf16_pos(mk.x & 0xffffu)) v[0] = 0.f;
      if (!bf16_pos(mk.x >> 16)) v[1] = 0.f;
      if (!bf16_pos(mk.y & 0xffffu)) v[2] = 0.f;
      if (!bf16_pos(mk.y >> 16)) v[3] = 0.f;
    }
    *reinterpret_cast<uint2 *>(out + m * a.s_own + cl0 * 2) =
        make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
  }
}

// diagnostics: stamps go to LDS and leave at the end of the workgroup
#define CL_STAMP(k)                                                                  \
  do {                                                                               \
    if (a.stamps && tid == 0) s_stamp[(k)] = wall_clock64();                         \
  } while (0)

// stamp slots: 0 start, 1 x0 in; fwd layer l: 2+4l poll, 3+4l peers in, 4+4l done,
// 5+4l published (L <= 3 fits; deeper towers stamp the first three); 14 z published,
// 15 z in, 16 dh_L published; bwd step j (layer L-1-j): 17+4j poll, 18+4j in,
// 19+4j done, 20+4j published; 31 end
__global__ __launch_bounds__(CL_THREADS) void tower_cl_kernel(ClArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  __shared__ unsigned long long s_stamp[32];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  // cluster of this workgroup: with a grid of whole multiples of 32 the 4 members
  // are blocks b, b + 8, b + 16, b + 24 (one XCD under the observed round-robin
  // placement: their hand-offs can stay in its L2), else 4 consecutive blocks
  const int bid = static_cast<int>(blockIdx.x);
  const int grid = static_cast<int>(gridDim.x);
  int cluster, c;
  if ((grid & 31) == 0) {
    const int q = bid >> 3;
    cluster = (bid & 7) * (grid >> 5) + (q >> 2);
    c = q & 3;
  } else {
    cluster = bid >> 2;
    c = bid & 3;
  }
  const int64_t row0 = static_cast<int64_t>(cluster) * CL_ROWS;
  const int L = a.L;
  __shared__ unsigned s_sync[2];  // epoch, local
  char *in = lds + a.off_in;
  float *f_z = reinterpret_cast<float *>(lds + a.off_f);
  float *f_dz = f_z + CL_ROWS;
  float *f_loss = f_dz + CL_ROWS;
  float *prm = reinterpret_cast<float *>(lds + a.off_p);
  float *p_hw = prm + CL_MAXL * 128;
  float *p_y = p_hw + 128;
  float *p_base = p_y + CL_ROWS;
  float *p_b0 = p_base + CL_ROWS;
  float *p_ws = p_b0 + 4;             // ns side-linear weights (c == 0)
  float *p_xs = p_ws + 64;            // [64][ns] side-linear inputs (c == 0)
  const int H = a.width[L];
  const int ns = c == 0 ? a.ns : 0;
  unsigned long long *stp = a.stamps ? s_stamp : nullptr;
  auto slot = [&](int k) -> unsigned long long * { return (stp && k < 31) ? stp + k : nullptr; };
  CL_STAMP(0);
  if (tid == 0) {  // this launch's epoch; announce this member's XCD to the cluster
    const unsigned ep = __hip_atomic_load(a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_sync[0] = ep;
    __hip_atomic_store(a.xcc + cluster * CL_WG + c, ((ep + 1) << 4) | cl_xcc_id(), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  bf16x8 wfr[CL_KS];  // the next layer's weight fragments of this wave's tile

  // ---- prologue: x0 rows and layer 0's weights in flight together; zero IN (pad
  // columns), stage the slice's parameters, x0 -> IN, x0's k-fragment image ----------
  {
    const int xch = tw_ceil(a.width[0], 8);
    constexpr int XQ = (CL_ROWS * 64) / CL_THREADS;  // <= 64 chunks per row (512 columns)
    const int xrows = static_cast<int>(min<int64_t>(CL_ROWS, a.B - row0));
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(a.x0 + row0 * a.ld_x0), 0, static_cast<int>(xrows * a.ld_x0 * 2),
        0x00020000);
    u32x4 xr[XQ];  // unconditional loads (out-of-range offsets read zeros), one wait
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int i = tid + q * CL_THREADS;
      const int r = i / xch, k = i - r * xch;
      const int off = (i < CL_ROWS * xch && r < xrows) ? static_cast<int>((r * a.ld_x0 + k * 8) * 2)
                                                       : 0x40000000;
      xr[q] = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0);
    }
    {
      const int T = tw_ceil(a.width[1], 16);
      const int t0 = cl_t0(T, c);
      const int ks = tw_ceil(a.width[0], 32);
      cl_issue(wfr, a.wf[0], a.wf_bytes[0], ks, t0 + wave, cl_rot_of(a, cluster, ks),
               wave < cl_t0(T, c + 1) - t0, a.diag);
    }
    float pb[CL_MAXL];
#pragma unroll
    for (int l = 0; l < CL_MAXL; ++l) {  // own columns of each layer's output (<= 128)
      pb[l] = 0.f;
      if (l < L && tid < 128 && a.bias[l]) {
        const int T = tw_ceil(a.width[l + 1], 16);
        const int col = 16 * cl_t0(T, c) + tid;
        if (col < a.width[l + 1] && tid < 16 * (cl_t0(T, c + 1) - cl_t0(T, c))) pb[l] = a.bias[l][col];
      }
    }
    float phw = 0.f, py = 0.f, pbase = 0.f, pb0 = 0.f, pws = 0.f;
    {
      const int T = tw_ceil(H, 16);
      const int col = 16 * cl_t0(T, c) + tid;
      if (tid < 128 && col < H && tid < 16 * (cl_t0(T, c + 1) - cl_t0(T, c))) phw = a.head_w[col];
    }
    const bool yrow = tid < CL_ROWS && row0 + tid < a.B;
    const float *ysrc = a.mode == MREC_TOWER_GIVEN_DZ ? a.dz_in : a.y;
    py = (yrow && ysrc) ? ysrc[row0 + tid] : 0.f;
    pbase = (yrow && a.base) ? a.base[row0 + tid] : 0.f;
    if (tid == 0) pb0 = (a.head_b ? a.head_b[0] : 0.f) + (a.b2 ? a.b2[0] : 0.f);
    if (tid < ns) pws = a.ws[tid];
    float pxs[8];  // [64][ns <= 64] side inputs: 8 per thread
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = tid + q * CL_THREADS;
      const int r = ns ? i / ns : 0, j = i - r * ns;
      pxs[q] = (i < CL_ROWS * ns && row0 + r < a.B) ? a.xs[(row0 + r) * a.ld_xs + j] : 0.f;
    }
    for (int i = tid * 16; i < CL_ROWS * a.s_in; i += CL_THREADS * 16)
      *reinterpret_cast<uint4 *>(in + i) = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int l = 0; l < CL_MAXL; ++l)
      if (l < L && tid < 128) prm[l * 128 + tid] = pb[l];
    if (tid < 128) p_hw[tid] = phw;
    if (tid < CL_ROWS) {
      p_y[tid] = py;
      p_base[tid] = pbase;
    }
    if (tid == 0) p_b0[0] = pb0;
    if (tid < 64) p_ws[tid] = pws;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = tid + q * CL_THREADS;
      if (i < CL_ROWS * ns) p_xs[i] = pxs[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int i = tid + q * CL_THREADS;
      const int r = i / xch, k = i - r * xch;
      if (i < CL_ROWS * xch) *reinterpret_cast<u32x4 *>(in + r * a.s_in + k * 16) = xr[q];
    }
    __syncthreads();
    CL_STAMP(1);
    // all 4 members on one XCD?  (their announcements are long out by now)
    if (tid == 0) {
      const unsigned want = (s_sync[0] + 1) << 4;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(a.xcc + cluster * CL_WG, 0, 16, 0x00020000);
      unsigned n = 0;
      u32x4 f;
      while (true) {
        f = __builtin_amdgcn_raw_buffer_load_b128(rs, 0, 0, kSc1);
        if ((f[0] >> 4) == (want >> 4) && (f[1] >> 4) == (want >> 4) && (f[2] >> 4) == (want >> 4) &&
            (f[3] >> 4) == (want >> 4))
          break;
        __builtin_amdgcn_s_sleep(1);
        if (++n == CL_SPIN_MAX) {
          __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      const bool same = f[0] == f[1] && f[1] == f[2] && f[2] == f[3];
      s_sync[1] = (same && !a.force_sc1) ? 1u : 0u;
    }
    __syncthreads();
    if (a.kfrag && a.x0_img && a.mode != MREC_TOWER_FORWARD) {
      // x0's k-fragment image (this workgroup's column slice), out while layer 0 runs
      const int T0 = tw_ceil(a.width[0], 16);
      const int s0 = cl_t0(T0, c), s1 = cl_t0(T0, c + 1);
      cl_store_kfrag(a, in + 32 * s0, a.s_in, s0, s1 - s0, a.width[0], a.x0_img, row0);
    }
  }

  const ClSync sy{a.flags + cluster * CL_WG, s_sync[0] * 64u, c, static_cast<int>(s_sync[1])};

  // ---- forward -------------------------------------------------------------------
  int hand = 0;  // hand-offs completed
  for (int l = 0; l < L; ++l) {
    const int w_out = a.width[l + 1];
    const int T = tw_ceil(w_out, 16);
    const int t0 = cl_t0(T, c), t1 = cl_t0(T, c + 1);
    const int Tin = tw_ceil(a.width[l], 16);
    ClWait w{slot(2 + 4 * l), slot(3 + 4 * l), sy, l == 0 ? -1 : hand - 1,
             a.xb[(hand - 1) & 1], Tin, cl_t0(Tin, c), cl_t0(Tin, c + 1), row0};
    char *own = lds + a.off_own[l];
    cl_layer<false>(a, wfr, tw_ceil(a.width[l], 32), w_out, t0, t1 - t0, in, own, prm + l * 128,
                    nullptr, w, cluster);
    __syncthreads();  // OWN[l] complete, IN free
    if (l < 3) CL_STAMP(4 + 4 * l);
    if (l + 1 < L) {
      uint16_t *xb = a.xb[hand & 1];
      cl_publish(a, own, in, xb, t0, t1 - t0, row0, sy.local);
      cl_signal(sy, static_cast<unsigned>(hand));
      ++hand;
      if (l < 3) CL_STAMP(5 + 4 * l);
      // the next layer's weights load while this workgroup waits for its peers
      const int Tn = tw_ceil(a.width[l + 2], 16);
      const int n0 = cl_t0(Tn, c);
      const int ks = tw_ceil(w_out, 32);
      cl_issue(wfr, a.wf[l + 1], a.wf_bytes[l + 1], ks, n0 + wave, cl_rot_of(a, cluster, ks),
               wave < cl_t0(Tn, c + 1) - n0, a.diag);
      if (a.mode != MREC_TOWER_FORWARD)
        cl_out(a, own, t0, t1 - t0, w_out, a.h_out[l], a.ld_h[l], row0);
    }
  }

  // ---- head: partial logits over the own columns of h_L, swapped by all 4 --------
  const char *hL = lds + a.off_own[L - 1];
  const int TH = tw_ceil(H, 16);
  const int h0 = cl_t0(TH, c), h1 = cl_t0(TH, c + 1);
  const int hcols = min(16 * (h1 - h0), H - 16 * h0);  // real own columns
  {
    const int m = tid >> 3, j = tid & 7;  // 64 rows x 8 lanes
    float dot = 0.f;
    for (int k = j; k * 8 < hcols; k += 8) {  // p_hw is zero past the real columns
      const uint4 hv = *reinterpret_cast<const uint4 *>(hL + m * a.s_own + k * 16);
      float hf[8];
      Vec<uint16_t>::to_f32(hv, hf);
#pragma unroll
      for (int q = 0; q < 8; ++q) dot = fmaf(hf[q], p_hw[k * 8 + q], dot);
    }
    for (int q = j; q < ns; q += 8) dot = fmaf(p_xs[m * ns + q], p_ws[q], dot);
    dot += __shfl_xor(dot, 1);
    dot += __shfl_xor(dot, 2);
    dot += __shfl_xor(dot, 4);
    if (j == 0) {
      float *zd = a.zx + (static_cast<int64_t>(cluster) * CL_WG + c) * CL_ROWS + m;
      if (sy.local)
        *reinterpret_cast<volatile float *>(zd) = dot;
      else
        __hip_atomic_store(zd, dot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  cl_signal(sy, static_cast<unsigned>(hand));
  ++hand;
  CL_STAMP(14);
  if (a.mode != MREC_TOWER_FORWARD) {  // the backward's first weights load meanwhile
    const int T = tw_ceil(a.width[L - 1], 16);
    const int t0 = cl_t0(T, c);
    const int ks = tw_ceil(H, 32);
    cl_issue(wfr, a.wb[L - 1], a.wb_bytes[L - 1], ks, t0 + wave, cl_rot_of(a, cluster, ks),
             wave < cl_t0(T, c + 1) - t0, a.diag);
  }
  cl_wait(a, sy, static_cast<unsigned>(hand - 1));
  CL_STAMP(15);
  if (tid < CL_ROWS) {
    const float *zp = a.zx + static_cast<int64_t>(cluster) * CL_WG * CL_ROWS + tid;
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < CL_WG; ++p)
      s += __hip_atomic_load(zp + p * CL_ROWS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool ok = row0 + tid < a.B;
    float d = 0.f, lo = 0.f, zz = 0.f;
    if (ok && a.mode == MREC_TOWER_GIVEN_DZ) {
      d = p_y[tid];
    } else if (ok) {
      zz = s + p_b0[0] + p_base[tid];
      const float yy = p_y[tid];
      d = (1.f / (1.f + __expf(-zz)) - yy) * a.invB;
      lo = fmaxf(zz, 0.f) - zz * yy + log1pf(__expf(-fabsf(zz)));
    }
    f_z[tid] = zz;
    f_dz[tid] = d;
    f_loss[tid] = lo;
  }
  __syncthreads();
  if (a.mode == MREC_TOWER_FORWARD) {
    if (c == 0 && tid < CL_ROWS && row0 + tid < a.B) a.z[row0 + tid] = f_z[tid];
  } else {
    // head-parameter partials (registers: h_L is overwritten by dh_L below), one row
    // per 16 rows, [sum_m dz h_L (own columns) | sum dz | sum dz xs] (c == 0: the
    // last two), as the 16-row kernel and mrec_ctr_head_finish lay them out
    const int q = tid >> 7, k = tid & 127;  // 4 quarters x 128 columns
    float hp = 0.f;
    if (k < hcols) {
#pragma unroll
      for (int m = 0; m < 16; ++m)
        hp = fmaf(f_dz[16 * q + m],
                  bf16_to_f32(*reinterpret_cast<const uint16_t *>(hL + (16 * q + m) * a.s_own + k * 2)),
                  hp);
    }
    float sp = 0.f;  // c == 0: sum dz (j = 0) / sum dz xs_j (j = 1..ns) of quarter q
    const int qs = tid / (1 + ns), js = tid - qs * (1 + ns);
    const bool side = c == 0 && qs < 4;
    if (side) {
      if (js == 0) {
        for (int m = 0; m < 16; ++m) sp += f_dz[16 * qs + m];
      } else {
        for (int m = 0; m < 16; ++m) sp = fmaf(f_dz[16 * qs + m], p_xs[(16 * qs + m) * ns + js - 1], sp);
      }
    }
    __syncthreads();  // h_L reads done before dh_L overwrites it
    // dh_L = dz * head_w * [h_L > 0], in place over the own h_L slice
    {
      char *g0 = lds + a.off_own[L - 1];
      const int m = tid >> 3, j = tid & 7;
      const float d = f_dz[m];
      for (int kk = j; kk < 2 * (h1 - h0); kk += 8) {
        const uint4 hv = *reinterpret_cast<const uint4 *>(g0 + m * a.s_own + kk * 16);
        const uint32_t hwd[4] = {hv.x, hv.y, hv.z, hv.w};
        float gv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t hb = (e & 1) ? (hwd[e >> 1] >> 16) : (hwd[e >> 1] & 0xffffu);
          gv[e] = bf16_pos(hb) ? d * p_hw[kk * 8 + e] : 0.f;  // pad columns: h = 0
        }
        *reinterpret_cast<uint4 *>(g0 + m * a.s_own + kk * 16) =
            make_uint4(pack_bf16x2(gv[0], gv[1]), pack_bf16x2(gv[2], gv[3]),
                       pack_bf16x2(gv[4], gv[5]), pack_bf16x2(gv[6], gv[7]));
      }
    }
    __syncthreads();
    {
      uint16_t *xb = a.xb[hand & 1];
      cl_publish(a, lds + a.off_own[L - 1], in, xb, h0, h1 - h0, row0, sy.local);
      cl_signal(sy, static_cast<unsigned>(hand));
      ++hand;
      CL_STAMP(16);
    }
    // the head's outputs leave behind the hand-off
    {
      const int64_t prow = (row0 >> 4) + q;
      if (k < hcols && prow * 16 < a.B) a.part[prow * a.ldp + 16 * h0 + k] = hp;
      if (side && (row0 >> 4) + qs < (a.B + 15) / 16)
        a.part[((row0 >> 4) + qs) * a.ldp + H + js] = sp;
    }
    if (c == 0) {
      if (tid < CL_ROWS && row0 + tid < a.B) {
        if (a.dz) a.dz[row0 + tid] = f_dz[tid];
        if (a.z && a.mode == MREC_TOWER_BCE) a.z[row0 + tid] = f_z[tid];
      }
      if (a.mode == MREC_TOWER_BCE && tid < 4) {
        const int64_t prow = (row0 >> 4) + tid;
        if (prow * 16 < a.B) {
          float lp = 0.f;
          for (int m = 0; m < 16; ++m) lp += f_loss[16 * tid + m];
          __hip_atomic_store(a.loss_part + prow, lp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    cl_out(a, lds + a.off_own[L - 1], h0, h1 - h0, H, a.dh_out[L - 1], a.ld_dh[L - 1], row0);

    // ---- backward: dh_l = (dh_{l+1} W_l) * [h_l > 0] (own columns of width[l]) ----
    for (int l = L - 1; l >= 0; --l) {
      const int w_out = a.width[l];
      const int T = tw_ceil(w_out, 16);
      const int t0 = cl_t0(T, c), t1 = cl_t0(T, c + 1);
      const int Tin = tw_ceil(a.width[l + 1], 16);
      const int sb = 17 + 4 * (L - 1 - l);
      ClWait w{slot(sb), slot(sb + 1), sy, hand - 1, a.xb[(hand - 1) & 1], Tin,
               cl_t0(Tin, c), cl_t0(Tin, c + 1), row0};
      // output: in place over the mask h_l (OWN[l-1]); dx0 (l == 0) into OWN[L-1]
      char *out = lds + (l > 0 ? a.off_own[l - 1] : a.off_own[L - 1]);
      cl_layer<true>(a, wfr, tw_ceil(a.width[l + 1], 32), w_out, t0, t1 - t0, in, out, nullptr,
                     l > 0 ? out : nullptr, w, cluster);
      __syncthreads();
      CL_STAMP(min(sb + 2, 30));
      if (l > 0) {
        uint16_t *xb = a.xb[hand & 1];
        cl_publish(a, out, in, xb, t0, t1 - t0, row0, sy.local);
        cl_signal(sy, static_cast<unsigned>(hand));
        ++hand;
        CL_STAMP(min(sb + 3, 30));
        const int Tn = tw_ceil(a.width[l - 1], 16);
        const int n0 = cl_t0(Tn, c);
        const int ks = tw_ceil(w_out, 32);
        cl_issue(wfr, a.wb[l - 1], a.wb_bytes[l - 1], ks, n0 + wave, cl_rot_of(a, cluster, ks),
                 wave < cl_t0(Tn, c + 1) - n0, a.diag);
        cl_out(a, out, t0, t1 - t0, w_out, a.dh_out[l - 1], a.ld_dh[l - 1], row0);
      } else {
        cl_store_rows(a, out, a.s_own, t0, t1 - t0, w_out, a.dx0, a.ld_dx0, row0);
      }
    }
  }

  // ---- teardown: the loss (last ticket holder, fixed order) and the counter reset --
  CL_STAMP(31);
  if (a.stamps && tid < 32) a.stamps[blockIdx.x * 32 + tid] = s_stamp[tid];
  __shared__ unsigned s_last;
  if (tid == 0) {
    s_last = 0u;
    if (a.mode == MREC_TOWER_BCE && c == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == static_cast<unsigned>(a.nclus) - 1 ? 1u : 0u;
    }
    // the last workgroup of the launch advances the epoch (the next launch's flags)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(a.gticket, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old == static_cast<unsigned>(grid) - 1) {
      __hip_atomic_store(a.gticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.epoch, (s_sync[0] + 1) & 0x3ffffffu, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!s_last) return;
  if (tid == 0) __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int nparts = static_cast<int>((a.B + 15) / 16);
  float t = 0.f;
  for (int k = tid; k < nparts; k += CL_THREADS)
    t += __hip_atomic_load(a.loss_part + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
  float *wsum = f_loss;
  __syncthreads();
  if (lane == 0) wsum[tid >> 6] = t;
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
    for (int w = 0; w < CL_WAVES; ++w) s += wsum[w];
    a.loss[0] = s * a.invB;
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

unsigned long long *tower_debug_stamps();  // tower.hip (mrec_tower_debug_stamps)

int64_t cl_nclus(int64_t B) { return (B + CL_ROWS - 1) / CL_ROWS; }

// workspace layout: [err, epoch, gticket | pad to 256 B][flags nclus x 16 B]
// [xcc nclus x 16 B][zx nclus x 4 x 64 f32][xb0 B x 512 bf16][xb1], parts 256-B aligned
struct ClWs {
  int64_t off_flags, off_xcc, off_zx, off_xb0, off_xb1, bytes;
};

ClWs cl_ws_layout(int64_t B) {
  auto al = [](int64_t x) { return (x + 255) / 256 * 256; };
  ClWs w{};
  const int64_t n = cl_nclus(B);
  w.off_flags = 256;
  w.off_xcc = al(w.off_flags + n * 16);
  w.off_zx = al(w.off_xcc + n * 16);
  w.off_xb0 = al(w.off_zx + n * CL_WG * CL_ROWS * 4);
  w.off_xb1 = al(w.off_xb0 + B * CL_LDX * 2);
  w.bytes = al(w.off_xb1 + B * CL_LDX * 2);
  return w;
}

static int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cus[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) v = 0;
    cus[dev] = v;
    (void)hipGetLastError();
  }
  return cus[dev];
}

}  // namespace mrec

using namespace mrec;

extern "C" {

int64_t mrec_tower_cluster_ws_bytes(int64_t batch) {
  return batch > 0 ? cl_ws_layout(batch).bytes : 0;
}

}  // extern "C"

namespace mrec {

// Launches the cluster kernel for `s` when it applies (returns true), else false
// (the caller runs the 16-row kernel).  Arguments are already validated.
bool tower_cluster_launch(const mrec_tower_args &s, hipStream_t st, mrec_status *status) {
  static const int env_off = [] {
    const char *e = getenv("MREC_TOWER_CLUSTER");
    return (e && e[0] == '0') ? 1 : 0;
  }();
  if (env_off || !s.cl_ws || s.batch <= 0) return false;
  const ClWs ws = cl_ws_layout(s.batch);
  if (s.cl_ws_bytes < ws.bytes || (reinterpret_cast<uintptr_t>(s.cl_ws) & 255)) return false;
  const int64_t nclus = cl_nclus(s.batch);
  const int cus = device_cus();
  if (cus <= 0 || nclus * CL_WG > cus) return false;  // all workgroups must be resident
  const int L = s.n_layers;
  ClArgs a{};
  a.B = s.batch;
  a.L = L;
  for (int l = 0; l <= L; ++l) a.width[l] = s.width[l];
  a.x0 = static_cast<const uint16_t *>(s.x0);
  a.ld_x0 = s.ld_x0;
  for (int l = 0; l < L; ++l) {
    a.wf[l] = static_cast<const uint16_t *>(s.w_fwd[l]);
    a.wb[l] = static_cast<const uint16_t *>(s.w_bwd[l]);
    a.wf_bytes[l] = static_cast<int>(tower_img_elems_fwd(s.width[l + 1], s.width[l]) * 2);
    a.wb_bytes[l] = static_cast<int>(tower_img_elems_bwd(s.width[l + 1], s.width[l]) * 2);
    a.bias[l] = s.bias[l];
    a.h_out[l] = static_cast<uint16_t *>(s.h_out[l]);
    a.ld_h[l] = s.ld_h[l];
    a.dh_out[l] = static_cast<uint16_t *>(s.dh_out[l]);
    a.ld_dh[l] = s.ld_dh[l];
  }
  a.head_w = s.head_w;
  a.head_b = s.head_b;
  a.base = s.base;
  a.xs = s.xs;
  a.ld_xs = s.ld_xs;
  a.ns = s.ns;
  a.ws = s.ws;
  a.b2 = s.b2;
  a.y = s.y;
  a.dx0 = static_cast<uint16_t *>(s.dx0);
  a.ld_dx0 = s.ld_dx0;
  a.z = s.z;
  a.dz = s.dz;
  a.part = s.part;
  a.ldp = s.ldp;
  a.loss_part = s.loss_part;
  a.ticket = s.ticket;
  a.loss = s.loss;
  a.invB = 1.f / static_cast<float>(s.batch);
  a.kfrag = s.kfrag ? 1 : 0;
  a.nsteps = static_cast<int>((s.batch + 31) / 32);
  a.x0_img = s.kfrag ? static_cast<uint16_t *>(s.x0_img) : nullptr;
  a.mode = s.mode;
  a.dz_in = s.dz_in;
  static const int store_env = [] {
    const char *e = getenv("MREC_TOWER_STORE");
    return e ? atoi(e) : 1;
  }();
  a.store_mode = store_env;
  static const int rot_env = [] {
    const char *e = getenv("MREC_TOWER_ROT");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  a.rotate = rot_env;
  a.stamps = tower_debug_stamps();
  static const int diag_env = [] {
    const char *e = getenv("MREC_TOWER_CL_DIAG");
    return e ? atoi(e) : 0;
  }();
  a.diag = diag_env;
  static const int sc1_env = [] {
    const char *e = getenv("MREC_TOWER_CL_SC1");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  a.force_sc1 = sc1_env;
  if (a.mode == MREC_TOWER_FORWARD) {
    a.x0_img = nullptr;
    for (int l = 0; l < L; ++l) a.h_out[l] = nullptr;
  }
  char *base = static_cast<char *>(s.cl_ws);
  a.err = reinterpret_cast<unsigned *>(base);
  a.epoch = reinterpret_cast<unsigned *>(base) + 1;
  a.gticket = reinterpret_cast<unsigned *>(base) + 2;
  a.flags = reinterpret_cast<unsigned *>(base + ws.off_flags);
  a.xcc = reinterpret_cast<unsigned *>(base + ws.off_xcc);
  a.zx = reinterpret_cast<float *>(base + ws.off_zx);
  a.xb[0] = reinterpret_cast<uint16_t *>(base + ws.off_xb0);
  a.xb[1] = reinterpret_cast<uint16_t *>(base + ws.off_xb1);
  a.nclus = static_cast<int>(nclus);
  int wmax_in = s.width[0];
  for (int l = 1; l <= L; ++l) wmax_in = std::max(wmax_in, s.width[l]);
  int off = 0;
  a.off_in = off;
  a.s_in = tw_stride(wmax_in);
  off += CL_ROWS * a.s_in;
  a.s_own = tw_stride(16 * CL_MAXT);
  for (int l = 0; l < L; ++l) {
    a.off_own[l] = off;
    off += CL_ROWS * a.s_own;
  }
  a.off_f = off;
  off += 3 * CL_ROWS * 4;
  a.off_p = off;
  off += (CL_MAXL * 128 + 128 + 2 * CL_ROWS + 4 + 64 + CL_ROWS * std::max(0, s.ns)) * 4;
  a.lds_bytes = (off + 15) / 16 * 16;
  constexpr int kMaxDyn = 160 * 1024 - 256;
  if (a.lds_bytes > kMaxDyn) return false;
  static int attr_set = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(tower_cl_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kMaxDyn);
    (void)hipGetLastError();
    return 1;
  }();
  (void)attr_set;
  tower_cl_kernel<<<dim3(static_cast<unsigned>(nclus * CL_WG)), CL_THREADS, a.lds_bytes, st>>>(a);
  *status = launch_status("mrec_tower_fwd_bwd (cluster)");
  return true;
}

}  // namespace mrec
