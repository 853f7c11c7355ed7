// Weight gradients of the fused MLP tower, dW_l = dY_l^T X_l (+ the bias gradient
// sum_b dY_l[b] in column n_in), over the batch, as split-K partial slabs
// (include/mrec.h mrec_tower_dw).
//
// Why not the generic GEMM (gemm.hip): its COL x COL path stages both operands in
// LDS through a barrier-coupled 3-deep ring and ran the tower's three dW at
// 24 us (~60 TFLOP/s, bench_gemm dw3), with every k group of a workgroup waiting on
// its slowest wave.  Here the operands are stored by the tower itself in the
// k-fragment layout (tower_common.h, kfrag_idx): one 1 KiB block per 16 columns x
// 32 batch rows, in v_mfma_f32_16x16x32_bf16 operand order for BOTH operands (lane
// l: column l % 16, rows 8 (l / 16) .. + 8).  Every wave streams its own fragments
// straight into VGPRs (one fully coalesced 1 KiB buffer load per fragment, PF k
// steps in flight, no LDS, no barrier) -- the fused tower's weight-stream pattern,
// which runs at the CU's L2 read rate.
//
// Geometry: one wave per workgroup owns a 64 x 64 output tile (4 x 4 MFMA tiles)
// for one K slice (C2: 147 tiles x 4 slices = 588 waves, ~2.3 per CU); the bias
// column's fragments are synthesised (ones).  Steps past the slice load from an
// out-of-range offset (zeros) so the pipeline never branches.  Measured (bench_gemm
// tdw, C2 tower): 15.7 us, of which ~6 us is launch + first-fragment latency +
// slab stores (a loop-free build) and the loop streams ~150 MB of fragments at
// ~65 GB/s per CU (the L2 read rate); a 256-thread variant sharing each step's 16
// fragments through LDS (half the bytes) ran 17.6-20.4 us: its per-step barrier
// serialised the waves.  Slices: 4 (8 ran equal, with twice the partial slabs).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "feed_common.h"
#include "head_common.h"
#include "tower_common.h"

namespace mrec {

#ifndef MREC_TDW_EXP
#define MREC_TDW_EXP 0
#endif
#ifndef MREC_DW_PF
#define MREC_DW_PF 4
#endif
constexpr int DW_PF = MREC_DW_PF;  // k steps of fragments in flight per wave
constexpr int DW_MAXL = 8;
constexpr int DW_TILE = 64;    // output tile edge of one wave (4 MFMA tiles)
constexpr int DW_OOB = 1 << 30;  // a voffset past every image: the load returns zeros

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct DwLayer {
  const uint16_t *dy;  // k-fragment image of dY [B, n_out]
  const uint16_t *x;   // k-fragment image of X [B, n_in]
  float *ws;           // partial slabs [splits][n_out][ldws]
  int64_t ldws;
  int n_out, n_in;
  int dy_bytes, x_bytes;
  int nbn, nbk;        // output blocks along n_out / (n_in + 1)
  int start;           // first workgroup of this layer (after the finish blocks)
};

struct DwArgs {
  int L;
  int nsteps;          // k steps of 32 batch rows
  int splits;
  int steps_per_split;
  DwLayer lay[DW_MAXL];
  int fin_blocks;
  HeadFinishArgs fin;
  FeedCopy feed;   // the batch feed's copy in workgroups [fin_blocks, fin_blocks + feed.blocks)
};

// One wave per workgroup, one 64 x 64 output tile (4 x 4 MFMA tiles) per wave.
// FEED: the launch also hosts the batch feed's copy (mrec_tower_dw_ex with a feed
// job).  Only that instantiation carries the copy body: its 32 loads in flight per
// lane cost 39 VGPRs, which every wave of the launch would reserve (164 -> 203
// VGPRs + 90 AGPRs: 2 -> 1 waves/SIMD; C3's ~980 dW tiles ran 19.5 -> 24.8 us
// without any feed job).
template <int PF, bool KC, bool FEED>
__global__ __launch_bounds__(64) void tower_dw_kernel(DwArgs a, KClock kc) {
  KcScope<KC> kc_scope(kc);
  __shared__ __attribute__((aligned(16))) float tile[64 * 68];  // epilogue transpose
  if (static_cast<int>(blockIdx.x) < a.fin_blocks) {  // uniform
    if (static_cast<int>(blockIdx.x) < head_finish_blocks(a.fin.H, a.fin.ns))
      ctr_head_finish_body<64>(a.fin, blockIdx.x, reinterpret_cast<float (*)[9]>(tile));
    return;
  }
  if constexpr (FEED) {
    if (static_cast<int>(blockIdx.x) < a.fin_blocks + a.feed.blocks) {  // uniform
      feed_copy_body<64>(a.feed, blockIdx.x - a.fin_blocks, reinterpret_cast<long long *>(tile));
      return;
    }
  }
  const int b = blockIdx.x - a.fin_blocks - a.feed.blocks;
  int l = 0;
  while (l + 1 < a.L && b >= a.lay[l + 1].start) ++l;  // uniform
  const DwLayer &y = a.lay[l];
  const int local = b - y.start;
  const int z = local % a.splits, blk = local / a.splits;
  if (blk >= y.nbn * y.nbk) return;
  const int bn = blk / y.nbk, bk = blk - bn * y.nbk;
  const int lane = threadIdx.x & 63;
  const int nt0 = bn * 4;  // the wave's first n_out tile
  const int kt0 = bk * 4;  // its first n_in (+ bias) tile
  const int s_beg = z * a.steps_per_split;
  const int s_n = max(0, min(a.nsteps, s_beg + a.steps_per_split) - s_beg);

  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(y.dy), 0, y.dy_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(y.x), 0, y.x_bytes, 0x00020000);
  // byte offset of this lane's 16 B in step s_beg of each tile (tiles past the
  // image read zeros through the range check)
  int va[4], vb[4];
  const int atiles = (y.n_out + 15) / 16, btiles = (y.n_in + 15) / 16;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    va[i] = nt0 + i < atiles ? ((nt0 + i) * a.nsteps + s_beg) * 1024 + lane * 16 : DW_OOB;
    vb[i] = kt0 + i < btiles ? ((kt0 + i) * a.nsteps + s_beg) * 1024 + lane * 16 : DW_OOB;
  }
  // the bias column n_in: its tile gets ones in that column (its other columns
  // hold X's zero padding, or nothing past the image)
  const int ones_tile = y.n_in / 16;
  const bool ones_lane = (lane & 15) == (y.n_in & 15);
  const bf16x8 ones = bf16x8{0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80};
  bool ones_j[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) ones_j[j] = kt0 + j == ones_tile && ones_lane;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[PF][4], fb[PF][4];
  auto load = [&](int p, int s) {  // step s of the slice (past it: zeros)
    const int so = s < s_n ? s * 1024 : DW_OOB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[p][i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, va[i] + so, 0, 0));
      fb[p][i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rb, vb[i] + so, 0, 0));
    }
  };
#pragma unroll
  for (int p = 0; p < PF; ++p) {
    load(p, p);
    __builtin_amdgcn_sched_barrier(0);  // issue order = consumption order (waitcnt)
  }
#if MREC_TDW_EXP == 4  // diagnostics: no main loop
  const int total = 0;
#else
  const int total = (s_n + PF - 1) / PF * PF;
#endif
  for (int base = 0; base < total; base += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      bf16x8 bj[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bj[j] = ones_j[j] ? ones : fb[p][j];
#if MREC_TDW_EXP == 1  // diagnostics: loads only
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][0][0] += __builtin_bit_cast(float, int(fa[p][i][0] ^ bj[i][1]));
#else
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[p][i], bj[j], acc[i][j], 0, 0, 0);
#endif
#if MREC_TDW_EXP != 2  // 2: MFMAs on the prologue's fragments only
      load(p, base + p + PF);
#endif
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // partial slab z: lane holds rows 16 i + 4 (lane / 16) + r of column 16 j +
  // lane % 16 of the tile; through LDS so that the slab rows leave as 16-B stores
  // (16 lanes = one 256-B row segment)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) tile[(i * 16 + 4 * (lane >> 4) + r) * 68 + j * 16 + (lane & 15)] = acc[i][j][r];
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): one wave, no barrier needed
  __builtin_amdgcn_wave_barrier();
  float *slab = y.ws + static_cast<int64_t>(z) * y.n_out * y.ldws;
  const int m0 = nt0 * 16, n = kt0 * 16 + (lane & 15) * 4;
#pragma unroll 4
  for (int it = 0; it < 16; ++it) {
    const int row = it * 4 + (lane >> 4);
    const int m = m0 + row;
    if (m < y.n_out && n < y.ldws) {
      const float4 v = *reinterpret_cast<const float4 *>(tile + row * 68 + (lane & 15) * 4);
#if MREC_TDW_EXP == 3  // diagnostics: no slab stores (kept alive)
      if (v.x == 1.2345e-30f)
#endif
      *reinterpret_cast<float4 *>(slab + static_cast<int64_t>(m) * y.ldws + n) = v;
    }
  }
}

// row-major bf16 [rows, cols] (row stride ld) -> k-fragment image (pad rows /
// columns zero); one thread per 16-B lane slot of the image
__global__ __launch_bounds__(256) void kfrag_pack_kernel(const uint16_t *__restrict__ x, int64_t rows,
                                                         int64_t cols, int64_t ld,
                                                         uint16_t *__restrict__ img, int64_t slots) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= slots) return;
  const int64_t nsteps = (rows + 31) / 32;
  const int64_t blk = i / 64, lane = i % 64;
  const int64_t t = blk / nsteps, s = blk - t * nsteps;
  const int64_t c = t * 16 + (lane & 15);
  const int64_t r0 = s * 32 + 8 * (lane >> 4);
  uint16_t v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (c < cols && r0 + e < rows) ? x[(r0 + e) * ld + c] : uint16_t(0);
  *reinterpret_cast<uint4 *>(img + i * 8) =
      make_uint4(v[0] | (uint32_t(v[1]) << 16), v[2] | (uint32_t(v[3]) << 16),
                 v[4] | (uint32_t(v[5]) << 16), v[6] | (uint32_t(v[7]) << 16));
}

}  // namespace mrec

using namespace mrec;

extern "C" {

int64_t mrec_kfrag_elems(int64_t rows, int64_t cols) { return kfrag_elems(rows, cols); }

mrec_status mrec_kfrag_pack(const void *x, int64_t rows, int64_t cols, int64_t ld, void *img,
                            mrec_stream stream) {
  MREC_CHECK_ARG(x && img, "NULL pointer");
  MREC_CHECK_ARG(rows >= 0 && cols >= 0 && ld >= cols, "bad shape");
  const int64_t slots = kfrag_elems(rows, cols) / 8;
  if (slots == 0) return MREC_OK;
  kfrag_pack_kernel<<<dim3(static_cast<unsigned>((slots + 255) / 256)), 256, 0,
                      static_cast<hipStream_t>(stream)>>>(static_cast<const uint16_t *>(x), rows, cols,
                                                          ld, static_cast<uint16_t *>(img), slots);
  return launch_status("mrec_kfrag_pack");
}

mrec_status mrec_tower_dw(const mrec_tower_dw_args *p, const mrec_head_finish_job *finish,
                          mrec_stream stream) {
  return mrec_tower_dw_ex(p, finish, nullptr, stream);
}

mrec_status mrec_tower_dw_ex(const mrec_tower_dw_args *p, const mrec_head_finish_job *finish,
                             const mrec_feed_job *feed, mrec_stream stream) {
  MREC_CHECK_ARG(p != nullptr, "NULL args");
  const mrec_tower_dw_args &s = *p;
  MREC_CHECK_ARG(s.n_layers >= 1 && s.n_layers <= DW_MAXL, "n_layers must be in [1, 8]");
  MREC_CHECK_ARG(s.batch >= 0, "negative batch");
  MREC_CHECK_ARG(s.splits >= 1 && s.splits <= 64, "splits out of [1, 64]");
  {  // the split count the REDUCE jobs use (mrec_gemm_workspace_size(.., K = batch, splits))
    const int64_t k = ((s.batch + s.splits - 1) / s.splits + 63) / 64 * 64;
    const int64_t eff = s.batch > 0 ? (s.batch + std::max<int64_t>(k, 64) - 1) / std::max<int64_t>(k, 64) : 1;
    MREC_CHECK_ARG(eff == s.splits, "splits must be an effective split-K count for this batch "
                                    "(ceil(B / round64(ceil(B / splits))) == splits)");
  }
  DwArgs a{};
  a.L = s.n_layers;
  a.nsteps = static_cast<int>((s.batch + 31) / 32);
  a.splits = s.splits;
  a.steps_per_split = (a.nsteps + s.splits - 1) / s.splits;
  if (finish) {
    const mrec_head_finish_job &f = *finish;
    mrec_status st = build_head_finish(f.part, f.ldp, f.batch, f.H, f.ns, f.g, f.update, f.lr,
                                       f.w, f.bias, f.ws, f.b2, f.dw_out, f.db_out, f.dws_out,
                                       f.db2_out, &a.fin);
    if (st != MREC_OK) return st;
    a.fin_blocks = (f.H + 1 + f.ns + 7) / 8;
  }
  int blocks = 0;
  for (int l = 0; l < a.L; ++l) {
    const int no = s.n_out[l], ni = s.n_in[l];
    MREC_CHECK_ARG(no >= 1 && ni >= 1, "n_out / n_in must be >= 1");
    MREC_CHECK_ARG(s.dy_img[l] && s.x_img[l] && s.ws[l], "NULL image / workspace");
    MREC_CHECK_ARG(s.ldws[l] >= ni + 1, "ldws < n_in + 1");
    MREC_CHECK_ARG(kfrag_elems(s.batch, no) * 2 < DW_OOB && kfrag_elems(s.batch, ni) * 2 < DW_OOB,
                   "k-fragment image exceeds 1 GiB");
    DwLayer &y = a.lay[l];
    y.dy = static_cast<const uint16_t *>(s.dy_img[l]);
    y.x = static_cast<const uint16_t *>(s.x_img[l]);
    y.ws = s.ws[l];
    y.ldws = s.ldws[l];
    y.n_out = no;
    y.n_in = ni;
    y.dy_bytes = static_cast<int>(kfrag_elems(s.batch, no) * 2);
    y.x_bytes = static_cast<int>(kfrag_elems(s.batch, ni) * 2);
    MREC_CHECK_ARG(s.ldws[l] % 4 == 0 && reinterpret_cast<uintptr_t>(s.ws[l]) % 16 == 0,
                   "ws rows must be 16-B aligned (ldws % 4 == 0)");
    y.nbn = (no + DW_TILE - 1) / DW_TILE;
    y.nbk = (ni + 1 + DW_TILE - 1) / DW_TILE;
    y.start = blocks;
    blocks += y.nbn * y.nbk * s.splits;
  }
  if (feed) {
    if (mrec_status st = build_feed_copy(feed, 64, &a.feed); st != MREC_OK) return st;
  }
  const int grid = a.fin_blocks + a.feed.blocks + blocks;
  if (grid == 0) return MREC_OK;
  const KClock kc = kclock_take();
  const dim3 g(static_cast<unsigned>(grid));
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (a.feed.blocks > 0) {
    if (kc.buf)
      tower_dw_kernel<DW_PF, true, true><<<g, 64, 0, st>>>(a, kc);
    else
      tower_dw_kernel<DW_PF, false, true><<<g, 64, 0, st>>>(a, kc);
  } else {
    if (kc.buf)
      tower_dw_kernel<DW_PF, true, false><<<g, 64, 0, st>>>(a, kc);
    else
      tower_dw_kernel<DW_PF, false, false><<<g, 64, 0, st>>>(a, kc);
  }
  return launch_status("mrec_tower_dw");
}

}  // extern "C"
