// MFMA bf16 GEMM for the dense towers (MLP, DCN-v2 cross, DIN attention unit).
//
//   C[m, n] = epi( sum_k A(m, k) * B(k, n) ),  A, B bf16, fp32 accumulation
//
// Operands are ROW (k contiguous) or COL (m / n contiguous).  One 256-thread
// workgroup computes a 64x64 output tile over a K slice (4 waves in 2x2, each wave
// 2x2 v_mfma_f32_16x16x32_bf16 tiles).  Operands move into LDS with
// global_load_lds_dwordx4 (LDS-DMA: no VGPR staging, no per-element VALU) in
// 64-wide k groups through a 3-deep ring (48 KiB, three workgroups per CU): group
// g+2 is in flight while the MFMAs consume group g (s_waitcnt vmcnt + barrier).
//
// LDS images (per operand, per k group of 64: 64 rows x 64 k = 8 KiB):
//   ROW: [row][8 slots of 16 B], chunk c (8 k) of row r in slot c ^ (r & 7) — the
//        XOR swizzle is applied to the per-lane DMA *source* address (the DMA
//        destination is lane-linear), so fragment reads are bank-conflict free;
//   COL: [k/8][row/16][8 k][16 rows] 256-B blocks, read back transposed with
//        ds_read_b64_tr_b16 straight into MFMA operand layout.
// Pieces outside the operand (rows >= ilim, k >= kend) are DMA'd from a zero page;
// a 16-B piece straddling the last valid k (or row, for COL) reads the operand's
// pad elements, which must be zero (every buffer libmrec writes is zero-padded).
//
// Epilogue (through LDS, 8 columns per 16-B store):
//   v = acc + bias[n]; aux = v; v = relu(v); v *= mul; v += add; v = mask>0 ? v : 0.
// b_ones_col = N appends a ones column to B: column N of the product is the row
// sum of A (the bias gradient) and goes to `ones_out` (fp32 [M]).  Split-K partial
// tiles go to a workspace and are reduced in fixed order (deterministic).
#include <algorithm>

#include "common.h"
#include "gemm_common.h"
#include "head_common.h"

namespace mrec {

constexpr int BM = 64, BN = 64;
constexpr int GEMM_THREADS = 256;
constexpr int KG = 64;                 // k per staging group
#ifndef MREC_GEMM_NBUF
#define MREC_GEMM_NBUF 3
#endif
constexpr int NBUF = MREC_GEMM_NBUF;   // k-group ring depth, 16 KiB per group: 3 -> 48 KiB, 3 WG/CU (4: +3%, 5: +5%, 6: +50% measured)
constexpr int GROUP_ELEMS = 64 * KG;   // one operand's group image (bf16 elements)
constexpr int TLD = BN + 4;            // fp32 row stride of the C tile staged in LDS

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

__device__ __attribute__((aligned(64))) uint4 g_zero_page[64];

// s_waitcnt vmcnt(n) with expcnt / lgkmcnt left unconstrained (gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
// Per-lane DMA source walker for one operand.  Every wave issues 2 instructions per
// k group (pieces t = wave and wave + 4 of the group's 8), each moving 1 KiB.
template <bool COL>
struct DmaSrc {
  const uint16_t *p[2];  // source of this lane's piece for group 0
  bool iok[2];           // row (ROW) / row-chunk (COL) inside the operand
  int kofs[2];           // this lane's k offset within a group
  int64_t step;          // elements between consecutive groups

  __device__ __forceinline__ DmaSrc(const uint16_t *base, int64_t ld, int64_t ilim, int64_t i0,
                                    int64_t k0, int wave, int lane) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = wave + 4 * u;
      int64_t i, k;
      if constexpr (!COL) {
        const int rr = lane >> 3;
        i = i0 + t * 8 + rr;
        k = ((lane & 7) ^ rr) * 8;
      } else {
        i = i0 + (lane >> 4) * 16 + (lane & 1) * 8;
        k = t * 8 + ((lane & 15) >> 1);
      }
      iok[u] = i < ilim;
      kofs[u] = static_cast<int>(k);
      p[u] = COL ? base + (k0 + k) * ld + i : base + i * ld + (k0 + k);
    }
    step = COL ? KG * ld : KG;
  }
  // issue group `kg` (k range [k0 + 64 kg, ...), valid below kend - k0) into img
  __device__ __forceinline__ void issue(int kg, int64_t krel_end, uint16_t *gimg, int wave) const {
    const uint16_t *zero = reinterpret_cast<const uint16_t *>(g_zero_page);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool ok = iok[u] && (kg * KG + kofs[u]) < krel_end;
      const uint16_t *src = ok ? p[u] + kg * step : zero;
      __builtin_amdgcn_global_load_lds(src, gimg + (wave + 4 * u) * 512, 16, 0, 0);
    }
  }
};

__device__ __forceinline__ void unpack8(const uint4 r, float (&f)[8]) {
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(w[j] << 16);
    f[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}

// 16-B epilogue of columns [n, n + 8) of row m (n % 8 == 0, n < max(N + ones, pad_to))
__device__ __forceinline__ void epilogue_chunk(const GemmArgs &g, int64_t m, int64_t n,
                                               float (&v)[8]) {
  if (g.update) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (n + j < g.N || n + j == g.b_ones_col) epilogue_elem(g, m, n + j, v[j]);
    return;
  }
  if (g.b_ones_col >= n && g.b_ones_col < n + 8 && g.ones_out) {
    float o = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (n + j == g.b_ones_col) o = v[j];
    g.ones_out[m] = o;
  }
  if (!g.vec) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (n + j < g.N || n + j < g.pad_to) epilogue_elem(g, m, n + j, v[j]);
    return;
  }
  if (n >= g.N && n >= g.pad_to) return;
  const int cnt = static_cast<int>(min<int64_t>(8, max<int64_t>(0, g.N - n)));
  if (g.bias) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += j < cnt ? g.bias[n + j] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = j < cnt ? v[j] : 0.f;
  if (g.aux)
    *reinterpret_cast<uint4 *>(g.aux + m * g.ld_aux + n) =
        make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                   pack_bf16x2(v[6], v[7]));
  if (g.act == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
  }
  if (g.mul) {
    float t[8];
    unpack8(*reinterpret_cast<const uint4 *>(g.mul + m * g.ld_mul + n), t);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= t[j];
  }
  if (g.add) {
    float t[8];
    unpack8(*reinterpret_cast<const uint4 *>(g.add + m * g.ld_add + n), t);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += t[j];
  }
  if (g.mask) {
    float t[8];
    unpack8(*reinterpret_cast<const uint4 *>(g.mask + m * g.ld_mask + n), t);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = t[j] > 0.f ? v[j] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = j < cnt ? v[j] : 0.f;
  if (n >= g.pad_to && n < g.N) return;  // (cannot happen: pad_to >= N when vec)
  if (g.c_f32) {
    float *c = static_cast<float *>(g.C) + m * g.ldc + n;
    *reinterpret_cast<float4 *>(c) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4 *>(c + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    *reinterpret_cast<uint4 *>(static_cast<uint16_t *>(g.C) + m * g.ldc + n) =
        make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                   pack_bf16x2(v[6], v[7]));
  }
}

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
#ifdef MREC_GEMM_PROF
// per-workgroup wall-clock stamps (100 MHz) of the last launch: start, first
// k group landed, main loop done, epilogue stores retired (tools/bench_gemm.py --prof)
__device__ uint64_t g_gemm_prof[4096][4];
#define GEMM_STAMP(k)                                                          \
  do {                                                                         \
    if (threadIdx.x == 0 && bz == 0 && bx < 4096) g_gemm_prof[bx][k] = wall_clock64(); \
  } while (0)
#else
#define GEMM_STAMP(k) \
  do {                \
  } while (0)
#endif

// one output tile (workgroup `bx` of the tile grid, K slice `bz`)
template <bool A_COL, bool B_COL>
__device__ __forceinline__ void gemm_tile(const GemmArgs &g, int bx, int bz, uint16_t *smem) {
  GEMM_STAMP(0);
  const int64_t kb = static_cast<int64_t>(bz) * g.k_per_split;
  const int64_t ke = min(g.K, kb + g.k_per_split);
  const int64_t krel = ke > kb ? ke - kb : 0;
  const int nkg = static_cast<int>((krel + KG - 1) / KG);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order: workgroup b runs on XCD b % 8 (dispatch round-robin; a
  // speed heuristic only), so XCD x gets the contiguous m-major tile range
  // [x * xchunk, (x + 1) * xchunk) and the N-tiles sharing an A row panel meet in
  // one XCD's L2 instead of being fetched by all eight.
  const int tile = (bx & 7) * g.xchunk + (bx >> 3);
  if (tile >= g.ntiles) return;  // uniform: padding workgroups of the last XCD slots
  const int64_t m0 = static_cast<int64_t>(tile / g.ntn) * BM;
  const int64_t n0 = static_cast<int64_t>(tile % g.ntn) * BN;
  // ring of NBUF k-group buffers, each [A group image | B group image]
  auto a_buf = [&](int kg) { return smem + (kg % NBUF) * 2 * GROUP_ELEMS; };
  auto b_buf = [&](int kg) { return smem + (kg % NBUF) * 2 * GROUP_ELEMS + GROUP_ELEMS; };
  const DmaSrc<A_COL> da(g.A, g.lda, g.M, m0, kb, wave, lane);
  const DmaSrc<B_COL> db(g.B, g.ldb, g.b_cols, n0, kb, wave, lane);
  for (int kg = 0; kg < NBUF - 1 && kg < nkg; ++kg) {
    da.issue(kg, krel, a_buf(kg), wave);
    db.issue(kg, krel, b_buf(kg), wave);
  }
  const bool ones_here = g.b_ones_col >= n0 && g.b_ones_col < n0 + BN;  // uniform

  // per-lane fragment offsets within a group image, for the group's two k steps
  const int g4 = lane >> 4, l15 = lane & 15;
  int aoff[2], boff[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if constexpr (!A_COL)
      aoff[s] = (wm * 32 + l15) * KG + ((((s * 4 + g4) ^ (lane & 7))) << 3);
    else
      aoff[s] = (s * 4 + g4) * 512 + (wm * 32 >> 4) * 128 + (l15 >> 2) * 16 + 4 * (l15 & 3);
    if constexpr (!B_COL)
      boff[s] = (wn * 32 + l15) * KG + ((((s * 4 + g4) ^ (lane & 7))) << 3);
    else
      boff[s] = (s * 4 + g4) * 512 + (wn * 32 >> 4) * 128 + (l15 >> 2) * 16 + 4 * (l15 & 3);
  }

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int kg = 0; kg < nkg; ++kg) {
    // group kg has landed for this wave when at most the one group issued after it
    // (4 DMAs per wave) is still in flight; the barrier makes that true for every
    // wave and also retires every wave's reads of the buffer about to be refilled.
    // A bare s_barrier (with a compiler memory clobber): __syncthreads' release
    // fence would wait for vmcnt(0), i.e. drain the prefetch too.
    switch (min(nkg - 1 - kg, NBUF - 2)) {  // groups allowed in flight after group kg
      case 0: wait_vmcnt<0>(); break;
      case 1: wait_vmcnt<4>(); break;
      case 2: wait_vmcnt<8>(); break;
      case 3: wait_vmcnt<12>(); break;
      case 4: wait_vmcnt<16>(); break;
      case 5: wait_vmcnt<20>(); break;
      default: wait_vmcnt<24>(); break;
    }
    asm volatile("s_barrier" ::: "memory");
    if (kg == 0) GEMM_STAMP(1);
    if (kg + NBUF - 1 < nkg) {
      da.issue(kg + NBUF - 1, krel, a_buf(kg + NBUF - 1), wave);
      db.issue(kg + NBUF - 1, krel, b_buf(kg + NBUF - 1), wave);
    }
    if (ones_here) {  // the bias-gradient ones column of this group (rare, uniform)
      uint16_t *bimg = b_buf(kg);
      const int col = static_cast<int>(g.b_ones_col - n0);
      if (tid < KG) {
        const int k = tid;
        const uint16_t v = kg * KG + k < krel ? uint16_t(0x3f80) : uint16_t(0);
        if constexpr (!B_COL)
          bimg[col * KG + ((((k >> 3) & 7) ^ (col & 7)) << 3) + (k & 7)] = v;
        else
          bimg[(k >> 3) * 512 + (col >> 4) * 128 + (k & 7) * 16 + (col & 15)] = v;
      }
      __syncthreads();
    }
    const uint16_t *ag = a_buf(kg), *bg = b_buf(kg);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if constexpr (!A_COL) {
          a[i] = *reinterpret_cast<const bf16x8 *>(ag + aoff[s] + i * 16 * KG);
        } else {
          const uint16_t *q = ag + aoff[s] + i * 128;
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)(q));
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)(q + 64));
          a[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
        if constexpr (!B_COL) {
          b[i] = *reinterpret_cast<const bf16x8 *>(bg + boff[s] + i * 16 * KG);
        } else {
          const uint16_t *q = bg + boff[s] + i * 128;
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)(q));
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s *)(q + 64));
          b[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue: C tile -> LDS (fp32) -> 8-column chunks ----
  __syncthreads();
  GEMM_STAMP(2);
  float *T = reinterpret_cast<float *>(smem);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        T[(wm * 32 + i * 16 + g4 * 4 + r) * TLD + wn * 32 + j * 16 + l15] = acc[i][j][r];
  __syncthreads();
  const int row = tid >> 2;
  const int64_t m = m0 + row;
  if (m >= g.M) return;
  const int64_t ncols = g.b_ones_col >= 0 ? g.b_ones_col + 1 : g.N;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = (tid & 3) * 16 + h * 8;
    const int64_t n = n0 + c;
    float v[8];
    const float4 x0 = *reinterpret_cast<const float4 *>(T + row * TLD + c);
    const float4 x1 = *reinterpret_cast<const float4 *>(T + row * TLD + c + 4);
    v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
    v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    if (g.split_k > 1) {
      if (n < ncols) {
        float *w = g.ws + (static_cast<int64_t>(bz) * g.M + m) * g.ldws + n;
        *reinterpret_cast<float4 *>(w) = x0;
        *reinterpret_cast<float4 *>(w + 4) = x1;
      }
    } else if (n < ncols || n < g.pad_to) {
      epilogue_chunk(g, m, n, v);
    }
  }
#ifdef MREC_GEMM_PROF
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  GEMM_STAMP(3);
#endif
}

template <bool A_COL, bool B_COL>
__global__ __launch_bounds__(GEMM_THREADS) void gemm_dma_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  gemm_tile<A_COL, B_COL>(g, blockIdx.x, blockIdx.z, smem);
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs g) {
  splitk_reduce_body(g, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------
// several independent problems in ONE launch (a backward layer's dx GEMM, its dW
// partial slabs and the previous layer's deferred dW reduction + fused SGD): the
// workgroups of problem p are [start[p], start[p+1]), starts multiples of 8 so the
// XCD-aware tile order holds inside each problem.  Latency-bound neighbours
// overlap instead of paying a launch boundary each.
// ---------------------------------------------------------------------------
constexpr int MULTI_MAX = 4;
constexpr size_t kGemmLdsMin = NBUF * 2 * GROUP_ELEMS * sizeof(uint16_t);  // <= kGemmLds
enum : int { JOB_GEMM_RR = 0, JOB_GEMM_RC = 1, JOB_GEMM_CR = 2, JOB_GEMM_CC = 3, JOB_REDUCE = 4 };

struct MultiArgs {
  int n;
  int plan_blocks;  // 0 (the embedding-backward plan rides in the interaction launch)
  int fin_blocks;   // then the CTR head finish (padded to 8)
  HeadFinishArgs fin;
  int kind[MULTI_MAX];
  int tile_blocks[MULTI_MAX];  // workgroups per K slice (GEMM jobs)
  int nblk[MULTI_MAX];         // workgroups with work (the rest pad to a multiple of 8)
  int start[MULTI_MAX + 1];
  GemmArgs g[MULTI_MAX];
};

__global__ __launch_bounds__(GEMM_THREADS) void gemm_multi_kernel(MultiArgs ma) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  if (static_cast<int>(blockIdx.x) < ma.plan_blocks + ma.fin_blocks) {  // uniform
    const int fb = blockIdx.x - ma.plan_blocks;
    if (fb < head_finish_blocks(ma.fin.H, ma.fin.ns))
      ctr_head_finish_body(ma.fin, fb, reinterpret_cast<float (*)[9]>(smem));
    return;
  }
  const int b = blockIdx.x - ma.plan_blocks - ma.fin_blocks;
  int p = 0;
  while (p + 1 < ma.n && b >= ma.start[p + 1]) ++p;  // uniform
  const int local = b - ma.start[p];
  if (local >= ma.nblk[p]) return;
  const GemmArgs &g = ma.g[p];
  switch (ma.kind[p]) {
    case JOB_GEMM_RR: gemm_tile<false, false>(g, local % ma.tile_blocks[p], local / ma.tile_blocks[p], smem); break;
    case JOB_GEMM_RC: gemm_tile<false, true>(g, local % ma.tile_blocks[p], local / ma.tile_blocks[p], smem); break;
    case JOB_GEMM_CR: gemm_tile<true, false>(g, local % ma.tile_blocks[p], local / ma.tile_blocks[p], smem); break;
    case JOB_GEMM_CC: gemm_tile<true, true>(g, local % ma.tile_blocks[p], local / ma.tile_blocks[p], smem); break;
    default: splitk_reduce_body(g, local, ma.nblk[p]); break;
  }
}

// ---------------------------------------------------------------------------
// weight prep: fp32 [N, K] -> bf16 row image [N, ldr] and/or transposed [K, ldt]
// (pad columns written as zeros)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void weight_prep_kernel(const float *__restrict__ W, int64_t N,
                                                          int64_t K, int64_t ldw,
                                                          uint16_t *__restrict__ row, int64_t ldr,
                                                          uint16_t *__restrict__ tr, int64_t ldt) {
  __shared__ float tile[32][33];
  const int64_t k0 = static_cast<int64_t>(blockIdx.x) * 32, n0 = static_cast<int64_t>(blockIdx.y) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int64_t n = n0 + r, k = k0 + tx;
    const float v = (n < N && k < K) ? W[n * ldw + k] : 0.f;
    tile[r][tx] = v;
    if (row && n < N && k < ldr) row[n * ldr + k] = f32_to_bf16_rne(v);
  }
  __syncthreads();
  if (tr) {
    for (int r = ty; r < 32; r += 8) {
      const int64_t k = k0 + r, n = n0 + tx;
      if (k < K && n < ldt) tr[k * ldt + n] = f32_to_bf16_rne(tile[tx][r]);
    }
  }
}

static bool aligned16(const void *p, int64_t ld, int es) {
  return p && (reinterpret_cast<uintptr_t>(p) & 15) == 0 && (ld * es) % 16 == 0;
}

// K slab per workgroup (multiple of 64) and the resulting split count
static void plan_split(int64_t K, int32_t split_req, int64_t *kps, int32_t *splits) {
  const int64_t s = split_req < 1 ? 1 : split_req;
  int64_t k = ((K + s - 1) / s + KG - 1) / KG * KG;
  if (k < KG) k = KG;
  *kps = k;
  *splits = static_cast<int32_t>(K > 0 ? (K + k - 1) / k : 1);
}

constexpr size_t kGemmLds = std::max<size_t>(NBUF * 2 * GROUP_ELEMS * sizeof(uint16_t),
                                             BM * TLD * sizeof(float));

template <bool AC, bool BC>
static void launch_dma(const GemmArgs &g, dim3 grid, hipStream_t s) {
  static const bool attr = [] {  // > 64 KiB of dynamic LDS must be opted into, once
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(gemm_dma_kernel<AC, BC>),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(kGemmLds));
    return true;
  }();
  (void)attr;
  gemm_dma_kernel<AC, BC><<<grid, GEMM_THREADS, kGemmLds, s>>>(g);
}

}  // namespace mrec

using namespace mrec;

extern "C" {

size_t mrec_gemm_workspace_size(int64_t M, int64_t N, int64_t K, int32_t split_k) {
  int64_t kps;
  int32_t splits;
  plan_split(K, split_k, &kps, &splits);
  if (splits <= 1) return 0;
  return static_cast<size_t>(splits) * static_cast<size_t>(M) *
         static_cast<size_t>((N + 1 + 7) / 8 * 8) * 4;
}

}  // extern "C"

namespace mrec {

// validate one GEMM call and fill its kernel arguments; *ncols_out = 0 means "no work"
static mrec_status build_gemm(int64_t M, int64_t N, int64_t K, const mrec_operand *A,
                              const mrec_operand *B, int64_t b_ones_col, int64_t b_cols,
                              const mrec_epilogue *epi, void *C, mrec_dtype c_dtype, int64_t ldc,
                              int32_t split_k, void *workspace, size_t ws_bytes, GemmArgs *out,
                              int *kind, int64_t *ncols_out) {
  MREC_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "negative size");
  MREC_CHECK_ARG(A && A->ptr && B && B->ptr && C, "NULL operand");
  MREC_CHECK_ARG(A->dtype == MREC_BF16 && B->dtype == MREC_BF16,
                 "A and B must be bf16 (prepare fp32 weights with mrec_weight_prep)");
  MREC_CHECK_ARG(aligned16(A->ptr, A->ld, 2) && aligned16(B->ptr, B->ld, 2),
                 "A/B rows must be 16-byte aligned (pointer % 16 == 0, ld % 8 == 0)");
  MREC_CHECK_ARG(c_dtype == MREC_BF16 || c_dtype == MREC_F32, "C must be bf16 or f32");
  MREC_CHECK_ARG(b_ones_col < 0 || b_ones_col == N, "b_ones_col must be -1 or N");
  MREC_CHECK_ARG(b_cols >= 0 && b_cols <= N, "b_cols must be in [0, N]");
  MREC_CHECK_ARG(split_k >= 1 && split_k <= 64, "split_k out of [1, 64]");
  MREC_CHECK_ARG(ldc >= N, "ldc too small");
  int64_t kps;
  int32_t splits;
  plan_split(K, split_k, &kps, &splits);
  if (splits > 1 && ws_bytes < mrec_gemm_workspace_size(M, N, K, split_k)) {
    set_error("mrec_gemm: workspace too small");
    return MREC_ENOSPC;
  }
  MREC_CHECK_ARG(splits == 1 || workspace, "split-K needs a workspace");
  const int64_t ncols = b_ones_col >= 0 ? N + 1 : N;
  *ncols_out = (M == 0) ? 0 : ncols;
  GemmArgs g = {};
  g.M = M;
  g.N = N;
  g.K = K;
  g.A = static_cast<const uint16_t *>(A->ptr);
  g.lda = A->ld;
  g.B = static_cast<const uint16_t *>(B->ptr);
  g.ldb = B->ld;
  *kind = (A->layout == MREC_LAYOUT_COL ? 2 : 0) | (B->layout == MREC_LAYOUT_COL ? 1 : 0);
  g.b_ones_col = b_ones_col;
  g.b_cols = b_cols;
  if (epi) {
    g.bias = epi->bias;
    g.act = epi->act;
    g.mul = static_cast<const uint16_t *>(epi->mul);
    g.ld_mul = epi->ld_mul;
    g.add = static_cast<const uint16_t *>(epi->add);
    g.ld_add = epi->ld_add;
    g.aux = static_cast<uint16_t *>(epi->aux);
    g.ld_aux = epi->ld_aux;
    g.mask = static_cast<const uint16_t *>(epi->mask);
    g.ld_mask = epi->ld_mask;
    g.ones_out = epi->ones_out;
    g.update = epi->update ? 1 : 0;
    g.lr = epi->lr;
    g.img_row = static_cast<uint16_t *>(epi->img_row);
    g.ld_img_row = epi->ld_img_row;
    g.img_tr = static_cast<uint16_t *>(epi->img_tr);
    g.ld_img_tr = epi->ld_img_tr;
    g.img_kind = epi->img_kind;
    MREC_CHECK_ARG(g.img_kind == kImgRowTr || g.img_kind == kImgTower, "bad img_kind");
    MREC_CHECK_ARG(!g.update || (c_dtype == MREC_F32 && !g.bias && !g.act && !g.mul && !g.add &&
                                 !g.aux && !g.mask),
                   "update epilogue: C must be fp32 and bias/act/mul/add/aux/mask unset");
    MREC_CHECK_ARG(g.img_kind == kImgTower || !g.img_row || g.ld_img_row >= N, "ld_img_row < N");
    MREC_CHECK_ARG(g.img_kind == kImgTower || !g.img_tr || g.ld_img_tr >= M, "ld_img_tr < M");
  }
  g.C = C;
  g.ldc = ldc;
  g.c_f32 = c_dtype == MREC_F32;
  g.pad_to = g.update ? N : std::min<int64_t>(ldc, (N + 7) / 8 * 8);
  g.ldws = (ncols + 7) / 8 * 8;
  // 16-B epilogue stores write whole 8-column chunks: only when C's rows hold
  // round8(N) columns (an [M, N] fp32 C with N = 4 mod 8 is 16-B aligned per row
  // but an 8-wide chunk at the row end would spill into the next row)
  g.vec = aligned16(C, ldc, g.c_f32 ? 4 : 2) && ldc >= (N + 7) / 8 * 8 &&
          (!g.mul || aligned16(g.mul, g.ld_mul, 2)) &&
          (!g.add || aligned16(g.add, g.ld_add, 2)) && (!g.aux || aligned16(g.aux, g.ld_aux, 2)) &&
          (!g.mask || aligned16(g.mask, g.ld_mask, 2));
  g.ws = static_cast<float *>(workspace);
  g.split_k = splits;
  g.k_per_split = kps;
  g.ntn = static_cast<int>((ncols + BN - 1) / BN);
  g.ntiles = g.ntn * static_cast<int>((M + BM - 1) / BM);
  g.xchunk = (g.ntiles + 7) / 8;
  *out = g;
  return MREC_OK;
}

int64_t reduce_blocks(const GemmArgs &g) {
  const int64_t total = g.M * (g.ldws / 4);
  return std::min<int64_t>((total + 255) / 256, 2048);
}

mrec_status build_reduce_job(const mrec_gemm_call &c, GemmArgs *g, int64_t *nblk) {
  int kind;
  int64_t ncols;
  mrec_status st = build_gemm(c.M, c.N, c.K, c.A, c.B, c.b_ones_col, c.b_cols, c.epi, c.C,
                              c.c_dtype, c.ldc, c.split_k, c.workspace, c.ws_bytes, g, &kind,
                              &ncols);
  if (st != MREC_OK) return st;
  MREC_CHECK_ARG(c.phase == MREC_GEMM_REDUCE && g->split_k > 1,
                 "a co-launched GEMM job must be a split-K REDUCE");
  *nblk = ncols > 0 ? reduce_blocks(*g) : 0;
  return MREC_OK;
}

mrec_status build_co_reduce(int32_t n_reduce, const mrec_gemm_call *reduce, CoReduce *co,
                            int *blocks) {
  *co = {};
  *blocks = 0;
  MREC_CHECK_ARG(n_reduce >= 0 && n_reduce <= kMaxCoReduce && (n_reduce == 0 || reduce),
                 "n_reduce out of [0, 6]");
  for (int i = 0; i < n_reduce; ++i) {
    int64_t nb = 0;
    mrec_status st = build_reduce_job(reduce[i], &co->g[co->n], &nb);
    if (st != MREC_OK) return st;
    if (nb == 0) continue;
    co->nblk[co->n] = static_cast<int>(nb);
    co->start[co->n] = *blocks;
    *blocks += static_cast<int>(nb);
    ++co->n;
  }
  co->start[co->n] = *blocks;
  return MREC_OK;
}

}  // namespace mrec

extern "C" {

mrec_status mrec_gemm(int64_t M, int64_t N, int64_t K, const mrec_operand *A,
                      const mrec_operand *B, int64_t b_ones_col, int64_t b_cols,
                      const mrec_epilogue *epi, void *C, mrec_dtype c_dtype, int64_t ldc,
                      int32_t split_k, void *workspace, size_t ws_bytes, mrec_stream stream) {
  GemmArgs g;
  int kind;
  int64_t ncols;
  mrec_status st = build_gemm(M, N, K, A, B, b_ones_col, b_cols, epi, C, c_dtype, ldc, split_k,
                              workspace, ws_bytes, &g, &kind, &ncols);
  if (st != MREC_OK || ncols == 0) return st;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>(8 * g.xchunk), 1u, static_cast<unsigned>(g.split_k));
  switch (kind) {
    case 0: launch_dma<false, false>(g, grid, s); break;
    case 1: launch_dma<false, true>(g, grid, s); break;
    case 2: launch_dma<true, false>(g, grid, s); break;
    default: launch_dma<true, true>(g, grid, s); break;
  }
  st = launch_status("mrec_gemm");
  if (st != MREC_OK || g.split_k == 1) return st;
  splitk_reduce_kernel<<<dim3(static_cast<unsigned>(reduce_blocks(g))), 256, 0, s>>>(g);
  return launch_status("mrec_gemm(split-k reduce)");
}

#ifdef MREC_GEMM_PROF
void mrec_gemm_prof_read(uint64_t *out, int n) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gemm_prof), sizeof(uint64_t) * 4 * n);
}
#endif

mrec_status mrec_gemm_multi(int32_t n, const mrec_gemm_call *calls, mrec_stream stream) {
  return mrec_gemm_multi_ex(n, calls, nullptr, nullptr, stream);
}

mrec_status mrec_gemm_multi_ex(int32_t n, const mrec_gemm_call *calls, const mrec_plan_job *plan,
                               const mrec_head_finish_job *finish, mrec_stream stream) {
  MREC_CHECK_ARG(n >= 0 && n <= MULTI_MAX && (n == 0 || calls), "n out of [0, 4]");
  MultiArgs ma = {};
  if (finish) {
    const mrec_head_finish_job &f = *finish;
    mrec_status st = build_head_finish(f.part, f.ldp, f.batch, f.H, f.ns, f.g, f.update, f.lr,
                                       f.w, f.bias, f.ws, f.b2, f.dw_out, f.db_out, f.dws_out,
                                       f.db2_out, &ma.fin);
    if (st != MREC_OK) return st;
    ma.fin_blocks = (f.H + 1 + f.ns + 7) / 8;
    ma.fin_blocks = (ma.fin_blocks + 7) / 8 * 8;
  }
  // the embedding-backward plan runs in the interaction launch (mrec_interact_fwd_ex):
  // inside a GEMM launch it held the GEMM at half occupancy (the plan body's registers)
  MREC_CHECK_ARG(plan == nullptr, "a plan job inside a GEMM launch is no longer supported: "
                                  "pass it to mrec_interact_fwd_ex");
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    const mrec_gemm_call &c = calls[i];
    GemmArgs g;
    int kind;
    int64_t ncols;
    mrec_status st = build_gemm(c.M, c.N, c.K, c.A, c.B, c.b_ones_col, c.b_cols, c.epi, c.C,
                                c.c_dtype, c.ldc, c.split_k, c.workspace, c.ws_bytes, &g, &kind,
                                &ncols);
    if (st != MREC_OK) return st;
    MREC_CHECK_ARG(c.phase == MREC_GEMM_FULL || c.phase == MREC_GEMM_PARTIAL ||
                       c.phase == MREC_GEMM_REDUCE, "bad phase");
    MREC_CHECK_ARG(c.phase != MREC_GEMM_FULL || g.split_k == 1,
                   "a split-K GEMM in mrec_gemm_multi must be PARTIAL (then REDUCE later)");
    MREC_CHECK_ARG(c.phase == MREC_GEMM_FULL || g.split_k > 1, "PARTIAL / REDUCE need split-K");
    const int j = ma.n;
    int64_t nb = 0;
    if (ncols > 0) {
      if (c.phase == MREC_GEMM_REDUCE) {
        ma.kind[j] = JOB_REDUCE;
        nb = reduce_blocks(g);
      } else {
        ma.kind[j] = kind;
        ma.tile_blocks[j] = 8 * g.xchunk;
        nb = static_cast<int64_t>(8) * g.xchunk * g.split_k;
      }
    }
    if (nb == 0) continue;
    ma.nblk[j] = static_cast<int>(nb);
    ma.g[j] = g;
    ma.start[j] = blocks;
    blocks += static_cast<int>((nb + 7) / 8 * 8);
    ma.n = j + 1;
  }
  if (ma.n == 0 && ma.plan_blocks == 0 && ma.fin_blocks == 0) return MREC_OK;
  ma.start[ma.n] = blocks;
  static const bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(gemm_multi_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(kGemmLds));
    return true;
  }();
  (void)attr;
  gemm_multi_kernel<<<dim3(static_cast<unsigned>(ma.plan_blocks + ma.fin_blocks + blocks)), GEMM_THREADS,
                      kGemmLds, static_cast<hipStream_t>(stream)>>>(ma);
  return launch_status("mrec_gemm_multi");
}

mrec_status mrec_weight_prep(const float *W, int64_t N, int64_t K, int64_t ldw, void *row,
                             int64_t ldr, void *tr, int64_t ldt, mrec_stream stream) {
  MREC_CHECK_ARG(W != nullptr && (row || tr), "NULL pointer");
  MREC_CHECK_ARG(N >= 0 && K >= 0 && ldw >= K, "bad shape");
  MREC_CHECK_ARG(!row || ldr >= K, "ldr < K");
  MREC_CHECK_ARG(!tr || ldt >= N, "ldt < N");
  if (N == 0 || K == 0) return MREC_OK;
  const int64_t kx = std::max<int64_t>(K, row ? ldr : K);
  const int64_t nx = std::max<int64_t>(N, tr ? ldt : N);
  const dim3 grid(static_cast<unsigned>((kx + 31) / 32), static_cast<unsigned>((nx + 31) / 32));
  weight_prep_kernel<<<grid, 256, 0, static_cast<hipStream_t>(stream)>>>(
      W, N, K, ldw, static_cast<uint16_t *>(row), ldr, static_cast<uint16_t *>(tr), ldt);
  return launch_status("mrec_weight_prep");
}

}  // extern "C"
