// GEMM argument block and the split-K reduction body, shared by gemm.hip and the
// launches that run a deferred weight-gradient reduction (+ fused SGD) beside
// their own work (emb_bwd.hip: mrec_emb_bwd_apply_ex).
#pragma once
#include "common.h"
#include "tower_common.h"

namespace mrec {

struct GemmArgs {
  int64_t M, N, K;
  const uint16_t *A;
  int64_t lda;
  const uint16_t *B;
  int64_t ldb;
  int64_t b_ones_col;
  int64_t b_cols;
  const float *bias;
  int act;
  const uint16_t *mul;
  int64_t ld_mul;
  const uint16_t *add;
  int64_t ld_add;
  uint16_t *aux;
  int64_t ld_aux;
  const uint16_t *mask;
  int64_t ld_mask;
  void *C;
  int64_t ldc;
  int c_f32;
  int vec;         // C / aux / mul / add / mask rows 16-B aligned: 16-B epilogue stores
  int64_t pad_to;  // columns [N, pad_to) of C are written as 0
  float *ones_out;
  int split_k;
  int64_t k_per_split;
  float *ws;
  int64_t ldws;    // row stride of a split-K partial slab (round8(ncols))
  int ntn;         // output tiles along N
  int ntiles;      // output tiles (M x N)
  int xchunk;      // tiles per XCD slot: ceil(ntiles / 8)
  int update;      // fused SGD: C -= lr * v (fp32 master), images re-emitted
  float lr;
  uint16_t *img_row;
  int64_t ld_img_row;
  uint16_t *img_tr;
  int64_t ld_img_tr;
  int img_kind;    // kImgRowTr / kImgTower (tower_common.h)
};

__device__ __forceinline__ float bf(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }

// scalar epilogue of one element (split-K reduce and unaligned outputs)
__device__ __forceinline__ void epilogue_elem(const GemmArgs &g, int64_t m, int64_t n, float acc) {
  if (g.update) {  // fused SGD step of a master weight (+ its bias through the ones column)
    if (n == g.b_ones_col) {
      if (g.ones_out) g.ones_out[m] = fmaf(-g.lr, acc, g.ones_out[m]);
      return;
    }
    if (n >= g.N) return;
    float *c = static_cast<float *>(g.C) + m * g.ldc + n;
    const float w = fmaf(-g.lr, acc, *c);
    *c = w;
    const uint16_t h = f32_to_bf16_rne(w);
    if (g.img_kind == kImgTower) {  // W [M, N]: the fused tower's fragment images
      if (g.img_row) g.img_row[tower_idx_fwd(m, n, g.N)] = h;
      if (g.img_tr) g.img_tr[tower_idx_bwd(m, n, g.M)] = h;
      return;
    }
    if (g.img_row) g.img_row[m * g.ld_img_row + n] = h;
    if (g.img_tr) g.img_tr[n * g.ld_img_tr + m] = h;
    return;
  }
  if (n == g.b_ones_col) {
    if (g.ones_out) g.ones_out[m] = acc;
    if (n < g.pad_to) {
      if (g.c_f32)
        static_cast<float *>(g.C)[m * g.ldc + n] = 0.f;
      else
        static_cast<uint16_t *>(g.C)[m * g.ldc + n] = 0;
    }
    return;
  }
  if (n >= g.N) {
    if (n < g.pad_to) {
      if (g.c_f32)
        static_cast<float *>(g.C)[m * g.ldc + n] = 0.f;
      else
        static_cast<uint16_t *>(g.C)[m * g.ldc + n] = 0;
    }
    return;
  }
  float v = acc + (g.bias ? g.bias[n] : 0.f);
  if (g.aux) g.aux[m * g.ld_aux + n] = f32_to_bf16_rne(v);
  if (g.act == 1) v = fmaxf(v, 0.f);
  if (g.mul) v *= bf(g.mul[m * g.ld_mul + n]);
  if (g.add) v += bf(g.add[m * g.ld_add + n]);
  if (g.mask) {
    const uint16_t mv = g.mask[m * g.ld_mask + n];
    if (mv == 0 || (mv & 0x8000u)) v = 0.f;
  }
  if (g.c_f32)
    static_cast<float *>(g.C)[m * g.ldc + n] = v;
  else
    static_cast<uint16_t *>(g.C)[m * g.ldc + n] = f32_to_bf16_rne(v);
}

// the fused-SGD update of a 4 x 4 block (rows m0..m0+3, columns n..n+3 < N, m0 % 4
// == n % 4 == 0) of a weight with tower images: the fp32 master rows as float4,
// each image as four 8-byte stores -- tower_idx_fwd keeps 4 consecutive k (= n)
// of a row together, tower_idx_bwd 4 consecutive n (= m) of a column (instead of
// 32 scattered 2-byte stores)
__device__ __forceinline__ void update_block4_tower(const GemmArgs &g, int64_t m0, int64_t n,
                                                    const float4 (&v)[4]) {
  float w[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float *c = static_cast<float *>(g.C) + (m0 + r) * g.ldc + n;
    const float4 old = *reinterpret_cast<const float4 *>(c);
    w[r][0] = fmaf(-g.lr, v[r].x, old.x);
    w[r][1] = fmaf(-g.lr, v[r].y, old.y);
    w[r][2] = fmaf(-g.lr, v[r].z, old.z);
    w[r][3] = fmaf(-g.lr, v[r].w, old.w);
    *reinterpret_cast<float4 *>(c) = make_float4(w[r][0], w[r][1], w[r][2], w[r][3]);
    if (g.img_row)
      *reinterpret_cast<uint2 *>(g.img_row + tower_idx_fwd(m0 + r, n, g.N)) =
          make_uint2(pack_bf16x2(w[r][0], w[r][1]), pack_bf16x2(w[r][2], w[r][3]));
  }
  if (g.img_tr) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<uint2 *>(g.img_tr + tower_idx_bwd(m0, n + j, g.M)) =
          make_uint2(pack_bf16x2(w[0][j], w[1][j]), pack_bf16x2(w[2][j], w[3][j]));
  }
}

// slab 0 + slab 1 + ... + slab sk-1 of 4 columns, in slab order.  DEEP: the loads
// of 8 slabs are issued before their adds (one memory round trip per 8 slabs
// instead of one per slab: the DIN top tower's 16-slice reduce took 28 us as a
// dependent chain); the embedding apply's co-launched reduce (4 slices) keeps the
// plain loop, whose registers do not weigh on the apply
template <bool DEEP>
__device__ __forceinline__ float4 splitk_sum4(const float *p, int64_t slab, int sk) {
  float4 s = *reinterpret_cast<const float4 *>(p);
  int z = 1;
  if constexpr (DEEP) {
    for (; z + 8 <= sk; z += 8) {
      float4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = *reinterpret_cast<const float4 *>(p + (z + u) * slab);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s.x += t[u].x; s.y += t[u].y; s.z += t[u].z; s.w += t[u].w;
      }
    }
  }
  for (; z < sk; ++z) {
    const float4 t = *reinterpret_cast<const float4 *>(p + z * slab);
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  }
  return s;
}

// fixed-order reduction of the split-K partial slabs + epilogue (4 columns / thread)
template <bool DEEP = true>
__device__ __forceinline__ void splitk_reduce_body(const GemmArgs &g, int64_t bid, int64_t nblk) {
  const int64_t ncols = g.b_ones_col >= 0 ? g.b_ones_col + 1 : g.N;
  const int64_t q = g.ldws / 4;
  const int64_t slab = g.M * g.ldws;
  // fused SGD into tower images: 4 x 4 blocks over rows [0, M4), columns < N in
  // whole fours, the same fixed summation order per element
#ifdef MREC_NO_BLK4  // diagnostics: the per-element path only
  const bool blk4 = false;
#else
  const bool blk4 = g.update && g.img_kind == kImgTower && (g.ldc % 4) == 0 &&
                    (reinterpret_cast<uintptr_t>(g.C) & 15) == 0;
#endif
  const int64_t M4 = blk4 ? g.M / 4 * 4 : 0;
  const int64_t N4 = blk4 ? g.N / 4 : 0;  // whole column fours inside W
  if (blk4) {
    // one row of a block per lane (4 lanes per block: a quarter of the dependent slab
    // loads per thread), the block gathered by the first of the 4 lanes
    const int64_t tot4 = (M4 / 4) * N4;
    const int base = (threadIdx.x & 63) & ~3;
    for (int64_t i = bid * 256 + threadIdx.x; i < tot4 * 4; i += nblk * 256) {
      const int64_t j = i >> 2;
      const int r = static_cast<int>(i & 3);
      const int64_t m0 = (j / N4) * 4, n = (j % N4) * 4;
      const float4 mine = splitk_sum4<DEEP>(g.ws + (m0 + r) * g.ldws + n, slab, g.split_k);
      float4 v[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        v[rr] = make_float4(__shfl(mine.x, base + rr), __shfl(mine.y, base + rr),
                            __shfl(mine.z, base + rr), __shfl(mine.w, base + rr));
      if (r == 0) update_block4_tower(g, m0, n, v);
    }
  }
  const int64_t total = g.M * q;
  for (int64_t i = bid * 256 + threadIdx.x; i < total; i += nblk * 256) {
    const int64_t m = i / q, n = (i - m * q) * 4;
    if (n >= ncols && n >= g.pad_to) continue;
    if (m < M4 && n + 4 <= N4 * 4) continue;  // done above in a 4 x 4 block
    const float4 s = splitk_sum4<DEEP>(g.ws + m * g.ldws + n, slab, g.split_k);
    const float e[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (n + j < ncols || n + j < g.pad_to) epilogue_elem(g, m, n + j, e[j]);
  }
}

// host: validate a REDUCE-phase mrec_gemm_call and fill its arguments and
// workgroup count (gemm.hip)
mrec_status build_reduce_job(const mrec_gemm_call &c, GemmArgs *g, int64_t *nblk);
int64_t reduce_blocks(const GemmArgs &g);

// deferred split-K weight-gradient reductions (+ fused SGD) run by trailing
// workgroups of an embedding-update launch (emb_bwd.hip's apply kernels,
// emb_bwd_large.hip's bucket kernel): independent of the embedding update, and a
// launch of their own would cost a kernel boundary on the step's serial path
constexpr int kMaxCoReduce = 6;  // (C3: 3 cross + 2 MLP layers; kernel args stay < 4 KB)
struct CoReduce {
  int n;
  int nblk[kMaxCoReduce];
  int start[kMaxCoReduce + 1];  // workgroup offsets after the host launch's own blocks
  GemmArgs g[kMaxCoReduce];
};

__device__ __forceinline__ bool co_reduce(const CoReduce &co, int b) {
  int p = 0;
  while (p + 1 < co.n && b >= co.start[p + 1]) ++p;
  const int local = b - co.start[p];
  if (local < co.nblk[p]) splitk_reduce_body<false>(co.g[p], local, co.nblk[p]);
  return true;
}

// host: validate n_reduce REDUCE-phase calls into *co (jobs with no work dropped);
// *blocks = the workgroups they take (gemm.hip)
mrec_status build_co_reduce(int32_t n_reduce, const mrec_gemm_call *reduce, CoReduce *co,
                            int *blocks);

}  // namespace mrec
