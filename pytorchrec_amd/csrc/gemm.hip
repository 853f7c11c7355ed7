// MFMA bf16 GEMM for the dense towers (MLP, DCN-v2 cross, DIN attention unit).
//
//   C[m, n] = epi( sum_k A'(m, k) * B(k, n) )
//
// A'(m, k) = A(m, k) [* (Amod(m, k) > 0) | * Amod(m, k)]   (ReLU' mask / dz = g*x0)
// Operands are ROW (k contiguous) or COL (m / n contiguous); B may be fp32 (read
// and converted while staging) or bf16.  Everything is staged into LDS as
// [row][k] images (COL operands transposed on the way in, 8x8 blocks per thread)
// and consumed by v_mfma_f32_16x16x32_bf16 with fp32 accumulation.  Output tile
// 64x64 per 256-thread workgroup, 4 waves in 2x2, each wave 2x2 MFMA tiles.
//
// Two schedules:
//  * panel  (K <= 448, the MLP / cross / attention shapes): the whole K extent of
//    the A row panel and the B column panel is loaded into LDS in ONE phase with
//    every load in flight at once, then the block runs K/32 MFMA steps out of LDS
//    with no further global traffic.  At these small K the per-tile load latency,
//    not the MFMA rate, is what a K-loop pays; this pays it once.
//  * stream (long K: weight gradients reduce over the batch): BK = 64 tiles,
//    double-buffered, the next tile's loads issued before the current MFMAs;
//    split-K over workgroups with a fixed-order fp32 slab reduction.
//
// Epilogue: v = acc + bias[n]; aux = v; v = relu(v); v *= mul; v += add; C = v.
// b_ones_col = N appends a ones column to B: column N of the product is the row
// sum of A' (the bias gradient) and is written to `ones_out` (fp32 [M]).
#include <algorithm>

#include "common.h"

namespace mrec {

constexpr int BM = 64, BN = 64;
constexpr int GEMM_THREADS = 256;
constexpr int PANEL_KMAX = 448;
constexpr int PANEL_LD = PANEL_KMAX + 8;  // 912 B rows: 16 rows of a ds_read_b128 group hit distinct banks

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct GemmArgs {
  int64_t M, N, K;
  const void *A;
  int64_t lda;
  int a_col;
  const void *amod;
  int64_t ld_amod;
  int amod_kind;  // 0 none, 1 relu mask, 2 multiply
  const void *B;
  int64_t ldb;
  int b_col;
  int64_t b_ones_col;
  int64_t b_cols;
  const float *bias;
  int act;
  const void *mul;
  int64_t ld_mul;
  const void *add;
  int64_t ld_add;
  void *aux;
  int64_t ld_aux;
  void *C;
  int64_t ldc;
  int c_f32;
  float *ones_out;
  int a_vec, amod_vec, b_vec;
  int split_k;
  int64_t k_per_split;
  float *ws;
};

__device__ __forceinline__ float bf(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }

// ---- slab staging --------------------------------------------------------
// A workgroup stages a [64 rows][klen] slab of A and of B (klen <= 448) into
// LDS [row][k] images.  Every thread first issues ALL of its 16-byte loads for
// the slab (registers are the staging buffer: up to 16 per operand, plus 16 for
// the A modifier), then applies the modifier / 8x8 transpose and writes LDS.
//   ROW operand: 8 threads per row, 32 rows per pass, 2 passes, <= 7 chunks per pass
//   COL operand: unit = 8x8 block (8 k rows x 8 rows), 8 * kc units, <= 2 per
//                thread, 8 loads each
constexpr int ROW_UNITS = 14;  // 2 passes x 7 chunks (56 chunks = 448 per row / 8 threads)
constexpr int COL_UNITS = 2;   // ceil(8 * 56 / 256)
constexpr int MAX_LOADS = 16;

__device__ __forceinline__ uint16_t h16(const uint4 &w, int j) {
  const uint32_t x = (j < 2) ? w.x : (j < 4) ? w.y : (j < 6) ? w.z : w.w;
  return uint16_t((j & 1) ? (x >> 16) : (x & 0xffffu));
}

__device__ __forceinline__ uint4 mod16(int kind, const uint4 &a, const uint4 &m) {
  uint16_t t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint16_t av = h16(a, j), mv = h16(m, j);
    t[j] = (kind == 1) ? ((mv != 0 && !(mv & 0x8000u)) ? av : uint16_t(0))
                       : f32_to_bf16_rne(bf(av) * bf(mv));
  }
  return make_uint4(uint32_t(t[0]) | (uint32_t(t[1]) << 16), uint32_t(t[2]) | (uint32_t(t[3]) << 16),
                    uint32_t(t[4]) | (uint32_t(t[5]) << 16), uint32_t(t[6]) | (uint32_t(t[7]) << 16));
}

// Operand view: element (i, k) of the GEMM operand (i = output row for A, output
// column for B) lives at ptr[i*ld + k] (ROW) or ptr[k*ld + i] (COL).
struct OpView {
  const uint16_t *p;
  int64_t ld;
  int64_t ilim;  // valid i (rows of A = M; columns of B = b_cols)
  bool vec;
};

template <bool COL>
struct Stager {
  static constexpr int NL = COL ? COL_UNITS * 8 : ROW_UNITS;
  uint4 r[NL];

  // Issue every load of this thread for slab rows [i0, i0+64), k in [k0, k0+klen):
  // unconditional 16-B loads from clamped addresses — no branch, no wait between
  // them; out-of-range elements are zeroed in mask().  Rows are 16-B aligned with
  // ld a multiple of 8 (checked on the host), so a chunk never leaves its row.
  __device__ __forceinline__ void issue(const OpView &v, int64_t i0, int64_t k0, int klen,
                                        int64_t kend) {
    const int tid = threadIdx.x;
    const int kc = klen / 8;
    if constexpr (!COL) {
      // 8 threads per row (128 contiguous bytes per row per instruction), 32 rows
      // per pass, 2 passes; chunk j of a thread is k8 = (8j + q) * 8
      const int q = tid & 7;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int64_t i = i0 + (tid >> 3) + 32 * p;
        const uint16_t *rowp = v.p + (i < v.ilim ? i : 0) * v.ld + k0;
#pragma unroll
        for (int j = 0; j < ROW_UNITS / 2; ++j) {
          const int ch = 8 * j + q;
          const bool ok = ch < kc && i < v.ilim && k0 + ch * 8 < kend;
          r[p * (ROW_UNITS / 2) + j] =
              *reinterpret_cast<const uint4 *>(ok ? rowp + ch * 8 : v.p);
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < COL_UNITS; ++u) {
        const int c = tid + u * GEMM_THREADS;
        const int rb = c & 7, k8 = (c >> 3) * 8;
        const int64_t i = i0 + rb * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int64_t k = k0 + k8 + j;
          const bool ok = c < 8 * kc && k < kend && i < v.ilim;
          r[u * 8 + j] = *reinterpret_cast<const uint4 *>(v.p + (ok ? k * v.ld + i : 0));
        }
      }
    }
  }

  // zero every element outside [0, ilim) x [k0, kend) (after the loads landed);
  // branch-free word selects so the compiler never drains the load queue early
  __device__ __forceinline__ static uint4 keep_first(const uint4 &x, int keep) {
    uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t lo = (2 * q < keep) ? 0x0000ffffu : 0u;
      const uint32_t hi = (2 * q + 1 < keep) ? 0xffff0000u : 0u;
      w[q] &= (lo | hi);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
  __device__ __forceinline__ void mask(const OpView &v, int64_t i0, int64_t k0, int klen,
                                       int64_t kend) {
    const int tid = threadIdx.x;
    const int kc = klen / 8;
    if constexpr (!COL) {
      const int q = tid & 7;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int64_t i = i0 + (tid >> 3) + 32 * p;
#pragma unroll
        for (int j = 0; j < ROW_UNITS / 2; ++j) {
          const int ch = 8 * j + q;
          const int64_t k = k0 + ch * 8;
          const bool ok = ch < kc && i < v.ilim && k < kend;
          const int keep = ok ? static_cast<int>(min<int64_t>(8, kend - k)) : 0;
          r[p * (ROW_UNITS / 2) + j] = keep_first(r[p * (ROW_UNITS / 2) + j], keep);
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < COL_UNITS; ++u) {
        const int c = tid + u * GEMM_THREADS;
        const int rb = c & 7, k8 = (c >> 3) * 8;
        const int64_t i = i0 + rb * 8;
        const int keep_i = static_cast<int>(min<int64_t>(8, max<int64_t>(0, v.ilim - i)));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const bool ok = c < 8 * kc && k0 + k8 + j < kend;
          r[u * 8 + j] = keep_first(r[u * 8 + j], ok ? keep_i : 0);
        }
      }
    }
  }

  __device__ __forceinline__ void apply(int kind, const Stager &m) {
#pragma unroll
    for (int u = 0; u < NL; ++u) r[u] = mod16(kind, r[u], m.r[u]);
  }

  // write the staged registers into the [64][ld] LDS image
  __device__ __forceinline__ void commit(uint16_t *S, int ld, int klen) const {
    const int tid = threadIdx.x;
    const int kc = klen / 8;
    if constexpr (!COL) {
      const int q = tid & 7;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        uint16_t *rowS = S + ((tid >> 3) + 32 * p) * ld;
#pragma unroll
        for (int j = 0; j < ROW_UNITS / 2; ++j) {
          const int ch = 8 * j + q;
          if (ch < kc) *reinterpret_cast<uint4 *>(rowS + ch * 8) = r[p * (ROW_UNITS / 2) + j];
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < COL_UNITS; ++u) {
        const int c = tid + u * GEMM_THREADS;
        if (c < 8 * kc) {
          const int rb = c & 7, k8 = (c >> 3) * 8;
#pragma unroll
          for (int jn = 0; jn < 8; ++jn) {  // row rb*8+jn gets k8..k8+7 = column jn of the block
            uint16_t t[8];
#pragma unroll
            for (int jk = 0; jk < 8; ++jk) t[jk] = h16(r[u * 8 + jk], jn);
            *reinterpret_cast<uint4 *>(S + (rb * 8 + jn) * ld + k8) =
                make_uint4(uint32_t(t[0]) | (uint32_t(t[1]) << 16),
                           uint32_t(t[2]) | (uint32_t(t[3]) << 16),
                           uint32_t(t[4]) | (uint32_t(t[5]) << 16),
                           uint32_t(t[6]) | (uint32_t(t[7]) << 16));
          }
        }
      }
    }
  }
};

__device__ __forceinline__ void epilogue_elem(const GemmArgs &g, int64_t m, int64_t n, float acc) {
  if (n == g.b_ones_col) {
    if (g.ones_out) g.ones_out[m] = acc;
    return;
  }
  float v = acc + (g.bias ? g.bias[n] : 0.f);
  if (g.aux) static_cast<uint16_t *>(g.aux)[m * g.ld_aux + n] = f32_to_bf16_rne(v);
  if (g.act == 1) v = fmaxf(v, 0.f);
  if (g.mul) v *= bf(static_cast<const uint16_t *>(g.mul)[m * g.ld_mul + n]);
  if (g.add) v += bf(static_cast<const uint16_t *>(g.add)[m * g.ld_add + n]);
  if (g.c_f32)
    static_cast<float *>(g.C)[m * g.ldc + n] = v;
  else
    static_cast<uint16_t *>(g.C)[m * g.ldc + n] = f32_to_bf16_rne(v);
}

__device__ __forceinline__ void mfma_step(const uint16_t *As, const uint16_t *Bs, int ld, int k,
                                          int wm, int wn, int lane, f32x4 (&acc)[2][2]) {
  const int fr = lane & 15, fk = k + (lane >> 4) * 8;
  bf16x8 a[2], b[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
    a[i] = *reinterpret_cast<const bf16x8 *>(As + (wm * 32 + i * 16 + fr) * ld + fk);
#pragma unroll
  for (int j = 0; j < 2; ++j)
    b[j] = *reinterpret_cast<const bf16x8 *>(Bs + (wn * 32 + j * 16 + fr) * ld + fk);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
}

__device__ __forceinline__ void write_tile(const GemmArgs &g, int64_t m0, int64_t n0, int wm,
                                           int wn, int lane, const f32x4 (&acc)[2][2]) {
  const int64_t ncols = g.b_ones_col >= 0 ? g.b_ones_col + 1 : g.N;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t n = n0 + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (m < g.M && n < ncols) {
          if (g.split_k > 1)
            g.ws[(static_cast<int64_t>(blockIdx.z) * g.M + m) * ncols + n] = acc[i][j][r];
          else
            epilogue_elem(g, m, n, acc[i][j][r]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// slab kernel: one K slab (<= 448) per workgroup, staged in one phase
// ---------------------------------------------------------------------------
template <bool A_COL, bool B_COL, bool AMOD>
__global__ __launch_bounds__(GEMM_THREADS) void gemm_slab_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t *As = smem;
  uint16_t *Bs = smem + BM * PANEL_LD;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = static_cast<int64_t>(blockIdx.y) * BM;
  const int64_t n0 = static_cast<int64_t>(blockIdx.x) * BN;
  const int64_t kb = static_cast<int64_t>(blockIdx.z) * g.k_per_split;
  const int64_t ke = min(g.K, kb + g.k_per_split);
  const int klen = ke > kb ? static_cast<int>((ke - kb + 31) / 32 * 32) : 0;
  const OpView va{static_cast<const uint16_t *>(g.A), g.lda, g.M, static_cast<bool>(g.a_vec)};
  const OpView vb{static_cast<const uint16_t *>(g.B), g.ldb, g.b_cols, static_cast<bool>(g.b_vec)};
  {
    Stager<A_COL> sa;
    Stager<B_COL> sb;
    sa.issue(va, m0, kb, klen, ke);
    sb.issue(vb, n0, kb, klen, ke);
    if constexpr (AMOD) {
      const OpView vm{static_cast<const uint16_t *>(g.amod), g.ld_amod, g.M,
                      static_cast<bool>(g.amod_vec)};
      Stager<A_COL> sm;
      sm.issue(vm, m0, kb, klen, ke);
      sa.mask(va, m0, kb, klen, ke);
      sa.apply(g.amod_kind, sm);  // masked-out A elements are 0 whatever the modifier
    } else {
      sa.mask(va, m0, kb, klen, ke);
    }
    sb.mask(vb, n0, kb, klen, ke);
    sa.commit(As, PANEL_LD, klen);
    sb.commit(Bs, PANEL_LD, klen);
    if (g.b_ones_col >= 0 && n0 <= g.b_ones_col && g.b_ones_col < n0 + BN) {
      __syncthreads();  // the commit above wrote zeros into this row (uniform branch)
      // the appended ones column of B: row (b_ones_col - n0) of the B image = 1 for k < ke
      const int rowo = static_cast<int>(g.b_ones_col - n0);
      for (int k = tid; k < klen; k += GEMM_THREADS)
        Bs[rowo * PANEL_LD + k] = (kb + k < ke) ? uint16_t(0x3f80) : uint16_t(0);
    }
  }
  __syncthreads();
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < klen; k += 32) mfma_step(As, Bs, PANEL_LD, k, wm, wn, lane, acc);
  write_tile(g, m0, n0, wm, wn, lane, acc);
}

// fixed-order reduction of split-K partial slabs + epilogue
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs g) {
  const int64_t ncols = g.b_ones_col >= 0 ? g.b_ones_col + 1 : g.N;
  const int64_t total = g.M * ncols;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    float s = 0.f;
    for (int z = 0; z < g.split_k; ++z) s += g.ws[z * total + i];
    epilogue_elem(g, i / ncols, i % ncols, s);
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

// K slab per workgroup (multiple of 32, <= PANEL_KMAX) and the resulting split count
static void plan_split(int64_t K, int32_t split_req, int64_t *kps, int32_t *splits) {
  int64_t s = split_req < 1 ? 1 : split_req;
  int64_t k = ((K + s - 1) / s + 31) / 32 * 32;
  if (k > PANEL_KMAX) {
    s = (K + PANEL_KMAX - 1) / PANEL_KMAX;
    k = ((K + s - 1) / s + 31) / 32 * 32;
  }
  if (k < 32) k = 32;
  *kps = k;
  *splits = static_cast<int32_t>(K > 0 ? (K + k - 1) / k : 1);
}

template <bool AC, bool BC, bool AM>
static void launch_slab(const GemmArgs &g, dim3 grid, hipStream_t s) {
  static bool attr = false;
  const size_t lds = 2 * static_cast<size_t>(BM) * PANEL_LD * sizeof(uint16_t);
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(gemm_slab_kernel<AC, BC, AM>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr = true;
  }
  gemm_slab_kernel<AC, BC, AM><<<grid, GEMM_THREADS, lds, s>>>(g);
}

}  // namespace mrec

using namespace mrec;

extern "C" {

size_t mrec_gemm_workspace_size(int64_t M, int64_t N, int64_t K, int32_t split_k) {
  int64_t kps;
  int32_t splits;
  plan_split(K, split_k, &kps, &splits);
  if (splits <= 1) return 0;
  return static_cast<size_t>(splits) * static_cast<size_t>(M) * static_cast<size_t>(N + 1) * 4;
}

mrec_status mrec_gemm(int64_t M, int64_t N, int64_t K, const mrec_operand *A,
                      const mrec_operand *B, const mrec_operand *a_mod, int32_t a_mod_kind,
                      int64_t b_ones_col, int64_t b_cols, const mrec_epilogue *epi, void *C,
                      mrec_dtype c_dtype, int64_t ldc, int32_t split_k, void *workspace,
                      size_t ws_bytes, mrec_stream stream) {
  MREC_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "negative size");
  MREC_CHECK_ARG(A && A->ptr && B && B->ptr && C, "NULL operand");
  MREC_CHECK_ARG(A->dtype == MREC_BF16 && B->dtype == MREC_BF16,
                 "A and B must be bf16 (prepare fp32 weights with mrec_weight_prep)");
  MREC_CHECK_ARG(c_dtype == MREC_BF16 || c_dtype == MREC_F32, "C must be bf16 or f32");
  MREC_CHECK_ARG(a_mod_kind >= 0 && a_mod_kind <= 2, "bad a_mod_kind");
  MREC_CHECK_ARG(a_mod_kind == 0 || (a_mod && a_mod->ptr && a_mod->dtype == MREC_BF16 &&
                                     a_mod->layout == A->layout),
                 "a_mod must be bf16 with A's layout");
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
  if (M == 0 || ncols == 0) return MREC_OK;
  GemmArgs g = {};
  g.M = M;
  g.N = N;
  g.K = K;
  g.A = A->ptr;
  g.lda = A->ld;
  g.a_col = A->layout == MREC_LAYOUT_COL;
  g.amod = a_mod_kind ? a_mod->ptr : nullptr;
  g.ld_amod = a_mod_kind ? a_mod->ld : 0;
  g.amod_kind = a_mod_kind;
  g.B = B->ptr;
  g.ldb = B->ld;
  g.b_col = B->layout == MREC_LAYOUT_COL;
  g.b_ones_col = b_ones_col;
  g.b_cols = b_cols;
  if (epi) {
    g.bias = epi->bias;
    g.act = epi->act;
    g.mul = epi->mul;
    g.ld_mul = epi->ld_mul;
    g.add = epi->add;
    g.ld_add = epi->ld_add;
    g.aux = epi->aux;
    g.ld_aux = epi->ld_aux;
    g.ones_out = epi->ones_out;
  }
  g.C = C;
  g.ldc = ldc;
  g.c_f32 = c_dtype == MREC_F32;
  g.a_vec = aligned16(g.A, g.lda, 2);
  g.amod_vec = g.amod ? aligned16(g.amod, g.ld_amod, 2) : 1;
  g.b_vec = aligned16(g.B, g.ldb, 2);
  MREC_CHECK_ARG(g.a_vec && g.b_vec && g.amod_vec,
                 "A/B/a_mod rows must be 16-byte aligned (pointer % 16 == 0, ld % 8 == 0)");
  g.ws = static_cast<float *>(workspace);
  g.split_k = splits;
  g.k_per_split = kps;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>((ncols + BN - 1) / BN),
                  static_cast<unsigned>((M + BM - 1) / BM), static_cast<unsigned>(splits));
  const bool am = a_mod_kind != 0;
  if (!g.a_col && !g.b_col) {
    am ? launch_slab<false, false, true>(g, grid, s) : launch_slab<false, false, false>(g, grid, s);
  } else if (!g.a_col && g.b_col) {
    am ? launch_slab<false, true, true>(g, grid, s) : launch_slab<false, true, false>(g, grid, s);
  } else if (g.a_col && !g.b_col) {
    am ? launch_slab<true, false, true>(g, grid, s) : launch_slab<true, false, false>(g, grid, s);
  } else {
    am ? launch_slab<true, true, true>(g, grid, s) : launch_slab<true, true, false>(g, grid, s);
  }
  mrec_status st = launch_status("mrec_gemm");
  if (st != MREC_OK || splits == 1) return st;
  const int64_t total = M * ncols;
  const unsigned rb = static_cast<unsigned>(std::min<int64_t>((total + 255) / 256, 2048));
  splitk_reduce_kernel<<<rb, 256, 0, s>>>(g);
  return launch_status("mrec_gemm(split-k reduce)");
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
