// MFMA bf16 GEMM for the dense towers (MLP, DCN-v2 cross, DIN attention unit).
//
//   C[m, n] = epi( sum_k A'(m, k) * B(k, n) )
//
// A'(m, k) = A(m, k) [* (Amod(m, k) > 0) | * Amod(m, k)]   (ReLU' mask / dz = g*x0)
// Operands are ROW (k contiguous) or COL (m / n contiguous); B may be fp32 (the
// fp32 master weights, converted to bf16 while staging) or bf16.  Tiles are staged
// global -> registers -> LDS as [row][k] images (transposed on the way in for COL
// operands) and consumed by v_mfma_f32_16x16x32_bf16 with fp32 accumulation.
//
// Block 64x64, BK 32, 4 waves in 2x2, each wave 32x32 = 2x2 MFMA tiles; LDS rows
// padded to 80 B so the 16 rows a ds_read_b128 lane group touches hit distinct
// banks.  Double-buffered: tile t+1 is loaded into registers before the MFMAs of
// tile t and written to the other LDS buffer after them (one barrier per tile).
//
// Epilogue (split_k == 1): v = acc + bias[n]; aux = v; v = relu(v); v = mul * v;
// v = v + add; C = v (bf16 or fp32).  split_k > 1 writes fp32 partial slabs that a
// second kernel reduces in fixed order and then runs the same epilogue
// (deterministic).  b_ones_col = K' makes B(k, K') = 1 so column K' of C is the
// row-sum of A' over k: the bias gradient rides along the weight-gradient GEMM.
#include <algorithm>

#include "common.h"

namespace mrec {

constexpr int BM = 64, BN = 64, BK = 32, LDSK = BK + 8;  // LDS row = 80 B
constexpr int GEMM_THREADS = 256;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct GemmArgs {
  int64_t M, N, K;
  const void *A;
  int64_t lda;
  int a_col;  // 1: A(m,k) at A[k*lda + m]
  const void *amod;
  int64_t ld_amod;
  int amod_kind;  // 0 none, 1 relu mask, 2 multiply
  const void *B;
  int64_t ldb;
  int b_col;  // 1: B(k,n) at B[k*ldb + n]; 0: at B[n*ldb + k]
  int b_f32;
  int64_t b_ones_col;
  int64_t b_cols;  // B(k, n) = 0 for n >= b_cols
  // epilogue
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
  int a_vec, amod_vec, b_vec;  // 16-byte vector loads legal
  int split_k;
  int64_t k_per_split;
  float *ws;  // [split_k, M, N] partials
};

__device__ __forceinline__ float bf(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }

// 8 consecutive bf16 (as raw bits) along the contiguous dim, zero outside [0, lim)
__device__ __forceinline__ void load8_bf16(const uint16_t *p, int64_t c0, int64_t lim, bool vec,
                                           uint16_t *o) {
  if (vec && c0 + 8 <= lim) {
    const uint4 r = *reinterpret_cast<const uint4 *>(p + c0);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = uint16_t(w[i] & 0xffffu);
      o[2 * i + 1] = uint16_t(w[i] >> 16);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (c0 + j < lim) ? p[c0 + j] : uint16_t(0);
  }
}

__device__ __forceinline__ void load8_f32(const float *p, int64_t c0, int64_t lim, bool vec,
                                          uint16_t *o) {
  float v[8];
  if (vec && c0 + 8 <= lim) {
    const float4 a = *reinterpret_cast<const float4 *>(p + c0);
    const float4 b = *reinterpret_cast<const float4 *>(p + c0 + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (c0 + j < lim) ? p[c0 + j] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f32_to_bf16_rne(v[j]);
}

// One staging chunk = 8 elements; the per-thread state between load and LDS write.
struct Chunk {
  uint16_t v[8];
};

// A tile chunk: ROW -> row m = r, k = k0 + c*8..; COL -> k row, 8 m values
__device__ __forceinline__ void load_a_chunk(const GemmArgs &g, int64_t m0, int64_t k0, int64_t kend,
                                             Chunk &c) {
  const int tid = threadIdx.x;
  const uint16_t *A = static_cast<const uint16_t *>(g.A);
  const uint16_t *Mo = static_cast<const uint16_t *>(g.amod);
  if (!g.a_col) {
    const int r = tid >> 2, cc = (tid & 3) * 8;
    const int64_t m = m0 + r;
    if (m < g.M) {
      load8_bf16(A + m * g.lda, k0 + cc, kend, g.a_vec, c.v);
      if (g.amod_kind) {
        uint16_t mv[8];
        load8_bf16(Mo + m * g.ld_amod, k0 + cc, kend, g.amod_vec, mv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (g.amod_kind == 1)
            c.v[j] = (mv[j] != 0 && !(mv[j] & 0x8000u)) ? c.v[j] : uint16_t(0);
          else
            c.v[j] = f32_to_bf16_rne(bf(c.v[j]) * bf(mv[j]));
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) c.v[j] = 0;
    }
  } else {
    const int kr = tid >> 3, mc = (tid & 7) * 8;
    const int64_t k = k0 + kr;
    if (k < kend) {
      load8_bf16(A + k * g.lda, m0 + mc, g.M, g.a_vec, c.v);
      if (g.amod_kind) {
        uint16_t mv[8];
        load8_bf16(Mo + k * g.ld_amod, m0 + mc, g.M, g.amod_vec, mv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (g.amod_kind == 1)
            c.v[j] = (mv[j] != 0 && !(mv[j] & 0x8000u)) ? c.v[j] : uint16_t(0);
          else
            c.v[j] = f32_to_bf16_rne(bf(c.v[j]) * bf(mv[j]));
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) c.v[j] = 0;
    }
  }
}

__device__ __forceinline__ void load_b_chunk(const GemmArgs &g, int64_t n0, int64_t k0, int64_t kend,
                                             Chunk &c) {
  const int tid = threadIdx.x;
  if (!g.b_col) {  // B(k, n) at B[n*ldb + k]: rows are n
    const int r = tid >> 2, cc = (tid & 3) * 8;
    const int64_t n = n0 + r;
    if (n == g.b_ones_col) {
#pragma unroll
      for (int j = 0; j < 8; ++j) c.v[j] = (k0 + cc + j < kend) ? uint16_t(0x3f80) : uint16_t(0);
    } else if (n < g.b_cols) {
      if (g.b_f32)
        load8_f32(static_cast<const float *>(g.B) + n * g.ldb, k0 + cc, kend, g.b_vec, c.v);
      else
        load8_bf16(static_cast<const uint16_t *>(g.B) + n * g.ldb, k0 + cc, kend, g.b_vec, c.v);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) c.v[j] = 0;
    }
  } else {  // B(k, n) at B[k*ldb + n]: rows are k, 8 n values
    const int kr = tid >> 3, nc = (tid & 7) * 8;
    const int64_t k = k0 + kr;
    if (k < kend) {
      const int64_t nlim = g.b_cols;
      if (g.b_f32)
        load8_f32(static_cast<const float *>(g.B) + k * g.ldb, n0 + nc, nlim, g.b_vec, c.v);
      else
        load8_bf16(static_cast<const uint16_t *>(g.B) + k * g.ldb, n0 + nc, nlim, g.b_vec, c.v);
      if (g.b_ones_col >= 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (n0 + nc + j == g.b_ones_col) c.v[j] = uint16_t(0x3f80);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) c.v[j] = 0;
    }
  }
}

// write a chunk into the [row][k] LDS image
__device__ __forceinline__ void store_chunk(uint16_t (*S)[LDSK], bool col_layout, const Chunk &c) {
  const int tid = threadIdx.x;
  if (!col_layout) {
    const int r = tid >> 2, cc = (tid & 3) * 8;
    uint4 w;
    w.x = uint32_t(c.v[0]) | (uint32_t(c.v[1]) << 16);
    w.y = uint32_t(c.v[2]) | (uint32_t(c.v[3]) << 16);
    w.z = uint32_t(c.v[4]) | (uint32_t(c.v[5]) << 16);
    w.w = uint32_t(c.v[6]) | (uint32_t(c.v[7]) << 16);
    *reinterpret_cast<uint4 *>(&S[r][cc]) = w;
  } else {
    const int kr = tid >> 3, mc = (tid & 7) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) S[mc + j][kr] = c.v[j];
  }
}

__device__ __forceinline__ float load_elem(const void *p, int64_t idx, bool f32) {
  return f32 ? static_cast<const float *>(p)[idx] : bf(static_cast<const uint16_t *>(p)[idx]);
}

// epilogue on one element (m, n) with fp32 pre-activation acc
__device__ __forceinline__ void epilogue_elem(const GemmArgs &g, int64_t m, int64_t n, float acc) {
  float v = acc + ((g.bias && n < g.N) ? g.bias[n] : 0.f);
  if (g.aux) static_cast<uint16_t *>(g.aux)[m * g.ld_aux + n] = f32_to_bf16_rne(v);
  if (g.act == 1) v = fmaxf(v, 0.f);
  if (g.mul) v *= bf(static_cast<const uint16_t *>(g.mul)[m * g.ld_mul + n]);
  if (g.add) v += bf(static_cast<const uint16_t *>(g.add)[m * g.ld_add + n]);
  if (g.c_f32)
    static_cast<float *>(g.C)[m * g.ldc + n] = v;
  else
    static_cast<uint16_t *>(g.C)[m * g.ldc + n] = f32_to_bf16_rne(v);
}

__global__ __launch_bounds__(GEMM_THREADS) void gemm_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) uint16_t As[2][BM][LDSK];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][BN][LDSK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = static_cast<int64_t>(blockIdx.y) * BM;
  const int64_t n0 = static_cast<int64_t>(blockIdx.x) * BN;
  const int64_t kb = static_cast<int64_t>(blockIdx.z) * g.k_per_split;
  const int64_t ke = min(g.K, kb + g.k_per_split);
  const int ntiles = ke > kb ? static_cast<int>((ke - kb + BK - 1) / BK) : 0;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Chunk ca, cb;
  if (ntiles > 0) {
    load_a_chunk(g, m0, kb, ke, ca);
    load_b_chunk(g, n0, kb, ke, cb);
    store_chunk(As[0], g.a_col, ca);
    store_chunk(Bs[0], g.b_col, cb);
  }
  __syncthreads();
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < ntiles;
    if (more) {
      const int64_t k0 = kb + static_cast<int64_t>(t + 1) * BK;
      load_a_chunk(g, m0, k0, ke, ca);
      load_b_chunk(g, n0, k0, ke, cb);
    }
    bf16x8 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      a[i] = *reinterpret_cast<const bf16x8 *>(&As[cur][wm * 32 + i * 16 + fr][fk]);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      b[j] = *reinterpret_cast<const bf16x8 *>(&Bs[cur][wn * 32 + j * 16 + fr][fk]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    if (more) {
      store_chunk(As[cur ^ 1], g.a_col, ca);
      store_chunk(Bs[cur ^ 1], g.b_col, cb);
    }
    __syncthreads();
  }

  // C/D layout of 16x16: col = lane & 15, row = (lane >> 4) * 4 + r
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

static bool aligned16(const void *p, int64_t ld, int es) {
  return p && (reinterpret_cast<uintptr_t>(p) & 15) == 0 && (ld * es) % 16 == 0;
}

}  // namespace mrec

using namespace mrec;

extern "C" {

size_t mrec_gemm_workspace_size(int64_t M, int64_t N, int32_t split_k) {
  if (split_k <= 1) return 0;
  return static_cast<size_t>(split_k) * static_cast<size_t>(M) * static_cast<size_t>(N + 1) * 4;
}

mrec_status mrec_gemm(int64_t M, int64_t N, int64_t K, const mrec_operand *A,
                      const mrec_operand *B, const mrec_operand *a_mod, int32_t a_mod_kind,
                      int64_t b_ones_col, int64_t b_cols, const mrec_epilogue *epi, void *C,
                      mrec_dtype c_dtype, int64_t ldc, int32_t split_k, void *workspace,
                      size_t ws_bytes, mrec_stream stream) {
  MREC_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "negative size");
  MREC_CHECK_ARG(A && A->ptr && B && B->ptr && C, "NULL operand");
  MREC_CHECK_ARG(A->dtype == MREC_BF16, "A must be bf16");
  MREC_CHECK_ARG(B->dtype == MREC_BF16 || B->dtype == MREC_F32, "B must be bf16 or f32");
  MREC_CHECK_ARG(c_dtype == MREC_BF16 || c_dtype == MREC_F32, "C must be bf16 or f32");
  MREC_CHECK_ARG(a_mod_kind >= 0 && a_mod_kind <= 2, "bad a_mod_kind");
  MREC_CHECK_ARG(a_mod_kind == 0 || (a_mod && a_mod->ptr && a_mod->dtype == MREC_BF16 &&
                                     a_mod->layout == A->layout),
                 "a_mod must be bf16 with A's layout");
  MREC_CHECK_ARG(b_ones_col < 0 || b_ones_col == N, "b_ones_col must be -1 or N");
  MREC_CHECK_ARG(b_cols >= 0 && b_cols <= N, "b_cols must be in [0, N]");
  MREC_CHECK_ARG(split_k >= 1 && split_k <= 64, "split_k out of [1, 64]");
  const int64_t ncols = b_ones_col >= 0 ? N + 1 : N;
  MREC_CHECK_ARG(ldc >= ncols, "ldc too small");
  if (split_k > 1 && ws_bytes < mrec_gemm_workspace_size(M, N, split_k)) {
    set_error("mrec_gemm: workspace too small");
    return MREC_ENOSPC;
  }
  MREC_CHECK_ARG(split_k == 1 || workspace, "split_k needs a workspace");
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
  g.b_f32 = B->dtype == MREC_F32;
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
  }
  g.C = C;
  g.ldc = ldc;
  g.c_f32 = c_dtype == MREC_F32;
  g.a_vec = aligned16(g.A, g.lda, 2);
  g.amod_vec = g.amod ? aligned16(g.amod, g.ld_amod, 2) : 0;
  g.b_vec = aligned16(g.B, g.ldb, g.b_f32 ? 4 : 2);
  g.split_k = split_k;
  const int64_t kps = ((K + split_k - 1) / split_k + BK - 1) / BK * BK;
  g.k_per_split = kps > 0 ? kps : BK;
  g.ws = static_cast<float *>(workspace);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>((ncols + BN - 1) / BN), static_cast<unsigned>((M + BM - 1) / BM),
                  static_cast<unsigned>(split_k));
  gemm_kernel<<<grid, GEMM_THREADS, 0, s>>>(g);
  mrec_status st = launch_status("mrec_gemm");
  if (st != MREC_OK || split_k == 1) return st;
  const int64_t total = M * ncols;
  const unsigned rb = static_cast<unsigned>(std::min<int64_t>((total + 255) / 256, 2048));
  splitk_reduce_kernel<<<rb, 256, 0, s>>>(g);
  return launch_status("mrec_gemm(split-k reduce)");
}

}  // extern "C"
