// DIN attention unit fused per sample (config C4).
//
// One workgroup (8 waves) per sample b at a time, persistent over samples.  The
// attention-unit input X = [q | k_j | q - k_j | q * k_j] (64 padded history rows x
// 4E), the MLP activations and every gradient live in LDS only; the MLP weights
// are staged once per workgroup as bf16 in both operand orders.  What the layered
// path (mrec_din_feat_fwd + three mrec_gemm layers + mrec_din_pool_*) moved
// through HBM per step at C4 -- the [B L, 128] input, the [B L, 80] / [B L, 40]
// activations and their gradients, ~0.4 GB -- never leaves the CU.
//
//   forward   s_j = w3 . relu(W2 relu(W1 x_j + b1) + b2) + b3
//             a   = softmax_j over valid j (his[b, j] > 0 or j == 0), invalid -> 0
//             top[b] = [q | sum_j a_j k_j | 0-pad]          (same math as din.hip)
//   backward  (given dtop and the saved a) ds_j = a_j (du.k_j - sum_i a_i du.k_i),
//             the MLP recomputed and back-propagated with bf16 MFMA operands
//             (fp32 accumulation, as the layered GEMMs), dX in fp32 straight into
//             dk_j = a_j du + df_k - df_(q-k) + df_(q*k) q and
//             dq   = dtop_q + sum_j (df_q + df_(q-k) + df_(q*k) k_j), written as
//             ONE bf16 gradient of the gathered rows; weight gradients accumulated
//             in MFMA registers across the workgroup's samples, one partial per
//             workgroup, summed in fixed order by din_att_wgrad_kernel.
//
// All GEMMs are v_mfma_f32_16x16x32_bf16 with both operands read as 16-B LDS
// vectors: lane l holds A[m = l % 16][k = 8 (l / 16) .. + 8] and the B^T row
// B[k .. + 8][n = l % 16]; so every operand buffer is stored "row = output index,
// contiguous along k" and the reductions over history rows read transposed copies
// ([feature][row]) written beside the row-major ones.
#include <cstdlib>

#include "common.h"

namespace mrec {

typedef short da_bf16x8 __attribute__((ext_vector_type(8)));
typedef float da_f32x4 __attribute__((ext_vector_type(4)));

constexpr int DA_ROWS = 64;              // history positions per sample, padded
constexpr int DA_CG = 2;                 // column groups: 8 waves = 4 row tiles x 2
constexpr int DA_THREADS = 64 * 4 * DA_CG;
constexpr int DA_LDT = DA_ROWS + 8;      // row stride of the [feature][row] buffers

struct DinAttArgs {
  const uint16_t *rows;  // gathered rows [q (batch) | k (batch L)] bf16
  int64_t ld_rows;
  const int32_t *his;
  int64_t ld_his;
  const float *w1, *b1, *w2, *b2, *w3, *b3;  // fp32 masters, nn.Linear layout
  int64_t ldw1, ldw2;
  int64_t batch;
  int L, H1, H2;
  float *a;  // [batch, L] softmax weights (written by fwd, read by bwd)
  uint16_t *top;
  int64_t ldt;
  const uint16_t *dtop;
  int64_t lddt;
  uint16_t *drows;
  int64_t ld_drows;
  float *part;  // [gridDim.x][P] weight-gradient partials
  int64_t P;
  unsigned long long *stamps;  // diagnostics: workgroup 0's phase clocks (NULL: off)
};

// diagnostics: s_memtime stamps of workgroup 0 (thread 0) at the backward's phase
// boundaries, samples 0..5: [0] start, [1] weights staged, then 8 per sample
#define DA_STAMP(k)                                                   \
  do {                                                                \
    if (p.stamps && blockIdx.x == 0 && tid == 0 && (k) < 64)          \
      p.stamps[(k)] = __builtin_amdgcn_s_memtime();                   \
  } while (0)

__device__ __forceinline__ da_bf16x8 da_frag(const uint16_t *base, int ld, int r0, int k0,
                                             int lane) {
  return *reinterpret_cast<const da_bf16x8 *>(base + (r0 + (lane & 15)) * ld + k0 +
                                              8 * (lane >> 4));
}

__device__ __forceinline__ da_f32x4 da_mfma(da_bf16x8 a, da_bf16x8 b, da_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// sum over the 16 lanes of a row group (lanes 16 g .. 16 g + 15)
// (DPP row rotations, no LDS crossbar; lanes may differ in the last bit, callers
// use one lane's value)
__device__ __forceinline__ float da_sum16(float v) {
  v += dpp_f32<0x128>(v);  // row_ror:8
  v += dpp_f32<0x124>(v);  // row_ror:4
  v += dpp_f32<0x122>(v);  // row_ror:2
  return v + dpp_f32<0x121>(v);  // row_ror:1
}

template <int E, int H1T, int H1K, int H2T, int H2K>
struct DaShape {
  static constexpr int E4 = 4 * E;
  static constexpr int KT1 = E4 / 32;  // k steps of layer 1
  static constexpr int NTX = E4 / 16;  // column tiles of X
  static constexpr int LDX = E4 + 8;
  static constexpr int H1N = 16 * H1T;  // layer-1 outputs, tile padded
  static constexpr int H1P = 32 * H1K;  // ... k-step padded
  static constexpr int LDH = H1P + 8;
  static constexpr int H2N = 16 * H2T;
  static constexpr int H2P = 32 * H2K;
  static constexpr int LDW2T = H2P + 8;
  static_assert(E % 16 == 0 && E4 % 32 == 0, "E must be a multiple of 16");
  static_assert(H1N <= H1P && H2N <= H2P, "k-step padding covers the tiles");
  static_assert(H2P <= H1P, "dZ2 aliases H1 with H1's row stride");
  static_assert(H1P <= E4, "dZ1 aliases X");
  // bf16 element offsets of the LDS buffers (16-B aligned: every size % 8 == 0)
  static constexpr int oX = 0;                       // X [64][LDX]   (bwd: dZ1 [64][LDH])
  static constexpr int oH1 = oX + DA_ROWS * LDX;     // H1 [64][LDH]  (bwd: dZ2 [64][LDH])
  static constexpr int oW1 = oH1 + DA_ROWS * LDH;    // W1 [H1N][LDX]
  static constexpr int oW2 = oW1 + H1N * LDX;        // W2 [H2N][LDH]
  static constexpr int fwd_end = oW2 + H2N * LDH;
  static constexpr int oXT = fwd_end;                // X^T [E4][LDT]
  static constexpr int oH1T = oXT + E4 * DA_LDT;     // H1^T [H1N][LDT]
  static constexpr int oZ1T = oH1T + H1N * DA_LDT;   // dZ1^T [H1N][LDT]
  static constexpr int oZ2T = oZ1T + H1N * DA_LDT;   // dZ2^T [H2N][LDT]
  static constexpr int oW1T = oZ2T + H2N * DA_LDT;   // W1^T [E4][LDH]
  static constexpr int oW2T = oW1T + E4 * LDH;       // W2^T [H1N][LDW2T]
  static constexpr int bwd_end = oW2T + H1N * LDW2T;
  // fp32 tail: b1 [H1N], b2 [H2N], w3 [H2N], q [E], du [E], g [64], dq parts [4][E]
  static constexpr int nf32 = H1N + 2 * H2N + 2 * E + DA_ROWS + 4 * E;
  static constexpr size_t fwd_bytes =
      fwd_end * 2 + (H1N + 2 * H2N + (DA_CG + 1) * DA_ROWS + DA_THREADS) * 4;
  static constexpr size_t bwd_bytes = bwd_end * 2 + nf32 * 4;
};

__device__ __forceinline__ void da_zero_lds(char *lds, size_t bytes) {
  for (size_t o = threadIdx.x * 16; o < bytes; o += DA_THREADS * 16)
    *reinterpret_cast<uint4 *>(lds + o) = make_uint4(0, 0, 0, 0);
}

// Weights once per workgroup: every float4 load of a thread is issued before any
// is converted (a load -> store loop of ~55 dependent L2 round trips per thread
// cost ~40 us per launch).  Needs ldw1, ldw2, H1 multiples of 4, 16-B aligned w1 / w2.
template <class S, bool BWD>
__device__ void da_stage_weights(const DinAttArgs &p, uint16_t *sm, float *sb1, float *sb2,
                                 float *sw3) {
  const int tid = threadIdx.x;
  constexpr int Q1 = S::H1N * S::E4 / 4, N1 = (Q1 + DA_THREADS - 1) / DA_THREADS;
  constexpr int Q2 = S::H2N * S::H1N / 4, N2 = (Q2 + DA_THREADS - 1) / DA_THREADS;
  float4 v1[N1], v2[N2];
  // unconditional loads (padding reads element 0, zeroed at the conversion): a
  // conditional load's value is copied out of its branch and that copy waits for it
  bool ok1[N1], ok2[N2];
#pragma unroll
  for (int it = 0; it < N1; ++it) {
    const int i = (tid + it * DA_THREADS) * 4, n = i / S::E4, k = i - n * S::E4;
    ok1[it] = i < S::H1N * S::E4 && n < p.H1;
    v1[it] = *reinterpret_cast<const float4 *>(p.w1 + (ok1[it] ? n * p.ldw1 + k : 0));
  }
#pragma unroll
  for (int it = 0; it < N2; ++it) {
    const int i = (tid + it * DA_THREADS) * 4, n = i / S::H1N, k = i - n * S::H1N;
    ok2[it] = i < S::H2N * S::H1N && n < p.H2 && k < p.H1;
    v2[it] = *reinterpret_cast<const float4 *>(p.w2 + (ok2[it] ? n * p.ldw2 + k : 0));
  }
  DA_STAMP(61);
  for (int i = tid; i < S::H1N; i += DA_THREADS) sb1[i] = i < p.H1 ? p.b1[i] : 0.f;
  for (int i = tid; i < S::H2N; i += DA_THREADS) {
    sb2[i] = i < p.H2 ? p.b2[i] : 0.f;
    sw3[i] = i < p.H2 ? p.w3[i] : 0.f;
  }
#pragma unroll
  for (int it = 0; it < N1; ++it) {
    const int i = (tid + it * DA_THREADS) * 4, n = i / S::E4, k = i - n * S::E4;
    if (i >= S::H1N * S::E4) continue;
    if (!ok1[it]) v1[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    const uint16_t h[4] = {f32_to_bf16_rne(v1[it].x), f32_to_bf16_rne(v1[it].y),
                           f32_to_bf16_rne(v1[it].z), f32_to_bf16_rne(v1[it].w)};
    *reinterpret_cast<uint2 *>(sm + S::oW1 + n * S::LDX + k) =
        make_uint2(h[0] | (static_cast<uint32_t>(h[1]) << 16),
                   h[2] | (static_cast<uint32_t>(h[3]) << 16));
    if constexpr (BWD) {
#pragma unroll
      for (int c = 0; c < 4; ++c) sm[S::oW1T + (k + c) * S::LDH + n] = h[c];
    }
  }
  DA_STAMP(62);
#pragma unroll
  for (int it = 0; it < N2; ++it) {
    const int i = (tid + it * DA_THREADS) * 4, n = i / S::H1N, k = i - n * S::H1N;
    if (i >= S::H2N * S::H1N) continue;
    if (!ok2[it]) v2[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    const uint16_t h[4] = {f32_to_bf16_rne(v2[it].x), f32_to_bf16_rne(v2[it].y),
                           f32_to_bf16_rne(v2[it].z), f32_to_bf16_rne(v2[it].w)};
    *reinterpret_cast<uint2 *>(sm + S::oW2 + n * S::LDH + k) =
        make_uint2(h[0] | (static_cast<uint32_t>(h[1]) << 16),
                   h[2] | (static_cast<uint32_t>(h[3]) << 16));
    if constexpr (BWD) {
#pragma unroll
      for (int c = 0; c < 4; ++c) sm[S::oW2T + (k + c) * S::LDW2T + n] = h[c];
    }
  }
}

// row chunk task of the X builders: thread t -> history row j, 8 columns at c
template <int E>
struct DaTask {
  static constexpr int CH = E / 8;  // 16-B chunks per q / k row
  int j, c;
  bool on;
  __device__ DaTask(int t) : j(t / CH), c((t % CH) * 8), on(t < DA_ROWS * CH) {}
};

// global inputs of one sample for thread t, loaded one sample ahead (their
// latency overlaps the previous sample's LDS / MFMA phases)
struct DaRaw {
  uint4 q, k, du;  // q / k chunk (bf16 x 8), du chunk (bwd)
  float a;         // bwd: a[b, lane]
  int valid;       // fwd: history position `lane` valid
};

template <int E, bool BWD>
__device__ __forceinline__ DaRaw da_load(const DinAttArgs &p, int64_t b, const DaTask<E> &t,
                                         int lane) {
  DaRaw r;
  r.q = r.k = r.du = make_uint4(0, 0, 0, 0);
  r.a = 0.f;
  r.valid = 0;
  if (t.on) {
    r.q = *reinterpret_cast<const uint4 *>(p.rows + b * p.ld_rows + t.c);
    if (t.j < p.L)
      r.k = *reinterpret_cast<const uint4 *>(p.rows + (p.batch + b * p.L + t.j) * p.ld_rows + t.c);
    if constexpr (BWD)
      r.du = *reinterpret_cast<const uint4 *>(p.dtop + b * p.lddt + E + t.c);
  }
  if constexpr (BWD) {
    if (lane < p.L) r.a = p.a[b * p.L + lane];
  } else {
    r.valid = lane < p.L && (lane == 0 || p.his[b * p.ld_his + lane] > 0);
  }
  return r;
}

// X row j of sample b: [q | k | q - k | q * k] as bf16 (the rounding of
// din_feat_fwd_kernel); rows j >= L are zero.  Returns k (fp32) and q (fp32).
template <class S, int E, bool TR>
__device__ __forceinline__ void da_build_x(const DinAttArgs &p, const DaRaw &raw,
                                           const DaTask<E> &t, uint16_t *sm, float (&qv)[8],
                                           float (&kv)[8]) {
  const uint4 qraw = raw.q, kraw = raw.k;
  const bool real = t.j < p.L;
  Vec<uint16_t>::to_f32(qraw, qv);
  Vec<uint16_t>::to_f32(kraw, kv);
  float d[8], m[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    d[i] = qv[i] - kv[i];
    m[i] = qv[i] * kv[i];
  }
  uint4 dq = make_uint4(pack_bf16x2(d[0], d[1]), pack_bf16x2(d[2], d[3]), pack_bf16x2(d[4], d[5]),
                        pack_bf16x2(d[6], d[7]));
  uint4 mq = make_uint4(pack_bf16x2(m[0], m[1]), pack_bf16x2(m[2], m[3]), pack_bf16x2(m[4], m[5]),
                        pack_bf16x2(m[6], m[7]));
  uint4 qq = qraw;
  if (!real) qq = dq = mq = make_uint4(0, 0, 0, 0);
  uint16_t *x = sm + S::oX + t.j * S::LDX + t.c;
  *reinterpret_cast<uint4 *>(x) = qq;
  *reinterpret_cast<uint4 *>(x + E) = kraw;
  *reinterpret_cast<uint4 *>(x + 2 * E) = dq;
  *reinterpret_cast<uint4 *>(x + 3 * E) = mq;
  if constexpr (TR) {
    uint16_t *xt = sm + S::oXT + t.c * DA_LDT + t.j;
    const uint4 parts[4] = {qq, kraw, dq, mq};
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint32_t u[4] = {parts[g].x, parts[g].y, parts[g].z, parts[g].w};
#pragma unroll
      for (int i = 0; i < 8; ++i)
        xt[(g * E + i) * DA_LDT] = static_cast<uint16_t>(u[i >> 1] >> (16 * (i & 1)));
    }
  }
}

// Wave w = (row tile rt = w / 2: rows 16 rt .. + 15, column group cg = w % 2; the
// waves of one SIMD, w and w + 4, hold different row tiles):
// a GEMM's 16-column output tiles n = cg, cg + DA_CG, ... of the wave's rows.
// layer 1: acc[jn] = X[rows] W1^T (tile n = cg + DA_CG jn)
template <class S, int H1T>
__device__ __forceinline__ void da_layer1(const uint16_t *sm, int rt, int cg, int lane, bool on,
                                          da_f32x4 (&acc)[(H1T + DA_CG - 1) / DA_CG]) {
  constexpr int J = (H1T + DA_CG - 1) / DA_CG;
#pragma unroll
  for (int jn = 0; jn < J; ++jn) acc[jn] = da_f32x4{0.f, 0.f, 0.f, 0.f};
  if (!on) return;
#pragma unroll
  for (int s = 0; s < S::KT1; ++s) {
    const da_bf16x8 a = da_frag(sm + S::oX, S::LDX, 16 * rt, 32 * s, lane);
#pragma unroll
    for (int jn = 0; jn < J; ++jn) {
      const int n = cg + DA_CG * jn;
      if (n < H1T) acc[jn] = da_mfma(a, da_frag(sm + S::oW1, S::LDX, 16 * n, 32 * s, lane), acc[jn]);
    }
  }
}

// layer 2: acc[jn] = H1[rows] W2^T
template <class S, int H1K, int H2T>
__device__ __forceinline__ void da_layer2(const uint16_t *sm, int rt, int cg, int lane, bool on,
                                          da_f32x4 (&acc)[(H2T + DA_CG - 1) / DA_CG]) {
  constexpr int J = (H2T + DA_CG - 1) / DA_CG;
#pragma unroll
  for (int jn = 0; jn < J; ++jn) acc[jn] = da_f32x4{0.f, 0.f, 0.f, 0.f};
  if (!on) return;
#pragma unroll
  for (int s = 0; s < H1K; ++s) {
    const da_bf16x8 a = da_frag(sm + S::oH1, S::LDH, 16 * rt, 32 * s, lane);
#pragma unroll
    for (int jn = 0; jn < J; ++jn) {
      const int n = cg + DA_CG * jn;
      if (n < H2T) acc[jn] = da_mfma(a, da_frag(sm + S::oW2, S::LDH, 16 * n, 32 * s, lane), acc[jn]);
    }
  }
}

// ---------------------------------------------------------------------------
// forward: scores, masked softmax, pooling -> top, a
// ---------------------------------------------------------------------------
template <int E, int H1T, int H1K, int H2T, int H2K>
__global__ __launch_bounds__(DA_THREADS) void din_att_fwd_kernel(DinAttArgs p) {
  using S = DaShape<E, H1T, H1K, H2T, H2K>;
  constexpr int J1 = (H1T + DA_CG - 1) / DA_CG, J2 = (H2T + DA_CG - 1) / DA_CG;
  extern __shared__ __attribute__((aligned(16))) char da_lds[];
  uint16_t *sm = reinterpret_cast<uint16_t *>(da_lds);
  float *sb1 = reinterpret_cast<float *>(da_lds + S::fwd_end * 2);
  float *sb2 = sb1 + S::H1N;
  float *sw3 = sb2 + S::H2N;
  float *ss = sw3 + S::H2N;        // score parts [DA_CG][64]
  float *sa = ss + DA_CG * DA_ROWS;  // softmax weights [64]
  float *su = sa + DA_ROWS;        // pooled-sum parts [DA_THREADS / E][E]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, rt = w >> 1, cg = w & 1;
  da_zero_lds(da_lds, S::fwd_end * 2);
  __syncthreads();
  da_stage_weights<S, false>(p, sm, sb1, sb2, sw3);
  const float b3 = p.b3[0];
  const DaTask<E> task(tid);
  DaRaw cur = {};
  if (blockIdx.x < p.batch) cur = da_load<E, false>(p, blockIdx.x, task, lane);
  for (int64_t b = blockIdx.x; b < p.batch; b += gridDim.x) {
    if (task.on) {
      float qv[8], kv[8];
      da_build_x<S, E, false>(p, cur, task, sm, qv, kv);
    }
    // rows past the last valid history position only feed masked scores: their
    // row tiles skip the MLP (wave-uniform: every wave holds all 64 validity bits)
    const uint64_t vm = __ballot(cur.valid);
    const bool act = 16 * rt < (vm ? 64 - __clzll(vm) : 0);
    // the next sample's inputs, issued once this sample's are consumed (issued before
    // the X build, the build's wait covered them too)
    DaRaw nxt = {};
    if (b + gridDim.x < p.batch) nxt = da_load<E, false>(p, b + gridDim.x, task, lane);
    __syncthreads();
    {
      da_f32x4 acc[J1];
      da_layer1<S, H1T>(sm, rt, cg, lane, act, acc);
#pragma unroll
      for (int jn = 0; jn < J1; ++jn) {
        const int n = cg + DA_CG * jn;
        if (n >= H1T) continue;
        const int col = 16 * n + (lane & 15);
        const float bias = sb1[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * rt + 4 * (lane >> 4) + i;
          sm[S::oH1 + r * S::LDH + col] = f32_to_bf16_rne(fmaxf(acc[jn][i] + bias, 0.f));
        }
      }
    }
    __syncthreads();
    {
      da_f32x4 acc[J2];
      da_layer2<S, H1K, H2T>(sm, rt, cg, lane, act, acc);
      float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int jn = 0; jn < J2; ++jn) {
        const int n = cg + DA_CG * jn;
        if (n >= H2T) continue;
        const int col = 16 * n + (lane & 15);
        const float bias = sb2[col], wv = sw3[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) part[i] = fmaf(fmaxf(acc[jn][i] + bias, 0.f), wv, part[i]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = da_sum16(part[i]);
        if ((lane & 15) == 0) ss[cg * DA_ROWS + 16 * rt + 4 * (lane >> 4) + i] = v;
      }
    }
    __syncthreads();
    // masked softmax over history positions (lane j), as din_pool_fwd_kernel, in
    // every wave (no extra barrier); wave 0 stores a
    {
      float sc = b3;
#pragma unroll
      for (int g = 0; g < DA_CG; ++g) sc += ss[g * DA_ROWS + lane];
      const float sj = cur.valid ? sc : -INFINITY;
      float m = sj;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
      const float e = cur.valid ? __expf(sj - m) : 0.f;
      const float a = e / sum_wave(e);
      if (w == 0) {
        sa[lane] = a;
        if (lane < p.L) p.a[b * p.L + lane] = a;
      }
    }
    __syncthreads();
    // u[e] = sum_j a_j k_j[e]: thread (part g, column e) sums positions j = g mod G,
    // the G parts are then added in part order (fixed order, deterministic)
    constexpr int G = DA_THREADS / E;
    {
      const int e = tid % E, g = tid / E;
      float u = 0.f;
      for (int j = g; j < p.L; j += G)
        u = fmaf(sa[j], bf16_to_f32(sm[S::oX + j * S::LDX + E + e]), u);
      su[g * E + e] = u;
    }
    __syncthreads();
    if (tid < E) {
      float u = 0.f;
#pragma unroll
      for (int g = 0; g < G; ++g) u += su[g * E + tid];
      uint16_t *tp = p.top + b * p.ldt;
      tp[tid] = sm[S::oX + tid];  // q (row 0's q block)
      tp[E + tid] = f32_to_bf16_rne(u);
    }
    for (int c = 2 * E + tid; c < p.ldt; c += DA_THREADS) p.top[b * p.ldt + c] = 0;
    cur = nxt;
    __syncthreads();  // the next sample's X build overwrites X, read by the pooled sum
  }
}

// ---------------------------------------------------------------------------
// forward, one wave per sample: no workgroup barrier after the weights are staged.
//
// The attention MLP is row-independent, so a wave can take a sample's 64 history
// rows as 4 row tiles of its own: layer 1's A operand is built in registers straight
// from the lane's 16-B q / k chunks (lane l holds X[row l % 16][k = 8 (l / 16) .. + 8]
// of each 32-wide k step, and with E >= 16 that is one block of [q | k | q - k | q k]
// at column offset 8 (l / 16) mod E), layer 1's B fragments live in VGPRs for the
// launch, and only H1 (one 16-row tile), the scores, a and the pooling parts pass
// through the wave's own LDS scratch.  Every sum runs in the order of
// din_att_fwd_kernel (k steps ascending, score parts of column group 0 then 1, the
// pooled sum's DA_THREADS / E parts in part order), so the two kernels agree
// bitwise (tests/test_gpu_din_att.py).  The one-workgroup-per-sample kernel spent
// ~4.6 us per sample on barriers and LDS round trips (37 us at C4); the MFMA work of
// a sample is 116 16x16x32 steps (~1.9k cycles).
// ---------------------------------------------------------------------------
template <int E, int H1T, int H1K, int H2T, int H2K>
struct DaShapeF : DaShape<E, H1T, H1K, H2T, H2K> {
  using B = DaShape<E, H1T, H1K, H2T, H2K>;
  static constexpr int WAVES = DA_THREADS / 64;
  static constexpr int G = DA_THREADS / E;  // pooling parts (din_att_fwd_kernel's order)
  // bf16 elements: the weights, shared by the workgroup's waves while they load
  // their fragments
  static constexpr int oW1 = 0;
  static constexpr int oW2 = B::H1N * B::LDX;
  static constexpr int w_end = oW2 + B::H2N * B::LDH;
  static constexpr size_t fp_off = static_cast<size_t>(w_end) * 2;  // b1, b2, w3 fp32
  static constexpr size_t scratch_off = (fp_off + (B::H1N + 2 * B::H2N) * 4 + 15) / 16 * 16;
  // per wave: H [16][LDH] bf16; score parts [2][64], a [64], pooling parts [G][E] fp32
  static constexpr int s_end = 16 * B::LDH;
  static constexpr size_t wave_bytes =
      static_cast<size_t>(s_end) * 2 + (3 * DA_ROWS + G * E) * 4;
  static constexpr size_t bytes = scratch_off + WAVES * wave_bytes;
  static_assert(E == 16 || E == 32, "a lane's k-step chunk is one block of X at offset 8 g mod E");
  static_assert((s_end * 2) % 16 == 0 && wave_bytes % 16 == 0, "16-B aligned scratch");
  static_assert(bytes <= 160 * 1024, "LDS budget");
};

// Loaded unconditionally from clamped addresses (sample min(b, batch - 1), row
// min(j, L - 1), position min(lane, L - 1)) and masked where used: a conditional
// load's value is copied out of its branch, and that copy waits for the load -- the
// prologue's first-sample loads then stalled the weight staging behind them.
struct DaRawW {
  uint4 q;     // q chunk (bf16 x 8) at column offset 8 (lane / 16) mod E
  uint4 k[4];  // k chunk of history row min(16 rt + lane % 16, L - 1)
  int hv;      // his[b, min(lane, L - 1)]
};

template <int E>
__device__ __forceinline__ DaRawW da_load_w(const DinAttArgs &p, int64_t b, int lane, int off) {
  DaRawW r;
  b = b < p.batch ? b : p.batch - 1;
  r.q = *reinterpret_cast<const uint4 *>(p.rows + b * p.ld_rows + off);
#pragma unroll
  for (int rt = 0; rt < 4; ++rt) {
    const int j = min(16 * rt + (lane & 15), p.L - 1);
    r.k[rt] = *reinterpret_cast<const uint4 *>(p.rows + (p.batch + b * p.L + j) * p.ld_rows + off);
  }
  r.hv = p.his[b * p.ld_his + min(lane, p.L - 1)];
  return r;
}

// compiler + wave-order fence for a wave-local LDS round trip (the LDS executes one
// wave's instructions in order; this keeps the compiler from moving them)
#define DA_WAVE_SYNC()                                  \
  do {                                                  \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
    __builtin_amdgcn_wave_barrier();                    \
  } while (0)

// KC: the clocked instantiation (mrec_kernel_clock, common.h), launched only while
// the clock is on; the production one carries no clock code
template <int E, int H1T, int H1K, int H2T, int H2K, bool KC = false>
__global__ __launch_bounds__(DA_THREADS, 1) void din_att_fwd_wave_kernel(DinAttArgs p, KClock kc) {
  KcScope<KC> kc_scope(kc);
  using S = DaShapeF<E, H1T, H1K, H2T, H2K>;
  constexpr int KT1 = S::KT1, G = S::G, LDH = S::LDH;
  constexpr int PPL = G / 16;  // pooling parts per lane: rows j = 16 rt + lane % 16 -> j mod G
  extern __shared__ __attribute__((aligned(16))) char da_lds[];
  uint16_t *sm = reinterpret_cast<uint16_t *>(da_lds);
  float *sb1 = reinterpret_cast<float *>(da_lds + S::fp_off);
  float *sb2 = sb1 + S::H1N;
  float *sw3 = sb2 + S::H2N;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, r16 = lane & 15;
  char *ws = da_lds + S::scratch_off + w * S::wave_bytes;
  uint16_t *sHt = reinterpret_cast<uint16_t *>(ws);
  float *sSC = reinterpret_cast<float *>(ws + S::s_end * 2);
  float *sA = sSC + 2 * DA_ROWS;
  float *sP = sA + DA_ROWS;
  DA_STAMP(0);
  const int off = (8 * g) % E;
  const int64_t nw = static_cast<int64_t>(gridDim.x) * S::WAVES;
  int64_t b = blockIdx.x + static_cast<int64_t>(gridDim.x) * w;
  DaRawW cur = da_load_w<E>(p, b, lane, off);  // loads while the weights are staged
  // zero what is read but never written: W2's and H's padded k columns
  da_zero_lds(da_lds, S::scratch_off);
  for (int o = lane * 16; o < S::s_end * 2; o += 64 * 16)
    *reinterpret_cast<uint4 *>(ws + o) = make_uint4(0, 0, 0, 0);
  __syncthreads();
  DA_STAMP(60);
  da_stage_weights<S, false>(p, sm, sb1, sb2, sw3);
  __syncthreads();
  DA_STAMP(1);
  // layer 1's B fragments in VGPRs (80 at C4); layer 2's are read from the staged
  // copy per use (in VGPRs too they spill at 256)
  da_bf16x8 w1f[H1T][KT1];
  float b1v[H1T][4], b2v[H2T], w3v[H2T];
#pragma unroll
  for (int n = 0; n < H1T; ++n) {
#pragma unroll
    for (int i = 0; i < 4; ++i) b1v[n][i] = sb1[16 * n + 4 * g + i];
#pragma unroll
    for (int s = 0; s < KT1; ++s) w1f[n][s] = da_frag(sm + S::oW1, S::LDX, 16 * n, 32 * s, lane);
  }
#pragma unroll
  for (int n = 0; n < H2T; ++n) {
    b2v[n] = sb2[16 * n + r16];
    w3v[n] = sw3[16 * n + r16];
  }
  const float b3 = p.b3[0];
  int sidx = 0;
  for (; b < p.batch; b += nw) {
    const DaRawW nxt = da_load_w<E>(p, b + nw, lane, off);
    DA_WAVE_SYNC();  // the previous sample's pooling reads are done
    DA_STAMP(2 + 8 * sidx);
    const bool valid = lane < p.L && (lane == 0 || cur.hv > 0);
    const uint64_t vm = __ballot(valid);
    const int nact = vm ? 64 - __clzll(vm) : 0;
    float qv[8];
    Vec<uint16_t>::to_f32(cur.q, qv);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      if (16 * rt >= nact) continue;  // rows past the last valid position: masked
      const bool real = 16 * rt + r16 < p.L;
      const uint4 kk = real ? cur.k[rt] : make_uint4(0, 0, 0, 0);
      uint4 qq = cur.q, dq, mq;
      {
        float kv[8], d[8], m[8];
        Vec<uint16_t>::to_f32(kk, kv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          d[i] = qv[i] - kv[i];
          m[i] = qv[i] * kv[i];
        }
        dq = make_uint4(pack_bf16x2(d[0], d[1]), pack_bf16x2(d[2], d[3]),
                        pack_bf16x2(d[4], d[5]), pack_bf16x2(d[6], d[7]));
        mq = make_uint4(pack_bf16x2(m[0], m[1]), pack_bf16x2(m[2], m[3]),
                        pack_bf16x2(m[4], m[5]), pack_bf16x2(m[6], m[7]));
      }
      if (!real) qq = dq = mq = make_uint4(0, 0, 0, 0);
      da_f32x4 acc[H1T];
#pragma unroll
      for (int n = 0; n < H1T; ++n) acc[n] = da_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KT1; ++s) {
        const int blk = (32 * s + 8 * g) / E;
        const uint4 xv = blk == 0 ? qq : blk == 1 ? kk : blk == 2 ? dq : mq;
        const da_bf16x8 a = __builtin_bit_cast(da_bf16x8, xv);
#pragma unroll
        for (int n = 0; n < H1T; ++n) acc[n] = da_mfma(w1f[n][s], a, acc[n]);
      }
      // (operands swapped: acc[n] is H1^T, lane l holds row l % 16's outputs
      // 16 n + 4 (l / 16) .. + 3 -- the same products and k order, one 8-B store each)
      DA_WAVE_SYNC();  // the previous tile's H reads are done
#pragma unroll
      for (int n = 0; n < H1T; ++n) {
        float h[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) h[i] = fmaxf(acc[n][i] + b1v[n][i], 0.f);
        *reinterpret_cast<uint2 *>(sHt + r16 * LDH + 16 * n + 4 * g) =
            make_uint2(pack_bf16x2(h[0], h[1]), pack_bf16x2(h[2], h[3]));
      }
      DA_WAVE_SYNC();
      da_f32x4 acc2[H2T];
#pragma unroll
      for (int n = 0; n < H2T; ++n) acc2[n] = da_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < H1K; ++s) {
        const da_bf16x8 a = da_frag(sHt, LDH, 0, 32 * s, lane);
#pragma unroll
        for (int n = 0; n < H2T; ++n)
          acc2[n] = da_mfma(a, da_frag(sm + S::oW2, LDH, 16 * n, 32 * s, lane), acc2[n]);
      }
      float part[DA_CG][4] = {};
#pragma unroll
      for (int n = 0; n < H2T; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          part[n % DA_CG][i] = fmaf(fmaxf(acc2[n][i] + b2v[n], 0.f), w3v[n], part[n % DA_CG][i]);
#pragma unroll
      for (int cg = 0; cg < DA_CG; ++cg)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = da_sum16(part[cg][i]);
          if (r16 == 0) sSC[cg * DA_ROWS + 16 * rt + 4 * g + i] = v;
        }
    }
    DA_WAVE_SYNC();
    DA_STAMP(3 + 8 * sidx);
    // masked softmax over history positions (lane j)
    {
      float sc = b3;
#pragma unroll
      for (int cg = 0; cg < DA_CG; ++cg) sc += sSC[cg * DA_ROWS + lane];
      const float sj = valid ? sc : -INFINITY;
      const float m = max_wave(sj);
      const float e = valid ? __expf(sj - m) : 0.f;
      const float a = e / sum_wave(e);
      sA[lane] = a;
      if (lane < p.L) p.a[b * p.L + lane] = a;
    }
    DA_WAVE_SYNC();
    DA_STAMP(4 + 8 * sidx);
    // pooling parts from the lane's own k chunks: part gp = sum over rows j = gp mod G
    // in ascending j (= ascending row tile), columns off .. off + 7
    {
      float pu[PPL][8] = {};
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) {
        const int j = 16 * rt + r16;
        if (j >= p.L) continue;
        const float aj = sA[j];
        float kv[8];
        Vec<uint16_t>::to_f32(cur.k[rt], kv);
#pragma unroll
        for (int i = 0; i < 8; ++i) pu[rt % PPL][i] = fmaf(aj, kv[i], pu[rt % PPL][i]);
      }
      if (8 * g < E) {  // (E = 16: lanes g and g + 2 hold the same chunk)
#pragma unroll
        for (int t = 0; t < PPL; ++t) {
          float4 *dst = reinterpret_cast<float4 *>(sP + (16 * t + r16) * E + off);
          dst[0] = make_float4(pu[t][0], pu[t][1], pu[t][2], pu[t][3]);
          dst[1] = make_float4(pu[t][4], pu[t][5], pu[t][6], pu[t][7]);
        }
      }
    }
    DA_WAVE_SYNC();
    DA_STAMP(5 + 8 * sidx);
    uint16_t *tp = p.top + b * p.ldt;
    if (lane < E) {
      float u = 0.f;
#pragma unroll 8
      for (int gp = 0; gp < G; ++gp) u += sP[gp * E + lane];
      tp[E + lane] = f32_to_bf16_rne(u);
    }
    if (r16 == 0 && 8 * g < E) {  // q (row 0's q block: zero iff L == 0)
      const uint32_t qw[4] = {cur.q.x, cur.q.y, cur.q.z, cur.q.w};
#pragma unroll
      for (int i = 0; i < 8; ++i)
        tp[8 * g + i] = p.L > 0 ? static_cast<uint16_t>(qw[i >> 1] >> (16 * (i & 1))) : 0;
    }
    for (int c = 2 * E + lane; c < p.ldt; c += 64) tp[c] = 0;
    DA_STAMP(6 + 8 * sidx);
    ++sidx;
    cur = nxt;
  }
}

// ---------------------------------------------------------------------------
// backward: pooling backward, MLP recomputed + back-propagated, dX -> d rows,
// weight-gradient partials per workgroup
// ---------------------------------------------------------------------------
template <int E, int H1T, int H1K, int H2T, int H2K>
__global__ __launch_bounds__(DA_THREADS) void din_att_bwd_kernel(DinAttArgs p) {
  using S = DaShape<E, H1T, H1K, H2T, H2K>;
  constexpr int NTX = S::NTX;
  constexpr int EC = E / 16;  // column tiles per block of X
  constexpr int J1 = (H1T + DA_CG - 1) / DA_CG, J2 = (H2T + DA_CG - 1) / DA_CG;
  constexpr int JX = (EC + DA_CG - 1) / DA_CG;
  constexpr int NWV = DA_THREADS / 64;
  constexpr int NW1 = (H1T * NTX + NWV - 1) / NWV;  // dW1 tiles per wave
  constexpr int NW2 = (H2T * H1T + NWV - 1) / NWV;  // dW2 tiles per wave
  extern __shared__ __attribute__((aligned(16))) char da_lds[];
  uint16_t *sm = reinterpret_cast<uint16_t *>(da_lds);
  float *sb1 = reinterpret_cast<float *>(da_lds + S::bwd_end * 2);
  float *sb2 = sb1 + S::H1N;
  float *sw3 = sb2 + S::H2N;
  float *sq = sw3 + S::H2N;  // q [E] fp32
  float *sdu = sq + E;       // du = dtop[b, E:2E] [E]
  float *sg = sdu + E;       // g_j = du . k_j [64]
  float *sdq = sg + DA_ROWS;  // per-row-tile dq parts [4][E]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, rt = w >> 1, cg = w & 1;
  DA_STAMP(0);
  da_zero_lds(da_lds, S::bwd_end * 2);
  __syncthreads();
  da_stage_weights<S, true>(p, sm, sb1, sb2, sw3);
  const DaTask<E> task(tid);
  int sidx = 0;
  DA_STAMP(1);

  da_f32x4 gw1[NW1], gw2[NW2];
#pragma unroll
  for (int i = 0; i < NW1; ++i) gw1[i] = da_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NW2; ++i) gw2[i] = da_f32x4{0.f, 0.f, 0.f, 0.f};
  float gb1[J1], gb2[J2], gw3[J2];  // per-lane column partials (column 16 n + lane % 16)
#pragma unroll
  for (int n = 0; n < J1; ++n) gb1[n] = 0.f;
#pragma unroll
  for (int n = 0; n < J2; ++n) gb2[n] = gw3[n] = 0.f;
  float gb3 = 0.f;

  DaRaw cur = {};
  if (blockIdx.x < p.batch) cur = da_load<E, true>(p, blockIdx.x, task, lane);
  for (int64_t b = blockIdx.x; b < p.batch; b += gridDim.x) {
    DaRaw nxt = {};
    if (b + gridDim.x < p.batch) nxt = da_load<E, true>(p, b + gridDim.x, task, lane);
    // ---- phase 0: X / X^T, q, du, g_j = du . k_j ----
    if (task.on) {
      float qv[8], kv[8], dv[8];
      da_build_x<S, E, true>(p, cur, task, sm, qv, kv);
      Vec<uint16_t>::to_f32(cur.du, dv);
      float g = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) g = fmaf(dv[i], kv[i], g);
#pragma unroll
      for (int off = 1; off < DaTask<E>::CH; off <<= 1) g += __shfl_xor(g, off);
      if (task.c == 0) sg[task.j] = g;
      if (task.j == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          sq[task.c + i] = qv[i];
          sdu[task.c + i] = dv[i];
        }
      }
    }
    const float aj = cur.a;  // lane = history row
    // rows past the last one with a_j != 0 have ds = 0, dX = 0 and add nothing to the
    // weight gradients: their row tiles skip every MFMA (accumulators stay 0, so the
    // epilogues store the same zeros), and the dW k steps past them are skipped
    const uint64_t am = __ballot(aj != 0.f);
    const int nv = am ? 64 - __clzll(am) : 0;
    const bool act = 16 * rt < nv;
    const int kk = nv > 32 ? 2 : 1;
    __syncthreads();
    DA_STAMP(2 + 8 * sidx + 0);
    // ---- phase 1: ds (every wave, lane = row), layer 1 -> H1, H1^T ----
    const float gj = sg[lane];
    const float ag = sum_wave(aj * gj);
    const float dsj = aj * (gj - ag);
    if (w == 0) gb3 += sum_wave(dsj);  // lane 0's value is written
    {
      da_f32x4 acc[J1];
      da_layer1<S, H1T>(sm, rt, cg, lane, act, acc);
#pragma unroll
      for (int jn = 0; jn < J1; ++jn) {
        const int n = cg + DA_CG * jn;
        if (n >= H1T) continue;
        const int col = 16 * n + (lane & 15);
        const float bias = sb1[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * rt + 4 * (lane >> 4) + i;
          const uint16_t h = f32_to_bf16_rne(fmaxf(acc[jn][i] + bias, 0.f));
          sm[S::oH1 + r * S::LDH + col] = h;
          sm[S::oH1T + col * DA_LDT + r] = h;
        }
      }
    }
    __syncthreads();
    DA_STAMP(2 + 8 * sidx + 1);
    // ---- phase 2: layer 2, dZ2 = ds w3 relu'(z2) -> dZ2 (over H1), dZ2^T ----
    {
      da_f32x4 acc[J2];
      da_layer2<S, H1K, H2T>(sm, rt, cg, lane, act, acc);
      __syncthreads();  // both column groups' reads of these H1 rows precede the dZ2 stores
#pragma unroll
      for (int jn = 0; jn < J2; ++jn) {
        const int n = cg + DA_CG * jn;
        if (n >= H2T) continue;
        const int col = 16 * n + (lane & 15);
        const float bias = sb2[col], wv = sw3[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * rt + 4 * (lane >> 4) + i;
          const float dsr = __shfl(dsj, r);
          const float h2 = fmaxf(acc[jn][i] + bias, 0.f);
          const float dz = h2 > 0.f ? dsr * wv : 0.f;
          gw3[jn] = fmaf(dsr, h2, gw3[jn]);
          gb2[jn] += dz;
          const uint16_t hz = f32_to_bf16_rne(dz);
          sm[S::oH1 + r * S::LDH + col] = hz;
          sm[S::oZ2T + col * DA_LDT + r] = hz;
        }
      }
    }
    __syncthreads();
    DA_STAMP(2 + 8 * sidx + 2);
    // ---- phase 3: dH1 = dZ2 W2, dZ1 = dH1 relu'(H1) -> dZ1 (over X), dZ1^T; dW2 ----
    {
      da_f32x4 acc[J1];
#pragma unroll
      for (int jn = 0; jn < J1; ++jn) acc[jn] = da_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < H2K; ++s) {
        if (!act) break;
        const da_bf16x8 a = da_frag(sm + S::oH1, S::LDH, 16 * rt, 32 * s, lane);
#pragma unroll
        for (int jn = 0; jn < J1; ++jn) {
          const int n = cg + DA_CG * jn;
          if (n < H1T)
            acc[jn] = da_mfma(a, da_frag(sm + S::oW2T, S::LDW2T, 16 * n, 32 * s, lane), acc[jn]);
        }
      }
#pragma unroll
      for (int jn = 0; jn < J1; ++jn) {
        const int n = cg + DA_CG * jn;
        if (n >= H1T) continue;
        const int col = 16 * n + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * rt + 4 * (lane >> 4) + i;
          const uint16_t h = sm[S::oH1T + col * DA_LDT + r];
          const float dz = (h != 0 && !(h & 0x8000u)) ? acc[jn][i] : 0.f;
          gb1[jn] += dz;
          const uint16_t hz = f32_to_bf16_rne(dz);
          sm[S::oX + r * S::LDH + col] = hz;  // dZ1 over X (dead since phase 1)
          sm[S::oZ1T + col * DA_LDT + r] = hz;
        }
      }
#pragma unroll
      for (int i = 0; i < NW2; ++i) {
        const int t = w + NWV * i;
        if (t < H2T * H1T) {
          const int m = t / H1T, n = t - m * H1T;
#pragma unroll
          for (int s = 0; s < 2; ++s)
            if (s < kk)
            gw2[i] = da_mfma(da_frag(sm + S::oZ2T, DA_LDT, 16 * m, 32 * s, lane),
                             da_frag(sm + S::oH1T, DA_LDT, 16 * n, 32 * s, lane), gw2[i]);
        }
      }
    }
    __syncthreads();
    DA_STAMP(2 + 8 * sidx + 3);
    // ---- phase 4: dX = dZ1 W1 -> d rows (dk per row, dq parts); dW1 ----
    {
      // the wave's X column tiles: blocks q / k / q-k / q*k of column tiles c16 = cg + DA_CG jx
      da_f32x4 acc[JX][4];
#pragma unroll
      for (int jx = 0; jx < JX; ++jx)
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) acc[jx][blk] = da_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < H1K; ++s) {
        if (!act) break;
        const da_bf16x8 a = da_frag(sm + S::oX, S::LDH, 16 * rt, 32 * s, lane);
#pragma unroll
        for (int jx = 0; jx < JX; ++jx) {
          const int c16 = cg + DA_CG * jx;
          if (c16 >= EC) continue;
#pragma unroll
          for (int blk = 0; blk < 4; ++blk)
            acc[jx][blk] = da_mfma(
                a, da_frag(sm + S::oW1T, S::LDH, 16 * (blk * EC + c16), 32 * s, lane),
                acc[jx][blk]);
        }
      }
#pragma unroll
      for (int jx = 0; jx < JX; ++jx) {
        const int c16 = cg + DA_CG * jx;
        if (c16 >= EC) continue;
        const int e = 16 * c16 + (lane & 15);
        const float qe = sq[e], due = sdu[e];
        float dqp = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * rt + 4 * (lane >> 4) + i;
          const float dfq = acc[jx][0][i], dfk = acc[jx][1][i];
          const float dfd = acc[jx][2][i], dfm = acc[jx][3][i];
          const float ke = bf16_to_f32(sm[S::oXT + (E + e) * DA_LDT + r]);
          const float ar = __shfl(aj, r);
          const float dk = fmaf(ar, due, dfk - dfd + dfm * qe);
          if (r < p.L)
            p.drows[(p.batch + b * p.L + r) * p.ld_drows + e] = f32_to_bf16_rne(dk);
          dqp += dfq + dfd + dfm * ke;
        }
        dqp = swap32_sum(swap16_sum(dqp));  // the 4 row groups of column e
        if (lane < 16) sdq[rt * E + e] = dqp;
      }
#pragma unroll
      for (int i = 0; i < NW1; ++i) {
        const int t = w + NWV * i;
        if (t < H1T * NTX) {
          const int m = t / NTX, n = t - m * NTX;
#pragma unroll
          for (int s = 0; s < 2; ++s)
            if (s < kk)
            gw1[i] = da_mfma(da_frag(sm + S::oZ1T, DA_LDT, 16 * m, 32 * s, lane),
                             da_frag(sm + S::oXT, DA_LDT, 16 * n, 32 * s, lane), gw1[i]);
        }
      }
    }
    __syncthreads();
    DA_STAMP(2 + 8 * sidx + 4);
    if (tid < E) {
      const float v = bf16_to_f32(p.dtop[b * p.lddt + tid]) + sdq[tid] + sdq[E + tid] +
                      sdq[2 * E + tid] + sdq[3 * E + tid];
      p.drows[b * p.ld_drows + tid] = f32_to_bf16_rne(v);
    }
    cur = nxt;
    DA_STAMP(2 + 8 * sidx + 5);
    ++sidx;
  }

  // ---- weight-gradient partials of this workgroup ----
  float *part = p.part + static_cast<int64_t>(blockIdx.x) * p.P;
  const int E4 = S::E4, H1 = p.H1, H2 = p.H2;
  float *pw2 = part + H1 * E4, *pb1 = pw2 + H2 * H1, *pb2 = pb1 + H1, *pw3 = pb2 + H2,
        *pb3 = pw3 + H2;
#pragma unroll
  for (int i = 0; i < NW1; ++i) {
    const int t = w + NWV * i;
    if (t < H1T * NTX) {
      const int m = t / NTX, n = t - m * NTX;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int h = 16 * m + 4 * (lane >> 4) + j;
        if (h < H1) part[h * E4 + 16 * n + (lane & 15)] = gw1[i][j];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NW2; ++i) {
    const int t = w + NWV * i;
    if (t < H2T * H1T) {
      const int m = t / H1T, n = t - m * H1T;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int h2 = 16 * m + 4 * (lane >> 4) + j, h1 = 16 * n + (lane & 15);
        if (h2 < H2 && h1 < H1) pw2[h2 * H1 + h1] = gw2[i][j];
      }
    }
  }
  // column partials: lanes l, l + 16, l + 32, l + 48 hold the same column; then the
  // 4 row tiles (each column belongs to one column group)
  __syncthreads();
  float *red = reinterpret_cast<float *>(da_lds);  // [4][H1N + 2 H2N] (LDS now dead)
  constexpr int RW = S::H1N + 2 * S::H2N;
#pragma unroll
  for (int jn = 0; jn < J1; ++jn) {
    const int n = cg + DA_CG * jn;
    const float v = swap32_sum(swap16_sum(gb1[jn]));
    if (n < H1T && lane < 16) red[rt * RW + 16 * n + lane] = v;
  }
#pragma unroll
  for (int jn = 0; jn < J2; ++jn) {
    const int n = cg + DA_CG * jn;
    const float v = swap32_sum(swap16_sum(gb2[jn])), u = swap32_sum(swap16_sum(gw3[jn]));
    if (n < H2T && lane < 16) {
      red[rt * RW + S::H1N + 16 * n + lane] = v;
      red[rt * RW + S::H1N + S::H2N + 16 * n + lane] = u;
    }
  }
  __syncthreads();
  for (int c = tid; c < RW; c += DA_THREADS) {
    const float v = red[c] + red[RW + c] + red[2 * RW + c] + red[3 * RW + c];
    if (c < S::H1N) {
      if (c < H1) pb1[c] = v;
    } else if (c < S::H1N + S::H2N) {
      if (c - S::H1N < H2) pb2[c - S::H1N] = v;
    } else if (c - S::H1N - S::H2N < H2) {
      pw3[c - S::H1N - S::H2N] = v;
    }
  }
  if (tid == 0) pb3[0] = gb3;
}

// ---------------------------------------------------------------------------
// backward, two samples in flight per workgroup (the default): waves 0-3 take one
// sample, waves 4-7 the next, each wave one 16-row tile of its sample with ALL
// column tiles.  No transposed copies: the operands whose k runs along history
// rows (dW1 = dZ1^T X, dW2 = dZ2^T H1) and the weights' transposed uses (dH1 =
// dZ2 W2, dX = dZ1 W1) are read with ds_read_b64_tr_b16 from the row-major
// buffers, which leaves LDS for two samples' X / H1 / dZ2 / dZ1.  A wave's layer 1
// -> layer 2 -> dH1 chain only touches its own rows, so a pair of samples takes 3
// workgroup barriers (X built; all rows' dZ2 / H1 / dZ1 for the weight gradients;
// the pair done) where the one-sample kernel took 6 per sample.
// ---------------------------------------------------------------------------
template <int E, int H1T, int H1K, int H2T, int H2K>
struct DaShape2 : DaShape<E, H1T, H1K, H2T, H2K> {
  using B = DaShape<E, H1T, H1K, H2T, H2K>;
  static constexpr int LDZ2 = B::H2P + 8;
  static constexpr int oW1 = 0;                       // W1 [H1P][LDX] (rows >= H1 zero)
  static constexpr int oW2 = oW1 + B::H1P * B::LDX;   // W2 [H2P][LDH] (rows >= H2 zero)
  static constexpr int oS = oW2 + B::H2P * B::LDH;    // two slots of:
  static constexpr int sX = 0;                        //   X [64][LDX]
  static constexpr int sH1 = sX + DA_ROWS * B::LDX;   //   H1 [64][LDH]
  static constexpr int sZ2 = sH1 + DA_ROWS * B::LDH;  //   dZ2 [64][LDZ2]
  static constexpr int sZ1 = sZ2 + DA_ROWS * LDZ2;    //   dZ1 [64][LDH]
  static constexpr int slot_elems = sZ1 + DA_ROWS * B::LDH;
  static constexpr int bf_end = oS + 2 * slot_elems;
  // fp32 tail: b1 [H1N], b2 [H2N], w3 [H2N], then per slot q [E], du [E], g [64], dq [4][E]
  static constexpr int nslot32 = 2 * E + DA_ROWS + 4 * E;
  static constexpr int nf32 = B::H1N + 2 * B::H2N + 2 * nslot32;
  static constexpr size_t core_bytes = bf_end * 2 + nf32 * 4;
  // per wave: its 16 rows' bf16 gradient staged in LDS so that the rows leave as
  // whole 16-B pieces (one 2-B store per lane: 8x the store instructions; the PMC
  // write count is the same either way, the lines merge before HBM)
  static constexpr int SP = E + 8;  // staging row pitch (elements)
  static constexpr size_t stage_off = (core_bytes + 15) / 16 * 16;
  static constexpr size_t bytes = stage_off + (DA_THREADS / 64) * 16 * SP * 2;
  static_assert(bytes <= 160 * 1024, "LDS");
  // after the loop: column partials [8][H1N + 2 H2N] | b3 [2]
  static constexpr size_t red_bytes = (8 * (B::H1N + 2 * B::H2N) + 2) * 4;
  static_assert(red_bytes <= bytes, "the end reduction reuses the workgroup's LDS");
};

// MFMA operand fragment with k running down the rows of a row-major bf16 buffer:
// lane l gets column c0 + l % 16, rows r0 + 8 (l / 16) .. + 8 (two
// ds_read_b64_tr_b16: each 16-lane group addresses 4 rows x 4 column quads)
__device__ __forceinline__ da_bf16x8 da_frag_tr(const uint16_t *base, int ld, int c0, int r0,
                                                int lane) {
  typedef short v4s_t __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;
  const int i = lane & 15, g = lane >> 4;
  const uint16_t *q = base + (r0 + 8 * g + (i >> 2)) * ld + c0 + 4 * (i & 3);
  const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t *)(q));
  const v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t *)(q + 4 * ld));
  return da_bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// X rows of one sample, row-major only: [q | k | q - k | q * k] (rows >= L zero)
template <int E, int LDX>
__device__ __forceinline__ void da_build_x_rm(const DinAttArgs &p, const DaRaw &raw,
                                              const DaTask<E> &t, uint16_t *X, float (&qv)[8],
                                              float (&kv)[8]) {
  const uint4 qraw = raw.q, kraw = raw.k;
  const bool real = t.j < p.L;
  Vec<uint16_t>::to_f32(qraw, qv);
  Vec<uint16_t>::to_f32(kraw, kv);
  float d[8], m[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    d[i] = qv[i] - kv[i];
    m[i] = qv[i] * kv[i];
  }
  uint4 dq = make_uint4(pack_bf16x2(d[0], d[1]), pack_bf16x2(d[2], d[3]), pack_bf16x2(d[4], d[5]),
                        pack_bf16x2(d[6], d[7]));
  uint4 mq = make_uint4(pack_bf16x2(m[0], m[1]), pack_bf16x2(m[2], m[3]), pack_bf16x2(m[4], m[5]),
                        pack_bf16x2(m[6], m[7]));
  uint4 qq = qraw;
  if (!real) qq = dq = mq = make_uint4(0, 0, 0, 0);
  uint16_t *x = X + t.j * LDX + t.c;
  *reinterpret_cast<uint4 *>(x) = qq;
  *reinterpret_cast<uint4 *>(x + E) = kraw;
  *reinterpret_cast<uint4 *>(x + 2 * E) = dq;
  *reinterpret_cast<uint4 *>(x + 3 * E) = mq;
}

template <int E, int H1T, int H1K, int H2T, int H2K, bool KC = false>
__global__ __launch_bounds__(DA_THREADS) void din_att_bwd2_kernel(DinAttArgs p, KClock kc) {
  KcScope<KC> kc_scope(kc);
  using S = DaShape2<E, H1T, H1K, H2T, H2K>;
  constexpr int NTX = S::NTX, EC = E / 16, LDX = S::LDX, LDH = S::LDH, LDZ2 = S::LDZ2;
  constexpr int NWV = DA_THREADS / 64;
  constexpr int NW1 = (H1T * NTX + NWV - 1) / NWV;  // dW1 tiles per wave (over both slots' rows)
  constexpr int NW2 = (H2T * H1T + NWV - 1) / NWV;  // dW2 tiles per wave
  extern __shared__ __attribute__((aligned(16))) char da_lds[];
  uint16_t *sm = reinterpret_cast<uint16_t *>(da_lds);
  float *sb1 = reinterpret_cast<float *>(da_lds + S::bf_end * 2);
  float *sb2 = sb1 + S::H1N;
  float *sw3 = sb2 + S::H2N;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, slot = w >> 2, rt = w & 3;
  float *sq = sw3 + S::H2N + slot * S::nslot32;  // this slot's q [E]
  float *sdu = sq + E;                           // du [E]
  float *sg = sdu + E;                           // g_j = du . k_j [64]
  float *sdq = sg + DA_ROWS;                     // per-row-tile dq parts [4][E]
  uint16_t *X = sm + S::oS + slot * S::slot_elems + S::sX;
  uint16_t *Hb = sm + S::oS + slot * S::slot_elems + S::sH1;
  uint16_t *Z2 = sm + S::oS + slot * S::slot_elems + S::sZ2;
  uint16_t *Z1 = sm + S::oS + slot * S::slot_elems + S::sZ1;
  const uint16_t *W1 = sm + S::oW1, *W2 = sm + S::oW2;
  const uint16_t *slots = sm + S::oS;
  uint16_t *stg = reinterpret_cast<uint16_t *>(da_lds + S::stage_off) + w * 16 * S::SP;
  __shared__ int snv[2];  // per slot: rows up to the last one with a_j != 0
  DA_STAMP(0);
  da_zero_lds(da_lds, S::bf_end * 2);
  __syncthreads();
  da_stage_weights<S, false>(p, sm, sb1, sb2, sw3);
  const DaTask<E> task(tid & 255);  // X chunk tasks of this thread's slot
  int sidx = 0;
  DA_STAMP(1);

  da_f32x4 gw1[NW1], gw2[NW2];
#pragma unroll
  for (int i = 0; i < NW1; ++i) gw1[i] = da_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NW2; ++i) gw2[i] = da_f32x4{0.f, 0.f, 0.f, 0.f};
  float gb1[H1T], gb2[H2T], gw3[H2T];  // per-lane column partials (column 16 n + lane % 16)
#pragma unroll
  for (int n = 0; n < H1T; ++n) gb1[n] = 0.f;
#pragma unroll
  for (int n = 0; n < H2T; ++n) gb2[n] = gw3[n] = 0.f;
  float gb3 = 0.f;

  const int64_t G = gridDim.x;
  int64_t b = blockIdx.x + G * slot;  // this slot's sample (samples blockIdx + G i: i even / odd)
  DaRaw cur = {};
  uint16_t dtq = 0;  // dtop[b, lane] (q part, raw bf16) for the dq tail (waves rt == 0)
  if (b < p.batch) {
    cur = da_load<E, true>(p, b, task, lane);
    if (rt == 0 && lane < E) dtq = p.dtop[b * p.lddt + lane];
  }
  // the dq tail of a pair runs in the next iteration (after its first barrier): a
  // store just before the loop's end made the iteration wait for its write
  int64_t tb = -1;     // pending tail: this slot's sample
  uint16_t tdq = 0;
  for (int64_t b0 = blockIdx.x; b0 < p.batch; b0 += 2 * G, b += 2 * G) {
    const bool have = b < p.batch;  // uniform per slot (slot 1 may be idle in the last pair)
    // ---- X, q, du, g_j = du . k_j ----
    if (task.on) {
      float qv[8], kv[8], dv[8];
      da_build_x_rm<E, LDX>(p, cur, task, X, qv, kv);
      Vec<uint16_t>::to_f32(cur.du, dv);
      float g = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) g = fmaf(dv[i], kv[i], g);
#pragma unroll
      for (int off = 1; off < DaTask<E>::CH; off <<= 1) g += __shfl_xor(g, off);
      if (task.c == 0) sg[task.j] = g;
      if (task.j == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          sq[task.c + i] = qv[i];
          sdu[task.c + i] = dv[i];
        }
      }
    }
    const float aj = cur.a;  // lane = history row (0 when this slot is idle)
    // the next pair's inputs, issued once this pair's are consumed: loaded at the top
    // of the iteration they made the X build wait for them (one vmcnt for both)
    DaRaw nxt = {};
    uint16_t dtq_n = 0;
    if (b + 2 * G < p.batch) {
      nxt = da_load<E, true>(p, b + 2 * G, task, lane);
      if (rt == 0 && lane < E) dtq_n = p.dtop[(b + 2 * G) * p.lddt + lane];
    }
    const uint64_t am = __ballot(aj != 0.f);
    const int nv = am ? 64 - __clzll(am) : 0;
    const bool act = 16 * rt < nv;
    if (rt == 0 && lane == 0) snv[slot] = nv;
    __syncthreads();
    DA_STAMP(2 + 8 * sidx + 0);
    // the weight gradients' k steps per slot: rows past 32 add nothing when no row
    // there carries a gradient
    const int kk0 = snv[0] > 32 ? 2 : 1, kk1 = snv[1] > 32 ? 2 : 1;
    if (tb >= 0 && rt == 0 && lane < E) {  // the previous pair's dq (sdq is rewritten after B2)
      const float v = bf16_to_f32(tdq) + sdq[lane] + sdq[E + lane] + sdq[2 * E + lane] +
                      sdq[3 * E + lane];
      p.drows[tb * p.ld_drows + lane] = f32_to_bf16_rne(v);
    }
    // ---- ds; layer 1 -> H1 (own rows) ----
    const float gj = sg[lane];
    const float ag = sum_wave(aj * gj);
    const float dsj = aj * (gj - ag);
    if (rt == 0) gb3 += sum_wave(dsj);
    {
      da_f32x4 acc[H1T];
#pragma unroll
      for (int n = 0; n < H1T; ++n) acc[n] = da_f32x4{0.f, 0.f, 0.f, 0.f};
      if (act) {
#pragma unroll
        for (int s = 0; s < S::KT1; ++s) {
          const da_bf16x8 a = da_frag(X, LDX, 16 * rt, 32 * s, lane);
#pragma unroll
          for (int n = 0; n < H1T; ++n) acc[n] = da_mfma(a, da_frag(W1, LDX, 16 * n, 32 * s, lane), acc[n]);
        }
      }
#pragma unroll
      for (int n = 0; n < H1T; ++n) {
        const int col = 16 * n + (lane & 15);
        const float bias = sb1[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * rt + 4 * (lane >> 4) + i;
          Hb[r * LDH + col] = f32_to_bf16_rne(fmaxf(acc[n][i] + bias, 0.f));
        }
      }
    }
    // ---- layer 2, dZ2 = ds w3 relu'(z2) -> dZ2 (own rows) ----
    {
      da_f32x4 acc[H2T];
#pragma unroll
      for (int n = 0; n < H2T; ++n) acc[n] = da_f32x4{0.f, 0.f, 0.f, 0.f};
      if (act) {
#pragma unroll
        for (int s = 0; s < H1K; ++s) {
          const da_bf16x8 a = da_frag(Hb, LDH, 16 * rt, 32 * s, lane);
#pragma unroll
          for (int n = 0; n < H2T; ++n) acc[n] = da_mfma(a, da_frag(W2, LDH, 16 * n, 32 * s, lane), acc[n]);
        }
      }
#pragma unroll
      for (int n = 0; n < H2T; ++n) {
        const int col = 16 * n + (lane & 15);
        const float bias = sb2[col], wv = sw3[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * rt + 4 * (lane >> 4) + i;
          const float dsr = __shfl(dsj, r);
          const float h2 = fmaxf(acc[n][i] + bias, 0.f);
          const float dz = h2 > 0.f ? dsr * wv : 0.f;
          gw3[n] = fmaf(dsr, h2, gw3[n]);
          gb2[n] += dz;
          Z2[r * LDZ2 + col] = f32_to_bf16_rne(dz);
        }
      }
    }
    // ---- dH1 = dZ2 W2, dZ1 = dH1 relu'(H1) -> dZ1 (own rows) ----
    {
      da_f32x4 acc[H1T];
#pragma unroll
      for (int n = 0; n < H1T; ++n) acc[n] = da_f32x4{0.f, 0.f, 0.f, 0.f};
      if (act) {
#pragma unroll
        for (int s = 0; s < H2K; ++s) {
          const da_bf16x8 a = da_frag(Z2, LDZ2, 16 * rt, 32 * s, lane);
#pragma unroll
          for (int n = 0; n < H1T; ++n)
            acc[n] = da_mfma(a, da_frag_tr(W2, LDH, 16 * n, 32 * s, lane), acc[n]);
        }
      }
#pragma unroll
      for (int n = 0; n < H1T; ++n) {
        const int col = 16 * n + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * rt + 4 * (lane >> 4) + i;
          const uint16_t h = Hb[r * LDH + col];
          const float dz = (h != 0 && !(h & 0x8000u)) ? acc[n][i] : 0.f;
          gb1[n] += dz;
          Z1[r * LDH + col] = f32_to_bf16_rne(dz);
        }
      }
    }
    __syncthreads();
    DA_STAMP(2 + 8 * sidx + 1);
    // ---- dW2 += dZ2^T H1 over both slots' rows (k = history rows) ----
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const uint16_t *z2 = slots + sl * S::slot_elems + S::sZ2;
      const uint16_t *h1 = slots + sl * S::slot_elems + S::sH1;
      const int kks = sl ? kk1 : kk0;
#pragma unroll 1
      for (int s = 0; s < kks; ++s) {
#pragma unroll
        for (int i = 0; i < NW2; ++i) {
          const int t = w + NWV * i;
          if (t < H2T * H1T) {
            const int m = t / H1T, n = t - m * H1T;
            gw2[i] = da_mfma(da_frag_tr(z2, LDZ2, 16 * m, 32 * s, lane),
                             da_frag_tr(h1, LDH, 16 * n, 32 * s, lane), gw2[i]);
          }
        }
      }
    }
    // ---- dX = dZ1 W1 -> d rows (dk per row, dq parts), one 16-column chunk of
    // q / k / q-k / q*k at a time (registers) ----
#pragma unroll 1
    for (int c16 = 0; c16 < EC; ++c16) {
      da_f32x4 acc[4];
#pragma unroll
      for (int blk = 0; blk < 4; ++blk) acc[blk] = da_f32x4{0.f, 0.f, 0.f, 0.f};
      if (act) {
#pragma unroll
        for (int s = 0; s < H1K; ++s) {
          const da_bf16x8 a = da_frag(Z1, LDH, 16 * rt, 32 * s, lane);
#pragma unroll
          for (int blk = 0; blk < 4; ++blk)
            acc[blk] = da_mfma(a, da_frag_tr(W1, LDX, 16 * (blk * EC + c16), 32 * s, lane), acc[blk]);
        }
      }
      const int e = 16 * c16 + (lane & 15);
      const float qe = sq[e], due = sdu[e];
      float dqp = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * rt + 4 * (lane >> 4) + i;
        const float dfq = acc[0][i], dfk = acc[1][i];
        const float dfd = acc[2][i], dfm = acc[3][i];
        const float ke = bf16_to_f32(X[r * LDX + E + e]);
        const float ar = __shfl(aj, r);
        const float dk = fmaf(ar, due, dfk - dfd + dfm * qe);
        stg[(r - 16 * rt) * S::SP + e] = f32_to_bf16_rne(dk);
        dqp += dfq + dfd + dfm * ke;
      }
      dqp = swap32_sum(swap16_sum(dqp));  // the 4 row groups of column e
      if (lane < 16) sdq[rt * E + e] = dqp;
    }
    // the wave's 16 rows of dk leave as 16-B pieces (its own staging rows: a wave-local
    // LDS round trip, no barrier)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (have) {
      constexpr int QPR = E / 8;  // 16-B pieces per row
#pragma unroll
      for (int idx = lane; idx < 16 * QPR; idx += 64) {
        const int rr = idx / QPR, q = idx - rr * QPR, r = 16 * rt + rr;
        if (r < p.L)
          *reinterpret_cast<uint4 *>(p.drows + (p.batch + b * p.L + r) * p.ld_drows + 8 * q) =
              *reinterpret_cast<const uint4 *>(stg + rr * S::SP + 8 * q);
      }
    }
    // ---- dW1 += dZ1^T X over both slots' rows ----
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const uint16_t *z1 = slots + sl * S::slot_elems + S::sZ1;
      const uint16_t *x = slots + sl * S::slot_elems + S::sX;
      const int kks = sl ? kk1 : kk0;
#pragma unroll 1
      for (int s = 0; s < kks; ++s) {
#pragma unroll
        for (int i = 0; i < NW1; ++i) {
          const int t = w + NWV * i;
          if (t < H1T * NTX) {
            const int m = t / NTX, n = t - m * NTX;
            gw1[i] = da_mfma(da_frag_tr(z1, LDH, 16 * m, 32 * s, lane),
                             da_frag_tr(x, LDX, 16 * n, 32 * s, lane), gw1[i]);
          }
        }
      }
    }
    tb = have ? b : -1;
    tdq = dtq;
    cur = nxt;
    dtq = dtq_n;
    __syncthreads();
    DA_STAMP(2 + 8 * sidx + 2);
    ++sidx;
  }
  if (tb >= 0 && rt == 0 && lane < E) {  // the last pair's dq
    const float v = bf16_to_f32(tdq) + sdq[lane] + sdq[E + lane] + sdq[2 * E + lane] +
                    sdq[3 * E + lane];
    p.drows[tb * p.ld_drows + lane] = f32_to_bf16_rne(v);
  }

  // ---- weight-gradient partials of this workgroup ----
  float *part = p.part + static_cast<int64_t>(blockIdx.x) * p.P;
  const int E4 = S::E4, H1 = p.H1, H2 = p.H2;
  float *pw2 = part + H1 * E4, *pb1 = pw2 + H2 * H1, *pb2 = pb1 + H1, *pw3 = pb2 + H2,
        *pb3 = pw3 + H2;
#pragma unroll
  for (int i = 0; i < NW1; ++i) {
    const int t = w + NWV * i;
    if (t < H1T * NTX) {
      const int m = t / NTX, n = t - m * NTX;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int h = 16 * m + 4 * (lane >> 4) + j;
        if (h < H1) part[h * E4 + 16 * n + (lane & 15)] = gw1[i][j];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NW2; ++i) {
    const int t = w + NWV * i;
    if (t < H2T * H1T) {
      const int m = t / H1T, n = t - m * H1T;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int h2 = 16 * m + 4 * (lane >> 4) + j, h1 = 16 * n + (lane & 15);
        if (h2 < H2 && h1 < H1) pw2[h2 * H1 + h1] = gw2[i][j];
      }
    }
  }
  // column partials: the 4 row groups of a lane column, then the 8 (slot, row tile)
  // waves in fixed order
  constexpr int RW = S::H1N + 2 * S::H2N;
  float *red = reinterpret_cast<float *>(da_lds);  // [8][RW] | b3 [2]
  float *rb3 = red + 8 * RW;
  __syncthreads();  // the LDS buffers are dead
#pragma unroll
  for (int n = 0; n < H1T; ++n) {
    const float v = swap32_sum(swap16_sum(gb1[n]));
    if (lane < 16) red[w * RW + 16 * n + lane] = v;
  }
#pragma unroll
  for (int n = 0; n < H2T; ++n) {
    const float v = swap32_sum(swap16_sum(gb2[n])), u = swap32_sum(swap16_sum(gw3[n]));
    if (lane < 16) {
      red[w * RW + S::H1N + 16 * n + lane] = v;
      red[w * RW + S::H1N + S::H2N + 16 * n + lane] = u;
    }
  }
  if (rt == 0 && lane == 0) rb3[slot] = gb3;
  __syncthreads();
  for (int c = tid; c < RW; c += DA_THREADS) {
    float v = red[c];
#pragma unroll
    for (int q = 1; q < 8; ++q) v += red[q * RW + c];
    if (c < S::H1N) {
      if (c < H1) pb1[c] = v;
    } else if (c < S::H1N + S::H2N) {
      if (c - S::H1N < H2) pb2[c - S::H1N] = v;
    } else if (c - S::H1N - S::H2N < H2) {
      pw3[c - S::H1N - S::H2N] = v;
    }
  }
  if (tid == 0) pb3[0] = rb3[0] + rb3[1];
}

__global__ __launch_bounds__(1024) void din_att_wgrad_kernel(
    const float *__restrict__ part, int parts, int64_t P, int E4, int H1, int H2, float *grads,
    float lr, float *w1, int64_t ldw1, float *b1, float *w2, int64_t ldw2, float *b2, float *w3,
    float *b3) {
  // 16 waves per 64 parameters, each summing its slice of the partials with every
  // load of the slice in flight (parts <= 256: <= 16 per wave), then the 16 slice
  // sums in slice order: a fixed order, deterministic run to run
  constexpr int NS = 16;
  __shared__ float red[NS][64];
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 64 + cl;
  const int per = (parts + NS - 1) / NS, g0 = sl * per, g1 = min(parts, g0 + per);
  float v = 0.f;
  if (i < P) {
    int g = g0;
    for (; g + 16 <= g1; g += 16) {
      float x[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) x[u] = part[(g + u) * P + i];
#pragma unroll
      for (int u = 0; u < 16; ++u) v += x[u];
    }
    for (; g + 4 <= g1; g += 4) {
      const float x0 = part[(g + 0) * P + i], x1 = part[(g + 1) * P + i];
      const float x2 = part[(g + 2) * P + i], x3 = part[(g + 3) * P + i];
      v += x0;
      v += x1;
      v += x2;
      v += x3;
    }
    for (; g < g1; ++g) v += part[g * P + i];
  }
  red[sl][cl] = v;
  __syncthreads();
  if (sl != 0 || i >= P) return;
  v = red[0][cl];
#pragma unroll
  for (int q = 1; q < NS; ++q) v += red[q][cl];
  if (grads) {
    grads[i] = v;
    return;
  }
  int64_t o = i;
  if (o < H1 * E4) {
    float &x = w1[(o / E4) * ldw1 + o % E4];
    x -= lr * v;
    return;
  }
  o -= H1 * E4;
  if (o < H2 * H1) {
    float &x = w2[(o / H1) * ldw2 + o % H1];
    x -= lr * v;
    return;
  }
  o -= H2 * H1;
  if (o < H1) { b1[o] -= lr * v; return; }
  o -= H1;
  if (o < H2) { b2[o] -= lr * v; return; }
  o -= H2;
  if (o < H2) { w3[o] -= lr * v; return; }
  b3[0] -= lr * v;
}

}  // namespace mrec

using namespace mrec;

namespace {

// the compiled attention-unit shapes: (E, H1, H2) -> kernels
#define MREC_DA_SHAPES(X) \
  X(32, 5, 3, 3, 2)       \
  X(16, 2, 1, 1, 1)

template <int E, int H1T, int H1K, int H2T, int H2K>
bool da_match(int e, int h1, int h2) {
  return e == E && (h1 + 15) / 16 == H1T && (h1 + 31) / 32 == H1K && (h2 + 15) / 16 == H2T &&
         (h2 + 31) / 32 == H2K;
}

int da_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        v <= 0)
      v = 256;
    (void)hipGetLastError();
    return v;
  }();
  return n;
}

template <int E, int H1T, int H1K, int H2T, int H2K>
void da_set_attrs() {
  using S = DaShape<E, H1T, H1K, H2T, H2K>;
  (void)hipFuncSetAttribute(reinterpret_cast<const void *>(din_att_fwd_kernel<E, H1T, H1K, H2T, H2K>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(S::fwd_bytes));
  (void)hipFuncSetAttribute(reinterpret_cast<const void *>(din_att_bwd_kernel<E, H1T, H1K, H2T, H2K>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(S::bwd_bytes));
  for (const void *k : {reinterpret_cast<const void *>(din_att_bwd2_kernel<E, H1T, H1K, H2T, H2K, false>),
                        reinterpret_cast<const void *>(din_att_bwd2_kernel<E, H1T, H1K, H2T, H2K, true>)})
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(DaShape2<E, H1T, H1K, H2T, H2K>::bytes));
  for (const void *k : {reinterpret_cast<const void *>(din_att_fwd_wave_kernel<E, H1T, H1K, H2T, H2K, false>),
                        reinterpret_cast<const void *>(din_att_fwd_wave_kernel<E, H1T, H1K, H2T, H2K, true>)})
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(DaShapeF<E, H1T, H1K, H2T, H2K>::bytes));
  (void)hipGetLastError();
}

// MREC_DIN_FWD_WG=1: the one-workgroup-per-sample forward (A/B and parity yardstick;
// read per call so a test can switch it)
bool da_fwd_wg() {
  const char *e = std::getenv("MREC_DIN_FWD_WG");
  return e && e[0] == '1';
}

// MREC_DIN_BWD_ONE=1: the one-sample-per-workgroup backward (A/B and parity yardstick)
bool da_one_sample() {
  static const bool v = [] {
    const char *e = std::getenv("MREC_DIN_BWD_ONE");
    return e && e[0] == '1';
  }();
  return v;
}

bool da_supported(int E, int H1, int H2) {
  if (H1 % 4 != 0) return false;
#define X(e, a, b, c, d) if (da_match<e, a, b, c, d>(E, H1, H2)) return true;
  MREC_DA_SHAPES(X)
#undef X
  return false;
}

}  // namespace

static unsigned long long *g_da_stamps = nullptr;

// MREC_DA_STAMP_FWD=1: the debug stamps go to the wave forward, not the backward
static bool da_stamp_fwd() {
  const char *e = std::getenv("MREC_DA_STAMP_FWD");
  return e && e[0] == '1';
}

extern "C" {

// diagnostics (not in mrec.h): phase clocks of the next backward launches (NULL: off)
void mrec_din_att_debug_stamps(void *buf) { g_da_stamps = static_cast<unsigned long long *>(buf); }

int32_t mrec_din_att_supported(int32_t E, int32_t H1, int32_t H2) {
  return da_supported(E, H1, H2) ? 1 : 0;
}

int64_t mrec_din_att_parts(int64_t batch) {
  const int64_t g = da_cus();
  return batch < g ? (batch > 0 ? batch : 1) : g;
}

int64_t mrec_din_att_param_count(int32_t E, int32_t H1, int32_t H2) {
  return static_cast<int64_t>(H1) * 4 * E + static_cast<int64_t>(H2) * H1 + H1 + 2 * H2 + 1;
}

static mrec_status da_check(const void *rows, int64_t ld_rows, int64_t batch, int32_t L, int32_t E,
                            const float *w1, int64_t ldw1, const float *b1, int32_t H1,
                            const float *w2, int64_t ldw2, const float *b2, int32_t H2,
                            const float *w3, const float *b3) {
  MREC_CHECK_ARG(rows && w1 && b1 && w2 && b2 && w3 && b3, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0 && L >= 1 && L <= DA_ROWS, "need 1 <= L <= 64");
  MREC_CHECK_ARG(da_supported(E, H1, H2), "attention-unit shape (E, H1, H2) not compiled");
  MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(rows) & 15) == 0 && ld_rows % 8 == 0 &&
                     ld_rows >= E,
                 "rows must be 16-byte aligned bf16 rows of >= E elements");
  MREC_CHECK_ARG(ldw1 >= 4 * E && ldw2 >= H1 && ldw1 % 4 == 0 && ldw2 % 4 == 0 && H1 % 4 == 0 &&
                     (reinterpret_cast<uintptr_t>(w1) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(w2) & 15) == 0,
                 "w1 / w2 16-byte aligned, ldw1, ldw2 and H1 multiples of 4");
  return MREC_OK;
}

mrec_status mrec_din_att_fwd(const void *rows, int64_t ld_rows, const int32_t *his, int64_t ld_his,
                             int64_t batch, int32_t L, int32_t E, const float *w1, int64_t ldw1,
                             const float *b1, int32_t H1, const float *w2, int64_t ldw2,
                             const float *b2, int32_t H2, const float *w3, const float *b3,
                             float *a, void *top, int64_t ldt, mrec_stream stream) {
  const mrec_status st = da_check(rows, ld_rows, batch, L, E, w1, ldw1, b1, H1, w2, ldw2, b2, H2,
                                  w3, b3);
  if (st != MREC_OK) return st;
  MREC_CHECK_ARG(his && a && top, "NULL pointer");
  MREC_CHECK_ARG(ld_his >= L && ldt >= 2 * E, "bad strides");
  if (batch == 0) return MREC_OK;
  DinAttArgs p{};
  p.rows = static_cast<const uint16_t *>(rows);
  p.ld_rows = ld_rows;
  p.his = his;
  p.ld_his = ld_his;
  p.w1 = w1, p.b1 = b1, p.w2 = w2, p.b2 = b2, p.w3 = w3, p.b3 = b3;
  p.ldw1 = ldw1, p.ldw2 = ldw2;
  p.batch = batch, p.L = L, p.H1 = H1, p.H2 = H2;
  p.a = a;
  p.top = static_cast<uint16_t *>(top);
  p.ldt = ldt;
  p.stamps = da_stamp_fwd() ? g_da_stamps : nullptr;
  const bool wg = da_fwd_wg();
  // one workgroup (8 sample waves) per CU, or one sample per workgroup
  const int64_t grid = wg ? std::min<int64_t>(batch, 2 * static_cast<int64_t>(da_cus()))
                          : std::min<int64_t>((batch + 7) / 8, da_cus());
  hipStream_t s = static_cast<hipStream_t>(stream);
#define X(e, h1t, h1k, h2t, h2k)                                                              \
  if (da_match<e, h1t, h1k, h2t, h2k>(E, H1, H2)) {                                         \
    static const int once = (da_set_attrs<e, h1t, h1k, h2t, h2k>(), 1);                     \
    (void)once;                                                                             \
    if (wg)                                                                                 \
      din_att_fwd_kernel<e, h1t, h1k, h2t, h2k>                                             \
          <<<dim3(static_cast<unsigned>(grid)), DA_THREADS,                                 \
             DaShape<e, h1t, h1k, h2t, h2k>::fwd_bytes, s>>>(p);                            \
    else if (const KClock kc = kclock_take(); kc.buf)                                       \
      din_att_fwd_wave_kernel<e, h1t, h1k, h2t, h2k, true>                                  \
          <<<dim3(static_cast<unsigned>(grid)), DA_THREADS,                                 \
             DaShapeF<e, h1t, h1k, h2t, h2k>::bytes, s>>>(p, kc);                           \
    else                                                                                    \
      din_att_fwd_wave_kernel<e, h1t, h1k, h2t, h2k, false>                                 \
          <<<dim3(static_cast<unsigned>(grid)), DA_THREADS,                                 \
             DaShapeF<e, h1t, h1k, h2t, h2k>::bytes, s>>>(p, kc);                           \
    return launch_status("mrec_din_att_fwd");                                               \
  }
  MREC_DA_SHAPES(X)
#undef X
  return MREC_EINVAL;
}

mrec_status mrec_din_att_bwd(const void *rows, int64_t ld_rows, int64_t batch, int32_t L,
                             int32_t E, const float *w1, int64_t ldw1, const float *b1, int32_t H1,
                             const float *w2, int64_t ldw2, const float *b2, int32_t H2,
                             const float *w3, const float *b3, const float *a, const void *dtop,
                             int64_t lddt, void *d_rows, int64_t ld_drows, float *part,
                             int64_t parts, mrec_stream stream) {
  const mrec_status st = da_check(rows, ld_rows, batch, L, E, w1, ldw1, b1, H1, w2, ldw2, b2, H2,
                                  w3, b3);
  if (st != MREC_OK) return st;
  MREC_CHECK_ARG(a && dtop && d_rows && part, "NULL pointer");
  MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(dtop) & 15) == 0 && lddt % 8 == 0 && lddt >= 2 * E,
                 "dtop must be 16-byte aligned bf16 rows of >= 2E elements");
  MREC_CHECK_ARG(ld_drows >= E && ld_drows % 8 == 0 && (reinterpret_cast<uintptr_t>(d_rows) & 15) == 0,
                 "d_rows must be 16-byte aligned bf16 rows (ld_drows a multiple of 8, >= E)");
  MREC_CHECK_ARG(parts == mrec_din_att_parts(batch), "parts must be mrec_din_att_parts(batch)");
  if (batch == 0) return MREC_OK;
  DinAttArgs p{};
  p.rows = static_cast<const uint16_t *>(rows);
  p.ld_rows = ld_rows;
  p.w1 = w1, p.b1 = b1, p.w2 = w2, p.b2 = b2, p.w3 = w3, p.b3 = b3;
  p.ldw1 = ldw1, p.ldw2 = ldw2;
  p.batch = batch, p.L = L, p.H1 = H1, p.H2 = H2;
  p.a = const_cast<float *>(a);
  p.dtop = static_cast<const uint16_t *>(dtop);
  p.lddt = lddt;
  p.drows = static_cast<uint16_t *>(d_rows);
  p.ld_drows = ld_drows;
  p.part = part;
  p.P = mrec_din_att_param_count(E, H1, H2);
  p.stamps = da_stamp_fwd() ? nullptr : g_da_stamps;
  hipStream_t s = static_cast<hipStream_t>(stream);
#define X(e, h1t, h1k, h2t, h2k)                                                              \
  if (da_match<e, h1t, h1k, h2t, h2k>(E, H1, H2)) {                                         \
    static const int once = (da_set_attrs<e, h1t, h1k, h2t, h2k>(), 1);                     \
    (void)once;                                                                             \
    if (da_one_sample())                                                                    \
      din_att_bwd_kernel<e, h1t, h1k, h2t, h2k>                                             \
          <<<dim3(static_cast<unsigned>(parts)), DA_THREADS,                                \
             DaShape<e, h1t, h1k, h2t, h2k>::bwd_bytes, s>>>(p);                            \
    else if (const KClock kc = kclock_take(); kc.buf)                                       \
      din_att_bwd2_kernel<e, h1t, h1k, h2t, h2k, true>                                      \
          <<<dim3(static_cast<unsigned>(parts)), DA_THREADS,                                \
             DaShape2<e, h1t, h1k, h2t, h2k>::bytes, s>>>(p, kc);                           \
    else                                                                                    \
      din_att_bwd2_kernel<e, h1t, h1k, h2t, h2k, false>                                     \
          <<<dim3(static_cast<unsigned>(parts)), DA_THREADS,                                \
             DaShape2<e, h1t, h1k, h2t, h2k>::bytes, s>>>(p, kc);                           \
    return launch_status("mrec_din_att_bwd");                                               \
  }
  MREC_DA_SHAPES(X)
#undef X
  return MREC_EINVAL;
}

mrec_status mrec_din_att_wgrad(const float *part, int64_t parts, int32_t E, int32_t H1, int32_t H2,
                               float *grads, float lr, float *w1, int64_t ldw1, float *b1,
                               float *w2, int64_t ldw2, float *b2, float *w3, float *b3,
                               mrec_stream stream) {
  MREC_CHECK_ARG(part && parts >= 1, "NULL pointer / no partials");
  MREC_CHECK_ARG(grads || (w1 && b1 && w2 && b2 && w3 && b3), "need grads or the parameters");
  const int64_t P = mrec_din_att_param_count(E, H1, H2);
  din_att_wgrad_kernel<<<dim3(static_cast<unsigned>((P + 63) / 64)), 1024, 0,
                         static_cast<hipStream_t>(stream)>>>(
      part, static_cast<int>(parts), P, 4 * E, H1, H2, grads, lr, w1, ldw1, b1, w2, ldw2, b2, w3,
      b3);
  return launch_status("mrec_din_att_wgrad");
}

}  // extern "C"
