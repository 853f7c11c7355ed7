// CTR head: output projection + logit sum, BCE-with-logits loss and gradient,
// and a deterministic scaled column sum (bias / small weight gradients).
//
// These replace ~15 tiny ATen launches per step (addmm(400->1), add, cast,
// binary_cross_entropy_with_logits fwd/bwd, mean, sum, a rocBLAS GEMV for the
// dense first-order weight gradient) with four kernels.
#include <algorithm>

#include "common.h"
#include "head_common.h"

namespace mrec {

// z[b] = base[b] + bias + sum_h h[b, h] * w[h]   (one wave per row, bf16 h, fp32 w)
__global__ __launch_bounds__(256) void head_fwd_kernel(const uint16_t *__restrict__ h, int64_t ldh,
                                                       int64_t B, int H, const float *__restrict__ w,
                                                       const float *__restrict__ bias,
                                                       const float *__restrict__ base,
                                                       float *__restrict__ z) {
  const int lane = threadIdx.x & 63;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const uint16_t *row = h + b * ldh;
  float acc = 0.f;
  for (int c = lane * 8; c < H; c += 512) {
    if (c + 8 <= H) {
      const uint4 r = *reinterpret_cast<const uint4 *>(row + c);
      float v[8];
      Vec<uint16_t>::to_f32(r, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = fmaf(v[j], w[c + j], acc);
    } else {
      for (int j = 0; c + j < H; ++j) acc = fmaf(bf16_to_f32(row[c + j]), w[c + j], acc);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if (lane == 0) z[b] = acc + (bias ? bias[0] : 0.f) + (base ? base[b] : 0.f);
}

// dh[b, h] = dz[b] * w[h] (* relu'(mask[b, h]))  (bf16 out, row stride ldh; pad
// columns up to ldh zeroed)
__global__ __launch_bounds__(256) void head_bwd_kernel(const float *__restrict__ dz,
                                                       const float *__restrict__ w, int64_t B, int H,
                                                       const uint16_t *__restrict__ mask,
                                                       int64_t ld_mask, uint16_t *__restrict__ dh,
                                                       int64_t ldh) {
  const int64_t n8 = ldh / 8;
  const int64_t total = B * n8;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t b = i / n8;
    const int c = static_cast<int>(i - b * n8) * 8;
    const float g = dz[b];
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (c + j < H) ? g * w[c + j] : 0.f;
    if (mask) {
      const uint4 mv = *reinterpret_cast<const uint4 *>(mask + b * ld_mask + c);
      const uint32_t mw[4] = {mv.x, mv.y, mv.z, mv.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t h = (mw[j >> 1] >> ((j & 1) * 16)) & 0xffffu;
        if (h == 0 || (h & 0x8000u)) v[j] = 0.f;
      }
    }
    *reinterpret_cast<uint4 *>(dh + b * ldh + c) =
        make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                   pack_bf16x2(v[6], v[7]));
  }
}

// BCE with logits, mean over B.  One 1024-thread block, fixed-order reduction.
//   loss = mean( max(z,0) - z*y + log1p(exp(-|z|)) )
__global__ __launch_bounds__(1024) void bce_fwd_kernel(const float *__restrict__ z,
                                                       const float *__restrict__ y, int64_t B,
                                                       float *__restrict__ loss) {
  __shared__ float red[1024 / 64];
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < B; i += 1024) {
    const float zi = z[i], yi = y[i];
    acc += fmaxf(zi, 0.f) - zi * yi + log1pf(__expf(-fabsf(zi)));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < 1024 / 64; ++i) s += red[i];
    loss[0] = B > 0 ? s / static_cast<float>(B) : 0.f;
  }
}

// dz[b] = g * (sigmoid(z[b]) - y[b]) / B   (g = upstream grad of the mean loss)
__global__ __launch_bounds__(256) void bce_bwd_kernel(const float *__restrict__ z,
                                                      const float *__restrict__ y, int64_t B,
                                                      const float *__restrict__ g,
                                                      float *__restrict__ dz) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= B) return;
  const float scale = (g ? g[0] : 1.f) / static_cast<float>(B);
  const float zi = z[i];
  const float sig = 1.f / (1.f + __expf(-zi));
  dz[i] = scale * (sig - y[i]);
}

// column sums: one 1024-thread workgroup per 8 columns (the last one, when asked,
// sums s itself); rows strided over the threads (4 independent loads in flight per
// thread at B = 4096), then a fixed-order tree (wave butterfly, then the 16 wave
// partials summed in order): bitwise reproducible.
constexpr int CS_T = 1024;
constexpr int CS_W = CS_T / 64;

__global__ __launch_bounds__(CS_T) void colsum_kernel(const float *__restrict__ s,
                                                      const void *__restrict__ X, int x_bf16,
                                                      int vec, int64_t ldx, int64_t B, int64_t C,
                                                      float *__restrict__ out,
                                                      float *__restrict__ total, int update,
                                                      float lr) {
  __shared__ float red[CS_W][9];
  const int64_t c0 = static_cast<int64_t>(blockIdx.x) * 8;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool tot_block = c0 >= C;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int64_t b = tid; b < B; b += CS_T) {
    const float sb = s[b];
    if (tot_block) {
      acc[0] += sb;
      continue;
    }
    float x[8];
    if (vec) {
      Vec<uint16_t>::to_f32(*reinterpret_cast<const uint4 *>(static_cast<const uint16_t *>(X) +
                                                             b * ldx + c0), x);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t c = c0 + j;
        x[j] = c >= C ? 0.f
                      : (x_bf16 ? bf16_to_f32(static_cast<const uint16_t *>(X)[b * ldx + c])
                                : static_cast<const float *>(X)[b * ldx + c]);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = fmaf(sb, x[j], acc[j]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc[j] += __shfl_xor(acc[j], off);
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[w][j] = acc[j];
  }
  __syncthreads();
  if (tid < 8) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < CS_W; ++k) v += red[k][tid];
    if (tot_block) {
      if (tid == 0) total[0] = update ? fmaf(-lr, v, total[0]) : v;
    } else if (c0 + tid < C) {
      out[c0 + tid] = update ? fmaf(-lr, v, out[c0 + tid]) : v;
    }
  }
}

// ---------------------------------------------------------------------------
// fused CTR head + BCE-with-logits, forward and backward in one pass over h
// ---------------------------------------------------------------------------
constexpr int HEAD_RPW = 4;                     // rows per wave
constexpr int HEAD_RPB = 4 * HEAD_RPW;          // rows per 256-thread workgroup
constexpr int HEAD_MAXH = 1024;                 // h width handled (2 chunks of 8 per lane)

template <int NC>  // chunks of 8 columns per lane: H <= 512 * NC
__global__ __launch_bounds__(256) void ctr_head_kernel(
    const uint16_t *__restrict__ h, int64_t ldh, int64_t B, int H, const float *__restrict__ w,
    const float *__restrict__ bias, const float *__restrict__ base, const float *__restrict__ y,
    const float *__restrict__ xs, int64_t ldxs, int ns, const float *__restrict__ ws,
    const float *__restrict__ b2, int relu, float *__restrict__ z, float *__restrict__ dz,
    uint16_t *__restrict__ dh, int64_t lddh, float *__restrict__ part, int64_t ldp,
    float *__restrict__ loss_part, unsigned *__restrict__ ticket, float *__restrict__ loss) {
  __shared__ float red[4][HEAD_MAXH + 1 + 64];
  __shared__ float sred[4][2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t r0 = (static_cast<int64_t>(blockIdx.x) * 4 + wv) * HEAD_RPW;
  const float invB = 1.f / static_cast<float>(B);
  const float b0 = (bias ? bias[0] : 0.f) + (b2 ? b2[0] : 0.f);
  const float wsl = lane < ns ? ws[lane] : 0.f;  // side linear: lane j holds ws[j] (ns <= 64)
  float sacc = 0.f;
  float wr[NC][8], acc[NC][8];
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = (q * 64 + lane) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      wr[q][j] = c + j < H ? w[c + j] : 0.f;
      acc[q][j] = 0.f;
    }
  }
  float dzs = 0.f, ls = 0.f;
  // every load of the wave's rows in flight before any math
  uint4 hraw[HEAD_RPW][NC];
  float xsr[HEAD_RPW], baser[HEAD_RPW], yr[HEAD_RPW];
#pragma unroll
  for (int rr = 0; rr < HEAD_RPW; ++rr) {
    const int64_t r = r0 + rr;
    const bool ok = r < B;
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int c = (q * 64 + lane) * 8;
      hraw[rr][q] = (ok && c < H) ? *reinterpret_cast<const uint4 *>(h + r * ldh + c)
                                  : make_uint4(0u, 0u, 0u, 0u);
    }
    xsr[rr] = (ok && lane < ns) ? xs[r * ldxs + lane] : 0.f;
    baser[rr] = (ok && base) ? base[r] : 0.f;
    yr[rr] = ok ? y[r] : 0.f;
  }
#pragma unroll
  for (int rr = 0; rr < HEAD_RPW; ++rr) {
    const int64_t r = r0 + rr;
    if (r >= B) break;  // uniform per wave
    float hv[NC][8];
    float dot = 0.f;
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      Vec<uint16_t>::to_f32(hraw[rr][q], hv[q]);
#pragma unroll
      for (int j = 0; j < 8; ++j) dot = fmaf(hv[q][j], wr[q][j], dot);
    }
    const float xsv = xsr[rr];
    dot = fmaf(xsv, wsl, dot);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dot += __shfl_xor(dot, off);
    const float zz = dot + b0 + baser[rr];
    const float yy = yr[rr];
    const float d = (1.f / (1.f + __expf(-zz)) - yy) * invB;
    sacc = fmaf(d, xsv, sacc);
    if (lane == 0) {
      z[r] = zz;
      dz[r] = d;
      dzs += d;
      ls += fmaxf(zz, 0.f) - zz * yy + log1pf(__expf(-fabsf(zz)));
    }
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int c = (q * 64 + lane) * 8;
      if (c >= lddh) continue;
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        g[j] = d * wr[q][j];
        if (relu && !(hv[q][j] > 0.f)) g[j] = 0.f;
        acc[q][j] = fmaf(d, hv[q][j], acc[q][j]);
      }
      *reinterpret_cast<uint4 *>(dh + r * lddh + c) =
          make_uint4(pack_bf16x2(g[0], g[1]), pack_bf16x2(g[2], g[3]), pack_bf16x2(g[4], g[5]),
                     pack_bf16x2(g[6], g[7]));
    }
  }
  // workgroup partial of dW (4 waves summed in order), db and the loss
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int c = (q * 64 + lane) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (c + j < H) red[wv][c + j] = acc[q][j];
  }
  if (lane < ns) red[wv][H + 1 + lane] = sacc;
  if (lane == 0) {
    sred[wv][0] = dzs;
    sred[wv][1] = ls;
  }
  __syncthreads();
  float *prow = part + static_cast<int64_t>(blockIdx.x) * ldp;
  for (int c = threadIdx.x; c < H + 1 + ns; c += 256)
    if (c != H) prow[c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
  __shared__ unsigned s_last;
  if (threadIdx.x == 0) {
    prow[H] = (sred[0][0] + sred[1][0]) + (sred[2][0] + sred[3][0]);
    // the loss: per-workgroup partial as a write-through granule, a per-call ticket,
    // the last arriver sums the partials in a fixed order (deterministic).
    // cdna_hip_programming.md §6 G16 (granule stores + relaxed agent ticket).
    const float lp = (sred[0][1] + sred[1][1]) + (sred[2][1] + sred[3][1]);
    __hip_atomic_store(loss_part + blockIdx.x, lp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == gridDim.x - 1 ? 1u : 0u;
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!s_last) return;
  float t = 0.f;  // thread k sums partials k, k + 256, ...: every load in flight at once
  for (unsigned k = threadIdx.x; k < gridDim.x; k += 256)
    t += __hip_atomic_load(loss_part + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
  if (lane == 0) sred[wv][1] = t;
  __syncthreads();
  if (threadIdx.x == 0) loss[0] = ((sred[0][1] + sred[1][1]) + (sred[2][1] + sred[3][1])) * invB;
}

// sum the per-workgroup partials (fixed order) -> dW [H] and db; then either SGD on
// (w, bias) with lr * g, or write g * dW / g * db
__global__ __launch_bounds__(256) void ctr_head_finish_kernel(HeadFinishArgs a) {
  __shared__ float red[4][9];
  ctr_head_finish_body(a, blockIdx.x, red);
}

mrec_status build_head_finish(const float *part, int64_t ldp, int64_t batch, int32_t H,
                              int32_t ns, const float *g, int32_t update, float lr, float *w,
                              float *bias, float *ws, float *b2, float *dw_out, float *db_out,
                              float *dws_out, float *db2_out, HeadFinishArgs *out) {
  MREC_CHECK_ARG(part != nullptr && H >= 1 && batch >= 1 && ns >= 0 && ns <= 64, "bad arguments");
  MREC_CHECK_ARG(!update || (w && (ns == 0 || ws)), "update needs w (and ws)");
  MREC_CHECK_ARG(ldp >= H + 1 + ns, "ldp < H + 1 + ns");
  *out = HeadFinishArgs{part, ldp, static_cast<int>(mrec_ctr_head_parts(batch)), H, ns, g,
                        update, lr, w, bias, ws, b2, dw_out, db_out, dws_out, db2_out};
  return MREC_OK;
}

}  // namespace mrec

using namespace mrec;

extern "C" {

mrec_status mrec_head_fwd(const void *h, int64_t ldh, int64_t batch, int32_t H, const float *w,
                          const float *bias, const float *base, float *z, mrec_stream stream) {
  MREC_CHECK_ARG(h && w && z, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0 && H >= 1 && ldh >= H, "bad shape");
  MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(h) & 15) == 0 && ldh % 8 == 0,
                 "h rows must be 16-byte aligned");
  if (batch == 0) return MREC_OK;
  head_fwd_kernel<<<dim3(static_cast<unsigned>((batch + 3) / 4)), 256, 0,
                    static_cast<hipStream_t>(stream)>>>(static_cast<const uint16_t *>(h), ldh,
                                                        batch, H, w, bias, base, z);
  return launch_status("mrec_head_fwd");
}

mrec_status mrec_head_bwd(const float *dz, const float *w, int64_t batch, int32_t H,
                          const void *mask, int64_t ld_mask, void *dh, int64_t ldh,
                          mrec_stream stream) {
  MREC_CHECK_ARG(dz && w && dh, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0 && H >= 1 && ldh >= H && ldh % 8 == 0, "bad shape");
  MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(dh) & 15) == 0, "dh must be 16-byte aligned");
  MREC_CHECK_ARG(!mask || ((reinterpret_cast<uintptr_t>(mask) & 15) == 0 && ld_mask % 8 == 0 &&
                           ld_mask >= (H + 7) / 8 * 8),
                 "mask rows must be 16-byte aligned and cover round8(H) columns");
  if (batch == 0) return MREC_OK;
  const int64_t total = batch * (ldh / 8);
  const unsigned g = static_cast<unsigned>(std::min<int64_t>((total + 255) / 256, 4096));
  head_bwd_kernel<<<g, 256, 0, static_cast<hipStream_t>(stream)>>>(
      dz, w, batch, H, static_cast<const uint16_t *>(mask), ld_mask, static_cast<uint16_t *>(dh),
      ldh);
  return launch_status("mrec_head_bwd");
}

mrec_status mrec_bce_fwd(const float *z, const float *y, int64_t batch, float *loss,
                         mrec_stream stream) {
  MREC_CHECK_ARG(z && y && loss, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0, "bad shape");
  bce_fwd_kernel<<<1, 1024, 0, static_cast<hipStream_t>(stream)>>>(z, y, batch, loss);
  return launch_status("mrec_bce_fwd");
}

mrec_status mrec_bce_bwd(const float *z, const float *y, int64_t batch, const float *g, float *dz,
                         mrec_stream stream) {
  MREC_CHECK_ARG(z && y && dz, "NULL pointer");
  MREC_CHECK_ARG(batch >= 0, "bad shape");
  if (batch == 0) return MREC_OK;
  bce_bwd_kernel<<<dim3(static_cast<unsigned>((batch + 255) / 256)), 256, 0,
                   static_cast<hipStream_t>(stream)>>>(z, y, batch, g, dz);
  return launch_status("mrec_bce_bwd");
}

mrec_status mrec_colsum(const float *s, const void *X, mrec_dtype x_dtype, int64_t ldx,
                        int64_t batch, int64_t C, float *out, float *total, int32_t update,
                        float lr, mrec_stream stream) {
  MREC_CHECK_ARG(s != nullptr, "s is NULL");
  MREC_CHECK_ARG(C == 0 || (X && out), "X/out NULL");
  MREC_CHECK_ARG(x_dtype == MREC_F32 || x_dtype == MREC_BF16, "X must be f32 or bf16");
  MREC_CHECK_ARG(batch >= 0 && C >= 0 && (C == 0 || ldx >= C), "bad shape");
  if (C == 0 && !total) return MREC_OK;
  const int vec = x_dtype == MREC_BF16 && (reinterpret_cast<uintptr_t>(X) & 15) == 0 &&
                  ldx % 8 == 0;
  const unsigned blocks = static_cast<unsigned>((C + 7) / 8 + (total ? 1 : 0));
  colsum_kernel<<<dim3(blocks), CS_T, 0, static_cast<hipStream_t>(stream)>>>(
      s, X, x_dtype == MREC_BF16, vec, ldx, batch, C, out, total, update, lr);
  return launch_status("mrec_colsum");
}

int64_t mrec_ctr_head_parts(int64_t batch) { return (batch + HEAD_RPB - 1) / HEAD_RPB; }

mrec_status mrec_ctr_head_fwd(const void *h, int64_t ldh, int64_t batch, int32_t H, const float *w,
                              const float *bias, const float *base, const float *y,
                              const float *xs, int64_t ldxs, int32_t ns, const float *ws,
                              const float *b2, int32_t relu_mask, float *z, float *dz, void *dh,
                              int64_t lddh, float *part, int64_t ldp, float *loss_part,
                              uint32_t *ticket, float *loss, mrec_stream stream) {
  MREC_CHECK_ARG(h && w && y && z && dz && dh && part && loss_part && ticket && loss,
                 "NULL pointer");
  MREC_CHECK_ARG(batch >= 1 && H >= 1 && H <= HEAD_MAXH && ldh >= H && lddh >= H, "bad shape");
  MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(h) & 15) == 0 && ldh % 8 == 0 &&
                     (reinterpret_cast<uintptr_t>(dh) & 15) == 0 && lddh % 8 == 0,
                 "h / dh rows must be 16-byte aligned");
  MREC_CHECK_ARG(ns >= 0 && ns <= 64 && (ns == 0 || (xs && ws && ldxs >= ns)),
                 "side linear: 0 <= ns <= 64 with xs / ws");
  MREC_CHECK_ARG(ldp >= H + 1 + ns, "ldp < H + 1 + ns");
  const int64_t nb = mrec_ctr_head_parts(batch);
  const dim3 grid(static_cast<unsigned>(nb));
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (H <= 512)
    ctr_head_kernel<1><<<grid, 256, 0, st>>>(
        static_cast<const uint16_t *>(h), ldh, batch, H, w, bias, base, y, xs, ldxs, ns, ws, b2,
        relu_mask, z, dz, static_cast<uint16_t *>(dh), lddh, part, ldp, loss_part, ticket, loss);
  else
    ctr_head_kernel<2><<<grid, 256, 0, st>>>(
        static_cast<const uint16_t *>(h), ldh, batch, H, w, bias, base, y, xs, ldxs, ns, ws, b2,
        relu_mask, z, dz, static_cast<uint16_t *>(dh), lddh, part, ldp, loss_part, ticket, loss);
  return launch_status("mrec_ctr_head_fwd");
}

mrec_status mrec_ctr_head_finish(const float *part, int64_t ldp, int64_t batch, int32_t H,
                                 int32_t ns, const float *g, int32_t update, float lr, float *w,
                                 float *bias, float *ws, float *b2, float *dw_out, float *db_out,
                                 float *dws_out, float *db2_out, mrec_stream stream) {
  HeadFinishArgs a;
  mrec_status st = build_head_finish(part, ldp, batch, H, ns, g, update, lr, w, bias, ws, b2,
                                     dw_out, db_out, dws_out, db2_out, &a);
  if (st != MREC_OK) return st;
  ctr_head_finish_kernel<<<dim3(static_cast<unsigned>((H + 1 + ns + 7) / 8)), 256, 0,
                           static_cast<hipStream_t>(stream)>>>(a);
  return launch_status("mrec_ctr_head_finish");
}

}  // extern "C"
