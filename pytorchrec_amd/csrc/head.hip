// CTR head: output projection + logit sum, BCE-with-logits loss and gradient,
// and a deterministic scaled column sum (bias / small weight gradients).
//
// These replace ~15 tiny ATen launches per step (addmm(400->1), add, cast,
// binary_cross_entropy_with_logits fwd/bwd, mean, sum, a rocBLAS GEMV for the
// dense first-order weight gradient) with four kernels.
#include <algorithm>

#include "common.h"

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

// column sums: partial[r][c] = sum_{b in chunk r} s[b] * X[b, c]; chunk r of rows
constexpr int CS_COLS = 64, CS_ROWLANES = 4, CS_CHUNKS = 32;

__global__ __launch_bounds__(256) void colsum_partial_kernel(const float *__restrict__ s,
                                                             const void *__restrict__ X, int x_bf16,
                                                             int64_t ldx, int64_t B, int64_t C,
                                                             float *__restrict__ part,
                                                             int with_total) {
  __shared__ float red[CS_ROWLANES][CS_COLS + 1];
  const int cl = threadIdx.x % CS_COLS, rl = threadIdx.x / CS_COLS;
  const int64_t c = static_cast<int64_t>(blockIdx.x) * CS_COLS + cl;
  const int64_t rows_per = (B + CS_CHUNKS - 1) / CS_CHUNKS;
  const int64_t b0 = static_cast<int64_t>(blockIdx.y) * rows_per;
  const int64_t b1 = min(B, b0 + rows_per);
  const int64_t Ct = C + (with_total ? 1 : 0);  // column C = sum of s (the bias gradient)
  float acc = 0.f;
  if (c < Ct) {
    for (int64_t b = b0 + rl; b < b1; b += CS_ROWLANES) {
      float x = 1.f;
      if (c < C)
        x = x_bf16 ? bf16_to_f32(static_cast<const uint16_t *>(X)[b * ldx + c])
                   : static_cast<const float *>(X)[b * ldx + c];
      acc = fmaf(s[b], x, acc);
    }
  }
  red[rl][cl] = acc;
  __syncthreads();
  if (rl == 0 && c < Ct) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < CS_ROWLANES; ++k) t += red[k][cl];
    part[static_cast<int64_t>(blockIdx.y) * Ct + c] = t;
  }
}

__global__ __launch_bounds__(256) void colsum_final_kernel(const float *__restrict__ part,
                                                           int64_t C, int with_total,
                                                           float *__restrict__ out,
                                                           float *__restrict__ total) {
  const int64_t Ct = C + (with_total ? 1 : 0);
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (c >= Ct) return;
  float t = 0.f;
  for (int r = 0; r < CS_CHUNKS; ++r) t += part[r * Ct + c];
  if (c < C)
    out[c] = t;
  else
    total[0] = t;
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

size_t mrec_colsum_workspace_size(int64_t C) {
  return static_cast<size_t>(CS_CHUNKS) * static_cast<size_t>(C + 1) * 4;
}

mrec_status mrec_colsum(const float *s, const void *X, mrec_dtype x_dtype, int64_t ldx,
                        int64_t batch, int64_t C, float *out, float *total, void *workspace,
                        size_t ws_bytes, mrec_stream stream) {
  MREC_CHECK_ARG(s != nullptr, "s is NULL");
  MREC_CHECK_ARG(C == 0 || (X && out), "X/out NULL");
  MREC_CHECK_ARG(x_dtype == MREC_F32 || x_dtype == MREC_BF16, "X must be f32 or bf16");
  MREC_CHECK_ARG(batch >= 0 && C >= 0 && (C == 0 || ldx >= C), "bad shape");
  MREC_CHECK_ARG(workspace && ws_bytes >= mrec_colsum_workspace_size(C), "workspace too small");
  if (C == 0 && !total) return MREC_OK;
  const int wt = total ? 1 : 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  float *part = static_cast<float *>(workspace);
  const dim3 g1(static_cast<unsigned>((C + wt + CS_COLS - 1) / CS_COLS), CS_CHUNKS);
  colsum_partial_kernel<<<g1, 256, 0, st>>>(s, X, x_dtype == MREC_BF16, ldx, batch, C, part, wt);
  mrec_status r = launch_status("mrec_colsum(partial)");
  if (r != MREC_OK) return r;
  colsum_final_kernel<<<dim3(static_cast<unsigned>((C + wt + 255) / 256)), 256, 0, st>>>(
      part, C, wt, out, total);
  return launch_status("mrec_colsum(final)");
}

}  // extern "C"
