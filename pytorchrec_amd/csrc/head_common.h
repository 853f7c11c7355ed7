// The CTR head's parameter-gradient finish (fixed-order sum of the per-workgroup
// partials + SGD), shared by its own kernel (head.hip) and the GEMM launch that
// runs it beside the first backward GEMMs (gemm.hip, mrec_gemm_multi_ex).
#pragma once
#include "common.h"

namespace mrec {

struct HeadFinishArgs {
  const float *part;
  int64_t ldp;
  int nparts, H, ns;
  const float *gp;  // upstream gradient of the loss (NULL = 1)
  int update;
  float lr;
  float *w, *bias, *ws, *b2;
  float *dw_out, *db_out, *dws_out, *db2_out;
};

__device__ __forceinline__ int head_finish_blocks(int H, int ns) { return (H + 1 + ns + 7) / 8; }

// workgroup `bid` (T = 256 or 64 threads) finishes columns [8 bid, 8 bid + 8) of
// [w | bias | ws]; the same fixed summation order for either T (the 4 waves' lanes
// of the 256-thread form are the 64-thread form's 4 strides)
template <int T = 256>
__device__ __forceinline__ void ctr_head_finish_body(const HeadFinishArgs &a, int bid,
                                                     float (*red)[9]) {
  const int H = a.H, ns = a.ns;
  const int c0 = bid * 8;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if constexpr (T == 64) {
    for (int w = 0; w < 4; ++w) {  // the 4 "waves" of the 256-thread order, one after another
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int k = w * 64 + lane; k < a.nparts; k += 256) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (c0 + j <= H + ns) acc[j] += a.part[static_cast<int64_t>(k) * a.ldp + c0 + j];
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
    }
    __syncthreads();
  } else {
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int k = threadIdx.x; k < a.nparts; k += 256) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (c0 + j <= H + ns) acc[j] += a.part[static_cast<int64_t>(k) * a.ldp + c0 + j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc[j] += __shfl_xor(acc[j], off);
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wv][j] = acc[j];
  }
  __syncthreads();
  }
  if (threadIdx.x < 8) {
    const int c = c0 + threadIdx.x;
    if (c > H + ns) return;
    const float g = a.gp ? a.gp[0] : 1.f;
    const float v = ((red[0][threadIdx.x] + red[1][threadIdx.x]) +
                     (red[2][threadIdx.x] + red[3][threadIdx.x])) * g;
    if (c < H) {
      if (a.update)
        a.w[c] = fmaf(-a.lr, v, a.w[c]);
      else if (a.dw_out)
        a.dw_out[c] = v;
    } else if (c == H) {  // both biases have gradient sum(dz)
      if (a.update) {
        if (a.bias) a.bias[0] = fmaf(-a.lr, v, a.bias[0]);
        if (a.b2) a.b2[0] = fmaf(-a.lr, v, a.b2[0]);
      } else {
        if (a.db_out) a.db_out[0] = v;
        if (a.db2_out) a.db2_out[0] = v;
      }
    } else {
      const int j = c - H - 1;
      if (a.update)
        a.ws[j] = fmaf(-a.lr, v, a.ws[j]);
      else if (a.dws_out)
        a.dws_out[j] = v;
    }
  }
}

// host: validate and fill (head.hip)
mrec_status build_head_finish(const float *part, int64_t ldp, int64_t batch, int32_t H,
                              int32_t ns, const float *g, int32_t update, float lr, float *w,
                              float *bias, float *ws, float *b2, float *dw_out, float *db_out,
                              float *dws_out, float *db2_out, HeadFinishArgs *out);

}  // namespace mrec
