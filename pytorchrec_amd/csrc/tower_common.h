// MFMA-fragment ("tower") images of an fp32 master weight W [N, K] (nn.Linear
// layout: N out features, K in features), shared by the fused MLP tower
// (tower.hip), the fused-SGD weight-gradient epilogue (gemm_common.h) and the
// data-parallel SGD (optim.hip), which re-emit the images after every update.
//
// The tower computes y^T = W x^T, so W is the A operand of
// v_mfma_f32_16x16x32_bf16 (lane l holds A[row = l % 16][k = 8 (l / 16) .. + 8]).
// One 16-row tile x 32-deep k step of A is one 1 KiB block laid out in lane
// order, so a wave fetches it with ONE fully coalesced global_load_dwordx4:
//
//   fwd image (y = x W^T):  tile t = n / 16 (ceil(N/16) tiles), step s = k / 32
//                            (ks = ceil(K/32) steps), block (t * ks + s);
//   bwd image (dx = dy W):   A = W^T, tile t = k / 16 (ceil(K/16) tiles), step
//                            s = n / 32 (ns = ceil(N/32) steps), block (t * ns + s).
//
// Entries outside [0, N) x [0, K) are zero: the images are zero-initialised once
// and every writer touches only real elements.
#pragma once
#include <stdint.h>

namespace mrec {

constexpr int kImgRowTr = 0;   // mrec_epilogue / mrec_sgd_job img_kind: row-major images
constexpr int kImgTower = 1;   // img_row / img_tr are the tower fwd / bwd images

__host__ __device__ __forceinline__ int64_t tower_img_elems_fwd(int64_t N, int64_t K) {
  return ((N + 15) / 16) * ((K + 31) / 32) * 512;
}
__host__ __device__ __forceinline__ int64_t tower_img_elems_bwd(int64_t N, int64_t K) {
  return ((K + 15) / 16) * ((N + 31) / 32) * 512;
}

// element W[n][k] in the fwd image (K = in features)
__host__ __device__ __forceinline__ int64_t tower_idx_fwd(int64_t n, int64_t k, int64_t K) {
  const int64_t ks = (K + 31) >> 5;
  const int64_t blk = (n >> 4) * ks + (k >> 5);
  const int64_t lane = (n & 15) + 16 * ((k & 31) >> 3);
  return (blk * 64 + lane) * 8 + (k & 7);
}

// element W[n][k] in the bwd image (N = out features)
__host__ __device__ __forceinline__ int64_t tower_idx_bwd(int64_t n, int64_t k, int64_t N) {
  const int64_t ns = (N + 31) >> 5;
  const int64_t blk = (k >> 4) * ns + (n >> 5);
  const int64_t lane = (k & 15) + 16 * ((n & 31) >> 3);
  return (blk * 64 + lane) * 8 + (n & 7);
}

// k-fragment image of an activation / gradient matrix X [B, C] (batch-major), the
// operand layout of the tower's weight-gradient kernel (tower_dw.hip): one 1 KiB
// block per 16 columns x 32 batch rows (tile t = c / 16, k step s = b / 32, block
// t * ceil(B/32) + s), lane l of the block = column 16 t + l % 16, rows
// 32 s + 8 (l / 16) .. + 8 -- v_mfma_f32_16x16x32_bf16 operand order for A (dY^T)
// and B (X) alike.  Rows past B and columns past C are zero.
__host__ __device__ __forceinline__ int64_t kfrag_elems(int64_t rows, int64_t cols) {
  return ((cols + 15) / 16) * ((rows + 31) / 32) * 512;
}
__host__ __device__ __forceinline__ int64_t kfrag_idx(int64_t b, int64_t c, int64_t nsteps) {
  return (((c >> 4) * nsteps + (b >> 5)) * 64 + (c & 15) + 16 * ((b & 31) >> 3)) * 8 + (b & 7);
}

__host__ __device__ __forceinline__ int tw_ceil(int a, int b) { return (a + b - 1) / b; }
// readable columns of an LDS activation block: whole k steps of 32
__host__ __device__ __forceinline__ int tw_cols(int w) { return tw_ceil(w, 32) * 32; }
// LDS row stride: the readable columns rounded up to 32 (mod 256) bytes, which makes
// the MFMA operand reads (ds_read_b128, lane l: row l % 16, 16 B at k 8 (l / 16))
// bank-conflict free
__host__ __device__ __forceinline__ int tw_stride(int w) {
  return tw_ceil(tw_cols(w) * 2 - 32, 256) * 256 + 32;
}

__device__ __forceinline__ bool bf16_pos(uint32_t h) { return h != 0u && !(h & 0x8000u); }

}  // namespace mrec
