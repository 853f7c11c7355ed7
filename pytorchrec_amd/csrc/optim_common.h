// Dense-parameter SGD tiles over an all-reduced gradient buffer (optim.hip's
// mrec_sgd_multi launch; the same tiles ride in the row-sharded owner's embedding
// apply, mrec_emb_bwd_apply_wire_sgd).  Not part of the ABI.
#pragma once
#include "common.h"
#include "tower_common.h"

namespace mrec {

constexpr int kSgdMaxJobs = 16;
constexpr int kTile = 32;

struct SgdJobArgs {
  float *w;
  const float *g;
  uint16_t *img_row;
  uint16_t *img_tr;
  int64_t N, K, ldw, ldg, ld_row, ld_tr;
  float lr;
  int img_kind;  // kImgRowTr / kImgTower
  int tiles_k;  // 32-column tiles along K
  int first;    // first workgroup of this job
};

struct SgdArgs {
  SgdJobArgs job[kSgdMaxJobs];
  int n;
  int blocks;  // total tiles
};

// host: validate the jobs and fill *a (optim.hip)
mrec_status build_sgd_args(int32_t n, const mrec_sgd_job *jobs, SgdArgs *a);

// tile `blk` of the jobs in `a` (kernel arguments, or a device-resident copy): one
// 32x32 tile of one job per 256-thread workgroup: w -= lr * g, images from the new w
// (the transposed image goes through an LDS tile so both writes are coalesced)
__device__ __forceinline__ void sgd_tile(const SgdArgs &a, int blk) {
  __shared__ float tile[kTile][kTile + 1];
  int j = 0;
  while (j + 1 < a.n && blk >= a.job[j + 1].first) ++j;  // uniform
  const SgdJobArgs &J = a.job[j];
  const int t = blk - J.first;
  const int64_t n0 = static_cast<int64_t>(t / J.tiles_k) * kTile;
  const int64_t k0 = static_cast<int64_t>(t % J.tiles_k) * kTile;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int r = ty; r < kTile; r += 8) {
    const int64_t n = n0 + r, k = k0 + tx;
    float v = 0.f;
    if (n < J.N && k < J.K) {
      float *p = J.w + n * J.ldw + k;
      v = fmaf(-J.lr, J.g[n * J.ldg + k], *p);
      *p = v;
    }
    tile[r][tx] = v;
    if (J.img_kind == kImgTower) {  // the fused tower's fragment images (real elements)
      if (n < J.N && k < J.K) {
        const uint16_t h = f32_to_bf16_rne(v);
        if (J.img_row) J.img_row[tower_idx_fwd(n, k, J.K)] = h;
        if (J.img_tr) J.img_tr[tower_idx_bwd(n, k, J.N)] = h;
      }
      continue;
    }
    if (J.img_row && n < J.N && k < J.ld_row) J.img_row[n * J.ld_row + k] = f32_to_bf16_rne(v);
  }
  if (J.img_tr && J.img_kind != kImgTower) {  // uniform per workgroup
    __syncthreads();
    for (int r = ty; r < kTile; r += 8) {
      const int64_t k = k0 + r, n = n0 + tx;
      if (k < J.K && n < J.ld_tr) J.img_tr[k * J.ld_tr + n] = f32_to_bf16_rne(tile[tx][r]);
    }
  }
}

}  // namespace mrec
