// Dense-parameter SGD over an all-reduced gradient buffer, for data-parallel
// training: every parameter of the step in ONE launch, each weight's bf16 GEMM
// images re-emitted from the updated fp32 master in the same pass.
//
// Replaces torch.optim.SGD.step (reference: optimizers.py:7-11, called from
// IModel.train_step, IModel.py:122-124) + one mrec_weight_prep per layer.  On one
// process the SGD of these parameters is fused into their backward kernels
// instead; data parallelism must sum the gradients over ranks first.
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
};

// one 32x32 tile of one job per workgroup: w -= lr * g, images from the new w
// (the transposed image goes through an LDS tile so both writes are coalesced)
template <bool KC>
__global__ __launch_bounds__(256) void sgd_multi_kernel(SgdArgs a, KClock kc) {
  KcScope<KC> kc_scope(kc);
  __shared__ float tile[kTile][kTile + 1];
  int j = 0;
  while (j + 1 < a.n && static_cast<int>(blockIdx.x) >= a.job[j + 1].first) ++j;  // uniform
  const SgdJobArgs &J = a.job[j];
  const int t = static_cast<int>(blockIdx.x) - J.first;
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

using namespace mrec;

extern "C" {

mrec_status mrec_sgd_multi(int32_t n, const mrec_sgd_job *jobs, mrec_stream stream) {
  MREC_CHECK_ARG(n >= 0 && n <= kSgdMaxJobs, "n must be in [0, 16]");
  MREC_CHECK_ARG(n == 0 || jobs != nullptr, "jobs is NULL");
  SgdArgs a{};
  int total = 0;
  for (int i = 0; i < n; ++i) {
    const mrec_sgd_job &s = jobs[i];
    MREC_CHECK_ARG(s.w != nullptr && s.g != nullptr, "w or g is NULL");
    MREC_CHECK_ARG(s.N >= 0 && s.K >= 0 && s.ldw >= s.K && s.ldg >= s.K, "bad shape / ld");
    MREC_CHECK_ARG(s.img_kind == kImgRowTr || s.img_kind == kImgTower, "bad img_kind");
    const bool packed = s.img_kind == kImgTower;
    MREC_CHECK_ARG(packed || s.img_row == nullptr || s.ld_row >= s.K, "ld_row < K");
    MREC_CHECK_ARG(packed || s.img_tr == nullptr || s.ld_tr >= s.N, "ld_tr < N");
    SgdJobArgs &J = a.job[a.n];
    J.w = s.w;
    J.g = s.g;
    J.img_row = static_cast<uint16_t *>(s.img_row);
    J.img_tr = static_cast<uint16_t *>(s.img_tr);
    J.N = s.N;
    J.K = s.K;
    J.ldw = s.ldw;
    J.ldg = s.ldg;
    J.ld_row = s.ld_row;
    J.ld_tr = s.ld_tr;
    J.lr = s.lr;
    J.img_kind = s.img_kind;
    // the row-major images' pad columns (up to ld) are written as zero by the edge
    // tiles; tower images keep their (zero) pad entries untouched
    const int64_t kc = packed ? s.K : std::max<int64_t>(s.K, s.img_row ? s.ld_row : 0);
    const int64_t nc = packed ? s.N : std::max<int64_t>(s.N, s.img_tr ? s.ld_tr : 0);
    if (s.N == 0 || s.K == 0) continue;
    J.tiles_k = static_cast<int>((kc + kTile - 1) / kTile);
    const int64_t tiles = ((nc + kTile - 1) / kTile) * J.tiles_k;
    MREC_CHECK_ARG(total + tiles < (1 << 30), "too many tiles");
    J.first = total;
    total += static_cast<int>(tiles);
    ++a.n;
  }
  if (total == 0) return MREC_OK;
  const KClock kc = kclock_take();
  if (kc.buf)
    sgd_multi_kernel<true><<<dim3(static_cast<unsigned>(total)), 256, 0,
                             static_cast<hipStream_t>(stream)>>>(a, kc);
  else
    sgd_multi_kernel<false><<<dim3(static_cast<unsigned>(total)), 256, 0,
                              static_cast<hipStream_t>(stream)>>>(a, kc);
  return launch_status("mrec_sgd_multi");
}

}  // extern "C"
