// Dense-parameter SGD over an all-reduced gradient buffer, for data-parallel
// training: every parameter of the step in ONE launch, each weight's bf16 GEMM
// images re-emitted from the updated fp32 master in the same pass.
//
// Replaces torch.optim.SGD.step (reference: optimizers.py:7-11, called from
// IModel.train_step, IModel.py:122-124) + one mrec_weight_prep per layer.  On one
// process the SGD of these parameters is fused into their backward kernels
// instead; data parallelism must sum the gradients over ranks first.
#include <algorithm>
#include <cstring>

#include "optim_common.h"

namespace mrec {

template <bool KC>
__global__ __launch_bounds__(256) void sgd_multi_kernel(SgdArgs a, KClock kc) {
  KcScope<KC> kc_scope(kc);
  sgd_tile(a, static_cast<int>(blockIdx.x));
}

mrec_status build_sgd_args(int32_t n, const mrec_sgd_job *jobs, SgdArgs *out) {
  MREC_CHECK_ARG(n >= 0 && n <= kSgdMaxJobs, "n must be in [0, 16]");
  MREC_CHECK_ARG(n == 0 || jobs != nullptr, "jobs is NULL");
  SgdArgs &a = *out;
  a = SgdArgs{};
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
  a.blocks = total;
  return MREC_OK;
}

}  // namespace mrec

using namespace mrec;

extern "C" {

mrec_status mrec_sgd_multi(int32_t n, const mrec_sgd_job *jobs, mrec_stream stream) {
  SgdArgs a;
  if (mrec_status st = build_sgd_args(n, jobs, &a); st != MREC_OK) return st;
  if (a.blocks == 0) return MREC_OK;
  const KClock kc = kclock_take();
  if (kc.buf)
    sgd_multi_kernel<true><<<dim3(static_cast<unsigned>(a.blocks)), 256, 0,
                             static_cast<hipStream_t>(stream)>>>(a, kc);
  else
    sgd_multi_kernel<false><<<dim3(static_cast<unsigned>(a.blocks)), 256, 0,
                              static_cast<hipStream_t>(stream)>>>(a, kc);
  return launch_status("mrec_sgd_multi");
}

size_t mrec_sgd_table_bytes(void) { return sizeof(SgdArgs); }

mrec_status mrec_sgd_table_build(int32_t n, const mrec_sgd_job *jobs, void *out, size_t out_bytes,
                                 int32_t *blocks) {
  MREC_CHECK_ARG(out != nullptr && out_bytes >= sizeof(SgdArgs) && blocks != nullptr,
                 "out NULL or smaller than mrec_sgd_table_bytes()");
  SgdArgs a;
  if (mrec_status st = build_sgd_args(n, jobs, &a); st != MREC_OK) return st;
  std::memcpy(out, &a, sizeof(SgdArgs));
  *blocks = a.blocks;
  return MREC_OK;
}

}  // extern "C"
