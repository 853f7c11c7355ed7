// DCN-v2 cross-network backward elementwise stage (absent
// from the reference; layer x_{l+1} = x0 * (x_l W^T + b) + x_l, z = x_l W^T + b).
// For layer l with upstream gradient g (all [M, d], bf16 rows):
//   dz          = g * x0                     -> operand of the dx_l and dW GEMMs
//   acc        += g * z   (fp32, [M, d])     -> the x0-multiplier part of dx0, summed
//                                               over the layers in one buffer
//   addend      = acc + g (bf16, optional)   -> layer 0 only: its dx_l GEMM adds it,
//                                               so that GEMM's output IS dx0
// One pass over g / x0 / z replaces ~8 torch elementwise kernels per layer and the
// autograd sums of x0's gradient.  Pad columns [d, round8(d)) of dz / acc / addend
// are written as zero (the GEMMs stage whole 16-byte rows).
#include <algorithm>

#include "common.h"

namespace mrec {

__device__ __forceinline__ void unpack8(const uint4 r, float *f) {
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(w[j] << 16);
    f[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float *v) {
  return make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                    pack_bf16x2(v[6], v[7]));
}

// one thread per 8 consecutive columns (16-byte loads / stores; rows are round8)
__global__ __launch_bounds__(256) void cross_bwd_prep_kernel(
    int64_t M, int64_t d, int64_t dp, const uint16_t *__restrict__ g, int64_t ldg,
    const uint16_t *__restrict__ x0, int64_t ldx0, const uint16_t *__restrict__ z, int64_t ldz,
    uint16_t *__restrict__ dz, int64_t lddz, float *__restrict__ acc, int64_t ldacc, int acc_init,
    uint16_t *__restrict__ addend, int64_t ldadd) {
  const int64_t q = dp / 8;
  const int64_t total = M * q;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t m = i / q, n = (i - m * q) * 8;
    float gv[8], xv[8], zv[8], a[8], o[8];
    unpack8(*reinterpret_cast<const uint4 *>(g + m * ldg + n), gv);
    unpack8(*reinterpret_cast<const uint4 *>(x0 + m * ldx0 + n), xv);
    unpack8(*reinterpret_cast<const uint4 *>(z + m * ldz + n), zv);
    float *ap = acc + m * ldacc + n;
    if (!acc_init) {
      const float4 a0 = *reinterpret_cast<const float4 *>(ap);
      const float4 a1 = *reinterpret_cast<const float4 *>(ap + 4);
      a[0] = a0.x; a[1] = a0.y; a[2] = a0.z; a[3] = a0.w;
      a[4] = a1.x; a[5] = a1.y; a[6] = a1.z; a[7] = a1.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool live = n + j < d;  // pad columns of the inputs may hold anything
      if (acc_init) a[j] = 0.f;
      a[j] = live ? fmaf(gv[j], zv[j], a[j]) : 0.f;
      o[j] = live ? gv[j] * xv[j] : 0.f;
    }
    *reinterpret_cast<uint4 *>(dz + m * lddz + n) = pack8(o);
    *reinterpret_cast<float4 *>(ap) = make_float4(a[0], a[1], a[2], a[3]);
    *reinterpret_cast<float4 *>(ap + 4) = make_float4(a[4], a[5], a[6], a[7]);
    if (addend) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = n + j < d ? a[j] + gv[j] : 0.f;
      *reinterpret_cast<uint4 *>(addend + m * ldadd + n) = pack8(o);
    }
  }
}

}  // namespace mrec

using namespace mrec;

extern "C" {

mrec_status mrec_dcn_cross_bwd_prep(int64_t M, int64_t d, const void *g, int64_t ldg,
                                    const void *x0, int64_t ldx0, const void *z, int64_t ldz,
                                    void *dz, int64_t lddz, float *acc, int64_t ldacc,
                                    int32_t acc_init, void *addend, int64_t ldadd,
                                    mrec_stream stream) {
  MREC_CHECK_ARG(M >= 0 && d >= 1, "bad shape");
  MREC_CHECK_ARG(g && x0 && z && dz && acc, "NULL pointer");
  const int64_t dp = (d + 7) / 8 * 8;
  MREC_CHECK_ARG(ldg >= dp && ldx0 >= dp && ldz >= dp && ldacc >= dp && lddz >= dp &&
                     (!addend || ldadd >= dp),
                 "rows need round8(d) columns");
  MREC_CHECK_ARG(ldg % 8 == 0 && ldx0 % 8 == 0 && ldz % 8 == 0 && lddz % 8 == 0 &&
                     ldacc % 4 == 0 && (!addend || ldadd % 8 == 0),
                 "row strides must keep 16-byte alignment");
  const uintptr_t al = reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(x0) |
                       reinterpret_cast<uintptr_t>(z) | reinterpret_cast<uintptr_t>(dz) |
                       reinterpret_cast<uintptr_t>(acc) | reinterpret_cast<uintptr_t>(addend);
  MREC_CHECK_ARG((al & 15) == 0, "pointers must be 16-byte aligned");
  if (M == 0) return MREC_OK;
  const int64_t blocks = std::min<int64_t>((M * (dp / 8) + 255) / 256, 8192);
  cross_bwd_prep_kernel<<<dim3(static_cast<unsigned>(blocks)), 256, 0,
                          static_cast<hipStream_t>(stream)>>>(
      M, d, dp, static_cast<const uint16_t *>(g), ldg, static_cast<const uint16_t *>(x0), ldx0,
      static_cast<const uint16_t *>(z), ldz, static_cast<uint16_t *>(dz), lddz, acc, ldacc,
      acc_init, static_cast<uint16_t *>(addend), ldadd);
  return launch_status("mrec_dcn_cross_bwd_prep");
}

}  // extern "C"
