// Shared helpers for libmrec (gfx950 only).  Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "mrec.h"

namespace mrec {

// ---------------------------------------------------------------------------
// status / error reporting (thread-local last error, no exceptions cross ABI)
// ---------------------------------------------------------------------------
void set_error(const std::string &msg);

#define MREC_CHECK_ARG(cond, msg)                                                          \
  do {                                                                                     \
    if (!(cond)) {                                                                         \
      ::mrec::set_error(std::string(__func__) + ": " + (msg));                             \
      return MREC_EINVAL;                                                                  \
    }                                                                                      \
  } while (0)

mrec_status launch_status(const char *what);  // hipGetLastError -> status

// ---------------------------------------------------------------------------
// kernel argument blocks (passed by value; <= 4 KiB kernarg segment)
// ---------------------------------------------------------------------------
struct BankArgs {
  char *data;
  int64_t row_offset[MREC_MAX_TABLES];
  int64_t rows[MREC_MAX_TABLES];
  int32_t n_tables;
  int32_t dim;
  int32_t row_stride;  // elements
  int32_t has_w;
  int32_t lpr;  // lanes per row: row bytes / 16
};

struct IdsArgs {
  const void *ptr[MREC_MAX_TABLES];
  int64_t stride;
  int64_t chunk;         // 0: element b at b * stride
  int64_t chunk_stride;  // else at (b / chunk) * chunk_stride + b % chunk
  int32_t is64;
  int32_t pad_negative;
};

mrec_status make_bank_args(const mrec_table_bank *bank, BankArgs *out, int *elem_bytes,
                           int *lanes_per_row);
mrec_status make_ids_args(const mrec_ids *ids, int n_tables, IdsArgs *out);

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(static_cast<uint32_t>(h) << 16);
}

// round-to-nearest-even, NaN kept NaN (quiet bit set)
__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);
  return static_cast<uint16_t>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// stochastic rounding with 16 random bits (unbiased: E[result] = f)
__device__ __forceinline__ uint16_t f32_to_bf16_sr(float f, uint32_t rnd) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);
  return static_cast<uint16_t>((u + (rnd & 0xffffu)) >> 16);
}

__device__ __forceinline__ uint32_t hash3(uint64_t seed, uint64_t row, uint32_t col) {
  uint32_t x = static_cast<uint32_t>(seed) ^ static_cast<uint32_t>(seed >> 32) * 0x27d4eb2fu;
  x ^= static_cast<uint32_t>(row) * 0x9e3779b1u;
  x ^= static_cast<uint32_t>(row >> 32) * 0x85ebca77u;
  x ^= col * 0xc2b2ae3du;
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ int64_t load_id(const IdsArgs &ids, int f, int64_t b) {
  const int64_t off = ids.chunk ? (b / ids.chunk) * ids.chunk_stride + b % ids.chunk : b * ids.stride;
  if (ids.is64) return static_cast<const int64_t *>(ids.ptr[f])[off];
  return static_cast<int64_t>(static_cast<const int32_t *>(ids.ptr[f])[off]);
}

// 16 bytes of a row as floats: EPL = 8 (bf16) or 4 (f32)
template <typename T>
struct Vec;
template <>
struct Vec<uint16_t> {
  static constexpr int EPL = 8;
  __device__ __forceinline__ static void to_f32(const uint4 &r, float *v) {
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
};
template <>
struct Vec<float> {
  static constexpr int EPL = 4;
  __device__ __forceinline__ static void to_f32(const uint4 &r, float *v) {
    v[0] = __uint_as_float(r.x);
    v[1] = __uint_as_float(r.y);
    v[2] = __uint_as_float(r.z);
    v[3] = __uint_as_float(r.w);
  }
};

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return static_cast<uint32_t>(f32_to_bf16_rne(lo)) |
         (static_cast<uint32_t>(f32_to_bf16_rne(hi)) << 16);
}

}  // namespace mrec
