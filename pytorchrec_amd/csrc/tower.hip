// Fused MLP tower + CTR head + BCE: forward and the input-gradient backward of the
// whole dense tower in ONE launch (include/mrec.h mrec_tower_fwd_bwd).
//
// Why one launch: at B = 4096 each 400-wide layer is ~1.4 GFLOP, i.e. well under a
// microsecond of MFMA work, but as its own GEMM launch it costs ~9 us (dispatch,
// the first k group's latency, the epilogue drain) and the activations make an
// HBM round trip.  Every row is independent until the weight gradients, so one
// workgroup owns 16 rows for the whole chain (fwd layers -> head + loss -> dx
// chain) and nothing but the weights crosses workgroups.
//
// Layout (one 512-thread workgroup = 8 waves, 16 rows):
//   * LDS holds the 16-row activation blocks: x0, h_1..h_L (kept for the ReLU
//     masks of the backward) and two gradient blocks (ping-pong), row-major bf16
//     with a row stride = 32 (mod 256) bytes, which makes the fragment reads
//     (ds_read_b128, lane l: row l % 16, 16 B at k 8 (l / 16)) bank-conflict free;
//   * the product is computed transposed, y^T = W x^T: the weight is MFMA operand
//     A and streams from L2 in fragment order (tower_common.h: one 1 KiB
//     global_load_dwordx4 per 16x32 block), the activation block is operand B,
//     read from LDS once per k step and shared by the wave's (<= 4) output tiles;
//   * lane l of the 16x16 accumulator holds y[row l % 16][4 (l / 16) .. + 4]:
//     the epilogue writes 8 contiguous bytes (ds_write_b64) per tile;
//   * PF k steps of weight fragments are in flight per wave (8 waves x 4 tiles x
//     PF x 1 KiB = 128 KiB per CU): the layer is bound by the CU's L2 read rate.
// Outputs (h_l, dh_l, dx0) leave LDS as coalesced 16-B row stores behind each
// layer, overlapped with the next layer's weight stream.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "tower_common.h"

namespace mrec {

constexpr int TW_ROWS = 16;
constexpr int TW_THREADS = 512;
constexpr int TW_WAVES = TW_THREADS / 64;
constexpr int TW_MAXL = 4;
constexpr int TW_MAXW = 512;
constexpr int TW_PF_DEFAULT = 8;         // k steps of weight fragments in flight per wave (r04: 8 over 4, -0.5 % step)
constexpr int TW_TPW = 4;                // output tiles per wave (<= 32 tiles = 512 wide)
constexpr int TW_MAXNS = 64;             // side-linear width
constexpr int TW_MAXC = 3;               // DCN-v2 cross layers ahead of the MLP (ABI 27)

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct TowerArgs {
  int64_t B;
  int L;
  int width[TW_MAXL + 1];
  const uint16_t *x0;
  int64_t ld_x0;
  const uint16_t *wf[TW_MAXL];
  const uint16_t *wb[TW_MAXL];
  int wf_bytes[TW_MAXL], wb_bytes[TW_MAXL];
  const float *bias[TW_MAXL];
  const float *head_w;
  const float *head_b;
  const float *base;
  const float *xs;
  int64_t ld_xs;
  int ns;
  const float *ws;
  const float *b2;
  const float *y;
  uint16_t *h_out[TW_MAXL];
  int64_t ld_h[TW_MAXL];
  uint16_t *dh_out[TW_MAXL];
  int64_t ld_dh[TW_MAXL];
  uint16_t *dx0;
  int64_t ld_dx0;
  float *z;
  float *dz;
  float *part;
  int64_t ldp;
  float *loss_part;
  unsigned *ticket;
  float *loss;
  float invB;
  // LDS plan (bytes): buffer offsets and row strides
  int off_x, s_x;
  int off_h[TW_MAXL], s_h[TW_MAXL];
  int off_g[2], s_g;
  int off_f;   // 2 x 16 floats: dz and loss per row
  int off_p;   // staged parameters (floats): biases, head_w, ws, b0, y, base, xs
  int p_bias[TW_MAXL], p_hw, p_ws, p_b0, p_y, p_base, p_xs, p_z, p_part;
  int lds_bytes;
  int rotate;  // per-workgroup k-step rotation (MREC_TOWER_ROT=0 disables)
  unsigned long long *stamps;  // diagnostics: [grid][16] wall-clock stamps (NULL: off)
  int store_mode;  // tower_store (MREC_TOWER_STORE)
  int kfrag;       // h_out / dh_out / x0_img are k-fragment images (tower_common.h)
  int nsteps;      // their k steps: ceil(B / 32)
  uint16_t *x0_img;
  int mode;        // MREC_TOWER_BCE / _FORWARD / _GIVEN_DZ
  const float *dz_in;
  // DCN-v2 cross network (ABI 27): C layers of width d = width[0] ahead of the MLP
  int C;
  const uint16_t *cwf[TW_MAXC];
  const uint16_t *cwb[TW_MAXC];
  const float *cbias[TW_MAXC];
  int cw_bytes;    // fwd and bwd images of a [d, d] weight have the same size
  uint16_t *cx_img[TW_MAXC];   // k-fragment images of x_1 .. x_C
  uint16_t *cdz_img[TW_MAXC];  // k-fragment images of dz_0 .. dz_{C-1}
  int off_xc[2];               // ping-pong x_c blocks (stride s_x); off_xc[0] is G in the backward
  int p_cbias[TW_MAXC];
};


typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// The MFMA main loop of one layer for a wave with NT real output tiles and G
// groups of PF k steps (both compile-time: the loop is straight-line code, so the
// compiler's vmcnt accounting keeps (PF - 1) * NT weight fragments in flight
// instead of draining at a loop header).  Weight fragments come in by buffer
// loads: voffset = the lane's slot of the tile, soffset = the k step
// (wave-uniform); a step past `ksteps` uses soffset = the image size, which the
// descriptor's range check turns into zeros (their MFMAs add nothing).  One
// sched_barrier per step keeps the refill loads right behind the step's MFMAs.
// Every workgroup streams the same weight image; starting each at its own k step
// (rot = blockIdx % ksteps, the steps taken cyclically) spreads the CUs of an XCD
// over the image's lines instead of having them all request the same L2 lines at
// once.  (A different fp32 summation order per workgroup; deterministic.)
__device__ __forceinline__ int tw_rot(int s, int rot, int ksteps) {
  if (s >= ksteps) return 0;  // padded step: the range check zeroes its weights (any finite B)
  const int r = s + rot;
  return r >= ksteps ? r - ksteps : r;
}

template <int NT, int G, int TW_PF>
__device__ __forceinline__ void tower_mfma_g(f32x4 (&acc)[TW_TPW], __amdgpu_buffer_rsrc_t rsrc,
                                             const int (&voff)[TW_TPW], int img_bytes,
                                             const char *brow, int ksteps, int rot) {
  bf16x8 wfr[TW_PF][NT];
#pragma unroll
  for (int p = 0; p < TW_PF; ++p) {
    const int so = p < ksteps ? tw_rot(p, rot, ksteps) * 1024 : img_bytes;
#pragma unroll
    for (int i = 0; i < NT; ++i)
      wfr[p][i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff[i], so, 0));
  }
#pragma unroll
  for (int s = 0; s < G * TW_PF; ++s) {
    const int p = s % TW_PF;
    const bf16x8 b = *reinterpret_cast<const bf16x8 *>(brow + tw_rot(s, rot, ksteps) * 64);
#pragma unroll
    for (int i = 0; i < NT; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[p][i], b, acc[i], 0, 0, 0);
    const int sn = s + TW_PF;
    if (sn < G * TW_PF) {  // compile-time
      const int so = sn < ksteps ? tw_rot(sn, rot, ksteps) * 1024 : img_bytes;
#pragma unroll
      for (int i = 0; i < NT; ++i)
        wfr[p][i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff[i], so, 0));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// dispatch on the number of PF-step groups (ksteps <= 16: widths <= 512)
template <int NT, int TW_PF, int G = 1>
__device__ __forceinline__ void tower_mfma(f32x4 (&acc)[TW_TPW], __amdgpu_buffer_rsrc_t rsrc,
                                           const int (&voff)[TW_TPW], int img_bytes,
                                           const char *brow, int ksteps, int rot) {
  if constexpr (G * TW_PF >= 16) {
    tower_mfma_g<NT, G, TW_PF>(acc, rsrc, voff, img_bytes, brow, ksteps, rot);
  } else {
    if (ksteps <= G * TW_PF)
      tower_mfma_g<NT, G, TW_PF>(acc, rsrc, voff, img_bytes, brow, ksteps, rot);
    else
      tower_mfma<NT, TW_PF, G + 1>(acc, rsrc, voff, img_bytes, brow, ksteps, rot);
  }
}

// One layer on the MFMA pipe: out[m][c] for the wave's output tiles c in
// [16 t, 16 t + 16), t = wave + 8 i, from `in` (LDS block, k steps of 32) and the
// A-operand image (tiles x ksteps blocks of 1 KiB).  Epilogue per element:
//   FWD: relu(acc + bias[c]) (c < width_out, else 0);
//   BWD: acc, times [mask[m][c] > 0] when mask != NULL.
// Tiles in [ntiles, 2 ceil(width_out / 32)) are written as zeros (the next
// layer reads whole k steps of 32).
// The MFMA phase of a layer: acc[i] = the wave's output tile t = wave + 8 i (lane l:
// rows 16 t + 4 (l / 16) .. + 4 of batch row l % 16).
template <int TW_PF>
__device__ __forceinline__ void tower_layer_acc(f32x4 (&acc)[TW_TPW], const uint16_t *__restrict__ img,
                                                int img_bytes, int ksteps, int ntiles, const char *in,
                                                int s_in, int rotate) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  int nreal = 0;
#pragma unroll
  for (int i = 0; i < TW_TPW; ++i) nreal += (wave + TW_WAVES * i < ntiles) ? 1 : 0;

  int voff[TW_TPW];  // byte offset of this lane's 16 B in step 0 of each tile
#pragma unroll
  for (int i = 0; i < TW_TPW; ++i) voff[i] = ((wave + TW_WAVES * i) * ksteps * 512 + lane * 8) * 2;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(img), 0, img_bytes, 0x00020000);

#pragma unroll
  for (int i = 0; i < TW_TPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const char *brow = in + r16 * s_in + g * 16;
  // rotate 1: blockIdx % ksteps; 2: (blockIdx / 8) % ksteps -- workgroups are dealt to the
  // 8 XCDs round-robin, so this spreads the 32 workgroups of one XCD (one L2) over all
  // k steps where mode 1 gives only ksteps / gcd(8, ksteps) distinct starts
  const unsigned bq = rotate == 2 ? blockIdx.x >> 3 : blockIdx.x;
  const int rot = rotate ? static_cast<int>(bq % static_cast<unsigned>(ksteps)) : 0;
  switch (nreal) {  // uniform per wave
    case 4: tower_mfma<4, TW_PF>(acc, rsrc, voff, img_bytes, brow, ksteps, rot); break;
    case 3: tower_mfma<3, TW_PF>(acc, rsrc, voff, img_bytes, brow, ksteps, rot); break;
    case 2: tower_mfma<2, TW_PF>(acc, rsrc, voff, img_bytes, brow, ksteps, rot); break;
    case 1: tower_mfma<1, TW_PF>(acc, rsrc, voff, img_bytes, brow, ksteps, rot); break;
    default: break;
  }
}

template <bool BWD, int TW_PF>
__device__ __forceinline__ void tower_layer(const uint16_t *__restrict__ img, int img_bytes,
                                            int ksteps, int width_out, const char *in, int s_in, char *out,
                                            int s_out, const float *__restrict__ bias,
                                            const char *mask, int s_mask, int rotate) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int ntiles = tw_ceil(width_out, 16);
  const int ztiles = 2 * tw_ceil(width_out, 32);
  f32x4 acc[TW_TPW];
  tower_layer_acc<TW_PF>(acc, img, img_bytes, ksteps, ntiles, in, s_in, rotate);

  // epilogue: lane holds rows c = 16 t + 4 g + r (r = 0..3) of column m = r16
#pragma unroll
  for (int i = 0; i < TW_TPW; ++i) {
    const int t = wave + TW_WAVES * i;
    if (t >= ztiles) break;  // uniform
    const int c0 = 16 * t + 4 * g;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (t < ntiles) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = c0 + r;
        float x = acc[i][r];
        if constexpr (!BWD) {
          x = c < width_out ? fmaxf(x + (bias ? bias[c] : 0.f), 0.f) : 0.f;
        }
        v[r] = x;
      }
      if (BWD && mask) {
        const uint2 mk = *reinterpret_cast<const uint2 *>(mask + r16 * s_mask + c0 * 2);
        if (!bf16_pos(mk.x & 0xffffu)) v[0] = 0.f;
        if (!bf16_pos(mk.x >> 16)) v[1] = 0.f;
        if (!bf16_pos(mk.y & 0xffffu)) v[2] = 0.f;
        if (!bf16_pos(mk.y >> 16)) v[3] = 0.f;
      }
    }
    *reinterpret_cast<uint2 *>(out + r16 * s_out + c0 * 2) =
        make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
  }
}

__device__ __forceinline__ void unpack_bf16x4(uint2 v, float (&f)[4]) {
  f[0] = __uint_as_float(v.x << 16);
  f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16);
  f[3] = __uint_as_float(v.y & 0xffff0000u);
}
__device__ __forceinline__ uint2 pack_bf16x4(const float (&f)[4]) {
  return make_uint2(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]));
}

// ---- DCN-v2 cross network inside the tower (ABI 27) -------------------------------
// Layer c: z_c = x_c Wc_c^T + b_c, x_{c+1} = x0 * z_c + x_c (d = width[0] wide, the
// x0 block stays in LDS).  The epilogue lane mapping is the same for the forward and
// the backward of a layer (d outputs both ways), so z_c stays in the lane's registers
// as bf16 (4 x 8 B per layer) from the forward to the backward instead of crossing
// HBM.  Rounding points as the layered path (mrec_gemm's mul / add / aux epilogue):
// z and x_{c+1} are bf16, x_{c+1} is computed from the fp32 z.
template <int TW_PF>
__device__ __forceinline__ void tower_cross_fwd(const uint16_t *__restrict__ img, int img_bytes, int d,
                                                const char *x0b, const char *in, int s_x, char *out,
                                                const float *bias, int rotate, uint2 (&zq)[TW_TPW]) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int ntiles = tw_ceil(d, 16), ztiles = 2 * tw_ceil(d, 32);
  f32x4 acc[TW_TPW];
  tower_layer_acc<TW_PF>(acc, img, img_bytes, tw_ceil(d, 32), ntiles, in, s_x, rotate);
#pragma unroll
  for (int i = 0; i < TW_TPW; ++i) {
    const int t = wave + TW_WAVES * i;
    zq[i] = make_uint2(0u, 0u);
    if (t >= ztiles) continue;  // uniform
    const int c0 = 16 * t + 4 * g;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (t < ntiles) {
      float x0f[4], xlf[4], z[4] = {0.f, 0.f, 0.f, 0.f};
      unpack_bf16x4(*reinterpret_cast<const uint2 *>(x0b + r16 * s_x + c0 * 2), x0f);
      unpack_bf16x4(*reinterpret_cast<const uint2 *>(in + r16 * s_x + c0 * 2), xlf);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (c0 + r < d) {
          z[r] = acc[i][r] + bias[c0 + r];
          v[r] = z[r] * x0f[r] + xlf[r];
        }
      }
      zq[i] = pack_bf16x4(z);
    }
    *reinterpret_cast<uint2 *>(out + r16 * s_x + c0 * 2) = pack_bf16x4(v);
  }
}

// The MLP's first layer backward when a cross network precedes it: acc = dx_C tile
// -> G block = bf16(dx_C) (the cross backward's running G), dz_{C-1} = bf16(G x0) ->
// dzo (the next MFMA operand).
template <int TW_PF>
__device__ __forceinline__ void tower_cross_handoff(const uint16_t *__restrict__ img, int img_bytes,
                                                    int ksteps, int d, const char *gin, int s_g,
                                                    const char *x0b, char *G, int s_x, char *dzo,
                                                    int rotate) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int ntiles = tw_ceil(d, 16), ztiles = 2 * tw_ceil(d, 32);
  f32x4 acc[TW_TPW];
  tower_layer_acc<TW_PF>(acc, img, img_bytes, ksteps, ntiles, gin, s_g, rotate);
#pragma unroll
  for (int i = 0; i < TW_TPW; ++i) {
    const int t = wave + TW_WAVES * i;
    if (t >= ztiles) continue;  // uniform
    const int c0 = 16 * t + 4 * g;
    uint2 gq = make_uint2(0u, 0u), dq = make_uint2(0u, 0u);
    if (t < ntiles) {
      float gv[4] = {acc[i][0], acc[i][1], acc[i][2], acc[i][3]}, x0f[4], gr[4], dz[4];
      gq = pack_bf16x4(gv);
      unpack_bf16x4(gq, gr);
      unpack_bf16x4(*reinterpret_cast<const uint2 *>(x0b + r16 * s_x + c0 * 2), x0f);
#pragma unroll
      for (int r = 0; r < 4; ++r) dz[r] = gr[r] * x0f[r];
      dq = pack_bf16x4(dz);
    }
    *reinterpret_cast<uint2 *>(G + r16 * s_x + c0 * 2) = gq;
    *reinterpret_cast<uint2 *>(dzo + r16 * s_g + c0 * 2) = dq;
  }
}

// Cross layer c backward, G_{c+1} in the G block, dz_c = G_{c+1} x0 in dzi:
//   G_c = dz_c Wc_c + G_{c+1},  dacc += G_{c+1} z_c (fp32, the x0-multiplier gradient);
// LAST (c = 0): G block = bf16(G_0 + dacc) = dx0; else G block = bf16(G_c) and
// dz_{c-1} = bf16(G_c x0) -> dzo.  Every lane reads and writes only its own G
// elements (the MFMA operand is dzi), so G is updated in place.
template <int TW_PF>
__device__ __forceinline__ void tower_cross_bwd(const uint16_t *__restrict__ img, int img_bytes, int d,
                                                const char *x0b, char *G, int s_x, const char *dzi,
                                                char *dzo, int s_g, int rotate, const uint2 (&zq)[TW_TPW],
                                                f32x4 (&dacc)[TW_TPW], bool last) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r16 = lane & 15;
  const int ntiles = tw_ceil(d, 16), ztiles = 2 * tw_ceil(d, 32);
  f32x4 acc[TW_TPW];
  tower_layer_acc<TW_PF>(acc, img, img_bytes, tw_ceil(d, 32), ntiles, dzi, s_g, rotate);
#pragma unroll
  for (int i = 0; i < TW_TPW; ++i) {
    const int t = wave + TW_WAVES * i;
    if (t >= ztiles) continue;  // uniform
    const int c0 = 16 * t + 4 * g;
    char *gp = G + r16 * s_x + c0 * 2;
    uint2 gq = make_uint2(0u, 0u), dq = make_uint2(0u, 0u);
    if (t < ntiles) {  // pad columns: G, z, x0 and the weights are zero there
      float go[4], zf[4], gn[4];
      unpack_bf16x4(*reinterpret_cast<const uint2 *>(gp), go);
      unpack_bf16x4(zq[i], zf);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gn[r] = acc[i][r] + go[r];
        dacc[i][r] = fmaf(go[r], zf[r], dacc[i][r]);
      }
      if (last) {
#pragma unroll
        for (int r = 0; r < 4; ++r) gn[r] += dacc[i][r];
        gq = pack_bf16x4(gn);
      } else {
        float x0f[4], gr[4], dz[4];
        gq = pack_bf16x4(gn);
        unpack_bf16x4(gq, gr);
        unpack_bf16x4(*reinterpret_cast<const uint2 *>(x0b + r16 * s_x + c0 * 2), x0f);
#pragma unroll
        for (int r = 0; r < 4; ++r) dz[r] = gr[r] * x0f[r];
        dq = pack_bf16x4(dz);
      }
    }
    *reinterpret_cast<uint2 *>(gp) = gq;
    if (!last) *reinterpret_cast<uint2 *>(dzo + r16 * s_g + c0 * 2) = dq;
  }
}

// rows [0, 16) of an LDS block -> global bf16 [B, ld], columns [0, round8(width)).
// store_mode 1 (default): sc1 write-through stores, which do not keep the line in
// the XCD's L2 (MI355X_MICROARCH.md, store flavours), so the ~2.5 MB of
// activation / gradient rows an XCD writes per launch do not evict the weight
// images every workgroup re-reads; 0: plain stores; 2: no stores (timing only).
__device__ __forceinline__ void tower_store(const char *blk, int s_blk, int width, uint16_t *dst,
                                            int64_t ld, int64_t row0, int64_t B, int store_mode) {
  if (!dst || store_mode == 2) return;
  const int chunks = tw_ceil(width, 8);
  const int rows = static_cast<int>(min<int64_t>(TW_ROWS, B - row0));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      dst + row0 * ld, 0, static_cast<int>(rows * ld * 2), 0x00020000);
  for (int i = threadIdx.x; i < TW_ROWS * chunks; i += TW_THREADS) {
    const int r = i / chunks, c = i - r * chunks;
    if (r < rows) {
      const u32x4 v = *reinterpret_cast<const u32x4 *>(blk + r * s_blk + c * 16);
      const int off = static_cast<int>((r * ld + c * 8) * 2);
      if (store_mode == 1)
        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, off, 0, 16);
      else
        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, off, 0, 0);
    }
  }
}

// rows [0, 16) of an LDS block -> the k-fragment image `img` of [B, width]
// (tower_common.h kfrag_idx): per 16-column tile the workgroup's half of the
// 32-row step is 32 lanes x 16 B = one contiguous 512-B piece.  Rows >= B are
// written as zeros; the last workgroup also zeroes the other half of its step when
// no workgroup owns it, so the image never holds stale rows (the weight-gradient
// kernel multiplies whole steps).
__device__ __forceinline__ void tower_store_kfrag(const char *blk, int s_blk, int width, uint16_t *img,
                                                  int nsteps, int64_t row0, int64_t B, int store_mode) {
  if (!img || store_mode == 2) return;
  const int ctiles = tw_ceil(width, 16);
  const int st = static_cast<int>(row0 >> 5), h = static_cast<int>((row0 >> 4) & 1);
  const int bytes = static_cast<int>(kfrag_elems(B, width) * 2);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(img, 0, bytes, 0x00020000);
  auto put = [&](u32x4 v, int off) {  // store_mode 1: write-through (see tower_store)
    if (store_mode == 1)
      __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, off, 0, 16);
    else
      __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, off, 0, 0);
  };
  // 16 lanes per (tile t, 8-row group gl): two ds_read_b64_tr_b16 give lane i the 8
  // rows of column 16 t + i (lane i addresses row 8 gl + i / 4 (+ 4), columns
  // 16 t + 4 (i % 4) .. + 4; rows 32 B apart mod 256: conflict free).  Every lane
  // of a wave runs the reads (EXEC all ones), idle ones on tile 0.
  const int n = ctiles * 32;
  const int i16 = threadIdx.x & 15;
  for (int base = 0; base < n; base += TW_THREADS) {
    const int idx = base + static_cast<int>(threadIdx.x);
    const bool on = idx < n;
    const int t = on ? idx >> 5 : 0, gl = (idx >> 4) & 1;
    const char *q = blk + (8 * gl + (i16 >> 2)) * s_blk + (t * 16 + 4 * (i16 & 3)) * 2;
    typedef short v4s_t __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;
    const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t *)(q));
    const v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t *)(q + 4 * s_blk));
    if (!on) continue;
    uint32_t w[4] = {static_cast<uint16_t>(lo[0]) | (uint32_t(static_cast<uint16_t>(lo[1])) << 16),
                     static_cast<uint16_t>(lo[2]) | (uint32_t(static_cast<uint16_t>(lo[3])) << 16),
                     static_cast<uint16_t>(hi[0]) | (uint32_t(static_cast<uint16_t>(hi[1])) << 16),
                     static_cast<uint16_t>(hi[2]) | (uint32_t(static_cast<uint16_t>(hi[3])) << 16)};
    const int64_t rlim = B - row0 - 8 * gl;  // rows of this group inside the batch
    if (rlim < 8) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e >= rlim) w[e >> 1] &= (e & 1) ? 0x0000ffffu : 0xffff0000u;
    }
    const int off = ((t * nsteps + st) * 64 + i16 + 16 * (2 * h + gl)) * 16;
    put(u32x4{w[0], w[1], w[2], w[3]}, off);
  }
  // the last workgroup zeroes the step's other half when no workgroup owns it
  if (h == 0 && row0 + TW_ROWS >= B) {
    for (int idx = threadIdx.x; idx < n; idx += TW_THREADS) {
      const int t = idx >> 5, j = idx & 31;
      const int off = ((t * nsteps + st) * 64 + 32 + j) * 16;
      put(u32x4{0u, 0u, 0u, 0u}, off);
    }
  }
}

// an activation / gradient block leaves in the launch's layout
__device__ __forceinline__ void tower_out(const TowerArgs &a, const char *blk, int s_blk, int width,
                                          uint16_t *dst, int64_t ld, int64_t row0) {
  if (a.kfrag)
    tower_store_kfrag(blk, s_blk, width, dst, a.nsteps, row0, a.B, a.store_mode);
  else
    tower_store(blk, s_blk, width, dst, ld, row0, a.B, a.store_mode);
}

// diagnostics: stamps go to LDS (a global store before a barrier would be waited
// for by it) and leave at the end of the workgroup
#define TW_STAMP(k)                                                                  \
  do {                                                                               \
    if (a.stamps && tid == 0) s_stamp[(k)] = wall_clock64();                         \
  } while (0)

template <int TW_PF, bool KC, bool CROSS>
__global__ __launch_bounds__(TW_THREADS) void tower_kernel(TowerArgs a, KClock kc) {
  KcScope<KC> kc_scope(kc);
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  __shared__ unsigned long long s_stamp[16];
  TW_STAMP(0);
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * TW_ROWS;
  const int L = a.L;

  // ---- prologue: x0 rows into registers, zero LDS, stage the small parameters,
  // then x0 into its block (the loads' latency overlaps the fills) ------------
  const int xchunks = tw_ceil(a.width[0], 8);
  uint4 xr[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int i = tid + q * TW_THREADS;
    const int r = i / xchunks, c = i - r * xchunks;
    xr[q] = (i < TW_ROWS * xchunks && row0 + r < a.B)
                ? *reinterpret_cast<const uint4 *>(a.x0 + (row0 + r) * a.ld_x0 + c * 8)
                : make_uint4(0u, 0u, 0u, 0u);
  }
  // the small parameters: every global load of this thread is issued before any
  // is consumed (one memory round trip; as store-after-load loops they were ~7
  // dependent trips, 4.8 us in the training step with x0 and the labels fresh
  // from the previous launch: tools/step_tower_stamps.py)
  const int H = a.width[L];
  float pb[TW_MAXL], phw, pws, pyb[2], pxs[2];
#pragma unroll
  for (int l = 0; l < TW_MAXL; ++l)  // widths <= 512 = TW_THREADS: one column per thread
    pb[l] = (l < L && tid < a.width[l + 1] && a.bias[l]) ? a.bias[l][tid] : 0.f;
  phw = tid < H ? a.head_w[tid] : 0.f;
  pws = tid < a.ns ? a.ws[tid] : 0.f;
  const bool yrow = tid < TW_ROWS && row0 + tid < a.B;
  const float *ysrc = a.mode == MREC_TOWER_GIVEN_DZ ? a.dz_in : a.y;  // p_y: labels or given dz
  pyb[0] = (yrow && ysrc) ? ysrc[row0 + tid] : 0.f;
  pyb[1] = (yrow && a.base) ? a.base[row0 + tid] : 0.f;
#pragma unroll
  for (int q = 0; q < 2; ++q) {  // TW_ROWS * ns <= 16 * 64 = 2 per thread
    const int i = tid + q * TW_THREADS;
    const int r = a.ns ? i / a.ns : 0, j = i - r * a.ns;
    pxs[q] = (i < TW_ROWS * a.ns && row0 + r < a.B) ? a.xs[(row0 + r) * a.ld_xs + j] : 0.f;
  }
  const float pb0 = tid == 0 ? (a.head_b ? a.head_b[0] : 0.f) + (a.b2 ? a.b2[0] : 0.f) : 0.f;
  float pcb[TW_MAXC];
  if constexpr (CROSS) {
#pragma unroll
    for (int c = 0; c < TW_MAXC; ++c)
      pcb[c] = (c < a.C && tid < a.width[0] && a.cbias[c]) ? a.cbias[c][tid] : 0.f;
  }
  for (int i = tid * 16; i < a.off_p; i += TW_THREADS * 16)
    *reinterpret_cast<uint4 *>(lds + i) = make_uint4(0u, 0u, 0u, 0u);
  float *prm = reinterpret_cast<float *>(lds + a.off_p);
#pragma unroll
  for (int l = 0; l < TW_MAXL; ++l)
    if (l < L && tid < a.width[l + 1]) prm[a.p_bias[l] + tid] = pb[l];
  if constexpr (CROSS) {
#pragma unroll
    for (int c = 0; c < TW_MAXC; ++c)
      if (c < a.C && tid < a.width[0]) prm[a.p_cbias[c] + tid] = pcb[c];
  }
  if (tid < (H + 7) / 8 * 8) prm[a.p_hw + tid] = phw;  // zero past H: whole chunks
  if (tid < a.ns) prm[a.p_ws + tid] = pws;
  if (tid == 0) prm[a.p_b0] = pb0;
  if (tid < TW_ROWS) {
    prm[a.p_y + tid] = pyb[0];
    prm[a.p_base + tid] = pyb[1];
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int i = tid + q * TW_THREADS;
    if (i < TW_ROWS * a.ns) prm[a.p_xs + i] = pxs[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int i = tid + q * TW_THREADS;
    const int r = i / xchunks, c = i - r * xchunks;
    if (i < TW_ROWS * xchunks)
      *reinterpret_cast<uint4 *>(lds + a.off_x + r * a.s_x + c * 16) = xr[q];
  }
  __syncthreads();
  TW_STAMP(1);

  // ---- cross network (CROSS): x_{c+1} = x0 * (x_c Wc_c^T + b_c) + x_c ------------
  // z_c as bf16 in a shift register of the lane's registers: pushed here, popped in
  // reverse layer order by the backward (compile-time indices, a runtime layer loop)
  uint2 zs[CROSS ? TW_MAXC : 1][TW_TPW];
#pragma unroll
  for (int k = 0; k < (CROSS ? TW_MAXC : 1); ++k)
#pragma unroll
    for (int i = 0; i < TW_TPW; ++i) zs[k][i] = make_uint2(0u, 0u);
  int off_in0 = a.off_x;
  if constexpr (CROSS) {
    const int d = a.width[0];
    for (int c = 0; c < a.C; ++c) {
      const char *in = lds + (c == 0 ? a.off_x : a.off_xc[(c - 1) & 1]);
      char *out = lds + a.off_xc[c & 1];
      uint2 zq[TW_TPW];
      tower_cross_fwd<TW_PF>(a.cwf[c], a.cw_bytes, d, lds + a.off_x, in, a.s_x, out,
                             prm + a.p_cbias[c], a.rotate, zq);
#pragma unroll
      for (int i = 0; i < TW_TPW; ++i) {
#pragma unroll
        for (int k = TW_MAXC - 1; k > 0; --k) zs[k][i] = zs[k - 1][i];
        zs[0][i] = zq[i];
      }
      __syncthreads();
      if (a.kfrag) {  // the cross weight gradients' X operands: x_0 = x0, x_{c+1}
        if (c == 0)
          tower_store_kfrag(lds + a.off_x, a.s_x, d, a.x0_img, a.nsteps, row0, a.B, a.store_mode);
        tower_store_kfrag(out, a.s_x, d, a.cx_img[c], a.nsteps, row0, a.B, a.store_mode);
      }
    }
    off_in0 = a.off_xc[(a.C - 1) & 1];
    TW_STAMP(15);  // diagnostics: the cross forward's end (the backward's is stamp 11)
  }

  // ---- forward: h_l = relu(h_{l-1} W_l^T + b_l) --------------------------------
  for (int l = 0; l < L; ++l) {
    const char *in = lds + (l == 0 ? off_in0 : a.off_h[l - 1]);
    const int s_in = l == 0 ? a.s_x : a.s_h[l - 1];
    tower_layer<false, TW_PF>(a.wf[l], a.wf_bytes[l], tw_ceil(a.width[l], 32), a.width[l + 1], in, s_in,
                       lds + a.off_h[l], a.s_h[l], prm + a.p_bias[l], nullptr, 0, a.rotate);
    __syncthreads();
    TW_STAMP(2 + l);
    // x0's k-fragment image leaves behind layer 1 (x0's block stays in LDS): issued
    // before it, its stores delayed the first weight fragments by ~1 us
    if (!CROSS && l == 0 && a.kfrag)
      tower_store_kfrag(lds + a.off_x, a.s_x, a.width[0], a.x0_img, a.nsteps, row0, a.B,
                        a.store_mode);
    if (l + 1 < L) tower_out(a, lds + a.off_h[l], a.s_h[l], a.width[l + 1], a.h_out[l], a.ld_h[l], row0);
  }

  // ---- head + BCE: thread (m = tid / 32, c = tid % 32), parameters from LDS ----
  // (results go to LDS first: a barrier behind global stores would wait for them)
  const char *hL = lds + a.off_h[L - 1];
  const int s_hL = a.s_h[L - 1];
  float *f_dz = reinterpret_cast<float *>(lds + a.off_f);
  float *f_loss = f_dz + TW_ROWS;
  float *f_z = prm + a.p_z;
  float *f_part = prm + a.p_part;
  const float *hw = prm + a.p_hw;
  {
    const int m = tid >> 5, c = tid & 31;
    const bool ok = row0 + m < a.B;
    float dot = 0.f;
    for (int j = c; j * 8 < H; j += 32) {  // hw is zero past H (whole chunks in LDS)
      const uint4 hv = *reinterpret_cast<const uint4 *>(hL + m * s_hL + j * 16);
      const float4 w0 = *reinterpret_cast<const float4 *>(hw + j * 8);
      const float4 w1 = *reinterpret_cast<const float4 *>(hw + j * 8 + 4);
      const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      float hf[8];
      Vec<uint16_t>::to_f32(hv, hf);
#pragma unroll
      for (int q = 0; q < 8; ++q) dot = fmaf(hf[q], wv[q], dot);
    }
    for (int j = c; j < a.ns; j += 32) dot = fmaf(prm[a.p_xs + m * a.ns + j], prm[a.p_ws + j], dot);
    // sum over the 32 lanes of row m (two 16-lane rows): DPP + one permlane swap
    dot = sum_quad(dot);
    dot += dpp_f32<0x124>(dot);  // row_ror:4
    dot += dpp_f32<0x128>(dot);  // row_ror:8
    dot = swap16_sum(dot);
    if (c == 0) {
      float d = 0.f, lo = 0.f, zz = 0.f;
      if (ok && a.mode == MREC_TOWER_GIVEN_DZ) {
        d = prm[a.p_y + m];
      } else if (ok) {
        zz = dot + prm[a.p_b0] + prm[a.p_base + m];
        const float yy = prm[a.p_y + m];
        d = (1.f / (1.f + __expf(-zz)) - yy) * a.invB;
        lo = fmaxf(zz, 0.f) - zz * yy + log1pf(__expf(-fabsf(zz)));
      }
      f_dz[m] = d;
      f_loss[m] = lo;
      f_z[m] = zz;
    }
  }
  __syncthreads();
  TW_STAMP(5);
  if (a.mode == MREC_TOWER_FORWARD) {  // the scores only
    if (tid < TW_ROWS && row0 + tid < a.B) a.z[row0 + tid] = f_z[tid];
    return;
  }
  // dh_L = dz * head_w * [h_L > 0] -> gradient block 0
  {
    char *g0 = lds + a.off_g[0];
    const int m = tid >> 5, c = tid & 31;
    const float d = f_dz[m];
    for (int j = c; j * 8 < H; j += 32) {
      const uint4 hv = *reinterpret_cast<const uint4 *>(hL + m * s_hL + j * 16);
      const uint32_t hwd[4] = {hv.x, hv.y, hv.z, hv.w};
      const float4 w0 = *reinterpret_cast<const float4 *>(hw + j * 8);
      const float4 w1 = *reinterpret_cast<const float4 *>(hw + j * 8 + 4);
      const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      float gv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint32_t hb = (q & 1) ? (hwd[q >> 1] >> 16) : (hwd[q >> 1] & 0xffffu);
        gv[q] = bf16_pos(hb) ? d * wv[q] : 0.f;  // pad columns: h = 0 and hw = 0
      }
      *reinterpret_cast<uint4 *>(g0 + m * a.s_g + j * 16) =
          make_uint4(pack_bf16x2(gv[0], gv[1]), pack_bf16x2(gv[2], gv[3]),
                     pack_bf16x2(gv[4], gv[5]), pack_bf16x2(gv[6], gv[7]));
    }
  }
  TW_STAMP(13);
  // head-parameter partials: [sum_m dz_m h_L[m] | sum dz | sum_m dz_m xs[m]]
  for (int c = tid; c < H + 1 + a.ns; c += TW_THREADS) {
    float sacc = 0.f;
    if (c < H) {
      float dzv[TW_ROWS];
#pragma unroll
      for (int m4 = 0; m4 < TW_ROWS; m4 += 4) {
        const float4 t = *reinterpret_cast<const float4 *>(f_dz + m4);
        dzv[m4] = t.x; dzv[m4 + 1] = t.y; dzv[m4 + 2] = t.z; dzv[m4 + 3] = t.w;
      }
#pragma unroll
      for (int m = 0; m < TW_ROWS; ++m)
        sacc = fmaf(dzv[m], bf16_to_f32(*reinterpret_cast<const uint16_t *>(hL + m * s_hL + c * 2)), sacc);
    } else if (c == H) {
      for (int m = 0; m < TW_ROWS; ++m) sacc += f_dz[m];
    } else {
      const int j = c - H - 1;
      for (int m = 0; m < TW_ROWS; ++m) sacc = fmaf(f_dz[m], prm[a.p_xs + m * a.ns + j], sacc);
    }
    f_part[c] = sacc;
  }
  TW_STAMP(14);
  __syncthreads();
  TW_STAMP(6);
  // now the global stores, behind the backward's first weight stream
  {
    float *prow = a.part + static_cast<int64_t>(blockIdx.x) * a.ldp;
    for (int c = tid; c < H + 1 + a.ns; c += TW_THREADS) prow[c] = f_part[c];
    if (tid < TW_ROWS && row0 + tid < a.B) {
      if (a.dz) a.dz[row0 + tid] = f_dz[tid];
      if (a.z && a.mode == MREC_TOWER_BCE) a.z[row0 + tid] = f_z[tid];
    }
  }
  tower_out(a, lds + a.off_g[0], a.s_g, H, a.dh_out[L - 1], a.ld_dh[L - 1], row0);

  // ---- backward: dh_{l-1} = (dh_l W_l) * [h_{l-1} > 0], dx0 = dh_1 W_1 ----------
  __shared__ unsigned s_last;
  int cur = 0;
  for (int l = L - 1; l >= 0; --l) {
    const char *gin = lds + a.off_g[cur];
    char *gout = lds + a.off_g[cur ^ 1];
    const char *mask = l > 0 ? lds + a.off_h[l - 1] : nullptr;
    const int s_mask = l > 0 ? a.s_h[l - 1] : 0;
    if (CROSS && l == 0)  // dx_C -> G (off_xc[0], free in the backward), dz_{C-1} -> gout
      tower_cross_handoff<TW_PF>(a.wb[0], a.wb_bytes[0], tw_ceil(a.width[1], 32), a.width[0], gin,
                                 a.s_g, lds + a.off_x, lds + a.off_xc[0], a.s_x, gout, a.rotate);
    else
      tower_layer<true, TW_PF>(a.wb[l], a.wb_bytes[l], tw_ceil(a.width[l + 1], 32), a.width[l], gin,
                               a.s_g, gout, a.s_g, nullptr, mask, s_mask, a.rotate);
    __syncthreads();
    TW_STAMP(7 + (L - 1 - l));
    if (l > 0) {
      tower_out(a, gout, a.s_g, a.width[l], a.dh_out[l - 1], a.ld_dh[l - 1], row0);
    } else if (CROSS) {
      if (tid == 0 && a.mode != MREC_TOWER_BCE) s_last = 0u;
      if (tid == 0 && a.mode == MREC_TOWER_BCE) {
        float lp = 0.f;
        for (int m = 0; m < TW_ROWS; ++m) lp += f_loss[m];
        __hip_atomic_store(a.loss_part + blockIdx.x, lp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == gridDim.x - 1 ? 1u : 0u;
      }
      if (a.kfrag)
        tower_store_kfrag(gout, a.s_g, a.width[0], a.cdz_img[a.C - 1], a.nsteps, row0, a.B,
                          a.store_mode);
    } else {
      // the loss: this workgroup's partial as a write-through granule + a relaxed
      // agent ticket (cdna_hip_programming.md §6 G16), before the dx0 stores so the
      // wait drains little; the last arriver sums the partials below
      if (tid == 0 && a.mode != MREC_TOWER_BCE) s_last = 0u;
      if (tid == 0 && a.mode == MREC_TOWER_BCE) {
        float lp = 0.f;
        for (int m = 0; m < TW_ROWS; ++m) lp += f_loss[m];
        __hip_atomic_store(a.loss_part + blockIdx.x, lp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == gridDim.x - 1 ? 1u : 0u;
      }
      tower_store(gout, a.s_g, a.width[0], a.dx0, a.ld_dx0, row0, a.B, a.store_mode);
    }
    cur ^= 1;
  }

  // ---- cross backward (CROSS): dz_c in off_g[cur], G_{c+1} in off_xc[0] ------------
  if constexpr (CROSS) {
    const int d = a.width[0];
    char *G = lds + a.off_xc[0];
    f32x4 dacc[TW_TPW];
#pragma unroll
    for (int i = 0; i < TW_TPW; ++i) dacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c = a.C - 1; c >= 0; --c) {
      uint2 zq[TW_TPW];
#pragma unroll
      for (int i = 0; i < TW_TPW; ++i) {  // pop z_c
        zq[i] = zs[0][i];
#pragma unroll
        for (int k = 0; k + 1 < TW_MAXC; ++k) zs[k][i] = zs[k + 1][i];
      }
      char *dzo = lds + a.off_g[cur ^ 1];
      tower_cross_bwd<TW_PF>(a.cwb[c], a.cw_bytes, d, lds + a.off_x, G, a.s_x, lds + a.off_g[cur],
                             dzo, a.s_g, a.rotate, zq, dacc, c == 0);
      __syncthreads();
      if (c > 0) {
        if (a.kfrag)
          tower_store_kfrag(dzo, a.s_g, d, a.cdz_img[c - 1], a.nsteps, row0, a.B, a.store_mode);
      } else {
        tower_store(G, a.s_x, d, a.dx0, a.ld_dx0, row0, a.B, a.store_mode);
      }
      cur ^= 1;
    }
  }

  // ---- the last ticket holder sums the loss partials (fixed order) ------------------
  TW_STAMP(11);
  __syncthreads();
  if (tid == 0 && s_last) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  TW_STAMP(12);
  if (a.stamps && tid < 16) a.stamps[blockIdx.x * 16 + tid] = s_stamp[tid];
  if (!s_last) return;
  float t = 0.f;
  for (unsigned k = tid; k < gridDim.x; k += TW_THREADS)
    t += __hip_atomic_load(a.loss_part + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
  float *wsum = f_loss;  // 8 waves (the per-row losses are no longer needed)
  __syncthreads();
  if (lane == 0) wsum[tid >> 6] = t;
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
    for (int w = 0; w < TW_WAVES; ++w) s += wsum[w];
    a.loss[0] = s * a.invB;
  }
}

// ---------------------------------------------------------------------------
// image prep: fp32 W [N, K] -> tower fwd / bwd images (real elements only)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void tower_prep_kernel(const float *__restrict__ W, int64_t N,
                                                         int64_t K, int64_t ldw,
                                                         uint16_t *__restrict__ pf,
                                                         uint16_t *__restrict__ pb) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= N * K) return;
  const int64_t n = i / K, k = i - n * K;
  const uint16_t h = f32_to_bf16_rne(W[n * ldw + k]);
  if (pf) pf[tower_idx_fwd(n, k, K)] = h;
  if (pb) pb[tower_idx_bwd(n, k, N)] = h;
}

static unsigned long long *g_tower_stamps = nullptr;  // mrec_tower_debug_stamps

unsigned long long *tower_debug_stamps() { return g_tower_stamps; }


static bool al16(const void *p, int64_t ld) {
  return p && (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 8 == 0;
}

}  // namespace mrec

using namespace mrec;

extern "C" {

// diagnostics (not in mrec.h): route per-workgroup phase stamps ([grid][16] uint64,
// 100 MHz wall clock) of the next tower launches to `buf` (NULL: off)
void mrec_tower_debug_stamps(void *buf) { g_tower_stamps = static_cast<unsigned long long *>(buf); }

int64_t mrec_tower_image_elems(int64_t N, int64_t K, int32_t bwd) {
  return bwd ? tower_img_elems_bwd(N, K) : tower_img_elems_fwd(N, K);
}

mrec_status mrec_tower_weight_prep(const float *W, int64_t N, int64_t K, int64_t ldw,
                                   void *img_fwd, void *img_bwd, mrec_stream stream) {
  MREC_CHECK_ARG(W && (img_fwd || img_bwd), "NULL pointer");
  MREC_CHECK_ARG(N >= 0 && K >= 0 && ldw >= K, "bad shape");
  if (N == 0 || K == 0) return MREC_OK;
  const int64_t n = N * K;
  tower_prep_kernel<<<dim3(static_cast<unsigned>((n + 255) / 256)), 256, 0,
                      static_cast<hipStream_t>(stream)>>>(W, N, K, ldw,
                                                          static_cast<uint16_t *>(img_fwd),
                                                          static_cast<uint16_t *>(img_bwd));
  return launch_status("mrec_tower_weight_prep");
}

mrec_status mrec_tower_fwd_bwd(const mrec_tower_args *p, mrec_stream stream) {
  MREC_CHECK_ARG(p != nullptr, "NULL args");
  const mrec_tower_args &s = *p;
  MREC_CHECK_ARG(s.batch >= 0, "negative batch");
  MREC_CHECK_ARG(s.n_layers >= 1 && s.n_layers <= TW_MAXL, "n_layers must be in [1, 4]");
  const int L = s.n_layers;
  for (int l = 0; l <= L; ++l)
    MREC_CHECK_ARG(s.width[l] >= 1 && s.width[l] <= TW_MAXW, "every width must be in [1, 512]");
  MREC_CHECK_ARG(al16(s.x0, s.ld_x0) && s.ld_x0 >= (s.width[0] + 7) / 8 * 8,
                 "x0 rows must be 16-B aligned with ld_x0 >= round8(width[0])");
  const bool kf = s.kfrag != 0;
  auto al = [](const void *q) { return q && (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const bool fwd_only = s.mode == MREC_TOWER_FORWARD;  // nothing but z is written
  for (int l = 0; l < L; ++l) {
    MREC_CHECK_ARG(s.w_fwd[l] && s.w_bwd[l], "NULL weight image");
    const int w = s.width[l + 1];
    if (fwd_only) continue;
    if (kf) {
      MREC_CHECK_ARG(al(s.dh_out[l]) && (l + 1 >= L || !s.h_out[l] || al(s.h_out[l])),
                     "k-fragment images must be 16-B aligned");
      continue;
    }
    MREC_CHECK_ARG(al16(s.dh_out[l], s.ld_dh[l]) && s.ld_dh[l] >= (w + 7) / 8 * 8,
                   "dh_out rows must be 16-B aligned with ld >= round8(width)");
    if (l + 1 < L && s.h_out[l])
      MREC_CHECK_ARG(al16(s.h_out[l], s.ld_h[l]) && s.ld_h[l] >= (w + 7) / 8 * 8,
                     "h_out rows must be 16-B aligned with ld >= round8(width)");
  }
  MREC_CHECK_ARG(!kf || !s.x0_img || al(s.x0_img), "x0_img must be 16-B aligned");
  MREC_CHECK_ARG(!kf || kfrag_elems(s.batch, TW_MAXW) * 2 < (int64_t(1) << 31),
                 "batch too large for k-fragment images");
  MREC_CHECK_ARG(fwd_only || !s.dx0 || (al16(s.dx0, s.ld_dx0) && s.ld_dx0 >= (s.width[0] + 7) / 8 * 8),
                 "dx0 rows must be 16-B aligned with ld >= round8(width[0])");
  MREC_CHECK_ARG(s.mode >= MREC_TOWER_BCE && s.mode <= MREC_TOWER_GIVEN_DZ, "bad mode");
  MREC_CHECK_ARG(s.head_w, "NULL head_w");
  if (s.mode == MREC_TOWER_BCE)
    MREC_CHECK_ARG(s.y && s.dz && s.part && s.loss_part && s.ticket && s.loss,
                   "NULL head / loss pointer");
  else if (s.mode == MREC_TOWER_FORWARD)
    MREC_CHECK_ARG(s.z, "MREC_TOWER_FORWARD needs z");
  else
    MREC_CHECK_ARG(s.dz_in && s.part, "MREC_TOWER_GIVEN_DZ needs dz_in and part");
  MREC_CHECK_ARG(s.ns >= 0 && s.ns <= TW_MAXNS && (s.ns == 0 || (s.xs && s.ws)),
                 "side linear: ns in [0, 64] with xs and ws");
  MREC_CHECK_ARG(s.ldp >= s.width[L] + 1 + s.ns, "ldp < N_L + 1 + ns");
  const int C = s.n_cross;
  MREC_CHECK_ARG(C >= 0 && C <= TW_MAXC, "n_cross must be in [0, 3]");
  for (int c = 0; c < C; ++c) {
    MREC_CHECK_ARG(s.cross_w_fwd[c] && s.cross_w_bwd[c], "NULL cross weight image");
    if (kf && !fwd_only)
      MREC_CHECK_ARG(al(s.cross_x_img[c]) && al(s.cross_dz_img[c]) && al(s.x0_img),
                     "cross layers with kfrag need x0_img, cross_x_img and cross_dz_img "
                     "(16-B aligned)");
  }
  if (s.batch == 0) return MREC_OK;

  TowerArgs a{};
  a.B = s.batch;
  a.L = L;
  for (int l = 0; l <= L; ++l) a.width[l] = s.width[l];
  a.x0 = static_cast<const uint16_t *>(s.x0);
  a.ld_x0 = s.ld_x0;
  int wmax = s.width[0];
  for (int l = 0; l < L; ++l) {
    a.wf[l] = static_cast<const uint16_t *>(s.w_fwd[l]);
    a.wb[l] = static_cast<const uint16_t *>(s.w_bwd[l]);
    a.wf_bytes[l] = static_cast<int>(tower_img_elems_fwd(s.width[l + 1], s.width[l]) * 2);
    a.wb_bytes[l] = static_cast<int>(tower_img_elems_bwd(s.width[l + 1], s.width[l]) * 2);
    a.bias[l] = s.bias[l];
    a.h_out[l] = static_cast<uint16_t *>(s.h_out[l]);
    a.ld_h[l] = s.ld_h[l];
    a.dh_out[l] = static_cast<uint16_t *>(s.dh_out[l]);
    a.ld_dh[l] = s.ld_dh[l];
    wmax = std::max(wmax, s.width[l + 1]);
  }
  a.head_w = s.head_w;
  a.head_b = s.head_b;
  a.base = s.base;
  a.xs = s.xs;
  a.ld_xs = s.ld_xs;
  a.ns = s.ns;
  a.ws = s.ws;
  a.b2 = s.b2;
  a.y = s.y;
  a.dx0 = static_cast<uint16_t *>(s.dx0);
  a.ld_dx0 = s.ld_dx0;
  a.z = s.z;
  a.dz = s.dz;
  a.part = s.part;
  a.ldp = s.ldp;
  a.loss_part = s.loss_part;
  a.ticket = s.ticket;
  a.loss = s.loss;
  a.invB = 1.f / static_cast<float>(s.batch);
  static const int rot_env = [] {  // MREC_TOWER_ROT: 0 off, 1 blockIdx, 2 per-XCD index
    const char *e = getenv("MREC_TOWER_ROT");
    return e ? atoi(e) : 1;
  }();
  a.rotate = rot_env;
  a.stamps = g_tower_stamps;
  static const int store_env = [] {
    const char *e = getenv("MREC_TOWER_STORE");
    return e ? atoi(e) : 1;
  }();
  a.store_mode = store_env;
  a.kfrag = kf ? 1 : 0;
  a.nsteps = static_cast<int>((s.batch + 31) / 32);
  a.x0_img = kf ? static_cast<uint16_t *>(s.x0_img) : nullptr;
  a.mode = s.mode;
  a.dz_in = s.dz_in;
  a.C = C;
  a.cw_bytes = static_cast<int>(tower_img_elems_fwd(s.width[0], s.width[0]) * 2);
  for (int c = 0; c < C; ++c) {
    a.cwf[c] = static_cast<const uint16_t *>(s.cross_w_fwd[c]);
    a.cwb[c] = static_cast<const uint16_t *>(s.cross_w_bwd[c]);
    a.cbias[c] = s.cross_bias[c];
    a.cx_img[c] = kf ? static_cast<uint16_t *>(s.cross_x_img[c]) : nullptr;
    a.cdz_img[c] = kf ? static_cast<uint16_t *>(s.cross_dz_img[c]) : nullptr;
  }
  if (a.mode == MREC_TOWER_FORWARD) {  // nothing leaves but z
    a.x0_img = nullptr;
    for (int l = 0; l < L; ++l) a.h_out[l] = nullptr;
    a.kfrag = 0;  // (the cross images)
  }
  int off = 0;
  a.off_x = off;
  a.s_x = tw_stride(s.width[0]);
  off += TW_ROWS * a.s_x;
  for (int q = 0; q < (C > 0 ? 2 : 0); ++q) {  // x_c ping-pong (G in the backward)
    a.off_xc[q] = off;
    off += TW_ROWS * a.s_x;
  }
  for (int l = 0; l < L; ++l) {
    a.off_h[l] = off;
    a.s_h[l] = tw_stride(s.width[l + 1]);
    off += TW_ROWS * a.s_h[l];
  }
  a.s_g = tw_stride(wmax);
  a.off_g[0] = off;
  off += TW_ROWS * a.s_g;
  a.off_g[1] = off;
  off += TW_ROWS * a.s_g;
  a.off_f = off;
  off += 2 * TW_ROWS * 4;
  off = (off + 15) / 16 * 16;
  a.off_p = off;  // everything before off_p is zero-filled by the kernel
  int np = 0;
  for (int l = 0; l < L; ++l) {
    a.p_bias[l] = np;
    np += (s.width[l + 1] + 3) / 4 * 4;  // segments 16-B aligned (float4 reads)
  }
  a.p_hw = np;
  np += (s.width[L] + 7) / 8 * 8;  // whole 8-column chunks, pad zero (the LDS fill)
  a.p_ws = np;
  np += (s.ns + 3) / 4 * 4;
  a.p_b0 = np;
  np += 1;
  a.p_y = np;
  np += TW_ROWS;
  a.p_base = np;
  np += TW_ROWS;
  a.p_xs = np;
  np += TW_ROWS * s.ns;
  a.p_z = np;
  np += TW_ROWS;
  a.p_part = np;
  np += s.width[L] + 1 + s.ns;
  for (int c = 0; c < C; ++c) {
    np = (np + 3) / 4 * 4;
    a.p_cbias[c] = np;
    np += s.width[0];
  }
  off += np * 4;
  a.lds_bytes = (off + 15) / 16 * 16;
  constexpr int kMaxDyn = 160 * 1024 - 256;  // the kernel's static LDS (s_last) is on top
  MREC_CHECK_ARG(a.lds_bytes <= kMaxDyn, "activation blocks exceed the 160 KiB LDS");
  static int attr_set = [] {
    for (const void *k : {reinterpret_cast<const void *>(tower_kernel<4, false, false>),
                          reinterpret_cast<const void *>(tower_kernel<6, false, false>),
                          reinterpret_cast<const void *>(tower_kernel<8, false, false>),
                          reinterpret_cast<const void *>(tower_kernel<TW_PF_DEFAULT, true, false>),
                          reinterpret_cast<const void *>(tower_kernel<TW_PF_DEFAULT, false, true>),
                          reinterpret_cast<const void *>(tower_kernel<TW_PF_DEFAULT, true, true>)})
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxDyn);
    (void)hipGetLastError();  // a refused attribute must not read as a failed launch
    return 1;
  }();
  (void)attr_set;
  static const int pf_env = [] {  // MREC_TOWER_PF: weight k steps in flight per wave
    const char *e = getenv("MREC_TOWER_PF");
    const int v = e ? atoi(e) : TW_PF_DEFAULT;
    return (v == 4 || v == 6) ? v : 8;
  }();
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t grid = (s.batch + TW_ROWS - 1) / TW_ROWS;
  const dim3 gd(static_cast<unsigned>(grid));
  const KClock kc = kclock_take();
  if (C > 0) {  // the cross network runs at the default prefetch depth
    if (kc.buf)
      tower_kernel<TW_PF_DEFAULT, true, true><<<gd, TW_THREADS, a.lds_bytes, st>>>(a, kc);
    else
      tower_kernel<TW_PF_DEFAULT, false, true><<<gd, TW_THREADS, a.lds_bytes, st>>>(a, kc);
  } else if (kc.buf) {  // (the clocked instantiation is the default prefetch depth's)
    tower_kernel<TW_PF_DEFAULT, true, false><<<gd, TW_THREADS, a.lds_bytes, st>>>(a, kc);
  } else if (pf_env == 8) {
    tower_kernel<8, false, false><<<gd, TW_THREADS, a.lds_bytes, st>>>(a, kc);
  } else if (pf_env == 6) {
    tower_kernel<6, false, false><<<gd, TW_THREADS, a.lds_bytes, st>>>(a, kc);
  } else {
    tower_kernel<4, false, false><<<gd, TW_THREADS, a.lds_bytes, st>>>(a, kc);
  }
  return launch_status("mrec_tower_fwd_bwd");
}

}  // extern "C"
