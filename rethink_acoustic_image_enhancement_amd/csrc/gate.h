// The GDFN gate (KDLAE/KDLAE_model.py:101-104): depthwise 3x3 of x1 and x2 + exact-erf GELU gate, one
// 16-hidden-channel chunk at a time from a chunk's halo image in LDS.  Shared by the fused GDFN tail
// (gdfn.hip) and the fused feed-forward half (ffn.hip), so the two compute the same bits.
#pragma once
#include <hip/hip_runtime.h>

namespace kdlae {
namespace gdfnc {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr bool kGeluPacked = true;  // packed-FP32 GELU gate in the C = 48 / 96 kernels
constexpr int kTile = 16;                          // output tile width (pixels)
constexpr int kHalo = kTile + 2;                   // 18 halo columns
constexpr int kDwF4 = 128;                         // per-chunk dw block: [9][8] weights, [8] bias, pad

// Exact-erf GELU, 0.5 x (1 + erf(x / sqrt 2)), with erf from Abramowitz & Stegun 7.1.26
// (|error| <= 1.5e-7): branch-free, so the gate VALU stays in one basic block with the MFMAs it is
// interleaved with.  The GELU error is <= 7.5e-8 |x|, at the level of fp32 rounding of the result.
__device__ __forceinline__ float gelu_erf_g(float x) {
#pragma clang fp contract(off)  // every fused multiply-add is written out: the same bits in every kernel
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float poly = fmaf(1.061405429f, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  poly *= t;
  const float e = fmaf(-poly, __expf(-z * z), 1.0f);  // erf(|x| / sqrt 2)
  return 0.5f * x * (1.0f + copysignf(e, x));
}

// The same GELU on a pair, written on float2 so hipcc emits packed FP32 (v_pk_fma/v_pk_mul: two
// lanes' worth of the polynomial per instruction); rcp and exp stay per value.  The operations and
// their order match gelu_erf_g.  Measured (profiles/r02_gdfn_gelu_packed_probe.txt): C96 -1.9%,
// C48 -1%, C192 +1.5% per launch, so the wide (NT = 12) kernel keeps the scalar form.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_gate2(f32x2 x, f32x2 v) {
#pragma clang fp contract(off)
  const f32x2 z = f32x2{fabsf(x.x), fabsf(x.y)} * 0.70710678118654752f;
  const f32x2 a = __builtin_elementwise_fma(f32x2{0.3275911f, 0.3275911f}, z, f32x2{1.0f, 1.0f});
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(a.x), __builtin_amdgcn_rcpf(a.y)};
  f32x2 poly = __builtin_elementwise_fma(f32x2{1.061405429f, 1.061405429f}, t, f32x2{-1.453152027f, -1.453152027f});
  poly = __builtin_elementwise_fma(poly, t, f32x2{1.421413741f, 1.421413741f});
  poly = __builtin_elementwise_fma(poly, t, f32x2{-0.284496736f, -0.284496736f});
  poly = __builtin_elementwise_fma(poly, t, f32x2{0.254829592f, 0.254829592f});
  poly *= t;
  const f32x2 nz2 = -z * z;
  const f32x2 ex = f32x2{__expf(nz2.x), __expf(nz2.y)};
  const f32x2 e = __builtin_elementwise_fma(-poly, ex, f32x2{1.0f, 1.0f});
  const f32x2 se = f32x2{copysignf(e.x, x.x), copysignf(e.y, x.y)};
  return ((0.5f * x) * (1.0f + se)) * v;
}

// gate of one 16-hidden-channel chunk for RPW tile rows (the GDFN stencil): depthwise 3x3 of x1 and x2
// (rows of the wave, column cx, channels 4q..4q+3 of each half) + exact-erf gate -> the float4 that IS
// the lane's MFMA B operand.  sl: the chunk's halo image (lane-linear [pixel][slot], slot = quad ^
// (column & 7), kHalo columns per row); dw: the chunk's dw block ([9][8] weights, [8] bias at +72);
// lo[h][j]: the lane's read offset of half h, column tap j in the wave's first halo row.  The
// unfused gate kernel (mdta.hip dwconv_gate) computes the same bits.
// LOWREG: a scheduling fence between the column taps, so at most one tap's halo reads are in flight
// (for callers with little register room left; the values are the same)
template <int RPW, bool PACKED, bool LOWREG = false>
__device__ __forceinline__ void gate_rows(const f32x4* sl, const f32x4* dw, const int (&lo)[2][3], int q,
                                          f32x4 (&gb)[RPW]) {
  f32x4 d[2][RPW];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const f32x4 bb = dw[72 + 4 * h + q];
#pragma unroll
    for (int r = 0; r < RPW; ++r) d[h][r] = bb;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      f32x4 wv[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) wv[i] = dw[(3 * i + j) * 8 + 4 * h + q];
#pragma unroll
      for (int rr = 0; rr < RPW + 2; ++rr) {
        const f32x4 v = (sl + lo[h][j])[rr * kHalo * 8];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int r = rr - i;
          if (r >= 0 && r < RPW) d[h][r] = __builtin_elementwise_fma(v, wv[i], d[h][r]);
        }
      }
      if constexpr (LOWREG) __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    if constexpr (PACKED) {
      const f32x2 lo2 = gelu_gate2(f32x2{d[0][r].x, d[0][r].y}, f32x2{d[1][r].x, d[1][r].y});
      const f32x2 hi2 = gelu_gate2(f32x2{d[0][r].z, d[0][r].w}, f32x2{d[1][r].z, d[1][r].w});
      gb[r] = f32x4{lo2.x, lo2.y, hi2.x, hi2.y};
    } else {
      gb[r].x = gelu_erf_g(d[0][r].x) * d[1][r].x;
      gb[r].y = gelu_erf_g(d[0][r].y) * d[1][r].y;
      gb[r].z = gelu_erf_g(d[0][r].z) * d[1][r].z;
      gb[r].w = gelu_erf_g(d[0][r].w) * d[1][r].w;
    }
  }
}


}  // namespace gdfnc
}  // namespace kdlae
