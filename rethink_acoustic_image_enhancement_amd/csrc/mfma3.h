// FP32 matrix products on the bf16 matrix cores of gfx950 (v_mfma_f32_16x16x32_bf16), exact-split form.
//
// gfx950 has no xf32/tf32 MFMA, and its f32 MFMA (v_mfma_f32_16x16x4_f32) runs at 1/16 of the bf16
// rate.  Every fp32 operand is therefore split exactly into three bf16 pieces (round to nearest even):
//     x = x_h + x_m + x_l,   x_h = bf16(x), x_m = bf16(x - x_h), x_l = bf16(x - x_h - x_m)
// (8 + 8 + 8 significand bits: the sum is x itself for every normal fp32 x down to ~2^-110).  A
// product is the sum of the nine piece products, each exact in the MFMA's fp32 accumulator; mfma6
// keeps the six with magnitude >= 2^-16 |a b| and drops a_m b_l, a_l b_m, a_l b_l, which are below
// 2^-23 |a b| together — the size of one fp32 rounding.  Measured against float64
// (profiles/r05a_bf16x6_probe.txt, tools/micro/bf16x6_probe.hip): over K = 96..1024 the split is as
// accurate as the f32 MFMA, which is an exact f32 fma chain (max error / sum|a b| 2.1e-7 vs 3.5e-7,
// rms 2^-25.6 vs 2^-25.1), because it rounds the accumulator 6 times per 32-deep k-group instead of
// 32 times.  Six bf16 MFMAs (16 cycles each) replace eight f32 ones (32 cycles each) per 16 x 16 x 32
// block: 2.67x the f32 MFMA throughput.
//
// Operand layout of v_mfma_f32_16x16x32_bf16: lane l holds A[row l & 15][k = 8 (l >> 4) + j] and
// B[k = 8 (l >> 4) + j][col l & 15], j = 0..7; C/D as the f32 16x16x4 form (col l & 15, row 4 (l >> 4)
// + e), so the accumulator tiles, epilogues and stores of the f32 kernels stay as they were.
//
// K order.  The f32 fragment order holds, per 16-deep k-group g and lane l, channels
// 16 g + 4 (l >> 4) + e (e < 4): exactly the float4 an activation lane loads.  A "pair" G covers k-groups
// 2G and 2G + 1, and its bf16 k index 8q + j (q = l >> 4) is channel 32G + 4q + j for j < 4 and
// 32G + 16 + 4q + (j - 4) for j >= 4: the B operand of a pair is split3(a[2G], a[2G + 1]) of the lane's
// own two float4, with no lane movement.  An odd last k-group pairs with zeros.  Weights are stored
// pre-split in "split fragment order": the record of (output tile t, pair G) is [3 planes h, m, l][64
// lanes] x 16 B (8 bf16) = 3 KiB, records tile-major ([t][G]), so a wave reads one plane as one
// contiguous 1 KiB.
#pragma once
#include <hip/hip_runtime.h>

namespace kdlae {

typedef float f32x4_3 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct F3 {  // the three bf16 planes of 8 fp32 values (12 VGPRs)
  bf16x8 h, m, l;
};

constexpr int kRec3 = 3 * 64;  // 16-byte slots per split record (3 KiB)

__device__ __forceinline__ void split1(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;  // exact
  m = (__bf16)r1;
  const float r2 = r1 - (float)m;  // exact, <= 8 significant bits
  l = (__bf16)r2;
}

__device__ __forceinline__ F3 split3(f32x4_3 lo, f32x4_3 hi) {
  F3 s;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    __bf16 h, m, l;
    split1(j < 4 ? lo[j] : hi[j - 4], h, m, l);
    s.h[j] = h;
    s.m[j] = m;
    s.l[j] = l;
  }
  return s;
}

__device__ __forceinline__ f32x4_3 mfma_bf(bf16x8 a, bf16x8 b, f32x4_3 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// acc += W . X over one 32-deep pair.  The term order is part of the numerics contract (every kernel
// that can produce a given output uses it): smaller terms first, grouped by W plane so a kernel can
// load one plane at a time — (l,h) (m,m) (m,h) (h,l) (h,m) (h,h).
__device__ __forceinline__ f32x4_3 mfma6(const F3& w, const F3& x, f32x4_3 c) {
  c = mfma_bf(w.l, x.h, c);
  c = mfma_bf(w.m, x.m, c);
  c = mfma_bf(w.m, x.h, c);
  c = mfma_bf(w.h, x.l, c);
  c = mfma_bf(w.h, x.m, c);
  c = mfma_bf(w.h, x.h, c);
  return c;
}

// mfma6 for two output tiles sharing the B operands of R row subtiles, the W planes read one at a
// time from LDS (w0 / w1 = the tiles' records + lane): 2 x 4 VGPRs of W live instead of 2 x 12
template <int R, bool T2, class T>
__device__ __forceinline__ void mfma6_pair(const T* w0, const T* w1, const F3 (&x)[R], f32x4_3 (&c0)[R],
                                           f32x4_3 (&c1)[R]) {
  bf16x8 p0 = __builtin_bit_cast(bf16x8, w0[128]);
  bf16x8 p1 = T2 ? __builtin_bit_cast(bf16x8, w1[128]) : p0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    c0[r] = mfma_bf(p0, x[r].h, c0[r]);
    if (T2) c1[r] = mfma_bf(p1, x[r].h, c1[r]);
  }
  p0 = __builtin_bit_cast(bf16x8, w0[64]);
  p1 = T2 ? __builtin_bit_cast(bf16x8, w1[64]) : p0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    c0[r] = mfma_bf(p0, x[r].m, c0[r]);
    if (T2) c1[r] = mfma_bf(p1, x[r].m, c1[r]);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    c0[r] = mfma_bf(p0, x[r].h, c0[r]);
    if (T2) c1[r] = mfma_bf(p1, x[r].h, c1[r]);
  }
  p0 = __builtin_bit_cast(bf16x8, w0[0]);
  p1 = T2 ? __builtin_bit_cast(bf16x8, w1[0]) : p0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    c0[r] = mfma_bf(p0, x[r].l, c0[r]);
    if (T2) c1[r] = mfma_bf(p1, x[r].l, c1[r]);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    c0[r] = mfma_bf(p0, x[r].m, c0[r]);
    if (T2) c1[r] = mfma_bf(p1, x[r].m, c1[r]);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    c0[r] = mfma_bf(p0, x[r].h, c0[r]);
    if (T2) c1[r] = mfma_bf(p1, x[r].h, c1[r]);
  }
}

// one split record (3 planes) of lane `lane` from LDS or global memory laid out as 16-byte slots
template <class T>
__device__ __forceinline__ F3 load_w3(const T* rec, int lane) {
  F3 w;
  w.h = __builtin_bit_cast(bf16x8, rec[lane]);
  w.m = __builtin_bit_cast(bf16x8, rec[64 + lane]);
  w.l = __builtin_bit_cast(bf16x8, rec[128 + lane]);
  return w;
}

// split records of an f32-fragment-order weight block [ntiles][kgroups][64][4]: (ntiles x ceil(kgroups/2))
// records of 3 KiB (pack.hip; also used by the per-image attention projection and the self tests)
hipError_t launch_split3(const float* src, float* dst, int ntiles, int kgroups, int nimg, long long src_img_stride,
                         long long dst_img_stride, hipStream_t s);
__host__ __device__ inline long long split3_floats(int ntiles, int kgroups) { return (long long)ntiles * ((kgroups + 1) / 2) * kRec3 * 4; }

}  // namespace kdlae
