// 16 -> 16 channel 3x3x3 Conv3d (KT = 3: KDLAE-S full-resolution encoder / decoder convs,
// KDLAE/KDLAE_model.py:386-393) and 3x3 Conv2d (KT = 1: the ASDQE extractors' second conv,
// ASDQE/ASDQE_model.py:131-142) + bias + ReLU as an LDS-tiled implicit GEMM for gfx950.
//
// With 16 output channels the generic implicit GEMM (gemm.hip) gets one MFMA per activation fragment
// it loads through L1 (27 taps re-read every input pixel from cache), which caps it near 40% of the
// MFMA rate.  Here a block stages its input halo once in LDS — 3 frames x (TR+2) rows x (TC+2) columns
// x 16 channels, 64 B per pixel — and each wave keeps all 27 weight fragments in VGPRs for the whole
// block, so the inner loop is one conflict-free ds_read_b128 (16 pixels x 64 B) per 4 MFMAs.
//
// MFMA roles as in gemm.hip: A = weights (rows = output channels), B = pixels; lane (li, lq) ends with
// pixel li, output channels 4 lq .. 4 lq + 3.  Products (r05): split-bf16 (mfma3.h) over pairs of taps,
// the k index 8 lq + j being input channel 4 lq + j of tap 2P (j < 4) or of tap 2P + 1 (j >= 4).
#include "kernels.h"
#include "lds_dma.h"
#include "mfma3.h"

namespace kdlae {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TR = 4;             // output rows per block (one per wave)
constexpr int TC = 64;            // output columns per block (4 pixel tiles of 16 per wave)
constexpr int HR = TR + 2, HC = TC + 2;
constexpr int HALO_PX = 3 * HR * HC;  // up to 1188 pixels x 16 channels = 74.25 KiB (KT = 3)

}  // namespace

template <int KT>
__global__ __launch_bounds__(256, 2) void conv3d_c16_kernel(Conv3dC16Params p) {
  constexpr int NPX = KT * HR * HC, NTAP = 9 * KT;
  __shared__ __attribute__((aligned(16))) f32x4 tile[HALO_PX * 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int tx_n = (p.W + TC - 1) / TC, ty_n = (p.H + TR - 1) / TR;
  int bid = blockIdx.x;
  const int txi = bid % tx_n;
  bid /= tx_n;
  const int tyi = bid % ty_n;
  bid /= ty_n;
  const int fr = bid % p.F;
  const int b = bid / p.F;
  const int x0 = txi * TC, y0 = tyi * TR;
  const long long fhw = (long long)p.H * p.W;
  const float* inb = p.in + (long long)b * p.F * fhw * p.ldi;

  // stage the halo: item i = (pixel, channel quad)
  dma::stage_batched<NPX * 4, 8>(tile, tid, [&](int i) -> f32x4 {
    const int q = i & 3, px = i >> 2;
    const int c = px % HC, r = (px / HC) % HR, f = px / (HC * HR);
    const int ff = fr + f - (KT == 3 ? 1 : 0), yy = y0 + r - 1, xx = x0 + c - 1;
    if ((unsigned)ff < (unsigned)p.F && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W)
      return *reinterpret_cast<const f32x4*>(inb + ((long long)ff * fhw + (long long)yy * p.W + xx) * p.ldi + 4 * q);
    return f32x4{0.f, 0.f, 0.f, 0.f};
  });
  // the 9 KT weight fragments (record g = tap of the fragment-order pack, NT = 1, Cin_pad = 16)
  f32x4 w[NTAP];
#pragma unroll
  for (int g = 0; g < NTAP; ++g) w[g] = *reinterpret_cast<const f32x4*>(p.wp + ((size_t)g * 64 + lane) * 4);
  const f32x4 bias = *reinterpret_cast<const f32x4*>(p.bias + 4 * lq);
  __syncthreads();

  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // taps in pairs (2P, 2P + 1; an odd last tap pairs with zeros): both operands split in registers,
  // six bf16 MFMAs per 16 x 16 x 32 block (mfma3.h)
#pragma unroll
  for (int P = 0; P < (NTAP + 1) / 2; ++P) {
    f32x4 xv[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int tap = 2 * P + h;
      const int df = tap / 9, dy = (tap / 3) % 3, dx = tap % 3;
      const f32x4* row = tile + ((df * HR + wave + dy) * HC + dx + li) * 4 + lq;
#pragma unroll
      for (int t = 0; t < 4; ++t) xv[h][t] = tap < NTAP ? row[t * 16 * 4] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const F3 wp = split3(w[2 * P], 2 * P + 1 < NTAP ? w[2 * P + 1] : f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = mfma6(wp, split3(xv[0][t], xv[1][t]), acc[t]);
  }

  const int y = y0 + wave;
  if (y >= p.H) return;
  float* outb = p.out + ((long long)b * p.F * fhw + (long long)fr * fhw + (long long)y * p.W) * p.ldo;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int x = x0 + t * 16 + li;
    if (x >= p.W) continue;
    f32x4 v = acc[t] + bias;
    if (p.relu) {
      v.x = fmaxf(v.x, 0.f);
      v.y = fmaxf(v.y, 0.f);
      v.z = fmaxf(v.z, 0.f);
      v.w = fmaxf(v.w, 0.f);
    }
    *reinterpret_cast<f32x4*>(outb + (long long)x * p.ldo + 4 * lq) = v;
  }
}

hipError_t launch_conv3d_c16(const Conv3dC16Params& p, hipStream_t s) {
  if (p.ldi % 4 || p.ldo % 4 || p.ldi < 16 || p.ldo < 16 || p.F <= 0 || p.H <= 0 || p.W <= 0 || p.Bn <= 0)
    return hipErrorInvalidValue;
  const long long blocks = (long long)p.Bn * p.F * ((p.H + TR - 1) / TR) * ((p.W + TC - 1) / TC);
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
  if (p.kt == 3) hipLaunchKernelGGL(conv3d_c16_kernel<3>, dim3((unsigned)blocks), dim3(256), 0, s, p);
  else if (p.kt == 1) hipLaunchKernelGGL(conv3d_c16_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, s, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace kdlae
