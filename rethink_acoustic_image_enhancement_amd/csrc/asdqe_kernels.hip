// ASDQE-specific kernels (ASDQE/ASDQE_model.py): bilinear x2 upsample into a concat half, the
// deterministic global-average-pool and the fused regressor head.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace kdlae {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Up.up = nn.Upsample(scale_factor=2, mode='bilinear', align_corners=True) (ASDQE_model.py:53):
// src = dst * (in - 1) / (out - 1); weights and the (h0, w0)-major blend order follow aten's CPU
// upsample_bilinear2d.  One thread per (output pixel, 4 channels); float4 loads / stores.
__global__ __launch_bounds__(256) void upsample2x_kernel(const float* __restrict__ in, int ldi, float* __restrict__ out,
                                                         int ldo, int C, int N, int h, int w) {
  const int H2 = 2 * h, W2 = 2 * w, c4n = C >> 2;
  const float rh = H2 > 1 ? (float)(h - 1) / (float)(H2 - 1) : 0.f;
  const float rw = W2 > 1 ? (float)(w - 1) / (float)(W2 - 1) : 0.f;
  const long long total = (long long)N * H2 * W2 * c4n;
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    const int c = (int)(idx % c4n) * 4;
    long long r = idx / c4n;
    const int ox = (int)(r % W2);
    r /= W2;
    const int oy = (int)(r % H2);
    const long long n = r / H2;
    const float sy = rh * (float)oy, sx = rw * (float)ox;
    const int y0 = (int)sy, x0 = (int)sx;
    const int yp = y0 < h - 1 ? 1 : 0, xp = x0 < w - 1 ? 1 : 0;
    const float ly1 = sy - (float)y0, ly0 = 1.f - ly1;
    const float lx1 = sx - (float)x0, lx0 = 1.f - lx1;
    const float* base = in + ((n * h + y0) * w + x0) * (long long)ldi + c;
    const f32x4 a = *reinterpret_cast<const f32x4*>(base);
    const f32x4 b = *reinterpret_cast<const f32x4*>(base + xp * ldi);
    const f32x4 d = *reinterpret_cast<const f32x4*>(base + (long long)yp * w * ldi);
    const f32x4 e = *reinterpret_cast<const f32x4*>(base + ((long long)yp * w + xp) * ldi);
    const f32x4 v = ly0 * (lx0 * a + lx1 * b) + ly1 * (lx0 * d + lx1 * e);
    *reinterpret_cast<f32x4*>(out + ((n * H2 + oy) * W2 + ox) * (long long)ldo + c) = v;
  }
}

hipError_t launch_upsample2x(const float* in, int ldi, float* out, int ldo, int C, int N, int h, int w,
                             hipStream_t s) {
  if (C % 4 || ldi % 4 || ldo % 4) return hipErrorInvalidValue;
  const long long total = (long long)N * 4 * h * w * (C / 4);
  long long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(upsample2x_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, ldi, out, ldo, C, N, h, w);
  return hipGetLastError();
}

// AdaptiveAvgPool2d((1,1)) pass 1 (ASDQE_model.py:145).  Block (slot, b): thread = (channel quad,
// pixel lane); each lane sums a strided subset of the slot's pixel range, lanes are then combined
// in LDS in a fixed order — no atomics, bit-reproducible.
__global__ __launch_bounds__(256) void gap_partial_kernel(const float* __restrict__ in, int ld, int C, long long HW,
                                                          int slots, float* __restrict__ partial) {
  __shared__ f32x4 red[256];
  const int slot = blockIdx.x, b = blockIdx.y;
  const int c4n = C >> 2;
  const int lanes = 256 / c4n;
  const int cq = threadIdx.x % c4n, pl = threadIdx.x / c4n;
  const long long p0 = HW * slot / slots, p1 = HW * (slot + 1) / slots;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (pl < lanes) {
    const float* base = in + (long long)b * HW * ld + cq * 4;
    for (long long p = p0 + pl; p < p1; p += lanes) acc += *reinterpret_cast<const f32x4*>(base + p * ld);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x < c4n) {
    f32x4 t = red[threadIdx.x];
    for (int l = 1; l < lanes; ++l) t += red[l * c4n + threadIdx.x];
    *reinterpret_cast<f32x4*>(partial + ((long long)b * slots + slot) * C + threadIdx.x * 4) = t;
  }
}

hipError_t launch_gap_partial(const float* in, int ld, int C, int B, long long HW, int slots, float* partial,
                              hipStream_t s) {
  if (C % 4 || C > 1024 || ld % 4 || slots < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gap_partial_kernel, dim3(slots, B), dim3(256), 0, s, in, ld, C, HW, slots, partial);
  return hipGetLastError();
}

// Regressor (ASDQE_model.py:144-154) with outc (1x1 conv, :109) moved ahead of the pool — both are
// affine, so mean(outc(y)) == outc(mean(y)).  Dropout is the identity in eval mode.  One block per
// image; every dot product is a single thread's fixed-order loop.
__global__ __launch_bounds__(256) void asdqe_head_kernel(HeadParams p) {
  __shared__ float g[1024], f[1024], h1[1024], h2[1024];
  const int b = blockIdx.x;
  for (int c = threadIdx.x; c < p.C; c += 256) {
    float t = 0.f;
    for (int sl = 0; sl < p.slots; ++sl) t += p.partial[((long long)b * p.slots + sl) * p.C + c];
    g[c] = t * p.inv_hw;
  }
  __syncthreads();
  for (int o = threadIdx.x; o < p.M; o += 256) {
    float t = p.bo[o];
    for (int c = 0; c < p.C; ++c) t = fmaf(p.wo[o * p.C + c], g[c], t);
    f[o] = t;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < p.N1; j += 256) {
    float t = p.b1[j];
    for (int o = 0; o < p.M; ++o) t = fmaf(p.w1[j * p.M + o], f[o], t);
    h1[j] = fmaxf(t, 0.f);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < p.N2; k += 256) {
    float t = p.b2[k];
    for (int j = 0; j < p.N1; ++j) t = fmaf(p.w2[k * p.N1 + j], h1[j], t);
    h2[k] = fmaxf(t, 0.f);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = p.b3[0];
    for (int k = 0; k < p.N2; ++k) t = fmaf(p.w3[k], h2[k], t);
    p.score[b] = tanhf(t);
  }
}

hipError_t launch_asdqe_head(const HeadParams& p, hipStream_t s) {
  if (p.C > 1024 || p.M > 1024 || p.N1 > 1024 || p.N2 > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(asdqe_head_kernel, dim3(p.B), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace kdlae
