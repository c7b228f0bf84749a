// FP32 products from bf16 MFMAs (v_mfma_f32_16x16x32_bf16) by an exact 3-way split:
//   x = x_hi + x_mid + x_lo, every piece a bf16 (RNE), so x is represented exactly (8 + 8 + 8 bits);
//   a.b = sum of the 9 piece products; "x6" keeps the 6 with magnitude >= 2^-16 |a||b| and drops
//   a_mid b_lo, a_lo b_mid, a_lo b_lo (<= 2^-23 |a||b| together, one fp32 rounding's size).
// Part 1: accuracy of 16x16 output tiles over K vs a float64 host reference, for the f32 MFMA
//         (exact f32 fma chain), the split with 3 / 6 / 9 products, and the host's sequential fp32 fma.
// Part 2: throughput of a resident-GEMM-like loop: per 32-deep k-group a wave splits its B fragment
//         (8 floats of its pixel) once and multiplies it against NT weight tiles (pre-split planes in
//         registers), 6 MFMAs per tile; fp32-equivalent TF/s vs the f32 MFMA loop doing the same work.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma_f32(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_bf(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

struct Split3 {
  bf16x8 h, m, l;
};
__device__ __forceinline__ Split3 split8(const float (&x)[8]) {
  Split3 s;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = (__bf16)x[j];
    const float r1 = x[j] - (float)h;
    const __bf16 m = (__bf16)r1;
    const float r2 = r1 - (float)m;
    s.h[j] = h;
    s.m[j] = m;
    s.l[j] = (__bf16)r2;
  }
  return s;
}

// one 16x16 tile per wave: C = A (16 x K) . B (K x 16); A row-major [16][K], B col-major [16][K]
template <int MODE>
__global__ void tile_kernel(const float* __restrict__ A, const float* __restrict__ B, float* __restrict__ C, int K) {
  const int lane = threadIdx.x & 63, tile = blockIdx.x;
  const float* a = A + (size_t)tile * 16 * K;
  const float* b = B + (size_t)tile * 16 * K;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int r = lane & 15, q = lane >> 4;
  if (MODE == 0) {
    for (int k = 0; k < K; k += 4) acc = mfma_f32(a[r * K + k + q], b[r * K + k + q], acc);
  } else {
    for (int k = 0; k < K; k += 32) {
      float xa[8], xb[8];
      for (int j = 0; j < 8; ++j) {
        xa[j] = a[r * K + k + 8 * q + j];
        xb[j] = b[r * K + k + 8 * q + j];
      }
      const Split3 sa = split8(xa), sb = split8(xb);
      if (MODE == 3) {  // 3 products
        acc = mfma_bf(sa.m, sb.h, acc);
        acc = mfma_bf(sa.h, sb.m, acc);
        acc = mfma_bf(sa.h, sb.h, acc);
      } else if (MODE == 6) {  // small terms first
        acc = mfma_bf(sa.l, sb.h, acc);
        acc = mfma_bf(sa.h, sb.l, acc);
        acc = mfma_bf(sa.m, sb.m, acc);
        acc = mfma_bf(sa.m, sb.h, acc);
        acc = mfma_bf(sa.h, sb.m, acc);
        acc = mfma_bf(sa.h, sb.h, acc);
      } else if (MODE == 61) {  // the library's order (mfma3.h mfma6): grouped by the A plane
        acc = mfma_bf(sa.l, sb.h, acc);
        acc = mfma_bf(sa.m, sb.m, acc);
        acc = mfma_bf(sa.m, sb.h, acc);
        acc = mfma_bf(sa.h, sb.l, acc);
        acc = mfma_bf(sa.h, sb.m, acc);
        acc = mfma_bf(sa.h, sb.h, acc);
      } else if (MODE == 60) {  // big term first (order check)
        acc = mfma_bf(sa.h, sb.h, acc);
        acc = mfma_bf(sa.m, sb.h, acc);
        acc = mfma_bf(sa.h, sb.m, acc);
        acc = mfma_bf(sa.m, sb.m, acc);
        acc = mfma_bf(sa.l, sb.h, acc);
        acc = mfma_bf(sa.h, sb.l, acc);
      } else {  // 9 products
        acc = mfma_bf(sa.l, sb.l, acc);
        acc = mfma_bf(sa.m, sb.l, acc);
        acc = mfma_bf(sa.l, sb.m, acc);
        acc = mfma_bf(sa.l, sb.h, acc);
        acc = mfma_bf(sa.h, sb.l, acc);
        acc = mfma_bf(sa.m, sb.m, acc);
        acc = mfma_bf(sa.m, sb.h, acc);
        acc = mfma_bf(sa.h, sb.m, acc);
        acc = mfma_bf(sa.h, sb.h, acc);
      }
    }
  }
  // C/D: col = lane & 15 (B column), row = 4 (lane >> 4) + e (A row)
  for (int e = 0; e < 4; ++e) C[(size_t)tile * 256 + (4 * q + e) * 16 + r] = acc[e];
}

static unsigned long long rng = 88172645463325252ull;
static double urand() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (rng >> 11) * (1.0 / 9007199254740992.0);
}
static float nrand() {
  const double u = urand() + 1e-300, v = urand();
  return (float)(std::sqrt(-2 * std::log(u)) * std::cos(6.283185307179586 * v));
}

template <int MODE>
void run_mode(const char* name, int K, int tiles, const float* dA, const float* dB, float* dC, const std::vector<double>& ref,
              const std::vector<double>& scale) {
  hipLaunchKernelGGL(tile_kernel<MODE>, dim3(tiles), dim3(64), 0, 0, dA, dB, dC, K);
  std::vector<float> C((size_t)tiles * 256);
  hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
  double mx = 0, ms = 0, mxa = 0;
  for (size_t i = 0; i < C.size(); ++i) {
    const double e = std::fabs((double)C[i] - ref[i]);
    mx = std::max(mx, e / scale[i]);
    ms += (e / scale[i]) * (e / scale[i]);
    mxa = std::max(mxa, e / (std::fabs(ref[i]) + 1e-30));
  }
  printf("  %-22s max err/sum|ab| %.3e  rms %.3e  (2^%.1f)\n", name, mx, std::sqrt(ms / C.size()),
         std::log2(std::sqrt(ms / C.size())));
}

void accuracy(int K, int tiles, float spread) {
  std::vector<float> A((size_t)tiles * 16 * K), B((size_t)tiles * 16 * K);
  for (auto& v : A) v = nrand() * std::exp2f((float)(urand() * spread - spread / 2));
  for (auto& v : B) v = nrand() * std::exp2f((float)(urand() * spread - spread / 2));
  std::vector<double> ref((size_t)tiles * 256), scale((size_t)tiles * 256);
  std::vector<float> seq((size_t)tiles * 256);
  for (int t = 0; t < tiles; ++t)
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = 0, sa = 0;
        float f = 0.f;
        for (int k = 0; k < K; ++k) {
          const float a = A[((size_t)t * 16 + i) * K + k], b = B[((size_t)t * 16 + j) * K + k];
          s += (double)a * b;
          sa += std::fabs((double)a * b);
          f = std::fmaf(a, b, f);
        }
        ref[(size_t)t * 256 + i * 16 + j] = s;
        scale[(size_t)t * 256 + i * 16 + j] = sa;
        seq[(size_t)t * 256 + i * 16 + j] = f;
      }
  float *dA, *dB, *dC;
  hipMalloc(&dA, A.size() * 4);
  hipMalloc(&dB, B.size() * 4);
  hipMalloc(&dC, (size_t)tiles * 256 * 4);
  hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  printf("K = %d, %d tiles, operand exponent spread 2^+-%.0f\n", K, tiles, spread / 2);
  {
    double mx = 0, ms = 0;
    for (size_t i = 0; i < seq.size(); ++i) {
      const double e = std::fabs((double)seq[i] - ref[i]) / scale[i];
      mx = std::max(mx, e);
      ms += e * e;
    }
    printf("  %-22s max err/sum|ab| %.3e  rms %.3e  (2^%.1f)\n", "host fp32 fma chain", mx, std::sqrt(ms / seq.size()),
           std::log2(std::sqrt(ms / seq.size())));
  }
  run_mode<0>("f32 MFMA 16x16x4", K, tiles, dA, dB, dC, ref, scale);
  run_mode<3>("bf16 x3", K, tiles, dA, dB, dC, ref, scale);
  run_mode<6>("bf16 x6 (small first)", K, tiles, dA, dB, dC, ref, scale);
  run_mode<61>("bf16 x6 (library order)", K, tiles, dA, dB, dC, ref, scale);
  run_mode<60>("bf16 x6 (big first)", K, tiles, dA, dB, dC, ref, scale);
  run_mode<9>("bf16 x9", K, tiles, dA, dB, dC, ref, scale);
  hipFree(dA);
  hipFree(dB);
  hipFree(dC);
}

// ---- throughput: NT weight tiles resident in registers (pre-split), the B fragment of each k-group
// loaded (L2-resident buffer) and split per k-group
template <int NT, bool EMU>
__global__ __launch_bounds__(256) void tput_kernel(const float* __restrict__ X, float* out, int iters) {
  const int lane = threadIdx.x & 63;
  f32x4 acc[NT][2];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  Split3 w[NT];
  float wf[NT][8];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = __sinf(lane * 1.7f + t * 3.1f + j * 0.37f);
    w[t] = split8(x);
#pragma unroll
    for (int j = 0; j < 8; ++j) wf[t][j] = x[j];
  }
  const float* xp = X + (size_t)(blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 * 16 + lane * 16;
  for (int it = 0; it < iters; ++it) {
    const f32x4* src = reinterpret_cast<const f32x4*>(xp + (it & 7) * 0);
    float b[2][8];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const f32x4 u = src[2 * r] * (1.0f + it * 1e-7f), v = src[2 * r + 1];
      for (int j = 0; j < 4; ++j) {
        b[r][j] = u[j];
        b[r][4 + j] = v[j];
      }
    }
    if constexpr (EMU) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const Split3 s = split8(b[r]);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          acc[t][r] = mfma_bf(w[t].l, s.h, acc[t][r]);
          acc[t][r] = mfma_bf(w[t].h, s.l, acc[t][r]);
          acc[t][r] = mfma_bf(w[t].m, s.m, acc[t][r]);
          acc[t][r] = mfma_bf(w[t].m, s.h, acc[t][r]);
          acc[t][r] = mfma_bf(w[t].h, s.m, acc[t][r]);
          acc[t][r] = mfma_bf(w[t].h, s.h, acc[t][r]);
        }
      }
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 2; ++r) acc[t][r] = mfma_f32(wf[t][s], b[r][s], acc[t][r]);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) s += acc[t][0].x + acc[t][1].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NT, bool EMU>
void tput(int blocks_per_cu, int iters) {
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * blocks_per_cu;
  float *X, *out;
  hipMalloc(&X, (size_t)blocks * 4 * 64 * 16 * 4);
  hipMemset(X, 0, (size_t)blocks * 4 * 64 * 16 * 4);
  std::vector<float> hx((size_t)blocks * 4 * 64 * 16);
  for (auto& v : hx) v = nrand();
  hipMemcpy(X, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((tput_kernel<NT, EMU>), dim3(blocks), dim3(256), 0, 0, X, out, iters / 4);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((tput_kernel<NT, EMU>), dim3(blocks), dim3(256), 0, 0, X, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // fp32-equivalent work: per iteration NT tiles x 2 pixel tiles x 16 x 16 x 8 k, 2 flop
  const double flops = 5.0 * blocks * 4.0 * iters * NT * 2 * 16 * 16 * 8 * 2.0;
  printf("NT=%d %s waves/SIMD=%d: %.1f TF/s fp32-equivalent (%.2fx the f32 MFMA peak 157.3)\n", NT,
         EMU ? "bf16x6" : "f32   ", blocks_per_cu, flops / (ms * 1e-3) / 1e12, flops / (ms * 1e-3) / 1e12 / 157.3);
  hipFree(X);
  hipFree(out);
}

int main() {
  accuracy(96, 2048, 0.f);
  accuracy(96, 2048, 16.f);
  accuracy(512, 512, 0.f);
  accuracy(1024, 256, 8.f);
  tput<6, false>(1, 20000);
  tput<6, true>(1, 20000);
  tput<6, false>(2, 20000);
  tput<6, true>(2, 20000);
  tput<3, true>(2, 20000);
  return 0;
}
