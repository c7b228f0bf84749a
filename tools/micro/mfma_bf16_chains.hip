// Sustained v_mfma_f32_16x16x32_bf16 throughput vs the number of independent accumulator chains
// (1 and 2 waves per SIMD): the split-bf16 kernels (mfma3.h) issue their MFMAs in 3..12 chains per
// wave, so this is the dependent-issue cost those wave roles see.  No memory traffic in the loop.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int CHAINS>
__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters, float a0) {
  f32x4 acc[CHAINS];
  bf16x8 a[CHAINS], b[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) {
    acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[c][j] = (__bf16)(a0 * __sinf(threadIdx.x * 12.9898f + c * 78.233f + j));
      b[c][j] = (__bf16)(a0 * __cosf(threadIdx.x * 4.1414f + c * 17.17f + j));
    }
  }
  for (int i = 0; i < iters; i += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c], b[c], acc[c], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c].x + acc[c].y + acc[c].z + acc[c].w;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CHAINS>
void run(float* out, int wps, int iters) {
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * wps;  // 256-thread blocks: 4 waves = one per SIMD
  hipLaunchKernelGGL(mfma_loop<CHAINS>, dim3(blocks), dim3(256), 0, 0, out, 64, 0.5f);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma_loop<CHAINS>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.5f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)blocks * 4 * iters * CHAINS * 16.0 * 16 * 32 * 2;
  const double tf = flops / (ms * 1e-3) / 1e12;
  printf("bf16 16x16x32 chains=%d waves/SIMD=%d: %.1f TF/s (%.1f%% of 2516.6 dense bf16; %.1f cycles per MFMA per SIMD at 2.4 GHz)\n",
         CHAINS, wps, tf, 100.0 * tf / 2516.6, 16.0 * 2516.6 / tf);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 256 * 8 * sizeof(float));
  for (int wps = 1; wps <= 2; ++wps) {
    run<1>(out, wps, 1 << 14);
    run<2>(out, wps, 1 << 14);
    run<3>(out, wps, 1 << 14);
    run<4>(out, wps, 1 << 14);
    run<6>(out, wps, 1 << 14);
    run<8>(out, wps, 1 << 14);
    run<12>(out, wps, 1 << 13);
  }
  hipFree(out);
  return 0;
}
