// Sustained v_mfma_f32_16x16x4_f32 throughput: independent accumulator chains, no memory traffic
// in the loop.  Reports TF/s for 1 and 2 waves per SIMD and the effective clock implied at 100%.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int CHAINS>
__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters, float a0, float b0) {
  f32x4 acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
  }
  float s = 0.f;
  for (int c = 0; c < CHAINS; ++c) s += acc[c].x + acc[c].y + acc[c].z + acc[c].w;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CHAINS>
void run(int blocks_per_cu, int iters) {
  const int cus = 256, blocks = cus * blocks_per_cu;
  float* out;
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(mfma_loop<CHAINS>, dim3(blocks), dim3(256), 0, 0, out, iters / 4, 1.0f, 0.5f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL(mfma_loop<CHAINS>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f, 0.5f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 5.0 * blocks * 4.0 /*waves*/ * iters * CHAINS * 2048.0;
  const double tf = flops / (ms * 1e-3) / 1e12;
  printf("chains=%d waves/SIMD=%d: %.1f TF/s (%.1f%% of 157.3; implied clock at 100%% = %.2f GHz)\n", CHAINS,
         blocks_per_cu, tf, 100 * tf / 157.3, 2.4 * tf / 157.3);
  hipFree(out);
}

int main() {
  run<4>(1, 20000);
  run<8>(1, 20000);
  run<4>(2, 20000);
  run<8>(2, 20000);
  return 0;
}
