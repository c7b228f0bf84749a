// Sustained v_mfma_f32_16x16x4_f32 throughput: independent accumulator chains, no memory traffic
// in the loop.  Reports TF/s for 1 and 2 waves per SIMD and the effective clock implied at 100%.
//
// r02: the r01 version looped over 4-8 MFMAs per iteration and hipcc shuffled accumulators through
// v_accvgpr_read/mov/write plus an s_nop 7 every iteration (register-allocation artefact), so it
// measured the shuffle, not the pipe (123-135 TF/s).  The loop body is now 8 iterations x CHAINS
// MFMAs with the operands varied per chain, and the ISA (hipcc -S) is back-to-back MFMAs.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int CHAINS>
__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters, float a0, float b0) {
  f32x4 acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a[CHAINS], b[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) {
    // random-looking operands per lane and chain: the clock the chip holds depends on the data
    a[c] = a0 * __sinf(threadIdx.x * 12.9898f + c * 78.233f + blockIdx.x * 0.37f);
    b[c] = b0 * __cosf(threadIdx.x * 4.1414f + c * 17.17f);
  }
  for (int i = 0; i < iters; i += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c], b[c], acc[c], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c].x + acc[c].y + acc[c].z + acc[c].w;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CHAINS>
void run(int blocks_per_cu, int iters) {
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * blocks_per_cu;
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
  printf("chains=%d waves/SIMD=%d cus=%d: %.1f TF/s (%.1f%% of 157.3; implied clock at 100%% = %.2f GHz)\n", CHAINS,
         blocks_per_cu, cus, tf, 100 * tf / 157.3, 2.4 * tf / 157.3);
  hipFree(out);
}

int main() {
  run<4>(1, 40000);
  run<8>(1, 40000);
  run<4>(2, 40000);
  run<8>(2, 40000);
  return 0;
}
