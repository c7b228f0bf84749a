// Does a VALU stream on one wave slow the MFMA stream of the other wave on the same SIMD?  The fused
// FFN pairs a project_in (MFMA) wave with a gate (VALU) wave per SIMD.  Blocks of 8 waves (one block
// per CU, waves w and w + 4 on one SIMD): waves 0-3 run an MFMA loop, waves 4-7 a VALU loop, either
// role alone or both.  MFMA shapes 16x16x32 and 32x32x16 bf16 at equal FLOPs; VALU packed
// (v_pk_fma_f32) or scalar (v_fma_f32) FMAs at equal FLOPs.  No memory traffic in the loops.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// role: bit 0 = MFMA waves active, bit 1 = VALU waves active, 4 = VALU on all 8 waves (2 VALU waves per
// SIMD), 8 = waves 0-3 run the MFMA loop with the VALU work interleaved (one wave per SIMD)
template <bool BIG, bool PACKED>
__global__ __launch_bounds__(512) void coissue(float* out, int mfma_iters, int valu_iters, int role, float a0) {
  const int w = threadIdx.x >> 6;
  float s = 0.f;
  if (w < 4 && !(role & 4)) {
    if (role & 9) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a[c][j] = (__bf16)(a0 * __sinf(threadIdx.x * 12.9898f + c * 78.233f + j));
          b[c][j] = (__bf16)(a0 * __cosf(threadIdx.x * 4.1414f + c * 17.17f + j));
        }
      if constexpr (BIG) {
        f32x16 acc[2];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int j = 0; j < 16; ++j) acc[c][j] = 0.f;
        for (int i = 0; i < mfma_iters; i += 8) {  // 2 chains x 4 = 8 MFMAs of 32x32x16 = 16 of 16x16x32
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int c = 0; c < 2; ++c)
              acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[c], b[c], acc[c], 0, 0, 0);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int j = 0; j < 16; ++j) s += acc[c][j];
      } else {
        f32x4 acc[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (role & 8) {
          f32x2 x[8];
          const f32x2 m = f32x2{a0 * 0.999f, a0 * 0.998f}, k = f32x2{a0 * 2e-3f, a0 * 4e-3f};
#pragma unroll
          for (int c = 0; c < 8; ++c) x[c] = f32x2{a0 * __sinf(threadIdx.x + c), a0 * __cosf(threadIdx.x + c)};
          const int per = valu_iters / (mfma_iters / 8);  // VALU iterations per 16 MFMAs
          for (int i = 0; i < mfma_iters; i += 8) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
#pragma unroll
              for (int c = 0; c < 4; ++c)
                acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c], b[c], acc[c], 0, 0, 0);
              for (int j = 0; j < per; ++j) {  // 2 packed FMAs per j: per x 8 per 16 MFMAs, as the VALU role
                x[2 * (j & 3)] = __builtin_elementwise_fma(x[2 * (j & 3)], m, k);
                x[2 * (j & 3) + 1] = __builtin_elementwise_fma(x[2 * (j & 3) + 1], m, k);
              }
            }
          }
#pragma unroll
          for (int c = 0; c < 8; ++c) s += x[c].x + x[c].y;
        } else {
          for (int i = 0; i < mfma_iters; i += 8) {  // 16 MFMAs of 16x16x32
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
              for (int c = 0; c < 4; ++c)
                acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c], b[c], acc[c], 0, 0, 0);
          }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) s += acc[c].x + acc[c].y + acc[c].z + acc[c].w;
      }
    }
  } else if ((role & 2) || (role & 4)) {
    f32x2 x[8];
    const f32x2 m = f32x2{a0 * 0.999f, a0 * 0.998f}, k = f32x2{a0 * 2e-3f, a0 * 4e-3f};
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = f32x2{a0 * __sinf(threadIdx.x + c), a0 * __cosf(threadIdx.x + c)};
    for (int i = 0; i < valu_iters; ++i) {  // 8 packed FMAs = 16 scalar FMAs per iteration
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        if constexpr (PACKED) {
          x[c] = __builtin_elementwise_fma(x[c], m, k);
        } else {
          x[c].x = fmaf(x[c].x, m.x, k.x);
          x[c].y = fmaf(x[c].y, m.y, k.y);
          asm volatile("" : "+v"(x[c].x), "+v"(x[c].y));  // keep the two lanes' FMAs scalar
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) s += x[c].x + x[c].y;
  }
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <bool BIG, bool PACKED>
float run(float* out, int mi, int vi, int role) {
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipLaunchKernelGGL((coissue<BIG, PACKED>), dim3(cus), dim3(512), 0, 0, out, 64, 64, role, 0.5f);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((coissue<BIG, PACKED>), dim3(cus), dim3(512), 0, 0, out, mi, vi, role, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

template <bool BIG, bool PACKED>
void suite(float* out, int mi, int vi) {
  const float tm = run<BIG, PACKED>(out, mi, vi, 1), tv = run<BIG, PACKED>(out, mi, vi, 2),
              tb = run<BIG, PACKED>(out, mi, vi, 3);
  printf("mfma %-9s valu %-6s: MFMA alone %.3f ms, VALU alone %.3f ms, both %.3f ms (max %.3f, sum %.3f; "
         "both / max = %.2f)\n",
         BIG ? "32x32x16" : "16x16x32", PACKED ? "packed" : "scalar", tm, tv, tb, tm > tv ? tm : tv, tm + tv,
         tb / (tm > tv ? tm : tv));
}

void extra(float* out, int mi, int vi) {
  const float tm = run<false, true>(out, mi, vi, 1), tv = run<false, true>(out, mi, vi, 2),
              tv2 = run<false, true>(out, mi, vi, 4), tf = run<false, true>(out, mi, vi, 8);
  printf("16x16x32 + packed: MFMA alone %.3f, VALU alone (1 wave/SIMD) %.3f, VALU on 2 waves/SIMD (2x the work) %.3f, "
         "MFMA + VALU interleaved in one wave %.3f ms\n", tm, tv, tv2, tf);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 512 * 8 * sizeof(float));
  const int mi = 1 << 16;  // 16x16x32-equivalent MFMAs per MFMA wave
  // VALU iterations: 16 scalar FMAs each; sized so the VALU wave's issue roughly matches the MFMA time
  for (int vi : {1 << 14, 1 << 15, 1 << 16}) {
    printf("valu iterations %d\n", vi);
    suite<false, true>(out, mi, vi);
    suite<true, true>(out, mi, vi);
    suite<false, false>(out, mi, vi);
    suite<true, false>(out, mi, vi);
    extra(out, mi, vi);
  }
  hipFree(out);
  return 0;
}
