// Micro-benchmark: HBM store rate of the GEMM epilogue's access shape on MI355X.
//   A: 16 pixel rows x 64 B per wave-instruction (a 16x16 MFMA accumulator tile as it stands: lane
//      (li, lq) writes 16 B at row li, channels 16t + 4lq); consecutive instructions (t, t+1)
//      complete each 128-B line
//   B: 8 rows x 128 B per instruction (full lines)
//   C: 4 rows x 256 B per instruction
// Every variant writes the same bytes: rows of LD floats, each wave 32 rows x LD floats.
// build: hipcc --offload-arch=gfx950 -O3 -o store_pattern store_pattern.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int LD = 256;  // floats per pixel row (1 KiB)

template <int V>
__global__ __launch_bounds__(512) void store_kernel(float* out, long long rows, int iters) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f32x4 v = f32x4{1.f, 2.f, 3.f, (float)lane};
  for (int it = 0; it < iters; ++it) {
    const long long tile = (long long)blockIdx.x + (long long)it * gridDim.x;
    const long long row0 = tile * 256 + wave * 32;
    if (row0 + 32 > rows) return;
    float* base = out + row0 * LD;
    if (V == 0) {
      const int li = lane & 15, lq = lane >> 4;
#pragma unroll
      for (int t = 0; t < LD / 16; ++t)
#pragma unroll
        for (int r = 0; r < 2; ++r)
          *reinterpret_cast<f32x4*>(base + (16 * r + li) * LD + 16 * t + 4 * lq) = v;
    } else if (V == 1) {
      const int lr = lane >> 3, lc = lane & 7;
#pragma unroll
      for (int t = 0; t < LD / 32; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *reinterpret_cast<f32x4*>(base + (8 * r + lr) * LD + 32 * t + 4 * lc) = v;
    } else {
      const int lr = lane >> 4, lc = lane & 15;
#pragma unroll
      for (int t = 0; t < LD / 64; ++t)
#pragma unroll
        for (int r = 0; r < 8; ++r)
          *reinterpret_cast<f32x4*>(base + (4 * r + lr) * LD + 64 * t + 4 * lc) = v;
    }
  }
}

int main() {
  const long long rows = 16LL << 20;  // 16M rows x 1 KiB = 16 GiB
  float* out;
  if (hipMalloc(&out, rows * LD * sizeof(float)) != hipSuccess) return 1;
  const int grid = 2048;
  const int iters = (int)(rows / 256 / grid);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[3] = {"A 16 rows x 64 B / instr (MFMA tile as is)", "B 8 rows x 128 B / instr",
                          "C 4 rows x 256 B / instr"};
  for (int rep = 0; rep < 2; ++rep)
    for (int v = 0; v < 3; ++v) {
      auto launch = [&]() {
        if (v == 0) hipLaunchKernelGGL(store_kernel<0>, dim3(grid), dim3(512), 0, 0, out, rows, iters);
        if (v == 1) hipLaunchKernelGGL(store_kernel<1>, dim3(grid), dim3(512), 0, 0, out, rows, iters);
        if (v == 2) hipLaunchKernelGGL(store_kernel<2>, dim3(grid), dim3(512), 0, 0, out, rows, iters);
      };
      launch();
      hipEventRecord(e0);
      for (int k = 0; k < 3; ++k) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      const double bytes = 3.0 * (double)rows * LD * 4;
      printf("%s: %.2f TB/s\n", names[v], bytes / (ms * 1e-3) / 1e12);
    }
  hipFree(out);
  return 0;
}
