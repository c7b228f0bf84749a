// Micro-benchmark of the training GEMM (train.hip launch_tgemm) on the shapes a KDLAE-T training
// step at 6 x 128^2 issues most often.  Build (CPU container):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/tgemm_bench.cpp \
//     rethink_acoustic_image_enhancement_amd/csrc/train.hip -o tools/micro/tgemm_bench
// Run on the GPU box: ./tools/micro/tgemm_bench   (prints us / TFLOP/s / GB/s per shape)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../../rethink_acoustic_image_enhancement_amd/csrc/train_kernels.h"

using kdlae::train::TGemm;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

struct Shape {
  const char* name;
  int kind;  // 0 fwd (A[P,K] W[N,K]^T), 1 dX (dY[P,N'] W[N',K] -> [P,K]), 2 dW (dY^T X, split-K)
  int P, N, K;
};

int main() {
  const Shape shapes[] = {
      {"fwd qkv C96   P98k", 0, 98304, 288, 96},   {"fwd pin C96   P98k", 0, 98304, 510, 96},
      {"fwd pout C96  P98k", 0, 98304, 96, 255},   {"fwd proj C96  P98k", 0, 98304, 96, 96},
      {"dX qkv C96    P98k", 1, 98304, 96, 288},   {"dX pin C96    P98k", 1, 98304, 96, 510},
      {"dX pout C96   P98k", 1, 98304, 255, 96},   {"dW qkv C96    P98k", 2, 98304, 288, 96},
      {"dW pin C96    P98k", 2, 98304, 510, 96},   {"fwd pin C48  P393k", 0, 393216, 254, 48},
      {"dX pin C48   P393k", 1, 393216, 48, 254},  {"dW pin C48   P393k", 2, 393216, 254, 48},
  };
  const size_t maxe = (size_t)393216 * 512;
  float *A, *B, *C, *part;
  CK(hipMalloc(&A, maxe * 4));
  CK(hipMalloc(&B, maxe * 4));
  CK(hipMalloc(&C, maxe * 4));
  const size_t pcap = 8u << 20;
  CK(hipMalloc(&part, pcap * 4));
  CK(hipMemset(A, 0, maxe * 4));
  CK(hipMemset(B, 0, maxe * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& s : shapes) {
    TGemm g;
    size_t cap = 0;
    double bytes = 0;
    if (s.kind == 0) {  // Y[P,N] = X[P,K] W[N,K]^T
      g.A = A; g.sam = s.K; g.sak = 1;
      g.B = B; g.sbk = 1; g.sbn = s.K;
      g.C = C; g.scm = s.N; g.scn = 1;
      g.M = s.P; g.N = s.N; g.K = s.K;
      bytes = 4.0 * s.P * (s.K + s.N);
    } else if (s.kind == 1) {  // dX[P,N] = dY[P,K] W[K,N]
      g.A = A; g.sam = s.K; g.sak = 1;
      g.B = B; g.sbk = s.N; g.sbn = 1;
      g.C = C; g.scm = s.N; g.scn = 1;
      g.M = s.P; g.N = s.N; g.K = s.K;
      bytes = 4.0 * s.P * (s.K + s.N);
    } else {  // dW[N,K] = dY[P,N]^T X[P,K]
      g.A = A; g.sam = 1; g.sak = s.N;
      g.B = B; g.sbk = s.K; g.sbn = 1;
      g.C = C; g.scm = s.K; g.scn = 1;
      g.M = s.N; g.N = s.K; g.K = s.P;
      g.partial = part;
      cap = pcap;
      bytes = 4.0 * s.P * (s.K + s.N);
    }
    const double flops = 2.0 * s.P * s.N * s.K;
    for (int i = 0; i < 3; ++i) CK(kdlae::train::launch_tgemm(g, cap, 0));
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) CK(kdlae::train::launch_tgemm(g, cap, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    std::printf("%-22s M=%7d N=%4d K=%7d  %8.1f us  %6.1f TF/s  %6.0f GB/s\n", s.name, g.M, g.N, g.K, us,
                flops / us / 1e6, bytes / us / 1e3);
  }
  return 0;
}
