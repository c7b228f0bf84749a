// Timing of the training step's 1x1 / MDTA contractions through launch_tgemm (whatever kernel the
// build routes them to): per shape, the mean of 20 launches after 3 warm-ups, HIP events.
// Shapes: the top contractions of tools/train_trace.py at KDLAET.yml 6 x 128^2.
// Build several binaries with different -D switches (tools/micro/build_rows_check.sh) and compare.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../rethink_acoustic_image_enhancement_amd/csrc/train_kernels.h"

using kdlae::train::TGemm;
#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

struct S {
  const char* role;
  int M, N, K, z;  // rows-type: M pixels; dW-type (role "dW"): M = Cout, N = Cin, K = pixels
  int lda, ldc;    // rows-type: A row stride, C row stride (0 = K / N)
};

int main() {
  const S shapes[] = {
      {"fwd", 98304, 510, 96, 1, 96, 512},   {"dX", 98304, 96, 510, 1, 512, 96},
      {"fwd", 98304, 96, 255, 1, 256, 96},   {"dX", 98304, 96, 288, 1, 288, 96},
      {"fwd", 98304, 288, 96, 1, 96, 288},   {"dX", 98304, 255, 96, 1, 96, 256},
      {"fwd", 393216, 254, 48, 1, 48, 256},  {"fwd", 98304, 96, 96, 1, 96, 96},
      {"dX", 393216, 48, 254, 1, 256, 48},   {"fwd", 393216, 144, 48, 1, 48, 144},
      {"fwd", 393216, 48, 127, 1, 128, 48},  {"dX", 393216, 127, 48, 1, 48, 128},
      {"fwd", 24576, 510, 96, 1, 96, 512},   {"dX", 24576, 96, 510, 1, 512, 96},
      {"fwd", 6144, 1020, 192, 1, 192, 1020}, {"dX", 6144, 192, 1020, 1, 1020, 192},
      {"fwd", 1536, 2042, 384, 1, 384, 2044}, {"dX", 1536, 384, 2042, 1, 2044, 384},
      {"dq", 16384, 96, 96, 6, 288, 288},    {"dq", 65536, 48, 48, 6, 144, 144},
      {"dW", 510, 96, 98304, 1, 512, 96},    {"dW", 288, 96, 98304, 1, 288, 96},
      {"dW", 96, 255, 98304, 1, 96, 256},    {"dW", 254, 48, 393216, 1, 256, 48},
      {"dW", 1020, 192, 6144, 1, 1020, 192}, {"dW", 2042, 384, 1536, 1, 2044, 384},
      {"gram", 96, 96, 16384, 6, 288, 288},  {"dW", 96, 96, 98304, 1, 96, 96},
  };
  const size_t big = 160u << 20;  // floats per operand buffer
  float *dA, *dB, *dC, *dP;
  CK(hipMalloc(&dA, big * 4));
  CK(hipMalloc(&dB, big * 4));
  CK(hipMalloc(&dC, big * 4));
  const size_t cap = 8u << 20;
  CK(hipMalloc(&dP, cap * 4));
  CK(hipMemset(dA, 0, big * 4));
  CK(hipMemset(dB, 0, big * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  double total = 0;
  for (const S& s : shapes) {
    TGemm g;
    const bool dw = s.role[0] == 'd' && s.role[1] == 'W';
    const bool gram = s.role[0] == 'g';
    if (dw || gram) {
      g.A = dA; g.sam = 1; g.sak = s.lda; g.bA1 = (long long)s.K * s.lda;
      g.B = dB; g.sbk = s.ldc; g.sbn = 1; g.bB1 = (long long)s.K * s.ldc;
      g.C = dC; g.scm = s.N; g.scn = 1; g.bC1 = (long long)s.M * s.N;
      g.partial = dP;
    } else {
      g.A = dA; g.sam = s.lda; g.sak = 1; g.bA1 = (long long)s.M * s.lda;
      g.B = dB;
      if (s.role[0] == 'f') { g.sbk = 1; g.sbn = s.K; } else { g.sbk = s.N; g.sbn = 1; }
      g.bB1 = (long long)s.N * s.K;
      g.C = dC; g.scm = s.ldc; g.scn = 1; g.bC1 = (long long)s.M * s.ldc;
      g.c_pad_ok = s.ldc >= (s.N + 3) / 4 * 4;
    }
    g.M = s.M; g.N = s.N; g.K = s.K; g.nz1 = s.z;
    const size_t pc = (dw || gram) ? cap : 0;
    for (int i = 0; i < 3; ++i) CK(kdlae::train::launch_tgemm(g, pc, 0));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 20; ++i) CK(kdlae::train::launch_tgemm(g, pc, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1000.0 / 20;
    total += us;
    const double fl = 2.0 * s.M * s.N * s.K * s.z;
    printf("%-5s M%7d N%5d K%7d z%2d  %8.1f us  %6.1f TF/s\n", s.role, s.M, s.N, s.K, s.z, us, fl / us / 1e6);
  }
  printf("TOTAL %.1f us\n", total);
  return 0;
}
