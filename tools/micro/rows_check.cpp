// Standalone check of the training row-streaming GEMM (train_rows.hip) against a CPU double
// reference over the shapes the training step launches (1x1 fwd / dX, MDTA products), including
// K % 16 != 0 with garbage in the ld pad columns, N tails, residual + per-column scale, batching,
// channel-slice views.  Build: see tools/micro/build_rows_check.sh.  Prints one line per case.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

static unsigned long long rng = 88172645463325252ull;
static float frand() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (float)((rng >> 11) * (1.0 / 9007199254740992.0)) * 2.f - 1.f;
}

struct Case {
  const char* name;
  int M, N, K, lda, ldc, nz1, nz2;
  bool bt;      // B stored [N][K] (fwd: W) instead of [K][N] (dX: W)
  bool res, rs, bias, slice;
};

int main() {
  const Case cases[] = {
      {"fwd K96 N510", 98304, 510, 96, 96, 512, 1, 1, true, false, false, true, false},
      {"fwd K48 N254", 20000, 254, 48, 48, 256, 1, 1, true, false, false, true, false},
      {"fwd K127 N48 res", 9000, 48, 127, 128, 48, 1, 1, true, true, false, true, false},
      {"fwd K255 N96 res", 7777, 96, 255, 256, 96, 1, 1, true, true, false, true, false},
      {"dX K510 N96", 12345, 96, 510, 512, 96, 1, 1, false, false, false, false, false},
      {"dX K96 N255", 5000, 255, 96, 96, 256, 1, 1, false, false, false, false, false},
      {"dX K144 N48 res", 4096, 48, 144, 144, 48, 1, 1, false, true, false, false, false},
      {"dX K2042 N384", 1536, 384, 2042, 2044, 384, 1, 1, false, false, false, false, false},
      {"dX K96 N127", 3000, 127, 96, 96, 128, 1, 1, false, false, false, false, false},
      {"dq Ch48 z6 res rs slice", 4096, 48, 48, 144, 144, 3, 2, true, true, true, false, true},
      {"dv Ch96 z2 slice", 2048, 96, 96, 288, 288, 2, 1, false, false, false, false, true},
      {"small M", 100, 40, 20, 20, 40, 1, 1, true, false, false, true, false},
      {"fwd K96 N96 (NT6)", 5000, 96, 96, 96, 96, 1, 1, true, false, false, true, false},
      {"fwd K96 N510 padok", 7000, 510, 96, 96, 512, 1, 1, true, false, false, true, false},
      {"dX K96 N127 padok", 3000, 127, 96, 96, 128, 1, 1, false, false, false, false, false},
      {"fwd K16 N128 (NT8)", 1000, 128, 16, 16, 128, 1, 1, true, false, false, true, false},
      {"fwd K64 N112 (NT8 kc1)", 1000, 112, 64, 64, 112, 1, 1, true, false, false, true, false},
  };
  int bad = 0;
  for (const Case& c : cases) {
    const int nz = c.nz1 * c.nz2;
    // per batch entry z1: A rows [M][lda] (slice: the head z2 takes columns z2*K of a wider row)
    const long long lda = c.slice ? c.lda : c.lda, ldc = c.ldc;
    const long long arows = (long long)c.M * lda;
    const long long asz = arows * c.nz1 + 64, csz = (long long)c.M * ldc * c.nz1 + 64;
    const long long bsz = (long long)c.N * c.K * nz + 64;
    std::vector<float> hA(asz), hB(bsz), hC(csz), hR(csz), bias(c.N), rs((size_t)c.N * nz);
    for (auto& v : hA) v = frand();
    // pad columns of the A rows (k >= K within lda): garbage incl. NaN when K % 16 != 0
    if (!c.slice)
      for (long long m = 0; m < (long long)c.M * c.nz1; ++m)
        for (long long k = c.K; k < lda; ++k) hA[m * lda + k] = NAN;
    for (auto& v : hB) v = frand();
    for (auto& v : hR) v = frand();
    for (auto& v : bias) v = frand();
    for (auto& v : rs) v = frand();
    for (auto& v : hC) v = 12345.f;
    float *dA, *dB, *dC, *dR, *dbias, *drs;
    CK(hipMalloc(&dA, asz * 4));
    CK(hipMalloc(&dB, bsz * 4));
    CK(hipMalloc(&dC, csz * 4));
    CK(hipMalloc(&dR, csz * 4));
    CK(hipMalloc(&dbias, c.N * 4));
    CK(hipMalloc(&drs, (size_t)c.N * nz * 4));
    CK(hipMemcpy(dA, hA.data(), asz * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, hB.data(), bsz * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dC, hC.data(), csz * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dR, hR.data(), csz * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dbias, bias.data(), c.N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(drs, rs.data(), (size_t)c.N * nz * 4, hipMemcpyHostToDevice));
    TGemm g;
    g.A = dA; g.sam = lda; g.sak = 1; g.bA1 = arows; g.bA2 = c.slice ? c.K : 0;
    g.B = dB;
    if (c.bt) { g.sbk = 1; g.sbn = c.K; } else { g.sbk = c.N; g.sbn = 1; }
    g.bB1 = (long long)c.N * c.K * c.nz2; g.bB2 = (long long)c.N * c.K;
    g.C = dC; g.scm = ldc; g.scn = 1; g.bC1 = (long long)c.M * ldc; g.bC2 = c.slice ? c.N : 0;
    g.bias = c.bias ? dbias : nullptr;
    if (c.res) { g.R = dR; g.srm = ldc; g.srn = 1; g.bR1 = g.bC1; g.bR2 = g.bC2; }
    if (c.rs) { g.rs = drs; g.brs1 = (long long)c.N * c.nz2; g.brs2 = c.N; }
    g.M = c.M; g.N = c.N; g.K = c.K; g.nz1 = c.nz1; g.nz2 = c.nz2;
    const bool padok = std::strstr(c.name, "padok") != nullptr;
    g.c_pad_ok = padok;
    printf("%-28s rows-eligible %d\n", c.name, (int)kdlae::train::tgemm_rows_eligible(g));
    CK(kdlae::train::launch_tgemm(g, 0, 0));
    CK(hipDeviceSynchronize());
    std::vector<float> out(csz);
    CK(hipMemcpy(out.data(), dC, csz * 4, hipMemcpyDeviceToHost));
    double maxerr = 0, maxref = 0;
    long long clobber = 0, nbad = 0;
    int badt[64] = {0}, badr[8] = {0}, badq[4] = {0};
    std::vector<char> written(csz, 0);
    for (int z1 = 0; z1 < c.nz1; ++z1)
      for (int z2 = 0; z2 < c.nz2; ++z2) {
        const int z = z1 * c.nz2 + z2;
        const float* A = hA.data() + z1 * g.bA1 + z2 * g.bA2;
        const float* B = hB.data() + z1 * g.bB1 + z2 * g.bB2;
        for (int m = 0; m < c.M; ++m)
          for (int n = 0; n < c.N; ++n) {
            double s = 0;
            for (int k = 0; k < c.K; ++k) {
              const double b = c.bt ? B[(long long)n * c.K + k] : B[(long long)k * c.N + n];
              s += (double)A[(long long)m * lda + k] * b;
            }
            if (c.bias) s += bias[n];
            const long long o = z1 * g.bC1 + z2 * g.bC2 + (long long)m * ldc + n;
            if (c.res) s += (c.rs ? rs[(size_t)z * c.N + n] : 1.0) * hR[o];
            written[o] = 1;
            const double e = std::fabs(out[o] - s);
            if (!(e <= maxerr)) maxerr = std::isnan(e) ? INFINITY : e;
            if (!(e <= 1e-3 * (std::fabs(s) + 1))) {
              if (nbad < 1 && c.M <= 20000) {
                // which (row, col) of the reference does the wrong value belong to?
                int fm = -1, fn = -1;
                for (int m2 = 0; m2 < c.M && fm < 0; ++m2)
                  for (int n2 = 0; n2 < c.N; ++n2) {
                    double s2 = 0;
                    for (int k = 0; k < c.K; ++k) {
                      const double b = c.bt ? B[(long long)n2 * c.K + k] : B[(long long)k * c.N + n2];
                      s2 += (double)A[(long long)m2 * lda + k] * b;
                    }
                    if (c.bias) s2 += bias[n2];
                    if (std::fabs(s2 - out[o]) < 1e-4 * (std::fabs(s2) + 1)) { fm = m2; fn = n2; break; }
                  }
                printf("   bad m %d n %d got %.6f ref %.6f  (= ref at m %d n %d)\n", m, n, out[o], s, fm, fn);
                printf("   row %d got:", m);
                for (int q = 0; q < 8; ++q) printf(" %.4f", out[o - n + q]);
                printf("\n");
              }
              ++nbad;
              badt[(n / 16) % 64]++;
              badr[(m % 128) / 16]++;
              badq[(n % 16) / 4]++;
            }
            if (std::fabs(s) > maxref) maxref = std::fabs(s);
          }
      }
    for (long long o = 0; o < csz; ++o) {
      const long long col = o % ldc;
      const bool pad = padok && col >= c.N && col < (c.N + 3) / 4 * 4 && o < (long long)c.M * ldc * c.nz1;
      if (pad ? out[o] != 0.f : (!written[o] && out[o] != 12345.f)) ++clobber;
    }
    const bool ok = maxerr <= 1e-5 * (maxref + 1) * std::sqrt((double)c.K) && clobber == 0;
    printf("%-28s max|err| %.3e  max|ref| %.3e  clobbered %lld  %s\n", c.name, maxerr, maxref, clobber,
           ok ? "OK" : "FAIL");
    if (nbad) {
      printf("   bad %lld; by col tile:", nbad);
      for (int i = 0; i < 64 && i * 16 < c.N; ++i) printf(" %d", badt[i]);
      printf("; by row subtile:");
      for (int i = 0; i < 8; ++i) printf(" %d", badr[i]);
      printf("; by quad:");
      for (int i = 0; i < 4; ++i) printf(" %d", badq[i]);
      printf("\n");
    }
    if (!ok) ++bad;
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dR); hipFree(dbias); hipFree(drs);
  }
  // ---- pixel-reduction (dW / Gram) cases through launch_tgemm with a split-K buffer
  struct WCase {
    const char* name;
    int M, N, P, lda, ldb, nz1, nz2;  // A = dY [P][lda] (M channels), B = X [P][ldb] (N channels)
  };
  const WCase wcases[] = {
      {"dW 510x96 P98304", 510, 96, 98304, 512, 96, 1, 1},
      {"dW 96x255 P20000", 96, 255, 20000, 96, 256, 1, 1},
      {"dW 48x127 P9999", 48, 127, 9999, 48, 128, 1, 1},
      {"dW 1020x192 P6144", 1020, 192, 6144, 1020, 192, 1, 1},
      {"gram 48x48 z6x2 slice", 48, 48, 4096, 288, 288, 6, 2},
      {"dW 3x40 P77", 3, 40, 77, 4, 40, 1, 1},
  };
  const size_t cap = 8u << 20;
  float* dpart;
  CK(hipMalloc(&dpart, cap * 4));
  for (const WCase& c : wcases) {
    const int nz = c.nz1 * c.nz2;
    const long long asz = (long long)c.P * c.lda * c.nz1 + 64, bsz = (long long)c.P * c.ldb * c.nz1 + 64;
    const long long csz = (long long)c.M * c.N * nz + 64;
    std::vector<float> hA(asz), hB(bsz);
    for (auto& v : hA) v = frand();
    for (auto& v : hB) v = frand();
    float *dA, *dB, *dC;
    CK(hipMalloc(&dA, asz * 4));
    CK(hipMalloc(&dB, bsz * 4));
    CK(hipMalloc(&dC, csz * 4));
    CK(hipMemcpy(dA, hA.data(), asz * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, hB.data(), bsz * 4, hipMemcpyHostToDevice));
    TGemm g;
    const bool slice = c.nz2 > 1;
    g.A = dA; g.sam = 1; g.sak = c.lda; g.bA1 = (long long)c.P * c.lda; g.bA2 = slice ? c.M : 0;
    g.B = dB; g.sbk = c.ldb; g.sbn = 1; g.bB1 = (long long)c.P * c.ldb; g.bB2 = slice ? c.N : 0;
    g.C = dC; g.scm = c.N; g.scn = 1; g.bC1 = (long long)c.M * c.N * c.nz2; g.bC2 = (long long)c.M * c.N;
    g.M = c.M; g.N = c.N; g.K = c.P; g.nz1 = c.nz1; g.nz2 = c.nz2;
    g.partial = dpart;
    printf("%-28s eligible %d\n", c.name, (int)kdlae::train::tgemm_cols_eligible(g));
    CK(kdlae::train::launch_tgemm(g, cap, 0));
    CK(hipDeviceSynchronize());
    std::vector<float> out(csz);
    CK(hipMemcpy(out.data(), dC, csz * 4, hipMemcpyDeviceToHost));
    double maxerr = 0, maxref = 0;
    for (int z1 = 0; z1 < c.nz1; ++z1)
      for (int z2 = 0; z2 < c.nz2; ++z2)
        for (int m = 0; m < c.M; ++m)
          for (int n = 0; n < c.N; ++n) {
            double sacc = 0;
            const float* A = hA.data() + z1 * g.bA1 + z2 * g.bA2;
            const float* B = hB.data() + z1 * g.bB1 + z2 * g.bB2;
            for (int p = 0; p < c.P; ++p) sacc += (double)A[(long long)p * c.lda + m] * B[(long long)p * c.ldb + n];
            const double e = std::fabs(out[z1 * g.bC1 + z2 * g.bC2 + (long long)m * c.N + n] - sacc);
            if (!(e <= maxerr)) maxerr = std::isnan(e) ? INFINITY : e;
            if (std::fabs(sacc) > maxref) maxref = std::fabs(sacc);
          }
    const bool ok = maxerr <= 2e-6 * std::sqrt((double)c.P) * 4;
    printf("%-28s max|err| %.3e  max|ref| %.3e  %s\n", c.name, maxerr, maxref, ok ? "OK" : "FAIL");
    if (!ok) ++bad;
    hipFree(dA); hipFree(dB); hipFree(dC);
  }
  printf("%s\n", bad ? "ROWS CHECK FAILED" : "ROWS CHECK OK");
  return 0;  // results are in the output; a HIP error exits 1 (CK)
}
