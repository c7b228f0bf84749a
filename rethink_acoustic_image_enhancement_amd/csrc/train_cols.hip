// Pixel-reduction MFMA GEMM of the training step (gfx950): C(m, n) = sum_p A(m, p) B(p, n) where the
// contraction runs over pixels — the 1x1 conv weight gradient dW = dY^T X
// (Train/basicsr/models/image_restoration_model.py:213 l_pix.backward() through KDLAE_model.py:99-106,
// :127, :143) and the MDTA Gram G = q^T k / dA = dout^T v per (image, head) (KDLAE_model.py:137-138).
// Both operands are NHWC rows (channels contiguous): A(m, p) = A[p * lda + m], B(p, n) = B[p * ldb + n].
//
// Products on the bf16 matrix cores in the exact-split form of every inference GEMM (mfma3.h: each
// fp32 operand split into three bf16 planes, six v_mfma_f32_16x16x32_bf16 per 32-deep step, as
// accurate as an fp32 fma chain at 2.67x the f32 MFMA rate).  The MFMA takes k index 8 (lane >> 4)
// + j (j < 8) for both operands; any pixel order serves a contraction as long as A and B share it, so
// lane (li, lq) supplies A[pixel 4j + lq][16i + li] and B[pixel 4j + lq][16t + li], j = 0..7: one
// dword per operand tile per 4-pixel step, straight from HBM into VGPRs (16 lanes read 64 contiguous
// bytes of one pixel row; the tiles of a wave cover whole lines), the 8 dwords of a 32-pixel stage
// split in registers.  A wave owns TM x TN accumulator tiles over a pixel chunk; each loaded A value
// feeds TN MFMAs and each B value TM, so the wave moves (TM + TN) x 256 B per 4-pixel step.  The four waves of a block take neighbouring wave tiles of
// the same pixel chunk (their rows meet in L1/L2).  Pixel chunks are split-K partials
// [batch][chunk][M][N], summed in fixed order by tgemm_reduce_kernel: deterministic.
// Loads are unconditional buffer ops (rows past P / channels past M, N read 0 through the
// descriptor range), so the prefetch of the next k-steps is never drained by a dynamic vmcnt.
#include <stdint.h>

#include "mfma3.h"
#include "train_kernels.h"

namespace kdlae {
namespace train {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;  // at most 4 waves
constexpr int kU = 8;          // k-steps (4 pixels each) per pipeline stage = one 32-deep MFMA step

struct ColsArgs {
  TGemm g;
  int kchunk;     // pixels per chunk (multiple of 4 kU)
  int splits;     // chunks
  int mt, nt;     // 16-wide tiles along M and N
  int wtm, wtn;   // wave tiles along M and N
};


__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* base, long long bytes) {
  const long long cap = 0x7fffff00LL;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, (int)(bytes < cap ? bytes : cap), 0x00020000);
}
constexpr unsigned kOOB = 0x80000000u;

template <int TM, int TN, bool IMPB>
__global__ __launch_bounds__(kThreads, 2) void tgemm_cols_kernel(ColsArgs a) {
  const TGemm& g = a.g;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int wt = blockIdx.y * (int)(blockDim.x >> 6) + wave;
  if (wt >= a.wtm * a.wtn) return;  // wave-uniform; no block barrier below
  const int wm = wt / a.wtn, wn = wt - wm * a.wtn;
  const int z = blockIdx.z, z1 = z / g.nz2, z2 = z - z1 * g.nz2;
  const int ks = blockIdx.x;
  const int p0 = ks * a.kchunk, p1 = min(g.K, p0 + a.kchunk);
  // operands: A(m, p) = A[p * sak + m] (sam == 1), B(p, n) = B[p * sbk + n] (sbn == 1)
  const float* A = g.A + z1 * g.bA1 + z2 * g.bA2;
  const float* B = g.B + z1 * g.bB1 + z2 * g.bB2;
  const __amdgpu_buffer_rsrc_t ra = rsrc(A, (long long)(p1 - 1) * g.sak * 4 + 4LL * g.M);
  // (IMPB: a chunk's shifted rows reach past it, so the whole tensor; the chunks are whole 16-pixel
  // stages there, K = Bn F H W with W % 16 == 0)
  const __amdgpu_buffer_rsrc_t rb =
      IMPB ? rsrc(B, (long long)g.K * g.sbk * 4) : rsrc(B, (long long)(p1 - 1) * g.sbk * 4 + 4LL * g.N);
  // this lane's byte offset of pixel lq, column 16 tile + li, per tile (kOOB past M / N); a k-step
  // adds a wave-uniform pixel offset.  Pixels >= p1 fall past the descriptor range by themselves
  // (row stride >= M, N), so no load carries a per-lane condition.
  const unsigned sa = (unsigned)g.sak * 4u, sb = (unsigned)g.sbk * 4u;
  unsigned am[TM], bn[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = (wm * TM + i) * 16 + li;
    am[i] = m < g.M ? (unsigned)lq * sa + 4u * (unsigned)m : kOOB;
  }
  // IMPB: tile t's 16 columns are channels c0..c0+15 of one tap (Cg % 16 == 0)
  [[maybe_unused]] int tdf[TN], tdy[TN], tdx[TN], tdel[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int n = (wn * TN + t) * 16 + li;
    if constexpr (IMPB) {
      const int tap = ((wn * TN + t) * 16) / g.Cg;
      tdf[t] = tap / 9 - 1;
      tdy[t] = (tap / 3) % 3 - 1;
      tdx[t] = tap % 3 - 1;
      tdel[t] = (tdf[t] * g.H + tdy[t]) * g.W + tdx[t];
      bn[t] = n < g.N ? 4u * (unsigned)(n - tap * g.Cg) : kOOB;
    } else {
      bn[t] = n < g.N ? (unsigned)lq * sb + 4u * (unsigned)n : kOOB;
    }
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int t = 0; t < TN; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // stage = kU k-steps = 4 kU pixels: lane reads pixel q + 4u + lq for u < kU
  auto load = [&](int q, float (&av)[kU][TM], float (&bv)[kU][TN]) {
#pragma unroll
    for (int hf = 0; hf < kU / 4; ++hf) {
      // IMPB: the 16 pixels qh .. qh + 15 lie in one image row (qh % 16 == 0, W % 16 == 0)
      const int qh = q + 16 * hf;
      [[maybe_unused]] int x0 = 0, y = 0, f = 0;
      [[maybe_unused]] bool rok[TN];
      if constexpr (IMPB) {
        const int row = qh / g.W;
        x0 = qh - row * g.W;
        y = row % g.H;
        f = (row / g.H) % g.F;
#pragma unroll
        for (int t = 0; t < TN; ++t)
          rok[t] = (unsigned)(f + tdf[t]) < (unsigned)g.F && (unsigned)(y + tdy[t]) < (unsigned)g.H;
      }
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) {
        const int u = 4 * hf + uu;
        const unsigned pa = (unsigned)(q + 4 * u) * sa, pb = (unsigned)(q + 4 * u) * sb;
#pragma unroll
        for (int i = 0; i < TM; ++i)
          av[u][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra, (int)(am[i] + pa), 0, 0));
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          unsigned off;
          if constexpr (IMPB) {
            const int x = x0 + 4 * uu + lq;
            const bool ok = rok[t] && (unsigned)(x + tdx[t]) < (unsigned)g.W && bn[t] != kOOB;
            off = ok ? (unsigned)(q + 4 * u + lq + tdel[t]) * sb + bn[t] : kOOB;
          } else {
            off = bn[t] + pb;
          }
          bv[u][t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, (int)off, 0, 0));
        }
      }
    }
  };
  // One 32-deep step per stage: k index j of lane lq = pixel q + 4j + lq for both operands.  The raw
  // stage is split into bf16 planes first, then the next stage loads into the same registers while
  // this stage's MFMAs run (1.5 buffers: the planes and one raw stage).
  constexpr int kStage = 4 * kU;
  float av[kU][TM], bv[kU][TN];
  if (p0 < p1) {
    load(p0, av, bv);
    for (int q = p0; q < p1; q += kStage) {
      F3 xa[TM], xb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        xa[i] = split3(f32x4{av[0][i], av[1][i], av[2][i], av[3][i]}, f32x4{av[4][i], av[5][i], av[6][i], av[7][i]});
#pragma unroll
      for (int t = 0; t < TN; ++t)
        xb[t] = split3(f32x4{bv[0][t], bv[1][t], bv[2][t], bv[3][t]}, f32x4{bv[4][t], bv[5][t], bv[6][t], bv[7][t]});
      if (q + kStage < p1) load(q + kStage, av, bv);
#pragma unroll
      for (int t = 0; t < TN; ++t)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][t] = mfma6(xa[i], xb[t], acc[i][t]);
    }
  }
  // partial [z][ks][M][N]: lane (li, lq) of (i, t) holds rows 16(wm TM + i) + 4lq + r, column 16(wn TN + t) + li
  float* part = g.partial + ((long long)z * a.splits + ks) * g.M * g.N;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int n = (wn * TN + t) * 16 + li;
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = (wm * TM + i) * 16 + 4 * lq + r;
        if (m < g.M) part[(long long)m * g.N + n] = acc[i][t][r];
      }
    }
}

// blocks of this variant and block size (nw waves) resident on the whole chip (hipOccupancy..., cached)
template <int TM, int TN, bool IMPB>
int slots(int nw) {
  static int n[5] = {0, 0, 0, 0, 0};
  if (!n[nw]) {
    int b = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, reinterpret_cast<const void*>(&tgemm_cols_kernel<TM, TN, IMPB>),
                                                     64 * nw, 0) != hipSuccess || b < 1)
      b = 1;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || cus < 1)
      cus = 256;
    n[nw] = b * cus;
  }
  return n[nw];
}

// split count: whole rounds of resident blocks (r03 sweep: a fixed wave target was up to 40% off
// either way depending on the shape), chunks of at least KDLAE_COLS_MIN pixels, within the
// partial-buffer capacity
constexpr auto KDLAE_COLS_MIN = 256;
constexpr auto KDLAE_COLS_NARROW = 1;
template <int TM, int TN, bool IMPB>
hipError_t launch_tt(TGemm g, ColsArgs a, int nw, int gy, long long batch, size_t partial_cap, hipStream_t s) {
  long long splits = ((long long)slots<TM, TN, IMPB>(nw) + gy * batch - 1) / (gy * batch);
  const long long maxs = (g.K + KDLAE_COLS_MIN - 1) / KDLAE_COLS_MIN;
  if (splits > maxs) splits = maxs;
  const long long cap = (long long)(partial_cap / ((size_t)g.M * g.N * batch));
  if (splits > cap) splits = cap;
  if (splits < 1) return hipErrorInvalidValue;
  int kchunk = (int)((g.K + splits - 1) / splits);
  kchunk = (kchunk + 4 * kU - 1) / (4 * kU) * (4 * kU);
  splits = (g.K + kchunk - 1) / kchunk;
  a.kchunk = kchunk;
  a.splits = (int)splits;
  g.splits = (int)splits;
  a.g = g;
  hipLaunchKernelGGL((tgemm_cols_kernel<TM, TN, IMPB>), dim3((unsigned)splits, (unsigned)gy, (unsigned)batch),
                     dim3(64 * nw), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_tgemm_reduce(g, s);
}

}  // namespace

bool tgemm_cols_eligible(const TGemm& g) {
  if (g.amode != 0 || (g.bmode != 0 && g.bmode != 4) || g.alpha != 1.f || !g.partial) return false;
  if (g.sam != 1 || g.sbn != 1 || g.M <= 0 || g.N <= 0 || g.K <= 0) return false;
  if (g.bmode == 4 && (g.Cg <= 0 || g.Cg % 16 || g.W % 16 || g.N != 27 * g.Cg || g.nz1 * g.nz2 != 1 || g.F < 1 ||
                       (long long)g.Bn * g.F * g.H * g.W != g.K || g.sbk < g.Cg))
    return false;
  if ((long long)g.K * g.sak * 4 >= (1LL << 31) - 64 || (long long)g.K * g.sbk * 4 >= (1LL << 31) - 64) return false;
  return true;
}

hipError_t launch_tgemm_cols(TGemm g, size_t partial_cap, hipStream_t s) {
  if (!tgemm_cols_eligible(g)) return hipErrorInvalidValue;
  ColsArgs a;
  a.mt = (g.M + 15) / 16;
  a.nt = (g.N + 15) / 16;
  // wave tile: TM, TN in {2, 3, 4}, the least padded
  auto pick = [](int tiles) {
    int best = 4, pad = 1 << 30;
    for (int c = 4; c >= 2; --c) {
      const int p = (tiles + c - 1) / c * c;
      if (p < pad) best = c, pad = p;
    }
    return best;
  };
  const int TM = pick(a.mt), TN = (TM == 4 && pick(a.nt) == 4) ? 2 : pick(a.nt);  // 4 x 4 spills
  a.wtm = (a.mt + TM - 1) / TM;
  a.wtn = (a.nt + TN - 1) / TN;
  const int wtiles = a.wtm * a.wtn;
  // waves per block: up to 4 wave tiles of one pixel chunk; fewer wave tiles take smaller blocks
  // (a 4-wave block with one live wave puts every live wave of the CU on the same SIMD)
  const int nw = KDLAE_COLS_NARROW ? (wtiles < 4 ? wtiles : 4) : 4;
  const int gy = (wtiles + nw - 1) / nw;
  const long long batch = (long long)g.nz1 * g.nz2;
  // (bmode 4: N = 27 Cg is 27 * whole 16-tiles, so TN is 3 or 4, or 2 beside TM = 4; no other
  // implicit instance is compiled)
#define TT(m, n)                                                                                     \
  if (TM == m && TN == n) {                                                                          \
    if constexpr (n != 2 || m == 4)                                                                  \
      if (g.bmode == 4) return launch_tt<m, n, true>(g, a, nw, gy, batch, partial_cap, s);            \
    if (g.bmode == 4) return hipErrorInvalidValue;                                                    \
    return launch_tt<m, n, false>(g, a, nw, gy, batch, partial_cap, s);                               \
  }
  TT(2, 2) TT(2, 3) TT(2, 4) TT(3, 2) TT(3, 3) TT(3, 4) TT(4, 2) TT(4, 3)
#undef TT
  return hipErrorInvalidValue;
}

}  // namespace train
}  // namespace kdlae
