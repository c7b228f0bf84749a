// KDLAE-T training kernels for gfx950 (MI355X): generic MFMA GEMM with im2col / shifted-B modes and a
// deterministic split-K, LayerNorm forward/backward with wavefront-shuffle channel reductions,
// depthwise 3x3 forward (the GDFN's fused depthwise + gate and both backward passes are in
// train_dwg.hip), the MDTA softmax and its backward, PixelShuffle,
// L1LossSr, grad-norm clip and AdamW.  Every reduction over pixels is two-pass (per-block partials,
// then a fixed-order sum), so a training step is bit-reproducible run to run.
//
// Reference semantics: KDLAE/KDLAE_model.py (LayerNorm :38-83, FeedForward :89-106, Attention
// :112-145), Train/basicsr/models/losses/losses.py:135-194 (L1LossSr),
// Train/basicsr/models/image_restoration_model.py:198-218 (clip_grad_norm_ 0.01, optimizer step).
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "train_kernels.h"

namespace kdlae {
namespace train {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

static inline int grid_for(long long n, int threads, int cap = 1 << 20) {
  long long g = (n + threads - 1) / threads;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

// ---------------------------------------------------------------------------------------------- GEMM
constexpr int BN = 64, BK = 32, LDP = BN + 4;

struct Pix { int b, y, x; };

__device__ __forceinline__ Pix decompose(long long p, int H, int W) {
  const long long hw = (long long)H * W;
  Pix r;
  r.b = (int)(p / hw);
  const int rem = (int)(p - (long long)r.b * hw);
  r.y = rem / W;
  r.x = rem - r.y * W;
  return r;
}

template <int AM>
__device__ __forceinline__ float a_at(const TGemm& g, const float* A, int m, int k, const Pix& pm) {
  if (m >= g.M || k >= g.K) return 0.f;
  if (AM == 0) return A[(long long)m * g.sam + (long long)k * g.sak];
  const int tap = k / g.Cg, c = k - tap * g.Cg;
  const int yy = pm.y + (tap / 3 - 1) * g.dil, xx = pm.x + (tap % 3 - 1) * g.dil;
  if (yy < 0 || yy >= g.H || xx < 0 || xx >= g.W) return 0.f;
  return A[(((long long)pm.b * g.H + yy) * g.W + xx) * g.lda + c];
}

// address of A(m, k..k+3) when those four are contiguous (null -> out of image: zeros)
template <int AM>
__device__ __forceinline__ const float* a_vec_ptr(const TGemm& g, const float* A, int m, int k, const Pix& pm) {
  if (AM == 0) return A + (long long)m * g.sam + k;
  const int tap = k / g.Cg, c = k - tap * g.Cg;
  const int yy = pm.y + (tap / 3 - 1) * g.dil, xx = pm.x + (tap % 3 - 1) * g.dil;
  if (yy < 0 || yy >= g.H || xx < 0 || xx >= g.W) return nullptr;
  return A + (((long long)pm.b * g.H + yy) * g.W + xx) * g.lda + c;
}

template <int BMODE>
__device__ __forceinline__ float b_at(const TGemm& g, const float* B, int k, int n, const Pix& pk, int tap) {
  if (k >= g.K || n >= g.N) return 0.f;
  if (BMODE == 0) return B[(long long)k * g.sbk + (long long)n * g.sbn];
  if (BMODE == 1) {
    const int yy = pk.y + (tap / 3 - 1) * g.dil, xx = pk.x + (tap % 3 - 1) * g.dil;
    if (yy < 0 || yy >= g.H || xx < 0 || xx >= g.W) return 0.f;
    return B[(((long long)pk.b * g.H + yy) * g.W + xx) * g.ldb + n];
  }
  const int t = k / g.Cg, c = k - t * g.Cg;
  if (BMODE == 2) return B[((long long)n * g.Cg + c) * 9 + t];
  return B[((long long)c * g.N + n) * 9 + (8 - t)];
}

__device__ __forceinline__ float epi(const TGemm& g, float acc, int m, int n, const float* R, const float* rs) {
  float v = g.alpha * acc;
  if (g.bias) v += g.bias[n];
  if (R) {
    const float r = R[(long long)m * g.srm + (long long)n * g.srn];
    v += rs ? rs[n] * r : r;
  }
  return v;
}

__device__ __forceinline__ void put4(float* d, const float4& v) { *reinterpret_cast<float4*>(d) = v; }
__device__ __forceinline__ float4 get4(const float* s) { return *reinterpret_cast<const float4*>(s); }

// Shared GEMM epilogue: C/D lane map col = lane & 15, row = 4 * (lane >> 4) + r.  With flags & 4 the
// (64 RM) x 64 tile is staged in LDS (smem, >= 64 RM x (BN + 4) floats) and each thread writes 16
// consecutive columns of one row per round; split-K blocks store raw partial sums.
template <int RM>
__device__ __forceinline__ void store_tile(const TGemm& g, int flags, float* smem, const f32x4 (&acc)[2 * RM][2],
                                           int m0, int n0, int z, int z1, int z2, int ks) {
  constexpr int LDC = BN + 4;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv & 1, wn = wv >> 1;
  const bool split = g.splits > 1;
  float* C = g.C + z1 * g.bC1 + z2 * g.bC2;
  const float* R = g.R ? g.R + z1 * g.bR1 + z2 * g.bR2 : nullptr;
  const float* rs = g.rs ? g.rs + z1 * g.brs1 + z2 * g.brs2 : nullptr;
  float* part = split ? g.partial + ((long long)z * g.splits + ks) * g.M * g.N : nullptr;
  if (flags & 4) {
    // stage the tile in LDS, then each thread writes 16 consecutive columns of one row per round
    float* Cs = smem;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2 * RM; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(wm * 32 * RM + i * 16 + 4 * (lane >> 4) + r) * LDC + wn * 32 + j * 16 + (lane & 15)] = acc[i][j][r];
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < RM; ++rr) {
      const int row = 64 * rr + (tid >> 2), cb = (tid & 3) * 16;
      const int m = m0 + row;
      if (m >= g.M) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = n0 + cb + 4 * q;
        if (n >= g.N) break;
        float4 v = get4(Cs + row * LDC + cb + 4 * q);
        if (n + 3 < g.N) {
          if (split) {
            put4(part + (long long)m * g.N + n, v);
          } else {
            v.x = epi(g, v.x, m, n, R, rs);
            v.y = epi(g, v.y, m, n + 1, R, rs);
            v.z = epi(g, v.z, m, n + 2, R, rs);
            v.w = epi(g, v.w, m, n + 3, R, rs);
            put4(C + (long long)m * g.scm + n, v);
          }
        } else {
          const float vv[4] = {v.x, v.y, v.z, v.w};
          for (int e = 0; e < 4 && n + e < g.N; ++e) {
            if (split) part[(long long)m * g.N + n + e] = vv[e];
            else C[(long long)m * g.scm + n + e] = epi(g, vv[e], m, n + e, R, rs);
          }
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2 * RM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 * RM + i * 16 + 4 * (lane >> 4) + r;
        const int n = n0 + wn * 32 + j * 16 + (lane & 15);
        if (m >= g.M || n >= g.N) continue;
        if (split) part[(long long)m * g.N + n] = acc[i][j][r];
        else C[(long long)m * g.scm + (long long)n * g.scn] = epi(g, acc[i][j][r], m, n, R, rs);
      }
}

// (64*RM)x64 block tile, BK = 32, 4 waves of (32*RM)x32 (2RM x 2 v_mfma_f32_16x16x4_f32 tiles).
// Global -> register prefetch of the next k-tile overlaps the MFMAs of the current one; 8 consecutive
// elements per thread along the contiguous operand dimension, as two float4 loads when the `flags`
// say they are aligned.  The C tile is staged through LDS so stores go out as whole 256 B rows.
// RM = 2 (128-row tiles) halves the B-operand LDS traffic per MFMA on the tall activation GEMMs.
// flags: 1 = A vector loads, 2 = B vector loads, 4 = C row stores (scn == 1, aligned)
template <int AM, int BMODE, int RM>
__global__ __launch_bounds__(256) void tgemm_kernel(TGemm g, int kchunk, int flags) {
  constexpr int BMr = 64 * RM, LDA_S = BMr + 4, LDC = BN + 4;
  constexpr int SM_LOOP = BK * LDA_S + BK * LDP, SM_EPI = BMr * LDC;
  __shared__ float smem[SM_LOOP > SM_EPI ? SM_LOOP : SM_EPI];
  float (*As)[LDA_S] = reinterpret_cast<float (*)[LDA_S]>(smem);
  float (*Bs)[LDP] = reinterpret_cast<float (*)[LDP]>(smem + BK * LDA_S);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv & 1, wn = wv >> 1;
  const int tiles_n = (g.N + BN - 1) / BN;
  // XCD-aware order: dispatch id d runs on XCD d % 8; logical tiles [x*per, (x+1)*per) go to XCD x, so
  // the n-tiles of one row block (consecutive logical ids) share that XCD's L2 copy of their A rows.
  // The grid is padded to a multiple of 8; the padding blocks exit.
  // (flags & 8: remap on; only for single-split grids of >= 64 tiles, where every XCD gets work)
  const int tiles_m = (g.M + BMr - 1) / BMr;
  const int per = (int)(gridDim.x >> 3);
  const int tile = (flags & 8) ? (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  if (tile >= tiles_m * tiles_n) return;
  const int m0 = (tile / tiles_n) * BMr, n0 = (tile % tiles_n) * BN;
  const int z = blockIdx.z, z1 = z / g.nz2, z2 = z - z1 * g.nz2;
  const float* A = g.A + z1 * g.bA1 + z2 * g.bA2;
  const float* B = g.B + (BMODE == 1 ? z1 * g.bB1 : z1 * g.bB1 + z2 * g.bB2);
  const int ks = blockIdx.y;
  const int kbeg = ks * kchunk, kend = min(g.K, kbeg + kchunk);
  const bool vecA = flags & 1, vecB = flags & 2;

  // per-thread 8-element runs: a_kc -> (row m, k..k+7); else (k, m..m+7).  Same for B.
  const bool a_kc = (AM == 1) || (g.sak == 1);
  const bool b_nc = (BMODE == 1) || (BMODE == 0 && g.sbn == 1);
  const int a_m = a_kc ? (tid >> 2) : (tid & 7) * 8;
  const int a_k = a_kc ? (tid & 3) * 8 : (tid >> 3);
  const int b_k = b_nc ? (tid >> 3) : (tid & 3) * 8;
  const int b_n = b_nc ? (tid & 7) * 8 : (tid >> 2);
  Pix pa[RM];
#pragma unroll
  for (int rr = 0; rr < RM; ++rr) {
    pa[rr] = Pix{0, 0, 0};
    if (AM == 1 && m0 + 64 * rr + a_m < g.M) pa[rr] = decompose(m0 + 64 * rr + a_m, g.H, g.W);
  }

  float ra[8 * RM], rb[8];
  auto load = [&](int k0) {
#pragma unroll
    for (int rr = 0; rr < RM; ++rr) {
      float* r8 = ra + 8 * rr;
      if (a_kc) {
        const int m = m0 + 64 * rr + a_m;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int k = k0 + a_k + 4 * h;
          if (vecA && m < g.M && k + 3 < kend) {
            const float* ptr = a_vec_ptr<AM>(g, A, m, k, pa[rr]);
            const float4 v = ptr ? get4(ptr) : make_float4(0.f, 0.f, 0.f, 0.f);
            r8[4 * h] = v.x; r8[4 * h + 1] = v.y; r8[4 * h + 2] = v.z; r8[4 * h + 3] = v.w;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) r8[4 * h + e] = (k + e < kend) ? a_at<AM>(g, A, m, k + e, pa[rr]) : 0.f;
          }
        }
      } else {
        const int k = k0 + a_k;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int m = m0 + 64 * rr + a_m + 4 * h;
          if (vecA && k < kend && m + 3 < g.M) {
            const float4 v = get4(A + (long long)k * g.sak + m);
            r8[4 * h] = v.x; r8[4 * h + 1] = v.y; r8[4 * h + 2] = v.z; r8[4 * h + 3] = v.w;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) r8[4 * h + e] = (k < kend) ? a_at<AM>(g, A, m + e, k, pa[rr]) : 0.f;
          }
        }
      }
    }
    if (b_nc) {
      const int k = k0 + b_k;
      Pix pk{0, 0, 0};
      if (BMODE == 1 && k < kend) pk = decompose(k, g.H, g.W);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int n = n0 + b_n + 4 * h;
        if (vecB && k < kend && n + 3 < g.N) {
          const float* ptr = nullptr;
          if (BMODE == 0) ptr = B + (long long)k * g.sbk + n;
          else {
            const int yy = pk.y + (z2 / 3 - 1) * g.dil, xx = pk.x + (z2 % 3 - 1) * g.dil;
            if (yy >= 0 && yy < g.H && xx >= 0 && xx < g.W) ptr = B + (((long long)pk.b * g.H + yy) * g.W + xx) * g.ldb + n;
          }
          const float4 v = ptr ? get4(ptr) : make_float4(0.f, 0.f, 0.f, 0.f);
          rb[4 * h] = v.x; rb[4 * h + 1] = v.y; rb[4 * h + 2] = v.z; rb[4 * h + 3] = v.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) rb[4 * h + e] = (k < kend) ? b_at<BMODE>(g, B, k, n + e, pk, z2) : 0.f;
        }
      }
    } else {
      const int n = n0 + b_n;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = k0 + b_k + 4 * h;
        if (BMODE == 0 && vecB && n < g.N && k + 3 < kend) {
          const float4 v = get4(B + (long long)n * g.sbn + k);
          rb[4 * h] = v.x; rb[4 * h + 1] = v.y; rb[4 * h + 2] = v.z; rb[4 * h + 3] = v.w;
        } else {
          Pix pk{0, 0, 0};
#pragma unroll
          for (int e = 0; e < 4; ++e) rb[4 * h + e] = (k + e < kend) ? b_at<BMODE>(g, B, k + e, n, pk, z2) : 0.f;
        }
      }
    }
  };

  f32x4 acc[2 * RM][2];
#pragma unroll
  for (int i = 0; i < 2 * RM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kbeg < kend) load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < RM; ++rr)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (a_kc) As[a_k + e][64 * rr + a_m] = ra[8 * rr + e];
        else As[a_k][64 * rr + a_m + e] = ra[8 * rr + e];
      }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (b_nc) Bs[b_k][b_n + e] = rb[e];
      else Bs[b_k + e][b_n] = rb[e];
    }
    __syncthreads();
    if (k0 + BK < kend) load(k0 + BK);
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      const int kr = kk * 4 + (lane >> 4);
      float av[2 * RM], bv[2];
#pragma unroll
      for (int i = 0; i < 2 * RM; ++i) av[i] = As[kr][wm * 32 * RM + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = Bs[kr][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2 * RM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma4(av[i], bv[j], acc[i][j]);
    }
  }

  // epilogue: C/D lane map col = lane & 15, row = 4 * (lane >> 4) + r
  store_tile<RM>(g, flags, smem, acc, m0, n0, z, z1, z2, ks);
}

// Lean variant for plain strided operands whose 8-element runs are float4-aligned (amode 0, bmode 0,
// flags 1|2 — every 1x1 conv forward / dX / dW and every MDTA contraction of the training step): the
// operand layouts are template parameters (AKC: A k-contiguous, BNC: B n-contiguous), each thread's
// operand pointers are formed once, and per-element bounds checks run only in edge tiles (the generic
// kernel spent ~10 VALU/SALU instructions per MFMA on them: r01 PMC, `tools/micro/tgemm_bench.cpp`).
template <bool AKC, bool BNC, int RM>
__global__ __launch_bounds__(256) void tgemm_lean_kernel(TGemm g, int kchunk, int flags) {
  constexpr int BMr = 64 * RM, LDA_S = BMr + 4, LDC = BN + 4;
  constexpr int SM_LOOP = BK * LDA_S + BK * LDP, SM_EPI = BMr * LDC;
  __shared__ __attribute__((aligned(16))) float smem[SM_LOOP > SM_EPI ? SM_LOOP : SM_EPI];
  float (*As)[LDA_S] = reinterpret_cast<float (*)[LDA_S]>(smem);
  float (*Bs)[LDP] = reinterpret_cast<float (*)[LDP]>(smem + BK * LDA_S);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv & 1, wn = wv >> 1;
  const int tiles_n = (g.N + BN - 1) / BN;
  const int tiles_m = (g.M + BMr - 1) / BMr;
  const int per = (int)(gridDim.x >> 3);
  const int tile = (flags & 8) ? (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  if (tile >= tiles_m * tiles_n) return;
  const int m0 = (tile / tiles_n) * BMr, n0 = (tile % tiles_n) * BN;
  const int z = blockIdx.z, z1 = z / g.nz2, z2 = z - z1 * g.nz2;
  const float* A = g.A + z1 * g.bA1 + z2 * g.bA2;
  const float* B = g.B + z1 * g.bB1 + z2 * g.bB2;
  const int ks = blockIdx.y;
  const int kbeg = ks * kchunk, kend = min(g.K, kbeg + kchunk);

  const int a_m = AKC ? (tid >> 2) : (tid & 7) * 8;
  const int a_k = AKC ? (tid & 3) * 8 : (tid >> 3);
  const int b_k = BNC ? (tid >> 3) : (tid & 3) * 8;
  const int b_n = BNC ? (tid & 7) * 8 : (tid >> 2);
  const float* pa[RM];
  int mrow[RM];
#pragma unroll
  for (int rr = 0; rr < RM; ++rr) {
    mrow[rr] = m0 + 64 * rr + a_m;
    pa[rr] = AKC ? A + (long long)mrow[rr] * g.sam + a_k : A + mrow[rr] + (long long)a_k * g.sak;
  }
  const int ncol = n0 + b_n;
  const float* pb = BNC ? B + ncol + (long long)b_k * g.sbk : B + (long long)ncol * g.sbn + b_k;

  float ra[8 * RM], rb[8];
  auto put8 = [](float* r, const float4& v0, const float4& v1) {
    r[0] = v0.x; r[1] = v0.y; r[2] = v0.z; r[3] = v0.w;
    r[4] = v1.x; r[5] = v1.y; r[6] = v1.z; r[7] = v1.w;
  };
  auto load = [&](int k0) {
    const bool kfull = k0 + BK <= kend;  // uniform: only the last k-tile of a split needs k checks
#pragma unroll
    for (int rr = 0; rr < RM; ++rr) {
      float* r = ra + 8 * rr;
      if (AKC) {
        const float* q = pa[rr] + k0;
        if (mrow[rr] < g.M && kfull) {
          put8(r, get4(q), get4(q + 4));
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) r[e] = (mrow[rr] < g.M && k0 + a_k + e < kend) ? q[e] : 0.f;
        }
      } else {
        const float* q = pa[rr] + (long long)k0 * g.sak;
        const bool kok = k0 + a_k < kend;
        if (kok && mrow[rr] + 7 < g.M) {
          put8(r, get4(q), get4(q + 4));
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) r[e] = (kok && mrow[rr] + e < g.M) ? q[e] : 0.f;
        }
      }
    }
    if (BNC) {
      const float* q = pb + (long long)k0 * g.sbk;
      const bool kok = k0 + b_k < kend;
      if (kok && ncol + 7 < g.N) {
        put8(rb, get4(q), get4(q + 4));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) rb[e] = (kok && ncol + e < g.N) ? q[e] : 0.f;
      }
    } else {
      const float* q = pb + k0;
      if (ncol < g.N && kfull) {
        put8(rb, get4(q), get4(q + 4));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) rb[e] = (ncol < g.N && k0 + b_k + e < kend) ? q[e] : 0.f;
      }
    }
  };

  f32x4 acc[2 * RM][2];
#pragma unroll
  for (int i = 0; i < 2 * RM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kbeg < kend) load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < RM; ++rr)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (AKC) As[a_k + e][64 * rr + a_m] = ra[8 * rr + e];
        else As[a_k][64 * rr + a_m + e] = ra[8 * rr + e];
      }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (BNC) Bs[b_k][b_n + e] = rb[e];
      else Bs[b_k + e][b_n] = rb[e];
    }
    __syncthreads();
    if (k0 + BK < kend) load(k0 + BK);
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      const int kr = kk * 4 + (lane >> 4);
      float av[2 * RM], bv[2];
#pragma unroll
      for (int i = 0; i < 2 * RM; ++i) av[i] = As[kr][wm * 32 * RM + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = Bs[kr][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2 * RM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma4(av[i], bv[j], acc[i][j]);
    }
  }

  store_tile<RM>(g, flags, smem, acc, m0, n0, z, z1, z2, ks);
}

// split-K reduce: a block owns 64 consecutive outputs of one batch entry; 16 waves each sum every 16th
// split (4 independent chains), combined in fixed order, then the epilogue -> deterministic
// Fixed-order split-K sum: wave w of a 16-wave block sums splits w, w + 16, ... (4 interleaved
// accumulators), the 16 wave sums are added in order, then the epilogue.  With vec (M N % 4 == 0,
// 16-byte aligned partials) a lane sums 4 consecutive outputs as one float4 — the same arithmetic per
// output as the scalar path, in a quarter of the load instructions.
__global__ __launch_bounds__(1024) void tgemm_reduce_kernel(TGemm g, int vec) {
  __shared__ f32x4 red[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int V = vec ? 4 : 1;
  const long long MN = (long long)g.M * g.N;
  const long long mn = ((long long)blockIdx.x * 64 + lane) * V;
  const int z = blockIdx.y;
  f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
  if (mn < MN) {
    const float* part = g.partial + (long long)z * g.splits * MN + mn;
    f32x4 a0 = a, a1 = a, a2 = a, a3 = a;
    auto ld = [&](int k) -> f32x4 {
      const float* p = part + (long long)k * MN;
      return vec ? *reinterpret_cast<const f32x4*>(p) : f32x4{p[0], 0.f, 0.f, 0.f};
    };
    int k = wv;
    for (; k + 48 < g.splits; k += 64) {
      a0 += ld(k);
      a1 += ld(k + 16);
      a2 += ld(k + 32);
      a3 += ld(k + 48);
    }
    for (; k < g.splits; k += 16) a0 += ld(k);
    a = (a0 + a1) + (a2 + a3);
  }
  red[wv][lane] = a;
  __syncthreads();
  if (wv != 0 || mn >= MN) return;
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 16; ++k) s += red[k][lane];
  const int z1 = z / g.nz2, z2 = z - z1 * g.nz2;
  float* C = g.C + z1 * g.bC1 + z2 * g.bC2;
  const float* R = g.R ? g.R + z1 * g.bR1 + z2 * g.bR2 : nullptr;
  const float* rs = g.rs ? g.rs + z1 * g.brs1 + z2 * g.brs2 : nullptr;
  for (int e = 0; e < V; ++e) {
    const long long i = mn + e;
    const int m = (int)(i / g.N), n = (int)(i - (long long)m * g.N);
    C[(long long)m * g.scm + (long long)n * g.scn] = epi(g, s[e], m, n, R, rs);
  }
}

template <int AM, int BMODE>
static void launch_t(const TGemm& g, int kchunk, int flags, int rm, dim3 grid, hipStream_t s) {
  if (rm == 2) hipLaunchKernelGGL((tgemm_kernel<AM, BMODE, 2>), grid, dim3(256), 0, s, g, kchunk, flags);
  else hipLaunchKernelGGL((tgemm_kernel<AM, BMODE, 1>), grid, dim3(256), 0, s, g, kchunk, flags);
}

static inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

constexpr auto KDLAE_SPLITK_BLOCKS = 2048;
constexpr auto KDLAE_SPLITK_MIN = 256;
constexpr auto KDLAE_TRAIN_ROWS = 1;
constexpr auto KDLAE_TRAIN_COLS = 1;
constexpr auto KDLAE_RED_VEC = 1;
hipError_t launch_tgemm_reduce(const TGemm& g, hipStream_t s) {
  const long long MN = (long long)g.M * g.N;
  const int vec = KDLAE_RED_VEC && MN % 4 == 0 && al16(g.partial);
  const long long per = vec ? 256 : 64;
  hipLaunchKernelGGL(tgemm_reduce_kernel, dim3((unsigned)((MN + per - 1) / per), (unsigned)(g.nz1 * g.nz2)), dim3(1024),
                     0, s, g, vec);
  return hipGetLastError();
}

hipError_t launch_tgemm(TGemm g, size_t partial_cap, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  // r03 per-shape sweep (tools/micro/rows_bench.cpp, profiles/r03_train_gemm_bench.txt): the row-
  // streaming and pixel-reduction kernels win 25-55% on the tall contractions; on the 64^2 / 32^2
  // levels (a few thousand rows, K or N up to 2042) the tiled kernel's finer grid is faster
  const long long rows = (long long)g.M * g.nz1 * g.nz2;
  if (KDLAE_TRAIN_ROWS && !g.partial && (rows >= 65536 || (rows >= 24576 && g.K <= 256)) && tgemm_rows_eligible(g))
    return launch_tgemm_rows(g, s);
  if (KDLAE_TRAIN_COLS && g.partial && partial_cap > 0 && (long long)g.K * g.nz1 * g.nz2 >= 16384 &&
      tgemm_cols_eligible(g))
    return launch_tgemm_cols(g, partial_cap, s);
  return launch_tgemm_tiled(g, partial_cap, s);
}

hipError_t launch_tgemm_tiled(TGemm g, size_t partial_cap, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  const long long batch = (long long)g.nz1 * g.nz2;
  // 128-row tiles when the grid still holds >= 2 blocks per CU with them (tall activation GEMMs)
  const int rm = (g.bmode != 1 && (long long)((g.M + 127) / 128) * ((g.N + BN - 1) / BN) * batch >= 512) ? 2 : 1;
  const int tiles = ((g.M + 64 * rm - 1) / (64 * rm)) * ((g.N + BN - 1) / BN);
  int splits = 1;
  // implicit-GEMM convolutions (amode 1) split only when their tiles leave the chip mostly idle:
  // r03 trace, splitting the 384-768-tile shapes as well was 20-110% slower (the partial round trip
  // outweighs the fuller grid), the 72-144-tile Upsample convs 18-71% faster; of the 288-tile
  // shapes, the K = 3456 ones gain (16^2 / 32^2 Upsample fwd / dX 427 -> 318, 330 -> 205 us) and the
  // K = 864 ones lose 10-20% (r03 A/B, gpurun_out/ab_sp)
  const long long ctiles = (long long)tiles * batch;
  const bool split_ok = g.amode != 1 || ctiles < 256 || (ctiles < 512 && g.K >= 1728);
  if (g.partial && partial_cap > 0 && split_ok) {
    // fill ~KDLAE_SPLITK_BLOCKS blocks, each split at least KDLAE_SPLITK_MIN deep
    const long long blocks = tiles * batch;
    long long want = (KDLAE_SPLITK_BLOCKS + blocks - 1) / blocks;
    const long long maxk = (g.K + KDLAE_SPLITK_MIN - 1) / KDLAE_SPLITK_MIN;
    if (want > maxk) want = maxk;
    const long long cap = (long long)(partial_cap / ((size_t)g.M * g.N * batch));
    if (want > cap) want = cap;
    if (want > 1) splits = (int)want;
  }
  int kchunk = (g.K + splits - 1) / splits;
  kchunk = (kchunk + BK - 1) / BK * BK;
  splits = (g.K + kchunk - 1) / kchunk;
  if (splits < 1) splits = 1;
  g.splits = splits;
  // vector-load / row-store eligibility (all offsets multiples of 4 floats, bases 16 B aligned)
  auto m4 = [](long long v) { return (v & 3) == 0; };
  int flags = 0;
  const bool a_kc = g.amode == 1 || g.sak == 1;
  if (g.amode == 1) {
    if (al16(g.A) && m4(g.lda) && g.Cg % 4 == 0 && m4(g.bA1) && m4(g.bA2)) flags |= 1;
  } else if (al16(g.A) && m4(g.bA1) && m4(g.bA2) && (a_kc ? m4(g.sam) : (g.sam == 1 && m4(g.sak)))) {
    flags |= 1;
  }
  if (g.bmode == 1) {
    if (al16(g.B) && m4(g.ldb) && m4(g.bB1)) flags |= 2;
  } else if (g.bmode == 0 && al16(g.B) && m4(g.bB1) && m4(g.bB2) &&
             ((g.sbn == 1 && m4(g.sbk)) || (g.sbk == 1 && m4(g.sbn)))) {
    flags |= 2;
  }
  if (splits > 1 ? (g.N % 4 == 0 && al16(g.partial))
                 : (g.scn == 1 && al16(g.C) && m4(g.scm) && m4(g.bC1) && m4(g.bC2)))
    flags |= 4;
  const bool xcd = splits == 1 && batch == 1 && tiles >= 64;
  if (xcd) flags |= 8;
  dim3 grid(xcd ? (tiles + 7) / 8 * 8 : tiles, splits, (unsigned)batch);
  if (g.amode == 0 && g.bmode == 0 && (flags & 3) == 3) {
    const bool akc = g.sak == 1, bnc = g.sbn == 1;
#define LEAN(a, b, r) hipLaunchKernelGGL((tgemm_lean_kernel<a, b, r>), grid, dim3(256), 0, s, g, kchunk, flags)
    if (rm == 2) {
      if (akc && bnc) LEAN(true, true, 2); else if (akc) LEAN(true, false, 2);
      else if (bnc) LEAN(false, true, 2); else LEAN(false, false, 2);
    } else {
      if (akc && bnc) LEAN(true, true, 1); else if (akc) LEAN(true, false, 1);
      else if (bnc) LEAN(false, true, 1); else LEAN(false, false, 1);
    }
#undef LEAN
  } else if (g.amode == 0 && g.bmode == 0) {
    launch_t<0, 0>(g, kchunk, flags, rm, grid, s);
  }
  // (the conv weight gradient's M = C_out never reaches 512 tiles of 128 rows: 64-row tiles only)
  else if (g.amode == 0 && g.bmode == 1) hipLaunchKernelGGL((tgemm_kernel<0, 1, 1>), grid, dim3(256), 0, s, g, kchunk, flags);
  else if (g.amode == 1 && g.bmode == 0) launch_t<1, 0>(g, kchunk, flags, rm, grid, s);
  else if (g.amode == 1 && g.bmode == 2) launch_t<1, 2>(g, kchunk, flags, rm, grid, s);
  else if (g.amode == 1 && g.bmode == 3) launch_t<1, 3>(g, kchunk, flags, rm, grid, s);
  else return hipErrorInvalidValue;
  if (splits > 1) return launch_tgemm_reduce(g, s);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------- LayerNorm
// One wave per pixel, channel c = lane + 64 i (V values per lane), wavefront-shuffle sums; NP pixels
// per iteration so their loads are in flight together (the per-pixel chain is latency bound).
constexpr int LN_NP = 4;

template <int V>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, int ldx, const float* __restrict__ w,
                                                     const float* __restrict__ b, int C, long long P, int biasfree,
                                                     float* __restrict__ y, int ldy, float* __restrict__ stats) {
  const int lane = threadIdx.x & 63;
  const long long nw = (long long)gridDim.x * 4;
  for (long long p0 = blockIdx.x * 4LL + (threadIdx.x >> 6); p0 < P; p0 += nw * LN_NP) {
    float v[LN_NP][V];
#pragma unroll
    for (int q = 0; q < LN_NP; ++q) {
      const long long p = p0 + q * nw;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int c = lane + 64 * i;
        v[q][i] = (p < P && c < C) ? x[p * ldx + c] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < LN_NP; ++q) {
      const long long p = p0 + q * nw;
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < V; ++i) s += v[q][i];
      const float mu = wave_sum(s) / C;
      float qq = 0.f;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int c = lane + 64 * i;
        if (c < C) qq += (v[q][i] - mu) * (v[q][i] - mu);
      }
      const float var = wave_sum(qq) / C;
      const float sd = sqrtf(var + 1e-5f);
      if (p >= P) continue;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int c = lane + 64 * i;
        if (c < C) y[p * ldy + c] = biasfree ? v[q][i] / sd * w[c] : (v[q][i] - mu) / sd * w[c] + b[c];
      }
      if (lane == 0) {
        stats[2 * p] = mu;
        stats[2 * p + 1] = 1.f / sd;
      }
    }
  }
}

template <int V>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy, int ldd, const float* __restrict__ x,
                                                     int ldx, const float* __restrict__ w,
                                                     const float* __restrict__ stats, int C, long long P, int biasfree,
                                                     const float* R, int ldr, float* dx, int lddx,
                                                     float* __restrict__ part) {
  __shared__ float red[4][2 * 64 * V];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float aw[V], ab[V], wr[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    aw[i] = ab[i] = 0.f;
    const int c = lane + 64 * i;
    wr[i] = c < C ? w[c] : 0.f;
  }
  const long long nw = (long long)gridDim.x * 4;
  for (long long p0 = blockIdx.x * 4LL + wv; p0 < P; p0 += nw * LN_NP) {
    float xv[LN_NP][V], dv[LN_NP][V], rv[LN_NP][V], mu[LN_NP], r[LN_NP];
#pragma unroll
    for (int q = 0; q < LN_NP; ++q) {
      const long long p = p0 + q * nw;
      const bool ok = p < P;
      mu[q] = ok ? stats[2 * p] : 0.f;
      r[q] = ok ? stats[2 * p + 1] : 0.f;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int c = lane + 64 * i;
        const bool live = ok && c < C;
        dv[q][i] = live ? dy[p * ldd + c] : 0.f;
        xv[q][i] = live ? x[p * ldx + c] : 0.f;
        rv[q][i] = (live && R) ? R[p * ldr + c] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < LN_NP; ++q) {
      const long long p = p0 + q * nw;
      float s1 = 0.f, s2 = 0.f, gv[V];
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const float xh = biasfree ? xv[q][i] * r[q] : (xv[q][i] - mu[q]) * r[q];
        aw[i] += dv[q][i] * xh;
        ab[i] += dv[q][i];
        gv[i] = dv[q][i] * wr[i];
        s1 += gv[i] * (biasfree ? xv[q][i] : xh);
        s2 += gv[i];
      }
      s1 = wave_sum(s1) / C;
      s2 = wave_sum(s2) / C;
      if (p >= P) continue;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int c = lane + 64 * i;
        if (c >= C) continue;
        const float rq = r[q];
        float d;
        if (biasfree) d = rq * gv[i] - rq * rq * rq * (xv[q][i] - mu[q]) * s1;
        else d = rq * (gv[i] - s2 - (xv[q][i] - mu[q]) * rq * s1);
        dx[p * lddx + c] = d + rv[q][i];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) {
    red[wv][64 * i + lane] = aw[i];
    red[wv][64 * V + 64 * i + lane] = ab[i];
  }
  __syncthreads();
  const int ncol = biasfree ? C : 2 * C;
  for (int c = threadIdx.x; c < ncol; c += blockDim.x) {
    const int off = c < C ? c : 64 * V + (c - C);
    part[(long long)blockIdx.x * ncol + c] = ((red[0][off] + red[1][off]) + red[2][off]) + red[3][off];
  }
}

#define LN_DISPATCH(KERNEL, grid, ...)                                                           \
  do {                                                                                            \
    if (C <= 64) hipLaunchKernelGGL((KERNEL<1>), grid, dim3(256), 0, s, __VA_ARGS__);               \
    else if (C <= 128) hipLaunchKernelGGL((KERNEL<2>), grid, dim3(256), 0, s, __VA_ARGS__);         \
    else if (C <= 256) hipLaunchKernelGGL((KERNEL<4>), grid, dim3(256), 0, s, __VA_ARGS__);         \
    else hipLaunchKernelGGL((KERNEL<8>), grid, dim3(256), 0, s, __VA_ARGS__);                       \
  } while (0)

// Lane-group variant (r03) for float4-aligned views: G lanes share a pixel (G = 16 / 32 / 64 for
// C <= 64 / 128 / 256, and 64 lanes x 2 quads up to 512), each lane NV float4 quads, 64 / G pixels
// per wave, shuffle sums over log2(G) steps instead of a 6-step full-wave reduction per pixel and
// statistic.  The one-wave-per-pixel kernels above left 25-40 of 64 lanes idle at C = 48 / 96
// (1.9 TB/s on the 393216-pixel sr-branch LayerNorm).
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <int G, int NV>
__global__ __launch_bounds__(256) void ln2_fwd_kernel(const float* __restrict__ x, int ldx, const float* __restrict__ w,
                                                      const float* __restrict__ b, int C, long long P, int biasfree,
                                                      float* __restrict__ y, int ldy, float* __restrict__ stats) {
  constexpr int PPW = 64 / G;  // pixels per wave
  const int lane = threadIdx.x & 63, gl = lane % G, gp = lane / G;
  const int Cq = C >> 2;
  f32x4 wv[NV], bv[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int q = gl + G * j;
    wv[j] = q < Cq ? *reinterpret_cast<const f32x4*>(w + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    bv[j] = (q < Cq && b) ? *reinterpret_cast<const f32x4*>(b + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const long long nwave = (long long)gridDim.x * 4;
  const float invC = 1.f / C;
  for (long long p0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * PPW; p0 < P; p0 += nwave * PPW) {
    const long long p = p0 + gp;
    const bool live = p < P;
    f32x4 v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int q = gl + G * j;
      v[j] = (live && q < Cq) ? *reinterpret_cast<const f32x4*>(x + p * ldx + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
    const float mu = group_sum<G>(s) * invC;
    float qq = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j)
      if (gl + G * j < Cq)
#pragma unroll
        for (int e = 0; e < 4; ++e) qq += (v[j][e] - mu) * (v[j][e] - mu);
    const float var = group_sum<G>(qq) * invC;
    const float sd = sqrtf(var + 1e-5f);
    if (!live) continue;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int q = gl + G * j;
      if (q >= Cq) continue;
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = biasfree ? v[j][e] / sd * wv[j][e] : (v[j][e] - mu) / sd * wv[j][e] + bv[j][e];
      *reinterpret_cast<f32x4*>(y + p * ldy + 4 * q) = o;
    }
    if (gl == 0) {
      stats[2 * p] = mu;
      stats[2 * p + 1] = 1.f / sd;
    }
  }
}

template <int G, int NV>
__global__ __launch_bounds__(256) void ln2_bwd_kernel(const float* __restrict__ dy, int ldd, const float* __restrict__ x,
                                                      int ldx, const float* __restrict__ w,
                                                      const float* __restrict__ stats, int C, long long P, int biasfree,
                                                      const float* R, int ldr, float* dx, int lddx,
                                                      float* __restrict__ part) {
  constexpr int PPW = 64 / G;
  __shared__ f32x4 red[4][2][G * NV];
  const int lane = threadIdx.x & 63, wv_ = threadIdx.x >> 6, gl = lane % G, gp = lane / G;
  const int Cq = C >> 2;
  f32x4 wr[NV], aw[NV], ab[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int q = gl + G * j;
    wr[j] = q < Cq ? *reinterpret_cast<const f32x4*>(w + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    aw[j] = ab[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const long long nwave = (long long)gridDim.x * 4;
  const float invC = 1.f / C;
  for (long long p0 = ((long long)blockIdx.x * 4 + wv_) * PPW; p0 < P; p0 += nwave * PPW) {
    const long long p = p0 + gp;
    const bool live = p < P;
    const float mu = live ? stats[2 * p] : 0.f, r = live ? stats[2 * p + 1] : 0.f;
    f32x4 dv[NV], xv[NV], rv[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int q = gl + G * j;
      const bool ok = live && q < Cq;
      dv[j] = ok ? *reinterpret_cast<const f32x4*>(dy + p * ldd + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
      xv[j] = ok ? *reinterpret_cast<const f32x4*>(x + p * ldx + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
      rv[j] = (ok && R) ? *reinterpret_cast<const f32x4*>(R + p * ldr + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float s1 = 0.f, s2 = 0.f;
    f32x4 gv[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = biasfree ? xv[j][e] * r : (xv[j][e] - mu) * r;
        aw[j][e] += dv[j][e] * xh;
        ab[j][e] += dv[j][e];
        gv[j][e] = dv[j][e] * wr[j][e];
        s1 += gv[j][e] * (biasfree ? xv[j][e] : xh);
        s2 += gv[j][e];
      }
    s1 = group_sum<G>(s1) * invC;
    s2 = group_sum<G>(s2) * invC;
    if (!live) continue;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int q = gl + G * j;
      if (q >= Cq) continue;
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = biasfree ? r * gv[j][e] - r * r * r * (xv[j][e] - mu) * s1
                                 : r * (gv[j][e] - s2 - (xv[j][e] - mu) * r * s1);
        o[e] = d + rv[j][e];
      }
      *reinterpret_cast<f32x4*>(dx + p * lddx + 4 * q) = o;
    }
  }
  // per-channel partials: the PPW pixel groups of a wave (lanes gl, gl + G, ...) in fixed order,
  // then the 4 waves in fixed order
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int o = G; o < 64; o <<= 1) {
        aw[j][e] += __shfl_xor(aw[j][e], o);
        ab[j][e] += __shfl_xor(ab[j][e], o);
      }
  if (gp == 0)
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      red[wv_][0][gl + G * j] = aw[j];
      red[wv_][1][gl + G * j] = ab[j];
    }
  __syncthreads();
  const int ncol = biasfree ? C : 2 * C;
  for (int c = threadIdx.x; c < ncol; c += blockDim.x) {
    const int which = c < C ? 0 : 1, cc = c < C ? c : c - C;
    const int q = cc >> 2, e = cc & 3;
    part[(long long)blockIdx.x * ncol + c] =
        ((red[0][which][q][e] + red[1][which][q][e]) + red[2][which][q][e]) + red[3][which][q][e];
  }
}

static inline bool ln2_ok(const void* a, int lda, const void* b, int ldb, int C) {
  return C % 4 == 0 && C <= 512 && ((uintptr_t)a & 15) == 0 && ((uintptr_t)b & 15) == 0 && lda % 4 == 0 && ldb % 4 == 0;
}

#define LN2_DISPATCH(KERNEL, grid, ...)                                                              \
  do {                                                                                               \
    if (C <= 64) hipLaunchKernelGGL((KERNEL<16, 1>), grid, dim3(256), 0, s, __VA_ARGS__);              \
    else if (C <= 128) hipLaunchKernelGGL((KERNEL<32, 1>), grid, dim3(256), 0, s, __VA_ARGS__);        \
    else if (C <= 256) hipLaunchKernelGGL((KERNEL<64, 1>), grid, dim3(256), 0, s, __VA_ARGS__);        \
    else hipLaunchKernelGGL((KERNEL<64, 2>), grid, dim3(256), 0, s, __VA_ARGS__);                      \
  } while (0)

hipError_t launch_ln_fwd(const float* x, int ldx, const float* w, const float* b, int C, long long P, int biasfree,
                         float* y, int ldy, float* stats, hipStream_t s, bool generic) {
  if (C > 512) return hipErrorInvalidValue;
  if (!generic && ln2_ok(x, ldx, y, ldy, C) && ((uintptr_t)w & 15) == 0 && (!b || ((uintptr_t)b & 15) == 0)) {
    const int ppw = C <= 64 ? 4 : C <= 128 ? 2 : 1;
    LN2_DISPATCH(ln2_fwd_kernel, dim3(grid_for(P, 4 * ppw * 2, 16384)), x, ldx, w, b, C, P, biasfree, y, ldy, stats);
    return hipGetLastError();
  }
  LN_DISPATCH(ln_fwd_kernel, dim3(grid_for(P, 4 * LN_NP, 16384)), x, ldx, w, b, C, P, biasfree, y, ldy, stats);
  return hipGetLastError();
}

hipError_t launch_ln_bwd(const float* dy, int ldd, const float* x, int ldx, const float* w, const float* stats, int C,
                         long long P, int biasfree, const float* R, int ldr, float* dx, int lddx, float* part, int nblk,
                         hipStream_t s, bool generic) {
  if (C > 512) return hipErrorInvalidValue;
  if (!generic && ln2_ok(dy, ldd, x, ldx, C) && ln2_ok(dx, lddx, w, 4, C) && (!R || ln2_ok(R, ldr, R, ldr, C))) {
    LN2_DISPATCH(ln2_bwd_kernel, dim3(nblk), dy, ldd, x, ldx, w, stats, C, P, biasfree, R, ldr, dx, lddx, part);
    return hipGetLastError();
  }
  LN_DISPATCH(ln_bwd_kernel, dim3(nblk), dy, ldd, x, ldx, w, stats, C, P, biasfree, R, ldr, dx, lddx, part);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------- depthwise 3x3
// Row sweep: a wave owns 64 channels (one per lane, 256 B coalesced per pixel) of a 64-pixel row
// segment and slides a 3x3 register window along x, so each output costs 3 new loads instead of 9.
constexpr int DW_SEG = 64;

__device__ __forceinline__ void dw_load_col(const float* __restrict__ in, int ldi, long long img0, int y, int x, int H,
                                            int W, int c, bool live, float (&col)[3]) {
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int yy = y + r - 1;
    col[r] = (live && x >= 0 && x < W && yy >= 0 && yy < H) ? in[(img0 + (long long)yy * W + x) * ldi + c] : 0.f;
  }
}

constexpr int DW_U = 4;  // output columns per iteration: 3*DW_U loads in flight together

__global__ __launch_bounds__(256) void dw_row_fwd_kernel(const float* __restrict__ in, int ldi,
                                                         const float* __restrict__ w, const float* __restrict__ b,
                                                         int flip, int C, int Bn, int H, int W, int nrs,
                                                         float* __restrict__ out, int ldo) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nrs) return;
  const int c = blockIdx.y * 64 + lane;
  const bool live = c < C;
  const int nsx = (W + DW_SEG - 1) / DW_SEG;
  const int xs = r % nsx, row = r / nsx;
  const int y = row % H, bi = row / H;
  const long long img0 = (long long)bi * H * W;
  const int x0 = xs * DW_SEG, x1 = min(W, x0 + DW_SEG);
  float wr[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) wr[k] = live ? w[c * 9 + (flip ? 8 - k : k)] : 0.f;
  const float bias = (live && b) ? b[c] : 0.f;
  float col[DW_U + 2][3];  // columns x-1 .. x+DW_U
  dw_load_col(in, ldi, img0, y, x0 - 1, H, W, c, live, col[0]);
  dw_load_col(in, ldi, img0, y, x0, H, W, c, live, col[1]);
  for (int x = x0; x < x1; x += DW_U) {
#pragma unroll
    for (int u = 0; u < DW_U; ++u) dw_load_col(in, ldi, img0, y, x + 1 + u, H, W, c, live, col[2 + u]);
#pragma unroll
    for (int u = 0; u < DW_U; ++u) {
      float acc = bias;
#pragma unroll
      for (int ty = 0; ty < 3; ++ty)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) acc += wr[ty * 3 + tx] * col[u + tx][ty];
      if (live && x + u < x1) out[(img0 + (long long)y * W + x + u) * ldo + c] = acc;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      col[0][k] = col[DW_U][k];
      col[1][k] = col[DW_U + 1][k];
    }
  }
}

static int dw_rowsegs(int Bn, int H, int W) { return Bn * H * ((W + DW_SEG - 1) / DW_SEG); }

// LDS-tiled version for views with ldi, ldo % 4 == 0: a block owns TY = 8 rows x TX pixel columns x
// QB channel quads (QB * TX = 256 threads) of one image, stages the (TY + 2) x (TX + 2) halo of float4
// quads in LDS with every load issued up front, then thread (x, q) walks its column of TY outputs with
// a 3 x 3 float4 window read from LDS (consecutive lanes = consecutive quads: conflict-free b128).
// Same accumulation order (bias, then taps row-major) as dw_row_fwd_kernel.
constexpr int DWT_TY = 8;

template <int QB>
__global__ __launch_bounds__(256) void dw_tile_fwd_kernel(const float* __restrict__ in, int ldi,
                                                          const float* __restrict__ w, const float* __restrict__ b,
                                                          int flip, int C, int H, int W, int tiles_x,
                                                          float* __restrict__ out, int ldo) {
  constexpr int TX = 256 / QB, HX = TX + 2, HY = DWT_TY + 2;
  __shared__ f32x4 tile[HY * HX * QB];
  const int Cq = (C + 3) >> 2, ngrp = (Cq + QB - 1) / QB;
  // channel group fastest: the blocks sharing a pixel tile run together, so each pixel's channels
  // reach HBM as whole lines at about the same time
  const int q0 = (blockIdx.x % ngrp) * QB, tile_i = blockIdx.x / ngrp;
  const int tx0 = (tile_i % tiles_x) * TX, ty0 = (tile_i / tiles_x) * DWT_TY;
  const long long img0 = (long long)blockIdx.z * H * W;
  const float* src = in + img0 * ldi;
  // all of a thread's halo loads are issued before the first LDS write (one HBM latency per block)
  constexpr int NLD = (HY * HX * QB + 255) / 256;
  f32x4 v[NLD];
#pragma unroll
  for (int k = 0; k < NLD; ++k) {
    const int i = threadIdx.x + 256 * k;
    const int q = i % QB, px = i / QB;
    const int xx = tx0 + px % HX - 1, yy = ty0 + px / HX - 1;
    v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (i < HY * HX * QB && q0 + q < Cq && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
      v[k] = *reinterpret_cast<const f32x4*>(src + ((long long)yy * W + xx) * ldi + 4 * (q0 + q));
  }
#pragma unroll
  for (int k = 0; k < NLD; ++k)
    if (threadIdx.x + 256 * k < HY * HX * QB) tile[threadIdx.x + 256 * k] = v[k];
  const int q = threadIdx.x % QB, xl = threadIdx.x / QB;
  const int c0 = 4 * (q0 + q), x = tx0 + xl;
  f32x4 wr[9];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) wr[k][e] = c0 + e < C ? w[(c0 + e) * 9 + (flip ? 8 - k : k)] : 0.f;
  f32x4 bias = f32x4{0.f, 0.f, 0.f, 0.f};
  if (b)
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[e] = c0 + e < C ? b[c0 + e] : 0.f;
  __syncthreads();
  if (c0 >= C || x >= W) return;
  const f32x4* t = tile + xl * QB + q;
  f32x4 r0[3], r1[3], r2[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    r0[dx] = t[dx * QB];
    r1[dx] = t[(HX + dx) * QB];
  }
  const bool full = c0 + 4 <= C;
  float* dst = out + (img0 + (long long)ty0 * W + x) * ldo + c0;
#pragma unroll
  for (int r = 0; r < DWT_TY; ++r) {
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) r2[dx] = t[((r + 2) * HX + dx) * QB];
    f32x4 acc = bias;
#pragma unroll
    for (int tx = 0; tx < 3; ++tx) acc += wr[tx] * r0[tx];
#pragma unroll
    for (int tx = 0; tx < 3; ++tx) acc += wr[3 + tx] * r1[tx];
#pragma unroll
    for (int tx = 0; tx < 3; ++tx) acc += wr[6 + tx] * r2[tx];
    if (ty0 + r < H) {
      float* o = dst + (long long)r * W * ldo;
      if (full) *reinterpret_cast<f32x4*>(o) = acc;
      else
        for (int e = 0; e < C - c0; ++e) o[e] = acc[e];
    }
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      r0[dx] = r1[dx];
      r1[dx] = r2[dx];
    }
  }
}

hipError_t launch_dw_fwd(const float* in, int ldi, const float* w, const float* b, int flip, int C, int Bn, int H,
                         int W, float* out, int ldo, hipStream_t s) {
  if (ldi % 4 == 0 && ldo % 4 == 0 && ldi >= (C + 3) / 4 * 4) {
    // QB = 8 quads (32 channels) when 16-quad groups would leave more dead lanes
    const int Cq = (C + 3) / 4;
    const bool q8 = ((Cq + 7) / 8) * 8 < ((Cq + 15) / 16) * 16;
    const int TX = q8 ? 32 : 16, QB = q8 ? 8 : 16;
    const int tiles_x = (W + TX - 1) / TX;
    const dim3 grid(tiles_x * ((H + DWT_TY - 1) / DWT_TY) * ((Cq + QB - 1) / QB), 1, Bn);
    if (q8) hipLaunchKernelGGL(dw_tile_fwd_kernel<8>, grid, dim3(256), 0, s, in, ldi, w, b, flip, C, H, W, tiles_x, out, ldo);
    else hipLaunchKernelGGL(dw_tile_fwd_kernel<16>, grid, dim3(256), 0, s, in, ldi, w, b, flip, C, H, W, tiles_x, out, ldo);
    return hipGetLastError();
  }
  const int nrs = dw_rowsegs(Bn, H, W);
  hipLaunchKernelGGL(dw_row_fwd_kernel, dim3((nrs + 3) / 4, (C + 63) / 64), dim3(256), 0, s, in, ldi, w, b, flip, C,
                     Bn, H, W, nrs, out, ldo);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------- column reductions
// block (column group of 64, row chunk, segment): 4 waves take every 4th row, combined in fixed order
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ x, int ldx, int ncols,
                                                     long long rows_per_seg, int square, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, seg = blockIdx.z, nblk = gridDim.y;
  const long long per = (rows_per_seg + nblk - 1) / nblk;
  const long long r0 = blockIdx.y * per, r1 = min(rows_per_seg, r0 + per);
  const float* xs = x + (long long)seg * rows_per_seg * ldx;
  float a0 = 0.f, a1 = 0.f;
  if (c < ncols) {
    long long r = r0 + wv;
    for (; r + 4 < r1; r += 8) {
      const float v0 = xs[r * ldx + c], v1 = xs[(r + 4) * ldx + c];
      a0 += square ? v0 * v0 : v0;
      a1 += square ? v1 * v1 : v1;
    }
    for (; r < r1; r += 4) {
      const float v = xs[r * ldx + c];
      a0 += square ? v * v : v;
    }
  }
  red[wv][lane] = a0 + a1;
  __syncthreads();
  if (wv == 0 && c < ncols)
    part[((long long)seg * nblk + blockIdx.y) * ncols + c] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// float4 form (ncols, ldx % 4 == 0, 16-byte aligned x): lane = (row sub-index lane >> 4, channel quad
// lane & 15), so a wave reads 4 rows x 64 channels per step; rows r0 + 16 i + 4 wv + (lane >> 4).
// Fixed order: per lane in row order, then the 4 row sub-indices, then the 4 waves.
__global__ __launch_bounds__(256) void colsum4_kernel(const float* __restrict__ x, int ldx, int ncols,
                                                      long long rows_per_seg, int square, float* __restrict__ part) {
  __shared__ f32x4 red[4][16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, rsub = lane >> 4;
  const int c = blockIdx.x * 64 + 4 * (lane & 15), seg = blockIdx.z, nblk = gridDim.y;
  const long long per = (rows_per_seg + nblk - 1) / nblk;
  const long long r0 = blockIdx.y * per, r1 = min(rows_per_seg, r0 + per);
  const float* xs = x + (long long)seg * rows_per_seg * ldx;
  f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
  if (c < ncols) {
    long long r = r0 + 4 * wv + rsub;
    for (; r + 16 < r1; r += 32) {
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(xs + r * ldx + c);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(xs + (r + 16) * ldx + c);
      a0 += square ? v0 * v0 : v0;
      a1 += square ? v1 * v1 : v1;
    }
    for (; r < r1; r += 16) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(xs + r * ldx + c);
      a0 += square ? v * v : v;
    }
  }
  f32x4 a = a0 + a1;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    a[e] += __shfl_xor(a[e], 16);
    a[e] += __shfl_xor(a[e], 32);
  }
  if (rsub == 0) red[wv][lane] = a;
  __syncthreads();
  if (wv == 0 && lane < 16 && c < ncols) {
    const f32x4 t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    float* o = part + ((long long)seg * nblk + blockIdx.y) * ncols + c;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = t[e];
  }
}

__global__ __launch_bounds__(1024) void part_reduce_kernel(const float* __restrict__ part, int nblk, int ncols,
                                                           int pstride, int nseg, float* out, int accumulate,
                                                           float scale) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, seg = blockIdx.y;
  float a = 0.f;
  if (c < ncols) {
    const float* p = part + (long long)seg * nblk * pstride + c;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int b = wv;
    for (; b + 48 < nblk; b += 64) {
      a0 += p[(long long)b * pstride];
      a1 += p[(long long)(b + 16) * pstride];
      a2 += p[(long long)(b + 32) * pstride];
      a3 += p[(long long)(b + 48) * pstride];
    }
    for (; b < nblk; b += 16) a0 += p[(long long)b * pstride];
    a = (a0 + a1) + (a2 + a3);
  }
  red[wv][lane] = a;
  __syncthreads();
  if (wv == 0 && c < ncols) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][lane];
    s *= scale;
    const long long o = (long long)seg * ncols + c;
    out[o] = accumulate ? out[o] + s : s;
  }
}

// Several independent partial reductions in one launch (r03): a TransformerBlock's backward ends
// with ~5 small ones (two LayerNorm weight gradients, two depthwise weight + bias gradients, the
// temperature); one launch each cost ~6.5 us of mostly fixed overhead.  Block x serves column group
// x of the descriptor whose prefix range holds it; same fixed-order sums as part_reduce_kernel.
__global__ __launch_bounds__(1024) void part_reduce_multi_kernel(RedBatch rb) {
  __shared__ float red[16][64];
  int j = 0;
  while (j + 1 < rb.n && (int)blockIdx.x >= rb.cg_prefix[j + 1]) ++j;
  const RedDesc& d = rb.d[j];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = ((int)blockIdx.x - rb.cg_prefix[j]) * 64 + lane;
  float a = 0.f;
  if (c < d.ncols) {
    const float* p = d.part + c;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int b = wv;
    for (; b + 48 < d.nblk; b += 64) {
      a0 += p[(long long)b * d.pstride];
      a1 += p[(long long)(b + 16) * d.pstride];
      a2 += p[(long long)(b + 32) * d.pstride];
      a3 += p[(long long)(b + 48) * d.pstride];
    }
    for (; b < d.nblk; b += 16) a0 += p[(long long)b * d.pstride];
    a = (a0 + a1) + (a2 + a3);
  }
  red[wv][lane] = a;
  __syncthreads();
  if (wv == 0 && c < d.ncols) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][lane];
    d.out[c] = s * d.scale;
  }
}

hipError_t launch_part_reduce_multi(const RedDesc* d, int n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (n > kRedBatch) return hipErrorInvalidValue;
  RedBatch rb;
  rb.n = n;
  rb.cg_prefix[0] = 0;
  for (int j = 0; j < n; ++j) {
    rb.d[j] = d[j];
    rb.cg_prefix[j + 1] = rb.cg_prefix[j] + (d[j].ncols + 63) / 64;
  }
  hipLaunchKernelGGL(part_reduce_multi_kernel, dim3(rb.cg_prefix[n]), dim3(1024), 0, s, rb);
  return hipGetLastError();
}

hipError_t launch_colsum(const float* x, int ldx, int ncols, long long rows_per_seg, int nseg, int square, float* part,
                         int nblk, hipStream_t s) {
constexpr auto KDLAE_COLSUM4 = 1;
  if (KDLAE_COLSUM4 && ncols % 4 == 0 && ldx % 4 == 0 && al16(x)) {
    hipLaunchKernelGGL(colsum4_kernel, dim3((ncols + 63) / 64, nblk, nseg), dim3(256), 0, s, x, ldx, ncols,
                       rows_per_seg, square, part);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(colsum_kernel, dim3((ncols + 63) / 64, nblk, nseg), dim3(256), 0, s, x, ldx, ncols,
                     rows_per_seg, square, part);
  return hipGetLastError();
}

hipError_t launch_part_reduce(const float* part, int nblk, int ncols, int nseg, float* out, int accumulate,
                              float scale, hipStream_t s, int pstride) {
  hipLaunchKernelGGL(part_reduce_kernel, dim3((ncols + 63) / 64, nseg), dim3(1024), 0, s, part, nblk, ncols,
                     pstride > 0 ? pstride : ncols, nseg, out, accumulate, scale);
  return hipGetLastError();
}


// ---------------------------------------------------------------------------------------------- MDTA core
constexpr float kNormEps = 1e-12f;  // F.normalize eps (KDLAE_model.py:135-136)

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// One wave per attention row i (Ch <= 128: lane owns columns lane and lane + 64), four rows per block,
// grid (B * heads, ceil(Ch / 4)).
__global__ __launch_bounds__(256) void attn_softmax_kernel(const float* __restrict__ G, const float* __restrict__ sumsq,
                                                           const float* __restrict__ temp, int C, int heads,
                                                           float* __restrict__ Attn) {
  const int bh = blockIdx.x, b = bh / heads, h = bh - b * heads;
  const int Ch = C / heads;
  const int lane = threadIdx.x & 63, i = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= Ch) return;
  const float t = temp[h];
  const float* g = G + (long long)bh * Ch * Ch + (long long)i * Ch;
  float* a = Attn + (long long)bh * Ch * Ch + (long long)i * Ch;
  const float* sq = sumsq + (long long)b * 2 * C + h * Ch;
  const float* sk = sumsq + (long long)b * 2 * C + C + h * Ch;
  const float nq = fmaxf(sqrtf(sq[i]), kNormEps);
  const int j0 = lane, j1 = lane + 64;
  const float v0 = j0 < Ch ? g[j0] / (nq * fmaxf(sqrtf(sk[j0]), kNormEps)) * t : -INFINITY;
  const float v1 = j1 < Ch ? g[j1] / (nq * fmaxf(sqrtf(sk[j1]), kNormEps)) * t : -INFINITY;
  const float mx = wave_max(fmaxf(v0, v1));
  const float e0 = j0 < Ch ? expf(v0 - mx) : 0.f, e1 = j1 < Ch ? expf(v1 - mx) : 0.f;
  const float inv = 1.f / wave_sum(e0 + e1);
  if (j0 < Ch) a[j0] = e0 * inv;
  if (j1 < Ch) a[j1] = e1 * inv;
}

// One block per (image, head): wave w walks rows w, w + 4, ... with the row's columns across lanes
// (dS, Mq, the E = dGhat * Ghat row and its row sum), then one thread per column sums E's column.
__global__ __launch_bounds__(256) void attn_bwd_kernel(const float* __restrict__ G, const float* __restrict__ sumsq,
                                                       const float* __restrict__ temp, const float* __restrict__ Attn,
                                                       const float* __restrict__ dAttn, int C, int heads,
                                                       float* __restrict__ Mq, float* __restrict__ cq,
                                                       float* __restrict__ ck, float* __restrict__ dtemp_part) {
  extern __shared__ float E[];  // [Ch][Ch] = dGhat * Ghat, then [4] per-wave dt partials
  const int bh = blockIdx.x, b = bh / heads, h = bh - b * heads;
  const int Ch = C / heads;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float t = temp[h];
  const long long mo = (long long)bh * Ch * Ch;
  const float* sq = sumsq + (long long)b * 2 * C + h * Ch;
  const float* sk = sumsq + (long long)b * 2 * C + C + h * Ch;
  float* red = E + Ch * Ch;
  const int j0 = lane, j1 = lane + 64;
  const float nk0 = j0 < Ch ? fmaxf(sqrtf(sk[j0]), kNormEps) : 1.f;
  const float nk1 = j1 < Ch ? fmaxf(sqrtf(sk[j1]), kNormEps) : 1.f;
  float dt = 0.f;
  for (int i = wave; i < Ch; i += 4) {
    const long long ro = mo + (long long)i * Ch;
    const float nq = fmaxf(sqrtf(sq[i]), kNormEps);
    const float a0 = j0 < Ch ? Attn[ro + j0] : 0.f, d0 = j0 < Ch ? dAttn[ro + j0] : 0.f;
    const float a1 = j1 < Ch ? Attn[ro + j1] : 0.f, d1 = j1 < Ch ? dAttn[ro + j1] : 0.f;
    const float rd = wave_sum(a0 * d0 + a1 * d1);
    float rs = 0.f;
    if (j0 < Ch) {
      const float dS = a0 * (d0 - rd), gh = G[ro + j0] / (nq * nk0), dgh = t * dS;
      dt += dS * gh;
      Mq[ro + j0] = dgh / (nq * nk0);
      E[i * Ch + j0] = dgh * gh;
      rs += dgh * gh;
    }
    if (j1 < Ch) {
      const float dS = a1 * (d1 - rd), gh = G[ro + j1] / (nq * nk1), dgh = t * dS;
      dt += dS * gh;
      Mq[ro + j1] = dgh / (nq * nk1);
      E[i * Ch + j1] = dgh * gh;
      rs += dgh * gh;
    }
    rs = wave_sum(rs);
    if (lane == 0) {
      const float s = sqrtf(sq[i]);
      cq[(long long)bh * Ch + i] = s >= kNormEps ? -rs / (s * s) : 0.f;
    }
  }
  dt = wave_sum(dt);
  if (lane == 0) red[wave] = dt;
  __syncthreads();
  for (int j = threadIdx.x; j < Ch; j += blockDim.x) {
    const float sj = sqrtf(sk[j]);
    float csum = 0.f;
    for (int r = 0; r < Ch; ++r) csum += E[r * Ch + j];
    ck[(long long)bh * Ch + j] = sj >= kNormEps ? -csum / (sj * sj) : 0.f;
  }
  if (threadIdx.x == 0) dtemp_part[bh] = (red[0] + red[1]) + (red[2] + red[3]);
}

hipError_t launch_attn_softmax(const float* G, const float* sumsq, const float* temp, int Bn, int C, int heads,
                               float* Attn, hipStream_t s) {
  const int Ch = C / heads;
  if (Ch > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(attn_softmax_kernel, dim3(Bn * heads, (Ch + 3) / 4), dim3(256), 0, s, G, sumsq, temp, C, heads,
                     Attn);
  return hipGetLastError();
}

hipError_t launch_attn_bwd(const float* G, const float* sumsq, const float* temp, const float* Attn, const float* dAttn,
                           int Bn, int C, int heads, float* Mq, float* cq, float* ck, float* dtemp_part,
                           hipStream_t s) {
  const int Ch = C / heads;
  if (Ch > 128) return hipErrorInvalidValue;
  const size_t lds = ((size_t)Ch * Ch + 4) * sizeof(float);
  hipLaunchKernelGGL(attn_bwd_kernel, dim3(Bn * heads), dim3(256), lds, s, G, sumsq, temp, Attn, dAttn, C, heads, Mq,
                     cq, ck, dtemp_part);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------- layout
__global__ void shuffle_kernel(const float* __restrict__ in, int ldi, float* __restrict__ out, int ldo, int C, int Bn,
                               int h, int w, int dir) {
  // indexes the low-resolution side: (b, y, x, c, i, j) <-> high (b, 2y+i, 2x+j, c), low channel c*4+i*2+j
  const long long total = (long long)Bn * h * w * C * 4;
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int lc = (int)(idx % (4 * C));
    const long long lp = idx / (4 * C);
    const int x = (int)(lp % w);
    const long long t = lp / w;
    const int y = (int)(t % h);
    const long long b = t / h;
    const int c = lc >> 2, i = (lc >> 1) & 1, j = lc & 1;
    const long long hp = (b * 2 * h + 2 * y + i) * (2LL * w) + 2 * x + j;
    if (dir == 0) out[lp * ldo + lc] = in[hp * ldi + c];
    else out[hp * ldo + c] = in[lp * ldi + lc];
  }
}

// out[p, 0:C] (= or +=) in[p, 0:C], and out[p, C:Wd] = 0 (Wd > C: a zero-padded copy).  32-bit
// index math when the element count allows it (a 64-bit division per element was most of the cost)
__global__ void copy_cols_kernel(const float* __restrict__ in, int ldi, float* out, int ldo, int C, int Wd,
                                 long long P, int accumulate) {
  const long long total = P * Wd;
  const bool narrow = total < (1LL << 32);
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    long long p;
    int c;
    if (narrow) {
      const unsigned u = (unsigned)idx, pu = u / (unsigned)Wd;
      p = pu;
      c = (int)(u - pu * (unsigned)Wd);
    } else {
      p = idx / Wd;
      c = (int)(idx - p * Wd);
    }
    if (c < C) {
      const float v = in[p * ldi + c];
      out[p * ldo + c] = accumulate ? out[p * ldo + c] + v : v;
    } else {
      out[p * ldo + c] = 0.f;
    }
  }
}

__global__ void nchw_to_nhwc_kernel(const float* __restrict__ in, int C, long long HW, long long total, float* out,
                                    int ldo, int accumulate) {
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const long long p = idx / C;  // global pixel (b*HW + s)
    const int c = (int)(idx - p * C);
    const long long b = p / HW, sp = p - b * HW;
    const float v = in[(b * C + c) * HW + sp];
    out[p * ldo + c] = accumulate ? out[p * ldo + c] + v : v;
  }
}

__global__ void nhwc_to_nchw_kernel(const float* __restrict__ in, int ldi, const float* __restrict__ add, int C,
                                    long long HW, long long total, float* __restrict__ out) {
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const long long sp = idx % HW;
    const long long bc = idx / HW;
    const long long b = bc / C;
    const int c = (int)(bc - b * C);
    float v = in[(b * HW + sp) * ldi + c];
    if (add) v += add[idx];
    out[idx] = v;
  }
}

hipError_t launch_shuffle(const float* in, int ldi, float* out, int ldo, int C, int Bn, int h, int w, int dir,
                          hipStream_t s) {
  const long long total = (long long)Bn * h * w * C * 4;
  hipLaunchKernelGGL(shuffle_kernel, dim3(grid_for(total, 256, 65536)), dim3(256), 0, s, in, ldi, out, ldo, C, Bn, h, w,
                     dir);
  return hipGetLastError();
}

// 3x3 conv weights (OIHW) -> the implicit-GEMM B operand as a plain [K = 9 Cg][N] row-major matrix
// (mode 2: B(k = t Cg + c, n) = W[n][c][t], the conv; mode 3: W[c][n][8 - t], the transposed conv):
// the tiled kernel then reads B as float4 runs instead of one index computation (k / Cg) and one
// stride-9 load per element.  Same values, so the same sums.
__global__ __launch_bounds__(256) void pack_w3_kernel(const float* __restrict__ W, int Cg, int N, int mode,
                                                      float* __restrict__ out) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x, tot = 9LL * Cg * N;
  if (idx >= tot) return;
  const int k = (int)(idx / N), n = (int)(idx - (long long)k * N);
  const int t = k / Cg, c = k - t * Cg;
  out[idx] = mode == 2 ? W[((long long)n * Cg + c) * 9 + t] : W[((long long)c * N + n) * 9 + (8 - t)];
}

hipError_t launch_pack_w3(const float* W, int Cg, int N, int mode, float* out, hipStream_t s) {
  if ((mode != 2 && mode != 3) || Cg <= 0 || N <= 0) return hipErrorInvalidValue;
  const long long tot = 9LL * Cg * N;
  hipLaunchKernelGGL(pack_w3_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, W, Cg, N, mode, out);
  return hipGetLastError();
}

hipError_t launch_copy_cols(const float* in, int ldi, float* out, int ldo, int C, long long P, int accumulate,
                            hipStream_t s, int zero_to) {
  const int Wd = zero_to > C ? zero_to : C;
  hipLaunchKernelGGL(copy_cols_kernel, dim3(grid_for(P * Wd, 256, 65536)), dim3(256), 0, s, in, ldi, out, ldo, C, Wd,
                     P, accumulate);
  return hipGetLastError();
}

hipError_t launch_nchw_to_nhwc(const float* in, int C, int Bn, long long HW, float* out, int ldo, int accumulate,
                               hipStream_t s) {
  const long long total = (long long)Bn * HW * C;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for(total, 256, 65536)), dim3(256), 0, s, in, C, HW, total, out,
                     ldo, accumulate);
  return hipGetLastError();
}

hipError_t launch_nhwc_to_nchw(const float* in, int ldi, const float* add, int C, int Bn, long long HW, float* out,
                               hipStream_t s) {
  const long long total = (long long)Bn * HW * C;
  hipLaunchKernelGGL(nhwc_to_nchw_kernel, dim3(grid_for(total, 256, 65536)), dim3(256), 0, s, in, ldi, add, C, HW,
                     total, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------- loss, clip, AdamW
__device__ __forceinline__ float block_sum_256(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  return ((sh[0] + sh[1]) + sh[2]) + sh[3];
}

__global__ __launch_bounds__(256) void l1sr_kernel(const float* __restrict__ pred, const float* __restrict__ tgt,
                                                   long long n, float gscale, float* __restrict__ grad,
                                                   float* __restrict__ part) {
  __shared__ float sh[4];
  float a = 0.f, sb = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float d = pred[i] - tgt[i];
    a += fabsf(d);
    sb += fabsf((pred[i] > 0.1f ? 1.f : 0.f) - (tgt[i] > 0.1f ? 1.f : 0.f));
    if (grad) grad[i] = d > 0.f ? gscale : (d < 0.f ? -gscale : 0.f);
  }
  a = block_sum_256(a, sh);
  sb = block_sum_256(sb, sh);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = sb;
  }
}

__global__ void l1sr_final_kernel(const float* part0, int nblk0, double n0, float wl0, float ws0, const float* part1,
                                  int nblk1, double n1, float wl1, float ws1, float* out) {
  if (threadIdx.x != 0) return;
  float a0 = 0.f, s0 = 0.f, a1 = 0.f, s1 = 0.f;
  for (int b = 0; b < nblk0; ++b) {
    a0 += part0[2 * b];
    s0 += part0[2 * b + 1];
  }
  for (int b = 0; b < nblk1; ++b) {
    a1 += part1[2 * b];
    s1 += part1[2 * b + 1];
  }
  float loss = wl0 * (float)(a0 / n0) + ws0 * (float)(s0 / n0);
  if (part1) loss += wl1 * (float)(a1 / n1) + ws1 * (float)(s1 / n1);
  out[0] = loss;
}

hipError_t launch_l1sr(const float* pred, const float* target, long long n, float w_l1, float* grad, float* part,
                       int nblk, hipStream_t s) {
  hipLaunchKernelGGL(l1sr_kernel, dim3(nblk), dim3(256), 0, s, pred, target, n, (float)(w_l1 / (double)n), grad, part);
  return hipGetLastError();
}

hipError_t launch_l1sr_final(const float* part0, int nblk0, long long n0, float wl0, float ws0, const float* part1,
                             int nblk1, long long n1, float wl1, float ws1, float* out, hipStream_t s) {
  hipLaunchKernelGGL(l1sr_final_kernel, dim3(1), dim3(64), 0, s, part0, nblk0, (double)n0, wl0, ws0, part1, nblk1,
                     (double)n1, wl1, ws1, out);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, long long n, float* __restrict__ part) {
  __shared__ float sh[4];
  float a = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    a += g[i] * g[i];
  a = block_sum_256(a, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = a;
}

__global__ void clip_coef_kernel(const float* part, int nblk, float gscale, float max_norm, float* state) {
  if (threadIdx.x != 0) return;
  double a = 0.0;
  for (int b = 0; b < nblk; ++b) a += part[b];
  const float norm = (float)sqrt(a) * gscale;
  state[0] = norm;
  float coef = 1.f;
  if (max_norm > 0.f) coef = fminf(1.f, max_norm / (norm + 1e-6f));
  state[1] = gscale * coef;
}

__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, long long n, const float* __restrict__ state, float lr,
                             float beta1, float beta2, float eps, float wd, float bc1, float bc2s) {
  const float gs = state[1];
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float gr = g[i] * gs;
    float pv = p[i] * (1.f - lr * wd);
    const float mv = m[i] + (1.f - beta1) * (gr - m[i]);
    const float vv = v[i] * beta2 + (1.f - beta2) * gr * gr;
    const float denom = sqrtf(vv) / bc2s + eps;
    pv -= (lr / bc1) * mv / denom;
    p[i] = pv;
    m[i] = mv;
    v[i] = vv;
  }
}

hipError_t launch_sumsq(const float* g, long long n, float* part, int nblk, hipStream_t s) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblk), dim3(256), 0, s, g, n, part);
  return hipGetLastError();
}

hipError_t launch_clip_coef(const float* part, int nblk, float gscale, float max_norm, float* state, hipStream_t s) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(64), 0, s, part, nblk, gscale, max_norm, state);
  return hipGetLastError();
}

hipError_t launch_adamw(float* p, const float* g, float* m, float* v, long long n, const float* state, float lr,
                        float beta1, float beta2, float eps, float wd, int step, hipStream_t s) {
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2s = sqrtf(1.f - powf(beta2, (float)step));
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n, 256, 16384)), dim3(256), 0, s, p, g, m, v, n, state, lr, beta1,
                     beta2, eps, wd, bc1, bc2s);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------- mixup, EMA
// Mixing_Augment.mixup (image_restoration_model.py:32-34): out[b] = lam * in[b] + (1 - lam) * in[perm[b]]
__global__ void mixup_kernel(const float* __restrict__ in, float* __restrict__ out, int B, long long per,
                             const int* __restrict__ perm, float lam) {
  const long long total = (long long)B * per;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / per);
    const long long e = i - (long long)b * per;
    out[i] = lam * in[i] + (1.f - lam) * in[(long long)perm[b] * per + e];
  }
}

// BaseModel.model_ema (base_model.py:54-62): ema = decay * ema + (1 - decay) * theta
__global__ void ema_kernel(float* __restrict__ ema, const float* __restrict__ theta, long long n, float decay) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    ema[i] = ema[i] * decay + theta[i] * (1.f - decay);
}

hipError_t launch_mixup(const float* in, float* out, int B, long long per, const int* perm, float lam, hipStream_t s) {
  hipLaunchKernelGGL(mixup_kernel, dim3(grid_for((long long)B * per, 256, 65536)), dim3(256), 0, s, in, out, B, per,
                     perm, lam);
  return hipGetLastError();
}

hipError_t launch_ema(float* ema, const float* theta, long long n, float decay, hipStream_t s) {
  hipLaunchKernelGGL(ema_kernel, dim3(grid_for(n, 256, 16384)), dim3(256), 0, s, ema, theta, n, decay);
  return hipGetLastError();
}

}  // namespace train
}  // namespace kdlae
