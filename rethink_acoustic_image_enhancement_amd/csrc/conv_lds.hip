// LDS-tiled implicit-GEMM 3x3 Conv2d / 3x3x3 Conv3d (+ bias, ReLU) for the small-image U-Nets: the
// ASDQE DoubleConvs (ASDQE/ASDQE_model.py:20-34, 64 to 256 output channels) and the KDLAE-S 32- and
// 64-channel levels (KDLAE/KDLAE_model.py:386-393).  Output channels beyond 64 run as more blocks
// along grid.y (4 channel tiles each), every one staging the same halo.
//
// The generic implicit GEMM (gemm.hip) re-reads every input pixel through L1 for each of the 9 (27)
// taps.  Here a block owns a 4-row x 64-column output tile of one frame and NT x 16 output channels.
// It stages the input halo of CC channels at a time in LDS, channel-group-major
// ([16-ch group][frame][6 rows][66 cols][16 ch], so one wave's 16-pixel x 64-B fragment read is a
// contiguous, conflict-free 1 KiB), and walks the k-groups (tap, 16-ch group) with the NT weight
// fragments of the next k-group prefetched from global memory (fragment order, L2-resident) while the
// 16 NT MFMAs of the current one run.  Wave w computes output row w: 4 pixel tiles x NT channel tiles.
//
// MFMA roles as in gemm.hip: A = weights (rows = output channels), B = pixels; lane (li, lq) ends with
// pixel li and output channels 4 lq .. 4 lq + 3 of each channel tile.
// Products (r05): the split-bf16 form of every inference GEMM (mfma3.h): consecutive k-groups of the
// chunk's (tap, group) sequence pair up; both operands are split in registers — the pixel fragments
// from LDS and the weight fragments from L2 — and six v_mfma_f32_16x16x32_bf16 replace eight
// v_mfma_f32_16x16x4_f32 per 16 x 16 x 32 block.
#include "kernels.h"
#include "lds_dma.h"
#include "mfma3.h"

namespace kdlae {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TR = 4, TC = 64, HR = TR + 2, HC = TC + 2;

}  // namespace

template <int KT, int NT, int CC, bool PRE>
__global__ __launch_bounds__(256) void conv_lds_kernel(ConvLdsParams p) {
  constexpr int NG = CC / 16;                   // 16-channel groups per staged chunk
  constexpr int FPX = KT * HR * HC;             // halo pixels per group
  constexpr int NTAP = 9 * KT;
  // PRE: the chunk's two 16-channel groups staged already split, [plane][quad][pixel] of bf16x8 (quad q:
  // channels 4q..4q+3 of group 0, then of group 1 = one lane's B operand), pixels padded to 16
  constexpr int FPXP = (FPX + 15) / 16 * 16;
  // PRE3 (KT = 3): fp32 halo as without PRE, the weights from tap-pair split records (kdlae_s.cpp)
  constexpr bool PRE2 = PRE && KT == 1, PRE3 = PRE && KT == 3;
  __shared__ __attribute__((aligned(16))) f32x4 tile[PRE2 ? 12 * FPXP : NG * FPX * 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int tx_n = (p.W + TC - 1) / TC, ty_n = (p.H + TR - 1) / TR;
  int bid = blockIdx.x;
  const int txi = bid % tx_n;
  bid /= tx_n;
  const int tyi = bid % ty_n;
  bid /= ty_n;
  const int fr = bid % p.F;
  const int b = bid / p.F;
  const int x0 = txi * TC, y0 = tyi * TR;
  const int t0 = blockIdx.y * NT;               // first output channel tile of this block
  const long long fhw = (long long)p.H * p.W;
  const float* inb = p.in + (long long)b * p.F * fhw * p.ldi;
  const int cgt = p.cin_pad / 16;               // channel groups per tap
  static_assert(!PRE2 || CC == 32, "pre-split records: 2-D, 2-group chunks");
  static_assert(!PRE3 || CC == 16, "tap-pair records: 3-D, 1-group chunks");
  const int kpt = (p.kgroups + 1) / 2;           // record pairs per output tile

  f32x4 acc[NT][4];
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[n][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // weight fragment of (channel tile t0 + n, k-group g) for this lane; tiles past ntiles read zeros
  auto wfrag = [&](int n, int g) -> f32x4 {
    const int tt = t0 + n;
    if (tt >= p.ntiles) return f32x4{0.f, 0.f, 0.f, 0.f};
    return *reinterpret_cast<const f32x4*>(p.wp + (((size_t)tt * p.kgroups + g) * 64 + lane) * 4);
  };

  for (int c0 = 0; c0 < p.cin_pad; c0 += CC) {
    __syncthreads();  // previous chunk's reads are done
    // stage channels [c0, c0 + CC): item = (group, halo pixel, quad)
    if constexpr (PRE2) {
      // item = (quad, pixel): both groups' float4 of the quad, split, three 16-byte planes
      constexpr int SB = 4;
#pragma unroll 1
      for (int base = 0; base < 4 * FPX; base += 256 * SB) {
        f32x4 v[SB][2];
#pragma unroll
        for (int k = 0; k < SB; ++k) {
          const int i = base + tid + 256 * k;
          const int q = i / FPX, px = i - q * FPX;
          const int c = px % HC, r = px / HC;
          const int yy = y0 + r - 1, xx = x0 + c - 1;
          const bool ok = i < 4 * FPX && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
          const float* src = inb + ((long long)fr * fhw + (long long)yy * p.W + xx) * p.ldi + c0 + 4 * q;
#pragma unroll
          for (int h = 0; h < 2; ++h)
            v[k][h] = ok ? *reinterpret_cast<const f32x4*>(src + 16 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int k = 0; k < SB; ++k) {
          const int i = base + tid + 256 * k;
          if (i >= 4 * FPX) continue;
          const int q = i / FPX, px = i - q * FPX;
          const F3 sv = split3(v[k][0], v[k][1]);
          tile[(0 * 4 + q) * FPXP + px] = __builtin_bit_cast(f32x4, sv.h);
          tile[(1 * 4 + q) * FPXP + px] = __builtin_bit_cast(f32x4, sv.m);
          tile[(2 * 4 + q) * FPXP + px] = __builtin_bit_cast(f32x4, sv.l);
        }
      }
    } else
    dma::stage_batched<NG * FPX * 4, 8>(tile, tid, [&](int i) -> f32x4 {
      const int q = i & 3, gp = i >> 2;
      const int px = gp % FPX, grp = gp / FPX;
      const int c = px % HC, r = (px / HC) % HR, f = px / (HC * HR);
      const int ff = fr + f - (KT == 3 ? 1 : 0), yy = y0 + r - 1, xx = x0 + c - 1;
      if (c0 + grp * 16 < p.cin_pad && (unsigned)ff < (unsigned)p.F && (unsigned)yy < (unsigned)p.H &&
          (unsigned)xx < (unsigned)p.W)
        return *reinterpret_cast<const f32x4*>(inb + ((long long)ff * fhw + (long long)yy * p.W + xx) * p.ldi + c0 +
                                               grp * 16 + 4 * q);
      return f32x4{0.f, 0.f, 0.f, 0.f};
    });
    __syncthreads();
    const int ngrp = min(NG, (p.cin_pad - c0) / 16);
    const int nk = NTAP * ngrp;  // k-groups of this chunk: (tap, group) with group fastest
    const int np = (nk + 1) / 2;  // split pairs (k-groups 2P, 2P + 1; an odd last one pairs with zeros)
    // weight fragments of pair P (f32 fragment order, L2-resident), split in registers per pair
    auto wpair = [&](int P, f32x4 (&wv)[2][NT]) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kk = 2 * P + h;
        const int tap = kk / ngrp, grp = kk - tap * ngrp;
        const int g = tap * cgt + c0 / 16 + grp;
#pragma unroll
        for (int n = 0; n < NT; ++n) wv[h][n] = kk < nk ? wfrag(n, g) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    };
    if constexpr (PRE2) {
      // pre-split records: pair P of the chunk = k-groups (tap P, groups c0/16, c0/16 + 1) = the
      // record pair G = (P cgt + c0 / 16) / 2 of the GEMM pack (cgt and c0 / 16 even)
      auto wrec = [&](int P, F3 (&wv)[NT]) {
        const int G = (P * cgt + c0 / 16) >> 1;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int tt = t0 + n;
          if (tt < p.ntiles) {
            wv[n] = load_w3(reinterpret_cast<const f32x4*>(p.wp3) + ((size_t)tt * kpt + G) * kRec3, lane);
          } else {
            wv[n].h = wv[n].m = wv[n].l = bf16x8{};
          }
        }
      };
      F3 wq[NT];
      wrec(0, wq);
      for (int P = 0; P < np; ++P) {
        F3 wn3[NT];
        if (P + 1 < np) wrec(P + 1, wn3);  // the next pair's records load under this pair's MFMAs
        F3 xs[4];
        const f32x4* xp = tile + lq * FPXP + (wave + P / 3) * HC + P % 3 + li;  // tap P, plane h
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          xs[t].h = __builtin_bit_cast(bf16x8, xp[16 * t]);
          xs[t].m = __builtin_bit_cast(bf16x8, xp[4 * FPXP + 16 * t]);
          xs[t].l = __builtin_bit_cast(bf16x8, xp[8 * FPXP + 16 * t]);
        }
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[n][t] = mfma6(wq[n], xs[t], acc[n][t]);
        if (P + 1 < np) {
#pragma unroll
          for (int n = 0; n < NT; ++n) wq[n] = wn3[n];
        }
      }
    } else if constexpr (PRE3) {
      // tap-pair records: pair P of the chunk (one group, taps 2P and 2P + 1; tap 27 zeros) is record
      // (c0 / 16) * 14 + P of the tile; the same values and pairing as the in-register split below
      const int kp3 = (p.cin_pad / 16) * 14;
      auto wrec = [&](int P, F3 (&wv)[NT]) {
        const int G = (c0 / 16) * 14 + P;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int tt = t0 + n;
          if (tt < p.ntiles) {
            wv[n] = load_w3(reinterpret_cast<const f32x4*>(p.wp3) + ((size_t)tt * kp3 + G) * kRec3, lane);
          } else {
            wv[n].h = wv[n].m = wv[n].l = bf16x8{};
          }
        }
      };
      F3 wq[NT];
      wrec(0, wq);
      for (int P = 0; P < np; ++P) {
        F3 wn3[NT];
        if (P + 1 < np) wrec(P + 1, wn3);  // the next pair's records load under this pair's MFMAs
        f32x4 xv[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int tap = 2 * P + h;
          const int df = tap / 9, dy = (tap / 3) % 3, dx = tap % 3;
          const f32x4* row = tile + ((df * HR + wave + dy) * HC + dx + li) * 4 + lq;
#pragma unroll
          for (int t = 0; t < 4; ++t) xv[h][t] = tap < nk ? row[t * 16 * 4] : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        F3 xs[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) xs[t] = split3(xv[0][t], xv[1][t]);
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[n][t] = mfma6(wq[n], xs[t], acc[n][t]);
        if (P + 1 < np) {
#pragma unroll
          for (int n = 0; n < NT; ++n) wq[n] = wn3[n];
        }
      }
    } else {
    f32x4 wc[2][NT];
    wpair(0, wc);
    for (int P = 0; P < np; ++P) {
      f32x4 wn[2][NT];
      if (P + 1 < np) wpair(P + 1, wn);  // the next pair's weights load under this pair's MFMAs
      f32x4 xv[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kk = 2 * P + h;
        const int tap = kk / ngrp, grp = kk - tap * ngrp;
        const int df = tap / 9, dy = (tap / 3) % 3, dx = tap % 3;
        const f32x4* row = tile + (((grp * KT + df) * HR + wave + dy) * HC + dx + li) * 4 + lq;
#pragma unroll
        for (int t = 0; t < 4; ++t) xv[h][t] = kk < nk ? row[t * 16 * 4] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      F3 xs[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) xs[t] = split3(xv[0][t], xv[1][t]);
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const F3 w = split3(wc[0][n], wc[1][n]);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[n][t] = mfma6(w, xs[t], acc[n][t]);
      }
      if (P + 1 < np) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int n = 0; n < NT; ++n) wc[h][n] = wn[h][n];
      }
    }
    }
  }

  const int y = y0 + wave;
  if (y >= p.H) return;
  if (p.out_mode == 1) {  // PixelUnshuffle(2) store (block-uniform branch)
    const int Ho = p.H >> 1, Wo = p.W >> 1;
    float* ob = p.out + ((long long)b * p.F + fr) * Ho * Wo * p.ldo;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int tt = t0 + n;
      if (tt >= p.ntiles) break;
      const f32x4 bias = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + tt * 16 + 4 * lq) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int x = x0 + t * 16 + li;
        if (x >= p.W) continue;
        f32x4 v = acc[n][t] + bias;
        float* o = ob + ((long long)(y >> 1) * Wo + (x >> 1)) * p.ldo + 2 * (y & 1) + (x & 1);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ch = tt * 16 + 4 * lq + e;
          if (ch < p.nout) o[4 * ch] = p.relu ? fmaxf(v[e], 0.f) : v[e];
        }
      }
    }
    return;
  }
  if (p.out_mode == 2) {  // PixelShuffle(2) store: a lane's 4 outputs fill one 2 x 2 output block
    const int Wo = 2 * p.W;
    float* ob = p.out + ((long long)b * p.F + fr) * 4 * fhw * p.ldo;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int tt = t0 + n;
      if (tt >= p.ntiles) break;
      const f32x4 bias = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + tt * 16 + 4 * lq) : f32x4{0.f, 0.f, 0.f, 0.f};
      const int ch = tt * 4 + lq;  // (tt * 16 + 4 lq + e) >> 2
      if (4 * ch >= p.nout) continue;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int x = x0 + t * 16 + li;
        if (x >= p.W) continue;
        f32x4 v = acc[n][t] + bias;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          ob[((long long)(2 * y + (e >> 1)) * Wo + 2 * x + (e & 1)) * p.ldo + ch] = p.relu ? fmaxf(v[e], 0.f) : v[e];
      }
    }
    return;
  }
  float* outb = p.out + ((long long)b * p.F * fhw + (long long)fr * fhw + (long long)y * p.W) * p.ldo;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int tt = t0 + n;
    if (tt >= p.ntiles) break;
    const f32x4 bias = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + tt * 16 + 4 * lq) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int x = x0 + t * 16 + li;
      if (x >= p.W) continue;
      f32x4 v = acc[n][t] + bias;
      if (p.relu) {
        v.x = fmaxf(v.x, 0.f);
        v.y = fmaxf(v.y, 0.f);
        v.z = fmaxf(v.z, 0.f);
        v.w = fmaxf(v.w, 0.f);
      }
      *reinterpret_cast<f32x4*>(outb + (long long)x * p.ldo + tt * 16 + 4 * lq) = v;
    }
  }
}

bool conv_lds_supported(int kt, int ntiles, int cin_pad) {
  if (kt != 1 && kt != 3) return false;
  if (cin_pad % 16 || cin_pad <= 0) return false;
  return ntiles >= 2 && ntiles <= 16;
}

hipError_t launch_conv_lds(const ConvLdsParams& p, hipStream_t s) {
  if (!conv_lds_supported(p.kt, p.ntiles, p.cin_pad) || p.ldi % 4 || p.ldo % 4 || p.ldi < p.cin_pad ||
      p.kgroups != 9 * p.kt * (p.cin_pad / 16))
    return hipErrorInvalidValue;
  if (p.out_mode == 0 ? p.ldo < 16 * p.ntiles
      : p.out_mode == 1 ? (p.kt != 1 || p.H % 2 || p.W % 2 || p.nout <= 0 || p.nout > 16 * p.ntiles ||
                           p.ldo < 4 * p.nout)
      : p.out_mode == 2 ? (p.kt != 1 || p.nout <= 0 || p.nout % 4 || p.nout > 16 * p.ntiles || 4 * p.ldo < p.nout)
                        : true)
    return hipErrorInvalidValue;
  const long long blocks = (long long)p.Bn * p.F * ((p.H + TR - 1) / TR) * ((p.W + TC - 1) / TC);
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
  // 4 channel tiles per block at most: NT = 8 needs 271 VGPRs + AGPRs (one wave per SIMD) and measured
  // slower than two NT = 4 blocks that stage the same halo (r01, ASDQE 128-channel convs)
  const int nt = p.ntiles <= 2 ? 2 : 4;
  dim3 grid((unsigned)blocks, (unsigned)((p.ntiles + nt - 1) / nt));
  // staged chunk: 32 channels (2-D, 51 KiB) or 16 channels (3-D, 76 KiB) of halo; 2-D with split
  // weight records when the caller has them and the chunks pair like the records (cin_pad % 32 == 0)
  const bool pre = p.kt == 1 && p.wp3 && p.cin_pad % 32 == 0;  // (kt = 3: wp3 holds tap-pair records)
  if (p.kt == 1) {
    if (nt == 2) {
      if (pre) hipLaunchKernelGGL((conv_lds_kernel<1, 2, 32, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((conv_lds_kernel<1, 2, 32, false>), grid, dim3(256), 0, s, p);
    } else {
      if (pre) hipLaunchKernelGGL((conv_lds_kernel<1, 4, 32, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((conv_lds_kernel<1, 4, 32, false>), grid, dim3(256), 0, s, p);
    }
  } else {
    // tap-pair split records when the caller has them (KDLAE-S packs them for every conv_lds layer)
    if (p.wp3) {
      if (nt == 2) hipLaunchKernelGGL((conv_lds_kernel<3, 2, 16, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((conv_lds_kernel<3, 4, 16, true>), grid, dim3(256), 0, s, p);
    } else {
      if (nt == 2) hipLaunchKernelGGL((conv_lds_kernel<3, 2, 16, false>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((conv_lds_kernel<3, 4, 16, false>), grid, dim3(256), 0, s, p);
    }
  }
  return hipGetLastError();
}

}  // namespace kdlae
