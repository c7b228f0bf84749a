// MFMA implicit-GEMM convolution for gfx950 (CDNA4), NHWC activations, fp32 values.
//
// out[p][n] = epilogue( sum_k A'[p][k] * W[n][k] )
//   pointwise (ksize 1): k = input channel               — every 1x1 Conv2d of KDLAE-T
//                          (qkv / project_out / project_in / ffn.project_out / reduce_chan,
//                           KDLAE/KDLAE_model.py:95,99,118,120,238,243)
//   implicit 3x3 (ksize 3): k = tap * Cin_pad + c, zero padding = dilation
//                          (Downsample/Upsample body convs :186,:196, upen :266)
//   A' = A, or the LayerNorm of A over channels when `ln` is set (BiasFree :50-52 / WithBias
//        :67-70); the LN weight is pre-folded into W and the LN bias into `bias`.
//   epilogue: + bias[n] (+ residual R[p][n], TransformerBlock :160-161) (ReLU), stored plain or
//             through the PixelUnshuffle(2) / PixelShuffle(2) index map (:187, :197), so the
//             shuffle never materialises.
//
// Work decomposition: a block is 8 waves; each wave owns 2 x 16 pixel rows, holding its A rows
// for the current k-chunk in VGPRs (float4 per lane per 16-deep k-group: 16 rows x 64 B
// contiguous per wave load).  The weight chunk [NT tiles][KG/2 pairs] (split fragment order) is
// staged into LDS and shared by all 8 waves; when the whole K fits one chunk it stays resident
// while the block walks a contiguous run of 256-row pixel tiles.
// Products (r05): the split-bf16 MFMA of mfma3.h — the A rows are split once per tile after the
// LayerNorm, the weights are stored pre-split, and every accumulator sums its 32-deep pairs in
// ascending k order with mfma6's term order, so all schedules (resident / chunked / fused) give the
// same bits for a pixel as long as their k-chunks start on an even k-group (the host enforces it).
#include "kernels.h"
#include "mfma3.h"
#include "rowops.h"

#include <algorithm>
#include <cstdlib>

namespace kdlae {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// LDS bytes of `tiles` output tiles' split records over kg k-groups
static inline size_t w3_bytes(long long tiles, int kg) { return (size_t)tiles * ((kg + 1) / 2) * 3072; }

// OUT: 0 = plain NHWC store (N % 16 == 0), 1 = PixelUnshuffle(2) store, 2 = PixelShuffle(2) store.
// Operand roles: the MFMA's A operand is the packed weight tile (rows = output channels) and its
// B operand is the pixel tile, so the accumulator holds D^T: lane (li, lq) owns pixel li and the 4
// consecutive output channels 4*lq .. 4*lq+3 -> one 16-byte store (and residual load) per tile.
//
// Two schedules, chosen by the host:
//  * resident (group_tiles > 0, needs KG == kgroups): the block's whole weight group (grid.y selects the group of
//    group_tiles output tiles) sits in LDS for the block's lifetime; each wave keeps its A rows
//    (full K, LN applied) in VGPRs, walks the group's n-chunks of NT tiles, and — with PF — issues
//    the next tile's A loads before this tile's MFMAs so HBM latency hides under matrix work.
//  * chunked (group_tiles == 0: deep layers, implicit-GEMM 3x3, odd K): grid.y = n-chunk; the [NT][KG] weight chunk is restaged
//    per k-chunk and A is reloaded per k-chunk (LN then comes from precomputed row stats).

template <int KG, bool CONV3>
__device__ __forceinline__ void load_a(const GemmParams& p, const float* __restrict__ Ab, int row0, int kc,
                                       int li, int lq, int HW, f32x4 (&a)[kGemmRT][KG]) {
#pragma unroll
  for (int r = 0; r < kGemmRT; ++r) {
    const int prow = row0 + r * 16 + li;
    const bool pv = prow < HW;
    if (!CONV3) {
      const int off0 = prow * p.lda + 4 * lq + kc * KG * 16;
#pragma unroll
      for (int g = 0; g < KG; ++g) {
        const bool ok = pv && (kc * KG + g) < p.kgroups;
        const f32x4 v = *reinterpret_cast<const f32x4*>(Ab + (ok ? off0 + g * 16 : 0));
        a[r][g] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
      // pixel -> (frame, y, x); taps are (dt, dy, dx) for Conv3d (kt = 3) or (dy, dx) for 2-D
      const int fhw = p.H * p.W;
      const int pt = prow / fhw;
      const int rem = prow - pt * fhw;
      const int py = rem / p.W;
      const int px = rem - py * p.W;
#pragma unroll
      for (int g = 0; g < KG; ++g) {
        const int gg = kc * KG + g;
        const int tap = gg / p.cg_per_tap;
        const int cgi = gg - tap * p.cg_per_tap;
        const int t9 = p.kt == 3 ? tap - (tap / 9) * 9 : tap;
        const int tt = p.kt == 3 ? pt + tap / 9 - 1 : pt;
        const int ty = t9 / 3;
        const int yy = py + (ty - 1) * p.dil;
        const int xx = px + (t9 - 3 * ty - 1) * p.dil;
        const bool ok = pv && gg < p.kgroups && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W &&
                        (unsigned)tt < (unsigned)p.F;
        const int off = ((tt * p.H + yy) * p.W + xx) * p.lda + cgi * 16 + 4 * lq;
        const f32x4 v = *reinterpret_cast<const f32x4*>(Ab + (ok ? off : 0));
        a[r][g] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
}

// STATS = false: the caller guarantees p.stats == nullptr (the straight-line resident kernels).  A
// runtime stats branch there put its global load after the next tile's A prefetch, and the join of
// the two paths waited vmcnt(0): every tile drained the prefetch and the previous tile's stores.
// LayerNorm of the A rows: in registers (rowops.h ln_rows: the whole row is in the lane group; host:
// kchunks == 1, kgroups * 16 == ln_C), or from precomputed row statistics (STATS, K chunked).
template <int KG, bool STATS = true, int RT = kGemmRT>
__device__ __forceinline__ void apply_ln(const GemmParams& p, int b, int row0, int li, int HW,
                                         f32x4 (&a)[RT][KG]) {
#pragma clang fp contract(off)
  if (STATS && p.stats) {
    const float wb = (p.ln == 2) ? 1.f : 0.f;
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const int prow = min(row0 + r * 16 + li, HW - 1);
      const float2 st = *reinterpret_cast<const float2*>(p.stats + 2 * ((long long)b * HW + prow));
      const float sh = st.x * wb;
#pragma unroll
      for (int g = 0; g < KG; ++g) a[r][g] = (a[r][g] - sh) * st.y;
    }
    return;
  }
  ln_rows<KG, RT>(p.ln, p.ln_C, p.kgroups, a);
}

// acc[t][r] += W-tile(t) x A(r) over the KG k-groups of `a` (fp32 rows, LN applied): pair G's B
// operands are split right before its MFMAs (2 x 12 VGPRs live, not KP x 24); split records of tile t
// at wl + (t * ldk + G) * kRec3.  Tiles are walked in units of two (4 independent accumulators).
template <int NT, int KG, int RT = kGemmRT>
__device__ __forceinline__ void mfma_chunk3(const f32x4* __restrict__ wl, int ldk, int lane,
                                            const f32x4 (&a)[RT][KG], f32x4 (&acc)[NT][RT]) {
  constexpr int KP = (KG + 1) / 2, NU = (NT + 1) / 2;
#pragma unroll
  for (int G = 0; G < KP; ++G) {
    F3 x[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r)
      x[r] = split3(a[r][2 * G], 2 * G + 1 < KG ? a[r][2 * G + 1] : f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int t = 2 * u;
      const f32x4* w0 = wl + (t * ldk + G) * kRec3 + lane;
      if (t + 1 < NT)
        mfma6_pair<RT, true>(w0, w0 + ldk * kRec3, x, acc[t], acc[t + 1]);
      else
        mfma6_pair<RT, false>(w0, w0, x, acc[t], acc[t]);
    }
  }
}

template <int NT, int OUT, bool HASR>
__device__ __forceinline__ void epilogue(const GemmParams& p, int b, int row0, int nt0, int tmax, int li, int lq,
                                         int HW, f32x4 (&acc)[NT][kGemmRT], const f32x4* bl) {
  // bl: this n-chunk's bias in LDS, 4 float4 per output tile (zeros when the layer has none).
  // vmcnt retires in order, so waiting for a global load issued after a store also drains that
  // store.  The residual of tile t+1 is therefore loaded before tile t is stored (one tile ahead),
  // and the bias comes from LDS: no load ever waits behind the store it follows.
  const float* __restrict__ Rb = p.R ? p.R + (long long)b * HW * p.ldr : nullptr;
  float* __restrict__ Ob = p.out + (OUT == 0 ? (long long)b * HW * p.ldo : 0);
  if constexpr (OUT == 0) {
    // residual loads are unconditional (addresses clamped in bounds, value selected after) so the
    // epilogue stays one basic block and the compiler can count vmcnt exactly
    auto load_res = [&](int t, f32x4 (&rv)[kGemmRT]) {
      const int nq = (nt0 + t) * 16 + 4 * lq;
      const bool tok = t < tmax && nq < p.N;
#pragma unroll
      for (int r = 0; r < kGemmRT; ++r) {
        const int pl = row0 + r * 16 + li;
        const bool ok = tok && pl < HW;
        const f32x4 v = *reinterpret_cast<const f32x4*>(Rb + (ok ? pl * p.ldr + nq : 0));
        rv[r] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    };
    [[maybe_unused]] f32x4 rc[kGemmRT], rn[kGemmRT];
    if constexpr (HASR) load_res(0, rc);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if constexpr (HASR) {
        if (t + 1 < NT) load_res(t + 1, rn);
      }
      const int nq = (nt0 + t) * 16 + 4 * lq;
      if (t < tmax && nq < p.N) {
#pragma unroll
        for (int r = 0; r < kGemmRT; ++r) {
          const int pl = row0 + r * 16 + li;
          if (pl >= HW) continue;
          f32x4 v = acc[t][r] + bl[4 * t + lq];
          if constexpr (HASR) v += rc[r];
          if (p.relu) v = f32x4{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
          *reinterpret_cast<f32x4*>(Ob + pl * p.ldo + nq) = v;
        }
      }
      if constexpr (HASR) {
#pragma unroll
        for (int r = 0; r < kGemmRT; ++r) rc[r] = rn[r];
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n0 = (nt0 + t) * 16;
    if (t >= tmax || n0 >= p.N) continue;
    const int nq = n0 + 4 * lq;
    const f32x4 bias = bl[4 * t + lq];
#pragma unroll
    for (int r = 0; r < kGemmRT; ++r) {
      const int pl = row0 + r * 16 + li;
      if (pl >= HW) continue;
      f32x4 v = acc[t][r] + bias;
      {
        const int fhw = p.H * p.W;
        const int t = pl / fhw;
        const int rem = pl - t * fhw;
        const int y = rem / p.W, x = rem - y * p.W;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = nq + e;
          if (n >= p.N) continue;
          float val = v[e];
          long long dst;
          int ch;
          if (OUT == 1) {
            const int Wo = p.W >> 1, Ho = p.H >> 1;
            dst = ((long long)b * p.F + t) * Ho * Wo + (y >> 1) * Wo + (x >> 1);
            ch = n * 4 + (y & 1) * 2 + (x & 1);
          } else {
            dst = ((long long)b * p.F + t) * 4 * fhw + (2 * y + ((n >> 1) & 1)) * (2 * p.W) + 2 * x + (n & 1);
            ch = n >> 2;
          }
          if (p.R) val += p.R[dst * p.ldr + ch];  // residual in the OUTPUT geometry (ConvTranspose3d + skip)
          if (p.relu) val = fmaxf(val, 0.f);
          Ob[dst * p.ldo + ch] = val;
        }
      }
    }
  }
}

// WPE = waves per SIMD the register budget must allow: 2 (<= 256 VGPRs, one 8-wave block per CU)
// or 4 (<= 128 VGPRs, two blocks per CU: more latency hiding for the store-heavy small-K shapes).
template <int NT, int KG, bool CONV3, int OUT, bool PF, int WPE, bool RES>
__global__ __launch_bounds__(kGemmThreads, WPE) void conv_gemm_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) f32x4 wlds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int HW = p.F * p.H * p.W;  // pixels per image (x frames for 3-D sequences)
  const int t_begin = blockIdx.x * p.tiles_per_block;
  const int t_end = min(t_begin + p.tiles_per_block, p.total_tiles);
  if (t_begin >= t_end) return;

  constexpr int KP = (KG + 1) / 2;  // split pairs per k-chunk
  if constexpr (RES) {
    // ------------------------------------------------------------------ resident schedule
    const int g0 = blockIdx.y * p.group_tiles;                       // first output tile of the group
    const int gtiles = min(p.group_tiles, p.ntiles - g0);
    int staged = -1;
    f32x4 a[kGemmRT][KG];
    [[maybe_unused]] f32x4 an[kGemmRT][KG];
    if (PF) {
      const int b = t_begin / p.tiles_per_img;
      load_a<KG, CONV3>(p, p.A + (long long)b * HW * p.lda,
                        (t_begin - b * p.tiles_per_img) * kGemmRows + wave * (kGemmRT * 16), 0, li, lq, HW, an);
    }
    const int n4pad = ((gtiles + NT - 1) / NT) * NT * KP * kRec3;  // partial last chunk reads zeros
    for (int tile = t_begin; tile < t_end; ++tile) {
      const int b = tile / p.tiles_per_img;
      const int row0 = (tile - b * p.tiles_per_img) * kGemmRows + wave * (kGemmRT * 16);
      const int wkey = p.w_img_stride ? b : 0;
      if (staged != wkey) {
        __syncthreads();
        const f32x4* wbase =
            reinterpret_cast<const f32x4*>(p.Wp + (long long)wkey * p.w_img_stride) + (long long)g0 * KP * kRec3;
        const int n4 = gtiles * KP * kRec3;
        for (int idx = tid; idx < n4pad; idx += kGemmThreads)
          wlds[idx] = idx < n4 ? wbase[idx] : f32x4{0.f, 0.f, 0.f, 0.f};
        const int nb4 = ((gtiles + NT - 1) / NT) * NT * 4;                  // bias of the group's tiles
        for (int idx = tid; idx < nb4; idx += kGemmThreads) {
          const int n = g0 * 16 + 4 * idx;
          wlds[n4pad + idx] = (p.bias && idx < gtiles * 4 && n < p.N) ? *reinterpret_cast<const f32x4*>(p.bias + n)
                                                                         : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        __syncthreads();
        staged = wkey;
      }
      if (PF) {
#pragma unroll
        for (int r = 0; r < kGemmRT; ++r)
#pragma unroll
          for (int g = 0; g < KG; ++g) a[r][g] = an[r][g];
        if (tile + 1 < t_end) {
          const int bn = (tile + 1) / p.tiles_per_img;
          load_a<KG, CONV3>(p, p.A + (long long)bn * HW * p.lda,
                            (tile + 1 - bn * p.tiles_per_img) * kGemmRows + wave * (kGemmRT * 16), 0, li, lq,
                            HW, an);
        }
      } else {
        load_a<KG, CONV3>(p, p.A + (long long)b * HW * p.lda, row0, 0, li, lq, HW, a);
      }
      if (p.ln) apply_ln<KG>(p, b, row0, li, HW, a);
      for (int c0 = 0; c0 < gtiles; c0 += NT) {
        f32x4 acc[NT][kGemmRT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < kGemmRT; ++r) acc[t][r] = f32x4{0.f, 0.f, 0.f, 0.f};
        mfma_chunk3<NT, KG>(wlds + (size_t)c0 * KP * kRec3, KP, lane, a, acc);
        const f32x4* bl = wlds + n4pad + c0 * 4;
        if (p.R) epilogue<NT, OUT, true>(p, b, row0, g0 + c0, gtiles - c0, li, lq, HW, acc, bl);
        else epilogue<NT, OUT, false>(p, b, row0, g0 + c0, gtiles - c0, li, lq, HW, acc, bl);
      }
    }
  } else {
    // ------------------------------------------------------------------ chunked schedule (RES == false)
    // k-chunk kc holds pairs kc KP .. kc KP + KP - 1 (the host keeps KG even when K takes several chunks)
    const int nc = blockIdx.y;
    const int KPt = (p.kgroups + 1) / 2;
    for (int tile = t_begin; tile < t_end; ++tile) {
      const int b = tile / p.tiles_per_img;
      const int row0 = (tile - b * p.tiles_per_img) * kGemmRows + wave * (kGemmRT * 16);
      const float* __restrict__ Ab = p.A + (long long)b * HW * p.lda;
      f32x4 acc[NT][kGemmRT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < kGemmRT; ++r) acc[t][r] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int kc = 0; kc < p.kchunks; ++kc) {
        const int wkey = p.w_img_stride ? b : 0;
        __syncthreads();
        const f32x4* wbase = reinterpret_cast<const f32x4*>(p.Wp + (long long)wkey * p.w_img_stride);
        for (int idx = tid; idx < NT * KP * kRec3; idx += kGemmThreads) {
          const int t = idx / (KP * kRec3);
          const int rem = idx - t * (KP * kRec3);
          const int G = rem / kRec3, sl = rem - G * kRec3;
          const int gt = nc * NT + t, gp = kc * KP + G;
          f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
          if (gt < p.ntiles && gp < KPt) v = wbase[((long long)gt * KPt + gp) * kRec3 + sl];
          wlds[idx] = v;
        }
        if (kc == 0)
          for (int idx = tid; idx < NT * 4; idx += kGemmThreads) {  // bias of the block's NT tiles
            const int n = nc * NT * 16 + 4 * idx;
            wlds[NT * KP * kRec3 + idx] =
                (p.bias && n < p.N) ? *reinterpret_cast<const f32x4*>(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
          }
        __syncthreads();
        f32x4 a[kGemmRT][KG];
        load_a<KG, CONV3>(p, Ab, row0, kc, li, lq, HW, a);
        if (p.ln) apply_ln<KG>(p, b, row0, li, HW, a);
        mfma_chunk3<NT, KG>(wlds, KP, lane, a, acc);
      }
      if (p.R) epilogue<NT, OUT, true>(p, b, row0, nc * NT, NT, li, lq, HW, acc, wlds + NT * KP * kRec3);
      else epilogue<NT, OUT, false>(p, b, row0, nc * NT, NT, li, lq, HW, acc, wlds + NT * KP * kRec3);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Resident 1x1 schedule, r02 ("straight-line"): the same work decomposition as the RES branch of
// conv_gemm_kernel, restructured so the compiler can count every vector-memory op.
//  * The n-chunk loop is unrolled (NCH = ceil(group_tiles / NT) is a template parameter) and every
//    global access is a raw BUFFER load/store through a per-image descriptor: rows past the image
//    and channels past N fall outside the descriptor's range, so out-of-range loads return 0 and
//    out-of-range stores are dropped by the hardware.  No exec-masked branches remain, so hipcc's
//    waitcnt pass sees one straight-line tile body and waits for exactly the loads it needs
//    (r01's kernel drained every store with vmcnt(0) inside the n-chunk loop: the PMC profile showed
//    waves parked on waitcnt for 32% of their cycles and the matrix pipe 58% busy).
//  * The next tile's A rows are always prefetched (the last tile re-reads its own rows) so the
//    count of outstanding ops is the same on every path; the residual of a chunk is loaded before
//    that chunk's MFMAs and consumed after them.
//  * ReLU is max(v, floor) with floor = 0 or -inf: no branch.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const float* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, (int)bytes, 0x00020000);
}
// cache policy of the streaming activation loads / output stores: the default (0).  r05 A/B
// (profiles/r05zz4_cache_policy_ab.txt): non-temporal stores or loads were level or slower on every shape
constexpr int kLdPol = 0, kStPol = 0;
__device__ __forceinline__ f32x4 buf_load4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, kLdPol));
}
__device__ __forceinline__ void buf_store4(__amdgpu_buffer_rsrc_t r, unsigned off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, kStPol);
}
constexpr unsigned kOOB = 0x80000000u;  // a byte offset past every descriptor's range

// Block -> (tile block bx, weight group / n-chunk by) of the resident and chunked kernels.  A tile
// block's A rows are read once per group, so the gy blocks of one tile block are launched as
// consecutive dispatches on one XCD: 1-D grid, id = s * 8 gy + j * 8 + k -> bx = 8 s + k, by = j
// (the hardware deals consecutive ids round-robin over the 8 XCDs, so k is the XCD).  They run side
// by side over the same tiles, and all but the first read of each A tile hit that XCD's L2 instead
// of HBM (with x-fastest 2-D grids the first ceil(gx / CUs) rounds were all group 0: every group
// re-read A from HBM).  gy = 1 keeps bx = id.  Ids past gx (the round-up to 8) exit.
__device__ __forceinline__ void block_tile_group(int gy, int& bx, int& by) {
  const int id = blockIdx.x, sgrp = id / (8 * gy), r = id - sgrp * 8 * gy;
  by = r >> 3;
  bx = sgrp * 8 + (r & 7);
}
static dim3 gemm_grid(int grid_x, int grid_y) {
  return dim3((unsigned)(((grid_x + 7) / 8) * 8 * grid_y));
}

// WPE = 2: 8 waves x 2 row subtiles (RT) per wave; WPE = 4 (r05): 16 waves x 1 subtile — the same
// 256-pixel block tile with twice the waves in flight at <= 128 VGPRs each (more loads and stores
// outstanding per CU; every W plane read from LDS feeds 1 row subtile instead of 2).
template <int NT, int KG, int NCH, int WPE, bool HASR, bool PF>
__global__ __launch_bounds__(kGemmThreads * WPE / 2, WPE) void gemm_res_kernel(GemmParams p) {
  constexpr int RT = WPE == 4 ? 1 : kGemmRT;
  constexpr int THREADS = kGemmThreads * WPE / 2;
  extern __shared__ __attribute__((aligned(16))) f32x4 wlds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int HW = p.F * p.H * p.W;
  int bx, by;
  block_tile_group((p.ntiles + p.group_tiles - 1) / p.group_tiles, bx, by);
  const int t_begin = bx * p.tiles_per_block;
  const int t_end = min(t_begin + p.tiles_per_block, p.total_tiles);
  if (t_begin >= t_end) return;
  const int g0 = by * p.group_tiles;
  const int gtiles = min(p.group_tiles, p.ntiles - g0);
  constexpr int KP = (KG + 1) / 2;  // split pairs
  constexpr int TP = NT * NCH;      // tiles staged per group (zero weights past gtiles)
  constexpr int WS = TP * KP * kRec3;  // weight slots in LDS; the bias follows
  // weights are per image when w_img_stride != 0 (the MDTA-folded projection M = W_proj blockdiag(A))
  auto stage = [&](int wkey) {
    const f32x4* wbase =
        reinterpret_cast<const f32x4*>(p.Wp + (long long)wkey * p.w_img_stride) + (long long)g0 * KP * kRec3;
    const int n4 = gtiles * KP * kRec3;
    for (int idx = tid; idx < WS; idx += THREADS) wlds[idx] = idx < n4 ? wbase[idx] : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int idx = tid; idx < TP * 4; idx += THREADS) {
      const int n = g0 * 16 + 4 * idx;
      wlds[WS + idx] = (p.bias && idx < gtiles * 4 && n < p.N) ? *reinterpret_cast<const f32x4*>(p.bias + n)
                                                                : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  int staged = p.w_img_stride ? t_begin / p.tiles_per_img : 0;
  stage(staged);
  __syncthreads();
  const unsigned a_bytes = (unsigned)HW * (unsigned)p.lda * 4u;
  const unsigned o_bytes = (unsigned)HW * (unsigned)p.ldo * 4u;
  const unsigned r_bytes = (unsigned)HW * (unsigned)p.ldr * 4u;
  // Output / residual addresses: voffset = the lane's pixel row + the group's first channel + its
  // channel quad (computed once per tile; the buffer size for rows past the image), plus t * 64 for
  // staged tile t, a constant hipcc folds into the instruction's offset field.  Padding tiles of a
  // partial group select the buffer size (a block-uniform v_cndmask), so the range check drops them.
  // soffset stays 0: with an SGPR soffset hipcc stops padding the store-data hazard of the x4
  // stores it emits (the data VGPRs were rewritten right after issue: wrong outputs on the GPU).
  auto tile_voff = [&](int t, unsigned v, unsigned bytes) -> int {
    return (int)(((t < gtiles) ? v : bytes) + 64u * (unsigned)t);
  };
  auto rows_of = [&](int tile, int& b, int& row0) {
    b = tile / p.tiles_per_img;
    row0 = (tile - b * p.tiles_per_img) * kGemmRows + wave * (RT * 16);
  };
  auto load_rows = [&](int tile, f32x4 (&dst)[RT][KG]) {
    int b, row0;
    rows_of(tile, b, row0);
    const __amdgpu_buffer_rsrc_t ra = buf_rsrc(p.A + (long long)b * HW * p.lda, a_bytes);
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const unsigned pix = (unsigned)(row0 + r * 16 + li);
      const unsigned base = pix < (unsigned)HW ? pix * (unsigned)p.lda * 4u + 16u * lq : kOOB;
#pragma unroll
      for (int g = 0; g < KG; ++g) dst[r][g] = buf_load4(ra, base + 64u * g);
    }
  };
  [[maybe_unused]] f32x4 an[RT][KG];
  if constexpr (PF) load_rows(t_begin, an);
  // The tile body runs once peeled, then in the loop: hipcc's waitcnt pass merges the loop header's
  // predecessors and keeps the smaller outstanding count, so with the prologue (12 loads in flight)
  // as a predecessor it waited for the previous tile's stores before the next tile's first use of its
  // prefetched rows; peeled, both predecessors have stores behind the prefetch.
  auto body = [&](int tile) __attribute__((always_inline)) {
    int b, row0;
    rows_of(tile, b, row0);
    if (p.w_img_stride && b != staged) {  // block-uniform: the tile range crossed into the next image
      __syncthreads();
      stage(b);
      __syncthreads();
      staged = b;
    }
    f32x4 a[RT][KG];
    if constexpr (PF) {
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int g = 0; g < KG; ++g) a[r][g] = an[r][g];
      load_rows(min(tile + 1, t_end - 1), an);  // unconditional: same op count on every path
    } else {
      load_rows(tile, a);
    }
    if (p.ln) apply_ln<KG, false, RT>(p, b, row0, li, HW, a);
    // K = 96 (unit-major body below): every pair's B operands split once per tile
    [[maybe_unused]] F3 xg[KP][RT];
    if constexpr (KG == 6) {
#pragma unroll
      for (int G = 0; G < KP; ++G)
#pragma unroll
        for (int r = 0; r < RT; ++r) xg[G][r] = split3(a[r][2 * G], a[r][2 * G + 1]);
    }
    const __amdgpu_buffer_rsrc_t ro = buf_rsrc(p.out + (long long)b * HW * p.ldo, o_bytes);
    [[maybe_unused]] __amdgpu_buffer_rsrc_t rr;
    if constexpr (HASR) rr = buf_rsrc(p.R + (long long)b * HW * p.ldr, r_bytes);
    unsigned vo[RT], vr[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const unsigned pix = (unsigned)(row0 + r * 16 + li);
      vo[r] = pix < (unsigned)HW ? pix * (unsigned)p.ldo * 4u + 16u * lq + 64u * g0 : o_bytes;
      vr[r] = pix < (unsigned)HW ? pix * (unsigned)p.ldr * 4u + 16u * lq + 64u * g0 : r_bytes;
    }
    if constexpr (KG == 6) {
    // K = 96: unit-major chunk body.  Each tile pair is accumulated over every pair and stored before
    // the next tile pair starts, so a pair's stores issue beside the next pair's MFMAs instead of in
    // one burst after all of them; only 4 accumulators are live.  Same per-tile summation order (pair
    // ascending, mfma6's term order) as mfma_chunk3: identical outputs.
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const f32x4* wl = wlds + (size_t)ch * NT * KP * kRec3;
      const f32x4* bl = wlds + WS + ch * NT * 4;
      constexpr int NU = (NT + 1) / 2;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int t = 2 * u;
        [[maybe_unused]] f32x4 rs[2][RT];
        if constexpr (HASR) {
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int r = 0; r < RT; ++r)
              rs[q][r] = (t + q < NT)
                             ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                             rr, tile_voff(ch * NT + t + q, vr[r], r_bytes), 0, 0))
                             : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        f32x4 a0[RT], a1[RT];
#pragma unroll
        for (int r = 0; r < RT; ++r) a0[r] = a1[r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int G = 0; G < KP; ++G) {
          const f32x4* w0 = wl + (t * KP + G) * kRec3 + lane;
          if (t + 1 < NT)
            mfma6_pair<RT, true>(w0, w0 + KP * kRec3, xg[G], a0, a1);
          else
            mfma6_pair<RT, false>(w0, w0, xg[G], a0, a1);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (t + q >= NT) continue;
          const f32x4 bias = bl[4 * (t + q) + lq];
#pragma unroll
          for (int r = 0; r < RT; ++r) {
            f32x4 v = (q == 0 ? a0[r] : a1[r]) + bias;
            if constexpr (HASR) v += rs[q][r];
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ro,
                                                   tile_voff(ch * NT + t + q, vo[r], o_bytes), 0, kStPol);
          }
        }
      }
    }
    } else {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      [[maybe_unused]] f32x4 res[NT][RT];
      if constexpr (HASR) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < RT; ++r)
            res[t][r] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, tile_voff(ch * NT + t, vr[r], r_bytes), 0, 0));
      }
      f32x4 acc[NT][RT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < RT; ++r) acc[t][r] = f32x4{0.f, 0.f, 0.f, 0.f};
      mfma_chunk3<NT, KG, RT>(wlds + (size_t)ch * NT * KP * kRec3, KP, lane, a, acc);
      // bias after the K sum, as every other GEMM schedule does: a pixel's result must not depend
      // on which schedule (batch size) produced it
      const f32x4* bl = wlds + WS + ch * NT * 4;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f32x4 bias = bl[4 * t + lq];
#pragma unroll
        for (int r = 0; r < RT; ++r) {
          f32x4 v = acc[t][r] + bias;
          if constexpr (HASR) v += res[t][r];
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ro, tile_voff(ch * NT + t, vo[r], o_bytes),
                                                 0, kStPol);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // keep one chunk's accumulators live at a time
    }
    }
  };
  body(t_begin);
  for (int tile = t_begin + 1; tile < t_end; ++tile) body(tile);
}

// ---------------------------------------------------------------------------------------------
// Fused attention output + FFN input, r02 (C = 48 blocks: one head, one resident weight group):
//   x1  = x + M v (+ bias_m)        M = W_proj blockdiag(A) per image (attn_fold; :140-144, :160)
//   out = LN(x1) W_in^T (+ bias)     LayerNorm + ffn.project_in (:161, :99), chunk-interleaved rows
// in one pass over the pixel tiles.  The M GEMM's accumulator (lane: pixel li, channels 4 lq..+3 of
// output tile t) IS the A-row layout of the second GEMM (k-group t), so x1 goes from the MFMA
// accumulators through the residual add and LayerNorm into the project_in MFMAs without leaving
// registers; it is stored once (the FFN's residual) and never re-read.  The unfused pair wrote x1,
// then read it back, and its N = 48 GEMM ran at ~4.5 TB/s / 36 TF/s.
// Numerics: both GEMMs accumulate pair-major in mfma6's term order exactly as gemm_res_kernel does, and
// x1 = (acc + bias_m) + x in that order, so the result equals the unfused path bit for bit.
template <int NT, int KG, int NCH>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_attn_in_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) f32x4 wlds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int HW = p.F * p.H * p.W;
  const int t_begin = blockIdx.x * p.tiles_per_block;
  const int t_end = min(t_begin + p.tiles_per_block, p.total_tiles);
  if (t_begin >= t_end) return;
  constexpr int KP = (KG + 1) / 2;   // split pairs
  constexpr int TP = NT * NCH;       // project_in tiles staged (zero weights past ntiles)
  constexpr int WS = TP * KP * kRec3;
  f32x4* ml = wlds + WS + TP * 4;    // M split records [KG tiles][KP pairs][kRec3], then bias_m [KG][4]
  {
    const f32x4* wbase = reinterpret_cast<const f32x4*>(p.Wp);
    const int n4 = p.ntiles * KP * kRec3;
    for (int idx = tid; idx < WS; idx += kGemmThreads) wlds[idx] = idx < n4 ? wbase[idx] : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int idx = tid; idx < TP * 4; idx += kGemmThreads) {
      const int n = 4 * idx;
      wlds[WS + idx] = (p.bias && idx < p.ntiles * 4 && n < p.N) ? *reinterpret_cast<const f32x4*>(p.bias + n)
                                                                  : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  auto stage_m = [&](int b) {
    const f32x4* mb = reinterpret_cast<const f32x4*>(p.Wm + (long long)b * p.wm_img_stride);
    for (int idx = tid; idx < KG * KP * kRec3; idx += kGemmThreads) ml[idx] = mb[idx];
    for (int idx = tid; idx < KG * 4; idx += kGemmThreads)
      ml[KG * KP * kRec3 + idx] =
          p.bias_m ? *reinterpret_cast<const f32x4*>(p.bias_m + 4 * idx) : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  int staged = t_begin / p.tiles_per_img;
  stage_m(staged);
  __syncthreads();
  const unsigned a_bytes = (unsigned)HW * (unsigned)p.lda * 4u;
  const unsigned o_bytes = (unsigned)HW * (unsigned)p.ldo * 4u;
  const unsigned r_bytes = (unsigned)HW * (unsigned)p.ldr * 4u;
  const unsigned o1_bytes = (unsigned)HW * (unsigned)p.ldo1 * 4u;
  auto tile_voff = [&](int t, unsigned v, unsigned bytes) -> int {
    return (int)(((t < p.ntiles) ? v : bytes) + 64u * (unsigned)t);
  };
  auto rows_of = [&](int tile, int& b, int& row0) {
    b = tile / p.tiles_per_img;
    row0 = (tile - b * p.tiles_per_img) * kGemmRows + wave * (kGemmRT * 16);
  };
  auto load_rows = [&](const float* base, int ld, unsigned bytes, int tile, f32x4 (&dst)[kGemmRT][KG]) {
    int b, row0;
    rows_of(tile, b, row0);
    const __amdgpu_buffer_rsrc_t ra = buf_rsrc(base + (long long)b * HW * ld, bytes);
#pragma unroll
    for (int r = 0; r < kGemmRT; ++r) {
      const unsigned pix = (unsigned)(row0 + r * 16 + li);
      const unsigned off = pix < (unsigned)HW ? pix * (unsigned)ld * 4u + 16u * lq : kOOB;
#pragma unroll
      for (int g = 0; g < KG; ++g) dst[r][g] = buf_load4(ra, off + 64u * g);
    }
  };
  // v rows are prefetched a tile ahead at K = 48; at K = 96 the extra 48 VGPRs would spill, and the
  // SIMD partner wave's MFMAs cover the load instead
  constexpr bool PFV = KG < 6;
  constexpr bool PFX = false;  // x rows a tile ahead as well: r04 A/B no gain (kept for the layout notes)
  f32x4 a[kGemmRT][KG];
  [[maybe_unused]] f32x4 an[kGemmRT][KG];
  [[maybe_unused]] f32x4 xn[kGemmRT][KG];
  if constexpr (PFV) load_rows(p.A, p.lda, a_bytes, t_begin, an);
  if constexpr (PFX) load_rows(p.R, p.ldr, r_bytes, t_begin, xn);
  // first tile peeled, as in gemm_res_kernel: the loop header then has no predecessor without the
  // previous tile's stores queued behind the v prefetch, so the first use of v waits for the loads only
  auto body = [&](int tile) __attribute__((always_inline)) {
    int b, row0;
    rows_of(tile, b, row0);
    if (b != staged) {  // block-uniform: the tile range crossed into the next image
      __syncthreads();
      stage_m(b);
      __syncthreads();
      staged = b;
    }
    if constexpr (PFV) {
#pragma unroll
      for (int r = 0; r < kGemmRT; ++r)
#pragma unroll
        for (int g = 0; g < KG; ++g) a[r][g] = an[r][g];
    } else {
      load_rows(p.A, p.lda, a_bytes, tile, a);
    }
    // x of this tile (read before x1 overwrites the same rows, by the same lanes), waited for after
    // the M GEMM; a one-tile-ahead prefetch of x measured no faster (registers).  At K = 96 the
    // x rows are loaded after the M GEMM: live across it they would spill
    f32x4 xr[kGemmRT][KG];
    if constexpr (PFX) {
#pragma unroll
      for (int r = 0; r < kGemmRT; ++r)
#pragma unroll
        for (int g = 0; g < KG; ++g) xr[r][g] = xn[r][g];
    } else if constexpr (KG < 6) {
      load_rows(p.R, p.ldr, r_bytes, tile, xr);
    }
    if constexpr (PFV) load_rows(p.A, p.lda, a_bytes, min(tile + 1, t_end - 1), an);  // next tile's v
    if constexpr (PFX) load_rows(p.R, p.ldr, r_bytes, min(tile + 1, t_end - 1), xn);
    {
      f32x4 acc1[KG][kGemmRT];
#pragma unroll
      for (int t = 0; t < KG; ++t)
#pragma unroll
        for (int r = 0; r < kGemmRT; ++r) acc1[t][r] = f32x4{0.f, 0.f, 0.f, 0.f};
      mfma_chunk3<KG, KG>(ml, KP, lane, a, acc1);
      if constexpr (KG >= 6) load_rows(p.R, p.ldr, r_bytes, tile, xr);
      const f32x4* bm = ml + KG * KP * kRec3;
      const __amdgpu_buffer_rsrc_t r1 = buf_rsrc(p.out1 + (long long)b * HW * p.ldo1, o1_bytes);
#pragma unroll
      for (int r = 0; r < kGemmRT; ++r) {
        const unsigned pix = (unsigned)(row0 + r * 16 + li);
        const unsigned off = pix < (unsigned)HW ? pix * (unsigned)p.ldo1 * 4u + 16u * lq : o1_bytes;
#pragma unroll
        for (int g = 0; g < KG; ++g) {
          f32x4 v = acc1[g][r] + bm[4 * g + lq];
          v += xr[r][g];
          a[r][g] = v;
          buf_store4(r1, off + 64u * g, v);
        }
      }
    }
    apply_ln<KG, false>(p, b, row0, li, HW, a);
    const __amdgpu_buffer_rsrc_t ro = buf_rsrc(p.out + (long long)b * HW * p.ldo, o_bytes);
    unsigned vo[kGemmRT];
#pragma unroll
    for (int r = 0; r < kGemmRT; ++r) {
      const unsigned pix = (unsigned)(row0 + r * 16 + li);
      vo[r] = pix < (unsigned)HW ? pix * (unsigned)p.ldo * 4u + 16u * lq : o_bytes;
    }
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      f32x4 acc[NT][kGemmRT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < kGemmRT; ++r) acc[t][r] = f32x4{0.f, 0.f, 0.f, 0.f};
      mfma_chunk3<NT, KG>(wlds + (size_t)ch * NT * KP * kRec3, KP, lane, a, acc);
      const f32x4* bl = wlds + WS + ch * NT * 4;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f32x4 bias = bl[4 * t + lq];
#pragma unroll
        for (int r = 0; r < kGemmRT; ++r)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[t][r] + bias), ro,
                                                 tile_voff(ch * NT + t, vo[r], o_bytes), 0, kStPol);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep one chunk's accumulators live at a time
    }
  };
  body(t_begin);
  for (int tile = t_begin + 1; tile < t_end; ++tile) body(tile);
}

// ---------------------------------------------------------------------------------------------
// Chunked schedule, r02 (deep 1x1 layers with K > the LDS budget, every implicit 3x3 / 3x3x3 conv):
// the block walks its pixel tiles x k-chunks as one sequence of steps.  Per step:
//   s_waitcnt vmcnt(0) + barrier   (this step's weights and A rows were issued one step earlier);
//   issue the NEXT step's weight chunk by buffer-load-to-LDS (double-buffered slots; out-of-range
//   records come back as zeros) and its A rows into registers (buffer loads, zero outside the image
//   or past K, so the 3x3 zero padding needs no branch);
//   6 x NT x KG / 2 split MFMAs per row subtile on this step's operands; at a tile's last k-chunk the
//   epilogue.
// r01's version staged each weight chunk through VGPRs behind two __syncthreads and loaded A only
// after them, so every k-chunk exposed two memory latencies with both waves of a SIMD parked.
template <int NT, int KG, bool CONV3, int OUT, bool HASR>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_chunk_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) f32x4 wlds[];
  constexpr int KP = (KG + 1) / 2;                    // split pairs per k-chunk (KG even when K takes several)
  constexpr int SLOT = NT * KP * kRec3;               // f32x4 per weight slot
  constexpr int PIECES = NT * KP * 3;                 // 1 KiB planes per chunk
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int HW = p.F * p.H * p.W;
  int bx, nc;
  block_tile_group((p.ntiles + NT - 1) / NT, bx, nc);
  const int t_begin = bx * p.tiles_per_block;
  const int t_end = min(t_begin + p.tiles_per_block, p.total_tiles);
  if (t_begin >= t_end) return;
  const int KC = p.kchunks;
  f32x4* bias_l = wlds + 2 * SLOT;
  for (int idx = tid; idx < NT * 4; idx += kGemmThreads) {
    const int n = nc * NT * 16 + 4 * idx;
    bias_l[idx] = (p.bias && n < p.N) ? *reinterpret_cast<const f32x4*>(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int KPt = (p.kgroups + 1) / 2;
  const unsigned w_bytes = (unsigned)p.ntiles * (unsigned)KPt * 3072u;
  const unsigned a_bytes = (unsigned)HW * (unsigned)p.lda * 4u;
  // weights of step (tile, kc) -> slot; record (t, G) of the chunk = split record (nc*NT + t, kc*KP + G)
  auto issue_w = [&](int tile, int kc, int slot) {
    const int b = tile / p.tiles_per_img;
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.Wp + (p.w_img_stride ? (long long)b * p.w_img_stride : 0LL)),
                                          0, (int)w_bytes, 0x00020000);
    f32x4* dst = wlds + slot * SLOT;
#pragma unroll
    for (int j = 0; j < (PIECES + 7) / 8; ++j) {
      const int k = wave + 8 * j;
      if (k >= PIECES) break;
      const int t = k / (3 * KP), rem = k - t * (3 * KP);
      const int G = rem / 3, pl = rem - 3 * G;
      const int gt = nc * NT + t, gp = kc * KP + G;
      const unsigned off =
          (gt < p.ntiles && gp < KPt) ? (unsigned)((gt * KPt + gp) * 3 + pl) * 1024u + 16u * lane : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(dst + 64 * k), 16, (int)off,
                                               0, 0, 0);
    }
  };
  auto load_a2 = [&](int tile, int kc, f32x4 (&dst)[kGemmRT][KG]) {
    const int b = tile / p.tiles_per_img;
    const int row0 = (tile - b * p.tiles_per_img) * kGemmRows + wave * (kGemmRT * 16);
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.A + (long long)b * HW * p.lda), 0, (int)a_bytes, 0x00020000);
#pragma unroll
    for (int r = 0; r < kGemmRT; ++r) {
      const int prow = row0 + r * 16 + li;
      const bool pv = prow < HW;
      if constexpr (!CONV3) {
        const unsigned base = (unsigned)(prow * p.lda + 4 * lq) * 4u;
#pragma unroll
        for (int g = 0; g < KG; ++g) {
          const int gg = kc * KG + g;
          dst[r][g] = buf_load4(ra, (pv && gg < p.kgroups) ? base + 64u * gg : kOOB);
        }
      } else {
        const int fhw = p.H * p.W;
        const int pt = prow / fhw;
        const int rem = prow - pt * fhw;
        const int py = rem / p.W;
        const int px = rem - py * p.W;
#pragma unroll
        for (int g = 0; g < KG; ++g) {
          const int gg = kc * KG + g;
          const int tap = gg / p.cg_per_tap;
          const int cgi = gg - tap * p.cg_per_tap;
          const int t9 = p.kt == 3 ? tap - (tap / 9) * 9 : tap;
          const int tt = p.kt == 3 ? pt + tap / 9 - 1 : pt;
          const int ty = t9 / 3;
          const int yy = py + (ty - 1) * p.dil;
          const int xx = px + (t9 - 3 * ty - 1) * p.dil;
          const bool ok = pv && gg < p.kgroups && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W &&
                          (unsigned)tt < (unsigned)p.F;
          dst[r][g] = buf_load4(ra, ok ? (unsigned)(((tt * p.H + yy) * p.W + xx) * p.lda + cgi * 16 + 4 * lq) * 4u : kOOB);
        }
      }
    }
  };
  // LN row statistics (mean, rstd) of the chunk's rows, precomputed by ln_stats (K is chunked)
  // (p.stats is null when the whole LN row fits one k-chunk: then the row is normalised in registers)
  auto load_stats = [&](int b, int row0, float2 (&st)[kGemmRT]) {
    if (!p.stats) return;
#pragma unroll
    for (int r = 0; r < kGemmRT; ++r) {
      const int prow = min(row0 + r * 16 + li, HW - 1);
      st[r] = *reinterpret_cast<const float2*>(p.stats + 2 * ((long long)b * HW + prow));
    }
  };
  auto ln_apply = [&](int b, int row0, const float2 (&st)[kGemmRT], f32x4 (&x)[kGemmRT][KG]) {
#pragma clang fp contract(off)  // apply_ln's rounding (the r01 kernel's stats path)
    if (!p.stats) {
      apply_ln<KG>(p, b, row0, li, HW, x);
      return;
    }
    const float wb = (p.ln == 2) ? 1.f : 0.f;
#pragma unroll
    for (int r = 0; r < kGemmRT; ++r) {
      const float sh = st[r].x * wb;
#pragma unroll
      for (int g = 0; g < KG; ++g) x[r][g] = (x[r][g] - sh) * st[r].y;
    }
  };
  f32x4 a[kGemmRT][KG], an[kGemmRT][KG];
  f32x4 acc[NT][kGemmRT];
  issue_w(t_begin, 0, 0);
  load_a2(t_begin, 0, an);
  int slot = 0;
  for (int tile = t_begin; tile < t_end; ++tile) {
    const int b = tile / p.tiles_per_img;
    const int row0 = (tile - b * p.tiles_per_img) * kGemmRows + wave * (kGemmRT * 16);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < kGemmRT; ++r) acc[t][r] = f32x4{0.f, 0.f, 0.f, 0.f};
    // one step: wait + barrier, operands of step (ntile, nkc) in flight, MFMAs of this step
    auto begin_step = [&]() {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kGemmRT; ++r)
#pragma unroll
        for (int g = 0; g < KG; ++g) a[r][g] = an[r][g];
    };
    float2 st[kGemmRT];
    for (int kc = 0; kc + 1 < KC; ++kc) {
      begin_step();
      if (p.ln) load_stats(b, row0, st);
      issue_w(tile, kc + 1, slot ^ 1);
      load_a2(tile, kc + 1, an);
      if (p.ln) ln_apply(b, row0, st, a);
        mfma_chunk3<NT, KG>(wlds + slot * SLOT, KP, lane, a, acc);
      slot ^= 1;
    }
    // last k-chunk: residual loads, then the next tile's first operands (clamped, so the count of
    // memory ops is the same on every path), MFMAs, epilogue
    begin_step();
    if (p.ln) load_stats(b, row0, st);
    [[maybe_unused]] f32x4 res[NT][kGemmRT];
    if constexpr (HASR && OUT == 0) {
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(p.R + (long long)b * HW * p.ldr), 0, (int)((unsigned)HW * (unsigned)p.ldr * 4u), 0x00020000);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int nq = (nc * NT + t) * 16 + 4 * lq;
#pragma unroll
        for (int r = 0; r < kGemmRT; ++r) {
          const int pl = row0 + r * 16 + li;
          res[t][r] = buf_load4(rr, (pl < HW && nq < p.N) ? (unsigned)(pl * p.ldr + nq) * 4u : kOOB);
        }
      }
    }
    const int ntile = min(tile + 1, t_end - 1);
    issue_w(ntile, 0, slot ^ 1);
    load_a2(ntile, 0, an);
    if (p.ln) ln_apply(b, row0, st, a);
      mfma_chunk3<NT, KG>(wlds + slot * SLOT, KP, lane, a, acc);
    slot ^= 1;
    if constexpr (OUT == 0) {
      const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
          p.out + (long long)b * HW * p.ldo, 0, (int)((unsigned)HW * (unsigned)p.ldo * 4u), 0x00020000);
      const float relu_floor = p.relu ? 0.f : -__builtin_huge_valf();
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int nq = (nc * NT + t) * 16 + 4 * lq;
        const f32x4 bias = bias_l[4 * t + lq];
#pragma unroll
        for (int r = 0; r < kGemmRT; ++r) {
          const int pl = row0 + r * 16 + li;
          f32x4 v = acc[t][r] + bias;
          if constexpr (HASR) v += res[t][r];
          v = f32x4{fmaxf(v.x, relu_floor), fmaxf(v.y, relu_floor), fmaxf(v.z, relu_floor), fmaxf(v.w, relu_floor)};
          buf_store4(ro, (pl < HW && nq < p.N) ? (unsigned)(pl * p.ldo + nq) * 4u : kOOB, v);
        }
      }
    } else {
      epilogue<NT, OUT, HASR>(p, b, row0, nc * NT, NT, li, lq, HW, acc, bias_l);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped last prefetch lands before exit
}

// (NT, KG, CONV3, OUT, PF, WPE, RES).  Resident variants need KG == kgroups exactly.
#define KDLAE_GEMM_VARIANTS(X) \
  X(9, 3, false, 0, true, 2, true) X(8, 3, false, 0, true, 2, true) X(3, 3, false, 0, true, 2, true) \
  X(6, 3, false, 0, true, 2, true) X(9, 6, false, 0, true, 2, true) X(8, 6, false, 0, true, 2, true) \
  X(6, 6, false, 0, true, 2, true) X(3, 6, false, 0, true, 2, true) X(3, 8, false, 0, true, 2, true) \
  X(6, 8, false, 0, true, 2, true) X(6, 12, false, 0, false, 2, true) X(8, 12, false, 0, false, 2, true) \
  X(3, 12, false, 0, false, 2, true) X(6, 16, false, 0, false, 2, true) X(3, 16, false, 0, false, 2, true) \
  X(3, 3, false, 0, false, 2, false) X(6, 6, false, 0, false, 2, false) \
  X(8, 12, false, 0, false, 2, false) X(6, 12, false, 0, false, 2, false) X(3, 12, false, 0, false, 2, false) \
  X(6, 16, false, 0, false, 2, false) X(3, 16, false, 0, false, 2, false) \
  X(12, 8, false, 0, false, 2, false) \
  X(3, 6, true, 1, false, 2, false) X(6, 6, true, 1, false, 2, false) \
  X(6, 12, true, 1, false, 2, false) X(12, 6, true, 1, false, 2, false) \
  X(3, 6, true, 2, false, 2, false) X(6, 6, true, 2, false, 2, false) \
  X(6, 12, true, 2, false, 2, false) X(12, 6, true, 2, false, 2, false) \
  X(2, 6, true, 2, false, 2, false) X(2, 6, true, 1, false, 2, false) \
  \
  X(8, 6, true, 0, false, 2, false) X(4, 6, true, 0, false, 2, false) X(2, 6, true, 0, false, 2, false) \
  X(1, 3, false, 0, false, 2, false) X(3, 4, false, 0, false, 2, false) X(4, 4, false, 2, false, 2, false) \
  X(8, 4, false, 2, false, 2, false) X(4, 2, false, 2, false, 2, false) X(3, 3, false, 2, false, 2, false) \
  X(6, 4, true, 1, false, 2, false) X(8, 4, true, 1, false, 2, false) X(6, 4, true, 2, false, 2, false) \
  X(8, 4, true, 2, false, 2, false) X(8, 4, true, 0, false, 2, false) \
  X(4, 4, true, 0, false, 2, false) X(2, 4, true, 0, false, 2, false)

bool gemm_has_variant(int NT, int KG, bool conv3, int wpe, bool resident, int out_mode) {
#define X(a, b, c, o, f, w, r) \
  if (NT == a && KG == b && conv3 == c && wpe == w && resident == r && out_mode == o) return true;
  KDLAE_GEMM_VARIANTS(X)
#undef X
  return false;
}

template <int NT, int KG, bool C3, int OUT, bool PF, int WPE, bool RES>
static hipError_t launch_variant(const GemmParams& p, int grid_x, int grid_y, size_t lds, hipStream_t s) {
  // the dynamic-LDS attribute is per device: one high-water mark per device id
  static size_t attr_lds[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (lds > attr_lds[dev]) {
    hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&conv_gemm_kernel<NT, KG, C3, OUT, PF, WPE, RES>),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr_lds[dev] = lds;
  }
  hipLaunchKernelGGL((conv_gemm_kernel<NT, KG, C3, OUT, PF, WPE, RES>), dim3(grid_x, grid_y), dim3(kGemmThreads),
                     lds, s, p);
  return hipGetLastError();
}

// (NT, KG, NCH, PF) of the straight-line resident kernel; launched for both HASR values
#define KDLAE_GEMM_RES2_VARIANTS(X) \
  X(9, 3, 1, true) X(9, 3, 2, true) X(8, 3, 1, true) X(8, 3, 2, true) X(3, 3, 1, true) X(3, 3, 2, true) \
  X(6, 3, 1, true) X(6, 3, 2, true) X(9, 6, 1, true) X(8, 6, 1, true) X(8, 6, 2, true) \
  X(6, 6, 1, true) X(6, 6, 2, true) X(3, 6, 1, true) X(3, 6, 2, true) X(3, 8, 1, true) X(3, 8, 2, true) \
  X(6, 8, 1, true) X(6, 8, 2, true) X(6, 12, 1, false) X(8, 12, 1, false) \
  X(3, 12, 1, false) X(3, 12, 2, false) X(6, 16, 1, false) X(3, 16, 1, false)
// (choose_variant keeps an entry's NT x NCH x ceil(KG/2) x 3 KiB of split weights <= 158 KiB)

// residual (HASR) instance only where launch_gemm's no-spill rule (res_ok) can admit a residual
template <int NT, int KG, int NCH>
constexpr bool res2_hasr_ok() { return NT * NCH <= 12 && NT * NCH * KG <= 72 && KG <= 8; }

// waves per SIMD of the resident kernel: 2 = 8 waves x 32 rows (16 waves x 16 rows at K <= 96 measured
// no faster in r05)
template <int NT, int KG, int NCH, bool PF>
static hipError_t launch_res2(const GemmParams& p, int grid_x, int grid_y, size_t lds, hipStream_t s) {
  constexpr bool RK = res2_hasr_ok<NT, KG, NCH>();
  constexpr int W = 2;
  constexpr int TH = kGemmThreads * W / 2;
  static size_t attr_lds[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (lds > attr_lds[dev]) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_res_kernel<NT, KG, NCH, W, false, PF>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if constexpr (RK) {
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_res_kernel<NT, KG, NCH, W, true, PF>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    attr_lds[dev] = lds;
  }
  if constexpr (RK) {
    if (p.R) {
      hipLaunchKernelGGL((gemm_res_kernel<NT, KG, NCH, W, true, PF>), gemm_grid(grid_x, grid_y), dim3(TH), lds, s, p);
      return hipGetLastError();
    }
  }
  if (p.R) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm_res_kernel<NT, KG, NCH, W, false, PF>), gemm_grid(grid_x, grid_y), dim3(TH), lds, s, p);
  return hipGetLastError();
}

// (NT, KG, CONV3, OUT) of the r02 chunked kernel: two weight slots of NT x ceil(KG/2) x 3 KiB must fit
// the LDS
// (only shapes whose A double buffer + accumulators fit 256 VGPRs without spills: NT x KG <= ~64)
#define KDLAE_GEMM_CHUNK2_VARIANTS(X) \
  X(3, 3, false, 0) X(6, 6, false, 0) X(12, 4, false, 0) X(1, 3, false, 0) X(3, 4, false, 0) \
  X(3, 6, true, 1) X(2, 6, true, 1) \
  X(3, 6, true, 2) X(2, 6, true, 2) \
  X(4, 6, true, 0) X(2, 6, true, 0) \
  X(4, 4, false, 2) X(8, 4, false, 2) X(4, 2, false, 2) X(3, 3, false, 2) \
  X(6, 4, true, 1) X(8, 4, true, 1) X(6, 4, true, 2) X(8, 4, true, 2) X(8, 4, true, 0) \
  X(4, 4, true, 0) X(2, 4, true, 0)
// (r05: the split-MFMA instances that spill at 256 VGPRs — NT x KG = 36..48 on the implicit 3x3 convs,
// KG = 9 — were dropped; the 3x3 convs take 4-deep k-chunks instead)

// (NT, KG, NCH) of the fused attention-output + project_in kernel (C = 48: K = 3 groups)
#define KDLAE_GEMM_ATTN_IN_VARIANTS(X) X(8, 3, 2) X(9, 3, 2) X(6, 3, 3)

// the variant exists and its project_in weights + the per-image M (split records) fit the LDS
bool gemm_attn_in_variant(int NT, int KG, int nch) {
#define X(a, b, c) \
  if (NT == a && KG == b && nch == c)     \
    return w3_bytes((long long)NT * nch, KG) + (size_t)NT * nch * 64 + w3_bytes(KG, KG) + (size_t)KG * 64 <= 160 * 1024;
  KDLAE_GEMM_ATTN_IN_VARIANTS(X)
#undef X
  return false;
}

bool gemm_has_variant2(int NT, int KG, bool conv3, int out_mode) {
#define X(a, b, c, o) \
  if (NT == a && KG == b && conv3 == c && out_mode == o) return true;
  KDLAE_GEMM_CHUNK2_VARIANTS(X)
#undef X
  return false;
}

template <int NT, int KG, bool C3, int OUT>
static hipError_t launch_chunk2(const GemmParams& p, int grid_x, int grid_y, hipStream_t s) {
  const size_t lds = 2 * w3_bytes(NT, KG) + (size_t)NT * 64;
  static size_t attr_lds[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  constexpr bool R0 = (OUT == 0 && !C3 && NT * KG < 36);  // residual variants without spills
  if (lds > attr_lds[dev]) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_chunk_kernel<NT, KG, C3, OUT, false>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (R0) {
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_chunk_kernel<NT, KG, C3, OUT, R0>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    attr_lds[dev] = lds;
  }
  if (R0 && p.R)
    hipLaunchKernelGGL((gemm_chunk_kernel<NT, KG, C3, OUT, R0>), gemm_grid(grid_x, grid_y), dim3(kGemmThreads), lds, s, p);
  else if (OUT == 0 && p.R)
    return hipErrorInvalidValue;  // (no residual variant: the host picks another NT x KG)
  else
    hipLaunchKernelGGL((gemm_chunk_kernel<NT, KG, C3, OUT, false>), gemm_grid(grid_x, grid_y), dim3(kGemmThreads), lds, s,
                       p);
  return hipGetLastError();
}

// route 0: the production dispatch; route 1 (self-test only): skip the r02 straight-line resident
// and chunked kernels so the r01 conv_gemm_kernel instance of (NT, KG) runs — the fallback the
// production dispatch takes for views those kernels cannot address (ld % 4 != 0, > 2 GiB images)
hipError_t launch_gemm_route(const GemmParams& p, int NT, int KG, int wpe, int grid_x, int route, hipStream_t s) {
  const bool c3 = p.ksize == 3;
  const bool res = p.group_tiles > 0;
  if (p.ln && !p.stats && (p.kchunks > 1 || p.kgroups > KG)) return hipErrorInvalidValue;  // LN needs whole rows
  // split pairs must not straddle k-chunks: every chunk starts on an even k-group (mfma3.h)
  if (p.kchunks > 1 && KG % 2) return hipErrorInvalidValue;
  if (p.Wm) {  // fused attention output + LN + GEMM: one resident group, K = N of the M GEMM = C
    const int nch = (p.ntiles + NT - 1) / NT;
    const size_t lds = w3_bytes((long long)NT * nch, KG) + (size_t)NT * nch * 64 + w3_bytes(KG, KG) + (size_t)KG * 64;
    const long long HW = (long long)p.F * p.H * p.W;
    const long long mx = HW * std::max({p.lda, p.ldo, p.ldr, p.ldo1}) * 4;
    if (!res || c3 || p.out_mode || p.group_tiles < p.ntiles || p.kgroups != KG || p.kchunks != 1 || p.relu ||
        !p.R || !p.out1 || p.stats || mx >= (1LL << 31) || lds > 160 * 1024 || p.lda % 4 || p.ldo % 4 || p.ldr % 4 ||
        p.ldo1 % 4)
      return hipErrorInvalidValue;
#define X(a, b, c)                                                                                            \
    if (NT == a && KG == b && nch == c) {                                                                     \
      static size_t attr_lds[64] = {};                                                                        \
      int dev = 0;                                                                                            \
      if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;                                  \
      if (lds > attr_lds[dev]) {                                                                              \
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_attn_in_kernel<a, b, c>),      \
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);             \
        if (e != hipSuccess) return e;                                                                        \
        attr_lds[dev] = lds;                                                                                  \
      }                                                                                                       \
      hipLaunchKernelGGL((gemm_attn_in_kernel<a, b, c>), dim3(grid_x, 1), dim3(kGemmThreads), lds, s, p);    \
      return hipGetLastError();                                                                               \
    }
    KDLAE_GEMM_ATTN_IN_VARIANTS(X)
#undef X
    return hipErrorInvalidValue;
  }
  if (route == 0 && res && !c3 && p.out_mode == 0 && wpe == 2 && p.kgroups == KG && p.kchunks == 1 && !p.relu &&
      !p.stats) {
    const long long HW = (long long)p.F * p.H * p.W;
    const long long mx = HW * std::max(std::max(p.lda, p.ldo), p.R ? p.ldr : 0) * 4;
    const int nch = (p.group_tiles + NT - 1) / NT;
    const int grid_y = (p.ntiles + p.group_tiles - 1) / p.group_tiles;
    const size_t lds = w3_bytes((long long)NT * nch, KG) + (size_t)NT * nch * 64;
    // residual variants keep NT x 2 residual float4 live across the chunk's MFMAs: only where that
    // fits the 256-VGPR budget without spills (hipcc -Rpass-analysis), else the r01 kernel
    const bool res_ok = !p.R || (NT * nch <= 12 && NT * nch * KG <= 72 && KG <= 8 && p.ldr % 4 == 0);  // no VGPR spills
    // (res2_hasr_ok is this rule at compile time: keep the two in step)
    if (mx < (1LL << 31) && lds <= 160 * 1024 && p.lda % 4 == 0 && p.ldo % 4 == 0 && res_ok) {
#define X(a, b, c, f) \
      if (NT == a && KG == b && nch == c) return launch_res2<a, b, c, f>(p, grid_x, grid_y, lds, s);
      KDLAE_GEMM_RES2_VARIANTS(X)
#undef X
    }
  }
  if (p.out_mode == 0 && (p.N % 16)) return hipErrorInvalidValue;  // plain stores are whole 16-channel tiles
  int grid_y;
  size_t lds;
  // LDS: packed weights, then the bias of the same output tiles (64 B per tile)
  if (res) {
    if (p.kgroups != KG || p.kchunks != 1) return hipErrorInvalidValue;
    grid_y = (p.ntiles + p.group_tiles - 1) / p.group_tiles;
    const size_t tiles_pad = (size_t)((p.group_tiles + NT - 1) / NT) * NT;
    lds = w3_bytes((long long)tiles_pad, p.kgroups) + tiles_pad * 64;
  } else {
    grid_y = (p.ntiles + NT - 1) / NT;
    lds = w3_bytes(NT, KG) + (size_t)NT * 64;
  }
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (route == 0 && !res && gemm_has_variant2(NT, KG, c3, p.out_mode) && p.lda % 4 == 0) {
    const long long HW = (long long)p.F * p.H * p.W;
    const long long osz = p.out_mode == 2 ? 4 * HW : (p.out_mode == 1 ? HW / 4 : HW);
    const bool fits = HW * p.lda * 4 < (1LL << 31) && osz * p.ldo * 4 < (1LL << 31) &&
                      (!p.R || osz * p.ldr * 4 < (1LL << 31)) && (long long)w3_bytes(p.ntiles, p.kgroups) < (1LL << 31);
    if (fits) {
#define X(a, b, c, o) \
      if (NT == a && KG == b && c3 == c && p.out_mode == o) return launch_chunk2<a, b, c, o>(p, grid_x, grid_y, s);
      KDLAE_GEMM_CHUNK2_VARIANTS(X)
#undef X
    }
  }
#define X(a, b, c, o, f, w, r)                                                                 \
  if (NT == a && KG == b && c3 == c && p.out_mode == o && wpe == w && res == r)                \
    return launch_variant<a, b, c, o, f, w, r>(p, grid_x, grid_y, lds, s);
  KDLAE_GEMM_VARIANTS(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t launch_gemm(const GemmParams& p, int NT, int KG, int wpe, int grid_x, hipStream_t s) {
  return launch_gemm_route(p, NT, KG, wpe, grid_x, 0, s);
}

// Entry i of a variant table (self-test enumeration): family 0 = conv_gemm_kernel (NT, KG, CONV3,
// OUT, PF, WPE, RES), 1 = gemm_res_kernel (NT, KG, NCH, PF), 2 = gemm_chunk_kernel (NT, KG, CONV3,
// OUT), 3 = gemm_attn_in_kernel (NT, KG, NCH).  Returns false past the end.
bool gemm_variant_entry(int family, int i, int* v) {
  int n = 0;
  switch (family) {
    case 0:
#define X(a, b, c, o, f, w, r) \
  if (n++ == i) { v[0] = a; v[1] = b; v[2] = c; v[3] = o; v[4] = f; v[5] = w; v[6] = r; return true; }
      KDLAE_GEMM_VARIANTS(X)
#undef X
      return false;
    case 1:
#define X(a, b, c, f) \
  if (n++ == i) { v[0] = a; v[1] = b; v[2] = c; v[3] = f; return true; }
      KDLAE_GEMM_RES2_VARIANTS(X)
#undef X
      return false;
    case 2:
#define X(a, b, c, o) \
  if (n++ == i) { v[0] = a; v[1] = b; v[2] = c; v[3] = o; return true; }
      KDLAE_GEMM_CHUNK2_VARIANTS(X)
#undef X
      return false;
    case 3:
#define X(a, b, c) \
  if (n++ == i) { v[0] = a; v[1] = b; v[2] = c; return true; }
      KDLAE_GEMM_ATTN_IN_VARIANTS(X)
#undef X
      return false;
    default:
      return false;
  }
}

}  // namespace kdlae
