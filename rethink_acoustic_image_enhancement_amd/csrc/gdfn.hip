// Fused GDFN tail (KDLAE/KDLAE_model.py:101-106):
//   out = x_res + project_out( gelu_erf(dw3x3(x1)) * dw3x3(x2) )
// in ONE pass over the project_in output.  The gated hidden tensor (hid channels per pixel) never
// reaches HBM: it is produced in registers in exactly the layout the MFMA B operand wants.
//
// Input layout (written by the project_in GEMM): per pixel 2*hidS floats, chunk-interleaved —
// chunk g (16 hidden channels) occupies floats [32g, 32g+16) for x1 and [32g+16, 32g+32) for x2,
// so one chunk of one pixel is a contiguous 128 B line.
//
// Block = 256 threads (4 waves, one workgroup per CU) on a 16 x 16 pixel tile; wave w owns tile
// rows 4w..4w+3, lane l owns pixel column l & 15 and channel quad l >> 4.  Per hidden chunk g
// (16 channels of x1 and the same 16 of x2):
//   * LDS-DMA (global_load_lds, no VGPRs) brings the chunk's 18 x 18 halo tile (one 128 B line per
//     pixel) and its depthwise weights + bias (2 KiB, repacked per chunk on the host) into a
//     3-slot stage ring, and its project_out W fragments (NT x 1 KiB) into a 4-slot W ring.
//     Iteration k issues chunk k+3, so chunks k+2 and k+3 are in flight while k+1 is gated and k
//     is multiplied; waits are counted (vmcnt = one chunk's DMAs per wave) and barriers raw, so the
//     in-flight chunks are never drained.  Nothing else in the loop reads global memory (an
//     ordinary load would make hipcc drain the DMAs before its use);
//   * the halo image is lane-linear [pixel][slot] with slot = quad ^ (column & 7) applied on the
//     SOURCE address, so the column reads of the stencil are bank-conflict-free;
//   * each lane computes the depthwise 3x3 + exact-erf gate for its 4 pixels (one per tile row) and
//     4 channels — a float4 which IS its B operand for the chunk's 4 MFMA k-steps
//     (B[k = 4(l>>4)+e][pixel l&15]); iteration g issues the MFMAs of chunk g in the same basic
//     block as the gate VALU of chunk g+1, so the two overlap.
// Epilogue: bias + residual, float4 stores of 4 consecutive output channels per lane.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include <algorithm>

#include "kernels.h"
#include "runtime.h"

namespace kdlae {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

#ifndef KDLAE_GELU_PACKED
#define KDLAE_GELU_PACKED 1
#endif
constexpr bool kGeluPacked = KDLAE_GELU_PACKED != 0;  // A/B knob: packed-FP32 GELU gate in gdfn_out
constexpr int kTile = 16;                          // output tile width (pixels); height TH is a parameter
constexpr int kHalo = kTile + 2;                   // 18 halo columns
constexpr int kDwF4 = 128;                         // per-chunk dw block: [9][8] weights, [8] bias, pad

// Stage slot geometry of a 16 x TH tile: the (TH+2) x 18 halo, one 128 B line (x1|x2 of the chunk,
// 8 float4 items) per pixel, staged as lane-linear 1 KiB DMA wave-instructions (piece k -> items
// 64k..64k+63) dealt round-robin over the waves, then the chunk's dw block.
template <int TH> struct GdTile {
  static constexpr int kHaloPx = (TH + 2) * kHalo;                 // 324 at TH = 16
  static constexpr int kStageItems = kHaloPx * 8;
  static constexpr int kStagePieces = (kStageItems + 63) / 64;     // 41 at TH = 16, 23 at TH = 8
  static constexpr int kStageF4 = kStagePieces * 64;
  static constexpr int kStageSlot = kStageF4 + kDwF4;
  template <int WAVES> static constexpr int stage_pieces(int w) { return (kStagePieces - w + WAVES - 1) / WAVES; }
  // DMA wave-instructions wave w issues per chunk: its stage pieces, W records t with
  // (t+1)%WAVES == w, the 2 dw-block pieces on the last wave
  template <int NT, int WAVES> static constexpr int dma_per_chunk(int w) {
    int n = stage_pieces<WAVES>(w) + (w == WAVES - 1 ? 2 : 0);
    for (int t = 0; t < NT; ++t) n += ((t + 1) % WAVES == w) ? 1 : 0;
    return n;
  }
  // halo pieces + the dw block of wave w: one chunk's DMAs when W travels separately (W2)
  template <int WAVES> static constexpr int stage_dma(int w) {
    return stage_pieces<WAVES>(w) + (w == WAVES - 1 ? 2 : 0);
  }
};

// Exact-erf GELU, 0.5 x (1 + erf(x / sqrt 2)), with erf from Abramowitz & Stegun 7.1.26
// (|error| <= 1.5e-7): branch-free, so the gate VALU stays in one basic block with the MFMAs it is
// interleaved with.  The GELU error is <= 7.5e-8 |x|, at the level of fp32 rounding of the result.
__device__ __forceinline__ float gelu_erf_g(float x) {
#ifdef KDLAE_PRECISE_GELU  // diagnostics build (tools/config1_taps.py): the device library's erff
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
#endif
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float poly = fmaf(1.061405429f, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  poly *= t;
  const float e = 1.0f - poly * __expf(-z * z);     // erf(|x| / sqrt 2)
  return 0.5f * x * (1.0f + copysignf(e, x));
}

// The same GELU on a pair, written on float2 so hipcc emits packed FP32 (v_pk_fma/v_pk_mul: two
// lanes' worth of the polynomial per instruction); rcp and exp stay per value.  The operations and
// their order match gelu_erf_g.  Measured (profiles/r02_gdfn_gelu_packed_probe.txt): C96 -1.9%,
// C48 -1%, C192 +1.5% per launch, so the wide (NT = 12) kernel keeps the scalar form.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_gate2(f32x2 x, f32x2 v) {
#ifdef KDLAE_PRECISE_GELU
  return f32x2{gelu_erf_g(x.x) * v.x, gelu_erf_g(x.y) * v.y};
#endif
  const f32x2 z = f32x2{fabsf(x.x), fabsf(x.y)} * 0.70710678118654752f;
  const f32x2 a = __builtin_elementwise_fma(f32x2{0.3275911f, 0.3275911f}, z, f32x2{1.0f, 1.0f});
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(a.x), __builtin_amdgcn_rcpf(a.y)};
  f32x2 poly = __builtin_elementwise_fma(f32x2{1.061405429f, 1.061405429f}, t, f32x2{-1.453152027f, -1.453152027f});
  poly = __builtin_elementwise_fma(poly, t, f32x2{1.421413741f, 1.421413741f});
  poly = __builtin_elementwise_fma(poly, t, f32x2{-0.284496736f, -0.284496736f});
  poly = __builtin_elementwise_fma(poly, t, f32x2{0.254829592f, 0.254829592f});
  poly *= t;
  const f32x2 nz2 = -z * z;
  const f32x2 ex = f32x2{__expf(nz2.x), __expf(nz2.y)};
  const f32x2 e = 1.0f - poly * ex;
  const f32x2 se = f32x2{copysignf(e.x, x.x), copysignf(e.y, x.y)};
  return ((0.5f * x) * (1.0f + se)) * v;
}

typedef unsigned u32x4g __attribute__((ext_vector_type(4)));
constexpr unsigned kOOB2 = 0x80000000u;  // a byte offset past every descriptor's range

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// s_waitcnt with only a vmcnt limit (gfx9 encoding: vmcnt[3:0] + [15:14], expcnt/lgkmcnt at max)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

__device__ __forceinline__ void dma16(const void* src, f32x4* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)lds_wave_base, 16, 0, 0);
}
// buffer form: voffset per lane, soffset (wave-uniform, SGPR) added outside the VALU; offsets past
// the descriptor's range land zeros
__device__ __forceinline__ void dma_buf(__amdgpu_buffer_rsrc_t r, f32x4* lds_wave_base, unsigned voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lptr_t)lds_wave_base, 16, (int)voff, soff, 0, 0);
}

// gate of one 16-hidden-channel chunk for RPW tile rows (the GDFN stencil): depthwise 3x3 of x1 and x2
// (rows of the wave, column cx, channels 4q..4q+3 of each half) + exact-erf gate -> the float4 that IS
// the lane's MFMA B operand.  sl: the chunk's halo image (lane-linear [pixel][slot], slot = quad ^
// (column & 7), kHalo columns per row); dw: the chunk's dw block ([9][8] weights, [8] bias at +72);
// lo[h][j]: the lane's read offset of half h, column tap j in the wave's first halo row.  Shared by
// gdfn_out_kernel and ffn48_kernel, so the two compute the same bits.
// LOWREG: a scheduling fence between the column taps, so at most one tap's halo reads are in flight
// (for callers with little register room left; the values are the same)
template <int RPW, bool PACKED, bool LOWREG = false>
__device__ __forceinline__ void gate_rows(const f32x4* sl, const f32x4* dw, const int (&lo)[2][3], int q,
                                          f32x4 (&gb)[RPW]) {
  f32x4 d[2][RPW];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const f32x4 bb = dw[72 + 4 * h + q];
#pragma unroll
    for (int r = 0; r < RPW; ++r) d[h][r] = bb;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      f32x4 wv[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) wv[i] = dw[(3 * i + j) * 8 + 4 * h + q];
#pragma unroll
      for (int rr = 0; rr < RPW + 2; ++rr) {
        const f32x4 v = (sl + lo[h][j])[rr * kHalo * 8];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int r = rr - i;
          if (r >= 0 && r < RPW) d[h][r] = v * wv[i] + d[h][r];
        }
      }
      if constexpr (LOWREG) __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    if constexpr (PACKED) {
      const f32x2 lo2 = gelu_gate2(f32x2{d[0][r].x, d[0][r].y}, f32x2{d[1][r].x, d[1][r].y});
      const f32x2 hi2 = gelu_gate2(f32x2{d[0][r].z, d[0][r].w}, f32x2{d[1][r].z, d[1][r].w});
      gb[r] = f32x4{lo2.x, lo2.y, hi2.x, hi2.y};
    } else {
      gb[r].x = gelu_erf_g(d[0][r].x) * d[1][r].x;
      gb[r].y = gelu_erf_g(d[0][r].y) * d[1][r].y;
      gb[r].z = gelu_erf_g(d[0][r].z) * d[1][r].z;
      gb[r].w = gelu_erf_g(d[0][r].w) * d[1][r].w;
    }
  }
}

}  // namespace

// W2: the project_out W fragments travel one chunk ahead of their MFMAs in a 2-slot ring of their
// own (issued after the barrier that retires the slot's previous reader) instead of riding with the
// stage 2 chunks ahead in a 3-slot ring: one W slot less of LDS, which lets C = 96 use 16 x 12
// tiles at two blocks per CU (2 x 34 KiB stage + 2 x 6 KiB W = exactly 80 KiB).  Needs NSTG = 2.
template <int NT, int WAVES, int TH, int NSTG, bool W2 = false>
__global__ __launch_bounds__(64 * WAVES, W2 ? 2 : 1) void gdfn_out_kernel(GdfnParams p) {
  using T = GdTile<TH>;
  constexpr int kStageItems = T::kStageItems, kStagePieces = T::kStagePieces;
  constexpr int kStageF4 = T::kStageF4, kStageSlot = T::kStageSlot;
  constexpr int kNStage = NSTG;                                // stage ring (halo + dw block)
  constexpr int kNW = W2 ? 2 : NSTG + 1;  // W ring: chunk c is multiplied in iteration c, chunk c+NSTG issued then
  static_assert(!W2 || NSTG == 2, "the W2 schedule is written for a 2-slot stage ring");
  constexpr int RPW = TH / WAVES;                              // tile rows per wave
  static_assert(RPW * WAVES == TH && NSTG >= 2, "tile rows per wave / ring depth");
  constexpr int kRounds = (kStagePieces + WAVES - 1) / WAVES;  // stage pieces per wave (max)
  extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
  f32x4* wring = lds + kNStage * kStageSlot;        // [kNW][NT][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: per-wave branches and LDS bases stay in SGPRs
  const int cx = lane & 15, q = lane >> 4;
  const int kch = p.hidS >> 4;

  // XCD-aware tile order: logical tiles [k*per, (k+1)*per) run on XCD k, so tiles that share halo
  // rows/columns share an L2.  The grid is padded to a multiple of 8.
  // With nsplit > 1 the nsplit blocks of one pixel tile (adjacent logical ids: same XCD, so the second
  // reads the halo from L2) each own NT of the layer's output tiles (C = 384: 2 x 12).
  const int tx_n = (p.W + kTile - 1) / kTile, ty_n = (p.H + TH - 1) / TH;
  const int nsp = p.nsplit > 1 ? p.nsplit : 1;
  const int ntiles = p.Bn * tx_n * ty_n * nsp;
  const int per = (int)(gridDim.x >> 3);
  int bid = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (bid >= ntiles) return;
  const int sp = bid % nsp;
  bid /= nsp;
  const int tx = bid % tx_n;
  bid /= tx_n;
  const int ty = bid % ty_n;
  const int b = bid / ty_n;
  const int x0 = tx * kTile, y0 = ty * TH;
  const long long HW = (long long)p.H * p.W;
  const float* X = p.x + (long long)b * HW * p.ld;

  // per-thread halo sources as 32-bit byte offsets into the image; chunk g adds 128 g bytes through
  // the DMA's scalar offset, so issuing a chunk costs no VALU.  Out-of-image pixels and tail items
  // get an offset past the descriptor's range: the buffer load returns zeros (the conv padding).
  unsigned srco[kRounds];
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const int it = (wave + WAVES * j) * 64 + lane;
    const int px = it >> 3, slot = it & 7;
    const int hy = px / kHalo, hx = px - hy * kHalo;
    const int quad = slot ^ (hx & 7);  // column swizzle: the halo row pitch (18) is even, so a
                                       // column-only XOR keeps every row's reads conflict-free and
                                       // leaves the row as an immediate offset
    const int yy = y0 - 1 + hy, xx = x0 - 1 + hx;
    const bool ok = it < kStageItems && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
    srco[j] = ok ? (unsigned)(((yy * p.W + xx) * p.ld + 4 * quad) * 4) : kOOB2;
  }
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(X), 0, (int)(HW * p.ld * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.Wp + (size_t)sp * NT * kch * 256), 0, NT * kch * 1024, 0x00020000);
  const int n0 = 16 * NT * sp;  // first output channel of this block
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.dw), 0, kch * kDwF4 * 16, 0x00020000);
  auto issue = [&](int g) {
    f32x4* sl = lds + (g % kNStage) * kStageSlot;
#pragma unroll
    for (int j = 0; j < kRounds; ++j) {
      const int k = wave + WAVES * j;
      if (k >= kStagePieces) break;
      dma_buf(rx, sl + 64 * k, srco[j], 128 * g);
    }
    if (wave == WAVES - 1) {
      dma_buf(rd, sl + kStageF4, 16u * lane, g * (kDwF4 * 16));
      dma_buf(rd, sl + kStageF4 + 64, 16u * lane + 1024u, g * (kDwF4 * 16));
    }
    if constexpr (!W2) {
      f32x4* wl = wring + (g % kNW) * (64 * NT);
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if ((t + 1) % WAVES == wave) dma_buf(rw, wl + 64 * t, 16u * lane, (t * kch + g) * 1024);
    }
  };
  [[maybe_unused]] auto issue_w = [&](int g) {
    f32x4* wl = wring + (g % kNW) * (64 * NT);
#pragma unroll
    for (int t = 0; t < NT; ++t)
      if ((t + 1) % WAVES == wave) dma_buf(rw, wl + 64 * t, 16u * lane, (t * kch + g) * 1024);
  };
  // wait until only the youngest chunk's DMAs are outstanding, then a raw barrier (a
  // __syncthreads() would wait vmcnt(0) and drain the ring)
  auto wait_chunks = [&](auto nchunks) {
    constexpr int K = decltype(nchunks)::value;
    switch (wave) {
      case 0: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(0 % WAVES)>(); break;
      case 1: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(1 % WAVES)>(); break;
      case 2: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(2 % WAVES)>(); break;
      case 3: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(3 % WAVES)>(); break;
      case 4: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(4 % WAVES)>(); break;
      case 5: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(5 % WAVES)>(); break;
      case 6: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(6 % WAVES)>(); break;
      case 7: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(7 % WAVES)>(); break;
      case 8: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(8 % WAVES)>(); break;
      case 9: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(9 % WAVES)>(); break;
      case 10: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(10 % WAVES)>(); break;
      case 11: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(11 % WAVES)>(); break;
      case 12: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(12 % WAVES)>(); break;
      case 13: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(13 % WAVES)>(); break;
      case 14: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(14 % WAVES)>(); break;
      default: wait_vmcnt<K * T::template dma_per_chunk<NT, WAVES>(15 % WAVES)>(); break;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // no LDS read may move above the barrier
  };
  auto wait_all = [&]() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // no LDS read may move above the barrier
  };

  f32x4 acc[RPW][NT];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-lane halo read offsets (f32x4 units) of the wave's first input row, column tap j, half h:
  // the other rows are immediate offsets (rr * 18 * 8), so the stencil needs no address VALU
  int lo[2][3];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int hx = cx + j;
      lo[h][j] = (RPW * wave * kHalo + hx) * 8 + ((4 * h + q) ^ (hx & 7));
    }
  // gate(g): depthwise 3x3 (rows 4w..4w+3, column cx, channels 16g+4q..+3 of x1 and x2) + gate
  auto gate = [&](int g, f32x4 (&gb)[RPW]) {
    const f32x4* sl = lds + (g % kNStage) * kStageSlot;
    gate_rows<RPW, kGeluPacked && NT <= 6>(sl, sl + kStageF4, lo, q, gb);  // [9][8] then bias [8]
  };
  auto mfma_chunk = [&](int g, const f32x4 (&gb)[RPW]) {
    const f32x4* wl = wring + (g % kNW) * (64 * NT);
    f32x4 w[NT];                                   // every W fragment first: one LDS wait per chunk
#pragma unroll
    for (int t = 0; t < NT; ++t) w[t] = wl[64 * t + lane];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        acc[r][t] = mfma4(w[t].x, gb[r].x, acc[r][t]);
        acc[r][t] = mfma4(w[t].y, gb[r].y, acc[r][t]);
        acc[r][t] = mfma4(w[t].z, gb[r].z, acc[r][t]);
        acc[r][t] = mfma4(w[t].w, gb[r].w, acc[r][t]);
      }
    }
  };

  f32x4 gb[RPW];
  if constexpr (W2) {
    // S0, W0, S1 in flight; gate(0) needs S0 (and iteration 0 W0): wait for all but S1's DMAs
    issue(0);
    issue_w(0);
    if (kch > 1) {
      issue(1);
      switch (wave) {
        case 0: wait_vmcnt<T::template stage_dma<WAVES>(0 % WAVES)>(); break;
        case 1: wait_vmcnt<T::template stage_dma<WAVES>(1 % WAVES)>(); break;
        case 2: wait_vmcnt<T::template stage_dma<WAVES>(2 % WAVES)>(); break;
        case 3: wait_vmcnt<T::template stage_dma<WAVES>(3 % WAVES)>(); break;
        case 4: wait_vmcnt<T::template stage_dma<WAVES>(4 % WAVES)>(); break;
        case 5: wait_vmcnt<T::template stage_dma<WAVES>(5 % WAVES)>(); break;
        case 6: wait_vmcnt<T::template stage_dma<WAVES>(6 % WAVES)>(); break;
        default: wait_vmcnt<T::template stage_dma<WAVES>(7 % WAVES)>(); break;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      wait_all();
    }
    gate(0, gb);
    for (int g = 0; g + 1 < kch; ++g) {
      // S(g+1) and W(g) (issued one iteration ago) landed; past the barrier every wave is done with
      // gate(g) (stage slot g%2) and mfma(g-1) (W slot (g+1)%2)
      wait_all();
      if (g + 2 < kch) issue(g + 2);
      issue_w(g + 1);
      f32x4 gbn[RPW];
      gate(g + 1, gbn);
      mfma_chunk(g, gb);
#pragma unroll
      for (int r = 0; r < RPW; ++r) gb[r] = gbn[r];
    }
    if (kch > 1) wait_all();  // W(kch-1)
    mfma_chunk(kch - 1, gb);
  } else {
  // prologue: chunks 0 .. NSTG-1 in flight; gate(0) once chunk 0 has landed
#pragma unroll
  for (int c = 0; c < NSTG; ++c)
    if (c < kch) issue(c);
  if (kch >= NSTG) wait_chunks(std::integral_constant<int, NSTG - 1>{});
  else wait_all();
  gate(0, gb);
  for (int g = 0; g + 1 < kch; ++g) {
    // issued so far: chunks 0..g+NSTG-1.  gate(g+1) needs chunk g+1; younger chunks may stay in flight.
    if (g + NSTG - 1 < kch) wait_chunks(std::integral_constant<int, NSTG - 2>{});
    else wait_all();
    // past this barrier every wave is done with gate(g) (stage slot g%NSTG) and mfma(g-1) (W slot
    // (g-1)%kNW = (g+NSTG)%kNW): chunk g+NSTG can reuse both
    if (g + NSTG < kch) issue(g + NSTG);
    f32x4 gbn[RPW];
    gate(g + 1, gbn);
    mfma_chunk(g, gb);
#pragma unroll
    for (int r = 0; r < RPW; ++r) gb[r] = gbn[r];
  }
  mfma_chunk(kch - 1, gb);
  }

  // epilogue: lane holds output channels 16t + 4q .. +3 of pixel (y0 + 4w + r, x0 + cx)
  // All loads (bias, every row's residual; clamped rows, unconditional) before the first store: vmcnt
  // retires in order, so a load issued after a store would make its wait drain that store.
  const int xo = x0 + cx;
  if (xo >= p.W) return;
  f32x4 bias[NT], res[RPW][NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
    bias[t] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + n0 + 16 * t + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int yo = min(y0 + RPW * wave + r, p.H - 1);
    const long long pix = (long long)b * HW + (long long)yo * p.W + xo;
#pragma unroll
    for (int t = 0; t < NT; ++t)
      res[r][t] = p.R ? *reinterpret_cast<const f32x4*>(p.R + pix * p.ldr + n0 + 16 * t + 4 * q)
                      : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int yo = y0 + RPW * wave + r;
    if (yo >= p.H) continue;
    const long long pix = (long long)b * HW + (long long)yo * p.W + xo;
#pragma unroll
    for (int t = 0; t < NT; ++t)
      *reinterpret_cast<f32x4*>(p.out + pix * p.ldo + n0 + 16 * t + 4 * q) = acc[r][t] + res[r][t] + bias[t];
  }
}


bool gdfn_supported(int C, int hidS) {
  return (C == 48 || C == 96 || C == 192 || C == 384) && hidS % 16 == 0 && hidS <= (C >= 192 ? 1024 : 256);
}

template <int NT, int WAVES, int TH, int NSTG, bool W2 = false>
static hipError_t launch_gdfn1(const GdfnParams& p, hipStream_t s) {
  const size_t lds = (size_t)(NSTG * GdTile<TH>::kStageSlot + (W2 ? 2 : NSTG + 1) * 64 * NT) * sizeof(f32x4);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  static size_t attr[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (lds > 64 * 1024 && lds > attr[dev]) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gdfn_out_kernel<NT, WAVES, TH, NSTG, W2>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr[dev] = lds;
  }
  const long long tiles = (long long)p.Bn * ((p.H + TH - 1) / TH) * ((p.W + kTile - 1) / kTile) *
                          (p.nsplit > 1 ? p.nsplit : 1);
  const long long grid = (tiles + 7) / 8 * 8;
  hipLaunchKernelGGL((gdfn_out_kernel<NT, WAVES, TH, NSTG, W2>), dim3((unsigned)grid), dim3(64 * WAVES), lds, s, p);
  return hipGetLastError();
}

static hipError_t launch_gdfn_out_small(const GdfnParams& p, int C, hipStream_t s);

hipError_t launch_gdfn_out(const GdfnParams& p, int C, hipStream_t s) {
  if (!gdfn_supported(C, p.hidS) || p.ld != 2 * p.hidS || p.ldo % 4 || (p.R && p.ldr % 4) || !p.zeros)
    return hipErrorInvalidValue;
  if (C >= 192) {
    // C = 192 / 384 (r02): 16 x 8 tiles, 2-slot stage ring + 2-slot W ring (2 x 25.5 + 2 x 12 KiB =
    // 75 KiB: two blocks per CU) and 12 output tiles per block (96 MFMAs per wave and chunk against
    // the same stencil VALU); C = 384 runs two blocks per pixel tile
    GdfnParams q = p;
    q.nsplit = C / 192;
    return launch_gdfn1<12, 4, 8, 2, true>(q, s);
  }
  GdfnParams q = p;
  q.nsplit = 1;
  return launch_gdfn_out_small(q, C, s);
}

static hipError_t launch_gdfn_out_small(const GdfnParams& p, int C, hipStream_t s) {
  // C = 96: 16 x 12 tiles with the W ring 2 slots deep (exactly 80 KiB: two blocks per CU):
  // C96@512^2 3.52 -> 3.37 ms, @256^2 0.866 -> 0.848 ms (profiles/r02_gdfn_c96_tile12_probe.txt).
  // Measured and dropped (profiles/r02_gdfn_tile_variants_probe.txt, r02_gdfn_variants2_probe.txt,
  // r02_gdfn2_vs_gdfn1_probe.txt): 16 x 16 tiles with 3 stage slots at one block per CU (r01),
  // 16 x 4 / 16 x 8 tiles, 2-wave blocks, and a barrier-free persistent strip schedule.
  if (C == 96) return launch_gdfn1<6, 4, 12, 2, true>(p, s);
  // C = 48: 16 x 12 tiles, 3 rows per wave.  77 KB of LDS still fits two blocks per CU (the 3 KiB W
  // records of NT = 3 leave room), and the halo and W/dw refetch per pixel drop by a third:
  // C48@1024^2 5.68 -> 5.42 ms, @512^2 1.46 -> 1.42 ms (profiles/r02_gdfn_c48_tile12_probe.txt).
  return launch_gdfn1<3, 4, 12, 2>(p, s);
}

// ---------------------------------------------------------------------------------------------
// Fused C = 48 FFN (r04, KDLAE_model.py:140-144, :160-161, :101-106): one kernel from the attention's
// v and the block input x to the block output, replacing gemm_attn_in_kernel<8,3,2> (x1 = x + M v,
// LN, project_in -> 2 hid-wide rows in HBM) + gdfn_out_kernel<3,4,12,2> (those rows back with a halo,
// dwconv + gate + project_out + residual).  The C = 48 blocks run at 512^2 and 1024^2 and were
// HBM-bound: 3008 B of traffic per pixel for the pair, ~600 B here.  The price is project_in (and
// M v, LN) recomputed on the tile's halo ring: 252 halo pixels per 192 outputs.
//  * block = 4 waves (one per SIMD, up to 512 VGPRs each: the LN'd halo rows, both accumulator sets
//    and the gate fit without spills; 8-wave 16 x 24 tiles at 256 VGPRs spilled ~180), a 16 x 12 pixel
//    tile (wave w owns tile rows 3w..3w+2, as gdfn_out's lanes do), persistent over the tiles of its
//    XCD; all weights (project_in 48 KiB, project_out 24 KiB, dw 16 KiB, biases) resident in LDS, M
//    restaged when the image changes;
//  * phase A: the 18 x 14 halo = 14 row tiles of 16 pixels + 2 column tiles; wave w takes halo rows
//    3w+1..3w+3 (its output rows: their x1 is kept as the residual) and one of the 4 remaining
//    tiles.  x1 = (M v + bias_m) + x, LayerNorm, in registers (lane: pixel, channel quad);
//  * per 16-channel hidden chunk g: project_in of tiles 2g, 2g+1 (x1 and x2 halves) for the wave's
//    halo pixels -> the chunk's halo image in LDS (gdfn_out's layout; out-of-image pixels 0), barrier,
//    gate_rows (the gdfn_out stencil) -> project_out MFMAs; project_in of chunk g+1 is issued beside
//    the gate of chunk g.
//  Every value is computed by the same operation sequence as the kernel pair (same fragments, same
//  MFMA k order per accumulator, the same LN and gate code), so the output is bit-identical.
namespace {
constexpr int kF48RPW = 3, kF48Main = 4, kF48TH = kF48RPW * kF48Main;   // 12 tile rows
constexpr int kF48Waves = 2 * kF48Main;                                  // + 4 project_in waves
constexpr int kF48HR = kF48TH + 2;                                     // 14 halo rows
constexpr int kF48Px = kF48HR * kHalo;                                 // 252 halo pixels
constexpr int kF48Kch = 8;                                             // hidden chunks (hidS = 128)
constexpr int kF48Tin = 2 * kF48Kch;                                   // project_in output tiles
// LDS carve, f32x4 units
constexpr int kF48Hb = 0;                                // [2][252 px][8 slots] chunk halo images
constexpr int kF48Win = kF48Hb + 2 * kF48Px * 8;         // [16 tiles][3 k-groups][64]
constexpr int kF48Dw = kF48Win + kF48Tin * 3 * 64;       // [8 chunks][128]
constexpr int kF48M = kF48Dw + kF48Kch * kDwF4;          // [3][3][64] folded projection of the image
constexpr int kF48Bm = kF48M + 9 * 64;                   // [12] bias_m
constexpr int kF48Bin = kF48Bm + 12;                     // [64] bias_in
constexpr int kF48Bout = kF48Bin + kF48Tin * 4;          // [12] bias_out
constexpr int kF48Lds = (kF48Bout + 12) * 16;            // 140,672 bytes: one block per CU
static_assert(kF48Lds <= 160 * 1024, "ffn48 LDS");

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// x1 = (M v + bias_m) + x for one 16-pixel tile (lane: pixel li, channel quad lq), the M GEMM in
// gemm_attn_in's per-accumulator order (k-group major, k-step minor)
__device__ __forceinline__ void f48_x1(const f32x4* ml, const f32x4* bm, int lane, int lq, const f32x4 (&va)[3],
                                       const f32x4 (&xa)[3], f32x4 (&x1)[3]) {
  f32x4 a1[3] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    f32x4 wm[3];
#pragma unroll
    for (int tt = 0; tt < 3; ++tt) wm[tt] = ml[(tt * 3 + g) * 64 + lane];
#pragma unroll
    for (int ss = 0; ss < 4; ++ss)
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) a1[tt] = mfma4(wm[tt][ss], va[g][ss], a1[tt]);
  }
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    f32x4 v = a1[g] + bm[4 * g + lq];
    v += xa[g];
    x1[g] = v;
  }
}
}  // namespace

__global__ __launch_bounds__(64 * kF48Waves, 1) void ffn48_kernel(Ffn48Params p) {
  extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool main_w = wave < kF48Main;                    // gate + project_out of tile rows 3w..3w+2
  const int hw = main_w ? wave : wave - kF48Main;         // helper index / row group of the wave
  const int li = lane & 15, lq = lane >> 4;
  const int tx_n = p.W / kTile, ty_n = (p.H + kF48TH - 1) / kF48TH;
  const int per_img = tx_n * ty_n;
  const int ntiles = p.Bn * per_img;
  const long long HW = (long long)p.H * p.W;
  // persistent and XCD-aware: XCD k (blockIdx & 7) walks logical tiles [k T / 8, (k+1) T / 8), its
  // blocks interleaved, so tiles that share halo rows run together on one L2
  const int xcd = (int)(blockIdx.x & 7), nxb = (int)(gridDim.x >> 3), xb = (int)(blockIdx.x >> 3);
  const int t_lo = (int)((long long)ntiles * xcd / 8), t_hi = (int)((long long)ntiles * (xcd + 1) / 8);
  if (t_lo + xb >= t_hi) return;

  // resident weights (project_out's stream from L2 into the main waves' registers, a chunk ahead)
  {
    const f32x4* win = reinterpret_cast<const f32x4*>(p.Win);
    for (int i = tid; i < kF48Tin * 3 * 64; i += 64 * kF48Waves) lds[kF48Win + i] = win[i];
    const f32x4* dwg = reinterpret_cast<const f32x4*>(p.dw);
    for (int i = tid; i < kF48Kch * kDwF4; i += 64 * kF48Waves) lds[kF48Dw + i] = dwg[i];
    for (int i = tid; i < kF48Tin * 4; i += 64 * kF48Waves)
      lds[kF48Bin + i] = p.bias_in ? reinterpret_cast<const f32x4*>(p.bias_in)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int i = tid; i < 12; i += 64 * kF48Waves)
      lds[kF48Bout + i] = p.bias_out ? reinterpret_cast<const f32x4*>(p.bias_out)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float wb = (p.ln == 2) ? 1.f : 0.f;
  const f32x4* wout = reinterpret_cast<const f32x4*>(p.Wout);
  // stencil read offsets (gdfn_out's, for the main wave's first halo row)
  int lo[2][3];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int hx = li + j;
      lo[h][j] = (kF48RPW * hw * kHalo + hx) * 8 + ((4 * h + lq) ^ (hx & 7));
    }
  // pixel tiles of helper hw (and, pt 0..2, of main wave hw): pt 0..2 = halo rows 3hw+1..3hw+3 (the
  // main wave's output rows, interior columns), pt 3 = the top halo row (0), the bottom one (1), the
  // left (2) or right (3) halo column (14 pixels)
  int hy[4], hx[4];
  bool tv[4];
#pragma unroll
  for (int pt = 0; pt < 3; ++pt) {
    hy[pt] = kF48RPW * hw + 1 + pt;
    hx[pt] = li + 1;
    tv[pt] = true;
  }
  hy[3] = hw == 0 ? 0 : hw == 1 ? kF48HR - 1 : li;
  hx[3] = hw <= 1 ? li + 1 : (hw == 2 ? 0 : kHalo - 1);
  tv[3] = hw <= 1 || li < kF48HR;

  int staged = -1;
  for (int t = t_lo + xb; t < t_hi; t += nxb) {
    const int b = t / per_img;
    const int rem = t - b * per_img;
    const int ty = rem / tx_n;
    const int x0 = (rem - ty * tx_n) * kTile, y0 = ty * kF48TH;
    if (b != staged) {  // block-uniform
      __syncthreads();
      const f32x4* mb = reinterpret_cast<const f32x4*>(p.Wm + (long long)b * p.wm_img_stride);
      for (int i = tid; i < 9 * 64; i += 64 * kF48Waves) lds[kF48M + i] = mb[i];
      for (int i = tid; i < 12; i += 64 * kF48Waves)
        lds[kF48Bm + i] = p.bias_m ? reinterpret_cast<const f32x4*>(p.bias_m)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
      __syncthreads();
      staged = b;
    }
    const unsigned vbytes = (unsigned)HW * (unsigned)p.ldv * 4u, xbytes = (unsigned)HW * (unsigned)p.ldx * 4u;
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.v + (long long)b * HW * p.ldv), 0, (int)vbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rxx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.x + (long long)b * HW * p.ldx), 0, (int)xbytes, 0x00020000);
    bool in[4];
    // raw buffer loads: 32-bit offsets, zeros past the range (out-of-image pixels), no branches
    auto load = [&](int pt, f32x4 (&vv)[3], f32x4 (&xx3)[3]) {
      const int yy = y0 - 1 + hy[pt], xx = x0 - 1 + hx[pt];
      in[pt] = tv[pt] && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
      const unsigned px = (unsigned)(yy * p.W + xx);
      const unsigned ov = in[pt] ? px * (unsigned)p.ldv * 4u + 16u * lq : kOOB2;
      const unsigned ox = in[pt] ? px * (unsigned)p.ldx * 4u + 16u * lq : kOOB2;
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        vv[g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rv, (int)(ov + 64u * g), 0, 0));
        xx3[g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rxx, (int)(ox + 64u * g), 0, 0));
      }
    };
    const f32x4* ml = lds + kF48M;
    const f32x4* bm = lds + kF48Bm;
    if (main_w) {
      // ---- main wave: x1 of its output rows (the residual; the helper of the same rows forms the same
      // values for LN), then per chunk the gate and project_out
      // x1 is parked in `out` at the lane's own addresses (the epilogue reads it back: same thread, so
      // program order holds) instead of holding 36 registers across the chunk loop
      const unsigned obytes = (unsigned)HW * (unsigned)p.ldo * 4u;
      const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
          p.out + (long long)b * HW * p.ldo, 0, (int)obytes, 0x00020000);
      unsigned oo[kF48RPW];
#pragma unroll
      for (int r = 0; r < kF48RPW; ++r) {
        const int yo = y0 + kF48RPW * hw + r;
        oo[r] = yo < p.H ? (unsigned)(yo * p.W + x0 + li) * (unsigned)p.ldo * 4u + 16u * lq : kOOB2;
      }
      {
        f32x4 va[3][3], xa[3][3];
#pragma unroll
        for (int pt = 0; pt < 3; ++pt) load(pt, va[pt], xa[pt]);
#pragma unroll
        for (int pt = 0; pt < 3; ++pt) {
          f32x4 x1[3];
          f48_x1(ml, bm, lane, lq, va[pt], xa[pt], x1);
#pragma unroll
          for (int tt = 0; tt < 3; ++tt)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4g, x1[tt]), ro, (int)(oo[pt] + 64u * tt), 0, 0);
        }
      }
      f32x4 acc[kF48RPW][3];
#pragma unroll
      for (int r = 0; r < kF48RPW; ++r)
#pragma unroll
        for (int tt = 0; tt < 3; ++tt) acc[r][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 w[3];
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) w[tt] = wout[(tt * kF48Kch + 0) * 64 + lane];
      lds_barrier();  // chunk 0's halo image
#pragma unroll 1
      for (int c = 0; c < kF48Kch; ++c) {
        f32x4 wn[3];
        if (c + 1 < kF48Kch) {
#pragma unroll
          for (int tt = 0; tt < 3; ++tt) wn[tt] = wout[(tt * kF48Kch + c + 1) * 64 + lane];
        }
        f32x4 gb[kF48RPW];
        gate_rows<kF48RPW, kGeluPacked>(lds + kF48Hb + (c & 1) * kF48Px * 8, lds + kF48Dw + c * kDwF4, lo, lq, gb);
#pragma unroll
        for (int tt = 0; tt < 3; ++tt)
#pragma unroll
          for (int r = 0; r < kF48RPW; ++r) {
            acc[r][tt] = mfma4(w[tt].x, gb[r].x, acc[r][tt]);
            acc[r][tt] = mfma4(w[tt].y, gb[r].y, acc[r][tt]);
            acc[r][tt] = mfma4(w[tt].z, gb[r].z, acc[r][tt]);
            acc[r][tt] = mfma4(w[tt].w, gb[r].w, acc[r][tt]);
          }
        if (c + 1 < kF48Kch) {
#pragma unroll
          for (int tt = 0; tt < 3; ++tt) w[tt] = wn[tt];
        }
        lds_barrier();  // chunk c's image read; chunk c+1's written
      }
      // ---- epilogue: out = acc + x1 + bias (gdfn_out's order); rows past the image dropped
#pragma unroll
      for (int r = 0; r < kF48RPW; ++r) {
        f32x4 x1v[3];
#pragma unroll
        for (int tt = 0; tt < 3; ++tt)
          x1v[tt] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ro, (int)(oo[r] + 64u * tt), 0, 0));
#pragma unroll
        for (int tt = 0; tt < 3; ++tt)
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(u32x4g, acc[r][tt] + x1v[tt] + lds[kF48Bout + 4 * tt + lq]), ro, (int)(oo[r] + 64u * tt), 0,
              0);
      }
    } else {
      // ---- helper wave: x1 and LN(x1) of its 4 halo pixel tiles, then project_in chunk by chunk into
      // the double-buffered halo image (chunk c+1 is written while the main waves gate chunk c)
      f32x4 xn[4][3];
      {
        f32x4 va[2][3], xa[2][3];
        load(0, va[0], xa[0]);
#pragma unroll
        for (int pt = 0; pt < 4; ++pt) {
          const int cb = pt & 1;
          if (pt + 1 < 4) load(pt + 1, va[cb ^ 1], xa[cb ^ 1]);
          f32x4 a[3];
          f48_x1(ml, bm, lane, lq, va[cb], xa[cb], a);
          // LayerNorm over the 48 channels (gemm.hip apply_ln, row in registers)
          float sm = 0.f;
#pragma unroll
          for (int g = 0; g < 3; ++g) sm += (a[g].x + a[g].y) + (a[g].z + a[g].w);
          sm += __shfl_xor(sm, 16);
          sm += __shfl_xor(sm, 32);
          const float mean = sm / 48.0f;
          float v2 = 0.f;
#pragma unroll
          for (int g = 0; g < 3; ++g) {
            const f32x4 d = a[g] - mean;
            const float dd = (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
            v2 += dd;
          }
          v2 += __shfl_xor(v2, 16);
          v2 += __shfl_xor(v2, 32);
          const float rstd = 1.0f / sqrtf(v2 / 48.0f + 1e-5f);
          const float sh = mean * wb;
#pragma unroll
          for (int g = 0; g < 3; ++g) xn[pt][g] = (a[g] - sh) * rstd;
        }
      }
      // project_in of chunk c (tiles 2c, 2c+1) + bias -> halo image buffer c & 1 (out-of-image pixels 0)
      auto project_in = [&](int c) {
        f32x4 o[4][2];
#pragma unroll
        for (int pt = 0; pt < 4; ++pt)
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) o[pt][hh] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          const f32x4 w0 = lds[kF48Win + ((2 * c) * 3 + g) * 64 + lane];
          const f32x4 w1 = lds[kF48Win + ((2 * c + 1) * 3 + g) * 64 + lane];
#pragma unroll
          for (int ss = 0; ss < 4; ++ss)
#pragma unroll
            for (int pt = 0; pt < 4; ++pt) {
              o[pt][0] = mfma4(w0[ss], xn[pt][g][ss], o[pt][0]);
              o[pt][1] = mfma4(w1[ss], xn[pt][g][ss], o[pt][1]);
            }
        }
        f32x4* hb = lds + kF48Hb + (c & 1) * kF48Px * 8;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const f32x4 bias = lds[kF48Bin + 4 * (2 * c + hh) + lq];
#pragma unroll
          for (int pt = 0; pt < 4; ++pt) {
            const f32x4 v = o[pt][hh] + bias;
            if (tv[pt]) hb[(hy[pt] * kHalo + hx[pt]) * 8 + ((4 * hh + lq) ^ (hx[pt] & 7))] = in[pt] ? v : f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
      };
      project_in(0);
      lds_barrier();  // chunk 0's halo image
#pragma unroll 1
      for (int c = 0; c < kF48Kch; ++c) {
        if (c + 1 < kF48Kch) project_in(c + 1);
        lds_barrier();
      }
    }
  }
}

bool ffn48_supported(int C, int hidS, int W) { return C == 48 && hidS == 16 * kF48Kch && W % kTile == 0; }

hipError_t launch_ffn48(const Ffn48Params& p, hipStream_t s) {
  if (p.W % kTile || p.ldv % 4 || p.ldx % 4 || p.ldo % 4 || p.Bn <= 0 || p.H <= 0) return hipErrorInvalidValue;
  static bool attr[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!attr[dev]) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&ffn48_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kF48Lds);
    if (e != hipSuccess) return e;
    attr[dev] = true;
  }
  const long long tiles = (long long)p.Bn * ((p.H + kF48TH - 1) / kF48TH) * (p.W / kTile);
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  long long grid = std::min<long long>(tiles, cus);  // one resident block per CU
  grid = (grid + 7) / 8 * 8;
  hipLaunchKernelGGL(ffn48_kernel, dim3((unsigned)grid), dim3(64 * kF48Waves), kF48Lds, s, p);
  return hipGetLastError();
}


}  // namespace kdlae
