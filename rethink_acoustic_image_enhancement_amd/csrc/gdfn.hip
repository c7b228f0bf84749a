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
    const f32x4* dw = sl + kStageF4;               // [9][8] then bias [8]
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
      }
    }
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      if constexpr (kGeluPacked && NT <= 6) {
        const f32x2 lo = gelu_gate2(f32x2{d[0][r].x, d[0][r].y}, f32x2{d[1][r].x, d[1][r].y});
        const f32x2 hi = gelu_gate2(f32x2{d[0][r].z, d[0][r].w}, f32x2{d[1][r].z, d[1][r].w});
        gb[r] = f32x4{lo.x, lo.y, hi.x, hi.y};
      } else {
        gb[r].x = gelu_erf_g(d[0][r].x) * d[1][r].x;
        gb[r].y = gelu_erf_g(d[0][r].y) * d[1][r].y;
        gb[r].z = gelu_erf_g(d[0][r].z) * d[1][r].z;
        gb[r].w = gelu_erf_g(d[0][r].w) * d[1][r].w;
      }
    }
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


// ---------------------------------------------------------------------------------------------
// r02 schedule ("gdfn2"): no LDS halo, no per-chunk barrier.  A persistent grid of one 4-wave
// block per CU; after one barrier that stages every chunk's project_out W fragments and dw block
// in LDS (C = 96: 96 + 20 KiB), each WAVE runs on its own: it owns strips of 16 columns x R rows and,
// per hidden chunk g, walks the strip's R + 2 input rows top to bottom:
//   * the three column-shifted 16-pixel rows of x1 and x2 (6 buffer loads, 16 B per lane; rows and
//     columns outside the image fall outside the descriptor and load zeros = the conv's padding)
//     are prefetched two input rows ahead, straight into VGPRs (the shifted loads hit the L1/L2
//     lines of the centre load, so HBM sees each 128 B pixel line about once);
//   * input row k adds its 3 x 3 taps into the running depthwise sums of output rows k-2..k;
//   * output row r is complete after input row r+2, gated at r+3 and multiplied (24 MFMAs for
//     C = 96) at r+4, so the stencil VALU of one row, the gate of the row before and the MFMAs of
//     the row before that are independent instruction streams the scheduler interleaves.  The
//     last two rows' gate/MFMA are carried into the next chunk's first two input rows.
// One wave per SIMD with up to 512 VGPRs: the accumulators of the strip (R x C/16 float4), the
// three prefetched rows and the chunk's dw weights stay in registers.  r01's kernel spent about a
// third of its wave cycles parked on the per-chunk barrier / DMA waits (profiles/r02_pmc_*).
// DPP lane shift of one float.  The empty asm keeps each component a separate scalar: hipcc
// (ROCm 7.2, -O3) otherwise merges the four update_dpp calls of a float4 into ONE v_mov_b32_dpp of
// the x component and copies it into y, z and w (wrong results; seen in the ISA of gdfn2 and of a
// 10-line reproducer, tools/micro/dpp_probe.hip documents the lane mapping).
template <int CTRL>
__device__ __forceinline__ float dpp1(float old, float v) {
  int o = __builtin_bit_cast(int, old), x = __builtin_bit_cast(int, v);
  asm("" : "+v"(x));
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(o, x, CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ f32x4 dpp4(const f32x4& old, const f32x4& v) {
  return f32x4{dpp1<CTRL>(old.x, v.x), dpp1<CTRL>(old.y, v.y), dpp1<CTRL>(old.z, v.z), dpp1<CTRL>(old.w, v.w)};
}

template <int NT, int R, int WPS>
__global__ __launch_bounds__(256 * WPS) __attribute__((amdgpu_waves_per_eu(WPS, WPS)))
void gdfn2_kernel(GdfnParams p, int nunits) {
  constexpr int K = R + 2;             // input rows per strip and chunk
  constexpr int PD = WPS == 1 ? 2 : 1;  // rows prefetched ahead (the second wave of a SIMD hides more)
  constexpr int NS = PD + 1;           // row slots
  static_assert(K % NS == 0, "the prefetch slots must line up at chunk boundaries");
  // one wave per SIMD (512 VGPRs): the chunk's dw taps stay in registers; two waves per SIMD
  // (256 VGPRs): they are re-read from LDS where they are used.  W fragments: always from LDS.
  constexpr bool kWRegs = WPS == 1;
  constexpr int WAVES = 4 * WPS;
  extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
  const int kch = p.hidS >> 4;
  f32x4* wl = lds;                          // [kch][NT][64] project_out fragments, chunk-major
  f32x4* dl = lds + kch * NT * 64;          // [kch][80]     dw taps [9][8] + bias [8]
  {
    const f32x4* Wf = reinterpret_cast<const f32x4*>(p.Wp);  // [NT][kch][64]
    const f32x4* Dw = reinterpret_cast<const f32x4*>(p.dw);  // [kch][128]
    for (int i = threadIdx.x; i < kch * NT * 64; i += 64 * WAVES) {
      const int g = i / (NT * 64), rem = i - g * (NT * 64);
      wl[i] = Wf[((size_t)(rem >> 6) * kch + g) * 64 + (rem & 63)];
    }
    for (int i = threadIdx.x; i < kch * 80; i += 64 * WAVES) {
      const int g = i / 80;
      dl[i] = Dw[(size_t)g * 128 + (i - g * 80)];
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int sx_n = (p.W + 15) >> 4, sy_n = (p.H + R - 1) / R;
  // XCD-aware split: XCD k (blocks k, k+8, ...) takes a contiguous range of strips, so the strips
  // whose halos overlap run at the same time under one L2
  const int per_xcd = (nunits + 7) >> 3;
  const int u_begin = (int)(blockIdx.x & 7) * per_xcd;
  const int u_end = min(u_begin + per_xcd, nunits);
  const int wstride = (int)(gridDim.x >> 3) * WAVES;
  const unsigned row_bytes = (unsigned)p.W * (unsigned)p.ld * 4u;
  const unsigned img_bytes = (unsigned)p.H * row_bytes;
  constexpr unsigned kFar = 0x40000000u;  // row or column offset outside the image (img_bytes <= 2^30)

  for (int u = u_begin + (int)(blockIdx.x >> 3) * WAVES + wave; u < u_end; u += wstride) {
    const int sc = u % sx_n, t2 = u / sx_n;
    const int sr = t2 % sy_n, b = t2 / sy_n;
    const int x0 = sc * 16, y0 = sr * R;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.x + (long long)b * p.H * p.W * p.ld), 0, (int)img_bytes, 0x00020000);
    // centre column (lane li <-> column x0+li) and the two edge columns (lane 0 <-> x0-1,
    // lane 15 <-> x0+16; the other lanes' edge offsets fall outside the descriptor)
    const int xc = x0 + li, xe = li == 0 ? x0 - 1 : (li == 15 ? x0 + 16 : -1);
    const unsigned ccoff = ((unsigned)xc < (unsigned)p.W ? (unsigned)xc * (unsigned)p.ld * 4u : kFar) + 16u * lq;
    const unsigned ecoff = ((unsigned)xe < (unsigned)p.W ? (unsigned)xe * (unsigned)p.ld * 4u : kFar) + 16u * lq;
    // input row k (0..K-1 <-> image row y0-1+k) of chunk g: x1 (h=0) and x2 (h=1), centre and edge
    auto load_row = [&](int g, int k, f32x4 (&dst)[2][2]) {
      const int yy = y0 - 1 + k;
      const unsigned so = ((unsigned)yy < (unsigned)p.H ? (unsigned)yy * row_bytes : kFar) + 128u * (unsigned)g;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        dst[h][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(ccoff + so + 64u * h), 0, 0));
        dst[h][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(ecoff + so + 64u * h), 0, 0));
      }
    };
    f32x4 acc[R][NT];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 xs[NS][2][2];
#pragma unroll
    for (int k = 0; k < PD; ++k) load_row(0, k, xs[k]);
    // carried from the previous chunk: the depthwise sums of row R-1 (not yet gated) and the gated
    // row R-2 (not yet multiplied); zeros before chunk 0, so the carried MFMAs add nothing
    f32x4 dpend[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    f32x4 gpend = f32x4{0.f, 0.f, 0.f, 0.f};
    auto gate4 = [](const f32x4& a, const f32x4& v) {
      return f32x4{gelu_erf_g(a.x) * v.x, gelu_erf_g(a.y) * v.y, gelu_erf_g(a.z) * v.z, gelu_erf_g(a.w) * v.w};
    };
    auto mfma_row = [&](const f32x4 (&wf)[NT], const f32x4& gb, f32x4 (&ac)[NT]) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int t = 0; t < NT; ++t) ac[t] = mfma4(wf[t][e], gb[e], ac[t]);
    };
    for (int g = 0; g < kch; ++g) {
      const f32x4* dwl = dl + g * 80;
      const int gp = g > 0 ? g - 1 : 0;
      [[maybe_unused]] f32x4 wdw[9][2];
      if constexpr (kWRegs) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int tap = 0; tap < 9; ++tap) wdw[tap][h] = dwl[tap * 8 + 4 * h + lq];
      }
      // tap (row i, column c) of x_h, from registers or (opaque pointer: no hoisting) from LDS
      auto tapw = [&](const f32x4* dwk, int i, int c, int h) -> f32x4 {
        if constexpr (kWRegs) return wdw[3 * i + c][h];
        else return dwk[(3 * i + c) * 8 + 4 * h + lq];
      };
      auto mfma_lds = [&](auto prev, const f32x4& gbv, f32x4 (&ac)[NT]) {
        constexpr bool kPrev = decltype(prev)::value;
        const f32x4* wk = wl + (kPrev ? gp : g) * NT * 64 + lane;
        asm("" : "+v"(wk));  // W fragments are read where used (not hoisted into 24 live VGPRs)
        f32x4 w[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) w[t] = wk[64 * t];
        mfma_row(w, gbv, ac);
      };
      f32x4 d[R][2];      // depthwise sums per output row (only a window of 3 is live)
      f32x4 gb[R];        // gated rows
      f32x4 gq;           // gated carried row R-1
#pragma unroll
      for (int k = 0; k < K; ++k) {
        // prefetch input row k+PD (of this chunk, or the first rows of the next; the last chunk re-reads)
        if (k + PD < K) load_row(g, k + PD, xs[(k + PD) % NS]);
        else load_row(g + 1 < kch ? g + 1 : g, k + PD - K, xs[(k + PD) % NS]);
        const f32x4* dwk = dwl;
        if constexpr (!kWRegs) asm("" : "+v"(dwk));
        const f32x4 bdw[2] = {dwk[72 + lq], dwk[76 + lq]};
        // column neighbours by DPP within each 16-lane row (= one channel quad): row_shr:1 gives
        // lane i the value of lane i-1, lane 0 keeps the edge load (column x0-1); row_shl:1 alike
        f32x4 v[2][3];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          v[h][1] = xs[k % NS][h][0];
          v[h][0] = dpp4<0x111>(xs[k % NS][h][1], v[h][1]);
          v[h][2] = dpp4<0x101>(xs[k % NS][h][1], v[h][1]);
        }
        // stencil: input row k -> output rows k - i (tap row i)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int r = k - i;
          if (r < 0 || r >= R) continue;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            f32x4 s = (i == 0) ? bdw[h] : d[r][h];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              const f32x4 w = tapw(dwk, i, c, h);
              s.x = fmaf(v[h][c].x, w.x, s.x);
              s.y = fmaf(v[h][c].y, w.y, s.y);
              s.z = fmaf(v[h][c].z, w.z, s.z);
              s.w = fmaf(v[h][c].w, w.w, s.w);
            }
            d[r][h] = s;
          }
        }
        // the previous chunk's last rows
        if (k == 0) {
          gq = gate4(dpend[0], dpend[1]);
          mfma_lds(std::true_type{}, gpend, acc[R - 2]);
        }
        if (k == 1) mfma_lds(std::true_type{}, gq, acc[R - 1]);
        // this chunk: gate row k-3, multiply row k-4
        if (k - 3 >= 0 && k - 3 < R) gb[k - 3] = gate4(d[k - 3][0], d[k - 3][1]);
        if (k - 4 >= 0 && k - 4 < R) mfma_lds(std::false_type{}, gb[k - 4], acc[k - 4]);
      }
      dpend[0] = d[R - 1][0];
      dpend[1] = d[R - 1][1];
      gpend = gb[R - 2];
    }
    {  // drain the last chunk's carried rows
      const int gl = kch - 1;
      f32x4 wf[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) wf[t] = wl[(gl * NT + t) * 64 + lane];
      const f32x4 gq = gate4(dpend[0], dpend[1]);
      mfma_row(wf, gpend, acc[R - 2]);
      mfma_row(wf, gq, acc[R - 1]);
    }
    // epilogue: every residual (and the bias) loaded before the first store (vmcnt retires in order)
    const int xo = x0 + li;
    const unsigned o_bytes = (unsigned)p.H * (unsigned)p.W * (unsigned)p.ldo * 4u;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        p.out + (long long)b * p.H * p.W * p.ldo, 0, (int)o_bytes, 0x00020000);
    f32x4 bias[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
      bias[t] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + 16 * t + 4 * lq) : f32x4{0.f, 0.f, 0.f, 0.f};
    if (p.R) {
      const unsigned r_bytes = (unsigned)p.H * (unsigned)p.W * (unsigned)p.ldr * 4u;
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(p.R + (long long)b * p.H * p.W * p.ldr), 0, (int)r_bytes, 0x00020000);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int yo = y0 + r;
        const unsigned off = (yo < p.H && xo < p.W) ? ((unsigned)(yo * p.W + xo) * (unsigned)p.ldr + 4u * lq) * 4u : kOOB2;
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[r][t] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, (int)(off + 64u * t), 0, 0));
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int yo = y0 + r;
      const unsigned off = (yo < p.H && xo < p.W) ? ((unsigned)(yo * p.W + xo) * (unsigned)p.ldo + 4u * lq) * 4u : kOOB2;
#pragma unroll
      for (int t = 0; t < NT; ++t)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4g, acc[r][t] + bias[t]), ro, (int)(off + 64u * t), 0, 0);
    }
  }
}

bool gdfn_supported(int C, int hidS) {
  // A/B hooks: C = 192 / 384 back on dwconv_gate + the project_out GEMM
  if (C == 192 && getenv("KDLAE_NO_GDFN192")) return false;
  if (C == 384 && getenv("KDLAE_NO_GDFN384")) return false;
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

template <int NT, int R, int WPS>
static hipError_t launch_gdfn2(const GdfnParams& p, hipStream_t s) {
  static size_t attr[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  const int kch = p.hidS / 16;
  const size_t lds = (size_t)kch * (NT * 64 + 80) * sizeof(f32x4);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > attr[dev]) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gdfn2_kernel<NT, R, WPS>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr[dev] = lds;
  }
  const long long units = (long long)p.Bn * ((p.H + R - 1) / R) * ((p.W + 15) / 16);
  if (units >= (1LL << 31)) return hipErrorInvalidValue;
  const int grid = std::max(8, device_cu_count() / 8 * 8);  // persistent: one block per CU
  hipLaunchKernelGGL((gdfn2_kernel<NT, R, WPS>), dim3((unsigned)grid), dim3(256 * WPS), lds, s, p, (int)units);
  return hipGetLastError();
}

// gdfn2 needs each image's x (and out / residual) under 2^30 bytes (offset sentinels) and W/dw in LDS
static bool gdfn2_ok(const GdfnParams& p, int C) {
  const long long hw = (long long)p.H * p.W;
  static const bool on = getenv("KDLAE_GDFN2") != nullptr;  // opt-in until it beats r01's kernel
  return on && hw * p.ld * 4 <= (1LL << 30) && hw * p.ldo * 4 < (1LL << 31) &&
         (!p.R || hw * p.ldr * 4 < (1LL << 31)) && (size_t)(p.hidS / 16) * ((C / 16) * 64 + 80) * 16 <= 160 * 1024;
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
  if (gdfn2_ok(p, C)) {
    static const int rows = getenv("KDLAE_GDFN2_ROWS") ? atoi(getenv("KDLAE_GDFN2_ROWS")) : 10;
    if (C == 96) return launch_gdfn2<6, 4, 1>(p, s);  // R = 7 spills at NT = 6
    return rows == 4 ? launch_gdfn2<3, 4, 1>(p, s) : rows == 7 ? launch_gdfn2<3, 7, 1>(p, s) : launch_gdfn2<3, 10, 1>(p, s);
  }
  // r01 schedule.  KDLAE_GDFN_TILE picks the tile height / stage ring / waves:
  //   0: 16 rows, 3 stage slots, 8 waves (one block per CU, 156 KB of LDS; r01's configuration);
  //   1 (default): 12 rows, 2 slots, 4 waves (C = 96 with the 2-slot W ring: 80 KB; C = 48: 77 KB),
  //      two independent blocks per CU;
  //   2: 4 rows, 2 slots, 4 waves (three blocks per CU);  3: 8 rows, 2 slots, 2 waves.
  static const int tile = getenv("KDLAE_GDFN_TILE") ? atoi(getenv("KDLAE_GDFN_TILE")) : 1;
  if (C == 96) {
    if (tile == 0) return launch_gdfn1<6, 8, 16, 3>(p, s);
    if (tile == 2) return launch_gdfn1<6, 4, 4, 2>(p, s);
    if (tile == 3) return launch_gdfn1<6, 2, 8, 2>(p, s);
    // 8: r02's first two-block layout, 16 x 8 tiles with the 3-slot W ring
    if (tile == 8) return launch_gdfn1<6, 4, 8, 2>(p, s);
    // default: 16 x 12 tiles with the W ring 2 slots deep (exactly 80 KiB: two blocks per CU):
    // C96@512^2 3.52 -> 3.37 ms, @256^2 0.866 -> 0.848 ms (profiles/r02_gdfn_c96_tile12_probe.txt)
    return launch_gdfn1<6, 4, 12, 2, true>(p, s);
  }
  if (tile == 0) return launch_gdfn1<3, 8, 16, 3>(p, s);
  if (tile == 2) return launch_gdfn1<3, 4, 4, 2>(p, s);
  if (tile == 3) return launch_gdfn1<3, 2, 8, 2>(p, s);
  // C = 48 default: 16 x 12 tiles, 3 rows per wave.  77 KB of LDS still fits two blocks per CU (the
  // 3 KiB W records of NT = 3 leave room), and the halo and W/dw refetch per pixel drop by a third:
  // C48@1024^2 5.68 -> 5.42 ms, @512^2 1.46 -> 1.42 ms (profiles/r02_gdfn_c48_tile12_probe.txt).
  // 6: the 16 x 8 tiles of C = 96
  if (tile == 6) return launch_gdfn1<3, 4, 8, 2>(p, s);
  return launch_gdfn1<3, 4, 12, 2>(p, s);
}

}  // namespace kdlae
