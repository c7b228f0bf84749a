// Fused GDFN tail (KDLAE/KDLAE_model.py:101-106):
//   out = x_res + project_out( gelu_erf(dw3x3(x1)) * dw3x3(x2) )
// in ONE pass over the project_in output.  The gated hidden tensor (hid channels per pixel) never
// reaches HBM: it is produced in registers in exactly the layout the MFMA B operand wants.
//
// Input layout (written by the project_in GEMM): per pixel 2*hidS floats, chunk-interleaved —
// chunk g (16 hidden channels) occupies floats [32g, 32g+16) for x1 and [32g+16, 32g+32) for x2,
// so one chunk of one pixel is a contiguous 128 B line.
//
// Block = 256 threads (4 waves, two workgroups per CU) on a 16 x TH pixel tile; wave w owns tile
// rows RPW w .. RPW w + RPW - 1, lane l owns pixel column l & 15 and channel quad l >> 4.  Per hidden
// chunk g (16 channels of x1 and the same 16 of x2):
//   * LDS-DMA (buffer_load ... lds, no VGPRs) brings the chunk's (TH+2) x 18 halo tile (one 128 B line
//     per pixel) and its depthwise weights + bias (2 KiB, repacked per chunk on the host) into a
//     2-slot stage ring; iteration g issues chunk g+2, so chunk g+1 lands while g is gated.  Nothing
//     else in the loop reads global memory (an ordinary load would make hipcc drain the DMAs);
//   * the halo image is lane-linear [pixel][slot] with slot = quad ^ (column & 7) applied on the
//     SOURCE address, so the column reads of the stencil are bank-conflict-free;
//   * each lane computes the depthwise 3x3 + exact-erf gate for its RPW pixels and 4 channels — a
//     float4 per pixel which, with the next chunk's, IS its split-MFMA B operand (mfma3.h: chunks 2G
//     and 2G+1 form pair G, channels 32G + 4q + j / 32G + 16 + 4q + j - 4 — the pout GEMM's order);
//   * project_out runs once per chunk pair on the bf16 matrix cores (mfma6), its split weight records
//     (NT x 3 KiB for the block's NT output tiles) DMA'd into a one-pair W slot during the even chunk.
// Epilogue: bias + residual, float4 stores of 4 consecutive output channels per lane.
// C = 192 / 384 run C / 96 blocks per pixel tile (adjacent ids: the same XCD, halo from L2), each
// owning 6 output tiles.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include <algorithm>

#include "gate.h"
#include "kernels.h"
#include "mfma3.h"
#include "runtime.h"

namespace kdlae {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

using gdfnc::gate_rows;
using gdfnc::kDwF4;
using gdfnc::kGeluPacked;
using gdfnc::kHalo;
using gdfnc::kTile;

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

typedef unsigned u32x4g __attribute__((ext_vector_type(4)));
constexpr unsigned kOOB2 = 0x80000000u;  // a byte offset past every descriptor's range

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

template <int NT, int TH>
__global__ __launch_bounds__(256, 2) void gdfn_out_kernel(GdfnParams p) {
  constexpr int WAVES = 4;
  using T = GdTile<TH>;
  constexpr int kStageItems = T::kStageItems, kStagePieces = T::kStagePieces;
  constexpr int kStageF4 = T::kStageF4, kStageSlot = T::kStageSlot;
  constexpr int RPW = TH / WAVES;                              // tile rows per wave
  static_assert(RPW * WAVES == TH, "tile rows per wave");
  constexpr int kRounds = (kStagePieces + WAVES - 1) / WAVES;  // stage pieces per wave (max)
  extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
  f32x4* wslot = lds + 2 * kStageSlot;  // [NT][kRec3]: the current pair's split W records
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: per-wave branches and LDS bases stay in SGPRs
  const int cx = lane & 15, q = lane >> 4;
  const int kch = p.hidS >> 4;
  const int kpt = (kch + 1) / 2;  // W pairs of the layer (split arena layout [C/16 tiles][kpt][kRec3])

  // XCD-aware tile order: logical tiles [k*per, (k+1)*per) run on XCD k, so tiles that share halo
  // rows/columns share an L2.  The grid is padded to a multiple of 8.  With nsplit > 1 the nsplit
  // blocks of one pixel tile (adjacent logical ids: same XCD, so the others read the halo from L2)
  // each own NT of the layer's output tiles.
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
  // this block's NT output tiles: records (sp NT + t, G) of the split arena
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.Wp + (size_t)sp * NT * kpt * kRec3 * 4), 0, NT * kpt * kRec3 * 16, 0x00020000);
  const int n0 = 16 * NT * sp;  // first output channel of this block
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.dw), 0, kch * kDwF4 * 16, 0x00020000);
  auto issue = [&](int g) {
    f32x4* sl = lds + (g & 1) * kStageSlot;
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
  };
  // the split records of pair G (3 NT pieces of 1 KiB, dealt over the waves)
  auto issue_w = [&](int G) {
#pragma unroll
    for (int k = 0; k < 3 * NT; ++k)
      if (k % WAVES == wave) {
        const int t = k / 3, pl = k - 3 * t;
        dma_buf(rw, wslot + 64 * k, 16u * lane, ((t * kpt + G) * 3 + pl) * 1024);
      }
  };
  // every outstanding DMA of this wave landed, then a raw barrier: past it all waves' DMAs are
  // visible and every wave is done with what it read before (a __syncthreads() is the same here)
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
  auto gate = [&](int g, f32x4 (&gb)[RPW]) {
    const f32x4* sl = lds + (g & 1) * kStageSlot;
    gate_rows<RPW, kGeluPacked>(sl, sl + kStageF4, lo, q, gb);  // [9][8] then bias [8]
  };
  // project_out of one chunk pair: B = split3(gate of chunk 2G, gate of chunk 2G+1)
  auto mfma_pair = [&](const f32x4 (&ga)[RPW], const f32x4 (&gc)[RPW]) {
    F3 xs[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) xs[r] = split3(ga[r], gc[r]);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const F3 w = load_w3(wslot + t * kRec3, lane);
#pragma unroll
      for (int r = 0; r < RPW; ++r) acc[r][t] = mfma6(w, xs[r], acc[r][t]);
    }
  };

  // prologue: S0, W0, S1 in flight; gate(0) once everything has landed
  issue(0);
  issue_w(0);
  if (kch > 1) issue(1);
  wait_all();
  f32x4 gb[RPW], gbp[RPW];
  gate(0, gb);
  // two chunks per iteration.  Step A (even chunk g): gate(g + 1), W of pair g / 2 issued.  Step B:
  // gate(g + 2) and the pair's MFMAs in one basic block, so the matrix and vector work interleave.
  // Each step starts with every wave's DMAs landed and a barrier, past which every wave is done with
  // the stage slot the step refills and (step A) with the previous pair's W slot.
  for (int g = 0; g + 1 < kch; g += 2) {
    wait_all();
    if (g + 2 < kch) issue(g + 2);
    if (g > 0) issue_w(g >> 1);
    {
      f32x4 gbn[RPW];
      gate(g + 1, gbn);
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        gbp[r] = gb[r];
        gb[r] = gbn[r];
      }
    }
    if (g + 2 >= kch) break;  // even kch: the last pair's MFMAs follow the loop
    wait_all();
    if (g + 3 < kch) issue(g + 3);
    f32x4 gbn[RPW];
    gate(g + 2, gbn);
    mfma_pair(gbp, gb);  // chunks g, g + 1
#pragma unroll
    for (int r = 0; r < RPW; ++r) gb[r] = gbn[r];
  }
  if (kch & 1) {  // the last chunk pairs with zeros
    if (kch > 1) {
      wait_all();  // every wave past the previous pair's MFMAs
      issue_w(kch >> 1);
    }
    wait_all();
    f32x4 z[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) z[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    mfma_pair(gb, z);
  } else {
    wait_all();  // W of the last pair
    mfma_pair(gbp, gb);
  }

  // epilogue: lane holds output channels 16t + 4q .. +3 of pixel (y0 + RPW w + r, x0 + cx)
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

template <int NT, int TH>
static hipError_t launch_gdfn1(const GdfnParams& p, hipStream_t s) {
  const size_t lds = (size_t)(2 * GdTile<TH>::kStageSlot + NT * kRec3) * sizeof(f32x4);
  if (lds > 80 * 1024) return hipErrorInvalidValue;  // two blocks per CU
  static size_t attr[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (lds > 64 * 1024 && lds > attr[dev]) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gdfn_out_kernel<NT, TH>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr[dev] = lds;
  }
  const long long tiles = (long long)p.Bn * ((p.H + TH - 1) / TH) * ((p.W + kTile - 1) / kTile) *
                          (p.nsplit > 1 ? p.nsplit : 1);
  const long long grid = (tiles + 7) / 8 * 8;
  hipLaunchKernelGGL((gdfn_out_kernel<NT, TH>), dim3((unsigned)grid), dim3(256), lds, s, p);
  return hipGetLastError();
}

// Tile shapes (r05, split MFMAs): the stage ring is 2 x (halo + dw block), the W slot NT x 3 KiB; both
// must fit 80 KiB for two blocks per CU.  C = 48: 16 x 12 tiles (2 x 34 + 9 KiB); C >= 96: 16 x 8 tiles
// with 6 output tiles per block (2 x 25 + 18 KiB), C / 96 blocks per pixel tile.
hipError_t launch_gdfn_out(const GdfnParams& p, int C, hipStream_t s) {
  if (!gdfn_supported(C, p.hidS) || p.ld != 2 * p.hidS || p.ldo % 4 || (p.R && p.ldr % 4) || !p.zeros)
    return hipErrorInvalidValue;
  GdfnParams q = p;
  if (C == 48) {
    q.nsplit = 1;
    return launch_gdfn1<3, 12>(q, s);
  }
  q.nsplit = C / 96;
  return launch_gdfn1<6, 8>(q, s);
}

}  // namespace kdlae
