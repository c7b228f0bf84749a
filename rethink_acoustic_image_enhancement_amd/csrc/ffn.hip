// Fused feed-forward half of a TransformerBlock (KDLAE/KDLAE_model.py:161, :95-106), C = 48 and 96:
//   y = x1 + project_out( gelu_erf(dw3x3(u1)) * dw3x3(u2) ),   [u1 | u2] = project_in(LN(x1))
// in ONE pass: the 2 hid-wide project_in rows never reach HBM.  Unfused, project_in wrote 2 hidS floats
// per pixel and the GDFN tail read them back with a 3x3 halo (C = 96 at 512^2: ~5 KB per pixel of the
// ~6 KB the FFN half moved).  The price is project_in recomputed on the tile's halo ring (180 pixels per
// 128 outputs), cheap since the split-bf16 MFMAs (mfma3.h) run at 2.67x the f32 MFMA rate.
//
// Block = 8 waves on a 16 x 8 pixel tile, persistent over the tiles of its XCD (one block per CU):
//  * P waves (4-7) own 3 of the halo's 12 pixel tiles of 16 (halo rows 0..9 over the interior
//    columns, then halo columns 0 and 17).  Per tile they load x1, apply the LayerNorm and split the
//    rows into bf16 planes, held in registers for the tile; per hidden chunk g (16 channels of u1 and
//    the same 16 of u2) they run project_in (weights streamed from L2) and write the chunk's halo image
//    (gdfn.hip's layout: lane-linear [pixel][slot], slot = quad ^ (column & 7); zeros outside the
//    image = the dwconv padding) into one of two LDS slots;
//  * G waves (0-3) own 2 output rows each: per chunk the depthwise 3x3 + gate (gate.h) from the halo
//    image, and per chunk pair project_out (split records DMA'd into a 2-slot W ring), then
//    bias + residual x1 and the store.
//  One barrier per chunk: P waves produce chunk g + 1 while G waves consume chunk g.
// Numerics: every value is computed by the same operations as the unfused pair (LN + project_in on
// gemm_res_kernel, then gdfn_out_kernel): the same split records, pair order and mfma6 term order,
// ln_rows, gate_rows and epilogue order, so the output is bit-identical (tests/test_kdlae_gpu.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "gate.h"
#include "kernels.h"
#include "mfma3.h"
#include "rowops.h"
#include "runtime.h"

namespace kdlae {

namespace {

using gdfnc::gate_rows;
using gdfnc::kDwF4;
using gdfnc::kGeluPacked;
using gdfnc::kHalo;
using gdfnc::kTile;

constexpr unsigned kOOBf = 0x80000000u;

typedef unsigned u32x4f __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) void* gptr_f;
typedef __attribute__((address_space(3))) void* lptr_f;

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// every wave issues the same number of DMA pieces, straight-line (piece k = w + 4 j; the padding
// pieces past the chunk's last read nothing and land in a dummy slot): no per-piece branch.  A/B
// (profiles/r05r_ffn_dma_ab.txt): C = 48 -5%, C = 96 +4% (3 more spilled VGPRs), so C = 48 only
template <int C>
constexpr bool uniform_dma() {
  return C == 48;
}

// Tile shape and wave counts.  C = 96's LDS has room for nothing larger than its 16 x 8 tile with
// 4 P + 4 G waves; for C = 48 r05 same-box A/B on C48@1024^2 (profiles/r05zv_ffn48_shape_ab.txt): the
// 16 x 8 tile, 4 + 4 waves 8.09-8.11 ms; a 16 x 12 tile (halo 1.31x instead of 1.41x, 17 spilled
// VGPRs) 8.05 ms; 12 waves (3 per SIMD, 168 VGPRs each) spill 35-130 VGPRs: 4 P + 8 G 10.37 ms,
// 8 P + 4 G 11.65 ms.
template <int C>
struct FfnShape {
  static constexpr int TH = 8;                             // interior rows per tile
  static constexpr int HR = TH + 2;                        // halo rows
  static constexpr int NGW = 4;                            // G waves: TH / NGW output rows each
  static constexpr int RPW = TH / NGW;
  static constexpr int NPT = HR + 2;                       // halo pixel tiles of 16: HR rows, 2 columns
  static constexpr int NP = 4;                             // P waves
  static constexpr int PT = (NPT + NP - 1) / NP;           // halo pixel tiles per P wave
  static constexpr int NW = NP + NGW;
  static constexpr int Img = HR * kHalo * 8;               // f32x4 per halo image slot
  static_assert(TH % NGW == 0 && HR <= 16 && PT * NP >= NPT, "ffn tile shape");
  static constexpr bool kUniformDma = uniform_dma<C>();
  static constexpr int KG = C / 16;          // k-groups of project_in
  static constexpr int KP = (KG + 1) / 2;    // split pairs of project_in
  static constexpr int NTO = C / 16;         // project_out output tiles
  static constexpr int KCH = C == 48 ? 8 : 16;  // max hidden chunks (hidS <= 16 KCH)
  // LDS carve (f32x4): 2 halo image slots, every chunk's dw block, 2 W slots, biases
  static constexpr int kDw = 2 * Img;
  static constexpr int kW = kDw + KCH * kDwF4;
  static constexpr int kBin = kW + 2 * NTO * kRec3;
  static constexpr int kBout = kBin + KCH * 8;
  static constexpr int kWin = kBout + NTO * 4;                 // 2 slots of one chunk's project_in records
  static constexpr int kWinSlot = 2 * KP * kRec3;              // (tiles 2g, 2g + 1) x KP pairs
  static constexpr int kDummy = kWin + 2 * kWinSlot;           // 1 KiB landing slot of padding DMA pieces
  static constexpr int kLds = (kDummy + (kUniformDma ? 64 : 0)) * 16;
  // project_out W pieces (1 KiB) of one pair dealt over the 4 G waves: piece k -> wave k % 4
  static constexpr int pw(int w) { return kUniformDma ? (3 * NTO + NGW - 1) / NGW : (3 * NTO - w + NGW - 1) / NGW; }
  // project_in pieces of one chunk dealt over the NP P waves
  static constexpr int pwin(int w) { return kUniformDma ? (6 * KP + NP - 1) / NP : (6 * KP - w + NP - 1) / NP; }
};

// G wave wi: wait until at most its W pieces of this pair (+ E older ops) are outstanding
template <class S, int E, int W = 0>
__device__ __forceinline__ void wait_w_of(int wi) {
  if constexpr (S::kUniformDma || W + 1 == S::NGW) {
    wait_vm<S::pw(W) + E>();
  } else {
    if (wi == W) {
      wait_vm<S::pw(W) + E>();
      return;
    }
    wait_w_of<S, E, W + 1>(wi);
  }
}

// P wave wi at the last chunk of a tile: at most its W-in pieces of this chunk and the next tile's
// x1 loads outstanding (a compile-time count per wave)
template <class S, int W = 0>
__device__ __forceinline__ void wait_pin_last(int wi) {
  if constexpr (S::kUniformDma || W + 1 == S::NP) {
    wait_vm<S::pwin(W) + S::PT * S::KG>();
  } else {
    if (wi == W) {
      wait_vm<S::pwin(W) + S::PT * S::KG>();
      return;
    }
    wait_pin_last<S, W + 1>(wi);
  }
}

}  // namespace

template <int C>
__global__ __launch_bounds__(64 * FfnShape<C>::NW, FfnShape<C>::NW / 4) void ffn_fused_kernel(FfnParams p) {
  using S = FfnShape<C>;
  constexpr int KG = S::KG, KP = S::KP, NTO = S::NTO;
  constexpr int kTH = S::TH, kHR = S::HR, kRPW = S::RPW, kImg = S::Img, PT = S::PT, NP = S::NP;
  constexpr int NT = 64 * S::NW;
  extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int kch = p.hidS >> 4, npairs = (kch + 1) >> 1;
  const int tx_n = (p.W + kTile - 1) / kTile, ty_n = (p.H + kTH - 1) / kTH;
  const int per_img = tx_n * ty_n, ntiles = p.Bn * per_img;
  // persistent, XCD-aware: XCD k (blockIdx & 7) walks logical tiles [k T / 8, (k+1) T / 8), its blocks
  // interleaved, so tiles that share halo rows run together on one L2
  const int xcd = (int)(blockIdx.x & 7), nxb = (int)(gridDim.x >> 3), xb = (int)(blockIdx.x >> 3);
  const int t_lo = (int)((long long)ntiles * xcd / 8), t_hi = (int)((long long)ntiles * (xcd + 1) / 8);
  if (t_lo + xb >= t_hi) return;  // block-uniform

  // resident: every chunk's dw block, both biases
  for (int i = tid; i < kch * kDwF4; i += NT) lds[S::kDw + i] = reinterpret_cast<const f32x4*>(p.dw)[i];
  for (int i = tid; i < kch * 8; i += NT)
    lds[S::kBin + i] = p.bias_in ? reinterpret_cast<const f32x4*>(p.bias_in)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = tid; i < NTO * 4; i += NT)
    lds[S::kBout + i] = p.bias_out ? reinterpret_cast<const f32x4*>(p.bias_out)[i] : f32x4{0.f, 0.f, 0.f, 0.f};

  const long long HW = (long long)p.H * p.W;
  const bool gw = wave < S::NGW;            // G wave (gate + project_out) or P wave (project_in)
  const int wi = gw ? wave : wave - S::NGW;

  // ---- G-wave state
  // project_out split records [NTO][npairs][kRec3] -> W slot s: pieces k = 3 t + plane
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.Wout), 0, NTO * npairs * kRec3 * 16, 0x00020000);
  auto issue_w = [&](int pair, int slot) {
    f32x4* dst = lds + S::kW + slot * (NTO * kRec3);
    if constexpr (S::kUniformDma) {
#pragma unroll
      for (int j = 0; j < (3 * NTO + S::NGW - 1) / S::NGW; ++j) {
        const int k = wi + S::NGW * j;
        const bool real = k < 3 * NTO;
        const int t = k / 3, pl = k - 3 * t;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lptr_f)(real ? dst + 64 * k : lds + S::kDummy), 16,
                                                 (int)(real ? 16u * lane : kOOBf),
                                                 real ? ((t * npairs + pair) * 3 + pl) * 1024 : 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 3 * NTO; ++k)
        if (k % S::NGW == wi) {
          const int t = k / 3, pl = k - 3 * t;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lptr_f)(dst + 64 * k), 16, (int)(16u * lane),
                                                   ((t * npairs + pair) * 3 + pl) * 1024, 0, 0);
        }
    }
  };
  // wait until at most N VMEM ops of this G wave are outstanding (exact per-wave counts)
  auto wait_w = [&](auto extra) {
    constexpr int E = decltype(extra)::value;
    wait_w_of<S, E>(wi);
  };
  int lo[2][3];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int hx = li + j;
      lo[h][j] = (kRPW * wi * kHalo + hx) * 8 + ((4 * h + lq) ^ (hx & 7));
    }

  // ---- P-wave state: halo pixel tiles PT wi .. PT wi + PT - 1 (rows 0..HR-1 over the interior columns,
  // then columns 0 and 17)
  int phy[PT], phx[PT];
  bool plv[PT];
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    const int pt = PT * wi + k;
    phy[k] = pt < kHR ? pt : li;
    phx[k] = pt < kHR ? li + 1 : (pt == kHR ? 0 : kHalo - 1);
    plv[k] = pt < kHR || (pt < S::NPT && li < kHR);
  }

  // ---- P-wave state: project_in records of chunk g DMA'd into W-in slot g & 1 (issued two chunks
  // ahead; the weights are the same for every tile, so the last chunks of a tile issue the next
  // tile's first); the tile's x1 rows loaded one tile ahead into a
  const __amdgpu_buffer_rsrc_t rwin = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.Win), 0, 2 * kch * KP * kRec3 * 16, 0x00020000);
  auto issue_win = [&](int g) {
    f32x4* dst = lds + S::kWin + (g & 1) * S::kWinSlot;
    if constexpr (S::kUniformDma) {
#pragma unroll
      for (int i = 0; i < (6 * KP + NP - 1) / NP; ++i) {
        const int k = wi + NP * i;  // piece k = (tile j = k / (3 KP), pair G, plane) of records (2g + j, G)
        const bool real = k < 6 * KP;
        const int j = k / (3 * KP), rem = k - j * 3 * KP;
        const int G = rem / 3, pl = rem - 3 * G;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rwin, (lptr_f)(real ? dst + 64 * k : lds + S::kDummy), 16,
                                                 (int)(real ? 16u * lane : kOOBf),
                                                 real ? (((2 * g + j) * KP + G) * 3 + pl) * 1024 : 0, 0, 0);
      }
    } else {
      auto issue_case = [&](auto wtag) {
        constexpr int WI = decltype(wtag)::value;
#pragma unroll
        for (int k = WI; k < 6 * KP; k += NP) {
          const int j = k / (3 * KP), rem = k - j * 3 * KP;
          const int G = rem / 3, pl = rem - 3 * G;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rwin, (lptr_f)(dst + 64 * k), 16, (int)(16u * lane),
                                                   (((2 * g + j) * KP + G) * 3 + pl) * 1024, 0, 0);
        }
      };
      switch (wi) {
        case 0: issue_case(std::integral_constant<int, 0>{}); break;
        case 1: issue_case(std::integral_constant<int, 1>{}); break;
        case 2: issue_case(std::integral_constant<int, 2>{}); break;
        default: issue_case(std::integral_constant<int, 3>{}); break;
      }
    }
  };
  f32x4 a[PT][KG];  // P waves: the x1 rows of the next tile (loaded ahead)
  auto load_x1 = [&](int t) {
    const int b = t / per_img;
    const int rem = t - b * per_img;
    const int ty = rem / tx_n;
    const int x0 = (rem - ty * tx_n) * kTile, y0 = ty * kTH;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.x + (long long)b * HW * p.ldx), 0, (int)(HW * p.ldx * 4), 0x00020000);
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const int yy = y0 - 1 + phy[k], xx = x0 - 1 + phx[k];
      const bool ok = plv[k] && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
      const unsigned off = ok ? (unsigned)((yy * p.W + xx) * p.ldx) * 4u + 16u * lq : kOOBf;
#pragma unroll
      for (int g = 0; g < KG; ++g)
        a[k][g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(off + 64u * g), 0, 0));
    }
  };

  // The P waves at issue priority 1 (s_setprio): the SIMD's arbiter favours the project_in producer
  // over the gate wave it shares the SIMD with.  r05 A/B (profiles/r05p_ffn_prio_ab.txt): C48@1024^2
  // 8.17-8.34 -> 7.83-7.88 ms per launch, C96 unchanged within noise; the G waves raised instead, or
  // P priority only in the tile prologue: smaller gains.
  if (gw) {
    issue_w(0, 0);
    wait_vm<0>();
  } else {
    __builtin_amdgcn_s_setprio(1);
    issue_win(0);
    issue_win(1);
    wait_vm<0>();
    load_x1(t_lo + xb);
  }
  __syncthreads();

  // The two roles run their own tile loops (the same tiles, the same barrier count per tile), so the
  // register allocator sees each role's live state on its own.
  auto tile_geo = [&](int t, int& b, int& x0, int& y0) {
    b = t / per_img;
    const int rem = t - b * per_img;
    const int ty = rem / tx_n;
    x0 = (rem - ty * tx_n) * kTile;
    y0 = ty * kTH;
  };
  if (!gw) {
    for (int t = t_lo + xb; t < t_hi; t += nxb) {
      int b, x0, y0;
      tile_geo(t, b, x0, y0);
      (void)b;
      // ================================================================ P waves: project_in producer
      F3 xs[KP][PT];
      bool in[PT];
#pragma unroll
      for (int k = 0; k < PT; ++k) {
        const int yy = y0 - 1 + phy[k], xx = x0 - 1 + phx[k];
        in[k] = plv[k] && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
      }
      ln_rows<KG, PT>(p.ln, C, KG, a);
#pragma unroll
      for (int k = 0; k < PT; ++k)
#pragma unroll
        for (int G = 0; G < KP; ++G)
          xs[G][k] = split3(a[k][2 * G], 2 * G + 1 < KG ? a[k][2 * G + 1] : f32x4{0.f, 0.f, 0.f, 0.f});
      // project_in of chunk g (output tiles 2g: u1, 2g + 1: u2; records in W-in slot g & 1) -> halo
      // image slot g & 1
      auto pin = [&](int g) {
        const f32x4* wl = lds + S::kWin + (g & 1) * S::kWinSlot + lane;
        f32x4 a1[PT], a2[PT];
#pragma unroll
        for (int k = 0; k < PT; ++k) a1[k] = a2[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        // the W planes one step ahead of their MFMAs (steps = (pair, plane l / m / h): mfma6_pair's
        // term order), fenced so each step's reads issue under the previous step's MFMAs
        bf16x8 w[2][2];
        auto ld = [&](int st, int buf) {
          const int G = st / 3, off = (2 - (st - 3 * G)) * 64;  // planes l, m, h at +128, +64, +0
          w[buf][0] = __builtin_bit_cast(bf16x8, wl[G * kRec3 + off]);
          w[buf][1] = __builtin_bit_cast(bf16x8, wl[(KP + G) * kRec3 + off]);
        };
        ld(0, 0);
#pragma unroll
        for (int st = 0; st < 3 * KP; ++st) {
          if (st + 1 < 3 * KP) ld(st + 1, (st + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);
          const int G = st / 3, pl = st - 3 * G;
          const bf16x8 p0 = w[st & 1][0], p1 = w[st & 1][1];
          if (pl == 2) {
#pragma unroll
            for (int r = 0; r < PT; ++r) {
              a1[r] = mfma_bf(p0, xs[G][r].l, a1[r]);
              a2[r] = mfma_bf(p1, xs[G][r].l, a2[r]);
            }
          }
          if (pl >= 1) {
#pragma unroll
            for (int r = 0; r < PT; ++r) {
              a1[r] = mfma_bf(p0, xs[G][r].m, a1[r]);
              a2[r] = mfma_bf(p1, xs[G][r].m, a2[r]);
            }
          }
#pragma unroll
          for (int r = 0; r < PT; ++r) {
            a1[r] = mfma_bf(p0, xs[G][r].h, a1[r]);
            a2[r] = mfma_bf(p1, xs[G][r].h, a2[r]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        const f32x4 b1 = lds[S::kBin + 4 * (2 * g) + lq], b2 = lds[S::kBin + 4 * (2 * g + 1) + lq];
        f32x4* img = lds + (g & 1) * kImg;
#pragma unroll
        for (int k = 0; k < PT; ++k) {
          if (!plv[k]) continue;
          const int px = phy[k] * kHalo + phx[k], sw = phx[k] & 7;
          img[px * 8 + (lq ^ sw)] = in[k] ? a1[k] + b1 : f32x4{0.f, 0.f, 0.f, 0.f};
          img[px * 8 + ((4 + lq) ^ sw)] = in[k] ? a2[k] + b2 : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      };
      pin(0);
      lds_barrier();  // B_0
      const bool more = t + nxb < t_hi;
      // unrolled by chunk pairs (kch is even) with the last pair peeled: every image / W-in slot index
      // is a compile-time constant, and the loop carries no per-parity copies of the live state
      for (int g = 0; g < kch - 2; g += 2) {
        // chunk g (even): W-in slot 0 was last read by pin(g) (before B_g): chunk g + 2 into it;
        // project_in of chunk g + 1 into image slot 1
        issue_win(g + 2);
        pin(g + 1);
        wait_vm<0>();   // W-in of chunk g + 2 (read by pin(g + 2) in the next chunk)
        lds_barrier();  // B_{g+1}
        // chunk g + 1 (odd): chunk g + 3 into W-in slot 1; project_in of chunk g + 2 into image slot 0
        issue_win(g + 3);
        pin(g + 2);
        wait_vm<0>();
        lds_barrier();  // B_{g+2}
      }
      // the last pair: the next tile's chunks 0 and 1 into the W-in slots
      issue_win(0);
      pin(kch - 1);
      wait_vm<0>();
      lds_barrier();  // B_{kch-1}
      issue_win(1);
      if (more) load_x1(t + nxb);  // the next tile's rows, during this chunk and the G epilogue
      // past B_kch pin(0) of the next tile reads W-in slot 0 (issued at chunk kch - 2): at most this
      // chunk's W-in pieces and the x1 loads may still be outstanding
      wait_pin_last<S>(wi);
      lds_barrier();  // B_kch
    }
  } else {
    int pc = 0;  // pairs consumed by this block (W slot = pc & 1)
    for (int t = t_lo + xb; t < t_hi; t += nxb) {
      int b, x0, y0;
      tile_geo(t, b, x0, y0);
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(p.x + (long long)b * HW * p.ldx), 0, (int)(HW * p.ldx * 4), 0x00020000);
      // ================================================================ G waves: gate + project_out
      f32x4 acc[kRPW][NTO];
#pragma unroll
      for (int r = 0; r < kRPW; ++r)
#pragma unroll
        for (int q = 0; q < NTO; ++q) acc[r][q] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto mfma_pair = [&](const f32x4 (&ga)[kRPW], const f32x4 (&gc)[kRPW], int slot) {
        F3 xsg[kRPW];
#pragma unroll
        for (int r = 0; r < kRPW; ++r) xsg[r] = split3(ga[r], gc[r]);
        const f32x4* wl = lds + S::kW + slot * (NTO * kRec3);
#pragma unroll
        for (int q = 0; q < NTO; ++q) {
          const F3 w = load_w3(wl + q * kRec3, lane);
#pragma unroll
          for (int r = 0; r < kRPW; ++r) acc[r][q] = mfma6(w, xsg[r], acc[r][q]);
        }
      };
      f32x4 gbp[kRPW];
      lds_barrier();  // B_0: chunk 0's image
      // unrolled by chunk pairs (kch is even): chunk g reads image slot 0, chunk g + 1 slot 1, and the
      // accumulators stay in one register set (a parity branch made hipcc copy them every chunk)
      for (int g = 0; g < kch; g += 2) {
        // chunk g: the W of pair g / 2 + 1 (or of the next tile's pair 0) into the other W slot; its
        // last reader, pair g / 2 - 1, finished before this chunk's barrier
        issue_w((g >> 1) + 1 < npairs ? (g >> 1) + 1 : 0, (pc + 1) & 1);
        gate_rows<kRPW, kGeluPacked>(lds, lds + S::kDw + g * kDwF4, lo, lq, gbp);
        // chunk g + 1 consumes pair g / 2: its W DMA must have landed.  Issued after it by this wave:
        // this chunk's W issue (pw pieces) and, at a tile's first pair, the previous tile's output
        // stores (the previous pair 0 landed in the prologue or before the previous tile's epilogue
        // read its residual)
        if (g == 0)
          wait_w(std::integral_constant<int, kRPW * NTO>{});
        else
          wait_w(std::integral_constant<int, 0>{});
        lds_barrier();  // B_{g+1}: chunk g + 1's image
        f32x4 gn[kRPW];
        gate_rows<kRPW, kGeluPacked>(lds + kImg, lds + S::kDw + (g + 1) * kDwF4, lo, lq, gn);
        mfma_pair(gbp, gn, pc & 1);  // chunks g, g + 1
        ++pc;
        lds_barrier();  // B_{g+2}: chunk g + 2's image
      }
      // epilogue: y = acc + x1 + bias (gdfn_out's order); rows / columns past the image dropped
      const int xo = x0 + li;
      f32x4 res[kRPW][NTO];
#pragma unroll
      for (int r = 0; r < kRPW; ++r) {
        const int yo = min(y0 + kRPW * wi + r, p.H - 1);
        const unsigned off = xo < p.W ? (unsigned)((yo * p.W + xo) * p.ldx) * 4u + 16u * lq : kOOBf;
#pragma unroll
        for (int q = 0; q < NTO; ++q)
          res[r][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(off + 64u * q), 0, 0));
      }
      float* O = p.out + (long long)b * HW * p.ldo;
      const __amdgpu_buffer_rsrc_t ro =
          __builtin_amdgcn_make_buffer_rsrc(O, 0, (int)(HW * p.ldo * 4), 0x00020000);
#pragma unroll
      for (int r = 0; r < kRPW; ++r) {
        const int yo = y0 + kRPW * wi + r;
        const unsigned off =
            (xo < p.W && yo < p.H) ? (unsigned)((yo * p.W + xo) * p.ldo) * 4u + 16u * lq : kOOBf;
#pragma unroll
        for (int q = 0; q < NTO; ++q)
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(u32x4f, acc[r][q] + res[r][q] + lds[S::kBout + 4 * q + lq]), ro,
              (int)(off + 64u * q), 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (unused) W DMA lands before exit
}


// an even chunk count (the released config: hidS = 128 / 256), so every pair is full
bool ffn_fused_supported(int C, int hidS) {
  if (C != 48 && C != 96) return false;
  const int kch = hidS / 16;
  return hidS % 16 == 0 && kch >= 2 && kch % 2 == 0 && kch <= (C == 48 ? 8 : 16);
}

template <int C>
static hipError_t launch_ffn1(const FfnParams& p, hipStream_t s) {
  constexpr int lds = FfnShape<C>::kLds;
  static_assert(lds <= 160 * 1024, "ffn LDS");
  static bool attr[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!attr[dev]) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&ffn_fused_kernel<C>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr[dev] = true;
  }
  constexpr int TH = FfnShape<C>::TH;
  const long long tiles = (long long)p.Bn * ((p.H + TH - 1) / TH) * ((p.W + kTile - 1) / kTile);
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  long long grid = std::min<long long>(tiles, cus);  // one resident block per CU
  grid = (grid + 7) / 8 * 8;
  hipLaunchKernelGGL((ffn_fused_kernel<C>), dim3((unsigned)grid), dim3(64 * FfnShape<C>::NW), lds, s, p);
  return hipGetLastError();
}

hipError_t launch_ffn_fused(const FfnParams& p, int C, hipStream_t s) {
  if (!ffn_fused_supported(C, p.hidS) || p.ldx % 4 || p.ldo % 4 || p.Bn <= 0 || p.H <= 0 || p.W <= 0 ||
      (long long)p.H * p.W * std::max(p.ldx, p.ldo) * 4 >= (1LL << 31))
    return hipErrorInvalidValue;
  return C == 48 ? launch_ffn1<48>(p, s) : launch_ffn1<96>(p, s);
}

}  // namespace kdlae
