// Fused MDTA pass 1 of a single-head TransformerBlock attention half (KDLAE/KDLAE_model.py:118-119,
// :124-137; heads = 1, C = 48 and 96: encoder_level1, decoder_level1, refinement, refinement_out,
// enhance):
//   [q | k | v] = dwconv3x3( qkv( LN(x) ) ),  G = q k^T (over the pixels of a slot), |q|^2, |k|^2,  v -> HBM
// in ONE pass.  Unfused, the qkv GEMM wrote 3C floats per pixel that the Gram ring read back with a
// halo (C = 96 at 512^2: 1.5 KB written + 1.3 KB read per pixel, the write-heavy GEMM shape of the
// forward); fused, the kernel reads x with a halo and writes v: ~0.8 KB per pixel.  The price is the
// qkv projection recomputed on the tile's halo ring (180 pixels per 128), on the split-bf16 MFMAs.
//
// Block = 8 waves on a 16 x 8 pixel tile, persistent over the "units" of its XCD (one block per CU).
// A unit is one Gram slot of the unfused path (a 16-column strip x one row segment of an image,
// kdlae_t.cpp nslots_for), so the slot partition — and with it the fixed-order fp64 slot reduction,
// run-to-run determinism and batch invariance — is the ring kernel's.
//  * P waves (4-7): per tile, x rows of the 10 x 18 halo (12 pixel tiles of 16, 3 per wave), LayerNorm
//    in registers, split into bf16 planes; per chunk (16 output channels of qkv: q tiles, then k, then
//    v) the projection (split records LDS-DMA'd two chunks ahead into a 2-slot W ring) into the
//    chunk's halo image (LDS, [pixel][4 quads]; zeros outside the image = the dwconv padding).
//  * G waves (0-3): 2 output rows each; per chunk the depthwise 3x3 from the halo image, then
//      q chunk: the values split into bf16 planes into the q staging ([plane][channel][pixel]) and
//               their squares into the wave's norm partials;
//      k chunk: the same into a double-buffered k staging; in the NEXT chunk the Gram column of that
//               k tile: G[i][j] += q_i k_j^T on v_mfma_f32_16x16x32_bf16 (mfma6: the exact-split
//               fp32 product of mfma3.h), the 4 G waves splitting (pixel half x q-row half) for
//               C = 96, (pixel quarter) for C = 48, so each wave runs the same MFMA count per column;
//      v chunk: stored to HBM (the attention-output GEMM's input, as the ring kernel writes it).
//    At a unit's end the waves' Gram partials are summed in fixed order through LDS and written with
//    the norms into the unit's slot.
//  One barrier per chunk (P produces chunk c + 1 while G consumes chunk c), one more per unit.
// Numerics: the slot is the unfused slot; within it the Gram sums run over 32-pixel k-steps in split
// bf16 products (as accurate as an fp32 fma chain, mfma3.h) instead of the ring's f32 MFMA chain, so
// the fused and unfused results agree to fp32 rounding, not bit for bit (tests/test_kdlae_gpu.py).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kernels.h"
#include "mfma3.h"
#include "rowops.h"
#include "runtime.h"

namespace kdlae {

namespace {

constexpr unsigned kOOBm = 0x80000000u;
typedef unsigned u32x4m __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lptr_m;

template <int N>
__device__ __forceinline__ void wait_vmm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ void bar_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int C>
struct QShape {
  static constexpr int TW = 16, TH = 8, HR = TH + 2, HC = TW + 2;  // tile, halo rows / columns
  static constexpr int KG = C / 16, KP = (KG + 1) / 2;             // projection k-groups / split pairs
  static constexpr int CT = C / 16;                                 // channel tiles of q (= k = v), heads = 1
  static constexpr int NCH = 3 * CT;                                // chunks per tile: q, k, v tiles
  static constexpr int NPT = HR + 2, NP = 4, PT = 3;                // halo pixel tiles, P waves, per P wave
  static constexpr int NGW = 4, RPW = TH / NGW;                     // G waves, output rows per G wave
  // Gram split over the G waves: NPH pixel parts (of the tile's 4 k-steps of 32) x NIH q-row parts
  static constexpr int NPH = CT % 2 == 0 ? 2 : 4, NIH = 4 / NPH;
  static constexpr int IPW = CT / NIH, SPW = 4 / NPH;               // q rows / k-steps per G wave
  static constexpr int SP = 136;                                    // staging pixel stride (bf16)
  static constexpr int kPieces = 3 * KP;                            // 1 KiB W pieces per chunk
  static constexpr int kPPW = (kPieces + NP - 1) / NP;              // per P wave (uniform issue)
  // LDS carve (bytes)
  static constexpr int kImgF4 = HR * HC * 4;          // f32x4 per halo image slot: [pixel][4 quads]
  static constexpr int oImg = 0;                      // 2 slots
  static constexpr int kWSlot = kPieces * 1024;
  static constexpr int oW = oImg + 2 * kImgF4 * 16;   // 2 W slots
  static constexpr int oDw = oW + 2 * kWSlot;         // NCH x 40 f32x4: [9 taps][4 quads], bias [4]
  static constexpr int oBin = oDw + NCH * 40 * 16;    // NCH x 4 f32x4
  static constexpr int oQ = oBin + NCH * 4 * 16;      // q staging [3 planes][C][SP] bf16
  static constexpr int kKBuf = 3 * 16 * SP * 2;
  static constexpr int oK = oQ + 3 * C * SP * 2;      // 2 k buffers [3][16][SP] bf16
  static constexpr int oN = oK + 2 * kKBuf;           // norm partials [NGW][2C] f32
  static constexpr int oDummy = oN + NGW * 2 * C * 4; // 1 KiB landing slot of padding DMA pieces
  static constexpr int kLds = oDummy + 1024;
  static_assert(IPW * NIH == CT && SPW * NPH == 4, "gram split");
  static_assert(NGW * IPW * CT * 64 * 16 <= 3 * C * SP * 2, "gram partials fit the q staging");
  static_assert(TH % NGW == 0, "rows per G wave");
};

}  // namespace

template <int C>
__global__ __launch_bounds__(512, 1) void mdta_fused_kernel(MdtaFusedParams p) {
  using S = QShape<C>;
  constexpr int KG = S::KG, KP = S::KP, CT = S::CT, NCH = S::NCH, PT = S::PT, NP = S::NP;
  constexpr int kHR = S::HR, kHC = S::HC, kRPW = S::RPW, kImgF4 = S::kImgF4, SP = S::SP;
  // (a static member of S inside a builtin's scalar-offset argument made hipcc's host pass drop the
  // kernel's stub silently: local copies)
  constexpr int kWSlot = S::kWSlot, kPieces = S::kPieces, oW = S::oW, oDummy = S::oDummy;
  extern __shared__ __attribute__((aligned(16))) f32x4 lds[];
  char* ldsb = reinterpret_cast<char*>(lds);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int strips = p.W / 16;
  const int uper = strips * p.nseg, nunits = p.Bn * uper;
  // persistent, XCD-aware: XCD k walks units [k U / 8, (k + 1) U / 8), its blocks interleaved, so
  // neighbouring strips (whose halo columns overlap) run together on one L2
  const int xcd = (int)(blockIdx.x & 7), nxb = (int)(gridDim.x >> 3), xb = (int)(blockIdx.x >> 3);
  const int u_lo = (int)((long long)nunits * xcd / 8), u_hi = (int)((long long)nunits * (xcd + 1) / 8);
  if (u_lo + xb >= u_hi) return;  // block-uniform
  const long long HW = (long long)p.H * p.W;

  // resident: every chunk's dw taps + bias, the projection bias
  for (int i = tid; i < NCH * 40; i += 512) {
    const int c = i / 40, r = i - 40 * c;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (r < 36)
      v = *reinterpret_cast<const f32x4*>(p.wdw + (r >> 2) * 3 * C + 16 * c + 4 * (r & 3));
    else if (p.bdw)
      v = *reinterpret_cast<const f32x4*>(p.bdw + 16 * c + 4 * (r - 36));
    lds[S::oDw / 16 + i] = v;
  }
  for (int i = tid; i < NCH * 4; i += 512)
    lds[S::oBin / 16 + i] = p.bias ? reinterpret_cast<const f32x4*>(p.bias)[i] : f32x4{0.f, 0.f, 0.f, 0.f};

  const bool gw = wave < S::NGW;
  const int wi = gw ? wave : wave - S::NGW;

  // unit u -> image, strip, segment; tile k of a unit covers rows y0 + 8 k .. of rows [ys, ye)
  auto unit_geo = [&](int u, int& b, int& x0, int& ys, int& ye) {
    b = u / uper;
    const int slot = u - b * uper;
    const int seg = slot / strips;
    x0 = (slot - seg * strips) * 16;
    ys = seg * p.seg_rows;
    ye = min(p.H, ys + p.seg_rows);
  };

  // ---- P-wave state: halo pixel tiles PT wi .. PT wi + PT - 1 (rows 0..HR-1 over the interior
  // columns, then columns 0 and 17)
  int phy[PT], phx[PT];
  bool plv[PT];
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    const int pt = PT * wi + k;
    phy[k] = pt < kHR ? pt : li;
    phx[k] = pt < kHR ? li + 1 : (pt == kHR ? 0 : kHC - 1);
    plv[k] = pt < kHR || (pt < S::NPT && li < kHR);
  }
  const __amdgpu_buffer_rsrc_t rwin =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.Wqkv), 0, NCH * S::kWSlot, 0x00020000);
  // W of chunk c (its records are one contiguous kPieces KiB: tile-major split arena) into W slot s;
  // every P wave issues kPPW pieces straight-line, padding pieces land in the dummy slot
  auto issue_w = [&](int c, int s) {
#pragma unroll
    for (int i = 0; i < S::kPPW; ++i) {
      const int k = wi + NP * i;
      const bool real = k < kPieces;
      f32x4* dst = real ? lds + (oW + s * kWSlot) / 16 + 64 * k : lds + oDummy / 16;
      const int soff = real ? c * kWSlot + 1024 * k : 0;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rwin, (lptr_m)dst, 16, (int)(real ? 16u * lane : kOOBm), soff, 0, 0);
    }
  };
  f32x4 a[PT][KG];  // P waves: the x rows of the next tile (loaded ahead)
  int gbase = 0;    // P waves: global chunk count at the tile start (W slot of chunk c = (gbase + c) & 1)
  auto load_x = [&](int b, int x0, int y0) {
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.x + (long long)b * HW * p.ldx), 0, (int)(HW * p.ldx * 4), 0x00020000);
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const int yy = y0 - 1 + phy[k], xx = x0 - 1 + phx[k];
      const bool ok = plv[k] && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
      const unsigned off = ok ? (unsigned)((yy * p.W + xx) * p.ldx) * 4u + 16u * lq : kOOBm;
#pragma unroll
      for (int g = 0; g < KG; ++g)
        a[k][g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(off + 64u * g), 0, 0));
    }
  };

  // ---- G-wave state
  // halo image read offset (f32x4) of the wave's first input row, column tap j
  int lo[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) lo[j] = ((kRPW * wi) * kHC + li + j) * 4 + lq;
  const int ph = wi % S::NPH, ih = wi / S::NPH;  // Gram split: pixel part, q-row part
  f32x4 gacc[S::IPW][CT];                        // Gram partials of this wave (this unit)

  if (!gw) {
    __builtin_amdgcn_s_setprio(1);  // P waves first (the ffn.hip order)
    issue_w(0, 0);
    issue_w(1, 1);
    wait_vmm<0>();
    int b, x0, ys, ye;
    unit_geo(u_lo + xb, b, x0, ys, ye);
    load_x(b, x0, ys);
  } else {
#pragma unroll
    for (int i = 0; i < S::IPW; ++i)
#pragma unroll
      for (int j = 0; j < CT; ++j) gacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();

  // The two roles run their own unit / tile loops (the same tiles, the same barrier count per tile),
  // so the register allocator sees each role's live state on its own (as in ffn.hip).
  if (!gw) {
  for (int u = u_lo + xb; u < u_hi; u += nxb) {
    int b, x0, ys, ye;
    unit_geo(u, b, x0, ys, ye);
    const int ntile = (ye - ys + S::TH - 1) / S::TH;
    for (int tk = 0; tk < ntile; ++tk) {
      const int y0 = ys + S::TH * tk;
      {
        // ============================================================== P waves: qkv producer
        // the next tile (this unit's next, or the next unit's first) for the x prefetch
        int nb = -1, nx0 = 0, ny0 = 0;
        if (tk + 1 < ntile) {
          nb = b, nx0 = x0, ny0 = y0 + S::TH;
        } else if (u + nxb < u_hi) {
          int ye2;
          unit_geo(u + nxb, nb, nx0, ny0, ye2);
        }
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
        // projection of chunk c (W slot ws) -> halo image slot c & 1
        auto pin = [&](int c, int ws) {
          const f32x4* wl = lds + (S::oW + ws * S::kWSlot) / 16 + lane;
          f32x4 acc[PT];
#pragma unroll
          for (int k = 0; k < PT; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
          // every W plane of the chunk first (3 KP ds_read_b128), then the MFMAs in mfma6's term order
          // per pair: with one output tile per chunk a step holds only 3 - 9 MFMAs, too few to cover a
          // plane read issued one step ahead
          bf16x8 w[3 * KP];
#pragma unroll
          for (int st = 0; st < 3 * KP; ++st) {
            const int G = st / 3, off = (2 - (st - 3 * G)) * 64;  // planes l, m, h at +128, +64, +0
            w[st] = __builtin_bit_cast(bf16x8, wl[G * kRec3 + off]);
          }
#pragma unroll
          for (int st = 0; st < 3 * KP; ++st) {
            const int G = st / 3, pl = st - 3 * G;
            const bf16x8 p0 = w[st];
            if (pl == 2) {
#pragma unroll
              for (int r = 0; r < PT; ++r) acc[r] = mfma_bf(p0, xs[G][r].l, acc[r]);
            }
            if (pl >= 1) {
#pragma unroll
              for (int r = 0; r < PT; ++r) acc[r] = mfma_bf(p0, xs[G][r].m, acc[r]);
            }
#pragma unroll
            for (int r = 0; r < PT; ++r) acc[r] = mfma_bf(p0, xs[G][r].h, acc[r]);
          }
          const f32x4 bi = lds[S::oBin / 16 + 4 * c + lq];
          f32x4* img = lds + (c & 1) * kImgF4;
#pragma unroll
          for (int k = 0; k < PT; ++k) {
            if (!plv[k]) continue;
            img[(phy[k] * kHC + phx[k]) * 4 + lq] = in[k] ? acc[k] + bi : f32x4{0.f, 0.f, 0.f, 0.f};
          }
        };
        // W slots run on a global chunk count (NCH may be odd): chunk c of this tile is global chunk
        // gc0 + c, its W slot (gc0 + c) & 1.  The image slot is c & 1 within the tile.
        pin(0, gbase & 1);
        bar_lds();  // B_0
        for (int c = 0; c < NCH - 2; ++c) {
          // W slot of chunk c (read by pin(c) before B_c) takes chunk c + 2
          issue_w(c + 2, (gbase + c) & 1);
          pin(c + 1, (gbase + c + 1) & 1);
          wait_vmm<0>();  // W of chunk c + 2 (read by pin(c + 2) in the next chunk)
          bar_lds();      // B_{c+1}
        }
        // the last two chunks issue the next tile's chunks 0, 1 (global chunks gbase + NCH, + NCH + 1)
        if (nb >= 0) issue_w(0, (gbase + NCH) & 1);
        pin(NCH - 1, (gbase + NCH - 1) & 1);
        wait_vmm<0>();
        bar_lds();  // B_{NCH-1}
        if (nb >= 0) {
          issue_w(1, (gbase + NCH + 1) & 1);
          load_x(nb, nx0, ny0);  // during this chunk and the G epilogue
        }
        // past B_NCH pin(0) of the next tile reads the slot issued at chunk NCH - 2 (landed above); this
        // chunk's W pieces and the x loads may stay outstanding
        wait_vmm<S::kPPW + PT * KG>();
        bar_lds();  // B_NCH
        gbase += NCH;
        if (tk == ntile - 1) bar_lds();  // B_u: the G waves sum the unit's Gram partials
      }
    }
  }
  } else {
  for (int u = u_lo + xb; u < u_hi; u += nxb) {
    int b, x0, ys, ye;
    unit_geo(u, b, x0, ys, ye);
    const int ntile = (ye - ys + S::TH - 1) / S::TH;
    for (int tk = 0; tk < ntile; ++tk) {
      const int y0 = ys + S::TH * tk;
      {
        // ============================================================== G waves: stencil, Gram, v
        const int yv = y0 + kRPW * wi;  // this wave's first output row
        const bool first = tk == 0;
        bar_lds();  // B_0: chunk 0's image
        auto stencil = [&](int c, f32x4 (&d)[kRPW]) {
          const f32x4* sl = lds + (c & 1) * kImgF4;
          const f32x4* dw = lds + S::oDw / 16 + 40 * c;
          const f32x4 bb = dw[36 + lq];
#pragma unroll
          for (int r = 0; r < kRPW; ++r) d[r] = bb;
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            f32x4 wv[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) wv[i] = dw[(3 * i + j) * 4 + lq];
#pragma unroll
            for (int rr = 0; rr < kRPW + 2; ++rr) {
              const f32x4 v = sl[lo[j] + rr * kHC * 4];
#pragma unroll
              for (int i = 0; i < 3; ++i) {
                const int r = rr - i;
                if (r >= 0 && r < kRPW) d[r] = __builtin_elementwise_fma(v, wv[i], d[r]);
              }
            }
          }
        };
        // q / k chunk c in the transposed lane layout the Gram operands want: lane (li, lq) computes
        // channel li of the chunk at 8 pixels (tile row kRPW wi + (lq >> 1), columns 8 (lq & 1) .. + 7),
        // splits them into bf16 planes and writes each plane as one 16 B row piece of the
        // [3][rows][SP] staging block at channel row ch0 + li (r06: the pixel-per-lane layout took 24
        // 2-byte scatter writes per chunk, 1.1 ms of a C96@512^2 launch); pixels past the unit's rows
        // (or the image) as zeros; squares -> the wave's norm partials (nidx: q at 0, k at C)
        auto stage_qk = [&](int c, char* base, int rows, int ch0, int nidx) {
          const float* imgf = reinterpret_cast<const float*>(lds + (c & 1) * kImgF4);
          const float* dwf = reinterpret_cast<const float*>(lds + S::oDw / 16 + 40 * c);
          const int r = lq >> 1, cg = lq & 1;
          const int R = kRPW * wi + r;  // tile row; its halo rows are R .. R + 2
          float w[9], v[3][10], o[8];
#pragma unroll
          for (int t = 0; t < 9; ++t) w[t] = dwf[t * 16 + li];
          const float bb = dwf[144 + li];
#pragma unroll
          for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int hc = 0; hc < 10; ++hc) v[dy][hc] = imgf[((R + dy) * kHC + 8 * cg + hc) * 16 + li];
          const bool ok = y0 + R < ye;
          float s2 = 0.f;
#pragma unroll
          for (int x = 0; x < 8; ++x) {
            float a = bb;
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
              for (int dx = 0; dx < 3; ++dx) a = __builtin_fmaf(v[dy][x + dx], w[3 * dy + dx], a);
            o[x] = ok ? a : 0.f;
            s2 = __builtin_fmaf(o[x], o[x], s2);
          }
          const F3 pl = split3(f32x4{o[0], o[1], o[2], o[3]}, f32x4{o[4], o[5], o[6], o[7]});
          const int px = R * 16 + 8 * cg;
          *reinterpret_cast<bf16x8*>(base + ((0 * rows + ch0 + li) * SP + px) * 2) = pl.h;
          *reinterpret_cast<bf16x8*>(base + ((1 * rows + ch0 + li) * SP + px) * 2) = pl.m;
          *reinterpret_cast<bf16x8*>(base + ((2 * rows + ch0 + li) * SP + px) * 2) = pl.l;
          // the 4 pixel groups of a channel (lanes li, li + 16, li + 32, li + 48) in a fixed order
          s2 += __shfl_xor(s2, 16);
          s2 += __shfl_xor(s2, 32);
          if (lq == 0) {
            float* np = reinterpret_cast<float*>(ldsb + S::oN) + wi * 2 * C + nidx + li;
            *np = first ? s2 : *np + s2;
          }
        };
        // Gram column j (k tile j in k buffer j & 1): G[i][j] += sum over this wave's k-steps
        auto gram_col = [&](int j) {
          const char* kb = ldsb + S::oK + (j & 1) * S::kKBuf;
#pragma unroll
          for (int t = 0; t < S::SPW; ++t) {
            const int px = 32 * (ph * S::SPW + t) + 8 * lq;
            F3 kk;
            kk.h = *reinterpret_cast<const bf16x8*>(kb + ((0 * 16 + li) * SP + px) * 2);
            kk.m = *reinterpret_cast<const bf16x8*>(kb + ((1 * 16 + li) * SP + px) * 2);
            kk.l = *reinterpret_cast<const bf16x8*>(kb + ((2 * 16 + li) * SP + px) * 2);
#pragma unroll
            for (int ii = 0; ii < S::IPW; ++ii) {
              __builtin_amdgcn_sched_barrier(0);
              const int ch = 16 * (ih * S::IPW + ii) + li;
              F3 qq;
              qq.h = *reinterpret_cast<const bf16x8*>(ldsb + S::oQ + ((0 * C + ch) * SP + px) * 2);
              qq.m = *reinterpret_cast<const bf16x8*>(ldsb + S::oQ + ((1 * C + ch) * SP + px) * 2);
              qq.l = *reinterpret_cast<const bf16x8*>(ldsb + S::oQ + ((2 * C + ch) * SP + px) * 2);
              gacc[ii][j] = mfma6(qq, kk, gacc[ii][j]);
            }
          }
        };
        float* V = p.v_out + (long long)b * HW * p.ldv;
        auto store_v = [&](const f32x4 (&d)[kRPW], int c) {
#pragma unroll
          for (int r = 0; r < kRPW; ++r) {
            if (yv + r >= p.H) continue;
            *reinterpret_cast<f32x4*>(V + ((long long)(yv + r) * p.W + x0 + li) * p.ldv + 16 * (c - 2 * CT) + 4 * lq) = d[r];
          }
        };
        for (int c = 0; c < CT; ++c) {  // q chunks
          stage_qk(c, ldsb + S::oQ, C, 16 * c, 16 * c);
          bar_lds();  // B_{c+1}
        }
#pragma unroll
        for (int c = CT; c < 2 * CT; ++c) {  // k chunks; the Gram column of the previous k tile
          if (c > CT) gram_col(c - CT - 1);
          stage_qk(c, ldsb + S::oK + ((c - CT) & 1) * S::kKBuf, 16, 0, C + 16 * (c - CT));
          bar_lds();
        }
        {  // the first v chunk and the last Gram column
          gram_col(CT - 1);
          f32x4 d[kRPW];
          stencil(2 * CT, d);
          store_v(d, 2 * CT);
          bar_lds();
        }
        for (int c = 2 * CT + 1; c < NCH; ++c) {  // v chunks
          f32x4 d[kRPW];
          stencil(c, d);
          store_v(d, c);
          bar_lds();
        }
        if (tk == ntile - 1) {
          // unit end: the waves' Gram partials through LDS (the q staging is free until the next
          // tile's chunk 0), summed over the pixel parts in fixed order, + the norms -> the slot
          f32x4* gs = reinterpret_cast<f32x4*>(ldsb + S::oQ);
#pragma unroll
          for (int ii = 0; ii < S::IPW; ++ii)
#pragma unroll
            for (int j = 0; j < CT; ++j) gs[((wi * S::IPW + ii) * CT + j) * 64 + lane] = gacc[ii][j];
          bar_lds();  // B_u
          const int slot = u - b * uper;
          float* out = p.partial + ((long long)b * p.nslots + slot) * p.slot_floats;
          // pair (i, j) = q tile i, k tile j: wave wi writes pairs wi, wi + 4, ...
          for (int pi = wi; pi < CT * CT; pi += S::NGW) {
            const int i = pi / CT, j = pi - i * CT;
            const int ihh = i / S::IPW, ii = i - ihh * S::IPW;
            f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < S::NPH; ++q) s += gs[(((ihh * S::NPH + q) * S::IPW + ii) * CT + j) * 64 + lane];
            *reinterpret_cast<f32x4*>(out + (pi * 64 + lane) * 4) = s;
          }
          const float* nb = reinterpret_cast<const float*>(ldsb + S::oN);
          for (int idx = tid; idx < 2 * C; idx += 64 * S::NGW) {
            float t = 0.f;
#pragma unroll
            for (int w = 0; w < S::NGW; ++w) t += nb[w * 2 * C + idx];
            out[CT * CT * 256 + idx] = t;
          }
#pragma unroll
          for (int ii = 0; ii < S::IPW; ++ii)
#pragma unroll
            for (int j = 0; j < CT; ++j) gacc[ii][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (unused) W DMAs land before exit
}

bool mdta_fused_supported(int C, int heads, int H, int W, int nseg, int seg_rows) {
  if ((C != 48 && C != 96) || heads != 1) return false;
  return W % 16 == 0 && H % 8 == 0 && seg_rows % 8 == 0 && nseg >= 1 && seg_rows * nseg >= H;
}

template <int C>
static hipError_t launch_mdta1(const MdtaFusedParams& p, hipStream_t s) {
  constexpr int lds = QShape<C>::kLds;
  static_assert(lds <= 160 * 1024, "mdta_fused LDS");
  static bool attr[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!attr[dev]) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mdta_fused_kernel<C>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr[dev] = true;
  }
  const long long units = (long long)p.Bn * (p.W / 16) * p.nseg;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  long long grid = std::min<long long>(units, cus);  // one resident block per CU
  grid = (grid + 7) / 8 * 8;
  hipLaunchKernelGGL((mdta_fused_kernel<C>), dim3((unsigned)grid), dim3(512), lds, s, p);
  return hipGetLastError();
}

hipError_t launch_mdta_fused(const MdtaFusedParams& p, int C, hipStream_t s) {
  if (!mdta_fused_supported(C, 1, p.H, p.W, p.nseg, p.seg_rows) || p.ldx % 4 || p.ldv % 4 || p.Bn <= 0 ||
      p.nslots != (p.W / 16) * p.nseg || p.slot_floats != (C / 16) * (C / 16) * 256 + 2 * C ||
      (long long)p.H * p.W * std::max(p.ldx, p.ldv) * 4 >= (1LL << 31))
    return hipErrorInvalidValue;
  return C == 48 ? launch_mdta1<48>(p, s) : launch_mdta1<96>(p, s);
}

}  // namespace kdlae
