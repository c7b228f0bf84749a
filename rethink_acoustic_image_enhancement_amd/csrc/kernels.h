// Internal launch interface of the KDLAE HIP kernels (gfx950 / CDNA4).
//
// Activation layout in HBM: NHWC fp32 "views" — pixel-major, channels contiguous, a view is
// (base pointer, pixel stride `ld` in floats).  A view may be a channel slice of a wider buffer,
// which is how torch.cat in the reference (KDLAE_model.py:289,294,299,316) disappears: the
// producer writes straight into its half of the concatenated buffer.
//
// Packed 1x1 / implicit-GEMM weights ("fragment order"): for output tile t (16 channels) and
// k-group g (16 reduction indices) one 1 KiB record of 64 lanes x float4 holds
// W[16t + (lane & 15)][16g + 4*(lane >> 4) + e], e = 0..3 — the float4 an activation lane of the same
// k-group loads.  The GEMM kernels read the "split fragment order" derived from it (mfma3.h): per
// output tile and pair of k-groups, three bf16 planes of 1 KiB that feed v_mfma_f32_16x16x32_bf16.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdint.h>

namespace kdlae {

constexpr int kGemmThreads = 512;            // 8 waves
constexpr int kGemmRT = 2;                   // 16-row subtiles per wave
constexpr int kGemmRows = 8 * kGemmRT * 16;  // 256 pixels per block tile

struct GemmParams {
  const float* A;  int lda;        // input view
  int cg_per_tap;                  // channel groups (of 16) per tap = Cin_pad / 16
  int kgroups;                     // taps * cg_per_tap
  int ksize, dil;                  // 1 (pointwise) or 3 (implicit GEMM, zero padding = dil)
  const float* Wp; long long w_img_stride; int ntiles;  // split records [ntiles][ceil(kgroups/2)][kRec3]
  int N;                           // output channels stored (padded channels included)
  const float* bias;               // [ntiles*16] or null
  float* out; int ldo;
  const float* R; int ldr;         // residual view (may alias out) or null
  const float* stats;              // [P][2] = (mean, rstd) or null
  int ln;                          // 0 none, 1 BiasFree LN on A, 2 WithBias LN on A
  int ln_C;                        // LN channel count (true C)
  int relu;                        // apply ReLU after bias/residual
  int Bn, H, W;                    // geometry of the input grid
  int out_mode;                    // 0 plain, 1 PixelUnshuffle(2), 2 PixelShuffle(2)
  int tiles_per_img, total_tiles, tiles_per_block;
  int kchunks;
  int group_tiles;                 // resident schedule: output tiles whose weights one block keeps in LDS
  int F, kt;                       // frames per sequence (1 for 2-D) and temporal taps (1, or 3 for Conv3d)
  // fused attention output (gemm_attn_in_kernel): A = v rows, R = the block input x; the kernel
  // forms x1 = x + M v (+ bias_m) with the per-image folded projection M (KDLAE_model.py:140-144,
  // :160), stores x1 to out1, and runs LN + the GEMM on x1 (:161, :99) — x1 never round-trips HBM
  const float* Wm; long long wm_img_stride; const float* bias_m;
  float* out1; int ldo1;
};

struct GramParams {
  const float* qkv; int ld;        // [P][ld]: q at [0,C), k at [C,2C), v at [2C,3C)
  const float* wdw;                // [9][3C] tap-major
  const float* bdw;                // [3C] or null
  float* v_out; int ldv;
  float* partial;                  // [B][heads][nslots][slot_floats]
  int C, heads, Ch;
  int Bn, H, W;
  int nslots, slot_floats;
  const float* zeros;              // >= 16 zero floats (DMA source for padding); null -> no ring kernel
};

struct GateParams {
  const float* x; int ld;          // [P][ld]: x1 at [0,hidS), x2 at [hidS, 2 hidS)
  int hidS;
  const float* w;                  // [9][2 hidS]
  const float* b;                  // [2 hidS] or null
  float* out; int ldo;
  int Bn, H, W;
};

struct SmallInParams {             // 3x3 (kt=1) or 3x3x3 (kt=3) conv, Cin * 9 * kt <= 36, Cout % 16 == 0
  const float* in; long long sb, sc, sy, sx;
  int Cin, Cout, dil;
  const float* w; const float* bias;   // w: [Cout][Cin][kt][3][3]
  float* out; int ldo;
  int Bn, H, W;
  int F, kt; long long st;             // frames per sequence, temporal taps, frame stride of the input
  int relu;
  const float* in_sub;                 // if set, the conv input is (in - in_sub) (ASDQE diff extractor)
  int vh, vw;                          // valid input extent (zero pad bottom/right beyond it); 0 = H, W
  int wt;                              // > 0 (kt 1): w is the weight of the conv this one transposes, [Cin][wt][3][3]
                                       // with wt = this conv's total Cout, taps flipped (a training dX)
};

struct SmallOutParams {            // 3x3 (ks=3) or pointwise (ks=1) conv with Cout <= 4, Cin % 16 == 0
  const float* in; int ld; int Cin, Cout;
  const float* w; const float* bias;   // w: [Cout][Cin][ks][ks]
  int Bn, H, W;
  int F, ks;                           // frames per sequence (pixels per image = F*H*W), kernel size
  float* out; int out_nchw; int ldo;   // NCHW (ldo unused) or NHWC with pixel stride ldo
  const float* res;                    // NCHW residual (same shape as out) or null
  const float* extra;                  // NCHW [B,1,H,W] copied into channel Cout (NHWC mode) or null
  int wt;                              // 1 (ks 3): w is the weight of the conv this one transposes,
                                       // [Cin][Cout][3][3] with flipped taps (a training dX)
  const float* res_nhwc; int ldr;      // NHWC residual added before the store (NHWC mode; may alias out)
};

bool gemm_attn_in_variant(int NT, int KG, int nch);
hipError_t launch_gemm(const GemmParams& p, int NT, int KG, int wpe, int grid_x, hipStream_t s);
hipError_t launch_gemm_route(const GemmParams& p, int NT, int KG, int wpe, int grid_x, int route, hipStream_t s);
bool gemm_variant_entry(int family, int i, int* v);
bool gemm_has_variant(int NT, int KG, bool conv3, int wpe, bool resident, int out_mode);
bool gemm_has_variant2(int NT, int KG, bool conv3, int out_mode);  // r02 chunked kernel
hipError_t launch_ln_stats(const float* x, int ld, int C, long long P, float* stats, hipStream_t s);
hipError_t launch_dwconv_gram(const GramParams& p, hipStream_t s);
hipError_t launch_dwconv_gram_route(const GramParams& p, int route, hipStream_t s);  // 2: generic kernel
hipError_t launch_gram_reduce(const float* partial, float* reduced, int Bn, int heads, int nslots,
                              int slot_floats, hipStream_t s);
hipError_t launch_attn_fold(const float* reduced, int slot_floats, const float* proj, const float* temp,
                            float* Mpacked, int Bn, int C, int heads, hipStream_t s);
hipError_t launch_dwconv_gate(const GateParams& p, hipStream_t s);
hipError_t launch_conv_small_in(const SmallInParams& p, hipStream_t s);
hipError_t launch_conv_small_out(const SmallOutParams& p, hipStream_t s);
// MaxPool (1,2,2) / MaxPool2d(2) on NHWC views: [N frames][H][W][C] -> [N][H/2][W/2][C] (floor)
hipError_t launch_maxpool2(const float* in, int ldi, float* out, int ldo, int C, long long nframes, int H, int W,
                           hipStream_t s);

// Fused GDFN tail: out = R + project_out(gelu_erf(dw3x3(x1)) * dw3x3(x2)) (gdfn.hip).
struct GdfnParams {
  const float* x; int ld;          // project_in output, chunk-interleaved [g][x1 16 | x2 16] per pixel
  int hidS;                        // padded hidden width (multiple of 16)
  const float* dw;                 // per chunk g (hidS/16 of them) 512 floats: [9 taps][32 ch] weights,
                                   // [32] bias at +288, zero pad (channel order as in x)
  const float* Wp;                 // project_out split records [C/16][hidS/32][kRec3] (mfma3.h)
  const float* bias;               // [C] or null
  const float* R; int ldr;         // residual (may alias out) or null
  float* out; int ldo;
  int Bn, H, W;
  const float* zeros;              // >= 16 B of zeros in device memory (source of out-of-image halo lines)
  int nsplit;                      // set by launch_gdfn_out: blocks per pixel tile, each owning C/nsplit outputs
};
bool gdfn_supported(int C, int hidS);
hipError_t launch_gdfn_out(const GdfnParams& p, int C, hipStream_t s);

// Fused feed-forward half (ffn.hip): out = x + project_out(gate(dwconv(project_in(LN(x))))) for C = 48 /
// 96 — project_in recomputed on each tile's halo, so its 2 hidS-wide rows never reach HBM.  `out` must
// not overlap x (neighbouring tiles read x as halo).
struct FfnParams {
  const float* x; int ldx;         // block input after the attention half (x1), [P][ldx]
  float* out; int ldo;
  int ln;                          // 1 BiasFree, 2 WithBias
  int hidS;                        // padded hidden width
  const float* Win;                // project_in split records [2 hidS / 16][C / 32 (round up)][kRec3], chunk-interleaved rows
  const float* bias_in;            // [2 hidS] (chunk-interleaved) or null
  const float* dw;                 // [hidS / 16][512] dw blocks (gdfn.hip layout)
  const float* Wout;               // project_out split records [C / 16][hidS / 32][kRec3]
  const float* bias_out;           // [C] or null
  int Bn, H, W;
};
bool ffn_fused_supported(int C, int hidS);
hipError_t launch_ffn_fused(const FfnParams& p, int C, hipStream_t s);


// Fused MDTA pass 1 for single-head C = 48 / 96 blocks (mdta_fused.hip): LN + qkv projection recomputed
// on each tile's halo, depthwise 3x3, v -> v_out, Gram + |q|^2 / |k|^2 -> the Gram slots of
// launch_dwconv_gram (same slot partition and layout: 16-column strips x nseg row segments)
struct MdtaFusedParams {
  const float* x; int ldx;         // block input [P][ldx]
  int ln;                          // 1 BiasFree, 2 WithBias
  const float* Wqkv;               // qkv split records [3C / 16][C / 32 (round up)][kRec3]
  const float* bias;               // [3C] or null (LN bias / conv bias folded)
  const float* wdw;                // [9][3C] tap-major
  const float* bdw;                // [3C] or null
  float* v_out; int ldv;
  float* partial;                  // [B][nslots][slot_floats]
  int nslots, slot_floats, nseg, seg_rows;
  int Bn, H, W;
};
bool mdta_fused_supported(int C, int heads, int H, int W, int nseg, int seg_rows);
hipError_t launch_mdta_fused(const MdtaFusedParams& p, int C, hipStream_t s);

// Pre/post-processing around the forward (pipeline.hip)
struct PreParams {
  const uint8_t* in; int B, h, w, cin, cout, bgr;  // u8 [B][h][w][cin]
  int gray;                                          // 1: cv2 COLOR_BGR2GRAY of a BGR(A) pixel, cout = 1
  int H, W;                                          // padded size (reflect, bottom/right)
  float* img;                                        // f32 [B][cout][H][W]
  const float* rate; float* rate_map;                // per-image rate [B] -> [B][1][H][W] (optional)
};
struct PostParams {
  const float* src; int B, C, Hs, Ws;                // f32 [B][C][Hs][Ws] (model output)
  int h, w, scale;                                   // crop (h*scale, w*scale) of the output
  const uint8_t* lq; int cin;                        // u8 [B][h][w][cin] input for the black mask (optional)
  uint8_t* out;                                      // u8 [B][h*scale][w*scale][C]
};
hipError_t launch_preprocess_u8(const PreParams& p, hipStream_t s);
hipError_t launch_postprocess_u8(const PostParams& p, hipStream_t s);

// Bilinear x2, align_corners=True (ASDQE_model.py:53): NHWC [N][h][w][C] -> [N][2h][2w][C] into a
// strided destination (a concat half).  C % 4 == 0.
hipError_t launch_upsample2x(const float* in, int ldi, float* out, int ldo, int C, int N, int h, int w,
                             hipStream_t s);
// Global average pool, pass 1: partial[b][slot][C] = sum over the slot's pixel range (fixed order).
hipError_t launch_gap_partial(const float* in, int ld, int C, int B, long long HW, int slots, float* partial,
                              hipStream_t s);
// ASDQE head (ASDQE_model.py:144-154 + the linear outc folded ahead of the pool): per image
// g = mean(partial) [C]; f = Wo g + bo [M]; h1 = relu(W1 f + b1) [N1]; h2 = relu(W2 h1 + b2) [N2];
// score = tanh(w3 . h2 + b3).
struct HeadParams {
  const float* partial; int slots, C; float inv_hw;
  const float* wo; const float* bo; int M;
  const float* w1; const float* b1; int N1;
  const float* w2; const float* b2; int N2;
  const float* w3; const float* b3;
  float* score; int B;
};
hipError_t launch_asdqe_head(const HeadParams& p, hipStream_t s);

// 16 -> 16 channel 3x3x3 Conv3d / 3x3 Conv2d (+ bias, ReLU) on NDHWC views, LDS-tiled (conv3d_c16.hip).
// wp: fragment-order weights of a Gemm with ntiles = 1, cg_per_tap = 1, kgroups = 27 (runtime.h pack).
struct Conv3dC16Params {
  const float* in; int ldi;        // [B][F][H][W] pixels, 16 channels at stride ldi
  const float* wp;                 // [27][64][4]
  const float* bias;               // [16]
  float* out; int ldo;
  int Bn, F, H, W;
  int relu;
  int kt;                          // temporal taps: 3 (Conv3d) or 1 (Conv2d, F = 1)
};
hipError_t launch_conv3d_c16(const Conv3dC16Params& p, hipStream_t s);

// LDS-tiled implicit-GEMM 3x3 (kt 1) / 3x3x3 (kt 3) conv with 2..8 output tiles of 16 channels (conv_lds.hip):
// wp = fragment-order weights of a Gemm with k = tap * cin_pad + c (kgroups = 9 kt cin_pad / 16).
struct ConvLdsParams {
  const float* in; int ldi; int cin_pad;
  const float* wp; int ntiles, kgroups;
  const float* bias;               // [ntiles * 16] or null
  float* out; int ldo;
  int Bn, F, H, W;
  int kt, relu;
  // optional: the same weights as split records (mfma3.h, pairs of consecutive k-groups); used by the
  // 2-D kernel when cin_pad % 32 == 0, where its (tap, 2-group chunk) pairs are exactly those pairs
  const float* wp3 = nullptr;
  // store map: 0 plain [px][ldo]; 1 PixelUnshuffle(2) into the half-resolution image (KDLAE-T
  // Downsample, KDLAE_model.py:186-187: channel 4 n + 2 (y & 1) + (x & 1)); 2 PixelShuffle(2) into the
  // double-resolution image (Upsample, :196-197: output n -> pixel (2y + (n >> 1 & 1), 2x + (n & 1)),
  // channel n >> 2); outputs n < nout only
  int out_mode = 0, nout = 0;
};
bool conv_lds_supported(int kt, int ntiles, int cin_pad);
hipError_t launch_conv_lds(const ConvLdsParams& p, hipStream_t s);

}  // namespace kdlae
