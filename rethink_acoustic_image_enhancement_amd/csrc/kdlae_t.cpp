// KDLAE-T host runtime: config validation, state_dict staging, weight packing into the device
// layout, workspace planning and the forward launch sequence (one HIP stream, no host syncs).
//
// Forward = KDLAE_teacher.forward (KDLAE/KDLAE_model.py:270-336) restated on NHWC views:
//   patch_embed -> encoder_level1 (written straight into the second half of the level-1 concat
//   buffer, so torch.cat at :299 is free) -> down1_2 (implicit-GEMM 3x3 + PixelUnshuffle store) ->
//   ... -> latent -> up4_3 (3x3 + PixelShuffle store into the first half of the level-3 concat
//   buffer, :288-289) -> reduce_chan_level3 -> ... -> output / output_param / refinement_out /
//   output2 + img -> hq; static=="train": cen -> upen -> enhance -> outputen -> sr (:324-329).
// Each TransformerBlock (:159-163) is 7 launches:
//   [LN1+qkv GEMM] [dwconv+Gram] [slot reduce] [softmax+fold into W_proj] [A.v.proj GEMM + residual]
//   [LN2+project_in GEMM] [dwconv+GELU gate] [project_out GEMM + residual]   (+ LN stats when K is chunked)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "runtime.h"

namespace kdlae {

struct BlockW {
  int C = 0, heads = 0, Ch = 0, hid = 0, hidS = 0;
  Gemm qkv, pin, pout, proj_gemm;  // proj_gemm: geometry of the per-image M GEMM
  size_t dwqkv = kNone, dwqkv_b = kNone, proj = kNone, proj_b = kNone, temp = kNone;
  size_t dwffn = kNone, dwffn_b = kNone;
  bool fused_gdfn = false;  // project_in output chunk-interleaved; dwconv+gate+project_out in one kernel
  bool fused_attn_in = false;  // x1 = x + M v, LN and project_in in one GEMM kernel (gemm_attn_in_kernel)
  // when project_in needs two resident weight groups (C = 96): the fused kernel runs group 0 (and
  // forms x1), a plain LN GEMM on x1 runs group 1
  bool attn_in_split = false;
  Gemm pin_g0, pin_g1;
  // r05: the whole feed-forward half (LN, project_in, dwconv + gate, project_out, residual) in one
  // kernel (ffn.hip), project_in recomputed on each tile's halo; the block output goes to the other
  // buffer of a ping-pong pair (stage()).  Debug flag no_ffn_fusion keeps the unfused kernels.
  bool ffn_fused = false;
  // r06: MDTA pass 1 with LN + qkv recomputed on each tile's halo (mdta_fused.hip) for single-head
  // C = 48 / 96 blocks; opt-in (debug flag mdta_fusion), the qkv GEMM + Gram ring by default
  bool mdta_fused = false;
};

}  // namespace kdlae

using namespace kdlae;

struct kdlae_t_handle {
  kdlae_t_config cfg{};
  int device = 0;
  ParamStore ps;           // expected state_dict keys (ordered, flat offsets) + host-staged values
  bool built = false;      // pack program uploaded (depends on the config only)
  bool committed = false;  // arena filled from parameters at least once
  DeviceWeights dw;        // packed arena + pack program
  // model
  std::vector<BlockW> enc1, enc2, enc3, latent, dec3, dec2, dec1, refinement, refinement_out, enhance;
  SmallW patch_embed, output, output_param, output2, cen, outputen;
  Gemm down1_2, down2_3, down3_4, up4_3, up3_2, up2_1, upen, reduce3, reduce2;
  size_t zeros = kNone;  // 64 zero floats (halo source for the fused GDFN kernel)
  // probe
  int probe_class = 0, probe_level = 0;
  std::vector<hipEvent_t> ev;
  size_t ev_used = 0;
  double probe_bytes = 0, probe_flops = 0;
  long long probe_launches = 0;
  struct ProbeRec { std::string tag; double bytes, flops; };
  std::vector<ProbeRec> probe_recs;
  // diagnostics (kdlae_t_debug_taps): per TransformerBlock in execution order, a device buffer that
  // receives the block's output as compact NHWC [B][H_i][W_i][C_i] (nullptr: not tapped)
  std::vector<float*> taps;

  const float* P(size_t off) const { return dw.P(off); }
  const float* P3(size_t off) const { return dw.P3(off); }
};

namespace kdlae {

static int hid_of(const kdlae_t_config& c, int dim) { return (int)((double)dim * c.ffn_expansion_factor); }

static void add_key(kdlae_t_handle* h, const std::string& k, int64_t n) { h->ps.add(k, n); }

// Expected state_dict (KDLAE_model.py:220-268, TransformerBlock :150-157, Attention :113-120,
// FeedForward :90-99, LayerNorm :73-79).
static void build_keys(kdlae_t_handle* h) {
  const kdlae_t_config& c = h->cfg;
  auto conv = [&](const std::string& n, int co, int ci, int k, bool b) {
    add_key(h, n + ".weight", (int64_t)co * ci * k * k);
    if (b) add_key(h, n + ".bias", co);
  };
  auto block = [&](const std::string& p, int dim, int heads) {
    const int hid = hid_of(c, dim);
    add_key(h, p + ".norm1.body.weight", dim);
    if (!c.layernorm_biasfree) add_key(h, p + ".norm1.body.bias", dim);
    add_key(h, p + ".attn.temperature", heads);
    conv(p + ".attn.qkv", 3 * dim, dim, 1, c.bias);
    conv(p + ".attn.qkv_dwconv", 3 * dim, 1, 3, c.bias);
    conv(p + ".attn.project_out", dim, dim, 1, c.bias);
    add_key(h, p + ".norm2.body.weight", dim);
    if (!c.layernorm_biasfree) add_key(h, p + ".norm2.body.bias", dim);
    conv(p + ".ffn.project_in", 2 * hid, dim, 1, c.bias);
    conv(p + ".ffn.dwconv", 2 * hid, 1, 3, c.bias);
    conv(p + ".ffn.project_out", dim, hid, 1, c.bias);
  };
  auto stage = [&](const std::string& n, int cnt, int dim, int heads) {
    for (int i = 0; i < cnt; ++i) block(n + "." + std::to_string(i), dim, heads);
  };
  const int d = c.dim;
  const int* nb = c.num_blocks;
  const int* hd = c.heads;
  const int nr = c.num_refinement_blocks;
  conv("patch_embed.proj", d, c.inp_channels, 3, false);
  stage("encoder_level1", nb[0], d, hd[0]);
  conv("down1_2.body.0", d / 2, d, 3, false);
  stage("encoder_level2", nb[1], 2 * d, hd[1]);
  conv("down2_3.body.0", d, 2 * d, 3, false);
  stage("encoder_level3", nb[2], 4 * d, hd[2]);
  conv("down3_4.body.0", 2 * d, 4 * d, 3, false);
  stage("latent", nb[3], 8 * d, hd[3]);
  conv("up4_3.body.0", 16 * d, 8 * d, 3, false);
  conv("reduce_chan_level3", 4 * d, 8 * d, 1, c.bias);
  stage("decoder_level3", nb[2], 4 * d, hd[2]);
  conv("up3_2.body.0", 8 * d, 4 * d, 3, false);
  conv("reduce_chan_level2", 2 * d, 4 * d, 1, c.bias);
  stage("decoder_level2", nb[1], 2 * d, hd[1]);
  conv("up2_1.body.0", 4 * d, 2 * d, 3, false);
  stage("decoder_level1", nb[0], 2 * d, hd[0]);
  stage("refinement", nr, 2 * d, hd[0]);
  conv("output", c.out_channels, 2 * d, 3, c.bias);
  conv("output_param", 2 * d, c.out_channels + 1, 3, c.bias);
  stage("refinement_out", nr, 2 * d, hd[0]);
  conv("output2", c.out_channels, 2 * d, 3, c.bias);
  if (c.static_train) {
    const int hc = 2 * d;
    conv("cen", hc, c.out_channels, 3, c.bias);
    conv("upen.body.0", 2 * hc, hc, 3, false);
    stage("enhance", nr, hc / 2, hd[0]);
    conv("outputen", c.out_channels, hc / 2, 3, c.bias);
  }
}

static int validate(const kdlae_t_config& c) {
  if (c.dual_pixel_task)
    return fail(KDLAE_ENOTIMPL, "dual_pixel_task=True: the reference forward raises NameError (out_hq undefined, KDLAE_model.py:305-321)");
  if (c.dim <= 0 || c.dim % 16)
    return fail(KDLAE_EINVAL_CONFIG, "dim must be a positive multiple of 16 on the HIP path");
  if (c.inp_channels < 1 || c.inp_channels > 4 || c.out_channels < 1 || c.out_channels > 3)
    return fail(KDLAE_EINVAL_CONFIG, "inp_channels must be 1..4 and out_channels 1..3");
  if (c.inp_channels != c.out_channels)
    return fail(KDLAE_EINVAL_CONFIG, "inp_channels must equal out_channels (hq = out + inp_img, KDLAE_model.py:321)");
  for (int i = 0; i < 4; ++i)
    if (c.num_blocks[i] < 0 || c.heads[i] <= 0) return fail(KDLAE_EINVAL_CONFIG, "bad num_blocks/heads");
  if (c.num_refinement_blocks < 0) return fail(KDLAE_EINVAL_CONFIG, "bad num_refinement_blocks");
  auto head_ok = [&](int C, int heads) {
    if (C % heads) return false;
    const int ch = C / heads;
    if (ch % 16) return false;
    return ch / 16 >= 1 && ch / 16 <= 8;
  };
  const int d = c.dim;
  const int levels[4] = {d, 2 * d, 4 * d, 8 * d};
  for (int i = 0; i < 4; ++i)
    if (!head_ok(levels[i], c.heads[i]))
      return fail(KDLAE_EINVAL_CONFIG, "channels per head must be a multiple of 16 in [16, 128] at every level");
  if (!head_ok(2 * d, c.heads[0]))
    return fail(KDLAE_EINVAL_CONFIG, "channels per head of decoder_level1/refinement must be a multiple of 16 in [16, 128]");
  if (c.ffn_expansion_factor <= 0) return fail(KDLAE_EINVAL_CONFIG, "bad ffn_expansion_factor");
  return KDLAE_OK;
}

// ----------------------------------------------------------------------------- packing helpers
// The packer records the device layout as a pack program (runtime.h): every packed float names the
// flat-parameter entries it is gathered from.  Values are produced on the device (pack.hip).
struct Packer {
  kdlae_t_handle* h;
  PackProgram prog;
  int err = KDLAE_OK;

  int32_t get(const std::string& k) { return h->ps.base(k, &err); }

  // generic fragment-order pack: Wf(n, k) -> PEx over [ntiles*16] x [kgroups*16]
  template <class F>
  size_t pack(int ntiles, int kgroups, F Wf) {
    return prog.add(pack_fragments(ntiles, kgroups, Wf));
  }
  // f32 fragment block + its split-fragment-order copy (what the GEMM kernels read, mfma3.h)
  template <class F>
  void pack_gemm(Gemm& g, F Wf) {
    g.w = pack(g.ntiles, g.kgroups, Wf);
    g.w3 = prog.split(g.w, g.ntiles, g.kgroups);
  }

  // 1x1 conv [Cout][Cin] with optional LN(weight, bias) folded on the input side.
  // row_map(n) -> source output row or -1 (padding); stored N = nstore.
  template <class RowMap>
  Gemm pointwise(const std::string& name, int Cout, int Cin, int Kpad, int nstore, RowMap row_map,
                 const std::string& ln_prefix, bool conv_bias, bool prefer_single_k) {
    Gemm g;
    const int32_t W = get(name + ".weight");
    const int32_t lnw = ln_prefix.empty() ? -1 : get(ln_prefix + ".body.weight");
    const int32_t lnb = (!ln_prefix.empty() && !h->cfg.layernorm_biasfree) ? get(ln_prefix + ".body.bias") : -1;
    const int32_t cb = conv_bias ? get(name + ".bias") : -1;
    if (err) return g;
    g.ntiles = (nstore + 15) / 16;
    g.kgroups = Kpad / 16;
    g.N = nstore;
    g.K = Kpad;
    g.ksize = 1;
    g.n_true = Cout;
    g.k_true = Cin;
    pack_gemm(g, [&](int n, int k) -> PEx {
      if (n >= nstore || k >= Cin) return PEx{};
      const int src = row_map(n);
      if (src < 0) return PEx{};
      return PEx{W + src * Cin + k, lnw >= 0 ? lnw + k : -1};
    });
    if (cb >= 0 || lnb >= 0) {
      // bias' = conv bias + W . ln_bias (the WithBias LN shift pushed through the 1x1 conv)
      std::vector<PEx> bv((size_t)g.ntiles * 16);
      if (lnb < 0)
        for (int n = 0; n < nstore; ++n) {
          const int src = row_map(n);
          if (src >= 0) bv[n].a = cb + src;
        }
      g.bias = prog.add(bv);
      if (lnb >= 0)
        for (int n = 0; n < nstore; ++n) {
          const int src = row_map(n);
          if (src < 0) continue;
          PDot d;
          d.dst = (int64_t)g.bias + n;
          d.base = cb >= 0 ? cb + src : -1;
          d.w = W + src * Cin;
          d.v = lnb;
          d.K = Cin;
          prog.dots.push_back(d);
        }
    }
    choose_variant(g, prefer_single_k);
    return g;
  }

  // 3x3 conv [Cout][Cin][3][3] as implicit GEMM, k = tap * Cin + c (Cin % 16 == 0)
  Gemm conv3(const std::string& name, int Cout, int Cin, int out_mode) {
    Gemm g;
    g.out_mode = out_mode;
    const int32_t W = get(name + ".weight");
    if (err) return g;
    g.ksize = 3;
    g.cg_per_tap = Cin / 16;
    g.ntiles = (Cout + 15) / 16;
    g.kgroups = 9 * Cin / 16;
    g.N = Cout;
    g.K = 9 * Cin;
    g.n_true = Cout;
    g.k_true = 9 * Cin;
    pack_gemm(g, [&](int n, int k) -> PEx {
      if (n >= Cout) return PEx{};
      const int tap = k / Cin, c = k - tap * Cin;
      return PEx{W + (n * Cin + c) * 9 + tap, -1};
    });
    choose_variant(g, false);
    return g;
  }

  SmallW small(const std::string& name, int Cout, int Cin, bool bias) {
    SmallW s;
    s.Cout = Cout;
    s.Cin = Cin;
    const int32_t W = get(name + ".weight");
    const int32_t B = bias ? get(name + ".bias") : -1;
    if (err) return s;
    s.w = prog.copy(W, (size_t)Cout * Cin * 9);
    if (B >= 0) s.bias = prog.copy(B, Cout);
    return s;
  }

  BlockW block(const std::string& p, int C, int heads) {
    BlockW b;
    const kdlae_t_config& c = h->cfg;
    b.C = C;
    b.heads = heads;
    b.Ch = C / heads;
    b.hid = hid_of(c, C);
    b.hidS = ru16(b.hid);
    const int hid = b.hid, hidS = b.hidS;
    b.qkv = pointwise(p + ".attn.qkv", 3 * C, C, C, 3 * C, [](int n) { return n; }, p + ".norm1", c.bias, true);
    const int32_t dw = get(p + ".attn.qkv_dwconv.weight");
    const int32_t dwb = c.bias ? get(p + ".attn.qkv_dwconv.bias") : -1;
    const int32_t pw = get(p + ".attn.project_out.weight");
    const int32_t pb = c.bias ? get(p + ".attn.project_out.bias") : -1;
    const int32_t tp = get(p + ".attn.temperature");
    const int32_t fw = get(p + ".ffn.dwconv.weight");
    const int32_t fb = c.bias ? get(p + ".ffn.dwconv.bias") : -1;
    if (err) return b;
    {
      std::vector<PEx> v((size_t)9 * 3 * C);
      for (int ch = 0; ch < 3 * C; ++ch)
        for (int t = 0; t < 9; ++t) v[(size_t)t * 3 * C + ch].a = dw + ch * 9 + t;
      b.dwqkv = prog.add(v);
      if (dwb >= 0) b.dwqkv_b = prog.copy(dwb, (size_t)3 * C);
    }
    b.proj = prog.copy(pw, (size_t)C * C);
    if (pb >= 0) b.proj_b = prog.copy(pb, C);
    b.temp = prog.copy(tp, heads);
    b.proj_gemm.ntiles = C / 16;
    b.proj_gemm.kgroups = C / 16;
    b.proj_gemm.N = C;
    b.proj_gemm.K = C;
    b.proj_gemm.n_true = C;
    b.proj_gemm.k_true = C;
    b.proj_gemm.bias = b.proj_b;
    b.proj_gemm.has_res = true;
    choose_variant(b.proj_gemm, true);
    // FFN: project_in rows [x1 (hid) | x2 (hid)].  Unfused: stored [x1 padded to hidS | x2 padded
    // to hidS] for the gate kernel.  Fused (gdfn.hip): chunk-interleaved, 16 channels of x1 then the
    // same 16 of x2 per 32-channel chunk, so each chunk of a pixel is one 128 B line.
    b.fused_gdfn = gdfn_supported(C, hidS);
    const bool fz = b.fused_gdfn;
    auto rmap = [hid, hidS, fz](int n) -> int {
      if (fz) {
        const int c = 16 * (n >> 5) + (n & 15);
        if (c >= hid) return -1;
        return (n & 16) ? hid + c : c;
      }
      if (n < hidS) return n < hid ? n : -1;
      const int m = n - hidS;
      return m < hid ? hid + m : -1;
    };
    b.pin = pointwise(p + ".ffn.project_in", 2 * hid, C, C, 2 * hidS, rmap, p + ".norm2", c.bias, true);
    if (fz) {
      // per 32-channel chunk: [9 taps][32] weights, [32] bias at +288, zero pad to 512 (gdfn.hip)
      std::vector<PEx> v((size_t)(hidS / 16) * 512);
      for (int n = 0; n < 2 * hidS; ++n) {
        const int src = rmap(n);
        if (src < 0) continue;
        PEx* blk = v.data() + (size_t)(n >> 5) * 512;
        for (int t = 0; t < 9; ++t) blk[t * 32 + (n & 31)].a = fw + src * 9 + t;
        if (fb >= 0) blk[288 + (n & 31)].a = fb + src;
      }
      b.dwffn = prog.add(v);
    } else {
      std::vector<PEx> v((size_t)9 * 2 * hidS), vb((size_t)2 * hidS);
      for (int n = 0; n < 2 * hidS; ++n) {
        const int src = rmap(n);
        if (src < 0) continue;
        for (int t = 0; t < 9; ++t) v[(size_t)t * 2 * hidS + n].a = fw + src * 9 + t;
        if (fb >= 0) vb[n].a = fb + src;
      }
      b.dwffn = prog.add(v);
      if (fb >= 0) b.dwffn_b = prog.add(vb);
    }
    b.pout = pointwise(p + ".ffn.project_out", C, hid, hidS, C, [](int n) { return n; }, "", c.bias, false);
    b.pout.has_res = true;  // x += project_out(...) (unfused path)
    choose_variant(b.pout, false);
    // attention output + FFN input in one pass where project_in is one resident weight group
    // (C = 48); debug flag no_attn_in_fusion keeps the two GEMMs (bit-identity test)
    const bool no_ai = debug_flag("no_attn_in_fusion");
    b.fused_attn_in = b.pin.group_tiles >= b.pin.ntiles && b.pin.KG == C / 16 && b.pin.WPE == 2 &&
                      gemm_attn_in_variant(b.pin.NT, b.pin.KG, (b.pin.ntiles + b.pin.NT - 1) / b.pin.NT) && !no_ai;
    // (gemm_attn_in_variant also checks that the variant's weights + M fit the LDS)
    // C = 96 (two weight groups): the fused kernel on group 0 + a plain LN GEMM on group 1.  A wash in
    // r02 (profiles/r02_attn_in_probe.txt); since r04's fused-kernel waitcnt fix and XCD-paired GEMM
    // order -4.2% at 512^2 and -2.7% at 256^2 per block (profiles/r04k_attn_in_split_ab_probe.txt), so on
    // by default; debug flag no_attn_in_split keeps the unfused pair (bit-identity test)
    if (!b.fused_attn_in && !no_ai && !debug_flag("no_attn_in_split") && b.pin.group_tiles > 0 &&
        b.pin.group_tiles < b.pin.ntiles && 2 * b.pin.group_tiles >= b.pin.ntiles && b.pin.KG == C / 16 &&
        b.pin.WPE == 2 && gemm_attn_in_variant(b.pin.NT, b.pin.KG, (b.pin.group_tiles + b.pin.NT - 1) / b.pin.NT)) {
      const int gt = b.pin.group_tiles;
      b.pin_g0 = b.pin;
      b.pin_g0.ntiles = gt;
      b.pin_g0.N = 16 * gt;
      b.pin_g0.n_true = (int)((long long)b.pin.n_true * gt / b.pin.ntiles);
      b.pin_g1 = b.pin;
      b.pin_g1.w = b.pin.w + (size_t)gt * b.pin.kgroups * 256;
      b.pin_g1.w3 = b.pin.w3 + (size_t)split3_floats(gt, b.pin.kgroups);
      if (b.pin.bias != kNone) b.pin_g1.bias = b.pin.bias + (size_t)16 * gt;
      b.pin_g1.ntiles = b.pin.ntiles - gt;
      b.pin_g1.N = b.pin.N - 16 * gt;
      b.pin_g1.n_true = b.pin.n_true - b.pin_g0.n_true;
      b.pin_g1.group_tiles = b.pin_g1.ntiles;
      b.fused_attn_in = b.attn_in_split = true;
    }
    b.ffn_fused = b.fused_gdfn && ffn_fused_supported(C, hidS) && b.pin.ntiles == 2 * hidS / 16 &&
                  !debug_flag("no_ffn_fusion");
    // opt-in (debug flag mdta_fusion): r06 measured it slower than the qkv GEMM + Gram ring it replaces
    // (C96@512^2 3.54 vs 3.41 ms, C48@1024^2 5.93 vs 5.29 ms; DESIGN.md §4 "Fused MDTA pass 1")
    b.mdta_fused = heads == 1 && (C == 48 || C == 96) && b.qkv.ntiles == 3 * C / 16 && debug_flag("mdta_fusion");
    return b;
  }

  std::vector<BlockW> stage(const std::string& n, int cnt, int C, int heads) {
    std::vector<BlockW> v;
    for (int i = 0; i < cnt; ++i) v.push_back(block(n + "." + std::to_string(i), C, heads));
    return v;
  }
};

// ----------------------------------------------------------------------------- workspace plan
struct Plan {
  size_t total = 0;
  size_t catL1, catL2, catL3, lat, dec3, dec2, out4, refo, cenb, srs;
  size_t qkv, vbuf, fpre, fg, stats, part, red, Mp;
  size_t take(size_t floats) {
    size_t off = total;
    total += (floats * 4 + 255) / 256 * 256;
    return off;
  }
};

// Partial Gram slots per (image, head).  The slot partition depends on the image size only, never on
// the batch: image i of a batch then sums its Gram in exactly the order it does alone (bit-identical
// batch invariance).  Row-sweep kernel (W % 16 == 0): 16-column strips x at most 8 row segments of
// at least 32 rows (512^2: 64 rows, the 2-row halo costs 3%; 1024^2: 128 rows; 4 and 16 segments
// measured no better, profiles/r02_gram_nseg_probe.txt); generic kernel: 64-pixel steps grouped 16
// per slot.
constexpr auto KDLAE_T_DOWN_LDS = 1;  // Downsample convs on conv_lds (0: the implicit GEMM)
constexpr auto KDLAE_T_UP_LDS = 1;  // Upsample convs on conv_lds (0: the implicit GEMM)
constexpr int kGramMaxSeg = 8, kGramMinRows = 32;  // Gram slots: row segments per strip, rows per segment
static int nslots_for(int H, int W, int /*B*/, int /*heads*/) {
  if (W % 16 == 0) {
    const int strips = W / 16;
    const int nseg = std::max(1, std::min(kGramMaxSeg, (H + kGramMinRows - 1) / kGramMinRows));
    return strips * nseg;
  }
  const int steps = (H * W + 63) / 64;
  int n = (steps + 15) / 16;
  return std::max(1, std::min(64, n));
}

static Plan make_plan(const kdlae_t_handle* h, int B, int H, int W) {
  const kdlae_t_config& c = h->cfg;
  const long long d = c.dim;
  const long long P1 = (long long)B * H * W, P2 = P1 / 4, P3 = P1 / 16, P4 = P1 / 64, Psr = 4 * P1;
  Plan pl;
  pl.catL1 = pl.take(P1 * 2 * d);
  pl.catL2 = pl.take(P2 * 4 * d);
  pl.catL3 = pl.take(P3 * 8 * d);
  pl.lat = pl.take(P4 * 8 * d);
  pl.dec3 = pl.take(P3 * 4 * d);
  pl.dec2 = pl.take(P2 * 2 * d);
  pl.out4 = pl.take(P1 * 4);
  pl.refo = pl.take(P1 * 2 * d);
  pl.cenb = c.static_train ? pl.take(P1 * 2 * d) : 0;
  pl.srs = c.static_train ? pl.take(Psr * d) : 0;
  // per-block scratch: max over every stage that runs
  long long mq = 0, mv = 0, mfp = 0, mfg = 0, mst = 0, mpart = 0, mred = 0, mM = 0;
  auto acc = [&](const std::vector<BlockW>& st, long long P, int Hh, int Ww) {
    for (const BlockW& b : st) {
      const int CT = b.Ch / 16;
      const long long slot = (long long)CT * CT * 256 + 2 * b.Ch;
      mq = std::max(mq, P * 3 * b.C);
      mv = std::max(mv, P * b.C);
      mfp = std::max(mfp, P * 2 * b.hidS);
      if (!b.fused_gdfn) mfg = std::max(mfg, P * b.hidS);  // gated tensor: unfused FFN tails only
      mst = std::max(mst, P * 2);
      mpart = std::max(mpart, (long long)B * b.heads * nslots_for(Hh, Ww, B, b.heads) * slot);
      mred = std::max(mred, (long long)B * b.heads * slot);
      mM = std::max(mM, (long long)B * split3_floats(b.C / 16, b.C / 16));
    }
  };
  acc(h->enc1, P1, H, W);
  acc(h->enc2, P2, H / 2, W / 2);
  acc(h->enc3, P3, H / 4, W / 4);
  acc(h->latent, P4, H / 8, W / 8);
  acc(h->dec3, P3, H / 4, W / 4);
  acc(h->dec2, P2, H / 2, W / 2);
  acc(h->dec1, P1, H, W);
  acc(h->refinement, P1, H, W);
  acc(h->refinement_out, P1, H, W);
  acc(h->enhance, Psr, 2 * H, 2 * W);
  pl.qkv = pl.take(mq);
  pl.vbuf = pl.take(mv);
  pl.fpre = pl.take(mfp);
  pl.fg = pl.take(mfg);
  pl.stats = pl.take(mst);
  pl.part = pl.take(mpart);
  pl.red = pl.take(mred);
  pl.Mp = pl.take(mM);
  return pl;
}

// ----------------------------------------------------------------------------- forward
struct Fwd {
  kdlae_t_handle* h;
  hipStream_t s;
  char* ws;
  Plan pl;
  int B;

  float* buf(size_t off) { return reinterpret_cast<float*>(ws + off); }

  bool probing(int cls, int C) const {
    return h->probe_class == cls && (h->probe_level == 0 || h->probe_level == C);
  }
  int probe_begin(int cls, int C) {
    if (!probing(cls, C)) return KDLAE_OK;
    if (h->ev_used + 2 > h->ev.size()) {
      for (int i = 0; i < 256; ++i) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        h->ev.push_back(e);
      }
    }
    HIPCHK(hipEventRecord(h->ev[h->ev_used], s));
    return KDLAE_OK;
  }
  std::string tag;  // layer label of the launch being probed (per-launch dump)
  int probe_end(int cls, int C, double bytes, double flops) {
    if (!probing(cls, C)) return KDLAE_OK;
    HIPCHK(hipEventRecord(h->ev[h->ev_used + 1], s));
    h->ev_used += 2;
    h->probe_bytes += bytes;
    h->probe_flops += flops;
    h->probe_launches += 1;
    h->probe_recs.push_back({tag, bytes, flops});
    return KDLAE_OK;
  }

  // GEMM launch on views (probe-wrapped)
  int gemm(const Gemm& g, const float* W, long long w_img_stride, View in, int Hh, int Ww, View out,
           int out_mode, const float* R, int ldr, int ln, int ln_C, int probeC) {
    const int HW = Hh * Ww;
    GemmCall c;
    c.g = &g;
    c.W = W;
    c.w_img_stride = w_img_stride;
    c.bias = h->P(g.bias);
    c.in = in;
    c.out = out;
    c.B = B;
    c.F = 1;
    c.H = Hh;
    c.Wd = Ww;
    c.out_mode = out_mode;
    c.R = R;
    c.ldr = ldr;
    c.ln = ln;
    c.ln_C = ln_C;
    c.stats_buf = buf(pl.stats);
    int rc = probe_begin(1, probeC);
    if (rc) return rc;
    // the Downsample convs (3x3, PixelUnshuffle store) on the LDS-tiled conv (conv_lds.hip): the
    // implicit GEMM gathers every input pixel through L1 for each of the 9 taps and, with 24..96
    // outputs, feeds each gathered fragment to only 2..6 MFMAs
    const bool lds_conv = g.ksize == 3 && ((KDLAE_T_DOWN_LDS && out_mode == 1) || (KDLAE_T_UP_LDS && out_mode == 2)) &&
                          !R && !ln && conv_lds_supported(1, g.ntiles, g.cg_per_tap * 16);
    if (h->probe_class == 1)
      tag = "gemm C" + std::to_string(probeC) + " HW" + std::to_string(HW) + " N" + std::to_string(g.n_true) + " K" +
            std::to_string(g.k_true) + " k" + std::to_string(g.ksize) +
            (lds_conv ? std::string(" conv_lds") : " v" + std::to_string(g.NT) + "x" + std::to_string(g.KG) +
                                                       (g.group_tiles ? "r" : "c") + "w" + std::to_string(g.WPE)) +
            (ln ? " ln" : "") + (R ? " res" : "");
    if (lds_conv) {
      ConvLdsParams q{};
      q.in = in.p;
      q.ldi = in.ld;
      q.cin_pad = g.cg_per_tap * 16;
      q.wp = h->P(g.w);
      q.wp3 = W;
      q.ntiles = g.ntiles;
      q.kgroups = g.kgroups;
      q.bias = h->P(g.bias);
      q.out = out.p;
      q.ldo = out.ld;
      q.Bn = B;
      q.F = 1;
      q.H = Hh;
      q.W = Ww;
      q.kt = 1;
      q.relu = 0;
      q.out_mode = out_mode;
      q.nout = g.n_true;
      HIPCHK(launch_conv_lds(q, s));
    } else if ((rc = run_gemm(c, s))) {
      return rc;
    }
    const double P = (double)B * HW;
    const double kin = g.ksize == 3 ? g.k_true / 9.0 : g.k_true;
    const double bytes = 4.0 * (P * kin + P * g.n_true * (R ? 2.0 : 1.0) + (double)g.n_true * g.k_true);
    return probe_end(1, probeC, bytes, 2.0 * P * g.n_true * g.k_true);
  }

  // One TransformerBlock (:159-163) in place on x, or — with ffn (b.ffn_fused) — its attention half in
  // place and its feed-forward half from x into *ffn (which must not overlap x).
  int block(const BlockW& b, View x, int Hh, int Ww, const View* ffn = nullptr) {
    const int HW = Hh * Ww;
    const int ln = h->cfg.layernorm_biasfree ? 1 : 2;
    const long long P = (long long)B * HW;
    int rc;
    // --- attention
    const int nslots = nslots_for(Hh, Ww, B, b.heads);
    const int nseg = Ww % 16 == 0 ? nslots / (Ww / 16) : 0;
    const int seg_rows = nseg ? (Hh + nseg - 1) / nseg : 0;
    if (b.mdta_fused && mdta_fused_supported(b.C, b.heads, Hh, Ww, nseg, seg_rows)) {
      // LN + qkv + dwconv + Gram in one pass (mdta_fused.hip): qkv never reaches HBM
      const int CT = b.Ch / 16;
      MdtaFusedParams q{};
      q.x = x.p;
      q.ldx = x.ld;
      q.ln = ln;
      q.Wqkv = h->P3(b.qkv.w3);
      q.bias = h->P(b.qkv.bias);
      q.wdw = h->P(b.dwqkv);
      q.bdw = h->P(b.dwqkv_b);
      q.v_out = buf(pl.vbuf);
      q.ldv = b.C;
      q.partial = buf(pl.part);
      q.nslots = nslots;
      q.slot_floats = CT * CT * 256 + 2 * b.Ch;
      q.nseg = nseg;
      q.seg_rows = seg_rows;
      q.Bn = B;
      q.H = Hh;
      q.W = Ww;
      if ((rc = probe_begin(2, b.C))) return rc;
      tag = "mdta_fused C" + std::to_string(b.C) + " HW" + std::to_string(HW);
      HIPCHK(launch_mdta_fused(q, b.C, s));
      // algorithmic: read x, write v; qkv projection, dwconv and Gram FLOPs
      if ((rc = probe_end(2, b.C, 4.0 * P * 2 * b.C,
                          2.0 * P * (3.0 * b.C * b.C + 27.0 * b.C + (double)b.C * b.Ch))))
        return rc;
      HIPCHK(launch_gram_reduce(q.partial, buf(pl.red), B, b.heads, nslots, q.slot_floats, s));
      HIPCHK(launch_attn_fold(buf(pl.red), q.slot_floats, h->P(b.proj), h->P(b.temp), buf(pl.Mp), B, b.C, b.heads, s));
    } else {
    View qkv{buf(pl.qkv), 3 * b.C};
    rc = gemm(b.qkv, h->P3(b.qkv.w3), 0, x, Hh, Ww, qkv, 0, nullptr, 0, ln, b.C, b.C);
    if (rc) return rc;
    GramParams gp{};
    gp.qkv = qkv.p;
    gp.ld = qkv.ld;
    gp.wdw = h->P(b.dwqkv);
    gp.bdw = h->P(b.dwqkv_b);
    gp.v_out = buf(pl.vbuf);
    gp.ldv = b.C;
    gp.partial = buf(pl.part);
    gp.C = b.C;
    gp.heads = b.heads;
    gp.Ch = b.Ch;
    gp.Bn = B;
    gp.H = Hh;
    gp.W = Ww;
    gp.nslots = nslots;
    gp.zeros = h->P(h->zeros);
    const int CT = b.Ch / 16;
    gp.slot_floats = CT * CT * 256 + 2 * b.Ch;
    if ((rc = probe_begin(2, b.C))) return rc;
    tag = "gram C" + std::to_string(b.C) + " Ch" + std::to_string(b.Ch) + " HW" + std::to_string(HW);
    HIPCHK(launch_dwconv_gram(gp, s));
    if ((rc = probe_end(2, b.C, 4.0 * P * 4 * b.C, 2.0 * P * (27.0 * b.C + (double)b.C * b.Ch)))) return rc;
    HIPCHK(launch_gram_reduce(gp.partial, buf(pl.red), B, b.heads, gp.nslots, gp.slot_floats, s));
    HIPCHK(launch_attn_fold(buf(pl.red), gp.slot_floats, h->P(b.proj), h->P(b.temp), buf(pl.Mp), B, b.C, b.heads, s));
    }
    View fpre{buf(pl.fpre), 2 * b.hidS};
    const bool fuse_in = b.fused_attn_in && !ffn;
    if (fuse_in) {
      // x1 = x + M v written back into x, LN(x1) -> project_in into fpre, one kernel
      const Gemm& g0 = b.attn_in_split ? b.pin_g0 : b.pin;
      GemmCall c;
      c.g = &g0;
      c.W = h->P3(g0.w3);
      c.bias = h->P(g0.bias);
      c.in = View{buf(pl.vbuf), b.C};
      c.out = fpre;
      c.B = B;
      c.F = 1;
      c.H = Hh;
      c.Wd = Ww;
      c.R = x.p;
      c.ldr = x.ld;
      c.ln = ln;
      c.ln_C = b.C;
      c.stats_buf = buf(pl.stats);
      c.Wm = buf(pl.Mp);
      c.wm_img_stride = split3_floats(b.C / 16, b.C / 16);
      c.bias_m = h->P(b.proj_b);
      c.out1 = x;
      if ((rc = probe_begin(1, b.C))) return rc;
      if (h->probe_class == 1)
        tag = "gemm C" + std::to_string(b.C) + " HW" + std::to_string(HW) + " N" + std::to_string(g0.n_true) +
              " K" + std::to_string(b.C) + " attn_out+ln+project_in v" + std::to_string(g0.NT) + "x" +
              std::to_string(g0.KG);
      if ((rc = run_gemm(c, s))) return rc;
      const double Pd = (double)P;
      // read v and x, write x1 and the project_in rows; M per image + W_in; both GEMMs' FLOPs
      const double bytes = 4.0 * (Pd * 3.0 * b.C + Pd * g0.n_true + (double)B * b.C * b.C +
                                  (double)g0.n_true * b.C);
      if ((rc = probe_end(1, b.C, bytes, 2.0 * Pd * ((double)b.C * b.C + (double)b.C * g0.n_true)))) return rc;
      if (b.attn_in_split) {  // project_in's second weight group on x1 (now in x)
        rc = gemm(b.pin_g1, h->P3(b.pin_g1.w3), 0, x, Hh, Ww, View{fpre.p + 16 * b.pin_g0.ntiles, fpre.ld}, 0, nullptr,
                  0, ln, b.C, b.C);
        if (rc) return rc;
      }
    } else {
      rc = gemm(b.proj_gemm, buf(pl.Mp), split3_floats(b.C / 16, b.C / 16), View{buf(pl.vbuf), b.C}, Hh, Ww, x, 0,
                x.p, x.ld, 0,
                0, b.C);
      if (rc) return rc;
    }
    // --- feed-forward
    if ((rc = tap(x, b.C, Hh, Ww))) return rc;  // x1 (diagnostics only)
    if (ffn) {
      FfnParams q{};
      q.x = x.p;
      q.ldx = x.ld;
      q.out = ffn->p;
      q.ldo = ffn->ld;
      q.ln = ln;
      q.hidS = b.hidS;
      q.Win = h->P3(b.pin.w3);
      q.bias_in = h->P(b.pin.bias);
      q.dw = h->P(b.dwffn);
      q.Wout = h->P3(b.pout.w3);
      q.bias_out = h->P(b.pout.bias);
      q.Bn = B;
      q.H = Hh;
      q.W = Ww;
      if ((rc = probe_begin(3, b.C))) return rc;
      tag = "ffn C" + std::to_string(b.C) + " hid" + std::to_string(b.hid) + " HW" + std::to_string(HW);
      HIPCHK(launch_ffn_fused(q, b.C, s));
      // algorithmic: read x1, write the block output; project_in, dwconv + gate, project_out FLOPs
      return probe_end(3, b.C, 4.0 * P * 2.0 * b.C,
                       2.0 * P * ((double)b.C * 2.0 * b.hid + 18.0 * b.hid + (double)b.hid * b.C));
    }
    if (!fuse_in) {
      rc = gemm(b.pin, h->P3(b.pin.w3), 0, x, Hh, Ww, fpre, 0, nullptr, 0, ln, b.C, b.C);
      if (rc) return rc;
    }
    if (b.fused_gdfn) {
      GdfnParams gd{};
      gd.x = fpre.p;
      gd.ld = fpre.ld;
      gd.hidS = b.hidS;
      gd.dw = h->P(b.dwffn);
      gd.Wp = h->P3(b.pout.w3);
      gd.bias = h->P(b.pout.bias);
      gd.R = x.p;
      gd.ldr = x.ld;
      gd.out = x.p;
      gd.ldo = x.ld;
      gd.Bn = B;
      gd.H = Hh;
      gd.W = Ww;
      gd.zeros = h->P(h->zeros);
      if ((rc = probe_begin(3, b.C))) return rc;
      tag = "gdfn C" + std::to_string(b.C) + " hid" + std::to_string(b.hid) + " HW" + std::to_string(HW);
      HIPCHK(launch_gdfn_out(gd, b.C, s));
      // algorithmic: read x1|x2 (2 hid) + residual (C), write C; dwconv + gate + project_out FLOPs
      return probe_end(3, b.C, 4.0 * P * (2.0 * b.hid + 2.0 * b.C),
                       2.0 * P * (18.0 * b.hid + (double)b.hid * b.C));
    }
    GateParams ga{};
    ga.x = fpre.p;
    ga.ld = fpre.ld;
    ga.hidS = b.hidS;
    ga.w = h->P(b.dwffn);
    ga.b = h->P(b.dwffn_b);
    ga.out = buf(pl.fg);
    ga.ldo = b.hidS;
    ga.Bn = B;
    ga.H = Hh;
    ga.W = Ww;
    if ((rc = probe_begin(3, b.C))) return rc;
    tag = "gate C" + std::to_string(b.C) + " hid" + std::to_string(b.hid) + " HW" + std::to_string(HW);
    HIPCHK(launch_dwconv_gate(ga, s));
    if ((rc = probe_end(3, b.C, 4.0 * P * 3 * b.hid, 2.0 * P * 18.0 * b.hid))) return rc;
    return gemm(b.pout, h->P3(b.pout.w3), 0, View{buf(pl.fg), b.hidS}, Hh, Ww, x, 0, x.p, x.ld, 0, 0, b.C);
  }

  // kdlae_t_debug_taps: taps passed so far in this forward; the order is tap_list's (per stage: its
  // input, then per block the attention half's output x1 and the block output)
  size_t tap_i = 0;
  int tap(View x, int C, int Hh, int Ww) {
    const size_t i = tap_i++;
    if (i < h->taps.size() && h->taps[i]) {
      const size_t P = (size_t)B * Hh * Ww;
      HIPCHK(hipMemcpy2DAsync(h->taps[i], (size_t)C * 4, x.p, (size_t)x.ld * 4, (size_t)C * 4, P,
                              hipMemcpyDeviceToDevice, s));
    }
    return KDLAE_OK;
  }
  // A stage whose blocks all take the fused feed-forward half (an even count) ping-pongs between x and
  // T = the project_in scratch (unused by the fused blocks), so its output lands in x.
  int stage(const std::vector<BlockW>& st, View x, int Hh, int Ww) {
    if (st.empty()) return KDLAE_OK;
    int rc = tap(x, st[0].C, Hh, Ww);
    if (rc) return rc;
    bool fused = st.size() % 2 == 0;
    for (const BlockW& b : st) fused = fused && b.ffn_fused;
    const View T{buf(pl.fpre), st[0].C};
    View cur = x;
    for (size_t i = 0; i < st.size(); ++i) {
      const BlockW& b = st[i];
      if (fused) {
        const View nxt = (i % 2 == 0) ? T : x;
        if ((rc = block(b, cur, Hh, Ww, &nxt))) return rc;
        cur = nxt;
      } else {
        if ((rc = block(b, x, Hh, Ww))) return rc;
      }
      if ((rc = tap(cur, b.C, Hh, Ww))) return rc;
    }
    return KDLAE_OK;
  }

  int small_in(const SmallW& w, const float* in, long long sb, long long sc, long long sy, long long sx, int Hh,
               int Ww, View out, int dil) {
    SmallInParams p{};
    p.in = in;
    p.sb = sb;
    p.sc = sc;
    p.sy = sy;
    p.sx = sx;
    p.Cin = w.Cin;
    p.Cout = w.Cout;
    p.dil = dil;
    p.w = h->P(w.w);
    p.bias = h->P(w.bias);
    p.out = out.p;
    p.ldo = out.ld;
    p.Bn = B;
    p.H = Hh;
    p.W = Ww;
    p.F = 1;
    p.kt = 1;
    p.st = 0;
    p.relu = 0;
    HIPCHK(launch_conv_small_in(p, s));
    return KDLAE_OK;
  }

  int small_out(const SmallW& w, View in, int Hh, int Ww, float* out, int nchw, int ldo, const float* res,
                const float* extra) {
    SmallOutParams p{};
    p.in = in.p;
    p.ld = in.ld;
    p.Cin = w.Cin;
    p.Cout = w.Cout;
    p.w = h->P(w.w);
    p.bias = h->P(w.bias);
    p.Bn = B;
    p.H = Hh;
    p.W = Ww;
    p.F = 1;
    p.ks = 3;
    p.out = out;
    p.out_nchw = nchw;
    p.ldo = ldo;
    p.res = res;
    p.extra = extra;
    HIPCHK(launch_conv_small_out(p, s));
    return KDLAE_OK;
  }

  int run(const float* img, const float* rate, int H, int W, float* hq, float* sr) {
    const kdlae_t_config& c = h->cfg;
    const int d = c.dim;
    int rc;
    const int H2 = H / 2, W2 = W / 2, H3 = H / 4, W3 = W / 4, H4 = H / 8, W4 = W / 8;
    float* L1 = buf(pl.catL1);
    float* L2 = buf(pl.catL2);
    float* L3 = buf(pl.catL3);
    View e1{L1 + d, 2 * d}, e2{L2 + 2 * d, 4 * d}, e3{L3 + 4 * d, 8 * d}, lat{buf(pl.lat), 8 * d};
    const long long HW = (long long)H * W;
    const int ci = c.inp_channels;
    // patch_embed (:275) from NCHW img into the level-1 concat buffer's second half
    if ((rc = small_in(h->patch_embed, img, ci * HW, HW, W, 1, H, W, e1, 1))) return rc;
    if ((rc = stage(h->enc1, e1, H, W))) return rc;
    if ((rc = gemm(h->down1_2, h->P3(h->down1_2.w3), 0, e1, H, W, e2, 1, nullptr, 0, 0, 0, -1))) return rc;
    if ((rc = stage(h->enc2, e2, H2, W2))) return rc;
    if ((rc = gemm(h->down2_3, h->P3(h->down2_3.w3), 0, e2, H2, W2, e3, 1, nullptr, 0, 0, 0, -1))) return rc;
    if ((rc = stage(h->enc3, e3, H3, W3))) return rc;
    if ((rc = gemm(h->down3_4, h->P3(h->down3_4.w3), 0, e3, H3, W3, lat, 1, nullptr, 0, 0, 0, -1))) return rc;
    if ((rc = stage(h->latent, lat, H4, W4))) return rc;
    // decoder level 3 (:288-291)
    if ((rc = gemm(h->up4_3, h->P3(h->up4_3.w3), 0, lat, H4, W4, View{L3, 8 * d}, 2, nullptr, 0, 0, 0, -1))) return rc;
    View d3{buf(pl.dec3), 4 * d};
    if ((rc = gemm(h->reduce3, h->P3(h->reduce3.w3), 0, View{L3, 8 * d}, H3, W3, d3, 0, nullptr, 0, 0, 0, -1))) return rc;
    if ((rc = stage(h->dec3, d3, H3, W3))) return rc;
    // decoder level 2 (:293-296)
    if ((rc = gemm(h->up3_2, h->P3(h->up3_2.w3), 0, d3, H3, W3, View{L2, 4 * d}, 2, nullptr, 0, 0, 0, -1))) return rc;
    View d2{buf(pl.dec2), 2 * d};
    if ((rc = gemm(h->reduce2, h->P3(h->reduce2.w3), 0, View{L2, 4 * d}, H2, W2, d2, 0, nullptr, 0, 0, 0, -1))) return rc;
    if ((rc = stage(h->dec2, d2, H2, W2))) return rc;
    // decoder level 1 + refinement (:298-302), in place on the full 2d-channel concat buffer
    if ((rc = gemm(h->up2_1, h->P3(h->up2_1.w3), 0, d2, H2, W2, View{L1, 2 * d}, 2, nullptr, 0, 0, 0, -1))) return rc;
    View d1{L1, 2 * d};
    if ((rc = stage(h->dec1, d1, H, W))) return rc;
    if ((rc = stage(h->refinement, d1, H, W))) return rc;
    const int co = c.out_channels;
    if (c.params_cat) {
      // output (:314) + cat denoise_rate (:316) -> output_param dil 2 (:317) -> refinement_out -> output2 + img
      float* o4 = buf(pl.out4);
      if ((rc = small_out(h->output, d1, H, W, o4, 0, 4, nullptr, rate))) return rc;
      View ro{buf(pl.refo), 2 * d};
      if ((rc = small_in(h->output_param, o4, 4 * HW, 1, 4LL * W, 4, H, W, ro, 2))) return rc;
      if ((rc = stage(h->refinement_out, ro, H, W))) return rc;
      if ((rc = small_out(h->output2, ro, H, W, hq, 1, 0, img, nullptr))) return rc;
    } else {
      if ((rc = small_out(h->output, d1, H, W, hq, 1, 0, img, nullptr))) return rc;
    }
    if (c.static_train) {
      // sr head on the UNclamped hq (:326-329)
      View cb{buf(pl.cenb), 2 * d};
      if ((rc = small_in(h->cen, hq, co * HW, HW, W, 1, H, W, cb, 1))) return rc;
      View sv{buf(pl.srs), d};
      if ((rc = gemm(h->upen, h->P3(h->upen.w3), 0, cb, H, W, sv, 2, nullptr, 0, 0, 0, -1))) return rc;
      if ((rc = stage(h->enhance, sv, 2 * H, 2 * W))) return rc;
      if ((rc = small_out(h->outputen, sv, 2 * H, 2 * W, sr, 1, 0, nullptr, nullptr))) return rc;
    }
    return KDLAE_OK;
  }
};

}  // namespace kdlae

// ============================================================================= C ABI
extern "C" {

const char* kdlae_last_error(void) { return kdlae::g_err.c_str(); }
int kdlae_abi_version(void) { return 1; }

int kdlae_t_create(const kdlae_t_config* cfg, int device, kdlae_t_handle** out) {
  if (!cfg || !out) return fail(KDLAE_ESTATE, "null argument");
  *out = nullptr;
  int rc = validate(*cfg);
  if (rc) return rc;
  auto* h = new kdlae_t_handle();
  h->cfg = *cfg;
  h->device = device;
  build_keys(h);
  *out = h;
  return KDLAE_OK;
}

int kdlae_t_destroy(kdlae_t_handle* h) {
  if (!h) return KDLAE_OK;
  {
    DeviceGuard g(h->device);
    h->dw.release();
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
  }
  delete h;
  return KDLAE_OK;
}

int kdlae_t_num_params(const kdlae_t_handle* h) { return h ? (int)h->ps.keys.size() : 0; }

int kdlae_t_param_info(const kdlae_t_handle* h, int index, const char** name, int64_t* numel) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  return h->ps.info(index, name, numel);
}

int64_t kdlae_t_params_numel(const kdlae_t_handle* h) { return h ? h->ps.total : -1; }

int kdlae_t_set_param(kdlae_t_handle* h, const char* name, const float* host_data, int64_t numel) {
  if (!h || !name || !host_data) return fail(KDLAE_ESTATE, "null argument");
  return h->ps.set(name, host_data, numel);
}

}  // extern "C"

// Records the packed layout of this configuration (once per handle) and uploads the program.
static int build_program(kdlae_t_handle* h) {
  if (h->built) return KDLAE_OK;
  const kdlae_t_config& c = h->cfg;
  Packer pk{h};
  pk.prog.nsrc = h->ps.total;
  h->zeros = pk.prog.add(std::vector<PEx>(64));
  const int d = c.dim;
  const int* nb = c.num_blocks;
  const int* hd = c.heads;
  const int nr = c.num_refinement_blocks;
  h->patch_embed = pk.small("patch_embed.proj", d, c.inp_channels, false);
  h->enc1 = pk.stage("encoder_level1", nb[0], d, hd[0]);
  h->down1_2 = pk.conv3("down1_2.body.0", d / 2, d, 1);
  h->enc2 = pk.stage("encoder_level2", nb[1], 2 * d, hd[1]);
  h->down2_3 = pk.conv3("down2_3.body.0", d, 2 * d, 1);
  h->enc3 = pk.stage("encoder_level3", nb[2], 4 * d, hd[2]);
  h->down3_4 = pk.conv3("down3_4.body.0", 2 * d, 4 * d, 1);
  h->latent = pk.stage("latent", nb[3], 8 * d, hd[3]);
  h->up4_3 = pk.conv3("up4_3.body.0", 16 * d, 8 * d, 2);
  h->reduce3 = pk.pointwise("reduce_chan_level3", 4 * d, 8 * d, 8 * d, 4 * d, [](int n) { return n; }, "", c.bias, false);
  h->dec3 = pk.stage("decoder_level3", nb[2], 4 * d, hd[2]);
  h->up3_2 = pk.conv3("up3_2.body.0", 8 * d, 4 * d, 2);
  h->reduce2 = pk.pointwise("reduce_chan_level2", 2 * d, 4 * d, 4 * d, 2 * d, [](int n) { return n; }, "", c.bias, false);
  h->dec2 = pk.stage("decoder_level2", nb[1], 2 * d, hd[1]);
  h->up2_1 = pk.conv3("up2_1.body.0", 4 * d, 2 * d, 2);
  h->dec1 = pk.stage("decoder_level1", nb[0], 2 * d, hd[0]);
  h->refinement = pk.stage("refinement", nr, 2 * d, hd[0]);
  h->output = pk.small("output", c.out_channels, 2 * d, c.bias);
  h->output_param = pk.small("output_param", 2 * d, c.out_channels + 1, c.bias);
  h->refinement_out = pk.stage("refinement_out", nr, 2 * d, hd[0]);
  h->output2 = pk.small("output2", c.out_channels, 2 * d, c.bias);
  if (c.static_train) {
    const int hc = 2 * d;
    h->cen = pk.small("cen", hc, c.out_channels, c.bias);
    h->upen = pk.conv3("upen.body.0", 2 * hc, hc, 2);
    h->enhance = pk.stage("enhance", nr, hc / 2, hd[0]);
    h->outputen = pk.small("outputen", c.out_channels, hc / 2, c.bias);
  }
  if (pk.err) return pk.err;
  DeviceGuard g(h->device);
  int rc = h->dw.upload_program(pk.prog);
  if (rc) return rc;
  h->built = true;
  return KDLAE_OK;
}

extern "C" {

int kdlae_t_commit_params(kdlae_t_handle* h, void* stream) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  int rc = h->ps.check_complete();
  if (rc) return rc;
  if ((rc = build_program(h))) return rc;
  DeviceGuard g(h->device);
  if ((rc = h->dw.run_host(h->ps.flat(), reinterpret_cast<hipStream_t>(stream)))) return rc;
  h->committed = true;
  return KDLAE_OK;
}

int kdlae_t_prepare(kdlae_t_handle* h) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  return build_program(h);
}

int kdlae_t_pack_device(kdlae_t_handle* h, const float* params, int64_t numel, void* stream) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  if (numel != h->ps.total)
    return fail(KDLAE_EPARAM, "flat parameter vector has " + std::to_string(numel) + " floats, expected " +
                                  std::to_string(h->ps.total));
  int rc = build_program(h);
  if (rc) return rc;
  DeviceGuard g(h->device);
  if ((rc = h->dw.run(params, reinterpret_cast<hipStream_t>(stream)))) return rc;
  h->committed = true;
  return KDLAE_OK;
}

int64_t kdlae_t_workspace_bytes(const kdlae_t_handle* h, int B, int H, int W) {
  if (!h || !h->committed) {
    fail(KDLAE_ESTATE, "workspace_bytes needs committed params");
    return -1;
  }
  if (B <= 0 || H <= 0 || W <= 0 || H % 8 || W % 8) {
    fail(KDLAE_EINVAL_SHAPE, "B, H, W must be positive with H % 8 == 0 and W % 8 == 0");
    return -1;
  }
  return (int64_t)make_plan(h, B, H, W).total;
}

int kdlae_t_forward(kdlae_t_handle* h, const float* img, const float* rate, int B, int H, int W, float* hq,
                    float* sr, void* workspace, int64_t workspace_bytes, void* stream) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  if (!h->committed) return fail(KDLAE_ESTATE, "forward before kdlae_t_commit_params / kdlae_t_pack_device");
  if (B <= 0 || H <= 0 || W <= 0 || H % 8 || W % 8)
    return fail(KDLAE_EINVAL_SHAPE, "KDLAE_teacher needs H % 8 == 0 and W % 8 == 0 (pixel_unshuffle x3, KDLAE_model.py:187)");
  if (!img || !hq) return fail(KDLAE_ESTATE, "img and hq are required");
  if (h->cfg.params_cat && !rate) return fail(KDLAE_ESTATE, "denoise_rate is required when params=='cat'");
  if ((sr != nullptr) != (h->cfg.static_train != 0))
    return fail(KDLAE_ESTATE, "sr must be non-null iff static=='train'");
  Fwd f{h, reinterpret_cast<hipStream_t>(stream), reinterpret_cast<char*>(workspace), make_plan(h, B, H, W), B};
  if ((int64_t)f.pl.total > workspace_bytes) return fail(KDLAE_ESTATE, "workspace too small");
  DeviceGuard g(h->device);
  return f.run(img, rate, H, W, hq, sr);
}

// TransformerBlocks in the order kdlae_t_forward runs them: (state_dict prefix, channels, resolution
// relative to the input as num / den)
struct TapInfo { std::string name; int C, num, den; };
static std::vector<TapInfo> tap_list(const kdlae_t_handle* h) {
  const kdlae_t_config& c = h->cfg;
  const int d = c.dim, nr = c.num_refinement_blocks;
  std::vector<TapInfo> v;
  auto add = [&](const char* n, int cnt, int C, int num, int den) {
    if (cnt <= 0) return;
    v.push_back({std::string(n) + ".in", C, num, den});
    for (int i = 0; i < cnt; ++i) {
      v.push_back({std::string(n) + "." + std::to_string(i) + ".attn", C, num, den});
      v.push_back({std::string(n) + "." + std::to_string(i), C, num, den});
    }
  };
  add("encoder_level1", c.num_blocks[0], d, 1, 1);
  add("encoder_level2", c.num_blocks[1], 2 * d, 1, 2);
  add("encoder_level3", c.num_blocks[2], 4 * d, 1, 4);
  add("latent", c.num_blocks[3], 8 * d, 1, 8);
  add("decoder_level3", c.num_blocks[2], 4 * d, 1, 4);
  add("decoder_level2", c.num_blocks[1], 2 * d, 1, 2);
  add("decoder_level1", c.num_blocks[0], 2 * d, 1, 1);
  add("refinement", nr, 2 * d, 1, 1);
  if (c.params_cat) add("refinement_out", nr, 2 * d, 1, 1);
  if (c.static_train) add("enhance", nr, d, 2, 1);
  return v;
}

int kdlae_t_debug_tap_count(const kdlae_t_handle* h) { return h ? (int)tap_list(h).size() : -1; }

int kdlae_t_debug_tap_info(const kdlae_t_handle* h, int i, char* name, int name_len, int* C, int* num, int* den) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  const std::vector<TapInfo> v = tap_list(h);
  if (i < 0 || i >= (int)v.size()) return fail(KDLAE_EPARAM, "tap index out of range");
  if (name && name_len > 0) snprintf(name, (size_t)name_len, "%s", v[i].name.c_str());
  if (C) *C = v[i].C;
  if (num) *num = v[i].num;
  if (den) *den = v[i].den;
  return KDLAE_OK;
}

int kdlae_t_debug_taps(kdlae_t_handle* h, int n, float* const* dst) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  if (n < 0 || (n > 0 && !dst)) return fail(KDLAE_EPARAM, "bad tap list");
  h->taps.assign(dst, dst + n);
  return KDLAE_OK;
}

int kdlae_t_probe_arm(kdlae_t_handle* h, int kernel_class, int level_filter) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  h->probe_class = kernel_class;
  h->probe_level = level_filter;
  h->ev_used = 0;
  h->probe_bytes = h->probe_flops = 0;
  h->probe_launches = 0;
  h->probe_recs.clear();
  return KDLAE_OK;
}

int kdlae_t_probe_read(kdlae_t_handle* h, double* ms, int64_t* launches, double* bytes, double* flops) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  double tot = 0;
  const char* dump = getenv("KDLAE_PROBE_DUMP");  // optional per-launch CSV (tag, ms, bytes, flops)
  FILE* f = dump ? fopen(dump, "w") : nullptr;
  if (f) fprintf(f, "tag,ms,bytes,flops\n");
  for (size_t i = 0; i + 1 < h->ev_used; i += 2) {
    HIPCHK(hipEventSynchronize(h->ev[i + 1]));
    float m = 0;
    HIPCHK(hipEventElapsedTime(&m, h->ev[i], h->ev[i + 1]));
    tot += m;
    if (f && i / 2 < h->probe_recs.size()) {
      const auto& r = h->probe_recs[i / 2];
      fprintf(f, "%s,%.6f,%.0f,%.0f\n", r.tag.c_str(), m, r.bytes, r.flops);
    }
  }
  if (f) fclose(f);
  if (ms) *ms = tot;
  if (launches) *launches = h->probe_launches;
  if (bytes) *bytes = h->probe_bytes;
  if (flops) *flops = h->probe_flops;
  return KDLAE_OK;
}

}  // extern "C"
