// KDLAE-S host runtime (KDLAE/KDLAE_model.py:340-431): multi-frame 3-D U-Net on NDHWC views.
//
//   x [B, F, H, W]  (== [B, 1, F, H, W] NDHWC with C = 1, the unsqueeze(1) of :397)
//   encoders[i]  Conv3d 3x3x3 + bias + ReLU, twice (:386-393)   -> skip_i (kept)
//   MaxPool3d (1,2,2) (:366)
//   st_fusion    the same block at the deepest level (:411)
//   decoders     ConvTranspose3d (1,2,2) s (1,2,2) + bias (:378-379), + skip (:417), block (:418)
//   out_conv     1x1x1 + bias (:384, :422), + x if residual (:425-426), squeeze(1) (:429)
//
// Conv3d = implicit GEMM over 27 taps x Cin (MFMA f32, bias + ReLU in the epilogue); the first conv
// (Cin = 1) is a direct VALU conv.  ConvTranspose3d = a 1x1 GEMM with N = 4*Cout whose epilogue
// stores through the PixelShuffle map and adds the skip tensor in place.  Channel counts are padded
// to 16 with zero weights (ReLU keeps pad channels at 0).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "runtime.h"

using namespace kdlae;

struct kdlae_s_handle {
  kdlae_s_config cfg{};
  int device = 0;
  int L = 0;               // levels = len(hidden_channels) - 1
  std::vector<int> hc, cs;  // hidden channels, padded to 16
  ParamStore ps;
  bool built = false, committed = false;
  DeviceWeights dw;        // packed arena + the pack program that fills it from the parameters
  struct Block { Gemm a, b; };
  SmallW first;             // encoders.0.0 (Cin = 1), stored padded [cs0][27]
  std::vector<Block> enc, dec;
  Block fusion;
  std::vector<Gemm> up;
  SmallW outc;              // out_conv, stored padded [1][cs0]
};

namespace {

struct SPlan {
  size_t total = 0;
  std::vector<size_t> skip;
  size_t tA = 0, tB = 0;
  size_t take(long long floats) {
    size_t off = total;
    total += ((size_t)floats * 4 + 255) / 256 * 256;
    return off;
  }
};

SPlan make_splan(const kdlae_s_handle* h, int B, int F, int H, int W) {
  SPlan pl;
  long long mx = 0;
  for (int i = 0; i < h->L; ++i) {
    const long long P = (long long)B * F * (H >> i) * (W >> i);
    pl.skip.push_back(pl.take(P * h->cs[i]));
  }
  int cmax = 0;
  for (int c : h->cs) cmax = std::max(cmax, c);
  mx = (long long)B * F * H * W * cmax;
  pl.tA = pl.take(mx);
  pl.tB = pl.take(mx);
  return pl;
}

int validate_s(const kdlae_s_config& c) {
  if (c.inp_channels != 1 || c.out_channels != 1)
    return fail(KDLAE_EINVAL_CONFIG, "KDLAE_student forward unsqueezes a [B,F,H,W] input: inp/out_channels must be 1");
  if (c.kernel_size != 3) return fail(KDLAE_EINVAL_CONFIG, "kernel_size must be 3 on the HIP path");
  if (c.num_hidden < 2 || c.num_hidden > 8) return fail(KDLAE_EINVAL_CONFIG, "2..8 hidden_channels supported");
  for (int i = 0; i < c.num_hidden; ++i)
    if (c.hidden_channels[i] <= 0 || c.hidden_channels[i] > 512) return fail(KDLAE_EINVAL_CONFIG, "bad hidden_channels");
  return KDLAE_OK;
}

}  // namespace

extern "C" {

int kdlae_s_create(const kdlae_s_config* cfg, int device, kdlae_s_handle** out) {
  if (!cfg || !out) return fail(KDLAE_ESTATE, "null argument");
  *out = nullptr;
  int rc = validate_s(*cfg);
  if (rc) return rc;
  auto* h = new kdlae_s_handle();
  h->cfg = *cfg;
  h->device = device;
  h->L = cfg->num_hidden - 1;
  for (int i = 0; i < cfg->num_hidden; ++i) {
    h->hc.push_back(cfg->hidden_channels[i]);
    h->cs.push_back(ru16(cfg->hidden_channels[i]));
  }
  // state_dict keys in registration order (KDLAE_model.py:359-384)
  auto blk = [&](const std::string& p, int cin, int cout) {
    h->ps.add(p + ".0.weight", (int64_t)cout * cin * 27);
    h->ps.add(p + ".0.bias", cout);
    h->ps.add(p + ".2.weight", (int64_t)cout * cout * 27);
    h->ps.add(p + ".2.bias", cout);
  };
  int cin = cfg->inp_channels;
  for (int i = 0; i < h->L; ++i) {
    blk("encoders." + std::to_string(i), cin, h->hc[i]);
    cin = h->hc[i];
  }
  blk("st_fusion", cin, h->hc[h->L]);
  for (int j = 0, i = h->L - 1; i >= 0; --i, ++j) {
    const int cu = (i == h->L - 1) ? h->hc[h->L] : h->hc[i + 1];
    h->ps.add("upconv_layers." + std::to_string(j) + ".weight", (int64_t)cu * h->hc[i] * 4);
    h->ps.add("upconv_layers." + std::to_string(j) + ".bias", h->hc[i]);
  }
  for (int j = 0, i = h->L - 1; i >= 0; --i, ++j) blk("decoders." + std::to_string(j), h->hc[i], h->hc[i]);
  h->ps.add("out_conv.weight", (int64_t)cfg->out_channels * h->hc[0]);
  h->ps.add("out_conv.bias", cfg->out_channels);
  // the reference registers encoders, pooling, st_fusion, upconv_layers, decoders, out_conv in that
  // attribute order; state_dict() lists encoders.*, st_fusion.*, upconv_layers.*, decoders.*, out_conv.*
  *out = h;
  return KDLAE_OK;
}

int kdlae_s_destroy(kdlae_s_handle* h) {
  if (!h) return KDLAE_OK;
  {
    DeviceGuard g(h->device);
    h->dw.release();
  }
  delete h;
  return KDLAE_OK;
}

int kdlae_s_num_params(const kdlae_s_handle* h) { return h ? (int)h->ps.keys.size() : 0; }

int kdlae_s_param_info(const kdlae_s_handle* h, int index, const char** name, int64_t* numel) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  return h->ps.info(index, name, numel);
}

int64_t kdlae_s_params_numel(const kdlae_s_handle* h) { return h ? h->ps.total : -1; }

int kdlae_s_set_param(kdlae_s_handle* h, const char* name, const float* host_data, int64_t numel) {
  if (!h || !name || !host_data) return fail(KDLAE_ESTATE, "null argument");
  return h->ps.set(name, host_data, numel);
}

}  // extern "C"

// Records the packed layout (pack program, runtime.h) of this configuration once per handle.
static int build_program_s(kdlae_s_handle* h) {
  if (h->built) return KDLAE_OK;
  PackProgram ar;
  ar.nsrc = h->ps.total;
  int err = KDLAE_OK;
  auto conv3d = [&](const std::string& name, int cin, int cout) {
    const int32_t W = h->ps.base(name + ".weight", &err);
    const int32_t Bv = h->ps.base(name + ".bias", &err);
    Gemm g;
    if (err) return g;
    const int cis = ru16(cin), cos = ru16(cout);
    g.ksize = 3;
    g.kt = 3;
    g.cg_per_tap = cis / 16;
    g.ntiles = cos / 16;
    g.kgroups = 27 * cis / 16;
    g.N = cos;
    g.K = 27 * cis;
    g.n_true = cout;
    g.k_true = 27 * cin;
    g.w = ar.add(pack_fragments(g.ntiles, g.kgroups, [&](int n, int k) -> PEx {
      const int tap = k / cis, c = k - tap * cis;
      if (n >= cout || c >= cin) return PEx{};
      return PEx{W + (n * cin + c) * 27 + tap, -1};
    }));
    g.w3 = ar.split(g.w, g.ntiles, g.kgroups);
    if (conv_lds_supported(3, g.ntiles, cis)) {
      // conv_lds stages one 16-channel group of the 3-frame halo at a time and pairs consecutive taps
      // of that group: records of k-groups (group c, tap 2j) + (group c, tap 2j + 1), tap 27 = zeros,
      // i.e. split records of the fragment block in k-group order c * 28 + tap
      const int kg28 = 28 * (cis / 16);
      const size_t wt = ar.add(pack_fragments(g.ntiles, kg28, [&](int n, int k) -> PEx {
        const int kg = k / 16, grp = kg / 28, tap = kg - 28 * grp, c = 16 * grp + (k & 15);
        if (n >= cout || c >= cin || tap >= 27) return PEx{};
        return PEx{W + (n * cin + c) * 27 + tap, -1};
      }));
      g.w3t = ar.split(wt, g.ntiles, kg28);
    }
    std::vector<PEx> b((size_t)g.ntiles * 16);
    for (int n = 0; n < cout; ++n) b[n].a = Bv + n;
    g.bias = ar.add(b);
    choose_variant(g);
    return g;
  };
  // first conv: Cin = 1 direct kernel, weights padded to [cs0][27]
  {
    const int32_t W = h->ps.base("encoders.0.0.weight", &err);
    const int32_t Bv = h->ps.base("encoders.0.0.bias", &err);
    if (err) return err;
    const int c0 = h->hc[0], cs0 = h->cs[0];
    std::vector<PEx> w((size_t)cs0 * 27), b((size_t)cs0);
    for (int n = 0; n < c0; ++n) {
      for (int t = 0; t < 27; ++t) w[(size_t)n * 27 + t].a = W + n * 27 + t;
      b[n].a = Bv + n;
    }
    h->first.w = ar.add(w);
    h->first.bias = ar.add(b);
    h->first.Cout = cs0;
    h->first.Cin = 1;
  }
  h->enc.clear();
  h->dec.clear();
  h->up.clear();
  for (int i = 0; i < h->L; ++i) {
    kdlae_s_handle::Block bl;
    const std::string p = "encoders." + std::to_string(i);
    if (i > 0) bl.a = conv3d(p + ".0", h->hc[i - 1], h->hc[i]);
    bl.b = conv3d(p + ".2", h->hc[i], h->hc[i]);
    h->enc.push_back(bl);
  }
  h->fusion.a = conv3d("st_fusion.0", h->hc[h->L - 1], h->hc[h->L]);
  h->fusion.b = conv3d("st_fusion.2", h->hc[h->L], h->hc[h->L]);
  for (int j = 0, i = h->L - 1; i >= 0; --i, ++j) {
    const std::string p = "upconv_layers." + std::to_string(j);
    const int32_t W = h->ps.base(p + ".weight", &err);  // [cin][cout][1][2][2]
    const int32_t Bv = h->ps.base(p + ".bias", &err);
    if (err) return err;
    const int cin = (i == h->L - 1) ? h->hc[h->L] : h->hc[i + 1], cout = h->hc[i];
    const int cis = ru16(cin), cos = ru16(cout);
    Gemm g;
    g.ksize = 1;
    g.out_mode = 2;
    g.ntiles = 4 * cos / 16;
    g.kgroups = cis / 16;
    g.N = 4 * cos;
    g.K = cis;
    g.n_true = 4 * cout;
    g.k_true = cin;
    g.w = ar.add(pack_fragments(g.ntiles, g.kgroups, [&](int n, int k) -> PEx {
      const int c = n >> 2, ii = (n >> 1) & 1, jj = n & 1;
      if (c >= cout || k >= cin) return PEx{};
      return PEx{W + ((k * cout + c) * 2 + ii) * 2 + jj, -1};
    }));
    g.w3 = ar.split(g.w, g.ntiles, g.kgroups);
    std::vector<PEx> b((size_t)g.ntiles * 16);
    for (int n = 0; n < 4 * cos; ++n)
      if ((n >> 2) < cout) b[n].a = Bv + (n >> 2);
    g.bias = ar.add(b);
    choose_variant(g);
    h->up.push_back(g);
    kdlae_s_handle::Block bl;
    const std::string d = "decoders." + std::to_string(j);
    bl.a = conv3d(d + ".0", cout, cout);
    bl.b = conv3d(d + ".2", cout, cout);
    h->dec.push_back(bl);
  }
  {
    const int32_t W = h->ps.base("out_conv.weight", &err);
    const int32_t Bv = h->ps.base("out_conv.bias", &err);
    if (err) return err;
    std::vector<PEx> w((size_t)h->cs[0]);
    for (int c = 0; c < h->hc[0]; ++c) w[c].a = W + c;
    h->outc.w = ar.add(w);
    h->outc.bias = ar.copy(Bv, h->cfg.out_channels);
    h->outc.Cin = h->cs[0];
    h->outc.Cout = 1;
  }
  if (err) return err;
  DeviceGuard g(h->device);
  int rc = h->dw.upload_program(ar);
  if (rc) return rc;
  h->built = true;
  return KDLAE_OK;
}

extern "C" {

int kdlae_s_commit_params(kdlae_s_handle* h, void* stream) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  int rc = h->ps.check_complete();
  if (rc) return rc;
  if ((rc = build_program_s(h))) return rc;
  DeviceGuard g(h->device);
  if ((rc = h->dw.run_host(h->ps.flat(), reinterpret_cast<hipStream_t>(stream)))) return rc;
  h->committed = true;
  return KDLAE_OK;
}

int kdlae_s_prepare(kdlae_s_handle* h) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  return build_program_s(h);
}

int kdlae_s_pack_device(kdlae_s_handle* h, const float* params, int64_t numel, void* stream) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  if (numel != h->ps.total)
    return fail(KDLAE_EPARAM, "flat parameter vector has " + std::to_string(numel) + " floats, expected " +
                                  std::to_string(h->ps.total));
  int rc = build_program_s(h);  // no-op after kdlae_s_prepare
  if (rc) return rc;
  DeviceGuard g(h->device);
  if ((rc = h->dw.run(params, reinterpret_cast<hipStream_t>(stream)))) return rc;
  h->committed = true;
  return KDLAE_OK;
}

int64_t kdlae_s_workspace_bytes(const kdlae_s_handle* h, int B, int F, int H, int W) {
  if (!h) return -1;
  const int m = 1 << h->L;
  if (B <= 0 || F <= 0 || H <= 0 || W <= 0 || H % m || W % m) {
    fail(KDLAE_EINVAL_SHAPE, "B, F, H, W must be positive with H, W divisible by 2^(levels)");
    return -1;
  }
  return (int64_t)make_splan(h, B, F, H, W).total;
}

int kdlae_s_forward(kdlae_s_handle* h, const float* x, int B, int F, int H, int W, float* out, void* workspace,
                    int64_t workspace_bytes, void* stream) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  if (!h->committed) return fail(KDLAE_ESTATE, "forward before kdlae_s_commit_params / kdlae_s_pack_device");
  const int m = 1 << h->L;
  if (B <= 0 || F <= 0 || H <= 0 || W <= 0 || H % m || W % m)
    return fail(KDLAE_EINVAL_SHAPE, "KDLAE_student needs H and W divisible by 2^(len(hidden_channels)-1) "
                                    "(MaxPool3d then ConvTranspose3d + skip, KDLAE_model.py:406,416-417)");
  if (!x || !out || !workspace) return fail(KDLAE_ESTATE, "null tensor");
  SPlan pl = make_splan(h, B, F, H, W);
  if ((int64_t)pl.total > workspace_bytes) return fail(KDLAE_ESTATE, "workspace too small");
  DeviceGuard dg(h->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  auto buf = [&](size_t off) { return reinterpret_cast<float*>(ws + off); };
  float* tA = buf(pl.tA);
  float* tB = buf(pl.tB);
  const DeviceWeights& D = h->dw;
  int rc;
  auto conv = [&](const Gemm& g, View in, View o, int Hh, int Ww, int relu) {
    if (g.kt == 3 && g.ntiles == 1 && g.cg_per_tap == 1 && g.kgroups == 27) {
      // 16 -> 16 channels: LDS-tiled kernel with the weights held in VGPRs (conv3d_c16.hip)
      Conv3dC16Params q{};
      q.in = in.p;
      q.ldi = in.ld;
      q.wp = D.P(g.w);
      q.bias = D.P(g.bias);
      q.out = o.p;
      q.ldo = o.ld;
      q.Bn = B;
      q.F = F;
      q.H = Hh;
      q.W = Ww;
      q.relu = relu;
      q.kt = 3;
      HIPCHK(launch_conv3d_c16(q, s));
      return (int)KDLAE_OK;
    }
    if (g.ksize == 3 && g.out_mode == 0 && g.kt == 3 && conv_lds_supported(g.kt, g.ntiles, g.cg_per_tap * 16)) {
      // LDS-tiled implicit GEMM (conv_lds.hip): halo staged once, no per-tap L1 re-reads
      ConvLdsParams q{};
      q.in = in.p;
      q.ldi = in.ld;
      q.cin_pad = g.cg_per_tap * 16;
      q.wp = D.P(g.w);
      q.ntiles = g.ntiles;
      q.kgroups = g.kgroups;
      q.bias = D.P(g.bias);
      q.out = o.p;
      q.ldo = o.ld;
      q.Bn = B;
      q.F = F;
      q.H = Hh;
      q.W = Ww;
      q.kt = g.kt;
      q.relu = relu;
      q.wp3 = D.P3(g.w3t);
      HIPCHK(launch_conv_lds(q, s));
      return (int)KDLAE_OK;
    }
    GemmCall c;
    c.g = &g;
    c.W = D.P3(g.w3);
    c.bias = D.P(g.bias);
    c.in = in;
    c.out = o;
    c.B = B;
    c.F = F;
    c.H = Hh;
    c.Wd = Ww;
    c.relu = relu;
    return run_gemm(c, s);
  };
  for (int i = 0; i < h->L; ++i) {
    const int Hi = H >> i, Wi = W >> i, ci = h->cs[i];
    if (i == 0) {
      SmallInParams p{};
      p.in = x;
      p.sb = (long long)F * H * W;
      p.sc = 0;
      p.st = (long long)H * W;
      p.sy = W;
      p.sx = 1;
      p.Cin = 1;
      p.Cout = h->first.Cout;
      p.dil = 1;
      p.w = D.P(h->first.w);
      p.bias = D.P(h->first.bias);
      p.out = tA;
      p.ldo = ci;
      p.Bn = B;
      p.H = H;
      p.W = W;
      p.F = F;
      p.kt = 3;
      p.relu = 1;
      HIPCHK(launch_conv_small_in(p, s));
    } else {
      if ((rc = conv(h->enc[i].a, View{tB, h->cs[i - 1]}, View{tA, ci}, Hi, Wi, 1))) return rc;
    }
    if ((rc = conv(h->enc[i].b, View{tA, ci}, View{buf(pl.skip[i]), ci}, Hi, Wi, 1))) return rc;
    HIPCHK(launch_maxpool2(buf(pl.skip[i]), ci, tB, ci, ci, (long long)B * F, Hi, Wi, s));
  }
  const int HL = H >> h->L, WL = W >> h->L;
  if ((rc = conv(h->fusion.a, View{tB, h->cs[h->L - 1]}, View{tA, h->cs[h->L]}, HL, WL, 1))) return rc;
  if ((rc = conv(h->fusion.b, View{tA, h->cs[h->L]}, View{tB, h->cs[h->L]}, HL, WL, 1))) return rc;
  int ccur = h->cs[h->L];
  for (int j = 0, i = h->L - 1; i >= 0; --i, ++j) {
    const int Hi = H >> i, Wi = W >> i, ci = h->cs[i];
    float* sk = buf(pl.skip[i]);
    GemmCall c;  // ConvTranspose3d (1,2,2) + bias, + skip, written in place over the skip tensor
    c.g = &h->up[j];
    c.W = D.P3(h->up[j].w3);
    c.bias = D.P(h->up[j].bias);
    c.in = View{tB, ccur};
    c.out = View{sk, ci};
    c.B = B;
    c.F = F;
    c.H = Hi >> 1;
    c.Wd = Wi >> 1;
    c.out_mode = 2;
    c.R = sk;
    c.ldr = ci;
    if ((rc = run_gemm(c, s))) return rc;
    if ((rc = conv(h->dec[j].a, View{sk, ci}, View{tA, ci}, Hi, Wi, 1))) return rc;
    if ((rc = conv(h->dec[j].b, View{tA, ci}, View{tB, ci}, Hi, Wi, 1))) return rc;
    ccur = ci;
  }
  SmallOutParams p{};
  p.in = tB;
  p.ld = h->cs[0];
  p.Cin = h->cs[0];
  p.Cout = 1;
  p.w = D.P(h->outc.w);
  p.bias = D.P(h->outc.bias);
  p.Bn = B;
  p.H = H;
  p.W = W;
  p.F = F;
  p.ks = 1;
  p.out = out;
  p.out_nchw = 1;
  p.res = h->cfg.residual ? x : nullptr;
  HIPCHK(launch_conv_small_out(p, s));
  return KDLAE_OK;
}

}  // extern "C"
