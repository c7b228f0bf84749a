#include <cstdlib>
// ASDQE host runtime: DenoiseRatePredictor forward in eval mode (ASDQE/ASDQE_model.py:123-171).
//
//   pad_to_multiple(lq / gt, dim) (:113-121, :159-160)   -> zero-extent bounds in the first convs
//   3 DoubleConv extractors on lq, gt, lq - gt (:131-135) -> merged [P][3*dim] (torch.cat :165)
//   UNet (:78-111): inc, down1..3 (maxpool + DoubleConv), up1..3 (bilinear x2 align_corners into
//   the concat's second half, cat [skip, up], DoubleConv), outc 1x1
//   regressor (:144-154): GAP, Linear-ReLU x2, Linear, Tanh
//
// Every conv3x3 + BatchNorm(eval) + ReLU is one implicit GEMM with BN folded into the packed weights
// and bias.  Skips are written by their producer straight into the first half of the concat buffer
// the decoder reads, and the upsample writes the second half, so torch.cat never materialises.
// outc is linear, so it is applied after the pool inside the head kernel (the full-resolution map is
// only produced when the caller asks for it).
#include <cmath>
#include <string>
#include <vector>

#include "runtime.h"

using namespace kdlae;

struct asdqe_handle {
  asdqe_config cfg{};
  int device = 0;
  ParamStore ps;
  bool built = false, committed = false;
  DeviceWeights dw;        // packed arena + the pack program that fills it from the parameters
  SmallW ext1[3];
  Gemm ext2[3];
  Gemm inc[2], dn[3][2], upc[3][2];
  Gemm outc;                                   // only for the optional feature-map output
  size_t wo = kNone, bo = kNone, w1 = kNone, b1 = kNone, w2 = kNone, b2 = kNone, w3 = kNone, b3 = kNone;
};

namespace {

const char* kExt[3] = {"lq_extractor", "gt_extractor", "diff_extractor"};
const char* kDown[3] = {"unet.down1.maxpool_conv.1.double_conv", "unet.down2.maxpool_conv.1.double_conv",
                        "unet.down3.maxpool_conv.1.double_conv"};
const char* kUp[3] = {"unet.up1.conv.double_conv", "unet.up2.conv.double_conv", "unet.up3.conv.double_conv"};
const int kDownC[3][2] = {{64, 128}, {128, 256}, {256, 256}};
const int kUpC[3][2] = {{512, 128}, {256, 64}, {128, 64}};

// GAP partial slots per image: a function of the padded image size only, so an image's pooled
// features are summed in the same order whatever the batch (bit-identical batch invariance).
int gap_slots(long long HW) {
  long long s = HW / 2048;
  return (int)std::max<long long>(1, std::min<long long>(256, s));
}

struct APlan {
  size_t total = 0;
  size_t e1, merged, t0, cat3, y3, p1, t1, cat2, y2, p2, t2, cat1, y1, p3, t3, x4, partial;
  int Hp, Wp, slots;
  size_t take(long long floats) {
    size_t off = total;
    total += ((size_t)floats * 4 + 255) / 256 * 256;
    return off;
  }
};

APlan make_aplan(const asdqe_handle* h, int B, int H, int W) {
  APlan pl;
  const int d = h->cfg.dim, m = 3 * d;
  pl.Hp = (H + d - 1) / d * d;
  pl.Wp = (W + d - 1) / d * d;
  const long long P0 = (long long)B * pl.Hp * pl.Wp, P1 = P0 / 4, P2 = P0 / 16, P3 = P0 / 64;
  pl.e1 = pl.take(P0 * m);
  pl.merged = pl.take(P0 * m);
  pl.t0 = pl.take(P0 * 64);
  pl.cat3 = pl.take(P0 * 128);
  pl.y3 = pl.take(P0 * 64);
  pl.p1 = pl.take(P1 * 64);
  pl.t1 = pl.take(P1 * 128);
  pl.cat2 = pl.take(P1 * 256);
  pl.y2 = pl.take(P1 * 64);
  pl.p2 = pl.take(P2 * 128);
  pl.t2 = pl.take(P2 * 256);
  pl.cat1 = pl.take(P2 * 512);
  pl.y1 = pl.take(P2 * 128);
  pl.p3 = pl.take(P3 * 256);
  pl.t3 = pl.take(P3 * 256);
  pl.x4 = pl.take(P3 * 256);
  pl.slots = gap_slots((long long)pl.Hp * pl.Wp);
  pl.partial = pl.take((long long)B * pl.slots * 64);
  return pl;
}

}  // namespace

extern "C" {

int asdqe_create(const asdqe_config* cfg, int device, asdqe_handle** out) {
  if (!cfg || !out) return fail(KDLAE_ESTATE, "null argument");
  *out = nullptr;
  if (cfg->in_channels < 1 || cfg->in_channels > 4)
    return fail(KDLAE_EINVAL_CONFIG, "in_channels must be 1..4 on the HIP path");
  if (cfg->dim < 16 || cfg->dim > 256 || cfg->dim % 16)
    return fail(KDLAE_EINVAL_CONFIG, "dim must be a multiple of 16 in 16..256 on the HIP path");
  auto* h = new asdqe_handle();
  h->cfg = *cfg;
  h->device = device;
  // state_dict keys in registration order (ASDQE_model.py:127-156), BN buffers included
  auto dc = [&](const std::string& p, int cin, int cout) {
    for (int i : {0, 3}) {
      const int ci = i == 0 ? cin : cout;
      h->ps.add(p + "." + std::to_string(i) + ".weight", (int64_t)cout * ci * 9);
      h->ps.add(p + "." + std::to_string(i) + ".bias", cout);
      const std::string bn = p + "." + std::to_string(i + 1) + ".";
      for (const char* s : {"weight", "bias", "running_mean", "running_var"}) h->ps.add(bn + s, cout);
      h->ps.add(bn + "num_batches_tracked", 1);
    }
  };
  const int d = cfg->dim, m = 3 * d;
  for (const char* e : kExt) dc(std::string(e) + ".double_conv", cfg->in_channels, d);
  dc("unet.inc.double_conv", m, 64);
  for (int i = 0; i < 3; ++i) dc(kDown[i], kDownC[i][0], kDownC[i][1]);
  for (int i = 0; i < 3; ++i) dc(kUp[i], kUpC[i][0], kUpC[i][1]);
  h->ps.add("unet.outc.conv.weight", (int64_t)m * 64);
  h->ps.add("unet.outc.conv.bias", m);
  h->ps.add("regressor.2.weight", (int64_t)256 * m);
  h->ps.add("regressor.2.bias", 256);
  h->ps.add("regressor.5.weight", 256 * 64);
  h->ps.add("regressor.5.bias", 64);
  h->ps.add("regressor.8.weight", 64);
  h->ps.add("regressor.8.bias", 1);
  *out = h;
  return KDLAE_OK;
}

int asdqe_destroy(asdqe_handle* h) {
  if (!h) return KDLAE_OK;
  {
    DeviceGuard g(h->device);
    h->dw.release();
  }
  delete h;
  return KDLAE_OK;
}

int asdqe_num_params(const asdqe_handle* h) { return h ? (int)h->ps.keys.size() : 0; }

int asdqe_param_info(const asdqe_handle* h, int index, const char** name, int64_t* numel) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  return h->ps.info(index, name, numel);
}

int64_t asdqe_params_numel(const asdqe_handle* h) { return h ? h->ps.total : -1; }

int asdqe_set_param(asdqe_handle* h, const char* name, const float* host_data, int64_t numel) {
  if (!h || !name || !host_data) return fail(KDLAE_ESTATE, "null argument");
  return h->ps.set(name, host_data, numel);
}

}  // extern "C"

// Records the packed layout (pack program, runtime.h) of this configuration once per handle.
static int build_program_a(asdqe_handle* h) {
  if (h->built) return KDLAE_OK;
  PackProgram ar;
  ar.nsrc = h->ps.total;
  int err = KDLAE_OK;
  // BatchNorm2d eval (eps 1e-5) folded into the preceding conv: W' = s W, b' = s (b - rm) + beta,
  // s = gamma / sqrt(rv + eps): s and b' are derived values computed on the device before the gathers
  auto bn_fold = [&](const std::string& conv, const std::string& bn, int cout, std::vector<int32_t>& sc,
                     std::vector<int32_t>& sh) {
    const int32_t B = h->ps.base(conv + ".bias", &err);
    const int32_t g = h->ps.base(bn + ".weight", &err);
    const int32_t be = h->ps.base(bn + ".bias", &err);
    const int32_t rm = h->ps.base(bn + ".running_mean", &err);
    const int32_t rv = h->ps.base(bn + ".running_var", &err);
    sc.assign(cout, -1);
    sh.assign(cout, -1);
    if (err) return;
    for (int n = 0; n < cout; ++n) {
      PDer d0;
      d0.kind = 0;
      d0.a = g + n;
      d0.b = rv + n;
      sc[n] = ar.derive(d0);
      PDer d1;
      d1.kind = 1;
      d1.a = B + n;
      d1.b = rm + n;
      d1.c = sc[n];
      d1.d = be + n;
      sh[n] = ar.derive(d1);
    }
  };
  auto conv3 = [&](const std::string& p, int i, int cin, int cout) {
    Gemm g;
    const std::string cv = p + "." + std::to_string(i), bn = p + "." + std::to_string(i + 1);
    const int32_t W = h->ps.base(cv + ".weight", &err);
    std::vector<int32_t> sc, sh;
    bn_fold(cv, bn, cout, sc, sh);
    if (err) return g;
    const int cis = ru16(cin), cos = ru16(cout);
    g.ksize = 3;
    g.cg_per_tap = cis / 16;
    g.ntiles = cos / 16;
    g.kgroups = 9 * cis / 16;
    g.N = cos;
    g.K = 9 * cis;
    g.n_true = cout;
    g.k_true = 9 * cin;
    g.w = ar.add(pack_fragments(g.ntiles, g.kgroups, [&](int n, int k) -> PEx {
      const int tap = k / cis, c = k - tap * cis;
      if (n >= cout || c >= cin) return PEx{};
      return PEx{W + (n * cin + c) * 9 + tap, sc[n]};
    }));
    g.w3 = ar.split(g.w, g.ntiles, g.kgroups);
    std::vector<PEx> b((size_t)cos);
    for (int n = 0; n < cout; ++n) b[n].a = sh[n];
    g.bias = ar.add(b);
    choose_variant(g);
    return g;
  };
  const int d = h->cfg.dim, m = 3 * d, ci = h->cfg.in_channels;
  for (int e = 0; e < 3; ++e) {
    const std::string p = std::string(kExt[e]) + ".double_conv";
    const int32_t W = h->ps.base(p + ".0.weight", &err);
    std::vector<int32_t> sc, sh;
    bn_fold(p + ".0", p + ".1", d, sc, sh);
    if (err) return err;
    std::vector<PEx> w((size_t)d * ci * 9), t((size_t)d);
    for (int n = 0; n < d; ++n) {
      for (int k = 0; k < ci * 9; ++k) w[(size_t)n * ci * 9 + k] = PEx{W + n * ci * 9 + k, sc[n]};
      t[n].a = sh[n];
    }
    h->ext1[e].w = ar.add(w);
    h->ext1[e].bias = ar.add(t);
    h->ext1[e].Cin = ci;
    h->ext1[e].Cout = d;
    h->ext2[e] = conv3(p, 3, d, d);
  }
  h->inc[0] = conv3("unet.inc.double_conv", 0, m, 64);
  h->inc[1] = conv3("unet.inc.double_conv", 3, 64, 64);
  for (int i = 0; i < 3; ++i) {
    h->dn[i][0] = conv3(kDown[i], 0, kDownC[i][0], kDownC[i][1]);
    h->dn[i][1] = conv3(kDown[i], 3, kDownC[i][1], kDownC[i][1]);
    h->upc[i][0] = conv3(kUp[i], 0, kUpC[i][0], kUpC[i][1]);
    h->upc[i][1] = conv3(kUp[i], 3, kUpC[i][1], kUpC[i][1]);
  }
  {
    const int32_t W = h->ps.base("unet.outc.conv.weight", &err);
    const int32_t Bv = h->ps.base("unet.outc.conv.bias", &err);
    if (err) return err;
    Gemm& g = h->outc;
    g.ntiles = ru16(m) / 16;
    g.kgroups = 4;
    g.N = ru16(m);
    g.K = 64;
    g.n_true = m;
    g.k_true = 64;
    g.w = ar.add(pack_fragments(g.ntiles, g.kgroups, [&](int n, int k) -> PEx {
      return n < m ? PEx{W + n * 64 + k, -1} : PEx{};
    }));
    g.w3 = ar.split(g.w, g.ntiles, g.kgroups);
    std::vector<PEx> b((size_t)g.N);
    for (int n = 0; n < m; ++n) b[n].a = Bv + n;
    g.bias = ar.add(b);
    choose_variant(g);
    h->wo = ar.copy(W, (size_t)m * 64);
    h->bo = ar.copy(Bv, m);
  }
  auto raw = [&](const char* k, size_t n) {
    const int32_t b = h->ps.base(k, &err);
    return b >= 0 ? ar.copy(b, n) : kNone;
  };
  h->w1 = raw("regressor.2.weight", (size_t)256 * m);
  h->b1 = raw("regressor.2.bias", 256);
  h->w2 = raw("regressor.5.weight", 256 * 64);
  h->b2 = raw("regressor.5.bias", 64);
  h->w3 = raw("regressor.8.weight", 64);
  h->b3 = raw("regressor.8.bias", 1);
  if (err) return err;
  DeviceGuard dg(h->device);
  int rc = h->dw.upload_program(ar);
  if (rc) return rc;
  h->built = true;
  return KDLAE_OK;
}

extern "C" {

int asdqe_commit_params(asdqe_handle* h, void* stream) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  int rc = h->ps.check_complete();
  if (rc) return rc;
  if ((rc = build_program_a(h))) return rc;
  DeviceGuard g(h->device);
  if ((rc = h->dw.run_host(h->ps.flat(), reinterpret_cast<hipStream_t>(stream)))) return rc;
  h->committed = true;
  return KDLAE_OK;
}

int asdqe_prepare(asdqe_handle* h) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  return build_program_a(h);
}

int asdqe_pack_device(asdqe_handle* h, const float* params, int64_t numel, void* stream) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  if (numel != h->ps.total)
    return fail(KDLAE_EPARAM, "flat parameter vector has " + std::to_string(numel) + " floats, expected " +
                                  std::to_string(h->ps.total));
  int rc = build_program_a(h);
  if (rc) return rc;
  DeviceGuard g(h->device);
  if ((rc = h->dw.run(params, reinterpret_cast<hipStream_t>(stream)))) return rc;
  h->committed = true;
  return KDLAE_OK;
}

int64_t asdqe_workspace_bytes(const asdqe_handle* h, int B, int H, int W) {
  if (!h) return -1;
  if (B <= 0 || H <= 0 || W <= 0) {
    fail(KDLAE_EINVAL_SHAPE, "B, H, W must be positive");
    return -1;
  }
  return (int64_t)make_aplan(h, B, H, W).total;
}

int asdqe_forward(asdqe_handle* h, const float* lq, const float* gt, int B, int H, int W, float* score, float* feat,
                  void* workspace, int64_t workspace_bytes, void* stream) {
  if (!h) return fail(KDLAE_ESTATE, "null handle");
  if (!h->committed) return fail(KDLAE_ESTATE, "forward before asdqe_commit_params / asdqe_pack_device");
  if (B <= 0 || H <= 0 || W <= 0) return fail(KDLAE_EINVAL_SHAPE, "B, H, W must be positive");
  if (!lq || !gt || !score || !workspace) return fail(KDLAE_ESTATE, "null tensor");
  APlan pl = make_aplan(h, B, H, W);
  if ((int64_t)pl.total > workspace_bytes) return fail(KDLAE_ESTATE, "workspace too small");
  DeviceGuard dg(h->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  auto buf = [&](size_t off) { return reinterpret_cast<float*>(ws + off); };
  const DeviceWeights& D = h->dw;
  const int d = h->cfg.dim, m = 3 * d, ci = h->cfg.in_channels;
  const int Hp = pl.Hp, Wp = pl.Wp;
  int rc;
  auto conv = [&](const Gemm& g, View in, View o, int Hh, int Ww, int relu) {
    if (g.kt == 1 && g.ksize == 3 && g.ntiles == 1 && g.cg_per_tap == 1 && g.kgroups == 9 &&
        g.out_mode == 0) {
      // 16 -> 16 channels: LDS-tiled kernel with VGPR-resident weights (conv3d_c16.hip)
      Conv3dC16Params q{};
      q.in = in.p;
      q.ldi = in.ld;
      q.wp = D.P(g.w);
      q.bias = D.P(g.bias);
      q.out = o.p;
      q.ldo = o.ld;
      q.Bn = B;
      q.F = 1;
      q.H = Hh;
      q.W = Ww;
      q.relu = relu;
      q.kt = 1;
      HIPCHK(launch_conv3d_c16(q, s));
      return (int)KDLAE_OK;
    }
    if (g.ksize == 3 && g.out_mode == 0 && g.kt == 1 && conv_lds_supported(g.kt, g.ntiles, g.cg_per_tap * 16)) {
      // LDS-tiled implicit GEMM (conv_lds.hip): halo staged once, no per-tap L1 re-reads
      ConvLdsParams q{};
      q.in = in.p;
      q.ldi = in.ld;
      q.cin_pad = g.cg_per_tap * 16;
      q.wp = D.P(g.w);
      q.wp3 = D.P3(g.w3);
      q.ntiles = g.ntiles;
      q.kgroups = g.kgroups;
      q.bias = D.P(g.bias);
      q.out = o.p;
      q.ldo = o.ld;
      q.Bn = B;
      q.F = 1;
      q.H = Hh;
      q.W = Ww;
      q.kt = g.kt;
      q.relu = relu;
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
    c.H = Hh;
    c.Wd = Ww;
    c.relu = relu;
    return run_gemm(c, s);
  };
  // extractors: conv1 (+BN+ReLU) reads the NCHW input with zero padding beyond H x W, conv2 writes merged
  float* e1 = buf(pl.e1);
  float* merged = buf(pl.merged);
  for (int e = 0; e < 3; ++e) {
    SmallInParams p{};
    p.in = e == 1 ? gt : lq;
    p.in_sub = e == 2 ? gt : nullptr;
    p.sb = (long long)ci * H * W;
    p.sc = (long long)H * W;
    p.sy = W;
    p.sx = 1;
    p.Cin = ci;
    p.Cout = d;
    p.dil = 1;
    p.w = D.P(h->ext1[e].w);
    p.bias = D.P(h->ext1[e].bias);
    p.out = e1 + e * d;
    p.ldo = m;
    p.Bn = B;
    p.H = Hp;
    p.W = Wp;
    p.vh = H;
    p.vw = W;
    p.F = 1;
    p.kt = 1;
    p.relu = 1;
    HIPCHK(launch_conv_small_in(p, s));
  }
  for (int e = 0; e < 3; ++e)
    if ((rc = conv(h->ext2[e], View{e1 + e * d, m}, View{merged + e * d, m}, Hp, Wp, 1))) return rc;
  // UNet encoder; each level's skip lands in the first half of the decoder's concat buffer
  float *t0 = buf(pl.t0), *cat3 = buf(pl.cat3), *y3 = buf(pl.y3);
  float *p1 = buf(pl.p1), *t1 = buf(pl.t1), *cat2 = buf(pl.cat2), *y2 = buf(pl.y2);
  float *p2 = buf(pl.p2), *t2 = buf(pl.t2), *cat1 = buf(pl.cat1), *y1 = buf(pl.y1);
  float *p3 = buf(pl.p3), *t3 = buf(pl.t3), *x4 = buf(pl.x4);
  const int H1 = Hp / 2, W1 = Wp / 2, H2 = Hp / 4, W2 = Wp / 4, H3 = Hp / 8, W3 = Wp / 8;
  if ((rc = conv(h->inc[0], View{merged, m}, View{t0, 64}, Hp, Wp, 1))) return rc;
  if ((rc = conv(h->inc[1], View{t0, 64}, View{cat3, 128}, Hp, Wp, 1))) return rc;
  HIPCHK(launch_maxpool2(cat3, 128, p1, 64, 64, B, Hp, Wp, s));
  if ((rc = conv(h->dn[0][0], View{p1, 64}, View{t1, 128}, H1, W1, 1))) return rc;
  if ((rc = conv(h->dn[0][1], View{t1, 128}, View{cat2, 256}, H1, W1, 1))) return rc;
  HIPCHK(launch_maxpool2(cat2, 256, p2, 128, 128, B, H1, W1, s));
  if ((rc = conv(h->dn[1][0], View{p2, 128}, View{t2, 256}, H2, W2, 1))) return rc;
  if ((rc = conv(h->dn[1][1], View{t2, 256}, View{cat1, 512}, H2, W2, 1))) return rc;
  HIPCHK(launch_maxpool2(cat1, 512, p3, 256, 256, B, H2, W2, s));
  if ((rc = conv(h->dn[2][0], View{p3, 256}, View{t3, 256}, H3, W3, 1))) return rc;
  if ((rc = conv(h->dn[2][1], View{t3, 256}, View{x4, 256}, H3, W3, 1))) return rc;
  // decoder: upsample into the concat's second half (F.pad is a no-op: sizes are exact multiples)
  HIPCHK(launch_upsample2x(x4, 256, cat1 + 256, 512, 256, B, H3, W3, s));
  if ((rc = conv(h->upc[0][0], View{cat1, 512}, View{t2, 128}, H2, W2, 1))) return rc;
  if ((rc = conv(h->upc[0][1], View{t2, 128}, View{y1, 128}, H2, W2, 1))) return rc;
  HIPCHK(launch_upsample2x(y1, 128, cat2 + 128, 256, 128, B, H2, W2, s));
  if ((rc = conv(h->upc[1][0], View{cat2, 256}, View{t1, 64}, H1, W1, 1))) return rc;
  if ((rc = conv(h->upc[1][1], View{t1, 64}, View{y2, 64}, H1, W1, 1))) return rc;
  HIPCHK(launch_upsample2x(y2, 64, cat3 + 64, 128, 64, B, H1, W1, s));
  if ((rc = conv(h->upc[2][0], View{cat3, 128}, View{t0, 64}, Hp, Wp, 1))) return rc;
  if ((rc = conv(h->upc[2][1], View{t0, 64}, View{y3, 64}, Hp, Wp, 1))) return rc;
  if (feat && (rc = conv(h->outc, View{y3, 64}, View{feat, m}, Hp, Wp, 0))) return rc;
  // regressor: GAP over the padded map (AdaptiveAvgPool2d sees H' x W'), outc folded after the pool
  float* partial = buf(pl.partial);
  HIPCHK(launch_gap_partial(y3, 64, 64, B, (long long)Hp * Wp, pl.slots, partial, s));
  HeadParams hp{};
  hp.partial = partial;
  hp.slots = pl.slots;
  hp.C = 64;
  hp.inv_hw = 1.f / (float)((long long)Hp * Wp);
  hp.wo = D.P(h->wo);
  hp.bo = D.P(h->bo);
  hp.M = m;
  hp.w1 = D.P(h->w1);
  hp.b1 = D.P(h->b1);
  hp.N1 = 256;
  hp.w2 = D.P(h->w2);
  hp.b2 = D.P(h->b2);
  hp.N2 = 64;
  hp.w3 = D.P(h->w3);
  hp.b3 = D.P(h->b3);
  hp.score = score;
  hp.B = B;
  HIPCHK(launch_asdqe_head(hp, s));
  return KDLAE_OK;
}

}  // extern "C"
