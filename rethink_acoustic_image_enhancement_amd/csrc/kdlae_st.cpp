// KDLAE-S training engine (the student of KDLAE/KDLAE_model.py:340-431 under BasicSR's
// ImageCleanModel with KDLAES.yml: Train/basicsr/models/image_restoration_model.py:198-218).
//
// Forward with every activation kept (NDHWC, ld = channels), then the hand-sequenced backward:
//   Conv3d 3x3x3 + bias + ReLU (:386-393)   fwd  Y = relu(Xcol . W'^T + b)           (train GEMM)
//                                           bwd  dZ = dY (Y > 0); db = colsum dZ;
//                                                dW' = dZ^T . Xcol; dX = col2im(dZ . W')
//                                           (W' = the weight in the columns' tap-major order, train_s.hip)
//   MaxPool3d (1,2,2) (:366)                fwd  inference kernel; bwd first-max routing
//   ConvTranspose3d (1,2,2) s2 (:378-379)   fwd  U = L . Wu (N = 4 Cout), D = shuffle(U) + b + skip (:417)
//                                           bwd  dU = unshuffle(dD); db = colsum dD; dWu = L^T dU; dL = dU Wu^T
//   out_conv 1x1x1 + residual (:422-426)    a K = C0 / N = 1 GEMM with the input as residual
// Parameters and gradients are flat buffers in state_dict order with every key 16-byte aligned (the
// KDLAE-T training layout), so kdlae_train_clip_adamw / _ema / the DDP all-reduce apply unchanged.
#include <hip/hip_runtime.h>

#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "kernels.h"
#include "runtime.h"
#include "train_kernels.h"
#include "train_s.h"

using namespace kdlae;
namespace tr = kdlae::train;

struct kdlae_st_handle {
  kdlae_s_config cfg{};
  int device = 0;
  int L = 0;
  std::vector<int> hc;
  std::vector<std::string> names;
  std::vector<int64_t> numel, offset;
  std::unordered_map<std::string, int64_t> off;
  int64_t total = 0;
  // the last forward (its activations live in the caller's workspace)
  bool valid = false;
  int B = 0, F = 0, H = 0, W = 0;
  const void* ws = nullptr;
  const float* x = nullptr;
  // backward side stream (non-blocking) for the Conv3d weight / bias gradients, and its fork / join
  // events (KDLAE_DEBUG=train_serial: everything on the caller's stream)
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  ~kdlae_st_handle() {
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    if (side) (void)hipStreamDestroy(side);
  }
};

namespace {

constexpr size_t kPartialFloats = 16u << 20;  // split-K partials of the weight-gradient GEMMs
constexpr auto KDLAE_ST_DX_CONV = 1;
constexpr auto KDLAE_ST_DIRECT = 1;
constexpr int kColsumBlocks = 256;

struct SPlanT {
  size_t total = 0;
  std::vector<size_t> ea, e, pool, ua, da, dd, dl, gskip;  // per level / decoder
  std::unordered_map<std::string, size_t> xcol;            // each Conv3d's forward column matrix
  size_t fa = 0, fo = 0, col = 0, gA = 0, gB = 0, partial = 0, part = 0, wp = 0, dwp = 0, wpk = 0, zb = 0;
  long long col2im_max = 0;  // the largest P * cin a col2im gathers (its element index is 32-bit)
  size_t take(long long floats) {
    const size_t o = total;
    total += ((size_t)floats * 4 + 255) / 256 * 256;
    return o;
  }
};

long long npx(const kdlae_st_handle* h, int lvl, int B, int F, int H, int W) {
  return (long long)B * F * (H >> lvl) * (W >> lvl);
}

// A Conv3d whose channel counts are multiples of 16 on a level at least 16 wide runs "direct": the
// forward on the inference conv kernels (conv3d_c16 for 16 -> 16, conv_lds for 2..16 output tiles) and
// the weight gradient on the pixel-reduction GEMM with an implicit im2col B (bmode 4); no column
// matrix.  The others (the 1-channel input conv, odd widths) go through Xcol.
bool conv_direct(int cin, int cout, int Wl) {
  if (!KDLAE_ST_DIRECT || cin % 16 || cout % 16 || Wl % 16) return false;
  return (cin == 16 && cout == 16) || conv_lds_supported(3, cout / 16, cin);
}
// the input gradient of a Conv3d on the inference conv kernels (flipped taps, cout -> cin)
bool dx_direct(int cin, int cout) {
  return KDLAE_ST_DX_CONV && cout % 16 == 0 && cin % 16 == 0 &&
         ((cin == 16 && cout == 16) || conv_lds_supported(3, cin / 16, cout));
}

SPlanT make_plan(const kdlae_st_handle* h, int B, int F, int H, int W) {
  SPlanT pl;
  const int L = h->L;
  long long colmax = 0, gmax = 0;  // colmax: set below
  for (int i = 0; i < L; ++i) {
    const long long P = npx(h, i, B, F, H, W);
    const int c = h->hc[i];
    pl.ea.push_back(pl.take(P * c));
    pl.e.push_back(pl.take(P * c));
    pl.pool.push_back(pl.take(P / 4 * c));
    pl.gskip.push_back(pl.take(P * c));
    gmax = std::max(gmax, P * c);
  }
  const long long PL = npx(h, L, B, F, H, W);
  pl.fa = pl.take(PL * h->hc[L]);
  pl.fo = pl.take(PL * h->hc[L]);
  gmax = std::max(gmax, PL * h->hc[L]);
  for (int j = 0; j < L; ++j) {
    const int i = L - 1 - j;
    const long long P = npx(h, i, B, F, H, W);
    const int c = h->hc[i];
    pl.ua.push_back(pl.take(P * c));  // U (= 4 c per low-resolution pixel)
    pl.dd.push_back(pl.take(P * c));  // D = shuffle(U) + b + skip
    pl.da.push_back(pl.take(P * c));
    pl.dl.push_back(pl.take(P * c));
  }
  // per Conv3d (name, input channels, output channels, level): its Xcol (only for the convs that are
  // not direct) is kept from the forward for its weight gradient
  std::vector<std::tuple<std::string, int, int, int>> convs;
  for (int i = 0; i < L; ++i) {
    const std::string p = "encoders." + std::to_string(i);
    convs.emplace_back(p + ".0", i ? h->hc[i - 1] : 1, h->hc[i], i);
    convs.emplace_back(p + ".2", h->hc[i], h->hc[i], i);
  }
  convs.emplace_back("st_fusion.0", h->hc[L - 1], h->hc[L], L);
  convs.emplace_back("st_fusion.2", h->hc[L], h->hc[L], L);
  for (int j = 0; j < L; ++j) {
    const int i = L - 1 - j;
    const std::string d = "decoders." + std::to_string(j);
    convs.emplace_back(d + ".0", h->hc[i], h->hc[i], i);
    convs.emplace_back(d + ".2", h->hc[i], h->hc[i], i);
  }
  // scratch: the dX columns of the convs whose dX is not direct, and the ConvTranspose dU
  for (int i = 0; i < L; ++i) colmax = std::max(colmax, npx(h, i, B, F, H, W) * h->hc[i]);
  for (auto& [name, ci, co, lvl] : convs) {
    const long long P = npx(h, lvl, B, F, H, W);
    if (!dx_direct(ci, co)) {
      colmax = std::max(colmax, P * 27 * ci);
      pl.col2im_max = std::max(pl.col2im_max, P * ci);
    }
    if (!conv_direct(ci, co, W >> lvl)) pl.xcol[name] = pl.take(P * 27 * ci);
  }
  pl.col = pl.take(colmax);
  long long wmax = 0;  // the largest Conv3d weight, for its tap-major copy and gradient
  for (int i = 0; i <= L; ++i) wmax = std::max(wmax, 27LL * h->hc[i] * std::max(i ? h->hc[i - 1] : 1, h->hc[i]));
  pl.wp = pl.take(wmax);
  pl.dwp = pl.take(wmax);
  pl.wpk = pl.take(wmax + 16LL * 27 * 16);  // packed dX weights (channel counts padded to 16)
  pl.zb = pl.take(64);                      // a zero bias for the inference conv kernels
  pl.gA = pl.take(gmax);
  pl.gB = pl.take(gmax);
  pl.partial = pl.take((long long)kPartialFloats);
  pl.part = pl.take((long long)kColsumBlocks * 64);
  return pl;
}

struct Ctx {
  kdlae_st_handle* h;
  const float* th;
  float* gr;
  char* ws;
  SPlanT pl;
  hipStream_t s;
  int B, F, H, W;
  hipStream_t side = nullptr;    // set by the backward unless KDLAE_DEBUG=train_serial
  hipStream_t main_s = nullptr;  // the caller's stream (c.s is the side stream inside a side segment)
  float* buf(size_t o) const { return reinterpret_cast<float*>(ws + o); }
  const float* P(const std::string& k) const { return th + h->off.at(k); }
  float* G(const std::string& k) const { return gr + h->off.at(k); }
};

#define TRY(x)                   \
  do {                           \
    int rc_ = (x);               \
    if (rc_) return rc_;         \
  } while (0)

int gemm(Ctx& c, tr::TGemm g, bool split) {
  if (split) {
    g.partial = c.buf(c.pl.partial);
    HIPCHK(tr::launch_tgemm(g, kPartialFloats, c.s));
  } else {
    HIPCHK(tr::launch_tgemm(g, 0, c.s));
  }
  return KDLAE_OK;
}

int colsum(Ctx& c, const float* x, int ld, int ncols, long long rows, float* out) {
  float* part = c.buf(c.pl.part);
  const int nb = (int)std::max<long long>(1, std::min<long long>(kColsumBlocks, rows / 128));
  const int nb2 = std::min(nb, (int)(kColsumBlocks * 64 / std::max(1, ncols)));
  HIPCHK(tr::launch_colsum(x, ld, ncols, rows, 1, 0, part, nb2, c.s));
  HIPCHK(tr::launch_part_reduce(part, nb2, ncols, 1, out, 0, 1.f, c.s));
  return KDLAE_OK;
}

// Y = relu(conv(X, W) + b) on the inference kernels (conv_direct) or as Xcol . W'^T + b (W' = the weight
// in the columns' tap-major order) over P pixels at level lvl
int conv_fwd(Ctx& c, const std::string& p, const float* X, int cin, float* Y, int cout, int lvl) {
  const int Hl = c.H >> lvl, Wl = c.W >> lvl;
  const long long P = (long long)c.B * c.F * Hl * Wl;
  if (conv_direct(cin, cout, Wl)) {
    float* wpk = c.buf(c.pl.wpk);
    HIPCHK(tr::launch_pack_conv(c.P(p + ".weight"), cout, cin, 0, wpk, c.s));
    if (cin == 16 && cout == 16) {
      Conv3dC16Params q{};
      q.in = X; q.ldi = cin;
      q.wp = wpk; q.bias = c.P(p + ".bias");
      q.out = Y; q.ldo = cout;
      q.Bn = c.B; q.F = c.F; q.H = Hl; q.W = Wl;
      q.relu = 1; q.kt = 3;
      HIPCHK(launch_conv3d_c16(q, c.s));
    } else {
      ConvLdsParams q{};
      q.in = X; q.ldi = cin; q.cin_pad = cin;
      q.wp = wpk; q.ntiles = cout / 16; q.kgroups = 27 * cin / 16;
      q.bias = c.P(p + ".bias");
      q.out = Y; q.ldo = cout;
      q.Bn = c.B; q.F = c.F; q.H = Hl; q.W = Wl;
      q.kt = 3; q.relu = 1;
      HIPCHK(launch_conv_lds(q, c.s));
    }
    return KDLAE_OK;
  }
  float* col = c.buf(c.pl.xcol.at(p));
  float* wp = c.buf(c.pl.wp);
  HIPCHK(tr::launch_wperm(c.P(p + ".weight"), wp, cout, cin, 0, c.s));
  HIPCHK(tr::launch_im2col3d(X, cin, cin, c.B, c.F, Hl, Wl, col, c.s));
  tr::TGemm g;
  g.A = col; g.sam = 27LL * cin; g.sak = 1;
  g.B = wp; g.sbk = 1; g.sbn = 27LL * cin;
  g.C = Y; g.scm = cout; g.scn = 1;
  g.bias = c.P(p + ".bias");
  g.M = (int)P; g.N = cout; g.K = 27 * cin;
  TRY(gemm(c, g, false));
  HIPCHK(tr::launch_relu(Y, cout, cout, P, c.s));
  return KDLAE_OK;
}

// the side stream waits for the main stream's current point; launches then go to the side stream
int side_fork(Ctx& c, hipStream_t main_s) {
  if (!c.side) return KDLAE_OK;
  HIPCHK(hipEventRecord(c.h->ev_fork, main_s));
  HIPCHK(hipStreamWaitEvent(c.side, c.h->ev_fork, 0));
  c.s = c.side;
  return KDLAE_OK;
}
// back to the main stream, which waits for the side stream's launches
int side_join(Ctx& c, hipStream_t main_s) {
  c.s = main_s;
  if (!c.side) return KDLAE_OK;
  HIPCHK(hipEventRecord(c.h->ev_join, c.side));
  HIPCHK(hipStreamWaitEvent(main_s, c.h->ev_join, 0));
  return KDLAE_OK;
}

// dY (grad of the ReLU output Y) -> weight / bias gradients and, when dX != null, the input gradient.
// The weight / bias gradients (which use the partial buffers, dwp and the gradient keys) run on the
// side stream beside the input gradient (which uses wpk / wp / col only); conv_bwd joins before returning.
int conv_bwd_body(Ctx& c, const std::string& p, const float* X, int cin, const float* Y, float* dY, int cout,
                  int lvl, float* dX) {
  const int Hl = c.H >> lvl, Wl = c.W >> lvl;
  const long long P = (long long)c.B * c.F * Hl * Wl;
  HIPCHK(tr::launch_relu_mask(dY, cout, Y, cout, cout, P, c.s));
  TRY(side_fork(c, c.main_s));
  TRY(colsum(c, dY, cout, cout, P, c.G(p + ".bias")));
  float* col = c.buf(c.pl.col);
  float* wp = c.buf(c.pl.wp);
  float* dwp = c.buf(c.pl.dwp);
  tr::TGemm g;  // dW'[o][k] = sum_p dZ[p][o] Xcol[p][k], then back to OIDHW order
  g.A = dY; g.sam = 1; g.sak = cout;
  g.C = dwp; g.scm = 27LL * cin; g.scn = 1;
  g.M = cout; g.N = 27 * cin; g.K = (int)P;
  if (conv_direct(cin, cout, Wl)) {  // Xcol implicit: the pixel-reduction kernel's bmode 4 reads X
    g.B = X; g.sbk = cin; g.sbn = 1; g.bmode = 4;
    g.Bn = c.B; g.F = c.F; g.H = Hl; g.W = Wl; g.Cg = cin;
    g.partial = c.buf(c.pl.partial);
    HIPCHK(tr::launch_tgemm_cols(g, kPartialFloats, c.s));
  } else {  // the forward's columns
    g.B = c.buf(c.pl.xcol.at(p)); g.sbk = 27LL * cin; g.sbn = 1;
    TRY(gemm(c, g, true));
  }
  HIPCHK(tr::launch_wperm(dwp, c.G(p + ".weight"), cout, cin, 1, c.s));
  c.s = c.main_s;
  if (!dX) return KDLAE_OK;
  // dX = the forward conv of dZ with flipped taps (cout -> cin channels) on the inference kernels:
  // conv3d_c16 for 16 -> 16, conv_lds for 2..16 output tiles; no column matrix, no col2im
  if (dx_direct(cin, cout)) {
    float* wpk = c.buf(c.pl.wpk);
    HIPCHK(tr::launch_pack_conv(c.P(p + ".weight"), cout, cin, 1, wpk, c.s));
    if (cin == 16 && cout == 16) {
      Conv3dC16Params q{};
      q.in = dY; q.ldi = cout;
      q.wp = wpk; q.bias = c.buf(c.pl.zb);
      q.out = dX; q.ldo = cin;
      q.Bn = c.B; q.F = c.F; q.H = Hl; q.W = Wl;
      q.relu = 0; q.kt = 3;
      HIPCHK(launch_conv3d_c16(q, c.s));
    } else {
      ConvLdsParams q{};
      q.in = dY; q.ldi = cout; q.cin_pad = cout;
      q.wp = wpk; q.ntiles = cin / 16; q.kgroups = 27 * cout / 16;
      q.bias = nullptr;
      q.out = dX; q.ldo = cin;
      q.Bn = c.B; q.F = c.F; q.H = Hl; q.W = Wl;
      q.kt = 3; q.relu = 0;
      HIPCHK(launch_conv_lds(q, c.s));
    }
    return KDLAE_OK;
  }
  HIPCHK(tr::launch_wperm(c.P(p + ".weight"), wp, cout, cin, 0, c.s));
  tr::TGemm d;  // dXcol = dZ . W', then the gather
  d.A = dY; d.sam = cout; d.sak = 1;
  d.B = wp; d.sbk = 27LL * cin; d.sbn = 1;
  d.C = col; d.scm = 27LL * cin; d.scn = 1;
  d.M = (int)P; d.N = 27 * cin; d.K = cout;
  TRY(gemm(c, d, false));
  HIPCHK(tr::launch_col2im3d(col, cin, c.B, c.F, Hl, Wl, dX, cin, 0, c.s));
  return KDLAE_OK;
}

int conv_bwd(Ctx& c, const std::string& p, const float* X, int cin, const float* Y, float* dY, int cout, int lvl,
             float* dX) {
  const int r = conv_bwd_body(c, p, X, cin, Y, dY, cout, lvl, dX);
  const int j = side_join(c, c.main_s);  // also on an error path: no side launch left unjoined
  return r ? r : j;
}

int net_fwd(Ctx& c, const float* x, float* out) {
  kdlae_st_handle* h = c.h;
  const int L = h->L;
  const float* cur = x;
  int ccur = 1;
  for (int i = 0; i < L; ++i) {
    const std::string p = "encoders." + std::to_string(i);
    const int ci = h->hc[i];
    TRY(conv_fwd(c, p + ".0", cur, ccur, c.buf(c.pl.ea[i]), ci, i));
    TRY(conv_fwd(c, p + ".2", c.buf(c.pl.ea[i]), ci, c.buf(c.pl.e[i]), ci, i));
    HIPCHK(launch_maxpool2(c.buf(c.pl.e[i]), ci, c.buf(c.pl.pool[i]), ci, ci, (long long)c.B * c.F, c.H >> i,
                           c.W >> i, c.s));
    cur = c.buf(c.pl.pool[i]);
    ccur = ci;
  }
  const int cL = h->hc[L];
  TRY(conv_fwd(c, "st_fusion.0", cur, ccur, c.buf(c.pl.fa), cL, L));
  TRY(conv_fwd(c, "st_fusion.2", c.buf(c.pl.fa), cL, c.buf(c.pl.fo), cL, L));
  cur = c.buf(c.pl.fo);
  ccur = cL;
  for (int j = 0; j < L; ++j) {
    const int i = L - 1 - j;
    const int ci = h->hc[i];
    const std::string u = "upconv_layers." + std::to_string(j), d = "decoders." + std::to_string(j);
    const long long Pl = npx(h, i + 1, c.B, c.F, c.H, c.W);
    tr::TGemm g;  // U = L . Wu, Wu = [cin][cout][1][2][2] = [cin][4 cout]
    g.A = cur; g.sam = ccur; g.sak = 1;
    g.B = c.P(u + ".weight"); g.sbk = 4LL * ci; g.sbn = 1;
    g.C = c.buf(c.pl.ua[j]); g.scm = 4LL * ci; g.scn = 1;
    g.M = (int)Pl; g.N = 4 * ci; g.K = ccur;
    TRY(gemm(c, g, false));
    HIPCHK(tr::launch_upshuffle_add(c.buf(c.pl.ua[j]), 4 * ci, c.P(u + ".bias"), c.buf(c.pl.e[i]), ci,
                                    c.buf(c.pl.dd[j]), ci, ci, c.B, c.F, c.H >> i, c.W >> i, c.s));
    TRY(conv_fwd(c, d + ".0", c.buf(c.pl.dd[j]), ci, c.buf(c.pl.da[j]), ci, i));
    TRY(conv_fwd(c, d + ".2", c.buf(c.pl.da[j]), ci, c.buf(c.pl.dl[j]), ci, i));
    cur = c.buf(c.pl.dl[j]);
    ccur = ci;
  }
  tr::TGemm g;  // out = d . w_out + b (+ x)
  const long long P0 = npx(h, 0, c.B, c.F, c.H, c.W);
  g.A = cur; g.sam = ccur; g.sak = 1;
  g.B = c.P("out_conv.weight"); g.sbk = 1; g.sbn = 0;
  g.C = out; g.scm = 1; g.scn = 0;
  g.bias = c.P("out_conv.bias");
  if (h->cfg.residual) {
    g.R = x; g.srm = 1; g.srn = 0;
  }
  g.M = (int)P0; g.N = 1; g.K = ccur;
  return gemm(c, g, false);
}

int net_bwd(Ctx& c, const float* x, const float* dout) {
  kdlae_st_handle* h = c.h;
  const int L = h->L;
  const long long P0 = npx(h, 0, c.B, c.F, c.H, c.W);
  const int c0 = h->hc[0];
  float* gA = c.buf(c.pl.gA);
  float* gB = c.buf(c.pl.gB);
  const float* dlast = c.buf(c.pl.dl[L - 1]);
  {  // out_conv
    tr::TGemm g;  // dW_out[c] = sum_p dout[p] d[p][c]
    g.A = dout; g.sam = 0; g.sak = 1;
    g.B = dlast; g.sbk = c0; g.sbn = 1;
    g.C = c.G("out_conv.weight"); g.scm = 0; g.scn = 1;
    g.M = 1; g.N = c0; g.K = (int)P0;
    TRY(gemm(c, g, true));
    TRY(colsum(c, dout, 1, 1, P0, c.G("out_conv.bias")));
    tr::TGemm d;  // dd[p][c] = dout[p] w_out[c]
    d.A = dout; d.sam = 1; d.sak = 0;
    d.B = c.P("out_conv.weight"); d.sbk = 0; d.sbn = 1;
    d.C = gA; d.scm = c0; d.scn = 1;
    d.M = (int)P0; d.N = c0; d.K = 1;
    TRY(gemm(c, d, false));
  }
  for (int j = L - 1; j >= 0; --j) {  // decoders, shallowest first
    const int i = L - 1 - j;
    const int ci = h->hc[i];
    const std::string u = "upconv_layers." + std::to_string(j), d = "decoders." + std::to_string(j);
    float* dD = c.buf(c.pl.gskip[i]);  // dD is also the skip tensor's gradient (D = U' + skip)
    TRY(conv_bwd(c, d + ".2", c.buf(c.pl.da[j]), ci, c.buf(c.pl.dl[j]), gA, ci, i, gB));
    TRY(conv_bwd(c, d + ".0", c.buf(c.pl.dd[j]), ci, c.buf(c.pl.da[j]), gB, ci, i, dD));
    // ConvTranspose3d: input L = the deeper level's output
    const int cin = (j == 0) ? h->hc[L] : h->hc[i + 1];
    const float* Lin = (j == 0) ? c.buf(c.pl.fo) : c.buf(c.pl.dl[j - 1]);
    const long long Pl = npx(h, i + 1, c.B, c.F, c.H, c.W);
    float* dU = c.buf(c.pl.col);
    HIPCHK(tr::launch_shuffle(dD, ci, dU, 4 * ci, ci, c.B * c.F, c.H >> (i + 1), c.W >> (i + 1), 0, c.s));
    TRY(colsum(c, dD, ci, ci, npx(h, i, c.B, c.F, c.H, c.W), c.G(u + ".bias")));
    tr::TGemm g;  // dWu[c][n] = sum_pl L[pl][c] dU[pl][n]
    g.A = Lin; g.sam = 1; g.sak = cin;
    g.B = dU; g.sbk = 4LL * ci; g.sbn = 1;
    g.C = c.G(u + ".weight"); g.scm = 4LL * ci; g.scn = 1;
    g.M = cin; g.N = 4 * ci; g.K = (int)Pl;
    TRY(gemm(c, g, true));
    tr::TGemm e;  // dL = dU . Wu^T
    e.A = dU; e.sam = 4LL * ci; e.sak = 1;
    e.B = c.P(u + ".weight"); e.sbk = 1; e.sbn = 4LL * ci;
    e.C = gA; e.scm = cin; e.scn = 1;
    e.M = (int)Pl; e.N = cin; e.K = 4 * ci;
    TRY(gemm(c, e, false));
  }
  const int cL = h->hc[L];
  TRY(conv_bwd(c, "st_fusion.2", c.buf(c.pl.fa), cL, c.buf(c.pl.fo), gA, cL, L, gB));
  TRY(conv_bwd(c, "st_fusion.0", c.buf(c.pl.pool[L - 1]), h->hc[L - 1], c.buf(c.pl.fa), gB, cL, L, gA));
  for (int i = L - 1; i >= 0; --i) {  // gA = gradient of pool[i]
    const int ci = h->hc[i];
    const std::string p = "encoders." + std::to_string(i);
    float* de = c.buf(c.pl.gskip[i]);  // in place: skip gradient + the pool's routed gradient
    HIPCHK(tr::launch_maxpool2_bwd(c.buf(c.pl.e[i]), ci, gA, ci, de, ci, de, ci, ci, c.B, c.F, c.H >> (i + 1),
                                   c.W >> (i + 1), c.s));
    TRY(conv_bwd(c, p + ".2", c.buf(c.pl.ea[i]), ci, c.buf(c.pl.e[i]), de, ci, i, gB));
    const float* Xin = i == 0 ? x : c.buf(c.pl.pool[i - 1]);
    const int cin = i == 0 ? 1 : h->hc[i - 1];
    TRY(conv_bwd(c, p + ".0", Xin, cin, c.buf(c.pl.ea[i]), gB, ci, i, i == 0 ? nullptr : gA));
  }
  return KDLAE_OK;
}

}  // namespace

extern "C" {

int kdlae_st_create(const kdlae_s_config* cfg, int device, kdlae_st_handle** out) {
  if (!cfg || !out) return fail(KDLAE_ESTATE, "null argument");
  *out = nullptr;
  if (cfg->inp_channels != 1 || cfg->out_channels != 1)
    return fail(KDLAE_EINVAL_CONFIG, "KDLAE_student training: inp/out_channels must be 1 (forward unsqueezes a [B,F,H,W] input)");
  if (cfg->kernel_size != 3) return fail(KDLAE_EINVAL_CONFIG, "kernel_size must be 3 on the HIP path");
  if (cfg->num_hidden < 2 || cfg->num_hidden > 8) return fail(KDLAE_EINVAL_CONFIG, "2..8 hidden_channels supported");
  auto* h = new kdlae_st_handle();
  h->cfg = *cfg;
  h->device = device;
  h->L = cfg->num_hidden - 1;
  for (int i = 0; i < cfg->num_hidden; ++i) {
    if (cfg->hidden_channels[i] <= 0 || cfg->hidden_channels[i] > 512) {
      delete h;
      return fail(KDLAE_EINVAL_CONFIG, "bad hidden_channels");
    }
    if (cfg->hidden_channels[i] % 4) {  // the step's pool / gather kernels move float4 channel groups
      delete h;
      return fail(KDLAE_EINVAL_CONFIG,
                  "KDLAE_student training on the HIP path needs hidden_channels divisible by 4 (inference takes any)");
    }
    h->hc.push_back(cfg->hidden_channels[i]);
  }
  auto add = [&](const std::string& k, int64_t n) {
    h->names.push_back(k);
    h->numel.push_back(n);
    h->offset.push_back(h->total);
    h->off[k] = h->total;
    h->total += (n + 3) / 4 * 4;  // 16-byte aligned keys (pads stay zero)
  };
  auto blk = [&](const std::string& p, int cin, int cout) {
    add(p + ".0.weight", (int64_t)cout * cin * 27);
    add(p + ".0.bias", cout);
    add(p + ".2.weight", (int64_t)cout * cout * 27);
    add(p + ".2.bias", cout);
  };
  int cin = 1;
  for (int i = 0; i < h->L; ++i) {
    blk("encoders." + std::to_string(i), cin, h->hc[i]);
    cin = h->hc[i];
  }
  blk("st_fusion", cin, h->hc[h->L]);
  for (int j = 0, i = h->L - 1; i >= 0; --i, ++j) {
    const int cu = (i == h->L - 1) ? h->hc[h->L] : h->hc[i + 1];
    add("upconv_layers." + std::to_string(j) + ".weight", (int64_t)cu * h->hc[i] * 4);
    add("upconv_layers." + std::to_string(j) + ".bias", h->hc[i]);
  }
  for (int j = 0, i = h->L - 1; i >= 0; --i, ++j) blk("decoders." + std::to_string(j), h->hc[i], h->hc[i]);
  add("out_conv.weight", h->hc[0]);
  add("out_conv.bias", 1);
  *out = h;
  return KDLAE_OK;
}

int kdlae_st_destroy(kdlae_st_handle* h) {
  delete h;
  return KDLAE_OK;
}

int kdlae_st_num_params(const kdlae_st_handle* h) { return h ? (int)h->names.size() : -1; }

int kdlae_st_param_info(const kdlae_st_handle* h, int i, const char** name, int64_t* numel, int64_t* offset) {
  if (!h || i < 0 || i >= (int)h->names.size()) return fail(KDLAE_EPARAM, "param index out of range");
  if (name) *name = h->names[i].c_str();
  if (numel) *numel = h->numel[i];
  if (offset) *offset = h->offset[i];
  return KDLAE_OK;
}

int64_t kdlae_st_num_floats(const kdlae_st_handle* h) { return h ? h->total : -1; }

int64_t kdlae_st_workspace_bytes(const kdlae_st_handle* h, int B, int F, int H, int W) {
  if (!h) return -1;
  const int m = 1 << h->L;
  if (B <= 0 || F <= 0 || H <= 0 || W <= 0 || H % m || W % m) {
    fail(KDLAE_EINVAL_SHAPE, "B, F, H, W must be positive with H, W divisible by 2^(levels)");
    return -1;
  }
  return (int64_t)make_plan(h, B, F, H, W).total;
}

int kdlae_st_forward(kdlae_st_handle* h, const float* theta, const float* x, int B, int F, int H, int W, float* out,
                     void* workspace, int64_t workspace_bytes, void* stream) {
  if (!h || !theta || !x || !out || !workspace) return fail(KDLAE_ESTATE, "null argument");
  const int m = 1 << h->L;
  if (B <= 0 || F <= 0 || H <= 0 || W <= 0 || H % m || W % m)
    return fail(KDLAE_EINVAL_SHAPE, "KDLAE_student needs H and W divisible by 2^(len(hidden_channels)-1)");
  Ctx c{h, theta, nullptr, reinterpret_cast<char*>(workspace), make_plan(h, B, F, H, W), (hipStream_t)stream,
        B, F, H, W};
  if ((int64_t)c.pl.total > workspace_bytes) return fail(KDLAE_ESTATE, "training workspace too small");
  // the 32-bit limits that apply: the GEMMs' M / K (pixel counts) are int, and so is col2im's element
  // index (P * cin) for the convs whose input gradient goes through columns; im2col, the column
  // matrices and the pixel-reduction kernel index in 64 bits (or fall back to the tiled GEMM)
  if ((long long)B * F * H * W >= (1LL << 31) || c.pl.col2im_max >= (1LL << 31))
    return fail(KDLAE_EINVAL_SHAPE, "batch too large: B*F*H*W and P*cin of a column-gradient conv must be < 2^31");
  DeviceGuard dg(h->device);
  h->valid = false;
  TRY(net_fwd(c, x, out));
  h->valid = true;
  h->B = B;
  h->F = F;
  h->H = H;
  h->W = W;
  h->ws = workspace;
  h->x = x;
  return KDLAE_OK;
}

int kdlae_st_backward(kdlae_st_handle* h, const float* theta, const float* dout, float* grad, void* workspace,
                      int64_t workspace_bytes, void* stream) {
  if (!h || !theta || !dout || !grad || !workspace) return fail(KDLAE_ESTATE, "null argument");
  if (!h->valid || h->ws != workspace)
    return fail(KDLAE_ESTATE, "kdlae_st_backward needs a preceding kdlae_st_forward on the same workspace");
  Ctx c{h, theta, grad, reinterpret_cast<char*>(workspace), make_plan(h, h->B, h->F, h->H, h->W),
        (hipStream_t)stream, h->B, h->F, h->H, h->W};
  if ((int64_t)c.pl.total > workspace_bytes) return fail(KDLAE_ESTATE, "training workspace too small");
  DeviceGuard dg(h->device);
  c.main_s = c.s;
  if (!debug_flag("train_serial")) {
    if (!h->side) {
      HIPCHK(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming));
    }
    c.side = h->side;
  }
  HIPCHK(hipMemsetAsync(grad, 0, (size_t)h->total * sizeof(float), c.s));  // the pad floats stay zero
  HIPCHK(hipMemsetAsync(c.buf(c.pl.zb), 0, 64 * sizeof(float), c.s));
  return net_bwd(c, h->x, dout);
}

int64_t kdlae_train_l1frames_scratch_floats(void) { return tr::l1frames_scratch_floats(); }

int kdlae_train_l1frames(const float* pred, const float* target, int N, int frames, int64_t hw, float l1loss_weight,
                         float temporal_weight, float binary, int reduction, float* dpred, float* loss, float* scratch,
                         void* stream) {
  if (!pred || !target || !dpred || !loss || !scratch) return fail(KDLAE_ESTATE, "null argument");
  if (N <= 0 || frames <= 0 || hw <= 0) return fail(KDLAE_EINVAL_SHAPE, "empty loss input");
  if (reduction != 0 && reduction != 1)
    return fail(KDLAE_EINVAL_CONFIG, "reduction: 0 = 'mean', 1 = 'sum' ('max' / 'mix' are not implemented)");
  HIPCHK(tr::launch_l1frames(pred, target, N, frames, hw, l1loss_weight, temporal_weight, binary, reduction, dpred,
                             loss, scratch, (hipStream_t)stream));
  return KDLAE_OK;
}

}  // extern "C"
