// Kernel self-test entry points (include/kdlae.h, "Kernel self-test entry points"): single launches
// of internal kernel families on caller buffers, so tests/test_kernel_variants_gpu.py can reach every
// compiled variant against a torch reference.  Not part of the drop-in boundary; nothing here is on
// a forward / training path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/kdlae.h"
#include "runtime.h"
#include "train_kernels.h"

namespace tr = kdlae::train;
using kdlae::fail;

extern "C" int kdlae_debug_tgemm(const kdlae_debug_tgemm_desc* d, void* stream) {
  if (!d) return fail(KDLAE_EINVAL_CONFIG, "null descriptor");
  tr::TGemm g;
  g.A = d->A; g.sam = d->sam; g.sak = d->sak; g.amode = d->amode;
  g.B = d->B; g.sbk = d->sbk; g.sbn = d->sbn; g.bmode = d->bmode;
  g.C = d->C; g.scm = d->scm; g.scn = d->scn;
  g.bias = d->bias;
  g.R = d->R; g.srm = d->srm; g.srn = d->srn;
  g.rs = d->rs;
  g.M = d->M; g.N = d->N; g.K = d->K; g.nz1 = d->nz1; g.nz2 = d->nz2;
  g.bA1 = d->bA1; g.bA2 = d->bA2; g.bB1 = d->bB1; g.bB2 = d->bB2; g.bC1 = d->bC1; g.bC2 = d->bC2;
  g.bR1 = d->bR1; g.bR2 = d->bR2; g.brs1 = d->brs1; g.brs2 = d->brs2;
  g.Bn = d->Bn; g.H = d->H; g.W = d->W; g.Cg = d->Cg; g.dil = d->dil; g.lda = d->lda; g.ldb = d->ldb;
  g.partial = d->partial;
  g.c_pad_ok = d->c_pad_ok != 0;
  g.F = d->F > 0 ? d->F : 1;
  const size_t cap = d->partial ? (size_t)d->partial_floats : 0;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (d->route) {
    case 0: e = tr::launch_tgemm(g, cap, s); break;
    case 1:
      if (!tr::tgemm_rows_eligible(g)) return fail(KDLAE_EINVAL_CONFIG, "not eligible for the row-streaming kernel");
      e = tr::launch_tgemm_rows(g, s);
      break;
    case 2:
      if (!cap || !tr::tgemm_cols_eligible(g)) return fail(KDLAE_EINVAL_CONFIG, "not eligible for the pixel kernel");
      e = tr::launch_tgemm_cols(g, cap, s);
      break;
    case 3: e = tr::launch_tgemm_tiled(g, cap, s); break;
    default: return fail(KDLAE_EINVAL_CONFIG, "route must be 0..3");
  }
  if (e != hipSuccess) return fail(KDLAE_EHIP, std::string("kdlae_debug_tgemm: ") + hipGetErrorString(e));
  return KDLAE_OK;
}

extern "C" int kdlae_debug_gemm_variant(int family, int i, int* v) {
  if (!v) return 0;
  return kdlae::gemm_variant_entry(family, i, v) ? 1 : 0;
}

extern "C" int kdlae_debug_gemm(const kdlae_debug_gemm_desc* d, void* stream) {
  using kdlae::ceil_div;
  if (!d || !d->A || !d->Wp || !d->out) return fail(KDLAE_EINVAL_CONFIG, "null descriptor or operand");
  if (d->Bn < 1 || d->F < 1 || d->H < 1 || d->W < 1 || d->ntiles < 1 || d->kgroups < 1 || d->N < 1 ||
      d->N > 16 * d->ntiles || d->NT < 1 || d->KG < 1)
    return fail(KDLAE_EINVAL_SHAPE, "bad GEMM geometry");
  if (d->ksize != 1 && d->ksize != 3) return fail(KDLAE_EINVAL_SHAPE, "ksize must be 1 or 3");
  const int kt = d->ksize == 3 ? d->kt : 1;
  if (d->ksize == 3 && ((kt != 1 && kt != 3) || d->kgroups != 9 * kt * d->cg_per_tap || d->lda < 16 * d->cg_per_tap))
    return fail(KDLAE_EINVAL_SHAPE, "implicit conv needs kgroups = 9 kt cg_per_tap and lda >= 16 cg_per_tap");
  if (d->ksize == 1 && d->lda < 16 * d->kgroups) return fail(KDLAE_EINVAL_SHAPE, "lda < K");
  if (d->out_mode == 0 && d->ldo < d->N) return fail(KDLAE_EINVAL_SHAPE, "ldo < N");
  if (d->out_mode == 1 && (d->H % 2 || d->W % 2 || d->ldo < 4 * d->N)) return fail(KDLAE_EINVAL_SHAPE, "unshuffle geometry");
  if (d->out_mode == 2 && (d->N % 4 || d->ldo < d->N / 4)) return fail(KDLAE_EINVAL_SHAPE, "shuffle geometry");
  if (d->route != 0 && d->route != 1) return fail(KDLAE_EINVAL_CONFIG, "route must be 0 or 1");
  const long long HW = (long long)d->F * d->H * d->W;
  kdlae::GemmParams p{};
  p.A = d->A;
  p.lda = d->lda;
  p.cg_per_tap = d->cg_per_tap;
  p.kgroups = d->kgroups;
  p.ksize = d->ksize;
  p.dil = d->dil > 0 ? d->dil : 1;
  // the caller hands f32 fragment order (runtime.h pack_fragments); the GEMM kernels read split
  // fragment order (mfma3.h): convert into scratch owned by this call
  hipStream_t s = (hipStream_t)stream;
  const int nimg_w = d->w_img_stride ? d->Bn : 1;
  const long long w3_img = kdlae::split3_floats(d->ntiles, d->kgroups);
  float* w3 = nullptr;
  float* m3 = nullptr;
  struct Scratch {
    float** a;
    float** b;
    hipStream_t s;
    ~Scratch() {
      (void)hipStreamSynchronize(s);
      if (*a) (void)hipFree(*a);
      if (*b) (void)hipFree(*b);
    }
  } scratch{&w3, &m3, s};
  HIPCHK(hipMalloc(&w3, (size_t)(w3_img * nimg_w) * sizeof(float)));
  HIPCHK(kdlae::launch_split3(d->Wp, w3, d->ntiles, d->kgroups, nimg_w, d->w_img_stride, w3_img, s));
  p.Wp = w3;
  p.w_img_stride = d->w_img_stride ? w3_img : 0;
  p.ntiles = d->ntiles;
  p.N = d->N;
  p.bias = d->bias;
  p.out = d->out;
  p.ldo = d->ldo;
  p.R = d->R;
  p.ldr = d->ldr;
  p.ln = d->ln;
  p.ln_C = d->ln_C;
  p.relu = d->relu;
  p.Bn = d->Bn;
  p.H = d->H;
  p.W = d->W;
  p.F = d->F;
  p.kt = kt;
  p.out_mode = d->out_mode;
  p.tiles_per_img = (int)ceil_div(HW, kdlae::kGemmRows);
  p.total_tiles = d->Bn * p.tiles_per_img;
  p.kchunks = d->group_tiles ? 1 : (int)ceil_div(d->kgroups, d->KG);
  p.group_tiles = d->group_tiles;
  if (d->Wm) {  // the per-image folded projection: kgroups x kgroups tiles per image
    const long long m3_img = kdlae::split3_floats(d->kgroups, d->kgroups);
    HIPCHK(hipMalloc(&m3, (size_t)(m3_img * d->Bn) * sizeof(float)));
    HIPCHK(kdlae::launch_split3(d->Wm, m3, d->kgroups, d->kgroups, d->Bn, d->wm_img_stride, m3_img, s));
    p.Wm = m3;
    p.wm_img_stride = m3_img;
  }
  p.bias_m = d->bias_m;
  p.out1 = d->out1;
  p.ldo1 = d->ldo1;
  if (d->ln && !d->Wm && (p.kchunks > 1 || d->kgroups * 16 != d->ln_C)) {
    if (!d->stats || d->ln_C > 512 || d->lda % 4) return fail(KDLAE_EINVAL_CONFIG, "chunked LN needs stats scratch");
    HIPCHK(kdlae::launch_ln_stats(d->A, d->lda, d->ln_C, (long long)d->Bn * HW, d->stats, s));
    p.stats = d->stats;
  }
  const int gy = d->group_tiles ? (int)ceil_div(d->ntiles, d->group_tiles) : (int)ceil_div(d->ntiles, d->NT);
  p.tiles_per_block = d->tiles_per_block > 0 ? d->tiles_per_block
                                             : kdlae::gemm_tiles_per_block(p.total_tiles, gy, d->group_tiles != 0, d->wpe);
  const int gx = (int)ceil_div(p.total_tiles, p.tiles_per_block);
  const hipError_t e = kdlae::launch_gemm_route(p, d->NT, d->KG, d->wpe, gx, d->route, s);
  if (e != hipSuccess) return fail(KDLAE_EHIP, std::string("kdlae_debug_gemm: ") + hipGetErrorString(e));
  return KDLAE_OK;
}

extern "C" int kdlae_debug_gram(const kdlae_debug_gram_desc* d, void* stream) {
  if (!d || !d->qkv || !d->wdw || !d->v_out || !d->partial || !d->reduced) return fail(KDLAE_EINVAL_CONFIG, "null operand");
  if (d->heads < 1 || d->C % d->heads || (d->C / d->heads) % 16 || d->C / d->heads > 128 || d->Bn < 1 || d->H < 1 ||
      d->W < 1 || d->ld < 3 * d->C || d->ldv < d->C)
    return fail(KDLAE_EINVAL_SHAPE, "bad Gram geometry (Ch = C / heads must be 16..128, a multiple of 16)");
  if (d->route < 0 || d->route > 2) return fail(KDLAE_EINVAL_CONFIG, "route must be 0..2");
  kdlae::GramParams p{};
  p.qkv = d->qkv;
  p.ld = d->ld;
  p.wdw = d->wdw;
  p.bdw = d->bdw;
  p.v_out = d->v_out;
  p.ldv = d->ldv;
  p.partial = d->partial;
  p.C = d->C;
  p.heads = d->heads;
  p.Ch = d->C / d->heads;
  p.Bn = d->Bn;
  p.H = d->H;
  p.W = d->W;
  // the engine's slot count (kdlae_t.cpp nslots_for)
  if (d->W % 16 == 0) {
    p.nslots = (d->W / 16) * std::max(1, std::min(8, (d->H + 31) / 32));
  } else {
    const int steps = (d->H * d->W + 63) / 64;
    p.nslots = std::max(1, std::min(64, (steps + 15) / 16));
  }
  const int CT = p.Ch / 16;
  p.slot_floats = CT * CT * 256 + 2 * p.Ch;
  p.zeros = d->route == 0 ? d->zeros : nullptr;
  if ((long long)d->Bn * d->heads * p.nslots * p.slot_floats > d->partial_floats)
    return fail(KDLAE_EINVAL_SHAPE, "partial scratch too small");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(kdlae::launch_dwconv_gram_route(p, d->route, s));
  HIPCHK(kdlae::launch_gram_reduce(p.partial, d->reduced, d->Bn, d->heads, p.nslots, p.slot_floats, s));
  return KDLAE_OK;
}

extern "C" int kdlae_debug_ln(const kdlae_debug_ln_desc* d, void* stream) {
  if (!d || d->C < 1 || d->C > 512 || d->P < 1) return fail(KDLAE_EINVAL_SHAPE, "bad LayerNorm geometry");
  hipStream_t s = (hipStream_t)stream;
  const bool generic = d->route == 1;
  hipError_t e;
  if (d->dir == 0) {
    if (!d->x || !d->w || !d->y || !d->stats) return fail(KDLAE_EINVAL_CONFIG, "null operand");
    e = tr::launch_ln_fwd(d->x, d->ldx, d->w, d->b, d->C, d->P, d->biasfree, d->y, d->ldy, d->stats, s, generic);
  } else {
    if (!d->x || !d->w || !d->dy || !d->dx || !d->stats || !d->part || d->nblk < 1)
      return fail(KDLAE_EINVAL_CONFIG, "null operand");
    e = tr::launch_ln_bwd(d->dy, d->ldd, d->x, d->ldx, d->w, d->stats, d->C, d->P, d->biasfree, d->R, d->ldr, d->dx,
                          d->lddx, d->part, d->nblk, s, generic);
  }
  if (e != hipSuccess) return fail(KDLAE_EHIP, std::string("kdlae_debug_ln: ") + hipGetErrorString(e));
  return KDLAE_OK;
}

extern "C" int kdlae_debug_small_in(const kdlae_debug_small_in_desc* d, void* stream) {
  if (!d || !d->in || !d->w || !d->out) return fail(KDLAE_EINVAL_CONFIG, "null operand");
  if (d->Bn < 1 || d->H < 1 || d->W < 1 || d->Cin < 1 || d->Cout < 16 || d->ldo < d->Cout)
    return fail(KDLAE_EINVAL_SHAPE, "bad small-input conv geometry");
  kdlae::SmallInParams p{};
  p.in = d->in;
  p.sb = d->sb;
  p.sc = d->sc;
  p.sy = d->sy;
  p.sx = d->sx;
  p.st = d->st;
  p.in_sub = d->in_sub;
  p.Cin = d->Cin;
  p.Cout = d->Cout;
  p.dil = d->dil > 0 ? d->dil : 1;
  p.kt = d->kt;
  p.F = d->F > 0 ? d->F : 1;
  p.w = d->w;
  p.bias = d->bias;
  p.out = d->out;
  p.ldo = d->ldo;
  p.Bn = d->Bn;
  p.H = d->H;
  p.W = d->W;
  p.vh = d->vh;
  p.vw = d->vw;
  p.relu = d->relu;
  const hipError_t e = kdlae::launch_conv_small_in(p, (hipStream_t)stream);
  if (e != hipSuccess) return fail(KDLAE_EHIP, std::string("kdlae_debug_small_in: ") + hipGetErrorString(e));
  return KDLAE_OK;
}
