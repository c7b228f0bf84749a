// Kernel self-test entry points (include/kdlae.h, "Kernel self-test entry points"): single launches
// of internal kernel families on caller buffers, so tests/test_kernel_variants_gpu.py can reach every
// compiled variant against a torch reference.  Not part of the drop-in boundary; nothing here is on
// a forward / training path.
#include <hip/hip_runtime.h>

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
