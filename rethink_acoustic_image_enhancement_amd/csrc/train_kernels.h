// Launch interface of the KDLAE-T training kernels (train.hip, gfx950).
//
// The training path keeps every activation NHWC fp32 (pixel-major, channels contiguous, pixel
// stride `ld`) like the inference path, but reads weights in their natural state_dict layout
// (OIHW) straight from the caller's flat parameter buffer: weights change every optimizer step,
// so there is no packed copy to keep in sync.
#pragma once
#include <hip/hip_runtime.h>

namespace kdlae {
namespace train {

// Generic batched MFMA GEMM:  C(m,n) = alpha * sum_k A(m,k) B(k,n)  [+ bias[n]]  [+ rs[n] * R(m,n)]
// (rs null -> coefficient 1).  R may alias C (read then written by the same lane).
//   amode 0: A(m,k) = A[m*sam + k*sak]
//   amode 1: implicit im2col of a 3x3 conv (dilation dil, zero padding dil) over an NHWC view A with
//            pixel stride lda: m = pixel, k = tap*Cg + c.
//   bmode 0: B(k,n) = B[k*sbk + n*sbn]
//   bmode 1: B(k = pixel, n = c) = B[(pixel shifted by tap z2)*ldb + c] with zero padding (conv dW).
//   bmode 2: 3x3 weight OIHW, k = tap*Cg + c: B = W[n][c][tap]      (conv forward)
//   bmode 3: 3x3 weight OIHW, k = tap*Cg + c: B = W[c][n][8 - tap]  (conv dX, a transposed conv)
//   bmode 4: implicit 3x3x3 im2col of an NDHWC view B ([Bn][F][H][W] pixels at stride sbk):
//            B(k = pixel, n = tap*Cg + c) = B[(pixel shifted by tap) * sbk + c], zero padding 1
//            (Conv3d weight gradient; pixel-reduction kernel only, Cg % 16 == 0, W % 16 == 0)
// Batch: z = z1 * nz2 + z2, every operand offset by z1*b?1 + z2*b?2.
// splits > 1: K is cut into `splits` chunks whose partial sums go to `partial`
// ([batch][splits][M][N]) and a fixed-order reduce applies the epilogue (deterministic).
struct TGemm {
  const float* A = nullptr; long long sam = 0, sak = 0; int amode = 0;
  const float* B = nullptr; long long sbk = 0, sbn = 0; int bmode = 0;
  float* C = nullptr; long long scm = 0, scn = 0;
  const float* bias = nullptr;
  const float* R = nullptr; long long srm = 0, srn = 0;
  const float* rs = nullptr;
  float alpha = 1.f;
  int M = 0, N = 0, K = 0;
  int nz1 = 1, nz2 = 1;
  long long bA1 = 0, bA2 = 0, bB1 = 0, bB2 = 0, bC1 = 0, bC2 = 0, bR1 = 0, bR2 = 0, brs1 = 0, brs2 = 0;
  // im2col geometry (amode 1 / bmode 1..4; F: frames of the 3x3x3 bmode 4)
  int Bn = 0, H = 0, W = 0, Cg = 0, dil = 1, F = 1; long long lda = 0, ldb = 0;
  int splits = 1; float* partial = nullptr;
  // the C view's row pad [N, ld4(N)) belongs to nobody else (a ld-rounded private buffer): a
  // kernel may store whole float4 quads there (zeros: the weights past N are zero)
  bool c_pad_ok = false;
};
// Launch; picks split-K itself when `partial` (capacity `partial_cap` floats) is given.
hipError_t launch_tgemm(TGemm g, size_t partial_cap, hipStream_t s);
// the tiled 64 x 64 / 128 x 64 kernels only (launch_tgemm's fallback: small grids, im2col modes)
hipError_t launch_tgemm_tiled(TGemm g, size_t partial_cap, hipStream_t s);
// Row-streaming kernel (train_rows.hip) for plain contractions with k-contiguous A rows and no
// split-K: weights staged in LDS in MFMA fragment order, A streamed to VGPRs.  launch_tgemm routes
// every eligible call there.
bool tgemm_rows_eligible(const TGemm& g);
hipError_t launch_tgemm_rows(const TGemm& g, hipStream_t s);
// Pixel-reduction kernel (train_cols.hip) for split-K contractions over pixels with channel-
// contiguous operands (1x1 dW, MDTA Gram / dA): split-K partials + launch_tgemm_reduce.
bool tgemm_cols_eligible(const TGemm& g);
hipError_t launch_tgemm_cols(TGemm g, size_t partial_cap, hipStream_t s);
// fixed-order sum of g.splits partials ([batch][splits][M][N] at g.partial) + the epilogue into C
hipError_t launch_tgemm_reduce(const TGemm& g, hipStream_t s);

// LayerNorm over channels per pixel (KDLAE_model.py:50-52 BiasFree, :67-70 WithBias), eps 1e-5.
// forward: y = LN(x) * w (+ b); stats[p] = (mean, rstd).  generic (self-test): the one-wave-per-pixel
// kernels the lane-group ones fall back to for misaligned views / C % 4 != 0
hipError_t launch_ln_fwd(const float* x, int ldx, const float* w, const float* b, int C, long long P, int biasfree,
                         float* y, int ldy, float* stats, hipStream_t s, bool generic = false);
// backward: dx = R + dLN(dy) (R may be null or alias dx); per-block partial dw [nblk][C], db [nblk][C]
// reduced into gw / gb by the caller's column reduce.  Returns the number of blocks used in *nblk.
hipError_t launch_ln_bwd(const float* dy, int ldd, const float* x, int ldx, const float* w, const float* stats,
                         int C, long long P, int biasfree, const float* R, int ldr, float* dx, int lddx,
                         float* part, int nblk, hipStream_t s, bool generic = false);

// depthwise 3x3 (padding 1) over NHWC: out[p,c] = sum_t w[c][t] in[p+off_t, c] (+ b[c]); flip=1 uses
// w[c][8-t] (dX of the same conv).
hipError_t launch_dw_fwd(const float* in, int ldi, const float* w, const float* b, int flip, int C, int Bn, int H,
                         int W, float* out, int ldo, hipStream_t s);
// Fused depthwise kernels (train_dwg.hip).  GDFN forward: yd = dw(y) (+b) over both halves
// (x1 at [0, hid), x2 at [hid, 2 hid)) and g = gelu_erf(yd1) * yd2 (yd may be null: not stored).  Backward: dy = dw^T(dyd) and the
// weight / bias gradient partials part[dwg_blocks][10 C] (C = 2 hid; columns [9 C weights | C biases]),
// with dyd = gate_bwd(dg, yd) computed on the fly (dwgate) or given (dw_bwd, C channels).
int dwg_blocks(int Bn, int H, int W);
hipError_t launch_dwgate_fwd(const float* y, int ldi, const float* w, const float* b, int hid, int Bn, int H, int W,
                             float* yd, int ldyd, float* g, int ldg, hipStream_t s);
hipError_t launch_dwgate_bwd(const float* dg, int ldg, const float* yd, int ldyd, const float* yin, int ldi,
                             const float* w, int hid, int Bn, int H, int W, float* dy, int lddy, float* part,
                             hipStream_t s);
// GDFN backward from (dg, y) alone: yd recomputed from y with the forward's arithmetic (same bits as
// launch_dwgate_bwd given the stored yd); the forward then passes yd = null to launch_dwgate_fwd.
hipError_t launch_dwgate_bwd_rc(const float* dg, int ldg, const float* yin, int ldi, const float* w, const float* b,
                                int hid, int Bn, int H, int W, float* dy, int lddy, float* part, hipStream_t s);
hipError_t launch_dw_bwd(const float* dyd, int ldd, const float* yin, int ldi, const float* w, int C, int Bn, int H,
                         int W, float* dy, int lddy, float* part, hipStream_t s);

// 3x3 conv weight gradient with a side of <= 4 channels (train_small.hip): part[nblk][Cout * Cin * 9]
// (OIHW order) partials of dW = sum_p dY[p] (x) X[p + off_t], summed by the caller's column reduce
bool dw3_small_ok(int Cin, int Cout);
int dw3_small_blocks(long long P, int Cin, int Cout, size_t part_cap);
hipError_t launch_dw3_small(const float* dy, int ldd, const float* x, int ldx, int Cin, int Cout, int Bn, int H, int W,
                            int dil, float* part, int nblk, hipStream_t s);

// column reductions: out[seg][c] = sum over rows of segment seg of f(x[r][c]); f = x or x^2.
// Two passes (partials then a fixed-order reduce), deterministic.
hipError_t launch_colsum(const float* x, int ldx, int ncols, long long rows_per_seg, int nseg, int square,
                         float* part, int nblk, hipStream_t s);
// out[seg][c] (= or +=) scale * sum_b part[(seg * nblk + b) * pstride + c], c < ncols (pstride 0 = ncols)
hipError_t launch_part_reduce(const float* part, int nblk, int ncols, int nseg, float* out, int accumulate,
                              float scale, hipStream_t s, int pstride = 0);

// out[c] = scale * sum_b part[b * pstride + c] for up to kRedBatch independent reductions, one launch
struct RedDesc {
  const float* part = nullptr;
  float* out = nullptr;
  int nblk = 0, ncols = 0, pstride = 0;
  float scale = 1.f;
};
constexpr int kRedBatch = 8;
struct RedBatch {
  RedDesc d[kRedBatch];
  int n;
  int cg_prefix[kRedBatch + 1];
};
hipError_t launch_part_reduce_multi(const RedDesc* d, int n, hipStream_t s);

// MDTA core (KDLAE_model.py:130-140), per (image, head) with Ch x Ch matrices:
// A = softmax(t[h] * G / (max(nq,eps) max(nk,eps)^T)), nq/nk from sumsq [B][2C] (q at [0,C), k at [C,2C)).
hipError_t launch_attn_softmax(const float* G, const float* sumsq, const float* temp, int Bn, int C, int heads,
                               float* Attn, hipStream_t s);
// Backward of the softmax and the normalisations: Mq = t dS / (nq nk^T); cq/ck = -(sum dS*Ghat)*t / n^2
// (0 where the norm was clamped); dtemp partial [B][heads].
hipError_t launch_attn_bwd(const float* G, const float* sumsq, const float* temp, const float* Attn,
                           const float* dAttn, int Bn, int C, int heads, float* Mq, float* cq, float* ck,
                           float* dtemp_part, hipStream_t s);

// PixelUnshuffle(2) (dir 0: [B,2h,2w,C] -> [B,h,w,4C]) / PixelShuffle(2) (dir 1: [B,h,w,4C] -> [B,2h,2w,C]);
// h, w are the low-resolution sizes, C the low-channel count.
hipError_t launch_shuffle(const float* in, int ldi, float* out, int ldo, int C, int Bn, int h, int w, int dir,
                          hipStream_t s);
// 3x3 weights OIHW -> [9 Cg][N] row-major implicit-GEMM B operand (mode 2: conv, B(t Cg + c, n) =
// W[n][c][t]; mode 3: transposed conv, W[c][n][8 - t]); then TGemm bmode 0 with sbk = N, sbn = 1
hipError_t launch_pack_w3(const float* W, int Cg, int N, int mode, float* out, hipStream_t s);
// out[p, 0:C] (= or +=) in[p, 0:C]; zero_to > C also zeroes out[p, C:zero_to] (a padded copy)
hipError_t launch_copy_cols(const float* in, int ldi, float* out, int ldo, int C, long long P, int accumulate,
                            hipStream_t s, int zero_to = 0);
// NCHW [B,C,H,W] -> NHWC view (out[p*ldo + c]); accumulate adds
hipError_t launch_nchw_to_nhwc(const float* in, int C, int Bn, long long HW, float* out, int ldo, int accumulate,
                               hipStream_t s);
// NHWC view -> NCHW [B,C,H,W]; out = in (+ add[B,C,H,W] if add)
hipError_t launch_nhwc_to_nchw(const float* in, int ldi, const float* add, int C, int Bn, long long HW, float* out,
                               hipStream_t s);

// L1LossSr term (Train/basicsr/models/losses/losses.py:135-194) for one (pred, target) pair:
// grad = w_l1 * sign(pred - target) / n;  part[blk] = (sum |pred-target|, sum |bin(pred)-bin(target)|)
hipError_t launch_l1sr(const float* pred, const float* target, long long n, float w_l1, float* grad, float* part,
                       int nblk, hipStream_t s);
// loss = sum_i (wl1_i / n_i * sum_l1_i + wsh_i / n_i * sum_sh_i) over up to two terms -> out[0]
hipError_t launch_l1sr_final(const float* part0, int nblk0, long long n0, float wl0, float ws0, const float* part1,
                             int nblk1, long long n1, float wl1, float ws1, float* out, hipStream_t s);

// grad-norm clip + AdamW (torch.nn.utils.clip_grad_norm_ + torch.optim.AdamW, base_model.py / image_restoration_model.py:216-218)
hipError_t launch_sumsq(const float* g, long long n, float* part, int nblk, hipStream_t s);
// state[0] = total norm of (gscale * g), state[1] = gscale * min(1, max_norm / (norm + 1e-6)) (or gscale if max_norm <= 0)
hipError_t launch_clip_coef(const float* part, int nblk, float gscale, float max_norm, float* state, hipStream_t s);
hipError_t launch_adamw(float* p, const float* g, float* m, float* v, long long n, const float* state, float lr,
                        float beta1, float beta2, float eps, float wd, int step, hipStream_t s);

// Mixing_Augment.mixup (image_restoration_model.py:32-34) on a [B][per] tensor, perm on device; out != in
hipError_t launch_mixup(const float* in, float* out, int B, long long per, const int* perm, float lam, hipStream_t s);
// BaseModel.model_ema (Train/basicsr/models/base_model.py:54-62)
hipError_t launch_ema(float* ema, const float* theta, long long n, float decay, hipStream_t s);

}  // namespace train
}  // namespace kdlae
