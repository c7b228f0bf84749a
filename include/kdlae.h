/*
 * kdlae.h — C ABI of the MI355X-native KDLAE path (libkdlae.so).
 *
 * The reference exposes no FFI: its boundary is the PyTorch nn.Module API
 * (SURVEY.md §8b).  These entry points are what a ctypes/cffi binding of
 * that module API binds; each one replaces the reference interface cited
 * beside it.  All pointers are device pointers unless marked host; tensors
 * are fp32, contiguous NCHW exactly as the reference consumes/produces them.
 * `stream` is a hipStream_t (0 = null stream).  Nothing here allocates,
 * frees or synchronises inside *_forward / *_pack_device: activations,
 * outputs, the flat parameter vector and the workspace are caller-owned;
 * the handle owns only the packed weights and their pack program.  Every
 * call makes the handle's device current and restores the caller's device
 * before returning.
 *
 * Error handling: every call returns KDLAE_OK (0) or one of the codes
 * below; kdlae_last_error() returns a thread-local message describing the
 * last failure on the calling thread.
 *
 * Environment: the library reads two variables, neither of which changes
 * results.  KDLAE_DEBUG (comma-separated flags, read when a KDLAE-T handle
 * builds its pack program: kdlae_t_prepare or the first pack) selects between kernel schedules that produce
 * the same bits: "no_attn_in_fusion" keeps the attention-output GEMM and the
 * LN + ffn.project_in GEMM separate (every block); "no_attn_in_split" keeps
 * them separate for the C = 96 blocks only (by default their first
 * project_in weight group is fused as well).  KDLAE_PROBE_DUMP
 * names a CSV file kdlae_t_probe_read writes per-launch timings to.
 * One more KDLAE_DEBUG flag is read on EVERY training call (kdlae_tt_forward /
 * kdlae_tt_backward / kdlae_tt_backward_marked), not at pack time:
 * "train_trace" brackets each training launch with a pair of HIP events and
 * synchronises the stream at the end of the call to dump them to
 * KDLAE_PROBE_DUMP.  It does not change results, but the synchronisation
 * removes the overlap of the bucketed all-reduce with the backward that the
 * gradient-ready marks exist for: diagnostics only, never in production.
 * "train_serial" (read by kdlae_tt_backward / kdlae_tt_backward_marked) keeps
 * every backward launch on the caller's stream; by default the weight-gradient
 * GEMMs and bias column sums run on a library-owned non-blocking side stream
 * that is forked from and joined back into the caller's stream inside the call
 * (every gradient-ready mark and the call's end follow a join), with the same
 * results either way.  "train_keep_yd" (read by kdlae_tt_forward; the backward
 * follows what the forward kept) stores the GDFN dwconv output for the
 * backward instead of having the backward recompute it from its input (A/B
 * only: same gradients bit for bit, 1 KiB per pixel more traffic each way);
 * "train_w3_raw" (read on every training call) has the 3x3 convs' implicit
 * GEMMs read the OIHW weights directly instead of a per-call [9 Cin][Cout]
 * repack (A/B only: same bits).
 */
#ifndef KDLAE_H_
#define KDLAE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  KDLAE_OK = 0,
  KDLAE_EINVAL_SHAPE = 1,   /* e.g. H or W not divisible by 8 (reference: RuntimeError from pixel_unshuffle) */
  KDLAE_EINVAL_CONFIG = 2,  /* ctor kwargs the HIP path does not support (message says which) */
  KDLAE_EHIP = 3,           /* a HIP runtime call failed; message carries hipGetErrorString */
  KDLAE_EPARAM = 4,         /* unknown / missing / wrongly sized state_dict entry */
  KDLAE_ENOTIMPL = 5,       /* dual_pixel_task=True: NameError in the reference (KDLAE_model.py:305-321) */
  KDLAE_ESTATE = 6          /* forward before commit_params, workspace too small, ... */
};

const char* kdlae_last_error(void);
int kdlae_abi_version(void);

/* ------------------------------------------------------------------ KDLAE-T
 * Ctor kwargs of KDLAE_teacher (KDLAE/KDLAE_model.py:205-218).  Strings are
 * mapped to flags: LayerNorm_type=='BiasFree' -> layernorm_biasfree=1,
 * static=="train" -> static_train=1, params=='cat' -> params_cat=1.
 */
typedef struct kdlae_t_config {
  int inp_channels;
  int out_channels;
  int dim;
  int num_blocks[4];
  int num_refinement_blocks;
  int heads[4];
  double ffn_expansion_factor;
  int bias;
  int layernorm_biasfree;
  int dual_pixel_task;
  int static_train;
  int params_cat;
} kdlae_t_config;

typedef struct kdlae_t_handle kdlae_t_handle;

/* replaces KDLAE_teacher.__init__ (KDLAE_model.py:205-268): validates the config, binds `device`. */
int kdlae_t_create(const kdlae_t_config* cfg, int device, kdlae_t_handle** out);
int kdlae_t_destroy(kdlae_t_handle* h);

/* state_dict surface (KDLAE_model.py:220-268 key layout; load_state_dict at KDLAE_T.ipynb:1074-1075).
 * kdlae_t_num_params / kdlae_t_param_info enumerate the expected keys and element counts, in
 * state_dict order.  The packed device layout (LN weight folded into 1x1 weights, NHWC/MFMA
 * fragment order) is produced ON THE DEVICE by the handle's pack program from the flat fp32
 * parameter vector (every key in that order, back to back; kdlae_t_params_numel floats):
 *   kdlae_t_pack_device(params = DEVICE flat vector) enqueues the pack on `stream` (no sync) and
 *     is what the nn.Module calls before every forward, so the packed copy never goes stale;
 *   kdlae_t_set_param stages one entry from HOST memory (strict: unknown key or numel mismatch
 *     -> KDLAE_EPARAM) and kdlae_t_commit_params packs the staged set (synchronous). */
int kdlae_t_num_params(const kdlae_t_handle* h);
int kdlae_t_param_info(const kdlae_t_handle* h, int index, const char** name, int64_t* numel);
int64_t kdlae_t_params_numel(const kdlae_t_handle* h);
/* Builds and uploads the handle's pack program (device allocation + one synchronous copy; the
 * program depends on the config only).  Optional: the first pack_device / commit_params does it
 * otherwise.  Call it once before capturing forwards into a HIP graph, so that no call inside the
 * capture allocates or synchronises. */
int kdlae_t_prepare(kdlae_t_handle* h);
int kdlae_t_pack_device(kdlae_t_handle* h, const float* params, int64_t numel, void* stream);
int kdlae_t_set_param(kdlae_t_handle* h, const char* name, const float* host_data, int64_t numel);
int kdlae_t_commit_params(kdlae_t_handle* h, void* stream);

/* Device bytes of caller-owned scratch needed by kdlae_t_forward for a B x H x W batch. */
int64_t kdlae_t_workspace_bytes(const kdlae_t_handle* h, int B, int H, int W);

/* replaces KDLAE_teacher.forward (KDLAE_model.py:270-336):
 *   img  [B, inp_channels, H, W]   ({"img"})
 *   rate [B, 1, H, W]              ({"denoise_rate"}; read only when params_cat)
 *   hq   [B, out_channels, H, W]   (out["hq"])
 *   sr   [B, out_channels, 2H, 2W] (out["sr"]; must be NULL iff static_train == 0)
 * H % 8 == 0 and W % 8 == 0 are required (else KDLAE_EINVAL_SHAPE).  Enqueued on `stream`. */
int kdlae_t_forward(kdlae_t_handle* h, const float* img, const float* rate, int B, int H, int W,
                    float* hq, float* sr, void* workspace, int64_t workspace_bytes, void* stream);

/* Measurement hook for bench.py (no effect on results).  When a probe class is armed, every
 * launch of that kernel class inside kdlae_t_forward is bracketed by a pair of HIP events on
 * `stream`; kdlae_t_probe_read synchronises those events and returns the summed device time (ms),
 * launch count and the algorithmic HBM bytes / FLOPs of the probed launches (SURVEY.md §8d model).
 * Classes: 0 = off, 1 = 1x1/implicit-GEMM conv (MFMA), 2 = dwconv+Gram (MDTA pass 1),
 * 3 = dwconv+GELU gate (GDFN).  A non-zero `level_filter` limits probing to blocks whose channel
 * count equals it.  */
int kdlae_t_probe_arm(kdlae_t_handle* h, int kernel_class, int level_filter);
int kdlae_t_probe_read(kdlae_t_handle* h, double* ms, int64_t* launches, double* bytes, double* flops);

/* Diagnostics (tools/config1_taps.py; not part of the drop-in boundary): activations at every
 * TransformerBlock stage in execution order — per stage its input ("<stage>.in"), then per block the
 * attention half's output x1 = x + attn(norm1 x) ("<stage>.<i>.attn", KDLAE_model.py:160) and the
 * block output ("<stage>.<i>", :161).  kdlae_t_debug_tap_info names tap i, its channel count C and its
 * resolution relative to the forward's input, H * num / den.  While kdlae_t_debug_taps(h, n, dst) is
 * armed (n = 0 disarms), every kdlae_t_forward copies tap i (i < n, dst[i] != NULL) into the device
 * buffer dst[i] as compact NHWC [B][H_i][W_i][C] on the forward's stream.  Results are unchanged. */
int kdlae_t_debug_tap_count(const kdlae_t_handle* h);
int kdlae_t_debug_tap_info(const kdlae_t_handle* h, int i, char* name, int name_len, int* C, int* num, int* den);
int kdlae_t_debug_taps(kdlae_t_handle* h, int n, float* const* dst);

/* ------------------------------------------------------------------ KDLAE-S
 * Ctor kwargs of KDLAE_student (KDLAE/KDLAE_model.py:340-384): a 3-D U-Net over a burst of frames.
 * hidden_channels has num_hidden entries (default [8, 16, 16, 32]); levels = num_hidden - 1.
 * The HIP path supports inp_channels == out_channels == 1 (forward unsqueezes a [B,F,H,W] input,
 * :397) and kernel_size == 3.
 */
typedef struct kdlae_s_config {
  int inp_channels;
  int out_channels;
  int residual;
  int num_hidden;
  int hidden_channels[8];
  int kernel_size;
} kdlae_s_config;

typedef struct kdlae_s_handle kdlae_s_handle;

/* replaces KDLAE_student.__init__ (KDLAE_model.py:341-384). */
int kdlae_s_create(const kdlae_s_config* cfg, int device, kdlae_s_handle** out);
int kdlae_s_destroy(kdlae_s_handle* h);
/* state_dict surface: encoders.{i}.{0,2}, st_fusion.{0,2}, upconv_layers.{j}, decoders.{j}.{0,2},
 * out_conv (same semantics as the kdlae_t_* calls). */
int kdlae_s_num_params(const kdlae_s_handle* h);
int kdlae_s_param_info(const kdlae_s_handle* h, int index, const char** name, int64_t* numel);
int64_t kdlae_s_params_numel(const kdlae_s_handle* h);
int kdlae_s_prepare(kdlae_s_handle* h);  /* as kdlae_t_prepare */
int kdlae_s_pack_device(kdlae_s_handle* h, const float* params, int64_t numel, void* stream);
int kdlae_s_set_param(kdlae_s_handle* h, const char* name, const float* host_data, int64_t numel);
int kdlae_s_commit_params(kdlae_s_handle* h, void* stream);
int64_t kdlae_s_workspace_bytes(const kdlae_s_handle* h, int B, int F, int H, int W);
/* replaces KDLAE_student.forward (KDLAE_model.py:395-431):
 *   x   [B, F, H, W]  (F = frames, the burst axis)
 *   out [B, F, H, W]  (= out_conv(...) + x when residual, squeezed)
 * H and W must be divisible by 2^levels (else KDLAE_EINVAL_SHAPE). */
int kdlae_s_forward(kdlae_s_handle* h, const float* x, int B, int F, int H, int W, float* out,
                    void* workspace, int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------ ASDQE
 * Ctor kwargs of DenoiseRatePredictor (ASDQE/ASDQE_model.py:127).  The HIP path supports
 * in_channels 1..4 and dim a multiple of 16 (16..256).  Eval-mode semantics only: BatchNorm uses
 * its running statistics (folded into the conv weights at commit), Dropout is the identity.
 */
typedef struct asdqe_config {
  int in_channels;
  int dim;
} asdqe_config;

typedef struct asdqe_handle asdqe_handle;

/* replaces DenoiseRatePredictor.__init__ (ASDQE_model.py:127-156). */
int asdqe_create(const asdqe_config* cfg, int device, asdqe_handle** out);
int asdqe_destroy(asdqe_handle* h);
/* state_dict surface incl. BatchNorm buffers (num_batches_tracked: 1 element, ignored).  The
 * reference loads its checkpoint with strict=False (ASDQE_test.py:79); this surface is strict.
 * The BatchNorm fold (W' = W g / sqrt(var + 1e-5), b' = (b - mean) g / sqrt(var + 1e-5) + beta) is
 * part of the device pack program (asdqe_pack_device, same contract as kdlae_t_pack_device). */
int asdqe_num_params(const asdqe_handle* h);
int asdqe_param_info(const asdqe_handle* h, int index, const char** name, int64_t* numel);
int64_t asdqe_params_numel(const asdqe_handle* h);
int asdqe_prepare(asdqe_handle* h);  /* as kdlae_t_prepare */
int asdqe_pack_device(asdqe_handle* h, const float* params, int64_t numel, void* stream);
int asdqe_set_param(asdqe_handle* h, const char* name, const float* host_data, int64_t numel);
int asdqe_commit_params(asdqe_handle* h, void* stream);
int64_t asdqe_workspace_bytes(const asdqe_handle* h, int B, int H, int W);
/* replaces DenoiseRatePredictor.forward (ASDQE_model.py:158-171) in eval mode:
 *   lq, gt [B, in_channels, H, W]  (any H, W: zero-padded bottom/right to a multiple of dim)
 *   score  [B, 1]                   (tanh output)
 *   feat   optional (NULL to skip): the UNet output map, NHWC [B, H', W', 3*dim] — an inspection
 *          hook; the score path folds the 1x1 outc after the pool and does not need it. */
int asdqe_forward(asdqe_handle* h, const float* lq, const float* gt, int B, int H, int W, float* score,
                  float* feat, void* workspace, int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------ pre/post-processing
 * The steps either side of the forward in KDLAE/KDLAE_T.ipynb (load_image_as_tensor, reflect pad,
 * denoise_rate map; clamp, crop, img_as_ubyte, zero-mask of black input pixels) and ASDQE's
 * ToTensor, on device buffers.
 */
#include <stdint.h>

/* (H, W) the notebook pads (h, w) to: ((h + m) / m) * m when h % m != 0, else h (same for w). */
void kdlae_padded_size(int h, int w, int multiple, int* H, int* W);

/* images u8 [B, h, w, channels] (channels 1, 3 or 4; alpha dropped; bgr != 0 swaps B and R like
 * cv2.cvtColor(BGR2RGB)) -> img f32 [B, min(channels, 3), H, W] = x / 255, reflect-padded on the
 * bottom/right to kdlae_padded_size(h, w, multiple) (multiple 1 = no padding: ASDQE ToTensor).
 * rate f32 [B] (nullable) -> rate_map f32 [B, 1, H, W] (nullable): the constant denoise_rate map. */
int kdlae_preprocess_u8(const uint8_t* images, int B, int h, int w, int channels, int bgr, int multiple,
                        const float* rate, float* img, float* rate_map, void* stream);

/* KDLAE/KDLAE-S.ipynb load_consecutive_stack + padding cell: frames u8 [B, F, h, w, channels]
 * (channels 1 = gray, 3 / 4 = BGR / BGRA as cv2.imread returns them) -> x f32 [B, F, H, W] =
 * cv2 COLOR_BGR2GRAY (8-bit fixed point) / 255, reflect-padded on the bottom/right to
 * kdlae_padded_size(h, w, multiple) (the notebook uses multiple 32).  Frames of one call share h, w
 * (the notebook cv2.resizes odd-sized frames first; that resize stays on the host). */
int kdlae_frames_preprocess_u8(const uint8_t* frames, int B, int F, int h, int w, int channels, int multiple,
                               float* x, void* stream);

/* out f32 [B, C, Hs, Ws] (model output, C <= 64: image channels, or the F frames of KDLAE-S) ->
 * dst u8 [B, h*scale, w*scale, C]:
 * clamp(0, 1), crop, rint(x * 255) (skimage img_as_ubyte), and 0 where the input pixel
 * lq u8 [B, h, w, lq_channels] (nullable) is black in every colour channel; scale 2 maps each
 * output pixel to its nearest input pixel (the notebook's np.repeat x2 mask for sr). */
int kdlae_postprocess_u8(const float* out, int B, int C, int Hs, int Ws, int h, int w, int scale,
                         const uint8_t* lq, int lq_channels, uint8_t* dst, void* stream);

/* ------------------------------------------------------------------ KDLAE-T training
 * One optimisation step of BasicSR's ImageCleanModel on KDLAE_teacher
 * (Train/basicsr/models/image_restoration_model.py:198-218): forward with saved activations,
 * L1LossSr (Train/basicsr/models/losses/losses.py:135-194), backward of every layer,
 * clip_grad_norm_(0.01) and AdamW.  Parameters and gradients are two flat caller-owned device
 * buffers of kdlae_tt_num_floats floats in state_dict order (offsets from kdlae_tt_param_info; each key
 * starts on a 16-byte boundary and the pad floats between keys must be zero);
 * weights are read in their OIHW state_dict layout, so an optimizer update needs no repacking.
 * The DDP gradient all-reduce (base_model.py:76-82) is done by the caller between the backward and
 * kdlae_train_clip_adamw: one collective over the flat gradient buffer, or bucketed and overlapped
 * with the backward through kdlae_tt_backward_marked's gradient-ready marks.
 */
typedef struct kdlae_tt_handle kdlae_tt_handle;

/* replaces KDLAE_teacher.__init__ for training (same config struct; dual_pixel_task -> ENOTIMPL). */
int kdlae_tt_create(const kdlae_t_config* cfg, int device, kdlae_tt_handle** out);
int kdlae_tt_destroy(kdlae_tt_handle* h);
/* net_g.state_dict() layout: key, element count and offset (floats) in the flat buffers. */
int kdlae_tt_num_params(const kdlae_tt_handle* h);
int kdlae_tt_param_info(const kdlae_tt_handle* h, int index, const char** name, int64_t* numel, int64_t* offset);
int64_t kdlae_tt_num_floats(const kdlae_tt_handle* h);
/* Device bytes of the caller-owned workspace (saved activations + backward scratch) for B x H x W. */
int64_t kdlae_tt_workspace_bytes(kdlae_tt_handle* h, int B, int H, int W);
/* replaces `preds = self.net_g(self.lq)` in optimize_parameters (image_restoration_model.py:200):
 * same tensors as kdlae_t_forward; theta = flat parameters.  Activations needed by the backward
 * stay in `workspace`, which must be passed unchanged to kdlae_tt_backward. */
int kdlae_tt_forward(kdlae_tt_handle* h, const float* theta, const float* img, const float* rate, int B, int H,
                     int W, float* hq, float* sr, void* workspace, size_t workspace_bytes, void* stream);
/* replaces `l_pix.backward()` (:213): dhq [B,C,H,W] / dsr [B,C,2H,2W] (nullable: zero) are the loss
 * gradients; grad (flat, overwritten) receives d loss / d theta.  Inputs get no gradient. */
int kdlae_tt_backward(kdlae_tt_handle* h, const float* theta, const float* dhq, const float* dsr, float* grad,
                      void* workspace, size_t workspace_bytes, void* stream);
/* kdlae_tt_backward plus gradient-ready marks for a bucketed DDP all-reduce that overlaps the backward
 * (DistributedDataParallel's gradient buckets, reducer.cpp behind base_model.py:76-82): the backward
 * walks the network deepest-first, i.e. the flat buffer from the end, and records event j when the
 * suffix [kdlae_tt_mark_lo(h, j), num_floats) of `grad` is final (offsets decrease with j).
 * kdlae_tt_mark_wait makes another stream wait for event j (enqueue that bucket's all-reduce behind
 * it); kdlae_tt_mark_sync waits on the host.  Marks stay valid until the next marked backward. */
int kdlae_tt_backward_marked(kdlae_tt_handle* h, const float* theta, const float* dhq, const float* dsr, float* grad,
                             void* workspace, size_t workspace_bytes, void* stream);
int kdlae_tt_mark_count(const kdlae_tt_handle* h);
int64_t kdlae_tt_mark_lo(const kdlae_tt_handle* h, int j);
int kdlae_tt_mark_wait(kdlae_tt_handle* h, int j, void* stream);
int kdlae_tt_mark_sync(kdlae_tt_handle* h, int j);

/* replaces self.cri_pix(pred, self.gt) with L1LossSr(loss_weight=1, reduction='mean') (losses.py:159-170):
 * loss[0] = 0.5 l1(hq) + 0.25 l1(sr) + 0.25 (shadow(hq) + shadow(sr)); dhq / dsr receive its gradient
 * (the shadow terms binarise at 0.1 and carry none).  pred_sr NULL = no sr term.  scratch: device
 * buffer of kdlae_train_l1sr_scratch_floats() floats. */
int64_t kdlae_train_l1sr_scratch_floats(void);
int kdlae_train_l1sr(const float* pred_hq, const float* gt_hq, int64_t n_hq, const float* pred_sr,
                     const float* gt_sr, int64_t n_sr, float* dhq, float* dsr, float* loss, float* scratch,
                     void* stream);
/* replaces torch.nn.utils.clip_grad_norm_(params, max_norm) + torch.optim.AdamW.step (:215-218) over
 * flat buffers: g = gscale * grad (gscale = 1/world_size after a summing all-reduce), clipped to
 * max_norm (<= 0: no clip); `step` counts from 1.  The norm covers all n gradients; the update
 * covers the host array `ranges` of nranges [begin, end) pairs (nranges 0: all n), mirroring
 * torch.optim skipping parameters whose .grad is None.  scratch: kdlae_train_adamw_scratch_floats()
 * floats; after the call scratch[2048] holds the gradient norm (after gscale, before clipping). */
int64_t kdlae_train_adamw_scratch_floats(void);
int kdlae_train_clip_adamw(float* theta, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                           float gscale, float max_norm, float lr, float beta1, float beta2, float eps,
                           float weight_decay, int step, const int64_t* ranges, int nranges, float* scratch,
                           void* stream);
/* replaces Mixing_Augment.mixup (image_restoration_model.py:25-61, KDLAET.yml mixing_augs):
 * out[b] = lam * in[b] + (1 - lam) * in[perm[b]] over B samples of per_sample floats; perm is a
 * device int[B]; lam and perm are drawn on the host exactly as the reference draws them. */
int kdlae_train_mixup(const float* in, float* out, int B, int64_t per_sample, const int* perm, float lam,
                      void* stream);
/* replaces BaseModel.model_ema(decay) (Train/basicsr/models/base_model.py:54-62) over the flat buffers. */
int kdlae_train_ema(float* ema, const float* theta, int64_t n, float decay, void* stream);

/* ------------------------------------------------------------------ KDLAE-S training
 * One optimisation step of BasicSR's ImageCleanModel on KDLAE_student with KDLAES.yml
 * (Train/Denoising/Options/paper202508/KDLAES.yml: L1LossForVideoFrames, clip_grad_norm_, AdamW):
 * forward with saved activations and the backward of every layer (Conv3d 3x3x3 + ReLU, MaxPool3d
 * (1,2,2), ConvTranspose3d (1,2,2) + skip, out_conv + residual; KDLAE/KDLAE_model.py:395-431).
 * Parameters / gradients: flat caller-owned buffers of kdlae_st_num_floats floats in state_dict order,
 * every key 16-byte aligned (pads zero), as for kdlae_tt_*; kdlae_train_clip_adamw / _ema / _mixup
 * apply unchanged. */
typedef struct kdlae_st_handle kdlae_st_handle;
/* replaces KDLAE_student.__init__ for training (KDLAE_model.py:341-384); inp/out_channels 1, kernel_size 3,
 * hidden_channels divisible by 4 (KDLAE_EINVAL_CONFIG otherwise) */
int kdlae_st_create(const kdlae_s_config* cfg, int device, kdlae_st_handle** out);
int kdlae_st_destroy(kdlae_st_handle* h);
int kdlae_st_num_params(const kdlae_st_handle* h);
int kdlae_st_param_info(const kdlae_st_handle* h, int index, const char** name, int64_t* numel, int64_t* offset);
int64_t kdlae_st_num_floats(const kdlae_st_handle* h);
int64_t kdlae_st_workspace_bytes(const kdlae_st_handle* h, int B, int F, int H, int W);
/* replaces `preds = self.net_g(self.lq)` (image_restoration_model.py:200) for KDLAE_student: x, out [B, F, H, W];
 * activations stay in `workspace` for kdlae_st_backward */
int kdlae_st_forward(kdlae_st_handle* h, const float* theta, const float* x, int B, int F, int H, int W, float* out,
                     void* workspace, int64_t workspace_bytes, void* stream);
/* replaces `l_pix.backward()` (:213): dout [B, F, H, W] -> grad (flat, overwritten); x gets no gradient */
int kdlae_st_backward(kdlae_st_handle* h, const float* theta, const float* dout, float* grad, void* workspace,
                      int64_t workspace_bytes, void* stream);
/* replaces L1LossForVideoFrames(l1loss_weight, reduction, temporal_weight, binary)(pred, target)
 * (Train/basicsr/models/losses/losses.py:409-526) for pred / target [N, frames, H, W] (hw = H W):
 * loss[0] = l1loss_weight (mean|p - t| + mean|bin(p) - bin(t)|) + temporal_weight mean|dp - dt| (frame
 * differences; frames == 1: no temporal term); reduction 0 = 'mean', 1 = 'sum' ('max' / 'mix': EINVAL_CONFIG).
 * dpred receives d loss / d pred.  scratch: kdlae_train_l1frames_scratch_floats() floats. */
int64_t kdlae_train_l1frames_scratch_floats(void);
int kdlae_train_l1frames(const float* pred, const float* target, int N, int frames, int64_t hw, float l1loss_weight,
                         float temporal_weight, float binary, int reduction, float* dpred, float* loss, float* scratch,
                         void* stream);

/* ---- Kernel self-test entry points (tests/test_kernel_variants_gpu.py; not part of the drop-in
 * boundary).  One launch of the training GEMM family on caller device buffers:
 *   C(m, n) = sum_k A(m, k) B(k, n) [+ bias[n]] [+ rs[n] R(m, n)], batch z = z1 * nz2 + z2, every
 *   operand offset by z1 * b?1 + z2 * b?2 (floats); amode 1 = implicit 3x3 im2col of the NHWC view A
 *   (pixel stride lda, k = tap * Cg + c, dilation dil, zero padding), bmode 1 = the NHWC view B shifted
 *   by tap z2 (conv weight gradient), bmode 2 / 3 = a 3x3 OIHW weight as the forward / transposed
 *   conv operand, bmode 4 = implicit 3x3x3 im2col of the NDHWC view B, n = tap * Cg + c (Conv3d weight
 *   gradient; pixel-reduction kernel) (see train_kernels.h TGemm).  route: 0 = the engine's own dispatch, 1 = the
 *   row-streaming kernel, 2 = the pixel-reduction kernel (needs partial), 3 = the tiled kernels. */
typedef struct kdlae_debug_tgemm_desc {
  const float* A; int64_t sam, sak; int amode;
  const float* B; int64_t sbk, sbn; int bmode;
  float* C; int64_t scm, scn;
  const float* bias;
  const float* R; int64_t srm, srn;
  const float* rs;
  int M, N, K, nz1, nz2;
  int64_t bA1, bA2, bB1, bB2, bC1, bC2, bR1, bR2, brs1, brs2;
  int Bn, H, W, Cg, dil;
  int64_t lda, ldb;
  float* partial; int64_t partial_floats;
  int route;
  int c_pad_ok;
  int F;  /* frames of the bmode 4 (implicit 3x3x3) B view; 0 = 1 */
} kdlae_debug_tgemm_desc;
int kdlae_debug_tgemm(const kdlae_debug_tgemm_desc* d, void* stream);

/* One launch of the inference implicit-GEMM family (gemm.hip) with the tile shape forced:
 *   out[b][p][n] = relu?( sum_k A'[b][p][k] Wp(n, k) + bias[n] (+ R) ), A' = A or LN(A) over ln_C
 *   (ln 1 BiasFree, 2 WithBias, unit weight); ksize 3: implicit 3x3 (kt 3: 3x3x3 over F frames),
 *   k = tap * 16 cg_per_tap + c, zero padding = dil; out_mode 1 / 2 stores through PixelUnshuffle(2)
 *   / PixelShuffle(2) (R then in the output geometry).  Wp: fragment-packed [ntiles][kgroups][64][4],
 *   element (l, e) of (t, g) = W(16 t + l % 16, 16 g + 4 (l / 16) + e); + b * w_img_stride per image.
 *   Wm != 0: fused attention output, x1 = R + Wm v (+ bias_m) stored to out1, then out = LN(x1) W.
 *   stats: [pixels][2] scratch when LN meets a chunked K.  group_tiles > 0: resident schedule.
 *   tiles_per_block 0: the engine's grid rule.  route 0: production dispatch; 1: the r01
 *   conv_gemm_kernel of (NT, KG) (the fallback for ld % 4 != 0 views). */
typedef struct kdlae_debug_gemm_desc {
  const float* A; int lda;
  int Bn, F, H, W;
  int ksize, kt, dil, cg_per_tap, kgroups;
  const float* Wp; int64_t w_img_stride; int ntiles, N;
  const float* bias;
  float* out; int ldo;
  const float* R; int ldr;
  int ln, ln_C, relu, out_mode;
  float* stats;
  const float* Wm; int64_t wm_img_stride; const float* bias_m; float* out1; int ldo1;
  int NT, KG, wpe, group_tiles, tiles_per_block;
  int route;
} kdlae_debug_gemm_desc;
int kdlae_debug_gemm(const kdlae_debug_gemm_desc* d, void* stream);
/* Entry i of a compiled variant table: family 0 conv_gemm_kernel (NT, KG, CONV3, OUT, PF, WPE, RES),
 * 1 gemm_res_kernel (NT, KG, NCH, PF), 2 gemm_chunk_kernel (NT, KG, CONV3, OUT), 3 gemm_attn_in_kernel
 * (NT, KG, NCH).  Fills v[0..6]; returns 1, or 0 past the end. */
int kdlae_debug_gemm_variant(int family, int i, int* v);

/* MDTA pass 1 + 2 (mdta.hip): depthwise 3x3 of qkv ([P][ld], wdw [9][3C] tap-major, bdw [3C]), v
 * stored to v_out, per (image, head) the Gram q k^T and the squared norms summed into
 * reduced[Bn * heads][Ch^2 + 2 Ch] (Gram in accumulator order: element (i * CT + j) * 256 + 4 l + e =
 * G[16 i + 4 (l / 16) + e][16 j + l % 16], CT = Ch / 16; then |q_c|^2, |k_c|^2).  partial: scratch of
 * partial_floats.  route 0: production (ring kernel where it applies), 1: without the ring kernel
 * (zeros ignored), 2: the generic 64-pixel-step kernel. */
typedef struct kdlae_debug_gram_desc {
  const float* qkv; int ld;
  const float* wdw; const float* bdw;
  float* v_out; int ldv;
  float* partial; int64_t partial_floats;
  float* reduced;
  const float* zeros;
  int C, heads, Bn, H, W;
  int route;
} kdlae_debug_gram_desc;
int kdlae_debug_gram(const kdlae_debug_gram_desc* d, void* stream);

/* Training LayerNorm (train.hip) over P pixels of C channels: dir 0 forward y = LN(x) w (+ b),
 * stats[P][2]; dir 1 backward dx = R + dLN(dy), part[nblk][C | 2 C] the per-block weight (and bias)
 * gradient partials.  route 0: production dispatch, 1: the one-wave-per-pixel kernels. */
typedef struct kdlae_debug_ln_desc {
  int dir;
  const float* x; int ldx;
  const float* w; const float* b;
  int C; int64_t P; int biasfree;
  float* y; int ldy;
  float* stats;
  const float* dy; int ldd;
  const float* R; int ldr;
  float* dx; int lddx;
  float* part; int nblk;
  int route;
} kdlae_debug_ln_desc;
int kdlae_debug_ln(const kdlae_debug_ln_desc* d, void* stream);

/* Small-input 3x3 / 3x3x3 conv (conv_small.hip), Cin * 9 * kt <= 36, Cout % 16 == 0: input element
 * (b, frame t, y, x, c) at in[b sb + t st + y sy + x sx + c sc] (minus in_sub at the same offset),
 * w [Cout][Cin][kt][3][3], NHWC output [Bn * F * H * W][ldo]; valid input extent vh x vw (0 = H, W). */
typedef struct kdlae_debug_small_in_desc {
  const float* in; int64_t sb, sc, sy, sx, st;
  const float* in_sub;
  int Cin, Cout, dil, kt, F;
  const float* w; const float* bias;
  float* out; int ldo;
  int Bn, H, W, vh, vw, relu;
} kdlae_debug_small_in_desc;
int kdlae_debug_small_in(const kdlae_debug_small_in_desc* d, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* KDLAE_H_ */
