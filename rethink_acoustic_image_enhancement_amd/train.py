"""KDLAE-T training on the MI355X HIP path.

Three layers, all backed by ``libkdlae.so`` (``kdlae_tt_*`` / ``kdlae_train_*`` in include/kdlae.h):

* ``TrainEngine`` — one training handle per (model, device): forward with saved activations and the
  hand-sequenced backward of every KDLAE_teacher layer over flat parameter / gradient buffers.
* Drop-in autograd: ``KDLAE_teacher.forward`` under grad mode routes through ``TeacherTrainFn`` and
  ``L1LossSr`` here is an autograd-aware HIP loss, so the reference's own loop
  (``preds = net_g(lq); l_pix = cri_pix(preds, gt); l_pix.backward(); clip_grad_norm_; opt.step()``,
  Train/basicsr/models/image_restoration_model.py:198-218) runs unchanged with any torch optimizer.
* ``KDLAETrainer`` — the fast path of that same loop: flat buffers end to end, the HIP L1LossSr, one
  RCCL all-reduce of the flat gradient for DDP (base_model.py:76-82), and the fused
  clip_grad_norm_ + AdamW kernel.  The model's parameters become views of the trainer's flat
  buffer, so ``state_dict()``/checkpoints and the inference path always see the trained weights.

There is no CPU fallback: every entry point raises on CPU tensors or a missing library.
"""
from __future__ import annotations

import ctypes
import math
import random

import torch
import torch.distributed as dist

from . import _lib

__all__ = ["TrainEngine", "TeacherTrainFn", "L1LossSr", "KDLAETrainer", "MixingAugment", "sync_gradients",
           "grad_buckets", "sync_gradients_bucketed", "StudentTrainEngine", "StudentTrainFn",
           "L1LossForVideoFrames", "KDLAESTrainer"]


def _vp(t):
    return ctypes.c_void_p(t.data_ptr() if t is not None else 0)


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


class TrainEngine:
    """``kdlae_tt_*`` handle for one KDLAE_teacher config on one device."""

    def __init__(self, model, device: torch.device):
        L = _lib.lib()
        self.device = device
        h = ctypes.c_void_p()
        idx = device.index if device.index is not None else torch.cuda.current_device()
        _lib.check(L.kdlae_tt_create(ctypes.byref(model._c_config()), idx, ctypes.byref(h)), "kdlae_tt_create")
        self.handle = h
        self._L = L
        self.keys = []
        for i in range(L.kdlae_tt_num_params(h)):
            name, numel, off = ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_int64()
            _lib.check(L.kdlae_tt_param_info(h, i, ctypes.byref(name), ctypes.byref(numel), ctypes.byref(off)),
                       "kdlae_tt_param_info")
            self.keys.append((name.value.decode(), int(numel.value), int(off.value)))
        self.numel = int(L.kdlae_tt_num_floats(h))
        names = [k for k, _, _ in self.keys]
        sd_names = [k for k, _ in model.named_parameters()]
        if names != sd_names:
            raise RuntimeError("KDLAE_teacher parameters do not match the training handle's state_dict layout")
        cfg = model._cfg
        self.static_train = cfg["static"] == "train"
        self.params_cat = cfg["params"] == "cat"
        self.out_channels = cfg["out_channels"]
        # parameters the reference forward never touches (KDLAE_model.py:315-319 when params != 'cat'):
        # autograd leaves their .grad None and torch.optim skips them
        unused = ("output_param.", "refinement_out.") if not self.params_cat else ()
        self.used = [not k.startswith(unused) for k in names]
        self.ws = None
        self.ws_shape = None
        self.generation = 0
        self._dtor = L.kdlae_tt_destroy

    def __del__(self):
        try:
            if self.handle:
                self._dtor(self.handle)
        except Exception:
            pass

    def used_ranges(self):
        """[begin, end) float ranges of the flat buffer that receive gradients (merged)."""
        out = []
        for (k, n, off), u in zip(self.keys, self.used):
            if not u:
                continue
            end = off + ((n + 3) & ~3)  # keys are 16-byte aligned; the zero pad floats ride along
            if out and out[-1][1] == off:
                out[-1][1] = end
            else:
                out.append([off, end])
        return out

    def flatten(self, tensors) -> torch.Tensor:
        """Parameters -> the handle's flat layout (state_dict order, each key 16-byte aligned, pads zero)."""
        tensors = list(tensors)
        flat = torch.zeros(self.numel, dtype=torch.float32, device=tensors[0].device)
        for (k, n, off), t in zip(self.keys, tensors):
            flat[off:off + n] = t.detach().reshape(-1).to(torch.float32)
        return flat

    def packed(self, flat) -> torch.Tensor:
        """The flat layout without its pad floats: torch.cat of the keys in state_dict order."""
        return torch.cat([flat[off:off + n] for _, n, off in self.keys])

    def _workspace(self, B, H, W):
        nbytes = int(self._L.kdlae_tt_workspace_bytes(self.handle, B, H, W))
        if nbytes < 0:
            _lib.check(1, "kdlae_tt_workspace_bytes")
        if self.ws is None or self.ws.numel() < nbytes:
            self.ws = None
            self.ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        return self.ws

    def forward(self, theta, img, rate):
        """KDLAE_teacher.forward (KDLAE_model.py:270-336) with activations kept for ``backward``."""
        if img.device.type != "cuda":
            raise RuntimeError("KDLAE training runs on ROCm devices only; there is no CPU fallback")
        img = img.detach().to(torch.float32).contiguous()
        B, _, H, W = img.shape
        if H % 8 or W % 8:
            raise RuntimeError(f"KDLAE_teacher needs H and W divisible by 8, got {H}x{W}")
        rate = rate.detach().to(device=img.device, dtype=torch.float32).contiguous() if self.params_cat else None
        oc = self.out_channels
        hq = torch.empty((B, oc, H, W), device=img.device, dtype=torch.float32)
        sr = torch.empty((B, oc, 2 * H, 2 * W), device=img.device, dtype=torch.float32) if self.static_train else None
        ws = self._workspace(B, H, W)
        rc = self._L.kdlae_tt_forward(self.handle, _vp(theta), _vp(img), _vp(rate), B, H, W, _vp(hq), _vp(sr),
                                      _vp(ws), ws.numel(), _stream(img.device))
        _lib.check(rc, "kdlae_tt_forward")
        self.generation += 1
        return hq, sr

    def backward(self, theta, dhq, dsr, grad, marked=False):
        """d loss / d theta into ``grad`` (flat, overwritten) from the output gradients.

        ``marked``: also record the gradient-ready events of ``kdlae_tt_backward_marked``; returns
        their suffix offsets (decreasing: the backward runs deepest-first, i.e. from the buffer's end)."""
        dhq = dhq.detach().to(torch.float32).contiguous() if dhq is not None else None
        dsr = dsr.detach().to(torch.float32).contiguous() if (dsr is not None and self.static_train) else None
        fn = self._L.kdlae_tt_backward_marked if marked else self._L.kdlae_tt_backward
        rc = fn(self.handle, _vp(theta), _vp(dhq), _vp(dsr), _vp(grad), _vp(self.ws), self.ws.numel(),
                _stream(grad.device))
        _lib.check(rc, "kdlae_tt_backward_marked" if marked else "kdlae_tt_backward")
        if not marked:
            return grad
        return [int(self._L.kdlae_tt_mark_lo(self.handle, j)) for j in range(self._L.kdlae_tt_mark_count(self.handle))]


class TeacherTrainFn(torch.autograd.Function):
    """Autograd node for one KDLAE_teacher forward on the training engine."""

    @staticmethod
    def forward(ctx, engine, img, rate, *params):
        theta = engine.flatten(params)
        hq, sr = engine.forward(theta, img, rate)
        # an output the loss ignores arrives as None (not zeros), so the branch that produced only it
        # gets None gradients and torch.optim skips those parameters, as with the reference module
        ctx.set_materialize_grads(False)
        ctx.engine = engine
        ctx.generation = engine.generation
        ctx.theta = theta
        ctx.shapes = [p.shape for p in params]
        if sr is None:
            return hq
        return hq, sr

    @staticmethod
    def backward(ctx, dhq, dsr=None):
        eng = ctx.engine
        if eng.generation != ctx.generation:
            raise RuntimeError("KDLAE_teacher: a second training forward ran before this graph's backward; "
                               "the HIP engine keeps one set of saved activations per model and device")
        if dhq is None and dsr is None:
            return (None, None, None, *[None] * len(ctx.shapes))
        grad = torch.empty(eng.numel, dtype=torch.float32, device=ctx.theta.device)
        eng.backward(ctx.theta, dhq, dsr, grad)  # a None output gradient is read as zero
        # sr = enhance(cen(hq)) (KDLAE_model.py:324-329): with no sr gradient that branch is untouched
        skip = ("cen.", "upen.", "enhance.", "outputen.") if dsr is None else None
        grads = []
        for (k, n, off), shape, used in zip(eng.keys, ctx.shapes, eng.used):
            live = used and not (skip and k.startswith(skip))
            grads.append(grad[off:off + n].view(shape) if live else None)
        return (None, None, None, *grads)


class _L1LossSrFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hq, gt_hq, sr, gt_sr, loss_weight):
        L = _lib.lib()
        dev = hq.device
        hq = hq.detach().contiguous()
        gt_hq = gt_hq.detach().to(torch.float32).contiguous()
        dhq = torch.empty_like(hq)
        dsr = None
        if sr is not None:
            sr = sr.detach().contiguous()
            gt_sr = gt_sr.detach().to(torch.float32).contiguous()
            dsr = torch.empty_like(sr)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        scratch = torch.empty(int(L.kdlae_train_l1sr_scratch_floats()), dtype=torch.float32, device=dev)
        rc = L.kdlae_train_l1sr(_vp(hq), _vp(gt_hq), hq.numel(), _vp(sr), _vp(gt_sr),
                                sr.numel() if sr is not None else 0, _vp(dhq), _vp(dsr), _vp(loss), _vp(scratch),
                                _stream(dev))
        _lib.check(rc, "kdlae_train_l1sr")
        ctx.save_for_backward(dhq, dsr if dsr is not None else torch.empty(0, device=dev))
        ctx.has_sr = sr is not None
        ctx.w = loss_weight
        return loss * loss_weight

    @staticmethod
    def backward(ctx, g):
        dhq, dsr = ctx.saved_tensors
        s = g * ctx.w
        return dhq * s, None, (dsr * s if ctx.has_sr else None), None, None


class L1LossSr(torch.nn.Module):
    """L1LossSr (Train/basicsr/models/losses/losses.py:135-194) on the HIP path, autograd-aware.

    loss = loss_weight * (0.5 l1(hq) + 0.25 l1(sr) + 0.25 (shadow(hq) + shadow(sr))), reduction 'mean'.
    """

    def __init__(self, loss_weight=1.0, reduction="mean"):
        super().__init__()
        if reduction not in ("none", "mean", "sum"):
            raise ValueError(f"Unsupported reduction mode: {reduction}. Supported ones are: ['none', 'mean', 'sum']")
        if reduction != "mean":
            raise NotImplementedError("the HIP L1LossSr implements reduction='mean' (the KDLAET.yml setting)")
        self.loss_weight = loss_weight
        self.reduction = reduction

    def forward(self, pred, target, weight=None, **kwargs):
        if weight is not None:
            raise NotImplementedError("element-wise loss weights are not used by the reference configs")
        if pred["hq"].device.type != "cuda":
            raise RuntimeError("L1LossSr (MI355X build) runs on ROCm devices only")
        return _L1LossSrFn.apply(pred["hq"], target["hq"], pred.get("sr"), target.get("sr") if pred.get("sr")
                                 is not None else None, float(self.loss_weight))


# ------------------------------------------------------------------ KDLAE-S (KDLAES.yml)
class StudentTrainEngine:
    """``kdlae_st_*`` handle for one KDLAE_student config on one device (KDLAE_model.py:340-431)."""

    def __init__(self, model, device: torch.device):
        L = _lib.lib()
        self.device = device
        h = ctypes.c_void_p()
        idx = device.index if device.index is not None else torch.cuda.current_device()
        _lib.check(L.kdlae_st_create(ctypes.byref(model._c_config()), idx, ctypes.byref(h)), "kdlae_st_create")
        self.handle = h
        self._L = L
        self.keys = []
        for i in range(L.kdlae_st_num_params(h)):
            name, numel, off = ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_int64()
            _lib.check(L.kdlae_st_param_info(h, i, ctypes.byref(name), ctypes.byref(numel), ctypes.byref(off)),
                       "kdlae_st_param_info")
            self.keys.append((name.value.decode(), int(numel.value), int(off.value)))
        self.numel = int(L.kdlae_st_num_floats(h))
        if [k for k, _, _ in self.keys] != [k for k, _ in model.named_parameters()]:
            raise RuntimeError("KDLAE_student parameters do not match the training handle's state_dict layout")
        self.ws = None
        self.generation = 0
        self._dtor = L.kdlae_st_destroy

    def __del__(self):
        try:
            if self.handle:
                self._dtor(self.handle)
        except Exception:
            pass

    def used_ranges(self):
        return [[0, self.numel]]

    flatten = TrainEngine.flatten
    packed = TrainEngine.packed

    def forward(self, theta, x):
        """KDLAE_student.forward with activations kept for ``backward``: x [B, F, H, W] -> [B, F, H, W]."""
        if x.device.type != "cuda":
            raise RuntimeError("KDLAE training runs on ROCm devices only; there is no CPU fallback")
        x = x.detach().to(torch.float32).contiguous()
        B, F, H, W = x.shape
        nbytes = int(self._L.kdlae_st_workspace_bytes(self.handle, B, F, H, W))
        if nbytes < 0:
            _lib.check(1, "kdlae_st_workspace_bytes")
        if self.ws is None or self.ws.numel() < nbytes:
            self.ws = None
            self.ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
        out = torch.empty_like(x)
        self._x = x  # the residual input must outlive the backward
        rc = self._L.kdlae_st_forward(self.handle, _vp(theta), _vp(x), B, F, H, W, _vp(out), _vp(self.ws),
                                      self.ws.numel(), _stream(x.device))
        _lib.check(rc, "kdlae_st_forward")
        self.generation += 1
        return out

    def backward(self, theta, dout, grad):
        dout = dout.detach().to(torch.float32).contiguous()
        rc = self._L.kdlae_st_backward(self.handle, _vp(theta), _vp(dout), _vp(grad), _vp(self.ws), self.ws.numel(),
                                       _stream(grad.device))
        _lib.check(rc, "kdlae_st_backward")
        return grad


class StudentTrainFn(torch.autograd.Function):
    """Autograd node for one KDLAE_student forward on the training engine (the input gets no gradient)."""

    @staticmethod
    def forward(ctx, engine, x, *params):
        theta = engine.flatten(params)
        out = engine.forward(theta, x)
        ctx.engine = engine
        ctx.generation = engine.generation
        ctx.theta = theta
        ctx.shapes = [p.shape for p in params]
        return out

    @staticmethod
    def backward(ctx, dout):
        eng = ctx.engine
        if eng.generation != ctx.generation:
            raise RuntimeError("KDLAE_student: a second training forward ran before this graph's backward; "
                               "the HIP engine keeps one set of saved activations per model and device")
        grad = torch.empty(eng.numel, dtype=torch.float32, device=ctx.theta.device)
        eng.backward(ctx.theta, dout, grad)
        return (None, None, *[grad[off:off + n].view(shape) for (k, n, off), shape in zip(eng.keys, ctx.shapes)])


class _L1FramesFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, l1w, tw, binary, red):
        L = _lib.lib()
        dev = pred.device
        p = pred.detach().to(torch.float32).contiguous()
        t = target.detach().to(device=dev, dtype=torch.float32).contiguous()
        N, Cf = p.shape[0], p.shape[1]
        hw = p.numel() // max(1, N * Cf)
        dp = torch.empty_like(p)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        scratch = torch.empty(int(L.kdlae_train_l1frames_scratch_floats()), dtype=torch.float32, device=dev)
        rc = L.kdlae_train_l1frames(_vp(p), _vp(t), N, Cf, hw, float(l1w), float(tw), float(binary), red, _vp(dp),
                                    _vp(loss), _vp(scratch), _stream(dev))
        _lib.check(rc, "kdlae_train_l1frames")
        ctx.save_for_backward(dp)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dp,) = ctx.saved_tensors
        return dp * g, None, None, None, None, None


class L1LossForVideoFrames(torch.nn.Module):
    """L1LossForVideoFrames (Train/basicsr/models/losses/losses.py:409-526) on the HIP path, autograd-aware:
    l1loss_weight * reduce(|p - t| + |bin(p) - bin(t)|) + temporal_weight * reduce(|dp - dt|) over the
    frame axis (dim 1) of [N, frames, H, W] tensors.  The reference's 'max' / 'mix' reductions (and
    element weights) are not used by its configs and raise NotImplementedError here."""

    def __init__(self, l1loss_weight=0.64, reduction="mean", sigma=2.0, weight=[1.5, 1.0], invert=False,
                 temporal_weight=0.36, binary=0.1):
        super().__init__()
        if reduction not in ["none", "mean", "sum", "max", "mix"]:
            raise ValueError(f"Unsupported reduction mode: {reduction}. "
                             f'Supported ones are: ["none", "mean", "sum", "max", "mix"]')
        self.l1loss_weight = l1loss_weight
        self.reduction = reduction
        self.temporal_weight = temporal_weight
        self.binary = binary

    def forward(self, pred, target, weight=None, **kwargs):
        if weight is not None:
            raise NotImplementedError("element-wise loss weights are not used by the reference configs")
        if self.reduction not in ("mean", "sum"):
            raise NotImplementedError(f"L1LossForVideoFrames reduction {self.reduction!r} on the HIP path "
                                      "(KDLAES.yml uses 'mean')")
        if pred.device.type != "cuda":
            raise RuntimeError("L1LossForVideoFrames (MI355X build) runs on ROCm devices only")
        return _L1FramesFn.apply(pred, target, self.l1loss_weight, self.temporal_weight, self.binary,
                                 0 if self.reduction == "mean" else 1)


class KDLAESTrainer:
    """ImageCleanModel.optimize_parameters for KDLAE_student with KDLAES.yml (AdamW lr 3e-4 wd 1e-4 betas
    (0.9, 0.999); use_grad_clip -> clip_grad_norm_(0.01); L1LossForVideoFrames(0.9, mean, temporal 0.1);
    mixup): flat buffers end to end, one RCCL all-reduce of the flat gradient for DDP."""

    def __init__(self, model, lr=3e-4, weight_decay=1e-4, betas=(0.9, 0.999), eps=1e-8, use_grad_clip=True,
                 max_norm=0.01, loss_kw=None, group=None, mixing_augs=None):
        params = list(model.parameters())
        if not params or params[0].device.type != "cuda":
            raise RuntimeError("KDLAESTrainer: move the model to a ROCm device first (no CPU fallback)")
        dev = params[0].device
        self.model = model
        self.engine = StudentTrainEngine(model, dev)
        eng = self.engine
        self.theta = eng.flatten(params).contiguous()
        with torch.no_grad():
            for (k, n, off), p in zip(eng.keys, params):
                p.data = self.theta[off:off + n].view(p.shape)
        self.grad = torch.zeros(eng.numel, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros_like(self.grad)
        self.exp_avg_sq = torch.zeros_like(self.grad)
        self.lr, self.weight_decay, self.betas, self.eps = lr, weight_decay, tuple(betas), eps
        self.max_norm = max_norm if use_grad_clip else 0.0
        kw = dict(l1loss_weight=0.9, temporal_weight=0.1, reduction="mean")
        kw.update(loss_kw or {})
        self.loss_fn = L1LossForVideoFrames(**kw)
        self.group = group
        self.step_count = 0
        self.loss = None
        L = _lib.lib()
        self._opt_scratch = torch.empty(int(L.kdlae_train_adamw_scratch_floats()), dtype=torch.float32, device=dev)
        self._l1_scratch = torch.empty(int(L.kdlae_train_l1frames_scratch_floats()), dtype=torch.float32,
                                       device=dev)
        self._loss = torch.zeros((), dtype=torch.float32, device=dev)
        m = mixing_augs or {}
        self.mixing = (MixingAugment(m.get("mixup_beta", 1.2), m.get("use_identity", False), dev)
                       if m.get("mixup", False) else None)

    def feed_train_data(self, lq, gt):
        if self.mixing is not None:
            gt, lq = self.mixing(gt, lq)
        return lq, gt

    def forward_backward(self, lq, gt):
        eng, L = self.engine, _lib.lib()
        out = eng.forward(self.theta, lq)
        self.output = out
        dout = torch.empty_like(out)
        # the same device move as _L1FramesFn: the loss kernel dereferences gt on the GPU
        gt = gt.to(device=out.device, dtype=torch.float32).contiguous()
        if gt.shape != out.shape:
            raise ValueError(f"gt shape {tuple(gt.shape)} != output shape {tuple(out.shape)}")
        N, Cf = out.shape[0], out.shape[1]
        lf = self.loss_fn
        if lf.reduction not in ("mean", "sum"):
            raise NotImplementedError(f"reduction {lf.reduction!r}")
        rc = L.kdlae_train_l1frames(_vp(out), _vp(gt), N, Cf, out.numel() // (N * Cf), float(lf.l1loss_weight),
                                    float(lf.temporal_weight), float(lf.binary), 0 if lf.reduction == "mean" else 1,
                                    _vp(dout), _vp(self._loss), _vp(self._l1_scratch), _stream(out.device))
        _lib.check(rc, "kdlae_train_l1frames")
        eng.backward(self.theta, dout, self.grad)
        self.loss = self._loss
        return self.loss

    def step(self, gscale: float = 1.0):
        self.step_count += 1
        b1, b2 = self.betas
        rc = _lib.lib().kdlae_train_clip_adamw(
            _vp(self.theta), _vp(self.grad), _vp(self.exp_avg), _vp(self.exp_avg_sq), self.engine.numel,
            float(gscale), float(self.max_norm), float(self.lr), float(b1), float(b2), float(self.eps),
            float(self.weight_decay), self.step_count, None, 0, _vp(self._opt_scratch), _stream(self.theta.device))
        _lib.check(rc, "kdlae_train_clip_adamw")

    def optimize_parameters(self, lq, gt):
        loss = self.forward_backward(lq, gt)
        self.step(sync_gradients(self.grad, self.group))
        return loss

    def grad_norm(self) -> torch.Tensor:
        return self._opt_scratch[2048]


def _mix(t, perm, lam):
    t = t.to(torch.float32).contiguous()
    out = torch.empty_like(t)
    per = t.numel() // t.shape[0]
    rc = _lib.lib().kdlae_train_mixup(_vp(t), _vp(out), t.shape[0], per, _vp(perm), float(lam), _stream(t.device))
    _lib.check(rc, "kdlae_train_mixup")
    return out


class MixingAugment:
    """Mixing_Augment (Train/basicsr/models/image_restoration_model.py:25-61), blend on the GPU.

    lam ~ Beta(mixup_beta, mixup_beta) and the batch permutation are drawn on the host exactly as the
    reference draws them (torch.distributions / torch.randperm / random.randint), so a seeded run
    picks the same mixes; the blend lam * x + (1 - lam) * x[perm] is ``kdlae_train_mixup``."""

    def __init__(self, mixup_beta=1.2, use_identity=False, device=None):
        self.dist = torch.distributions.beta.Beta(torch.tensor([mixup_beta]), torch.tensor([mixup_beta]))
        self.device = device
        self.use_identity = use_identity
        self.augments = [self.mixup]

    def mixup(self, target, input_):
        lam = self.dist.rsample((1, 1)).item()
        first = next(iter(target.values())) if isinstance(target, dict) else target
        if first.device.type != "cuda":
            raise RuntimeError("MixingAugment (MI355X build) blends ROCm tensors only")
        r_index = torch.randperm(first.size(0))
        perm = r_index.to(device=first.device, dtype=torch.int32)

        def blend(v):
            return _mix(v, perm, lam) if v is not None else None

        mixed_target = {k: blend(v) for k, v in target.items()} if isinstance(target, dict) else blend(target)
        mixed_input = {k: blend(v) for k, v in input_.items()} if isinstance(input_, dict) else blend(input_)
        return mixed_target, mixed_input

    def __call__(self, target, input_):
        if self.use_identity:
            augment_idx = random.randint(0, len(self.augments))  # includes "no augmentation"
        else:
            augment_idx = random.randint(0, len(self.augments) - 1)
        if augment_idx < len(self.augments):
            target, input_ = self.augments[augment_idx](target, input_)
        return target, input_


def sync_gradients(grad: torch.Tensor, group=None) -> float:
    """DDP gradient averaging (base_model.py:76-82) as ONE all-reduce over the flat gradient buffer.

    Sums in place over the process group (RCCL on ROCm, gloo on CPU) and returns the scale
    (1 / world size) that the clip + AdamW kernel folds in, so the mean never costs a pass."""
    if not (dist.is_available() and dist.is_initialized()):
        return 1.0
    ws = dist.get_world_size(group)
    if ws == 1:
        return 1.0
    if grad.is_cuda and dist.get_backend(group) != "nccl":
        host = grad.cpu()  # gloo reduces host memory (multi-process tests sharing one GPU)
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        grad.copy_(host)
    else:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
    return 1.0 / ws


def grad_buckets(mark_los, numel: int, cap_floats: int):
    """DDP-style gradient buckets over the flat buffer from the backward's gradient-ready marks.

    ``mark_los[j]``: the suffix [lo, numel) is final at mark j (decreasing).  Consecutive marks are
    merged until a bucket holds ``cap_floats`` (DistributedDataParallel's bucket_cap_mb, 25 MB by
    default); returns [(mark or None, lo, hi)] covering [0, numel) exactly, back to front.  A bucket
    waits on its mark's event; None = after the whole backward."""
    out, hi = [], numel
    for j, lo in enumerate(mark_los):
        if lo < hi and hi - lo >= cap_floats:
            out.append((j, lo, hi))
            hi = lo
    if hi > 0:
        last = len(mark_los) - 1 if mark_los and mark_los[-1] == 0 else None
        out.append((last, 0, hi))
    return out


def allreduce_buckets_rccl(grad: torch.Tensor, buckets, handle, group=None) -> None:
    """RCCL leg of ``sync_gradients_bucketed``: each bucket's SUM all-reduce is enqueued on the
    communication stream behind its gradient-ready event; the current stream waits for all of them."""
    L = _lib.lib()
    comm = _comm_stream(grad.device)
    cur = torch.cuda.current_stream(grad.device)
    works = []
    for j, lo, hi in buckets:
        if j is None:
            comm.wait_stream(cur)
        else:
            _lib.check(L.kdlae_tt_mark_wait(handle, j, ctypes.c_void_p(comm.cuda_stream)), "kdlae_tt_mark_wait")
        with torch.cuda.stream(comm):
            works.append(dist.all_reduce(grad[lo:hi], op=dist.ReduceOp.SUM, group=group, async_op=True))
    for w in works:
        w.wait()
    cur.wait_stream(comm)


def sync_gradients_bucketed(grad: torch.Tensor, buckets, handle=None, group=None) -> float:
    """The DDP all-reduce overlapped with the backward: bucket (j, lo, hi) of ``grad`` is all-reduced on
    a communication stream as soon as the backward has recorded gradient-ready event j
    (``kdlae_tt_mark_wait``), while the backward's later layers still run; the current stream then
    waits for every bucket.  Returns the 1 / world-size scale, like ``sync_gradients``.  On gloo
    (host collectives: the multi-process tests) each bucket waits for its event on the host."""
    if not (dist.is_available() and dist.is_initialized()):
        return 1.0
    ws = dist.get_world_size(group)
    if ws == 1:
        return 1.0
    L = _lib.lib()
    if grad.is_cuda and dist.get_backend(group) == "nccl":
        allreduce_buckets_rccl(grad, buckets, handle, group)
        return 1.0 / ws
    if not grad.is_cuda:
        for _, lo, hi in buckets:
            dist.all_reduce(grad[lo:hi], op=dist.ReduceOp.SUM, group=group)
        return 1.0 / ws
    # gloo on device gradients: the same event-ordered schedule as RCCL, with each bucket staged
    # through pinned host memory by a stream-ordered copy on the communication stream (so a bucket
    # leaves the device when its event fires, not after the whole backward)
    comm = _comm_stream(grad.device)
    cur = torch.cuda.current_stream(grad.device)
    staged = []
    for j, lo, hi in buckets:
        if j is None:
            comm.wait_stream(cur)
        else:
            _lib.check(L.kdlae_tt_mark_wait(handle, j, ctypes.c_void_p(comm.cuda_stream)), "kdlae_tt_mark_wait")
        host = torch.empty(hi - lo, dtype=grad.dtype, pin_memory=True)
        with torch.cuda.stream(comm):
            host.copy_(grad[lo:hi], non_blocking=True)
        comm.synchronize()  # this bucket's event wait and copy only
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        with torch.cuda.stream(comm):
            grad[lo:hi].copy_(host, non_blocking=True)
        staged.append(host)
    cur.wait_stream(comm)
    comm.synchronize()  # the pinned staging buffers outlive their copies
    return 1.0 / ws


_COMM = {}


def _comm_stream(device):
    key = torch.device(device).index
    if key not in _COMM:
        _COMM[key] = torch.cuda.Stream(device=device)
    return _COMM[key]


def _position_from_periods(iteration: int, cumulative_period) -> int:
    """get_position_from_periods (Train/basicsr/models/lr_scheduler.py:115-133)."""
    for i, period in enumerate(cumulative_period):
        if iteration <= period:
            return i
    return None


class CosineAnnealingRestartCyclicLR:
    """The LR schedule of KDLAET.yml (train.scheduler, :95-99), lr_scheduler.py:186-233 restated
    over the trainer's single parameter group: ``lr(last_epoch)`` is what the reference's
    ``get_lr`` returns after ``last_epoch`` scheduler steps."""

    def __init__(self, base_lr: float, periods, restart_weights=(1,), eta_mins=(0,)):
        if len(periods) != len(restart_weights):
            raise ValueError("periods and restart_weights should have the same length.")
        self.base_lr = float(base_lr)
        self.periods, self.restart_weights, self.eta_mins = list(periods), list(restart_weights), list(eta_mins)
        self.cumulative_period = [sum(self.periods[:i + 1]) for i in range(len(self.periods))]

    def lr(self, last_epoch: int) -> float:
        idx = _position_from_periods(last_epoch, self.cumulative_period)
        w = self.restart_weights[idx]
        nearest_restart = 0 if idx == 0 else self.cumulative_period[idx - 1]
        eta_min = self.eta_mins[idx]
        return eta_min + w * 0.5 * (self.base_lr - eta_min) * (
            1 + math.cos(math.pi * ((last_epoch - nearest_restart) / self.periods[idx])))


class KDLAETrainer:
    """ImageCleanModel.optimize_parameters for KDLAE_teacher (image_restoration_model.py:198-218).

    Defaults follow Train/Denoising/Options/paper202508/KDLAET.yml: AdamW lr 1e-5,
    weight_decay 5e-5, betas (0.2, 0.999); use_grad_clip -> clip_grad_norm_(0.01); L1LossSr."""

    def __init__(self, model, lr=1e-5, weight_decay=0.5e-4, betas=(0.2, 0.999), eps=1e-8, use_grad_clip=True,
                 max_norm=0.01, loss_weight=1.0, group=None, mixing_augs=None, ema_decay=0.0, scheduler=None,
                 bucket_cap_mb=25.0, overlap_grad_reduce=True):
        params = list(model.parameters())
        if not params or params[0].device.type != "cuda":
            raise RuntimeError("KDLAETrainer: move the model to a ROCm device first (no CPU fallback)")
        dev = params[0].device
        self.model = model
        self.engine = TrainEngine(model, dev)
        eng = self.engine
        # flat parameter buffer; the module's parameters become views of it
        self.theta = eng.flatten(params).contiguous()
        with torch.no_grad():
            for (k, n, off), p in zip(eng.keys, params):
                p.data = self.theta[off:off + n].view(p.shape)
        self.grad = torch.zeros(eng.numel, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros_like(self.grad)
        self.exp_avg_sq = torch.zeros_like(self.grad)
        self.lr, self.weight_decay, self.betas, self.eps = lr, weight_decay, tuple(betas), eps
        self.init_lr = lr
        # train.scheduler (e.g. CosineAnnealingRestartCyclicLR for KDLAET.yml); driven by the caller
        # through update_learning_rate(current_iter) like BaseModel's, else the lr stays fixed
        self.scheduler = scheduler
        self.max_norm = max_norm if use_grad_clip else 0.0
        self.loss_weight = loss_weight
        self.group = group
        # DDP gradient buckets (DistributedDataParallel(bucket_cap_mb=25), base_model.py:76-82):
        # all-reduced while the backward still runs; overlap_grad_reduce=False = one collective after it
        self.bucket_cap_floats = max(1, int(bucket_cap_mb * 1024 * 1024 / 4))
        self.overlap_grad_reduce = overlap_grad_reduce
        self.buckets = None
        self.step_count = 0
        self.output = None
        self.loss = None
        ranges = eng.used_ranges()
        self._ranges = (ctypes.c_int64 * (2 * len(ranges)))(*[v for r in ranges for v in r])
        self._nranges = len(ranges) if len(ranges) != 1 or ranges[0] != [0, eng.numel] else 0
        L = _lib.lib()
        self._l1_scratch = torch.empty(int(L.kdlae_train_l1sr_scratch_floats()), dtype=torch.float32, device=dev)
        self._opt_scratch = torch.empty(int(L.kdlae_train_adamw_scratch_floats()), dtype=torch.float32, device=dev)
        self._loss = torch.zeros((), dtype=torch.float32, device=dev)
        # KDLAET.yml train.mixing_augs ({mixup, mixup_beta, use_identity}); ImageCleanModel.__init__ :83-87
        m = mixing_augs or {}
        self.mixing = (MixingAugment(m.get("mixup_beta", 1.2), m.get("use_identity", False), dev)
                       if m.get("mixup", False) else None)
        # train.ema_decay (ImageCleanModel.__init__: net_g_ema starts as a copy of net_g, model_ema(0))
        self.ema_decay = float(ema_decay)
        self.theta_ema = self.theta.clone() if self.ema_decay > 0 else None

    def update_learning_rate(self, current_iter: int, warmup_iter: int = -1) -> float:
        """BaseModel.update_learning_rate (Train/basicsr/models/base_model.py:183-205): the scheduler
        has stepped current_iter - 1 times by iteration current_iter (train.py calls this before
        optimize_parameters); linear warm-up below warmup_iter.  Returns the lr now in force."""
        if self.scheduler is not None:
            self.lr = self.scheduler.lr(max(current_iter - 1, 0))
        if current_iter < warmup_iter:
            self.lr = self.init_lr / warmup_iter * current_iter
        return self.lr

    def feed_train_data(self, lq: dict, gt: dict):
        """ImageCleanModel.feed_train_data (:161-186): the optional mixup of (gt, lq)."""
        if self.mixing is not None:
            gt, lq = self.mixing(gt, lq)
        return lq, gt

    def ema_state_dict(self):
        """net_g_ema's parameters (``params_ema`` in BasicSR checkpoints) as views of the EMA buffer."""
        if self.theta_ema is None:
            raise RuntimeError("ema_decay is 0: there is no EMA copy")
        return {k: self.theta_ema[off:off + n].view(p.shape)
                for (k, n, off), p in zip(self.engine.keys, self.model.parameters())}

    def _distributed(self) -> bool:
        return dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1

    def forward_backward(self, lq: dict, gt: dict, marked: bool = False):
        """preds = net_g(lq); l_pix = cri_pix(preds, gt); l_pix.backward()  (:198-213).

        ``marked``: record gradient-ready marks and build ``self.buckets`` for the overlapped all-reduce."""
        eng, L = self.engine, _lib.lib()
        hq, sr = eng.forward(self.theta, lq["img"], lq.get("denoise_rate"))
        self.output = {"hq": hq, "sr": sr}
        dhq = torch.empty_like(hq)
        dsr = torch.empty_like(sr) if sr is not None else None
        gt_hq = gt["hq"].to(torch.float32).contiguous()
        gt_sr = gt["sr"].to(torch.float32).contiguous() if sr is not None else None
        rc = L.kdlae_train_l1sr(_vp(hq), _vp(gt_hq), hq.numel(), _vp(sr), _vp(gt_sr), sr.numel() if sr is not None
                                else 0, _vp(dhq), _vp(dsr), _vp(self._loss), _vp(self._l1_scratch),
                                _stream(hq.device))
        _lib.check(rc, "kdlae_train_l1sr")
        if self.loss_weight != 1.0:
            dhq.mul_(self.loss_weight)
            if dsr is not None:
                dsr.mul_(self.loss_weight)
        if marked:
            self.buckets = grad_buckets(eng.backward(self.theta, dhq, dsr, self.grad, marked=True), eng.numel,
                                        self.bucket_cap_floats)
        else:
            eng.backward(self.theta, dhq, dsr, self.grad)
        self.loss = self._loss * self.loss_weight
        return self.loss

    def step(self, gscale: float = 1.0):
        """clip_grad_norm_(net_g.parameters(), 0.01) + AdamW step (:215-218) over the flat buffers."""
        self.step_count += 1
        b1, b2 = self.betas
        rc = _lib.lib().kdlae_train_clip_adamw(
            _vp(self.theta), _vp(self.grad), _vp(self.exp_avg), _vp(self.exp_avg_sq), self.engine.numel,
            float(gscale), float(self.max_norm), float(self.lr), float(b1), float(b2), float(self.eps),
            float(self.weight_decay), self.step_count, self._ranges if self._nranges else None, self._nranges,
            _vp(self._opt_scratch), _stream(self.theta.device))
        _lib.check(rc, "kdlae_train_clip_adamw")
        if self.theta_ema is not None:  # model_ema(decay) after the step (:221-222)
            rc = _lib.lib().kdlae_train_ema(_vp(self.theta_ema), _vp(self.theta), self.engine.numel,
                                            self.ema_decay, _stream(self.theta.device))
            _lib.check(rc, "kdlae_train_ema")

    def optimize_parameters(self, lq: dict, gt: dict):
        """One full iteration: forward, L1LossSr, backward, DDP all-reduce, clip, AdamW.  With several
        ranks the all-reduce runs in gradient buckets overlapped with the backward (overlap_grad_reduce)."""
        if self._distributed() and self.overlap_grad_reduce:
            loss = self.forward_backward(lq, gt, marked=True)
            gscale = sync_gradients_bucketed(self.grad, self.buckets, self.engine.handle, self.group)
        else:
            loss = self.forward_backward(lq, gt)
            gscale = sync_gradients(self.grad, self.group)
        self.step(gscale)
        return loss

    def grad_norm(self) -> torch.Tensor:
        """Gradient norm of the last step (after DDP averaging, before clipping)."""
        return self._opt_scratch[2048]

    def get_current_log(self):
        return {"l_pix": float(self.loss)} if self.loss is not None else {}
