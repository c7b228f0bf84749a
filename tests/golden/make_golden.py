"""Generate golden fixtures from the IMPORTED REFERENCE (build container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

* Imports ``KDLAE/KDLAE_model.py`` and ``ASDQE/ASDQE_model.py`` from /root/reference (read
  only, no bytecode written).  Nothing from the reference is copied into this repository: only
  the numeric outputs below are saved.
* Weights: the §8c hash recipe (rethink_acoustic_image_enhancement_amd/hashweights.py).
* Inputs: hash images (key names stored in the fixture) and, for config 1, the decoded
  ``Sample/MDD/origin/0001_sort.jpg`` crop stored as uint8.
* Outputs: fp32 tensors (small shapes) or [::8, ::8] subsamples + float64 channel sums (512^2).
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from rethink_acoustic_image_enhancement_amd.hashweights import (  # noqa: E402
    hash_images, hash_normal, hash_state_dict)

REF = "/root/reference"
sys.dont_write_bytecode = True


def _import_ref():
    sys.path.insert(0, os.path.join(REF, "KDLAE"))
    sys.path.insert(0, os.path.join(REF, "ASDQE"))
    import ASDQE_model  # noqa: F401
    import KDLAE_model  # noqa: F401
    return KDLAE_model, ASDQE_model


def _load_hash(model):
    sd = model.state_dict()
    vals = hash_state_dict({k: tuple(v.shape) for k, v in sd.items()})
    model.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()}, strict=True)
    return model.eval()


TEACHER_CASES = {
    # name: (ctor kwargs, img shape, rate spec)
    "t_full_b2_32": (dict(dim=48, num_blocks=[4, 6, 6, 8], num_refinement_blocks=4,
                          heads=[1, 2, 4, 8], LayerNorm_type="BiasFree", bias=False,
                          static="train", params="cat"), (2, 3, 32, 32), "const:0.6,0.25"),
    "t_full_b1_48x80": (dict(dim=48, num_blocks=[4, 6, 6, 8], num_refinement_blocks=4,
                             heads=[1, 2, 4, 8], LayerNorm_type="BiasFree", bias=False,
                             static="train", params="cat"), (1, 3, 48, 80), "map"),
    "t_tiny_withbias": (dict(dim=16, num_blocks=[1, 2, 1, 1], num_refinement_blocks=1,
                             heads=[1, 2, 4, 8], LayerNorm_type="WithBias", bias=True,
                             static="train", params="cat"), (2, 3, 32, 48), "map"),
    "t_tiny_nocat_nosr": (dict(dim=16, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1,
                               heads=[1, 1, 2, 2], LayerNorm_type="BiasFree", bias=False,
                               static="no", params="plus"), (1, 3, 40, 24), "const:0.5"),
    "t_gray_1ch": (dict(inp_channels=1, out_channels=1, dim=16, num_blocks=[1, 1, 1, 1],
                        num_refinement_blocks=1, heads=[1, 2, 4, 8],
                        LayerNorm_type="BiasFree", bias=False, static="train", params="cat"),
                   (1, 1, 24, 32), "const:0.9"),
}


def make_rate(spec, b, h, w, key):
    if spec.startswith("const:"):
        vals = [float(v) for v in spec[6:].split(",")]
        vals = (vals * b)[:b]
        return np.stack([np.full((1, h, w), v, np.float32) for v in vals])
    return hash_images(key, (b, 1, h, w))


def teacher_goldens(KM, out):
    for name, (kw, shape, rspec) in TEACHER_CASES.items():
        t0 = time.time()
        m = _load_hash(KM.KDLAE_teacher(**kw))
        b, c, h, w = shape
        img = hash_images(f"img:{name}", shape)
        rate = make_rate(rspec, b, h, w, f"rate:{name}")
        with torch.no_grad():
            o = m({"img": torch.from_numpy(img), "denoise_rate": torch.from_numpy(rate)})
        d = dict(img=img, rate=rate, hq=o["hq"].numpy())
        if o["sr"] is not None:
            d["sr"] = o["sr"].numpy()
        d["cfg"] = np.frombuffer(json.dumps(kw).encode(), dtype=np.uint8)
        np.savez_compressed(os.path.join(out, f"{name}.npz"), **d)
        print(name, {k: v.shape for k, v in d.items()}, f"{time.time() - t0:.1f}s")


def mdd_input():
    """Config 1 input: 0001_sort.jpg rows 73:585, reflect-pad width 438 -> 512."""
    from PIL import Image

    im = np.asarray(Image.open(os.path.join(REF, "Sample/MDD/origin/0001_sort.jpg")).convert("RGB"))
    crop = im[73:585]                       # [512, 438, 3] uint8
    assert crop.shape[:2] == (512, 438), crop.shape
    return crop


def _run512(KM, img, kw, dtype):
    m = _load_hash(KM.KDLAE_teacher(**kw)).to(dtype)
    rate = torch.full((1, 1, 512, 512), 0.6, dtype=dtype)
    t0 = time.time()
    with torch.no_grad():
        o = m({"img": img.to(dtype), "denoise_rate": rate})
    return o["hq"], o["sr"], time.time() - t0


def teacher_512(KM, out):
    """512x512 KDLAE-T goldens: config-1 MDD input and a hash-uniform image, each from the
    reference in fp32 (the comparison target) AND in fp64 (the conditioning reference: on the MDD
    sonar image the reference's own fp32 result is ~3e-3 away from fp64)."""
    kw = dict(dim=48, num_blocks=[4, 6, 6, 8], num_refinement_blocks=4, heads=[1, 2, 4, 8],
              LayerNorm_type="BiasFree", bias=False, static="train", params="cat")
    crop = mdd_input()
    mdd = torch.from_numpy(crop.astype(np.float32) / 255.0).permute(2, 0, 1).unsqueeze(0)
    mdd = torch.nn.functional.pad(mdd, (0, 74, 0, 0), mode="reflect")
    rnd = torch.from_numpy(hash_images("img:t_rand_512", (1, 3, 512, 512)))
    for name, img, extra in (("t_mdd_512", mdd, dict(crop_u8=crop[..., 0] if (crop[..., 0] == crop[..., 1]).all()
                                                     and (crop[..., 0] == crop[..., 2]).all() else crop)),
                             ("t_rand_512", rnd, dict())):
        hq, sr, dt = _run512(KM, img, kw, torch.float32)
        hq64, sr64, dt64 = _run512(KM, img, kw, torch.float64)
        np.savez_compressed(
            os.path.join(out, f"{name}.npz"), **extra,
            hq_sub=hq[:, :, ::8, ::8].numpy(), sr_sub=sr[:, :, ::8, ::8].numpy(),
            hq64_sub=hq64[:, :, ::8, ::8].numpy(), sr64_sub=sr64[:, :, ::8, ::8].numpy(),
            hq_chsum=hq.double().sum(dim=(2, 3)).numpy(), sr_chsum=sr.double().sum(dim=(2, 3)).numpy(),
            hq64_chsum=hq64.sum(dim=(2, 3)).numpy(), sr64_chsum=sr64.sum(dim=(2, 3)).numpy(),
            hq_row257=hq[:, :, 257, :].numpy(), sr_row515=sr[:, :, 515, :].numpy(),
            hq64_row257=hq64[:, :, 257, :].numpy(), sr64_row515=sr64[:, :, 515, :].numpy(),
            ref_cpu_seconds=np.array([dt]), threads=np.array([torch.get_num_threads()]),
            cfg=np.frombuffer(json.dumps(kw).encode(), dtype=np.uint8))
        e = float((hq[:, :, ::8, ::8].double() - hq64[:, :, ::8, ::8]).abs().max())
        print(name, f"fp32 {dt:.1f}s fp64 {dt64:.1f}s  ref fp32-vs-fp64 hq_sub max-abs {e:.3e}")


STUDENT_CASES = {
    "s_default_b2": (dict(inp_channels=1, out_channels=1, residual=True, hidden_channels=[16, 32, 64]),
                     (2, 4, 32, 32)),
    "s_nores_3lvl": (dict(inp_channels=1, out_channels=1, residual=False, hidden_channels=[8, 16, 16, 32]),
                     (1, 3, 24, 40)),
}


def student_goldens(KM, out):
    for name, (kw, shape) in STUDENT_CASES.items():
        m = _load_hash(KM.KDLAE_student(**kw))
        x = hash_images(f"frames:{name}", shape)
        with torch.no_grad():
            y = m(torch.from_numpy(x)).numpy()
        np.savez_compressed(os.path.join(out, f"{name}.npz"), x=x, y=y,
                            cfg=np.frombuffer(json.dumps(kw).encode(), dtype=np.uint8))
        print(name, y.shape)


ASDQE_CASES = {
    "a_b4_64": (dict(in_channels=3, dim=16), (4, 3, 64, 64)),
    "a_b2_40x56": (dict(in_channels=3, dim=16), (2, 3, 40, 56)),   # exercises pad_to_multiple
}


def asdqe_goldens(AM, out):
    """Score plus the intermediates a near-constant score cannot pin: pooled UNet features (float64),
    a [::4, ::4] subsample of the UNet output map and of the merged extractor features.  Images
    differ per sample in brightness and noise level so that the score varies."""
    for name, (kw, shape) in ASDQE_CASES.items():
        m = _load_hash(AM.DenoiseRatePredictor(**kw))
        B = shape[0]
        scale = (0.3 + 0.7 * np.arange(1, B + 1) / B).reshape(B, 1, 1, 1)
        sigma = (0.02 + 0.2 * np.arange(B) / max(B - 1, 1)).reshape(B, 1, 1, 1)
        gt = (hash_images(f"gt:{name}", shape) * scale).astype(np.float32)
        lq = np.clip(gt + sigma * hash_normal(f"noise:{name}", shape), 0, 1).astype(np.float32)
        cap = {}
        h1 = m.unet.register_forward_hook(lambda mod, i, o: cap.__setitem__("feat", o.detach().clone()))
        h2 = m.unet.register_forward_pre_hook(lambda mod, i: cap.__setitem__("merged", i[0].detach().clone()))
        with torch.no_grad():
            y = m(torch.from_numpy(lq), torch.from_numpy(gt)).numpy()
        h1.remove()
        h2.remove()
        feat, merged = cap["feat"], cap["merged"]
        np.savez_compressed(os.path.join(out, f"{name}.npz"), lq=lq, gt=gt, score=y,
                            gap64=feat.double().mean(dim=(2, 3)).numpy(),
                            feat_sub=feat[:, :, ::4, ::4].numpy(), merged_sub=merged[:, :, ::4, ::4].numpy(),
                            cfg=np.frombuffer(json.dumps(kw).encode(), dtype=np.uint8))
        print(name, y.ravel(), tuple(feat.shape))


TRAIN_CASES = {
    # name: (ctor kwargs, img shape); training step goldens
    "train_tiny_biasfree": (dict(dim=8, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, heads=[1, 2, 4, 8],
                                 LayerNorm_type="BiasFree", bias=False, static="train", params="cat"), (2, 3, 32, 32)),
    "train_tiny_withbias": (dict(dim=8, num_blocks=[1, 2, 1, 1], num_refinement_blocks=1, heads=[1, 1, 2, 2],
                                 LayerNorm_type="WithBias", bias=True, static="train", params="cat"), (1, 3, 24, 40)),
    "train_nocat_nosr": (dict(dim=8, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, heads=[1, 1, 2, 2],
                              LayerNorm_type="BiasFree", bias=False, static="no", params="plus"), (1, 3, 32, 24)),
}
TRAIN_OPT = dict(lr=1e-3, weight_decay=0.5e-4, betas=(0.2, 0.999))  # KDLAET.yml betas/wd, larger lr
TRAIN_CLIP = 0.01
TRAIN_SUB = 5  # flat gradients / parameter deltas are stored at every 5th element (+ per-key float64 sums)


def train_goldens(KM, out):
    """Loss + every parameter gradient of the reference module under L1LossSr, then the parameters
    after two clip_grad_norm_(0.01) + AdamW steps (image_restoration_model.py:198-218).  The loss
    is the oracle's restatement of losses.py:135-194 (basicsr is not importable here)."""
    from oracle.train_oracle import l1sr_loss

    for name, (kw, shape) in TRAIN_CASES.items():
        t0 = time.time()
        m = _load_hash(KM.KDLAE_teacher(**kw)).train()
        b, c, h, w = shape
        img = hash_images(f"img:{name}", shape)
        rate = hash_images(f"rate:{name}", (b, 1, h, w))
        gt_hq = hash_images(f"gt_hq:{name}", shape)
        gt_sr = hash_images(f"gt_sr:{name}", (b, c, 2 * h, 2 * w))
        inp = {"img": torch.from_numpy(img), "denoise_rate": torch.from_numpy(rate)}
        gt = {"hq": torch.from_numpy(gt_hq), "sr": torch.from_numpy(gt_sr)}
        params = list(m.parameters())
        params0 = np.concatenate([p.detach().reshape(-1).numpy() for p in params]).astype(np.float64)
        opt = torch.optim.AdamW(params, **TRAIN_OPT)
        losses, norms = [], []
        for step in range(2):
            opt.zero_grad()
            loss = l1sr_loss(m(inp), gt)
            loss.backward()
            if step == 0:
                gl = [(p.grad if p.grad is not None else torch.zeros_like(p)).detach().reshape(-1).numpy()
                      for p in params]
                grad1 = np.concatenate(gl)
                gsums = np.array([[g.astype(np.float64).sum(), np.abs(g).astype(np.float64).sum()] for g in gl])
                used = np.array([p.grad is not None for p in params], np.uint8)
            norms.append(float(torch.nn.utils.clip_grad_norm_(params, TRAIN_CLIP)))
            opt.step()
            losses.append(float(loss))
        keys = [k for k, _ in m.named_parameters()]
        params2 = np.concatenate([p.detach().reshape(-1).numpy() for p in params]).astype(np.float64)
        d = dict(img=img, rate=rate, gt_hq=gt_hq, gt_sr=gt_sr, loss=np.array(losses, np.float64),
                 norm=np.array(norms, np.float64), grad1_sub=grad1[::TRAIN_SUB].astype(np.float32), grad_sums=gsums,
                 used=used, delta2_sub=(params2 - params0)[::TRAIN_SUB].astype(np.float32),
                 keys=np.frombuffer(json.dumps(keys).encode(), dtype=np.uint8),
                 cfg=np.frombuffer(json.dumps(kw).encode(), dtype=np.uint8),
                 opt=np.frombuffer(json.dumps(dict(TRAIN_OPT, clip=TRAIN_CLIP)).encode(), dtype=np.uint8))
        np.savez_compressed(os.path.join(out, f"{name}.npz"), **d)
        print(name, losses, norms, grad1.shape, f"{time.time() - t0:.1f}s")


# ---------------------------------------------------------------- KDLAE-S training (KDLAES.yml)
S_TRAIN_CASES = {
    # name: (ctor kwargs, x shape [B, F, H, W], loss kwargs)
    "train_s_kdlaes": (dict(inp_channels=1, out_channels=1, residual=True, hidden_channels=[16, 32, 64]), (2, 7, 32, 32),
                       dict(l1loss_weight=0.9, temporal_weight=0.1, reduction="mean")),
    "train_s_4lvl_sum": (dict(inp_channels=1, out_channels=1, residual=False, hidden_channels=[8, 16, 16, 32]),
                         (1, 3, 16, 24), dict(reduction="sum")),
    "train_s_1frame": (dict(inp_channels=1, out_channels=1, residual=True, hidden_channels=[12, 20]), (2, 1, 8, 12),
                       dict(l1loss_weight=0.9, temporal_weight=0.1, reduction="mean")),
}
S_TRAIN_OPT = dict(lr=3e-4, weight_decay=1e-4, betas=(0.9, 0.999))  # KDLAES.yml optim_g
S_TRAIN_SUB = 4  # flat gradients / parameter deltas kept at every 4th element (+ per-key float64 sums)


def _ref_video_loss():
    """L1LossForVideoFrames from the reference's own losses.py, loaded by path (its only import outside
    torch / numpy is basicsr.models.losses.loss_util, registered under that name from the reference's
    loss_util.py; the basicsr package itself needs cv2)."""
    import importlib.util
    import types
    base = os.path.join(REF, "Train", "basicsr", "models", "losses")
    for pkg in ("basicsr", "basicsr.models", "basicsr.models.losses"):
        if pkg not in sys.modules:
            m = types.ModuleType(pkg)
            m.__path__ = []
            sys.modules[pkg] = m
    for mod, fn in (("basicsr.models.losses.loss_util", "loss_util.py"), ("ref_losses", "losses.py")):
        spec = importlib.util.spec_from_file_location(mod, os.path.join(base, fn))
        m = importlib.util.module_from_spec(spec)
        sys.modules[mod] = m
        spec.loader.exec_module(m)
    return sys.modules["ref_losses"].L1LossForVideoFrames


def student_train_goldens(KM, out):
    """Loss + every parameter gradient of the reference KDLAE_student under the reference's
    L1LossForVideoFrames (autograd through both), then the parameters after two clip_grad_norm_(0.01)
    + AdamW steps (image_restoration_model.py:198-218, KDLAES.yml optim_g)."""
    Loss = _ref_video_loss()
    for name, (kw, shape, lkw) in S_TRAIN_CASES.items():
        t0 = time.time()
        m = _load_hash(KM.KDLAE_student(**kw)).train()
        x = hash_images(f"sx:{name}", shape)
        tgt = hash_images(f"st:{name}", shape)
        crit = Loss(**lkw)
        params = list(m.parameters())
        params0 = np.concatenate([p.detach().reshape(-1).numpy() for p in params]).astype(np.float64)
        opt = torch.optim.AdamW(params, **S_TRAIN_OPT)
        losses, norms = [], []
        for step in range(2):
            opt.zero_grad()
            loss = crit(m(torch.from_numpy(x)), torch.from_numpy(tgt))
            loss.backward()
            if step == 0:
                gl = [p.grad.detach().reshape(-1).numpy() for p in params]
                grad1 = np.concatenate(gl)
                gsums = np.array([[g.astype(np.float64).sum(), np.abs(g).astype(np.float64).sum()] for g in gl])
            norms.append(float(torch.nn.utils.clip_grad_norm_(params, TRAIN_CLIP)))
            opt.step()
            losses.append(float(loss))
        keys = [k for k, _ in m.named_parameters()]
        params2 = np.concatenate([p.detach().reshape(-1).numpy() for p in params]).astype(np.float64)
        d = dict(x=x, target=tgt, loss=np.array(losses, np.float64), norm=np.array(norms, np.float64),
                 grad1_sub=grad1[::S_TRAIN_SUB].astype(np.float32), grad_sums=gsums,
                 delta2_sub=(params2 - params0)[::S_TRAIN_SUB].astype(np.float32),
                 keys=np.frombuffer(json.dumps(keys).encode(), dtype=np.uint8),
                 cfg=np.frombuffer(json.dumps(kw).encode(), dtype=np.uint8),
                 loss_kw=np.frombuffer(json.dumps(lkw).encode(), dtype=np.uint8),
                 opt=np.frombuffer(json.dumps(dict(S_TRAIN_OPT, clip=TRAIN_CLIP)).encode(), dtype=np.uint8))
        np.savez_compressed(os.path.join(out, f"{name}.npz"), **d)
        print(name, losses, norms, grad1.shape, f"{time.time() - t0:.1f}s")


# ---------------------------------------------------------------- checkpoint layout
CKPT_CASES = {
    # name: (which model, ctor kwargs, input shape)
    "ckpt_t_tiny": ("teacher", dict(dim=16, num_blocks=[1, 2, 1, 1], num_refinement_blocks=1, heads=[1, 2, 4, 8],
                                    LayerNorm_type="BiasFree", bias=False, static="train", params="cat"), (1, 3, 32, 48)),
    "ckpt_s_default": ("student", dict(inp_channels=1, out_channels=1, residual=True, hidden_channels=[16, 32, 64]),
                       (1, 4, 32, 32)),
    "ckpt_a_default": ("asdqe", dict(in_channels=3, dim=16), (2, 3, 48, 48)),
}


def _two_level(sd):
    """Every float tensor snapped to its own {min, max}: the checkpoint keeps the reference's
    layout (keys, shapes, dtypes, BN buffers) but compresses to ~1 bit per value under xz."""
    out = {}
    for k, v in sd.items():
        if v.is_floating_point() and v.numel() > 1 and float(v.max()) > float(v.min()):
            lo, hi = v.min(), v.max()
            v = torch.where(v > (lo + hi) / 2, hi, lo).to(v.dtype)
        out[k] = v.clone()
    return out


def ckpt_goldens(KM, AM, out):
    """Checkpoints WRITTEN BY THE REFERENCE MODULES in the reference's on-disk layouts, plus the
    reference's outputs for them:
    * KDLAE-T / KDLAE-S: BasicSR save_network (Train/basicsr/models/base_model.py:213-244):
      torch.save({'params': sd, 'params_ema': sd_ema}) of net.state_dict() moved to CPU;
      consumers load ['params'] strictly (KDLAE_T.ipynb:1074-1075, KDLAE-S.ipynb:109-110).
    * ASDQE: torch.save(model.state_dict()) (Train/ASDQE.py:210,215,219), raw, BN buffers
      included; consumer load_state_dict(..., strict=False) (ASDQE/ASDQE_test.py:75-84).
    Files are committed xz-compressed (tests decompress them to a temp dir)."""
    import io
    import lzma

    for name, (kind, kw, shape) in CKPT_CASES.items():
        ctor = {"teacher": KM.KDLAE_teacher, "student": KM.KDLAE_student, "asdqe": AM.DenoiseRatePredictor}[kind]
        m = _load_hash(ctor(**kw))
        sd = _two_level(m.state_dict())
        m.load_state_dict(sd, strict=True)
        ema = {k: (v * 0.75 if v.is_floating_point() else v.clone()) for k, v in sd.items()}
        outs = {}
        for tag, weights in (("params", sd), ("params_ema", ema)):
            if kind == "asdqe" and tag == "params_ema":
                continue
            m.load_state_dict(weights, strict=True)
            m.eval()
            with torch.no_grad():
                if kind == "teacher":
                    b, c, h, w = shape
                    img = hash_images(f"img:{name}", shape)
                    rate = np.full((b, 1, h, w), 0.6, np.float32)
                    o = m({"img": torch.from_numpy(img), "denoise_rate": torch.from_numpy(rate)})
                    outs.update({f"{tag}_hq": o["hq"].numpy(), f"{tag}_sr": o["sr"].numpy(), "img": img, "rate": rate})
                elif kind == "student":
                    x = hash_images(f"frames:{name}", shape)
                    outs.update({f"{tag}_y": m(torch.from_numpy(x)).numpy(), "x": x})
                else:
                    gt = hash_images(f"gt:{name}", shape)
                    lq = np.clip(gt + 0.1 * hash_normal(f"noise:{name}", shape), 0, 1).astype(np.float32)
                    cap = {}
                    hk = m.unet.register_forward_hook(lambda mod, i, o: cap.__setitem__("feat", o.detach().clone()))
                    score = m(torch.from_numpy(lq), torch.from_numpy(gt)).numpy()
                    hk.remove()
                    outs.update({"score": score, "feat_sub": cap["feat"][:, :, ::4, ::4].numpy(), "lq": lq, "gt": gt})
        buf = io.BytesIO()
        if kind == "asdqe":
            torch.save(m.state_dict(), buf)        # raw state_dict, as Train/ASDQE.py writes it
        else:
            save = {}
            for tag, net_sd in (("params", sd), ("params_ema", ema)):
                net = ctor(**kw)                      # net_g and net_g_ema are separate modules
                net.load_state_dict(net_sd, strict=True)
                state_dict = net.state_dict()         # base_model.py:237-242
                for key, param in state_dict.items():
                    if key.startswith("module."):
                        key = key[7:]
                    state_dict[key] = param.cpu()
                save[tag] = state_dict
            torch.save(save, buf)                   # base_model.py:244
        raw = buf.getvalue()
        with open(os.path.join(out, f"{name}.pth.xz"), "wb") as f:
            f.write(lzma.compress(raw, preset=9 | lzma.PRESET_EXTREME))
        np.savez_compressed(os.path.join(out, f"{name}.npz"), **outs,
                            cfg=np.frombuffer(json.dumps(dict(kind=kind, kw=kw)).encode(), dtype=np.uint8))
        print(name, f"pth {len(raw) / 1e6:.2f} MB -> xz {os.path.getsize(os.path.join(out, name + '.pth.xz')) / 1e3:.0f} KB",
              {k: v.shape for k, v in outs.items()})


def _restormer_arch():
    import importlib.util
    path = os.path.join(REF, "Train/basicsr/models/archs/restormer_arch.py")
    spec = importlib.util.spec_from_file_location("ref_restormer_arch", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def key_lists(KM, AM, out):
    """state_dict key -> [shape, dtype] lists of the reference modules at the released configs
    (KDLAE_T.ipynb:1059-1071 / KDLAET.yml:65-78; KDLAE-S.ipynb:106 / KDLAES.yml:64-69; ASDQE
    defaults), the BasicSR alias RestormerSuperResolutionParam2 and the plain Restormer whose
    pretrained weights KDLAET.yml:82-83 loads with strict_load_g: false."""
    RA = _restormer_arch()
    t_kw = dict(inp_channels=3, out_channels=3, dim=48, num_blocks=[4, 6, 6, 8], num_refinement_blocks=4,
                heads=[1, 2, 4, 8], ffn_expansion_factor=2.66, bias=False, LayerNorm_type="BiasFree",
                dual_pixel_task=False, static="train", params="cat")
    mods = {
        "KDLAE_teacher_released": (KM.KDLAE_teacher, t_kw),
        "KDLAE_teacher_static_no": (KM.KDLAE_teacher, dict(t_kw, static="no")),
        "KDLAE_teacher_ctor_defaults": (KM.KDLAE_teacher, {}),
        "RestormerSuperResolutionParam2_KDLAET_yml": (RA.RestormerSuperResolutionParam2, t_kw),
        "Restormer_BiasFree": (RA.Restormer, dict(LayerNorm_type="BiasFree")),
        "KDLAE_student_released": (KM.KDLAE_student, dict(inp_channels=1, out_channels=1, residual=True,
                                                          hidden_channels=[16, 32, 64])),
        "DenoiseRatePredictor_default": (AM.DenoiseRatePredictor, {}),
    }
    res = {}
    for name, (ctor, kw) in mods.items():
        sd = ctor(**kw).state_dict()
        res[name] = {"kwargs": kw, "keys": [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in sd.items()]}
        print(name, len(sd), "keys")
    with open(os.path.join(out, "ref_state_dict_keys.json"), "w") as f:
        json.dump(res, f, separators=(",", ":"))


def lr_goldens(out):
    """KDLAET.yml's LR curve from the reference scheduler itself (Train/basicsr/models/lr_scheduler.py,
    imported by file path): lr in force at iteration i, where BasicSR steps the scheduler once per
    iteration from i = 2 on (base_model.py:183-193)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_lr_scheduler",
                                                  os.path.join(REF, "Train/basicsr/models/lr_scheduler.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    cfg = dict(periods=[90000, 8000], restart_weights=[1, 1], eta_mins=[0.0003, 0.000001])
    opt = torch.optim.AdamW([torch.nn.Parameter(torch.zeros(1))], lr=1e-5)
    sch = mod.CosineAnnealingRestartCyclicLR(opt, **cfg)
    marks = sorted(set([1, 2, 3, 100, 45000, 89999, 90000, 90001, 90002, 94000, 97999, 98000, 98001]
                       + list(range(1, 98001, 997))))
    res = {}
    for it in range(1, 98002):
        if it > 1:
            sch.step()
        if it in marks:
            res[str(it)] = opt.param_groups[0]["lr"]
    with open(os.path.join(out, "lr_kdlaet.json"), "w") as f:
        json.dump({"scheduler": cfg, "base_lr": 1e-5, "lr_at_iter": res}, f)
    print("lr", len(res), "points")


def frames_goldens(KM, out):
    """KDLAE-S.ipynb's default sample ('Sample for US': Sample/CAMUS/origin, inp_frames 7, KDLAE_student
    hidden [16,32,64] residual): the first 7 frames in sorted order (the notebook draws a random start),
    cropped to 70x60 to keep the fixture small.  The PNGs are lossless BGRA-equivalent RGBA, so the
    decoded bytes are what cv2.imread(IMREAD_UNCHANGED) returns (channels reordered to BGRA).  Saved:
    the u8 frames, and the reference module's output on load_consecutive_stack -> pad-to-32 input."""
    import glob as _glob

    from PIL import Image

    from oracle.pipeline_oracle import load_consecutive_stack, notebook_pad
    files = sorted(_glob.glob(os.path.join(REF, "Sample/CAMUS/origin/*.png")))[:7]
    frames = []
    for f in files:
        a = np.asarray(Image.open(f))                    # RGBA
        a = a[..., [2, 1, 0, 3]] if a.shape[2] == 4 else a[..., ::-1]  # cv2 order: BGRA / BGR
        frames.append(np.ascontiguousarray(a[240:310, 260:320]))
    frames = np.stack(frames)                            # [7, 70, 60, 4]
    kw = dict(inp_channels=1, out_channels=1, residual=True, hidden_channels=[16, 32, 64])
    m = _load_hash(KM.KDLAE_student(**kw))
    x = notebook_pad(load_consecutive_stack(list(frames)), 32)
    with torch.no_grad():
        y = m(x)
    np.savez_compressed(os.path.join(out, "frames_camus7.npz"), frames=frames, restored=y.numpy(),
                        files=np.frombuffer(json.dumps([os.path.basename(f) for f in files]).encode(), np.uint8),
                        cfg=np.frombuffer(json.dumps(kw).encode(), dtype=np.uint8))
    print("frames", frames.shape, tuple(x.shape), tuple(y.shape))


def asdqe_scoring_goldens(AM, out):
    """ASDQE/ASDQE_test.py __main__ on the reference's own MDD samples: methods origin / Teacher /
    Student@0.05 (:145-149), pairs from sorted folder listings (:42-50), PIL RGB + ToTensor (:59-65),
    bs=1 infer (:87-104), calculate_statistics (:107-120) and visualize_comparison's CSV (:123-133,
    written here by pandas exactly as the script does).  Each 658x438 JPEG is cropped to 64x64 so the
    fixture stays small; hash weights (the released ASDQE.pth is not available offline)."""
    import io as _io

    import pandas as pd
    from PIL import Image

    base = os.path.join(REF, "Sample/MDD/origin")
    methods = {"origin": base, "Teacher": os.path.join(REF, "Sample/MDD/denoise/KDLAE-T"),
               "Student@0.05": os.path.join(REF, "Sample/MDD/denoise/KDLAE-S_prob@0.05")}
    m = _load_hash(AM.DenoiseRatePredictor())
    crop = (slice(200, 264), slice(180, 244))
    load = lambda p: np.asarray(Image.open(p).convert("RGB"))[crop]  # noqa: E731
    lq_files = sorted(os.listdir(base))
    lq = np.stack([load(os.path.join(base, f)) for f in lq_files])
    arrays, preds, stats = {"lq": lq}, {}, []
    for name, d in methods.items():
        gt = np.stack([load(os.path.join(d, f)) for f in sorted(os.listdir(d))])
        arrays["gt_" + name] = gt
        p = []
        with torch.no_grad():
            for i in range(len(lq_files)):
                t = lambda a: torch.from_numpy(a[i].astype(np.float32) / 255.0).permute(2, 0, 1)[None]  # noqa: E731
                p.extend(m(t(lq), t(gt)).cpu().numpy().flatten())
        p = np.array(p)
        preds[name] = p
        stats.append({"mean": np.mean(p), "std": np.std(p), "min": np.min(p), "25%": np.percentile(p, 25),
                      "50%": np.percentile(p, 50), "75%": np.percentile(p, 75), "max": np.max(p)})
    df = pd.DataFrame(stats)
    df.index = list(methods)
    buf = _io.StringIO()
    df.T.to_csv(buf, float_format="%.6f", index=True)
    np.savez_compressed(os.path.join(out, "asdqe_scoring_mdd.npz"), **arrays,
                        **{"pred_" + k: v for k, v in preds.items()},
                        csv=np.frombuffer(buf.getvalue().encode(), np.uint8),
                        methods=np.frombuffer(json.dumps(list(methods)).encode(), np.uint8),
                        cfg=np.frombuffer(json.dumps(dict(in_channels=3, dim=16)).encode(), np.uint8))
    print("asdqe scoring", {k: v.round(5).tolist()[:3] for k, v in preds.items()})
    print(buf.getvalue())


def main():
    KM, AM = _import_ref()
    out = HERE
    which = sys.argv[1:] or ["teacher", "student", "asdqe", "t512", "train", "ckpt", "keys", "lr", "frames", "scoring",
                             "train_s"]
    if "train" in which:
        train_goldens(KM, out)
    if "train_s" in which:
        student_train_goldens(KM, out)
    if "teacher" in which:
        teacher_goldens(KM, out)
    if "student" in which:
        student_goldens(KM, out)
    if "asdqe" in which:
        asdqe_goldens(AM, out)
    if "t512" in which:
        teacher_512(KM, out)
    if "ckpt" in which:
        ckpt_goldens(KM, AM, out)
    if "keys" in which:
        key_lists(KM, AM, out)
    if "lr" in which:
        lr_goldens(out)
    if "frames" in which:
        frames_goldens(KM, out)
    if "scoring" in which:
        asdqe_scoring_goldens(AM, out)


if __name__ == "__main__":
    main()
