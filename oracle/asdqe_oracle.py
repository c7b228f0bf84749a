"""TEST INFRASTRUCTURE ONLY — CPU oracle for the ASDQE forward (DenoiseRatePredictor, eval mode).

A from-scratch functional restatement (torch CPU ops on a plain state_dict) of
``ASDQE/ASDQE_model.py``.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may call it; the product package never imports it.

Pinning: ``tests/golden/a_*.npz`` hold the imported reference's score, its pooled UNet features
(float64) and a [::4, ::4] subsample of the UNet output map, with the §8c hash weights
(``tests/golden/make_golden.py``); ``tests/test_oracle.py`` checks this module against them.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F


@dataclass
class AsdqeCfg:
    """Ctor kwargs of ``DenoiseRatePredictor`` (ASDQE/ASDQE_model.py:127)."""

    in_channels: int = 3
    dim: int = 16


def _bn(x, sd, p):
    """BatchNorm2d in eval mode: running statistics, eps 1e-5 (ASDQE_model.py:26, 29)."""
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        training=False, eps=1e-5)


def double_conv(x, sd, p):
    """(conv3x3 + bias -> BN -> ReLU) x 2 (ASDQE_model.py:20-34); p ends in '.double_conv'."""
    x = F.conv2d(x, sd[p + ".0.weight"], sd[p + ".0.bias"], padding=1)
    x = torch.relu(_bn(x, sd, p + ".1"))
    x = F.conv2d(x, sd[p + ".3.weight"], sd[p + ".3.bias"], padding=1)
    return torch.relu(_bn(x, sd, p + ".4"))


def down(x, sd, p):
    """MaxPool2d(2) then DoubleConv (ASDQE_model.py:36-46)."""
    return double_conv(F.max_pool2d(x, 2), sd, p + ".maxpool_conv.1.double_conv")


def up(x1, x2, sd, p):
    """Bilinear x2 (align_corners=True), pad to the skip's size, cat [skip, up], DoubleConv
    (ASDQE_model.py:48-68)."""
    x1 = F.interpolate(x1, scale_factor=2, mode="bilinear", align_corners=True)
    dy, dx = x2.shape[2] - x1.shape[2], x2.shape[3] - x1.shape[3]
    x1 = F.pad(x1, [dx // 2, dx - dx // 2, dy // 2, dy - dy // 2])
    return double_conv(torch.cat([x2, x1], dim=1), sd, p + ".conv.double_conv")


def unet(x, sd, p="unet"):
    """UNet.forward (ASDQE_model.py:96-111), bilinear=True."""
    x1 = double_conv(x, sd, p + ".inc.double_conv")
    x2 = down(x1, sd, p + ".down1")
    x3 = down(x2, sd, p + ".down2")
    x4 = down(x3, sd, p + ".down3")
    y = up(x4, x3, sd, p + ".up1")
    y = up(y, x2, sd, p + ".up2")
    y = up(y, x1, sd, p + ".up3")
    return F.conv2d(y, sd[p + ".outc.conv.weight"], sd[p + ".outc.conv.bias"])


def pad_to_multiple(x, multiple=16):
    """Zero pad bottom/right to a multiple (ASDQE_model.py:113-121)."""
    h, w = x.shape[-2:]
    ph, pw = (multiple - h % multiple) % multiple, (multiple - w % multiple) % multiple
    return F.pad(x, (0, pw, 0, ph)) if (ph or pw) else x


def asdqe_features(sd, lq, gt, cfg: AsdqeCfg):
    """DenoiseRatePredictor.forward (ASDQE_model.py:158-171) returning intermediates:
    'merged' [B,3d,H',W'], 'feat' (UNet output) [B,3d,H',W'], 'gap' [B,3d], 'score' [B,1]."""
    lq = pad_to_multiple(lq, cfg.dim)
    gt = pad_to_multiple(gt, cfg.dim)
    merged = torch.cat([double_conv(lq, sd, "lq_extractor.double_conv"),
                        double_conv(gt, sd, "gt_extractor.double_conv"),
                        double_conv(lq - gt, sd, "diff_extractor.double_conv")], dim=1)
    feat = unet(merged, sd)
    # regressor: AdaptiveAvgPool2d(1), Flatten, Linear-ReLU-Dropout x2, Linear, Tanh (:144-154);
    # Dropout is the identity in eval mode
    g = feat.mean(dim=(2, 3))
    h = torch.relu(F.linear(g, sd["regressor.2.weight"], sd["regressor.2.bias"]))
    h = torch.relu(F.linear(h, sd["regressor.5.weight"], sd["regressor.5.bias"]))
    score = torch.tanh(F.linear(h, sd["regressor.8.weight"], sd["regressor.8.bias"]))
    return {"merged": merged, "feat": feat, "gap": g, "score": score}


def asdqe_forward(sd, lq, gt, cfg: AsdqeCfg):
    return asdqe_features(sd, lq, gt, cfg)["score"]


def asdqe_param_shapes(cfg: AsdqeCfg) -> dict:
    """state_dict keys/shapes of DenoiseRatePredictor, registration order (ASDQE_model.py:127-156),
    including the BatchNorm buffers (num_batches_tracked is a 0-d int64)."""
    shapes = {}
    d = cfg.dim

    def dc(p, cin, cout):
        for i, (ci, co) in ((0, (cin, cout)), (3, (cout, cout))):
            shapes[f"{p}.{i}.weight"] = (co, ci, 3, 3)
            shapes[f"{p}.{i}.bias"] = (co,)
            for s in ("weight", "bias", "running_mean", "running_var"):
                shapes[f"{p}.{i + 1}.{s}"] = (co,)
            shapes[f"{p}.{i + 1}.num_batches_tracked"] = ()

    for e in ("lq", "gt", "diff"):
        dc(f"{e}_extractor.double_conv", cfg.in_channels, d)
    m = 3 * d
    dc("unet.inc.double_conv", m, 64)
    dc("unet.down1.maxpool_conv.1.double_conv", 64, 128)
    dc("unet.down2.maxpool_conv.1.double_conv", 128, 256)
    dc("unet.down3.maxpool_conv.1.double_conv", 256, 256)
    dc("unet.up1.conv.double_conv", 512, 128)
    dc("unet.up2.conv.double_conv", 256, 64)
    dc("unet.up3.conv.double_conv", 128, 64)
    shapes["unet.outc.conv.weight"] = (m, 64, 1, 1)
    shapes["unet.outc.conv.bias"] = (m,)
    for i, (ci, co) in ((2, (m, 256)), (5, (256, 64)), (8, (64, 1))):
        shapes[f"regressor.{i}.weight"] = (co, ci)
        shapes[f"regressor.{i}.bias"] = (co,)
    return shapes
