"""Drop-in ASDQE module whose forward runs on the MI355X HIP path (libkdlae.so, ``asdqe_*``).

Same public surface as ``ASDQE/ASDQE_model.py`` in the reference:
  * ``DenoiseRatePredictor(in_channels=3, dim=16)`` (:127) with an identical submodule tree, so the
    raw ``ASDQE.pth`` state_dict (148 keys incl. BatchNorm buffers, ``strict=False`` load at
    ASDQE_test.py:79) loads unchanged;
  * ``forward(lq, gt) -> score [B, 1]`` in ``[-1, 1]`` (:158-171), any H x W (zero-padded to a
    multiple of ``dim`` as ``pad_to_multiple`` does, :113-121).

Inference only, eval mode: BatchNorm uses running statistics (folded into the conv weights when the
weights are committed) and Dropout is the identity.  A module left in training mode raises, since the
reference would then use batch statistics and random dropout masks.  There is no CPU path.
"""
from __future__ import annotations

import ctypes
import warnings

import torch
import torch.nn as nn

from . import _lib
from .KDLAE_model import _Engine


class DoubleConv(nn.Module):
    """(conv3x3 + bias, BatchNorm2d, ReLU) x 2 (ASDQE_model.py:20-34) — parameter holder."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        c = out_channels
        self.double_conv = nn.Sequential(nn.Conv2d(in_channels, c, 3, padding=1), nn.BatchNorm2d(c), nn.ReLU(True),
                                         nn.Conv2d(c, c, 3, padding=1), nn.BatchNorm2d(c), nn.ReLU(True))


class Down(nn.Module):
    """MaxPool2d(2) + DoubleConv (ASDQE_model.py:36-46)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.maxpool_conv = nn.Sequential(nn.MaxPool2d(2), DoubleConv(in_channels, out_channels))


class Up(nn.Module):
    """Bilinear x2 (align_corners=True) + cat [skip, up] + DoubleConv (ASDQE_model.py:48-68)."""

    def __init__(self, in_channels, out_channels, bilinear=True):
        super().__init__()
        if not bilinear:
            raise NotImplementedError("ASDQE UNet is only instantiated with bilinear=True (ASDQE_model.py:81)")
        self.up = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
        self.conv = DoubleConv(in_channels, out_channels)


class OutConv(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size=1)


class UNet(nn.Module):
    """UNet(inp, out, bilinear=True) (ASDQE_model.py:78-94): 64-128-256-256 channels."""

    def __init__(self, inp_channels, out_channels, bilinear=True):
        super().__init__()
        self.n_channels = inp_channels
        self.out_channels = out_channels
        self.bilinear = bilinear
        self.inc = DoubleConv(inp_channels, 64)
        self.down1 = Down(64, 128)
        self.down2 = Down(128, 256)
        self.down3 = Down(256, 256)
        self.up1 = Up(512, 128, bilinear)
        self.up2 = Up(256, 64, bilinear)
        self.up3 = Up(128, 64, bilinear)
        self.outc = OutConv(64, out_channels)


class DenoiseRatePredictor(nn.Module):
    """ASDQE (ASDQE/ASDQE_model.py:123-171) with the forward on the MI355X HIP path."""

    def __init__(self, in_channels: int = 3, dim: int = 16) -> None:
        super().__init__()
        self.unet_multiple = dim
        self._cfg = dict(in_channels=in_channels, dim=dim)
        self.lq_extractor = DoubleConv(in_channels, dim)
        self.gt_extractor = DoubleConv(in_channels, dim)
        self.diff_extractor = DoubleConv(in_channels, dim)
        self.unet = UNet(inp_channels=3 * dim, out_channels=3 * dim)
        self.regressor = nn.Sequential(nn.AdaptiveAvgPool2d((1, 1)), nn.Flatten(), nn.Linear(3 * dim, 256),
                                       nn.ReLU(True), nn.Dropout(0.5), nn.Linear(256, 64), nn.ReLU(True),
                                       nn.Dropout(0.3), nn.Linear(64, 1), nn.Tanh())
        self.regressor[-2].bias.data.fill_(0.0)
        self._engines = {}
        self._warned_grad = False

    def _c_config(self) -> _lib.AConfig:
        cfg = _lib.AConfig()
        cfg.in_channels, cfg.dim = self._cfg["in_channels"], self._cfg["dim"]
        return cfg

    def engine(self, device: torch.device) -> _Engine:
        idx = device.index if device.index is not None else torch.cuda.current_device()
        eng = self._engines.get(idx)
        if eng is None:
            eng = _Engine(self._c_config(), idx, "asdqe")
            self._engines[idx] = eng
        return eng

    def forward(self, lq: torch.Tensor, gt: torch.Tensor, return_features: bool = False):
        """score [B, 1]; with ``return_features=True`` also the UNet output map [B, 3*dim, H', W']."""
        if self.training:
            raise RuntimeError("DenoiseRatePredictor (MI355X build) is inference-only: call .eval() first "
                               "(BatchNorm running statistics, Dropout off)")
        if lq.device.type != "cuda" or gt.device != lq.device:
            raise RuntimeError("DenoiseRatePredictor (MI355X build) runs on ROCm devices only; there is no CPU "
                               "fallback")
        ci = self._cfg["in_channels"]
        if lq.dim() != 4 or lq.shape[1] != ci or lq.shape != gt.shape:
            raise RuntimeError(f"expected lq, gt [B,{ci},H,W] of equal shape, got {tuple(lq.shape)}, {tuple(gt.shape)}")
        if torch.is_grad_enabled() and (lq.requires_grad or any(p.requires_grad for p in self.parameters())):
            if not self._warned_grad:
                warnings.warn("DenoiseRatePredictor HIP forward is inference-only: outputs carry no autograd graph")
                self._warned_grad = True
        B, _, H, W = lq.shape
        dev = lq.device
        stream = torch.cuda.current_stream(dev).cuda_stream
        eng = self.engine(dev)
        eng.sync_params(self, stream)
        lq_c = lq.detach().to(torch.float32).contiguous()
        gt_c = gt.detach().to(torch.float32).contiguous()
        score = torch.empty((B, 1), device=dev, dtype=torch.float32)
        d = self._cfg["dim"]
        Hp, Wp = -(-H // d) * d, -(-W // d) * d
        feat = torch.empty((B, Hp, Wp, 3 * d), device=dev, dtype=torch.float32) if return_features else None
        L = _lib.lib()
        nbytes = L.asdqe_workspace_bytes(eng.handle, B, H, W)
        if nbytes < 0:
            _lib.check(1, "asdqe_workspace_bytes")
        ws = eng.workspace(nbytes, dev)
        rc = L.asdqe_forward(eng.handle, ctypes.c_void_p(lq_c.data_ptr()), ctypes.c_void_p(gt_c.data_ptr()), B, H, W,
                             ctypes.c_void_p(score.data_ptr()),
                             ctypes.c_void_p(feat.data_ptr() if feat is not None else 0),
                             ctypes.c_void_p(ws.data_ptr()), ws.numel(), ctypes.c_void_p(stream))
        _lib.check(rc, "asdqe_forward")
        if return_features:
            return score, feat.permute(0, 3, 1, 2)
        return score


def pad_to_multiple(x: torch.Tensor, multiple: int = 16) -> torch.Tensor:
    """Zero pad bottom/right of a [B,C,H,W] tensor to a multiple (ASDQE_model.py:113-121)."""
    h, w = x.shape[-2:]
    ph, pw = (multiple - h % multiple) % multiple, (multiple - w % multiple) % multiple
    return torch.nn.functional.pad(x, (0, pw, 0, ph)) if (ph or pw) else x
