"""TEST INFRASTRUCTURE ONLY — CPU oracle for the steps either side of the forward.

Restates, on numpy/torch CPU tensors, the inference cell of KDLAE/KDLAE_T.ipynb (code cells:
``load_image_as_tensor``; the padding block ``H,W = ((h+m)//m)*m ...; F.pad(..., 'reflect')``;
``alpha = ones * denoise_rate``; ``clamp`` / crop / ``img_as_ubyte`` / the black-pixel mask and its
``np.repeat`` x2 for sr) and ASDQE_test.py's ToTensor + ``calculate_statistics`` (:107-120).

KDLAE/KDLAE-S.ipynb's ``load_consecutive_stack`` (cv2.imread -> COLOR_BGR2GRAY -> /255 -> stack) and its
padding / output cell (pad to a multiple of 32; clamp, crop, permute to [h, w, F], img_as_ubyte) are
restated too.  cv2 is not importable here either: ``bgr2gray_u8`` restates OpenCV's published 8-bit
fixed-point rule (yuv_shift 14, B2Y 1868 / G2Y 9617 / R2Y 4899), so it is "parity unpinned" by the
reference as well — except on gray-as-RGB frames (the MDD samples), where it is the identity.

``img_as_ubyte`` is scikit-image (not importable in this image; the reference pins no version):
restated from its published float->uint8 conversion, ``rint(x * 255)`` in float32 then clip.
That rounding rule is therefore "parity unpinned" by the reference; everything else follows the
notebook line for line.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def load_image_as_tensor(img_u8: np.ndarray, bgr: bool = False) -> torch.Tensor:
    """cv2 image (HWC u8) -> [1,C,h,w] float32 /255 (alpha dropped, BGR->RGB when bgr)."""
    img = img_u8
    if img.ndim == 2:
        img = img[:, :, None]
    if img.shape[2] == 4:
        img = img[:, :, :3]
    if img.shape[2] == 3 and bgr:
        img = img[:, :, ::-1]
    img = img.astype(np.float32) / 255.0
    return torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1).unsqueeze(0)


def notebook_pad(x: torch.Tensor, m: int = 8) -> torch.Tensor:
    h, w = x.shape[2], x.shape[3]
    H, W = ((h + m) // m) * m, ((w + m) // m) * m
    padh = H - h if h % m != 0 else 0
    padw = W - w if w % m != 0 else 0
    return F.pad(x, (0, padw, 0, padh), "reflect")


def img_as_ubyte(x: np.ndarray) -> np.ndarray:
    y = np.multiply(x.astype(np.float32), np.float32(255.0), dtype=np.float32)
    np.rint(y, out=y)
    return np.clip(y, 0, 255).astype(np.uint8)


def black_mask(lq_u8: np.ndarray) -> np.ndarray:
    """``(lq[...,0]==0)&(lq[...,1]==0)&(lq[...,2]==0)`` for 3 channels, ``lq.squeeze()==0`` for 1."""
    lq = lq_u8 if lq_u8.ndim == 3 else lq_u8[:, :, None]
    if lq.shape[2] == 4:
        lq = lq[:, :, :3]
    return np.all(lq == 0, axis=2)


def postprocess(pred: torch.Tensor, h: int, w: int, lq_u8: np.ndarray | None, scale: int = 1) -> np.ndarray:
    """[1,C,H,W] model output -> HWC u8 (clamp, crop, img_as_ubyte, zero-mask)."""
    r = torch.clamp(pred, 0, 1)[:, :, : h * scale, : w * scale]
    out = img_as_ubyte(r.permute(0, 2, 3, 1).numpy()[0])
    if lq_u8 is not None:
        m = black_mask(lq_u8)
        if scale == 2:
            m = np.repeat(np.repeat(m, 2, axis=0), 2, axis=1)
        out[m] = 0
    return out


def calculate_statistics(values) -> dict:
    v = np.asarray(values)
    return {"mean": np.mean(v), "std": np.std(v), "min": np.min(v), "25%": np.percentile(v, 25),
            "50%": np.percentile(v, 50), "75%": np.percentile(v, 75), "max": np.max(v)}


def bgr2gray_u8(img_u8: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(img, COLOR_BGR2GRAY) for 8-bit BGR / BGRA (alpha ignored)."""
    b, g, r = (img_u8[..., i].astype(np.uint32) for i in range(3))
    return ((1868 * b + 9617 * g + 4899 * r + 8192) >> 14).astype(np.uint8)


def load_consecutive_stack(frames_u8) -> torch.Tensor:
    """KDLAE-S.ipynb load_consecutive_stack for already-read equally sized frames (cv2.imread
    IMREAD_UNCHANGED arrays, in sequence order): gray, /255, stacked -> [1, F, h, w]."""
    out = []
    for img in frames_u8:
        if img.ndim == 3:
            img = bgr2gray_u8(img) if img.shape[2] >= 3 else img[:, :, 0]
        out.append(img.astype(np.float32) / 255.0)
    return torch.from_numpy(np.stack(out, axis=0)).unsqueeze(0)


def student_postprocess(restored: torch.Tensor, h: int, w: int) -> np.ndarray:
    """KDLAE-S.ipynb output cell: clamp, crop, permute(0, 2, 3, 1), img_as_ubyte(restored[0]) -> [h, w, F]."""
    r = torch.clamp(restored, 0, 1)[:, :, :h, :w]
    return img_as_ubyte(r.permute(0, 2, 3, 1).numpy()[0])
