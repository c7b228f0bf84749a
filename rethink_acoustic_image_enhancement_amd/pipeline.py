"""The steps either side of the forward, on the GPU.

* ``enhance_u8`` — KDLAE/KDLAE_T.ipynb's inference cell for a batch of equally sized uint8 images:
  ``load_image_as_tensor`` (u8 -> /255, alpha dropped, optional BGR->RGB), reflect pad to a
  multiple of 8, constant ``denoise_rate`` map, forward, then clamp / crop / ``img_as_ubyte`` and the
  zero-mask of input-black pixels (x2 nearest for ``sr``).  Pre and post are HIP kernels
  (``kdlae_preprocess_u8`` / ``kdlae_postprocess_u8``); images never round-trip through the host.
* ``frames_preprocess_u8`` / ``enhance_frames_u8`` — KDLAE/KDLAE-S.ipynb's cell: F frames (gray or
  cv2 BGR/BGRA u8) -> COLOR_BGR2GRAY -> /255 -> [B,F,H,W] reflect-padded to a multiple of 32 ->
  KDLAE_student -> clamp / crop / permute to [h,w,F] / ``img_as_ubyte``, pre and post on the GPU.
* ``asdqe_scores`` / ``score_statistics`` / ``write_statistics_csv`` — ASDQE/ASDQE_test.py's
  ``infer`` + ``calculate_statistics`` + ``visualize_comparison`` CSV (:87-133).
"""
from __future__ import annotations

import ctypes
import csv

import numpy as np
import torch

from . import _lib


def padded_size(h: int, w: int, multiple: int = 8):
    H, W = ctypes.c_int(), ctypes.c_int()
    _lib.lib().kdlae_padded_size(h, w, multiple, ctypes.byref(H), ctypes.byref(W))
    return H.value, W.value


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def preprocess_u8(images: torch.Tensor, denoise_rate=None, multiple: int = 8, bgr: bool = False):
    """u8 [B,h,w,C] (cuda) -> (img f32 [B,min(C,3),H,W], rate map f32 [B,1,H,W] or None)."""
    if images.device.type != "cuda" or images.dtype != torch.uint8 or images.dim() != 4:
        raise RuntimeError("preprocess_u8 expects a cuda uint8 tensor [B,h,w,C]")
    images = images.contiguous()
    B, h, w, C = images.shape
    H, W = padded_size(h, w, multiple)
    dev = images.device
    img = torch.empty((B, min(C, 3), H, W), device=dev, dtype=torch.float32)
    rate = rmap = None
    if denoise_rate is not None:
        rate = torch.as_tensor(denoise_rate, dtype=torch.float32).to(dev).expand(B).contiguous()
        rmap = torch.empty((B, 1, H, W), device=dev, dtype=torch.float32)
    rc = _lib.lib().kdlae_preprocess_u8(
        ctypes.c_void_p(images.data_ptr()), B, h, w, C, int(bgr), multiple,
        ctypes.c_void_p(rate.data_ptr() if rate is not None else 0), ctypes.c_void_p(img.data_ptr()),
        ctypes.c_void_p(rmap.data_ptr() if rmap is not None else 0), _stream(dev))
    _lib.check(rc, "kdlae_preprocess_u8")
    return img, rmap


def postprocess_u8(out: torch.Tensor, h: int, w: int, scale: int = 1, lq_u8: torch.Tensor | None = None):
    """Model output f32 [B,C,Hs,Ws] -> u8 [B,h*scale,w*scale,C] (clamp, crop, img_as_ubyte, black mask)."""
    out = out.contiguous()
    B, C, Hs, Ws = out.shape
    dst = torch.empty((B, h * scale, w * scale, C), device=out.device, dtype=torch.uint8)
    lq = lq_u8.contiguous() if lq_u8 is not None else None
    rc = _lib.lib().kdlae_postprocess_u8(
        ctypes.c_void_p(out.data_ptr()), B, C, Hs, Ws, h, w, scale,
        ctypes.c_void_p(lq.data_ptr() if lq is not None else 0), lq.shape[-1] if lq is not None else 0,
        ctypes.c_void_p(dst.data_ptr()), _stream(out.device))
    _lib.check(rc, "kdlae_postprocess_u8")
    return dst


def enhance_u8(model, images: torch.Tensor, denoise_rate, bgr: bool = False, multiple: int = 8):
    """KDLAE_T.ipynb inference for u8 images [B,h,w,C] on the model's device -> (hq u8, sr u8 or None)."""
    B, h, w, C = images.shape
    img, rmap = preprocess_u8(images, denoise_rate, multiple, bgr)
    with torch.no_grad():
        pred = model({"img": img, "denoise_rate": rmap})
    hq = postprocess_u8(pred["hq"], h, w, 1, images)
    sr = postprocess_u8(pred["sr"], h, w, 2, images) if pred.get("sr") is not None else None
    return hq, sr


def frames_preprocess_u8(frames: torch.Tensor, multiple: int = 32) -> torch.Tensor:
    """u8 frames (cuda) [B,F,h,w] (gray) or [B,F,h,w,C] (cv2 BGR / BGRA) -> f32 [B,F,H,W]."""
    if frames.device.type != "cuda" or frames.dtype != torch.uint8 or frames.dim() not in (4, 5):
        raise RuntimeError("frames_preprocess_u8 expects a cuda uint8 tensor [B,F,h,w] or [B,F,h,w,C]")
    frames = frames.contiguous()
    B, F, h, w = frames.shape[:4]
    C = frames.shape[4] if frames.dim() == 5 else 1
    H, W = padded_size(h, w, multiple)
    x = torch.empty((B, F, H, W), device=frames.device, dtype=torch.float32)
    rc = _lib.lib().kdlae_frames_preprocess_u8(ctypes.c_void_p(frames.data_ptr()), B, F, h, w, C, multiple,
                                               ctypes.c_void_p(x.data_ptr()), _stream(frames.device))
    _lib.check(rc, "kdlae_frames_preprocess_u8")
    return x


def enhance_frames_u8(model, frames: torch.Tensor, multiple: int = 32) -> torch.Tensor:
    """KDLAE-S.ipynb inference for u8 frame stacks [B,F,h,w(,C)] -> u8 [B,h,w,F] (restored frames)."""
    h, w = frames.shape[2], frames.shape[3]
    x = frames_preprocess_u8(frames, multiple)
    with torch.no_grad():
        y = model(x)
    return postprocess_u8(y, h, w, 1, None)


def to_tensor_u8(images: torch.Tensor) -> torch.Tensor:
    """torchvision ToTensor for u8 [B,h,w,C] RGB on the GPU: f32 [B,C,h,w] / 255 (no padding)."""
    img, _ = preprocess_u8(images, None, multiple=1)
    return img


def asdqe_scores(model, lq_u8: torch.Tensor, gt_u8: torch.Tensor, chunk: int = 64) -> np.ndarray:
    """ASDQE_test.py ``infer`` (:87-104) for equally sized RGB pairs u8 [N,h,w,3] -> float32 scores [N].
    The script scores one pair per forward; every pair is independent (GAP slots depend on the image
    size only), so scoring ``chunk`` pairs per forward gives the same values."""
    out = []
    with torch.no_grad():
        for c0 in range(0, lq_u8.shape[0], chunk):
            s = model(to_tensor_u8(lq_u8[c0:c0 + chunk]), to_tensor_u8(gt_u8[c0:c0 + chunk]))
            out.append(s.float().cpu().numpy().reshape(-1))
    return np.concatenate(out)


def score_statistics(values) -> dict:
    """ASDQE_test.py ``calculate_statistics`` (:107-120), on the float32 predictions as the script
    has them (np.mean / np.std of a float32 array accumulate in float32, pairwise)."""
    v = np.asarray(values)
    return {"mean": float(np.mean(v)), "std": float(np.std(v)), "min": float(np.min(v)),
            "25%": float(np.percentile(v, 25)), "50%": float(np.percentile(v, 50)),
            "75%": float(np.percentile(v, 75)), "max": float(np.max(v))}


def write_statistics_csv(stats_by_method: dict, path: str) -> None:
    """``visualize_comparison``'s transposed CSV (:123-133): rows = statistic, columns = method, %.6f."""
    methods = list(stats_by_method)
    keys = list(next(iter(stats_by_method.values())))
    with open(path, "w", newline="") as f:
        wr = csv.writer(f, lineterminator="\n")  # pandas DataFrame.to_csv line endings
        wr.writerow([""] + methods)
        for k in keys:
            wr.writerow([k] + [f"{stats_by_method[m][k]:.6f}" for m in methods])
