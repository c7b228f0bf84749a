"""TEST INFRASTRUCTURE ONLY — CPU oracle for the KDLAE-T / KDLAE-S forward.

This module is a from-scratch *functional* restatement (torch CPU ops on a plain state_dict)
of the reference math in ``KDLAE/KDLAE_model.py``.  It is the checker that the HIP path is
compared against; nothing in ``rethink_acoustic_image_enhancement_amd`` imports it, and only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may call it.

Pinning: ``tests/golden/`` holds outputs of the *imported reference* (generated in the build
container by ``tests/golden/make_golden.py`` with the §8c hash weights); the CPU test suite
checks this oracle against every one of them (``tests/test_oracle.py``).

Every function cites the reference line it restates.  All tensors are NCHW.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F


@dataclass
class TeacherCfg:
    """Ctor kwargs of ``KDLAE_teacher`` (KDLAE/KDLAE_model.py:205-218)."""

    inp_channels: int = 3
    out_channels: int = 3
    dim: int = 48
    num_blocks: list = field(default_factory=lambda: [4, 6, 6, 8])
    num_refinement_blocks: int = 4
    heads: list = field(default_factory=lambda: [1, 2, 4, 8])
    ffn_expansion_factor: float = 2.66
    bias: bool = False
    LayerNorm_type: str = "WithBias"
    dual_pixel_task: bool = False
    static: str = "train"
    params: str = "cat"


def _w(sd, name):
    return sd[name]


def _opt(sd, name):
    return sd.get(name)


def layer_norm(x, sd, prefix, ln_type):
    """BiasFree / WithBias LayerNorm over channels (KDLAE_model.py:50-52, 67-70, 81-83)."""
    w = _w(sd, prefix + ".body.weight").view(1, -1, 1, 1)
    var = x.var(dim=1, keepdim=True, unbiased=False)
    if ln_type == "BiasFree":
        return x / torch.sqrt(var + 1e-5) * w
    mu = x.mean(dim=1, keepdim=True)
    b = _w(sd, prefix + ".body.bias").view(1, -1, 1, 1)
    return (x - mu) / torch.sqrt(var + 1e-5) * w + b


def conv(x, sd, prefix, padding=0, dilation=1, groups=1):
    return F.conv2d(x, _w(sd, prefix + ".weight"), _opt(sd, prefix + ".bias"),
                    padding=padding, dilation=dilation, groups=groups)


def mdta(x, sd, p, heads):
    """Multi-Dconv head transposed attention (KDLAE_model.py:124-145)."""
    b, c, h, w = x.shape
    qkv = conv(x, sd, p + ".qkv")
    qkv = conv(qkv, sd, p + ".qkv_dwconv", padding=1, groups=3 * c)
    q, k, v = qkv.chunk(3, dim=1)
    ch = c // heads
    q = q.reshape(b, heads, ch, h * w)
    k = k.reshape(b, heads, ch, h * w)
    v = v.reshape(b, heads, ch, h * w)
    # F.normalize: x / max(||x||_2, 1e-12) along HW
    q = q / q.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    k = k / k.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    temp = _w(sd, p + ".temperature").view(1, heads, 1, 1)
    attn = torch.softmax(torch.matmul(q, k.transpose(-2, -1)) * temp, dim=-1)
    out = torch.matmul(attn, v).reshape(b, c, h, w)
    return conv(out, sd, p + ".project_out")


def gdfn(x, sd, p):
    """Gated-Dconv feed-forward (KDLAE_model.py:101-106), exact-erf GELU."""
    y = conv(x, sd, p + ".project_in")
    y = conv(y, sd, p + ".dwconv", padding=1, groups=y.shape[1])
    y1, y2 = y.chunk(2, dim=1)
    return conv(F.gelu(y1) * y2, sd, p + ".project_out")


def transformer_block(x, sd, p, heads, ln_type):
    """x += attn(norm1 x); x += ffn(norm2 x)  (KDLAE_model.py:159-163)."""
    x = x + mdta(layer_norm(x, sd, p + ".norm1", ln_type), sd, p + ".attn", heads)
    x = x + gdfn(layer_norm(x, sd, p + ".norm2", ln_type), sd, p + ".ffn")
    return x


def stage(x, sd, name, n, heads, ln_type):
    for i in range(n):
        x = transformer_block(x, sd, f"{name}.{i}", heads, ln_type)
    return x


def down(x, sd, p):
    """3x3 conv C->C/2 then PixelUnshuffle(2) (KDLAE_model.py:186-187)."""
    return F.pixel_unshuffle(conv(x, sd, p + ".body.0", padding=1), 2)


def up(x, sd, p):
    """3x3 conv C->2C then PixelShuffle(2) (KDLAE_model.py:196-197)."""
    return F.pixel_shuffle(conv(x, sd, p + ".body.0", padding=1), 2)


def teacher_forward(sd, img, denoise_rate, cfg: TeacherCfg):
    """KDLAE_teacher.forward (KDLAE_model.py:270-336). Returns {'hq', 'sr'}."""
    if cfg.dual_pixel_task:
        raise NotImplementedError("dual_pixel_task=True is broken in the reference (:305-321)")
    H, W = img.shape[-2:]
    if H % 8 or W % 8:
        raise RuntimeError("KDLAE_teacher needs H and W divisible by 8 (pixel_unshuffle x3)")
    nb, hd, lt = cfg.num_blocks, cfg.heads, cfg.LayerNorm_type
    e1 = stage(conv(img, sd, "patch_embed.proj", padding=1), sd, "encoder_level1", nb[0], hd[0], lt)
    e2 = stage(down(e1, sd, "down1_2"), sd, "encoder_level2", nb[1], hd[1], lt)
    e3 = stage(down(e2, sd, "down2_3"), sd, "encoder_level3", nb[2], hd[2], lt)
    lat = stage(down(e3, sd, "down3_4"), sd, "latent", nb[3], hd[3], lt)
    d3 = conv(torch.cat([up(lat, sd, "up4_3"), e3], 1), sd, "reduce_chan_level3")
    d3 = stage(d3, sd, "decoder_level3", nb[2], hd[2], lt)
    d2 = conv(torch.cat([up(d3, sd, "up3_2"), e2], 1), sd, "reduce_chan_level2")
    d2 = stage(d2, sd, "decoder_level2", nb[1], hd[1], lt)
    d1 = stage(torch.cat([up(d2, sd, "up2_1"), e1], 1), sd, "decoder_level1", nb[0], hd[0], lt)
    d1 = stage(d1, sd, "refinement", cfg.num_refinement_blocks, hd[0], lt)
    o = conv(d1, sd, "output", padding=1)
    if cfg.params == "cat":
        o = conv(torch.cat([o, denoise_rate], 1), sd, "output_param", padding=2, dilation=2)
        o = stage(o, sd, "refinement_out", cfg.num_refinement_blocks, hd[0], lt)
        o = conv(o, sd, "output2", padding=1)
    hq = o + img
    sr = None
    if cfg.static == "train":
        s = up(conv(hq, sd, "cen", padding=1), sd, "upen")
        s = stage(s, sd, "enhance", cfg.num_refinement_blocks, hd[0], lt)
        sr = conv(s, sd, "outputen", padding=1)
    return {"hq": hq, "sr": sr}


def teacher_param_shapes(cfg: TeacherCfg) -> dict:
    """state_dict key -> shape for a KDLAE_teacher config (KDLAE_model.py:220-268)."""
    shapes = {}
    bias = cfg.bias

    def c(name, cout, cin, k, b=bias):
        shapes[name + ".weight"] = (cout, cin, k, k)
        if b:
            shapes[name + ".bias"] = (cout,)

    def block(p, dim, heads):
        hid = int(dim * cfg.ffn_expansion_factor)
        for n in ("norm1", "norm2"):
            shapes[f"{p}.{n}.body.weight"] = (dim,)
            if cfg.LayerNorm_type != "BiasFree":
                shapes[f"{p}.{n}.body.bias"] = (dim,)
        shapes[f"{p}.attn.temperature"] = (heads, 1, 1)
        c(f"{p}.attn.qkv", 3 * dim, dim, 1)
        c(f"{p}.attn.qkv_dwconv", 3 * dim, 1, 3)
        c(f"{p}.attn.project_out", dim, dim, 1)
        c(f"{p}.ffn.project_in", 2 * hid, dim, 1)
        c(f"{p}.ffn.dwconv", 2 * hid, 1, 3)
        c(f"{p}.ffn.project_out", dim, hid, 1)

    def stg(name, n, dim, heads):
        for i in range(n):
            block(f"{name}.{i}", dim, heads)

    d, nb, hd = cfg.dim, cfg.num_blocks, cfg.heads
    c("patch_embed.proj", d, cfg.inp_channels, 3, b=False)
    stg("encoder_level1", nb[0], d, hd[0])
    c("down1_2.body.0", d // 2, d, 3, b=False)
    stg("encoder_level2", nb[1], 2 * d, hd[1])
    c("down2_3.body.0", d, 2 * d, 3, b=False)
    stg("encoder_level3", nb[2], 4 * d, hd[2])
    c("down3_4.body.0", 2 * d, 4 * d, 3, b=False)
    stg("latent", nb[3], 8 * d, hd[3])
    c("up4_3.body.0", 16 * d, 8 * d, 3, b=False)
    c("reduce_chan_level3", 4 * d, 8 * d, 1)
    stg("decoder_level3", nb[2], 4 * d, hd[2])
    c("up3_2.body.0", 8 * d, 4 * d, 3, b=False)
    c("reduce_chan_level2", 2 * d, 4 * d, 1)
    stg("decoder_level2", nb[1], 2 * d, hd[1])
    c("up2_1.body.0", 4 * d, 2 * d, 3, b=False)
    stg("decoder_level1", nb[0], 2 * d, hd[0])
    stg("refinement", cfg.num_refinement_blocks, 2 * d, hd[0])
    c("output", cfg.out_channels, 2 * d, 3)
    c("output_param", 2 * d, cfg.out_channels + 1, 3)
    stg("refinement_out", cfg.num_refinement_blocks, 2 * d, hd[0])
    c("output2", cfg.out_channels, 2 * d, 3)
    if cfg.static == "train":
        hc = 2 * d
        c("cen", hc, cfg.out_channels, 3)
        c("upen.body.0", 2 * hc, hc, 3, b=False)
        stg("enhance", cfg.num_refinement_blocks, hc // 2, hd[0])
        c("outputen", cfg.out_channels, hc // 2, 3)
    return shapes


# ----------------------------------------------------------------------------- KDLAE-S
@dataclass
class StudentCfg:
    """Ctor kwargs of ``KDLAE_student`` (KDLAE/KDLAE_model.py:341-342)."""

    inp_channels: int = 1
    out_channels: int = 1
    residual: bool = False
    hidden_channels: list = field(default_factory=lambda: [16, 32, 64])
    kernel_size: int = 3


def _conv3d(x, sd, p, padding):
    return F.conv3d(x, sd[p + ".weight"], sd.get(p + ".bias"), padding=padding)


def _block3d(x, sd, p, pad):
    """Conv3d-ReLU-Conv3d-ReLU (KDLAE_model.py:386-393)."""
    x = torch.relu(_conv3d(x, sd, p + ".0", pad))
    return torch.relu(_conv3d(x, sd, p + ".2", pad))


def student_forward(sd, x, cfg: StudentCfg):
    """KDLAE_student.forward (KDLAE_model.py:395-431): [B,F,H,W] -> [B,F,H,W]."""
    pad = cfg.kernel_size // 2
    levels = len(cfg.hidden_channels) - 1
    x = x.unsqueeze(1)
    cur, skips = x, []
    for i in range(levels):
        e = _block3d(cur, sd, f"encoders.{i}", pad)
        skips.append(e)
        cur = F.max_pool3d(e, kernel_size=(1, 2, 2))
    cur = _block3d(cur, sd, "st_fusion", pad)
    for i in range(levels):
        cur = F.conv_transpose3d(cur, sd[f"upconv_layers.{i}.weight"],
                                 sd.get(f"upconv_layers.{i}.bias"), stride=(1, 2, 2))
        cur = cur + skips[levels - 1 - i]
        cur = _block3d(cur, sd, f"decoders.{i}", pad)
    out = _conv3d(cur, sd, "out_conv", 0)
    if cfg.residual:
        out = out + x
    return out.squeeze(1)


def student_param_shapes(cfg: StudentCfg) -> dict:
    shapes = {}
    k = cfg.kernel_size
    hc = cfg.hidden_channels
    levels = len(hc) - 1

    def blk(p, cin, cout):
        shapes[p + ".0.weight"] = (cout, cin, k, k, k)
        shapes[p + ".0.bias"] = (cout,)
        shapes[p + ".2.weight"] = (cout, cout, k, k, k)
        shapes[p + ".2.bias"] = (cout,)

    cin = cfg.inp_channels
    for i in range(levels):
        blk(f"encoders.{i}", cin, hc[i])
        cin = hc[i]
    blk("st_fusion", cin, hc[-1])
    for j, i in enumerate(range(levels - 1, -1, -1)):
        cu_in = hc[-1] if i == levels - 1 else hc[i + 1]
        shapes[f"upconv_layers.{j}.weight"] = (cu_in, hc[i], 1, 2, 2)
        shapes[f"upconv_layers.{j}.bias"] = (hc[i],)
        blk(f"decoders.{j}", hc[i], hc[i])
    shapes["out_conv.weight"] = (cfg.out_channels, hc[0], 1, 1, 1)
    shapes["out_conv.bias"] = (cfg.out_channels,)
    return shapes


def psnr(a, b):
    """10 log10(1/MSE) over clamp(.,0,1), float64 (psnr_ssim.py:55-70)."""
    a = a.double().clamp(0, 1)
    b = b.double().clamp(0, 1)
    mse = torch.mean((a - b) ** 2).item()
    return float("inf") if mse == 0 else 10.0 * math.log10(1.0 / mse)
