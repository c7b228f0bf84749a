"""Config-1 (MDD sonar crop, 512x512, denoise_rate 0.6) precision analysis on the CPU oracle.

TEST/ANALYSIS INFRASTRUCTURE (imports oracle/): writes profiles/r03_config1_precision.txt.

1. Per stage: max-abs of the oracle's fp32 run against its fp64 run after every stage of
   KDLAE_teacher.forward (KDLAE/KDLAE_model.py:270-336), relative to the stage's max |x|.
2. Per op class: the fp32 forward with one op class promoted to fp64 (LayerNorm, MDTA, GDFN, every
   conv), then MDTA split further: only q.k^T / norms / softmax in fp64, and the HIP path's Gram
   scheme (fp32 partial sums over 1024-pixel slots, slots added in fp64; csrc/mdta.hip).
Errors are max-abs vs the fp64 output over the full maps and over the fixture's [::8, ::8]
subsample (what tests/test_kdlae_gpu.py::test_mdd_512_config1 compares).
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle.kdlae_oracle as O  # noqa: E402
from tests.util import hash_sd_for, load_fixture, mdd_input_tensor  # noqa: E402

ORIG = {n: getattr(O, n) for n in ("layer_norm", "mdta", "gdfn", "conv", "stage")}


def setup():
    d, kw = load_fixture("t_mdd_512")
    cfg = O.TeacherCfg(**kw)
    sd = hash_sd_for(O.teacher_param_shapes(cfg))
    return cfg, sd, {k: v.double() for k, v in sd.items()}, mdd_input_tensor(d), torch.full((1, 1, 512, 512), 0.6)


def restore():
    for n, f in ORIG.items():
        setattr(O, n, f)


def promote(fn, sd64):
    def g(x, sd, *a, **k):
        if x.dtype == torch.float64:
            return fn(x, sd, *a, **k)
        return fn(x.double(), sd64, *a, **k).float()
    return g


def mdta_core64(x, sd, p, heads):
    """MDTA with only the normalised Gram and softmax in fp64."""
    b, c, h, w = x.shape
    qkv = O.conv(O.conv(x, sd, p + ".qkv"), sd, p + ".qkv_dwconv", padding=1, groups=3 * c)
    q, k, v = qkv.chunk(3, dim=1)
    ch = c // heads
    q = q.reshape(b, heads, ch, h * w).double()
    k = k.reshape(b, heads, ch, h * w).double()
    q = q / q.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    k = k / k.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    temp = sd[p + ".temperature"].view(1, heads, 1, 1).double()
    attn = torch.softmax(torch.matmul(q, k.transpose(-2, -1)) * temp, dim=-1).float()
    out = torch.matmul(attn, v.reshape(b, heads, ch, h * w)).reshape(b, c, h, w)
    return O.conv(out, sd, p + ".project_out")


def mdta_slots(x, sd, p, heads, blk=1024):
    """fp32 everywhere; Gram and squared norms as fp32 sums over `blk`-pixel slots, slots added in
    fp64 (the HIP path's dwconv_gram + gram_reduce scheme)."""
    b, c, h, w = x.shape
    qkv = O.conv(O.conv(x, sd, p + ".qkv"), sd, p + ".qkv_dwconv", padding=1, groups=3 * c)
    q, k, v = qkv.chunk(3, dim=1)
    ch, n = c // heads, h * w
    nb = max(1, n // blk)
    qb = q.reshape(b, heads, ch, nb, n // nb).permute(0, 1, 3, 2, 4)
    kb = k.reshape(b, heads, ch, nb, n // nb).permute(0, 1, 3, 2, 4)
    G = torch.matmul(qb, kb.transpose(-2, -1)).double().sum(2)
    nq = (qb * qb).sum(-1).double().sum(2).sqrt().clamp_min(1e-12)
    nk = (kb * kb).sum(-1).double().sum(2).sqrt().clamp_min(1e-12)
    S = (G / (nq[..., :, None] * nk[..., None, :])).float() * sd[p + ".temperature"].view(1, heads, 1, 1)
    out = torch.matmul(torch.softmax(S, dim=-1), v.reshape(b, heads, ch, n)).reshape(b, c, h, w)
    return O.conv(out, sd, p + ".project_out")


def forward(cfg, sd, img, rate, rec=None):
    if rec is not None:
        def stage(x, sd_, name, n, heads, lt):
            y = ORIG["stage"](x, sd_, name, n, heads, lt)
            rec[name] = y.double()
            return y
        O.stage = stage
    with torch.no_grad():
        out = O.teacher_forward(sd, img, rate, cfg)
    O.stage = ORIG["stage"]
    return {k: v.double() for k, v in out.items()}


def errs(out, ref):
    r = {}
    for k in ("hq", "sr"):
        r[k] = float((out[k] - ref[k]).abs().max())
        r[k + "_sub"] = float((out[k][:, :, ::8, ::8] - ref[k][:, :, ::8, ::8]).abs().max())
    return r


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    cfg, sd32, sd64, img, rate = setup()
    lines = [__doc__.strip(), ""]
    rec64, rec32 = {}, {}
    t = time.time()
    ref = forward(cfg, sd64, img.double(), rate.double(), rec64)
    lines.append(f"fp64 forward {time.time() - t:.0f} s")
    base = forward(cfg, sd32, img, rate, rec32)
    lines += ["", "1. per stage: oracle fp32 vs fp64 (max-abs, and relative to max|x| of the stage output)",
              f"{'stage':<18}{'max|x|':>12}{'max-abs':>12}{'relative':>12}"]
    for name, y64 in rec64.items():
        m, e = float(y64.abs().max()), float((rec32[name] - y64).abs().max())
        lines.append(f"{name:<18}{m:>12.4g}{e:>12.3e}{e / max(m, 1e-30):>12.3e}")
    for k in ("hq", "sr"):
        m, e = float(ref[k].abs().max()), float((base[k] - ref[k]).abs().max())
        lines.append(f"{k:<18}{m:>12.4g}{e:>12.3e}{e / m:>12.3e}")
    lines += ["", "2. fp32 forward with one op class in fp64 (or the named MDTA variant): max-abs vs the fp64 output",
              f"{'variant':<34}{'hq':>11}{'sr':>11}{'hq[::8]':>11}{'sr[::8]':>11}"]

    def row(name, e):
        lines.append(f"{name:<34}{e['hq']:>11.3e}{e['sr']:>11.3e}{e['hq_sub']:>11.3e}{e['sr_sub']:>11.3e}")

    row("all fp32 (= the reference fp32)", errs(base, ref))
    for cls in ("layer_norm", "mdta", "gdfn", "conv"):
        restore()
        setattr(O, cls, promote(ORIG[cls], sd64))
        row(f"{cls} in fp64", errs(forward(cfg, sd32, img, rate), ref))
    for name, fn in (("mdta: Gram/norm/softmax in fp64", mdta_core64),
                     ("mdta: HIP slot scheme (f32 1024-px", mdta_slots)):
        restore()
        O.mdta = fn
        row(name if "slot" not in name else name + ")", errs(forward(cfg, sd32, img, rate), ref))
    restore()
    text = "\n".join(lines) + "\n"
    print(text)
    out = os.path.join(ROOT, "profiles", "r03_config1_precision.txt")
    with open(out, "w") as f:
        f.write(text)
    print(json.dumps({"written": out}))


if __name__ == "__main__":
    main()
