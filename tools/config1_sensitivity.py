"""Config-1 (MDD sonar crop 512x512): where the fp32-vs-fp64 error of KDLAE-T comes from.

ANALYSIS INFRASTRUCTURE (imports oracle/; the fp64 reference and the fp32 baselines come from
tools/config1_taps.py's cached oracle runs, gpurun_out/c1/oracle_cache.pt, recomputed if absent).

Baseline "slots32": the reference's fp32 forward with the HIP path's Gram scheme (fp32 sums over
1024-pixel slots, summed in fp64) — the best fp32 model of r03's analysis (3.4e-4 on hq[::8]).  Each
variant changes ONE thing in it and reports the error vs fp64 at a few taps and at the outputs:
  * ln_noise_*   every LayerNorm output times (1 + u 2^-24), u ~ U[-1, 1] per element (or per pixel):
                 a random half-ulp-scale perturbation, the control
  * deep_* / shallow_*   the same noise only in encoder_level3 / latent / decoder_level3, or only in
                 the other (full- and double-resolution) stages
  * ln_rcp       LN statistics in float64 but x * (1 / sqrt(var + eps)) instead of x / sqrt(var + eps)
  * gelu_as      GELU with the Abramowitz-Stegun 7.1.26 erf (|err| <= 1.5e-7)
A change whose error is no larger than the control's spread is not a defect: it is the input's
conditioning.  Writes profiles/<name>.txt.
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import config1_taps as T  # noqa: E402
import oracle.kdlae_oracle as O  # noqa: E402
from config1_precision import mdta_slots  # noqa: E402
from tests.util import hash_sd_for  # noqa: E402

ORIG_LN = O.layer_norm
DEEP = ("encoder_level3", "latent", "decoder_level3")


def ln_noise(mode, seed, where=None):
    g = torch.Generator().manual_seed(seed)

    def ln(x, sd, prefix, lt):
        y = ORIG_LN(x, sd, prefix, lt)
        if where is not None and prefix.startswith(DEEP) != (where == "deep"):
            return y
        shape = y.shape if mode == "elem" else (y.shape[0], 1, y.shape[2], y.shape[3])
        return y * (1 + (torch.rand(shape, generator=g) * 2 - 1) * 2.0 ** -24)
    return ln


def ln_rcp(x, sd, prefix, lt):
    x64 = x.double()
    mu64 = x64.mean(1, keepdim=True)
    var = ((x64 - mu64) ** 2).mean(1, keepdim=True).float()
    base = x if lt == "BiasFree" else x - mu64.float()
    y = base * (1.0 / torch.sqrt(var + 1e-5)) * sd[prefix + ".body.weight"].view(1, -1, 1, 1)
    if lt != "BiasFree":
        y = y + sd[prefix + ".body.bias"].view(1, -1, 1, 1)
    return y


def gelu_as(x):
    z = x.abs() * 0.70710678118654752
    t = 1.0 / (1.0 + 0.3275911 * z)
    poly = ((((1.061405429 * t - 1.453152027) * t + 1.421413741) * t - 0.284496736) * t + 0.254829592) * t
    return 0.5 * x * (1.0 + torch.copysign(1.0 - poly * torch.exp(-z * z), x))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", default="r04_config1_sensitivity")
    ap.add_argument("--cache", default=os.path.join(ROOT, "gpurun_out", "c1", "oracle_cache.pt"))
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    kw, img, rate = T.setup()
    cfg = O.TeacherCfg(**kw)
    sd32 = hash_sd_for(O.teacher_param_shapes(cfg))
    if os.path.exists(args.cache):
        c = torch.load(args.cache, weights_only=True)
        r64, base = c["r64"], c["slots32"]
    else:
        r64 = T.oracle_run(cfg, {k: v.double() for k, v in sd32.items()}, img.double(), rate.double())
        base = T.oracle_run(cfg, sd32, img, rate, mdta=mdta_slots)

    def run(ln=None, gelu=None):
        orig = (O.layer_norm, O.gdfn)
        if ln is not None:
            O.layer_norm = ln
        if gelu is not None:
            def gdfn(x, sd, p):
                y = O.conv(x, sd, p + ".project_in")
                y = O.conv(y, sd, p + ".dwconv", padding=1, groups=y.shape[1])
                y1, y2 = y.chunk(2, dim=1)
                return O.conv(gelu(y1) * y2, sd, p + ".project_out")
            O.gdfn = gdfn
        try:
            return T.oracle_run(cfg, sd32, img, rate, mdta=mdta_slots)
        finally:
            O.layer_norm, O.gdfn = orig

    cols = {"slots32": base}
    variants = [("noise_e0", dict(ln=ln_noise("elem", 0))), ("noise_e1", dict(ln=ln_noise("elem", 1))),
                ("noise_p0", dict(ln=ln_noise("pix", 0))), ("deep_e0", dict(ln=ln_noise("elem", 0, "deep"))),
                ("shallow_e0", dict(ln=ln_noise("elem", 0, "shallow"))), ("ln_rcp", dict(ln=ln_rcp)),
                ("gelu_as", dict(gelu=gelu_as))]
    for name, kw2 in variants:
        cols[name] = run(**kw2)
        print("done", name, flush=True)
    keys = ["encoder_level2.5", "encoder_level3.5", "latent.7", "decoder_level3.in", "decoder_level3.0",
            "decoder_level2.5", "refinement_out.3", "enhance.3"]
    lines = [__doc__.strip(), "", "relative max-abs error vs fp64 at taps (as tools/config1_taps.py); hq / sr: "
             "absolute max-abs over [::8, ::8]", "",
             f"{'tap':<20}" + "".join(f"{k:>12}" for k in cols)]
    for k in keys:
        ref = r64[k]
        m = float(ref.abs().max())
        lines.append(f"{k:<20}" + "".join(f"{float((cols[c][k] - ref).abs().max()) / m:>12.3e}" for c in cols))
    for k in ("hq", "sr"):
        lines.append(f"{k + '[::8]':<20}" + "".join(
            f"{float((cols[c][k][:, ::4, ::4] - r64[k][:, ::4, ::4]).abs().max()):>12.3e}" for c in cols))
    text = "\n".join(lines) + "\n"
    print(text)
    with open(os.path.join(ROOT, "profiles", args.name + ".txt"), "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
