"""Config-1 (MDD sonar crop 512x512, denoise_rate 0.6): how far fp32 evaluations of the reference land
from its fp64 output — the spread the config-1 parity test is judged against.

ANALYSIS INFRASTRUCTURE (imports oracle/, the CPU restatement pinned by the reference's own outputs).

The reference's fp32 forward (= the oracle in fp32) is run with every LayerNorm output multiplied by
(1 + u 2^-24), u ~ U[-1, 1] per element (a half-ulp-scale perturbation, what any other fp32 summation
order or rounding of those ops produces), once per seed.  For each run the max-abs / mean-abs error
against the reference's fp64 output is taken over exactly the samples tests/test_kdlae_gpu.py
::test_mdd_512_config1 compares (the fixture's [::8, ::8] subsample plus one full row).

Writes profiles/<name>.txt and tests/golden/t_mdd_512_ensemble.json.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle.kdlae_oracle as O  # noqa: E402
from tests.util import hash_sd_for, load_fixture, mdd_input_tensor  # noqa: E402

ORIG_LN = O.layer_norm


def sample_errors(out, d):
    """(max, mean) abs error vs the fixture's fp64 samples, per output, as the GPU test computes them."""
    res = {}
    for k, sub64, row64, row in (("hq", "hq64_sub", "hq64_row257", 257), ("sr", "sr64_sub", "sr64_row515", 515)):
        y = out[k].double()
        ours = torch.cat([y[:, :, ::8, ::8].flatten(), y[:, :, row, :].flatten()])
        ref = torch.cat([torch.from_numpy(d[sub64]).double().flatten(), torch.from_numpy(d[row64]).double().flatten()])
        e = (ours - ref).abs()
        res[k] = (float(e.max()), float(e.mean()))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=8)
    ap.add_argument("--name", default="r04_config1_ensemble")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    d, kw = load_fixture("t_mdd_512")
    cfg = O.TeacherCfg(**kw)
    sd = hash_sd_for(O.teacher_param_shapes(cfg))
    img = mdd_input_tensor(d)
    rate = torch.full((1, 1, 512, 512), 0.6)
    runs = []
    with torch.no_grad():
        base = sample_errors(O.teacher_forward(sd, img, rate, cfg), d)
        for seed in range(args.seeds):
            g = torch.Generator().manual_seed(seed)

            def ln(x, sd_, prefix, lt):
                y = ORIG_LN(x, sd_, prefix, lt)
                u = torch.rand(y.shape, generator=g) * 2 - 1
                return y * (1 + u * 2.0 ** -24)

            O.layer_norm = ln
            t = time.time()
            try:
                e = sample_errors(O.teacher_forward(sd, img, rate, cfg), d)
            finally:
                O.layer_norm = ORIG_LN
            runs.append(e)
            print(f"seed {seed}: hq {e['hq'][0]:.3e} sr {e['sr'][0]:.3e} ({time.time() - t:.0f} s)", flush=True)
    hq = sorted(r["hq"][0] for r in runs)
    sr = sorted(r["sr"][0] for r in runs)
    summary = {
        "what": "max-abs error vs the reference fp64 output over the config-1 test samples of the reference fp32 "
                "forward with LN outputs perturbed by (1 + u 2^-24), u ~ U[-1,1], one run per seed "
                "(tools/config1_ensemble.py)",
        "unperturbed_ref32": {"hq": base["hq"][0], "sr": base["sr"][0], "hq_mean": base["hq"][1],
                              "sr_mean": base["sr"][1]},
        "hq_max": [r["hq"][0] for r in runs], "sr_max": [r["sr"][0] for r in runs],
        "hq_mean": [r["hq"][1] for r in runs], "sr_mean": [r["sr"][1] for r in runs],
        "hq_median": float(np.median(hq)), "sr_median": float(np.median(sr)),
    }
    lines = [__doc__.strip(), "",
             f"unperturbed reference fp32: hq {base['hq'][0]:.3e} sr {base['sr'][0]:.3e} "
             f"(mean {base['hq'][1]:.2e} / {base['sr'][1]:.2e})",
             f"{'seed':>6}{'hq max':>12}{'sr max':>12}{'hq mean':>12}{'sr mean':>12}"]
    for i, r in enumerate(runs):
        lines.append(f"{i:>6}{r['hq'][0]:>12.3e}{r['sr'][0]:>12.3e}{r['hq'][1]:>12.2e}{r['sr'][1]:>12.2e}")
    lines.append(f"{'median':>6}{summary['hq_median']:>12.3e}{summary['sr_median']:>12.3e}")
    lines.append(f"{'range':>6}  hq {hq[0]:.3e} .. {hq[-1]:.3e}   sr {sr[0]:.3e} .. {sr[-1]:.3e}")
    text = "\n".join(lines) + "\n"
    print(text)
    with open(os.path.join(ROOT, "profiles", args.name + ".txt"), "w") as f:
        f.write(text)
    with open(os.path.join(ROOT, "tests", "golden", "t_mdd_512_ensemble.json"), "w") as f:
        json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
