"""Config-1 (MDD sonar crop 512x512): the reference's own fp32 CPU forward against itself.

ANALYSIS INFRASTRUCTURE (imports oracle/, the CPU restatement pinned by the reference's own outputs).

The reference fp32 forward (= the oracle in fp32, the same torch ops as KDLAE/KDLAE_model.py) is run
with torch intra-op thread counts 1, 2, 4 and 8 — the only change is how the CPU kernels split their
reductions.  Reported: each run's max-abs error vs the fp64 output and vs the 8-thread run over the
config-1 test samples (tools/config1_ensemble.sample_errors).  If two thread counts of the reference
differ by more than 1e-3 on this input, a 1e-3 max-abs bar against "the reference fp32 output" is not a
property any other implementation can be held to.  Writes profiles/<name>.txt.
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import oracle.kdlae_oracle as O  # noqa: E402
from config1_ensemble import sample_errors  # noqa: E402
from tests.util import hash_sd_for, load_fixture, mdd_input_tensor  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="8,4,2,1")
    ap.add_argument("--name", default="r04_config1_threads")
    args = ap.parse_args()
    d, kw = load_fixture("t_mdd_512")
    cfg = O.TeacherCfg(**kw)
    sd = hash_sd_for(O.teacher_param_shapes(cfg))
    img = mdd_input_tensor(d)
    rate = torch.full((1, 1, 512, 512), 0.6)
    outs = {}
    with torch.no_grad():
        for t in (int(v) for v in args.threads.split(",")):
            torch.set_num_threads(t)
            t0 = time.time()
            outs[t] = O.teacher_forward(sd, img, rate, cfg)
            print(f"threads {t}: {time.time() - t0:.0f} s", flush=True)
    first = next(iter(outs))
    lines = [__doc__.strip(), "",
             f"{'threads':>8}{'hq vs fp64':>13}{'sr vs fp64':>13}{'hq vs ' + str(first) + 't':>13}"
             f"{'sr vs ' + str(first) + 't':>13}   (max-abs; vs fp64 over the test samples, vs {first}t over the "
             "whole output)"]
    for t, o in outs.items():
        e = sample_errors(o, d)
        dh = float((o["hq"] - outs[first]["hq"]).abs().max())
        ds = float((o["sr"] - outs[first]["sr"]).abs().max())
        lines.append(f"{t:>8}{e['hq'][0]:>13.3e}{e['sr'][0]:>13.3e}{dh:>13.3e}{ds:>13.3e}")
    text = "\n".join(lines) + "\n"
    print(text)
    with open(os.path.join(ROOT, "profiles", args.name + ".txt"), "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
