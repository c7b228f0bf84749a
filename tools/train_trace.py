"""Per-launch timing of one KDLAE-T training step (bench.py --workload train setting, KDLAET.yml
6 x 128^2): the engine brackets every launch with HIP events under KDLAE_DEBUG=train_trace and
appends "phase,layer,kernel,ms" rows to KDLAE_PROBE_DUMP.  Prints the time per kernel and per GEMM
role (fwd / dX / dW / MDTA contractions) and the 25 slowest launches.
usage: python tools/train_trace.py OUT.csv"""
import collections
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import KW, make_inputs  # noqa: E402
from rethink_acoustic_image_enhancement_amd.hashweights import hash_images, load_hash_weights  # noqa: E402
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_teacher  # noqa: E402
from rethink_acoustic_image_enhancement_amd.train import KDLAETrainer  # noqa: E402

out = sys.argv[1]
dev = torch.device("cuda", 0)
B, H, W = 6, 128, 128
model = KDLAE_teacher(**KW)
load_hash_weights(model)
model = model.to(dev)
img, rate = make_inputs(1000, B, H, W)
gt_hq = torch.from_numpy(np.stack([hash_images(f"train_gt:{i}", (3, H, W)) for i in range(B)]))
gt_sr = torch.from_numpy(np.stack([hash_images(f"train_gtsr:{i}", (3, 2 * H, 2 * W)) for i in range(B)]))
batch = {"img": img.to(dev), "denoise_rate": rate.to(dev)}
gt = {"hq": gt_hq.to(dev), "sr": gt_sr.to(dev)}
trainer = KDLAETrainer(model, mixing_augs={"mixup": True, "mixup_beta": 1.2, "use_identity": True})
random.seed(0)
torch.manual_seed(0)


def step():
    lq_m, gt_m = trainer.feed_train_data(batch, gt)
    return trainer.optimize_parameters(lq_m, gt_m)


for _ in range(3):
    step()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    step()
e1.record()
torch.cuda.synchronize()
print(f"untraced step: {e0.elapsed_time(e1) / 5:.2f} ms")
if os.path.exists(out):
    os.remove(out)
# one stream for the traced step (the backward's side stream would overlap the launches being timed)
keep = os.environ.get("KDLAE_DEBUG")
os.environ["KDLAE_DEBUG"] = "train_trace,train_serial"
os.environ["KDLAE_PROBE_DUMP"] = out
step()
torch.cuda.synchronize()
if keep is None:
    del os.environ["KDLAE_DEBUG"]
else:
    os.environ["KDLAE_DEBUG"] = keep
ROLES = {"fwd", "dW", "dX", "fwd3", "dW3", "dX3", "gram", "av", "dA", "dv", "dq", "dk"}
rows = []
for line in open(out):
    ph, layer, kern, ms = line.rstrip("\n").rsplit(",", 3)
    rows.append((ph, layer, kern, float(ms)))
tot = sum(r[3] for r in rows)
print(f"traced launches: {len(rows)}, sum of launch times {tot:.2f} ms")
by_k = collections.Counter()
cnt = collections.Counter()
for ph, layer, kern, ms in rows:
    key = kern
    if kern == "launch_tgemm":
        roles = [t for t in layer.split(" ") if t in ROLES]
        role = roles[-1] if roles else "?"
        role = {"fwd": "fwd1x1", "dW": "dW1x1", "dX": "dX1x1"}.get(role, role)
        key = f"tgemm {role}"
    by_k[(ph, key)] += ms
    cnt[(ph, key)] += 1
for (ph, k), ms in sorted(by_k.items(), key=lambda kv: -kv[1]):
    print(f"{ph:4s} {k:32s} {ms:8.3f} ms  {cnt[(ph, k)]:5d} launches  {100 * ms / tot:5.1f}%")
print("slowest launches:")
for r in sorted(rows, key=lambda r: -r[3])[:25]:
    print(f"  {r[0]} {r[1]:70s} {r[2]:22s} {r[3] * 1e3:8.1f} us")
