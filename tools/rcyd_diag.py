"""Diagnostic: which gradient keys differ between the stored-yd GDFN backward (KDLAE_DEBUG=train_keep_yd)
and the recomputed-yd one, at the KDLAET.yml patch setting (6 x 128^2).
usage: python tools/rcyd_diag.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rethink_acoustic_image_enhancement_amd.hashweights import hash_images, load_hash_weights  # noqa: E402
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_teacher  # noqa: E402
from rethink_acoustic_image_enhancement_amd.train import KDLAETrainer  # noqa: E402

DEV = torch.device("cuda", 0)
m = KDLAE_teacher(LayerNorm_type="BiasFree")
load_hash_weights(m)
m = m.to(DEV).train()
B, H, W = 6, 128, 128
img = torch.from_numpy(hash_images("img:rcyd", (B, 3, H, W))).to(DEV)
rate = torch.full((B, 1, H, W), 0.6, device=DEV)
gt = {"hq": img.clamp(0.2, 0.8), "sr": torch.nn.functional.interpolate(img, scale_factor=2).clamp(0.2, 0.8)}
tr = KDLAETrainer(m)
inp = {"img": img, "denoise_rate": rate}
grads = {}
for flag in ("train_keep_yd,train_serial", "train_serial", "train_keep_yd,train_serial"):
    os.environ["KDLAE_DEBUG"] = flag
    tr.grad.fill_(float("nan"))
    tr.forward_backward(inp, gt)
    torch.cuda.synchronize()
    grads.setdefault(flag, []).append(tr.grad.clone())
a, b = grads["train_keep_yd,train_serial"], grads["train_serial"][0]
print("keep vs keep equal:", torch.equal(a[0], a[1]))
eng = tr.engine
rows = []
for k, n, off in eng.keys:
    d = (a[0][off:off + n] - b[off:off + n]).abs()
    if float(d.max()) > 0:
        rows.append((k, float(d.max()), int((d > 0).sum()), n, float(a[0][off:off + n].abs().max())))
print(f"{len(rows)} of {len(eng.keys)} keys differ")
print("equal:", [k for k, n, off in eng.keys if k not in {r[0] for r in rows}])
for r in rows[-30:]:
    print(f"{r[0]:55s} max {r[1]:.2e} count {r[2]:7d}/{r[3]:7d} scale {r[4]:.2e}")
