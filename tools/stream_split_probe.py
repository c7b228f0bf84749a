"""A/B probe: does running the T16 forward as two half-batches on two HIP streams beat one stream?

Two module copies (each with its own handle, workspace and HIP graphs) take images [0, 8) and [8, 16)
on two streams forked from / joined into the current stream; images are independent and the forward is
batch-invariant, so the outputs are the same bits as the one-stream full-batch forward (checked).
usage: python tools/stream_split_probe.py [steps]"""
import copy
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_teacher  # noqa: E402
from rethink_acoustic_image_enhancement_amd.hashweights import hash_images, load_hash_weights  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
kw = dict(LayerNorm_type="BiasFree")
m1 = KDLAE_teacher(**kw)
load_hash_weights(m1)
m1 = m1.to(dev).eval()
m2 = copy.deepcopy(m1)
B, H, W = 16, 512, 512
img = torch.from_numpy(hash_images("bench", (B, 3, H, W))).to(dev)
rate = torch.full((B, 1, H, W), 0.6, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def full():
    return m1({"img": img, "denoise_rate": rate})


def split(nstreams):
    cur = torch.cuda.current_stream(dev)
    h = B // 2
    outs = []
    for i, (m, s) in enumerate(((m1, s1), (m2, s2))):
        s = s if nstreams == 2 else cur
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            outs.append(m({"img": img[i * h:(i + 1) * h], "denoise_rate": rate[i * h:(i + 1) * h]}))
    if nstreams == 2:
        cur.wait_stream(s1)
        cur.wait_stream(s2)
    return {k: torch.cat([o[k] for o in outs]) for k in ("hq", "sr")}


def timed(fn):
    with torch.no_grad():
        for _ in range(3):  # eager, capture, replay
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            out = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / steps * 1e3, out


res = {}
ms, ref = timed(full)
res["one_stream_full_batch"] = ms
for n in (1, 2):
    ms, out = timed(lambda: split(n))
    res[f"{n}_stream_two_halves"] = ms
    res[f"{n}_stream_equal_bits"] = bool(torch.equal(out["hq"], ref["hq"]) and torch.equal(out["sr"], ref["sr"]))
res = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}
res["images_per_s"] = {k: round(B / v * 1e3, 2) for k, v in res.items() if k.endswith(("batch", "halves"))}
print(json.dumps(res))
