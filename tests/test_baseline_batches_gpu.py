"""Parity at the BASELINE.json batch sizes (configs[1..3]) on one MI355X, through the C ABI.

* T16 — KDLAE-T released config (KDLAE_T.ipynb:1059-1071), bs=16 at 512x512, static=train: every
  image of the batch is bit-identical to the same image run alone (the Gram slot partition depends
  on the image size only, kdlae_t.cpp nslots_for), and images 0 and 15 match the CPU oracle to
  1e-3 max-abs on hq and sr (BASELINE north_star).
* S8 — KDLAE-S bs=8, 4x512x512 (KDLAE-S.ipynb:106): every sample vs the oracle, samples bit-equal
  to single runs.
* A64 — ASDQE bs=64 at 256x256 (ASDQE/ASDQE_test.py): all 64 scores and UNet feature maps vs the
  oracle, singles bit-equal (GAP slots depend on the image size only, asdqe.cpp gap_slots).

Inputs are the bench's own synthetic workload (bench.py make_inputs / bench_secondary).
"""
import numpy as np
import pytest
import torch

from oracle.asdqe_oracle import AsdqeCfg, asdqe_features
from oracle.kdlae_oracle import StudentCfg, TeacherCfg, psnr, student_forward, teacher_forward
from rethink_acoustic_image_enhancement_amd.ASDQE_model import DenoiseRatePredictor
from rethink_acoustic_image_enhancement_amd.hashweights import hash_images, hash_uniform, load_hash_weights
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_student, KDLAE_teacher
from tests.util import max_abs

pytestmark = pytest.mark.gpu
TOL = 1e-3
DEV = "cuda:0"
T_KW = dict(inp_channels=3, out_channels=3, dim=48, num_blocks=[4, 6, 6, 8], num_refinement_blocks=4,
            heads=[1, 2, 4, 8], ffn_expansion_factor=2.66, bias=False, LayerNorm_type="BiasFree",
            dual_pixel_task=False, static="train", params="cat")
S_KW = dict(inp_channels=1, out_channels=1, residual=True, hidden_channels=[16, 32, 64])
A_KW = dict(in_channels=3, dim=16)


def _t16_inputs(n=16, H=512, W=512):
    """bench.py make_inputs(0, 16, 512, 512): hash images, per-image constant denoise_rate."""
    imgs = np.stack([hash_images(f"img16:{i}", (3, H, W)) for i in range(n)])
    rates = (hash_uniform("rate16", n) + 1.0) * 0.5
    rate = np.broadcast_to(rates.astype(np.float32)[:, None, None, None], (n, 1, H, W)).copy()
    return torch.from_numpy(imgs), torch.from_numpy(rate)


@pytest.fixture(scope="module")
def t16():
    m = KDLAE_teacher(**T_KW)
    load_hash_weights(m)
    m = m.to(DEV).eval()
    img, rate = _t16_inputs()
    with torch.no_grad():
        out = m({"img": img.to(DEV), "denoise_rate": rate.to(DEV)})
        full = {k: v.cpu() for k, v in out.items()}
        del out
        singles = []
        for i in range(img.shape[0]):
            o = m({"img": img[i:i + 1].to(DEV), "denoise_rate": rate[i:i + 1].to(DEV)})
            singles.append({k: v.cpu() for k, v in o.items()})
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    del m
    torch.cuda.empty_cache()
    return dict(img=img, rate=rate, full=full, singles=singles, sd=sd)


def test_t16_every_image_equals_single_run(t16):
    bad = [i for i, s in enumerate(t16["singles"])
           if not (torch.equal(t16["full"]["hq"][i:i + 1], s["hq"]) and torch.equal(t16["full"]["sr"][i:i + 1], s["sr"]))]
    assert not bad, f"images {bad} of the bs=16 batch differ from their single-image runs"
    assert torch.isfinite(t16["full"]["hq"]).all() and torch.isfinite(t16["full"]["sr"]).all()


@pytest.mark.parametrize("i", [0, 15])
def test_t16_image_vs_oracle(t16, i):
    with torch.no_grad():
        ref = teacher_forward(t16["sd"], t16["img"][i:i + 1], t16["rate"][i:i + 1], TeacherCfg(**T_KW))
    e_hq = max_abs(t16["full"]["hq"][i:i + 1], ref["hq"])
    e_sr = max_abs(t16["full"]["sr"][i:i + 1], ref["sr"])
    print(f"T16 image {i}: hq max-abs {e_hq:.3e} ({psnr(t16['full']['hq'][i:i + 1], ref['hq']):.1f} dB), "
          f"sr max-abs {e_sr:.3e} ({psnr(t16['full']['sr'][i:i + 1], ref['sr']):.1f} dB)")
    assert e_hq <= TOL and e_sr <= TOL


def test_s8_full_batch():
    m = KDLAE_student(**S_KW)
    load_hash_weights(m)
    m = m.to(DEV).eval()
    x = torch.from_numpy(np.stack([hash_images(f"s8:{i}", (4, 512, 512)) for i in range(8)]))
    with torch.no_grad():
        y = m(x.to(DEV)).cpu()
        singles = [m(x[i:i + 1].to(DEV)).cpu() for i in range(8)]
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    cfg = StudentCfg(**S_KW)
    errs = []
    for i in range(8):
        assert torch.equal(y[i:i + 1], singles[i]), f"sample {i} differs from its single run"
        with torch.no_grad():
            errs.append(max_abs(y[i:i + 1], student_forward(sd, x[i:i + 1], cfg)))
    print("S8 per-sample max-abs vs oracle:", " ".join(f"{e:.2e}" for e in errs))
    assert max(errs) <= TOL


def test_a64_full_batch():
    m = DenoiseRatePredictor(**A_KW)
    load_hash_weights(m)
    m = m.to(DEV).eval()
    # bench.py bench_secondary (a64): gt hash images, lq = clamp(gt + 0.1 u)
    g = torch.from_numpy(np.stack([hash_images(f"a64gt:{i}", (3, 256, 256)) for i in range(64)]))
    lq = (g + 0.1 * torch.from_numpy(hash_uniform("a64n", g.numel()).astype(np.float32)).view_as(g)).clamp(0, 1)
    with torch.no_grad():
        s_only = m(lq.to(DEV), g.to(DEV)).cpu()
        s, f = m(lq.to(DEV), g.to(DEV), return_features=True)
        s, f = s.cpu(), f.cpu()
        singles = {i: m(lq[i:i + 1].to(DEV), g[i:i + 1].to(DEV)).cpu() for i in (0, 31, 63)}
    assert torch.equal(s, s_only)
    for i, si in singles.items():
        assert torch.equal(s[i:i + 1], si), f"image {i} score differs from its single run"
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    cfg = AsdqeCfg(**A_KW)
    e_s = e_f = 0.0
    for c0 in range(0, 64, 16):
        with torch.no_grad():
            ref = asdqe_features(sd, lq[c0:c0 + 16], g[c0:c0 + 16], cfg)
        e_s = max(e_s, max_abs(s[c0:c0 + 16], ref["score"]))
        e_f = max(e_f, max_abs(f[c0:c0 + 16], ref["feat"]))
    print(f"A64: score max-abs {e_s:.3e}, UNet feature map max-abs {e_f:.3e} (64 images)")
    assert e_s <= TOL and e_f <= TOL
