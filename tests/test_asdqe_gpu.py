"""ASDQE (DenoiseRatePredictor, ASDQE/ASDQE_model.py:123-171, eval mode) on the HIP path vs the
reference's outputs (committed fixtures: score, pooled features, feature-map subsamples) and the CPU
oracle.  Tolerance: 1e-3 fp32 max-abs (north_star) on the score and on the UNet output map."""
import numpy as np
import pytest
import torch

from oracle.asdqe_oracle import AsdqeCfg, asdqe_features, asdqe_param_shapes
from rethink_acoustic_image_enhancement_amd.ASDQE_model import DenoiseRatePredictor
from rethink_acoustic_image_enhancement_amd.hashweights import hash_images, hash_normal, load_hash_weights
from tests.util import hash_sd_for, load_fixture, max_abs

pytestmark = pytest.mark.gpu
TOL = 1e-3
DEV = "cuda:0"


def _model(kw):
    m = DenoiseRatePredictor(**kw)
    load_hash_weights(m)
    return m.to(DEV).eval()


def _run(m, lq, gt):
    with torch.no_grad():
        s, f = m(lq.to(DEV), gt.to(DEV), return_features=True)
    torch.cuda.synchronize()
    return s.cpu(), f.cpu()


def _inputs(key, shape):
    B = shape[0]
    scale = torch.linspace(0.3, 1.0, B).view(B, 1, 1, 1)
    gt = torch.from_numpy(hash_images(f"gt:{key}", shape)) * scale
    lq = (gt + 0.1 * torch.from_numpy(hash_normal(f"n:{key}", shape))).clamp(0, 1)
    return lq.float().contiguous(), gt.float().contiguous()


@pytest.mark.parametrize("name", ["a_b4_64", "a_b2_40x56"])
def test_golden_fixture(name):
    d, kw = load_fixture(name)
    s, f = _run(_model(kw), torch.from_numpy(d["lq"]), torch.from_numpy(d["gt"]))
    e_s = max_abs(s, torch.from_numpy(d["score"]))
    e_f = max_abs(f[:, :, ::4, ::4], torch.from_numpy(d["feat_sub"]))
    e_g = float(np.abs(f.double().mean(dim=(2, 3)).numpy() - d["gap64"]).max())
    print(f"{name}: score {e_s:.3e} feat {e_f:.3e} gap {e_g:.3e}")
    assert e_s <= TOL and e_f <= TOL and e_g <= TOL


@pytest.mark.parametrize("kw,shape", [
    (dict(in_channels=3, dim=16), (2, 3, 37, 50)),      # ragged: pad_to_multiple on both axes
    (dict(in_channels=1, dim=32), (3, 1, 64, 96)),
    (dict(in_channels=3, dim=16), (2, 3, 256, 256)),    # the A64 per-image shape
])
def test_vs_oracle(kw, shape):
    lq, gt = _inputs(f"{kw}{shape}", shape)
    s, f = _run(_model(kw), lq, gt)
    cfg = AsdqeCfg(**kw)
    with torch.no_grad():
        ref = asdqe_features(hash_sd_for(asdqe_param_shapes(cfg)), lq, gt, cfg)
    e_s, e_f = max_abs(s, ref["score"]), max_abs(f, ref["feat"])
    print(f"{kw} {shape}: score {e_s:.3e} feat {e_f:.3e}")
    assert e_s <= TOL and e_f <= TOL


def test_score_only_path_batch_invariance_and_determinism():
    m = _model(dict())
    lq, gt = _inputs("inv", (4, 3, 48, 64))
    with torch.no_grad():
        s = m(lq.to(DEV), gt.to(DEV)).cpu()
        s2 = m(lq.to(DEV), gt.to(DEV)).cpu()
        s1 = m(lq[2:3].to(DEV), gt[2:3].to(DEV)).cpu()
    assert torch.equal(s, s2)
    assert torch.equal(s[2:3], s1)  # GAP slots depend on the image size only (asdqe.cpp gap_slots)
    s_f, _ = _run(m, lq, gt)
    assert torch.equal(s, s_f)


def test_eval_mode_and_device_errors():
    m = _model(dict())
    lq, gt = _inputs("err", (1, 3, 32, 32))
    m.train()
    with pytest.raises(RuntimeError, match="eval"):
        m(lq.to(DEV), gt.to(DEV))
    m.eval()
    with pytest.raises(RuntimeError, match="no CPU"):
        m(lq, gt)
