"""Reference-written checkpoints -> our modules -> HIP forward == the reference's outputs.

The ``tests/golden/ckpt_*`` files were written by the reference modules in the reference's own
layouts (make_golden.py ckpt_goldens): BasicSR ``{'params', 'params_ema'}`` (base_model.py:213-244)
for KDLAE-T and KDLAE-S, a raw state_dict with BatchNorm buffers for ASDQE (Train/ASDQE.py:210).
They are loaded the way the reference's consumers load them (KDLAE_T.ipynb:1074-1075 and
KDLAE-S.ipynb:109-110 strict on ['params']; ASDQE_test.py:75-84 strict=False), then run on cuda:0.
Tolerance 1e-3 max-abs (north_star).
"""
import lzma
import os

import pytest
import torch

from rethink_acoustic_image_enhancement_amd.ASDQE_model import DenoiseRatePredictor
from rethink_acoustic_image_enhancement_amd.checkpoint import load_checkpoint, load_network
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_student, KDLAE_teacher
from tests.util import GOLDEN, load_fixture, max_abs

pytestmark = pytest.mark.gpu
TOL = 1e-3
DEV = "cuda:0"


def _unpack(name, tmp_path):
    path = tmp_path / f"{name}.pth"
    with open(os.path.join(GOLDEN, f"{name}.pth.xz"), "rb") as f:
        path.write_bytes(lzma.decompress(f.read()))
    return str(path)


@pytest.mark.parametrize("key", ["params", "params_ema"])
def test_teacher_checkpoint_outputs(key, tmp_path):
    d, cfg = load_fixture("ckpt_t_tiny")
    m = KDLAE_teacher(**cfg["kw"])
    assert load_checkpoint(m, _unpack("ckpt_t_tiny", tmp_path), param_key=key, strict=True) == ([], [])
    m = m.to(DEV).eval()
    with torch.no_grad():
        o = m({"img": torch.from_numpy(d["img"]).to(DEV), "denoise_rate": torch.from_numpy(d["rate"]).to(DEV)})
    e_hq = max_abs(o["hq"].cpu(), torch.from_numpy(d[f"{key}_hq"]))
    e_sr = max_abs(o["sr"].cpu(), torch.from_numpy(d[f"{key}_sr"]))
    print(f"ckpt_t_tiny[{key}]: hq {e_hq:.3e} sr {e_sr:.3e}")
    assert e_hq <= TOL and e_sr <= TOL


def test_teacher_reload_switches_weights(tmp_path):
    """One module, two loads (params then params_ema) between forwards: the HIP handle repacks."""
    d, cfg = load_fixture("ckpt_t_tiny")
    path = _unpack("ckpt_t_tiny", tmp_path)
    m = KDLAE_teacher(**cfg["kw"]).to(DEV).eval()
    inp = {"img": torch.from_numpy(d["img"]).to(DEV), "denoise_rate": torch.from_numpy(d["rate"]).to(DEV)}
    for key in ("params", "params_ema", "params"):
        load_network(m, path, strict=True, param_key=key)
        with torch.no_grad():
            hq = m(inp)["hq"].cpu()
        assert max_abs(hq, torch.from_numpy(d[f"{key}_hq"])) <= TOL, key


@pytest.mark.parametrize("key", ["params", "params_ema"])
def test_student_checkpoint_outputs(key, tmp_path):
    d, cfg = load_fixture("ckpt_s_default")
    m = KDLAE_student(**cfg["kw"])
    m.load_state_dict(torch.load(_unpack("ckpt_s_default", tmp_path), map_location="cpu", weights_only=True)[key])
    with torch.no_grad():
        y = m.to(DEV).eval()(torch.from_numpy(d["x"]).to(DEV)).cpu()
    e = max_abs(y, torch.from_numpy(d[f"{key}_y"]))
    print(f"ckpt_s_default[{key}]: {e:.3e}")
    assert e <= TOL


def test_asdqe_raw_checkpoint_outputs(tmp_path):
    d, cfg = load_fixture("ckpt_a_default")
    m = DenoiseRatePredictor(**cfg["kw"])
    m.load_state_dict(torch.load(_unpack("ckpt_a_default", tmp_path), map_location=DEV, weights_only=True),
                      strict=False)                                   # ASDQE_test.py:79
    m = m.to(DEV).eval()
    with torch.no_grad():
        s, f = m(torch.from_numpy(d["lq"]).to(DEV), torch.from_numpy(d["gt"]).to(DEV), return_features=True)
    e_s = max_abs(s.cpu(), torch.from_numpy(d["score"]))
    e_f = max_abs(f.cpu()[:, :, ::4, ::4], torch.from_numpy(d["feat_sub"]))
    print(f"ckpt_a_default: score {e_s:.3e} feat {e_f:.3e}")
    assert e_s <= TOL and e_f <= TOL
