"""The CPU oracle (oracle/kdlae_oracle.py) against golden vectors of the imported reference."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle.kdlae_oracle import (StudentCfg, TeacherCfg, student_forward, student_param_shapes,
                                 teacher_forward, teacher_param_shapes)
from tests.util import GOLDEN, hash_sd_for, load_fixture, max_abs, mdd_input_tensor

TEACHER = sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, "t_*.npz"))
                 if "_512" not in f)
STUDENT = sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, "s_*.npz")))


@pytest.mark.parametrize("name", TEACHER)
def test_teacher_oracle_matches_reference(name):
    d, kw = load_fixture(name)
    cfg = TeacherCfg(**kw)
    sd = hash_sd_for(teacher_param_shapes(cfg))
    out = teacher_forward(sd, torch.from_numpy(d["img"]), torch.from_numpy(d["rate"]), cfg)
    assert max_abs(out["hq"], torch.from_numpy(d["hq"])) <= 1e-6
    if "sr" in d:
        assert max_abs(out["sr"], torch.from_numpy(d["sr"])) <= 1e-6
    else:
        assert out["sr"] is None


@pytest.mark.parametrize("name", STUDENT)
def test_student_oracle_matches_reference(name):
    d, kw = load_fixture(name)
    cfg = StudentCfg(**kw)
    sd = hash_sd_for(student_param_shapes(cfg))
    y = student_forward(sd, torch.from_numpy(d["x"]), cfg)
    assert max_abs(y, torch.from_numpy(d["y"])) <= 1e-6


def test_teacher_oracle_mdd_512():
    """Config 1 (1x3x512x512 MDD sample, denoise_rate 0.6) against the reference's subsamples."""
    d, kw = load_fixture("t_mdd_512")
    cfg = TeacherCfg(**kw)
    sd = hash_sd_for(teacher_param_shapes(cfg))
    img = mdd_input_tensor(d)
    with torch.no_grad():
        out = teacher_forward(sd, img, torch.full((1, 1, 512, 512), 0.6), cfg)
    assert max_abs(out["hq"][:, :, ::8, ::8], torch.from_numpy(d["hq_sub"])) <= 1e-5
    assert max_abs(out["sr"][:, :, ::8, ::8], torch.from_numpy(d["sr_sub"])) <= 1e-5
    np.testing.assert_allclose(out["hq"].double().sum(dim=(2, 3)).numpy(), d["hq_chsum"], rtol=1e-5)
    np.testing.assert_allclose(out["sr"].double().sum(dim=(2, 3)).numpy(), d["sr_chsum"], rtol=1e-5)


def test_oracle_rejects_bad_shapes():
    cfg = TeacherCfg(dim=16, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1)
    sd = hash_sd_for(teacher_param_shapes(cfg))
    with pytest.raises(RuntimeError):
        teacher_forward(sd, torch.zeros(1, 3, 20, 24), torch.zeros(1, 1, 20, 24), cfg)
    with pytest.raises(NotImplementedError):
        teacher_forward(sd, torch.zeros(1, 3, 16, 16), torch.zeros(1, 1, 16, 16),
                        TeacherCfg(dim=16, dual_pixel_task=True))


ASDQE = ["a_b4_64", "a_b2_40x56"]


@pytest.mark.parametrize("name", ASDQE)
def test_asdqe_oracle_matches_reference(name):
    from oracle.asdqe_oracle import AsdqeCfg, asdqe_features, asdqe_param_shapes
    d, kw = load_fixture(name)
    cfg = AsdqeCfg(**kw)
    shapes = asdqe_param_shapes(cfg)
    sd = hash_sd_for(shapes)
    with torch.no_grad():
        f = asdqe_features(sd, torch.from_numpy(d["lq"]), torch.from_numpy(d["gt"]), cfg)
    assert max_abs(f["feat"][:, :, ::4, ::4], torch.from_numpy(d["feat_sub"])) <= 1e-5
    assert max_abs(f["merged"][:, :, ::4, ::4], torch.from_numpy(d["merged_sub"])) <= 1e-5
    np.testing.assert_allclose(f["feat"].double().mean(dim=(2, 3)).numpy(), d["gap64"], rtol=0, atol=1e-6)
    assert max_abs(f["score"], torch.from_numpy(d["score"])) <= 1e-6
