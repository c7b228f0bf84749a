"""KDLAE-S training step (KDLAES.yml: KDLAE_student + L1LossForVideoFrames + clip + AdamW), CPU side:
the training oracle against goldens written by the *imported reference* (its KDLAE_student and its
own losses.py L1LossForVideoFrames, autograd through both), and the training handle's flat layout.
No GPU compute here.

Tolerances: loss 1e-6 relative; gradients 1e-4 of max |g| (fp32, a different reduction order than
oneDNN); per-key |g| sums 1e-4 relative; parameters after two AdamW steps (lr 3e-4) 2e-6 absolute.
"""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from oracle.kdlae_oracle import StudentCfg, student_param_shapes
from oracle.train_oracle import l1_video_frames, student_loss_and_grads
from rethink_acoustic_image_enhancement_amd import _lib
from tests.util import GOLDEN, hash_sd_for

CASES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("train_s_"))
SUB = 4  # tests/golden/make_golden.py S_TRAIN_SUB


def load_case(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    js = {k: json.loads(bytes(d[k]).decode()) for k in ("cfg", "loss_kw", "opt", "keys")}
    return d, js


def test_cases_present():
    assert len(CASES) >= 3


@pytest.mark.parametrize("name", CASES)
def test_oracle_grads_match_reference(name):
    d, js = load_case(name)
    cfg = StudentCfg(**js["cfg"])
    sd = hash_sd_for(student_param_shapes(cfg))
    keys = js["keys"]
    assert set(sd) == set(keys)
    sd = {k: sd[k] for k in keys}
    loss, grads = student_loss_and_grads(sd, torch.from_numpy(d["x"]), torch.from_numpy(d["target"]), cfg,
                                         **js["loss_kw"])
    assert abs(float(loss) - d["loss"][0]) <= 1e-6 * abs(d["loss"][0])
    flat = torch.cat([grads[k].reshape(-1) for k in keys]).numpy()
    sub = d["grad1_sub"]
    assert np.abs(flat[::SUB] - sub).max() <= 1e-4 * np.abs(sub).max()
    sums = np.array([[grads[k].double().sum(), grads[k].double().abs().sum()] for k in keys])
    np.testing.assert_allclose(sums[:, 1], d["grad_sums"][:, 1], rtol=1e-4, atol=1e-9)


@pytest.mark.parametrize("name", CASES)
def test_oracle_two_adamw_steps_match_reference(name):
    d, js = load_case(name)
    cfg = StudentCfg(**js["cfg"])
    keys = js["keys"]
    sd = hash_sd_for(student_param_shapes(cfg))
    params = {k: sd[k].clone().requires_grad_(True) for k in keys}
    opt = torch.optim.AdamW(list(params.values()), lr=js["opt"]["lr"], weight_decay=js["opt"]["weight_decay"],
                            betas=tuple(js["opt"]["betas"]))
    x, tgt = torch.from_numpy(d["x"]), torch.from_numpy(d["target"])
    from oracle.kdlae_oracle import student_forward
    losses, norms = [], []
    for _ in range(2):
        opt.zero_grad()
        loss = l1_video_frames(student_forward(params, x, cfg), tgt, **js["loss_kw"])
        loss.backward()
        norms.append(float(torch.nn.utils.clip_grad_norm_(list(params.values()), js["opt"]["clip"])))
        opt.step()
        losses.append(float(loss))
    np.testing.assert_allclose(losses, d["loss"], rtol=1e-6)
    np.testing.assert_allclose(norms, d["norm"], rtol=1e-5)
    p0 = torch.cat([sd[k].reshape(-1).double() for k in keys])
    p2 = torch.cat([params[k].detach().reshape(-1).double() for k in keys])
    assert np.abs((p2 - p0).numpy()[::SUB] - d["delta2_sub"]).max() <= 2e-6


def test_video_loss_restatement():
    """losses.py:440-526 on hand-checkable values: 2 frames of 2 pixels."""
    p = torch.tensor([[[[0.0, 0.5]], [[0.2, 0.05]]]])   # [1, 2, 1, 2]
    t = torch.tensor([[[[0.05, 0.3]], [[0.2, 0.3]]]])
    # per frame: |p-t| = (.05, .2, 0, .25), bins p (0,1,1,0) t (0,1,1,1) -> (0,0,0,1): mean (0.5 + 1) / 4
    # temporal: dp = (.2, -.45), dt = (.15, 0) -> |.05| + |.45| = .5, mean .25
    want = 0.64 * (0.5 + 1.0) / 4 + 0.36 * 0.25
    assert abs(float(l1_video_frames(p, t)) - want) < 1e-7
    assert abs(float(l1_video_frames(p, t, reduction="sum")) - (0.64 * 1.5 + 0.36 * 0.5)) < 1e-6


def test_training_handle_layout():
    L = _lib.lib()
    cfg = _lib.SConfig()
    cfg.inp_channels = cfg.out_channels = 1
    cfg.residual = 1
    cfg.num_hidden = 3
    for i, v in enumerate([16, 32, 64]):
        cfg.hidden_channels[i] = v
    cfg.kernel_size = 3
    h = ctypes.c_void_p()
    _lib.check(L.kdlae_st_create(ctypes.byref(cfg), 0, ctypes.byref(h)), "kdlae_st_create")
    try:
        shapes = student_param_shapes(StudentCfg(inp_channels=1, out_channels=1, residual=True,
                                                 hidden_channels=[16, 32, 64]))
        # named_parameters() order of the reference module (the golden's key list)
        _, js = load_case("train_s_kdlaes")
        shapes = {k: shapes[k] for k in js["keys"]}
        got, prev_end = [], 0
        for i in range(L.kdlae_st_num_params(h)):
            name, n, off = ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_int64()
            _lib.check(L.kdlae_st_param_info(h, i, ctypes.byref(name), ctypes.byref(n), ctypes.byref(off)), "info")
            got.append((name.value.decode(), n.value))
            assert off.value % 4 == 0 and off.value >= prev_end
            prev_end = off.value + n.value
        assert got == [(k, int(np.prod(s))) for k, s in shapes.items()]
        assert L.kdlae_st_num_floats(h) >= prev_end
        assert L.kdlae_st_workspace_bytes(h, 2, 7, 32, 32) > 0
        assert L.kdlae_st_workspace_bytes(h, 2, 7, 30, 32) == -1  # H % 4 != 0
    finally:
        L.kdlae_st_destroy(h)
