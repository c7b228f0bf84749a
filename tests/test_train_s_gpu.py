"""KDLAE-S training on the HIP path (KDLAES.yml: KDLAE_student + L1LossForVideoFrames + clip + AdamW)
against the CPU training oracle, which tests/test_train_s.py pins to the imported reference's own
autograd (KDLAE/KDLAE_model.py:340-431, Train/basicsr/models/losses/losses.py:409-526).

Tolerances: loss 1e-5 relative; every key's gradient within 2e-3 of that key's max |g| (fp32 GEMMs with
other summation orders than oneDNN's); AdamW deltas after two steps within 1e-6 + 2% of the delta scale.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle.kdlae_oracle import StudentCfg, student_forward, student_param_shapes
from oracle.train_oracle import l1_video_frames, student_loss_and_grads
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_student
from rethink_acoustic_image_enhancement_amd.hashweights import hash_images, load_hash_weights
from rethink_acoustic_image_enhancement_amd.train import KDLAESTrainer, L1LossForVideoFrames
from tests.util import GOLDEN, hash_sd_for

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CASES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("train_s_"))


def _case(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    js = {k: json.loads(bytes(d[k]).decode()) for k in ("cfg", "loss_kw", "opt", "keys")}
    return d, js


def _model(cfg):
    m = KDLAE_student(**cfg)
    load_hash_weights(m)
    return m.to(DEV).train()


def _check_grads(model, ref, what):
    for k, p in model.named_parameters():
        g, r = p.grad.detach().cpu(), ref[k]
        scale = float(r.abs().max()) + 1e-12
        err = float((g - r).abs().max())
        assert err <= 2e-3 * scale, f"{what} {k}: max |err| {err:.3e} vs max |g| {scale:.3e}"


@pytest.mark.parametrize("name", CASES)
def test_dropin_backward_matches_oracle(name):
    """model.train(); L1LossForVideoFrames(...)(model(x), target).backward() — the reference loop's own
    calls (image_restoration_model.py:200-213) — gives the oracle's loss and parameter gradients."""
    d, js = _case(name)
    cfg = StudentCfg(**js["cfg"])
    m = _model(js["cfg"])
    x, tgt = torch.from_numpy(d["x"]), torch.from_numpy(d["target"])
    loss = L1LossForVideoFrames(**js["loss_kw"])(m(x.to(DEV)), tgt.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    l_ref, g_ref = student_loss_and_grads(sd, x, tgt, cfg, **js["loss_kw"])
    assert abs(float(loss) - float(l_ref)) <= 1e-5 * abs(float(l_ref)), (float(loss), float(l_ref))
    _check_grads(m, g_ref, name)


def test_odd_channel_training_is_rejected():
    """Hidden widths not divisible by 4 ([6, 10]): the training handle refuses them with a clear error
    before anything launches (its pool / column-gather kernels move float4 channel groups); the eval
    forward of the same model still runs and matches the oracle."""
    cfg_kw = dict(inp_channels=1, out_channels=1, residual=True, hidden_channels=[6, 10])
    m = _model(cfg_kw)
    x = torch.from_numpy(hash_images("odd_s_x", (2, 3, 8, 12)))
    with pytest.raises((NotImplementedError, RuntimeError), match="divisible by 4"):
        m(x.to(DEV))
    m.eval()
    with torch.no_grad():
        out = m(x.to(DEV)).cpu()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref = student_forward(sd, x, StudentCfg(**cfg_kw))
    assert float((out - ref).abs().max()) <= 1e-5


def test_trainer_two_steps_match_oracle():
    """KDLAESTrainer (flat buffers, fused clip + AdamW) over two steps vs the oracle with torch AdamW."""
    d, js = _case("train_s_kdlaes")
    cfg = StudentCfg(**js["cfg"])
    m = _model(js["cfg"])
    keys = [k for k, _ in m.named_parameters()]
    sd0 = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    x, tgt = torch.from_numpy(d["x"]), torch.from_numpy(d["target"])
    tr = KDLAESTrainer(m, lr=js["opt"]["lr"], weight_decay=js["opt"]["weight_decay"], betas=tuple(js["opt"]["betas"]),
                       max_norm=js["opt"]["clip"], loss_kw=js["loss_kw"])
    losses = [float(tr.optimize_parameters(x.to(DEV), tgt.to(DEV))) for _ in range(2)]
    torch.cuda.synchronize()
    params = {k: sd0[k].clone().requires_grad_(True) for k in keys}
    opt = torch.optim.AdamW(list(params.values()), lr=js["opt"]["lr"], weight_decay=js["opt"]["weight_decay"],
                            betas=tuple(js["opt"]["betas"]))
    ref_losses = []
    for _ in range(2):
        opt.zero_grad()
        loss = l1_video_frames(student_forward(params, x, cfg), tgt, **js["loss_kw"])
        loss.backward()
        torch.nn.utils.clip_grad_norm_(list(params.values()), js["opt"]["clip"])
        opt.step()
        ref_losses.append(float(loss))
    np.testing.assert_allclose(losses, ref_losses, rtol=1e-5)
    for k in keys:
        got = m.state_dict()[k].detach().cpu() - sd0[k]
        want = params[k].detach() - sd0[k]
        scale = float(want.abs().max())
        assert float((got - want).abs().max()) <= 1e-6 + 0.02 * scale, k


@pytest.mark.parametrize("frames,red", [(1, "mean"), (4, "mean"), (3, "sum")])
def test_video_loss_and_gradient(frames, red):
    p = torch.from_numpy(hash_images(f"vl_p{frames}", (2, frames, 9, 13)))
    t = torch.from_numpy(hash_images(f"vl_t{frames}", (2, frames, 9, 13)))
    kw = dict(l1loss_weight=0.7, temporal_weight=0.3, reduction=red)
    pg = p.to(DEV).requires_grad_(True)
    loss = L1LossForVideoFrames(**kw)(pg, t.to(DEV))
    loss.backward()
    pr = p.clone().requires_grad_(True)
    ref = l1_video_frames(pr, t, **kw)
    ref.backward()
    assert abs(float(loss) - float(ref)) <= 1e-5 * abs(float(ref))
    assert float((pg.grad.cpu() - pr.grad).abs().max()) <= 1e-6 * (float(pr.grad.abs().max()) + 1e-12) + 1e-9


def test_backward_is_deterministic():
    d, js = _case("train_s_4lvl_sum")
    m = _model(js["cfg"])
    x, tgt = torch.from_numpy(d["x"]).to(DEV), torch.from_numpy(d["target"]).to(DEV)
    grads = []
    for _ in range(2):
        m.zero_grad()
        L1LossForVideoFrames(**js["loss_kw"])(m(x), tgt).backward()
        grads.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]).clone())
    assert torch.equal(grads[0], grads[1])


def test_side_stream_backward_equals_serial_backward():
    """Conv3d weight / bias gradients run on a forked side stream beside the input gradient; the result
    must equal the one-stream backward (KDLAE_DEBUG=train_serial) bit for bit, at the KDLAES.yml batch
    shape (4 x 7 x 128^2) where the streams overlap."""
    m = _model(dict(residual=True, hidden_channels=[16, 32, 64]))
    x = torch.from_numpy(hash_images("side_s_x", (4, 7, 128, 128))).to(DEV)
    tgt = torch.from_numpy(hash_images("side_s_t", (4, 7, 128, 128))).to(DEV)
    old = os.environ.get("KDLAE_DEBUG")
    grads = []
    try:
        for flag in ("train_serial", None, None):
            if flag:
                os.environ["KDLAE_DEBUG"] = flag
            else:
                os.environ.pop("KDLAE_DEBUG", None)
            m.zero_grad()
            L1LossForVideoFrames()(m(x), tgt).backward()
            torch.cuda.synchronize()
            grads.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]).clone())
    finally:
        if old is None:
            os.environ.pop("KDLAE_DEBUG", None)
        else:
            os.environ["KDLAE_DEBUG"] = old
    assert torch.isfinite(grads[0]).all()
    assert torch.equal(grads[0], grads[1]) and torch.equal(grads[0], grads[2])


@pytest.mark.parametrize("hw", [192, 384])
def test_progressive_patch_sizes_train(hw):
    """KDLAES.yml's progressive patches (gt_sizes up to 384, batch 4, 7 frames; train.py:381-418): one
    step must run (finite loss and gradients) and the side-stream backward must equal the one-stream one
    bit for bit.  r04 refused every batch above ~621k pixels through a hard-coded column-matrix guard."""
    m = _model(dict(residual=True, hidden_channels=[16, 32, 64]))
    x = torch.from_numpy(hash_images(f"pp_x{hw}", (4, 7, hw, hw))).to(DEV)
    tgt = torch.from_numpy(hash_images(f"pp_t{hw}", (4, 7, hw, hw)))  # on the host: the trainer moves it
    old = os.environ.get("KDLAE_DEBUG")
    grads, losses = [], []
    try:
        for flag in ("train_serial", None):
            if flag:
                os.environ["KDLAE_DEBUG"] = flag
            else:
                os.environ.pop("KDLAE_DEBUG", None)
            m.zero_grad()
            loss = L1LossForVideoFrames()(m(x), tgt.to(DEV))
            loss.backward()
            torch.cuda.synchronize()
            losses.append(float(loss))
            grads.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]).clone())
    finally:
        if old is None:
            os.environ.pop("KDLAE_DEBUG", None)
        else:
            os.environ["KDLAE_DEBUG"] = old
    assert all(np.isfinite(losses)) and torch.isfinite(grads[0]).all()
    assert torch.equal(grads[0], grads[1])
    # the trainer path with a CPU target (it used to hand the kernel a host pointer)
    tr = KDLAESTrainer(m, lr=3e-4, weight_decay=1e-4, betas=(0.9, 0.99), max_norm=0.01)
    assert np.isfinite(float(tr.optimize_parameters(x, tgt)))


def test_unsupported_reduction_raises():
    with pytest.raises(NotImplementedError):
        L1LossForVideoFrames(reduction="max")(torch.zeros(1, 2, 4, 4, device=DEV), torch.zeros(1, 2, 4, 4, device=DEV))
