"""KDLAE-T training step, CPU side: the training oracle against the reference
goldens, the training handle's flat-buffer layout against the module's parameters, workspace
sizing, and the DDP gradient sync over gloo (world size 2).  No GPU compute here.

Tolerances: loss 1e-6 relative; gradients 1e-4 of the tensor's max |g| (fp32, different reduction
order than oneDNN); parameters after two AdamW steps 2e-6 absolute on the delta (lr 1e-3).
"""
import ctypes
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle.kdlae_oracle import TeacherCfg, teacher_param_shapes
from oracle.train_oracle import TrainStep, l1sr_loss, loss_and_grads
from rethink_acoustic_image_enhancement_amd import _lib
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_teacher
from rethink_acoustic_image_enhancement_amd.train import sync_gradients
from tests.util import GOLDEN, hash_sd_for

CASES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith("train_") and not f.startswith("train_s_"))


def load_train_case(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    cfg = json.loads(bytes(d["cfg"]).decode())
    opt = json.loads(bytes(d["opt"]).decode())
    keys = json.loads(bytes(d["keys"]).decode())
    return d, cfg, opt, keys


def case_inputs(d):
    img = torch.from_numpy(d["img"])
    rate = torch.from_numpy(d["rate"])
    gt = {"hq": torch.from_numpy(d["gt_hq"]), "sr": torch.from_numpy(d["gt_sr"])}
    return img, rate, gt


def test_golden_cases_present():
    assert len(CASES) >= 3


@pytest.mark.parametrize("name", CASES)
def test_oracle_grads_match_reference(name):
    d, cfg, opt, keys = load_train_case(name)
    tc = TeacherCfg(**cfg)
    sd = hash_sd_for(teacher_param_shapes(tc))
    assert set(sd) == set(keys)
    sd = {k: sd[k] for k in keys}
    img, rate, gt = case_inputs(d)
    if tc.static != "train":
        gt = {"hq": gt["hq"]}
    loss, grads = loss_and_grads(sd, img, rate, gt, tc)
    assert abs(float(loss) - d["loss"][0]) <= 1e-6 * abs(d["loss"][0])
    flat = torch.cat([grads[k].reshape(-1) for k in keys]).numpy()
    sub = d["grad1_sub"]
    assert np.abs(flat[::5] - sub).max() <= 1e-4 * np.abs(sub).max()
    sums = np.array([[grads[k].double().sum(), grads[k].double().abs().sum()] for k in keys])
    np.testing.assert_allclose(sums[:, 1], d["grad_sums"][:, 1], rtol=1e-4, atol=1e-9)


@pytest.mark.parametrize("name", CASES)
def test_oracle_two_adamw_steps_match_reference(name):
    d, cfg, opt, keys = load_train_case(name)
    tc = TeacherCfg(**cfg)
    sd = hash_sd_for(teacher_param_shapes(tc))
    sd = {k: sd[k] for k in keys}
    img, rate, gt = case_inputs(d)
    if tc.static != "train":
        gt = {"hq": gt["hq"]}
    st = TrainStep(sd, tc, lr=opt["lr"], weight_decay=opt["weight_decay"], betas=tuple(opt["betas"]),
                   clip=opt["clip"])
    losses, norms = [], []
    for _ in range(2):
        loss, norm = st.step(img, rate, gt)
        losses.append(float(loss))
        norms.append(float(norm))
    np.testing.assert_allclose(losses, d["loss"], rtol=1e-6)
    np.testing.assert_allclose(norms, d["norm"], rtol=1e-5)
    p0 = torch.cat([sd[k].reshape(-1).double() for k in keys])
    p2 = torch.cat([st.state_dict()[k].reshape(-1).double() for k in keys])
    delta = (p2 - p0).numpy()[::5]
    assert np.abs(delta - d["delta2_sub"]).max() <= 2e-6


def test_l1sr_restatement():
    """losses.py:159-170 on hand-checkable values."""
    pred = {"hq": torch.tensor([[[[0.0, 0.5], [0.2, 1.0]]]]), "sr": None}
    tgt = {"hq": torch.tensor([[[[0.05, 0.3], [0.2, 0.0]]]])}
    # l1 = (0.05 + 0.2 + 0 + 1.0) / 4 = 0.3125; shadow: bins (0,1,1,1) vs (0,1,1,0) -> 0.25
    loss = l1sr_loss(pred, tgt)
    assert abs(float(loss) - (0.5 * 0.3125 + 0.25 * 0.25)) < 1e-7


def _tt_handle(m):
    L = _lib.lib()
    h = ctypes.c_void_p()
    _lib.check(L.kdlae_tt_create(ctypes.byref(m._c_config()), 0, ctypes.byref(h)), "kdlae_tt_create")
    return L, h


@pytest.mark.parametrize("kw", [
    dict(LayerNorm_type="BiasFree"),  # the released KDLAET.yml config
    dict(dim=16, num_blocks=[1, 2, 1, 1], num_refinement_blocks=1, LayerNorm_type="WithBias", bias=True),
    dict(dim=16, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, static="no", params="plus"),
])
def test_training_handle_layout_matches_module(kw):
    m = KDLAE_teacher(**kw)
    L, h = _tt_handle(m)
    try:
        named = list(m.named_parameters())
        assert L.kdlae_tt_num_params(h) == len(named)
        off_expect = 0
        for i, (k, p) in enumerate(named):
            name, numel, off = ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_int64()
            assert L.kdlae_tt_param_info(h, i, ctypes.byref(name), ctypes.byref(numel), ctypes.byref(off)) == 0
            assert name.value.decode() == k and numel.value == p.numel() and off.value == off_expect
            off_expect += (p.numel() + 3) // 4 * 4  # each key 16-byte aligned
        assert L.kdlae_tt_num_floats(h) == off_expect
        # workspace for the KDLAET.yml patch setting (6 x 128^2) and a ragged-size rejection
        nb = L.kdlae_tt_workspace_bytes(h, 6, 128, 128)
        assert 0 < nb < 64 << 30
        assert L.kdlae_tt_workspace_bytes(h, 1, 36, 40) == -1
    finally:
        L.kdlae_tt_destroy(h)


def test_training_handle_rejects_dual_pixel():
    m = KDLAE_teacher(dim=16, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1)
    cfg = m._c_config()
    cfg.dual_pixel_task = 1
    L = _lib.lib()
    h = ctypes.c_void_p()
    assert L.kdlae_tt_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ddp_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.arange(10, dtype=torch.float32) * (rank + 1)
    scale = sync_gradients(g)
    q.put((rank, scale, (g * scale).tolist()))
    dist.destroy_process_group()


def test_sync_gradients_gloo_world2():
    """One all-reduce over the flat gradient buffer; the returned scale turns the sum into DDP's mean."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    mean = (np.arange(10) * 1 + np.arange(10) * 2) / 2.0
    for rank, scale, vals in res:
        assert scale == 0.5
        np.testing.assert_allclose(vals, mean)


def test_grad_buckets_cover_the_buffer():
    """DDP-style buckets from gradient-ready marks: contiguous, back to front, exactly [0, numel), each
    closed by a mark whose suffix contains it, merged up to the cap."""
    from rethink_acoustic_image_enhancement_amd.train import grad_buckets
    marks = [990, 950, 900, 700, 690, 400, 120, 0]
    for cap in (1, 30, 100, 250, 5000):
        bk = grad_buckets(marks, 1000, cap)
        hi = 1000
        for j, lo, b_hi in bk:
            assert b_hi == hi and lo < b_hi
            if j is not None:
                assert marks[j] <= lo  # the mark's final suffix covers the bucket
            hi = lo
        assert hi == 0
        assert all(b_hi - lo >= cap for j, lo, b_hi in bk[:-1])
    assert grad_buckets(marks, 1000, 1) == [(j, lo, hi) for j, (lo, hi) in
                                            enumerate(zip(marks, [1000] + marks[:-1]))]
    # a backward whose last mark does not reach offset 0: the remainder waits for the whole backward
    assert grad_buckets([800, 300], 1000, 100)[-1] == (None, 0, 300)


def _bucket_worker(rank, world, port, q):
    import torch.distributed as dist

    from rethink_acoustic_image_enhancement_amd.train import grad_buckets, sync_gradients_bucketed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(rank)
    grad = torch.randn(1000, generator=g)
    full = grad.clone()
    dist.all_reduce(full)
    bk = grad_buckets([990, 950, 900, 700, 690, 400, 120, 0], 1000, 100)
    scale = sync_gradients_bucketed(grad, bk)
    q.put((rank, scale, bool(torch.equal(grad, full)), len(bk)))
    dist.destroy_process_group()


def test_sync_gradients_bucketed_gloo_world2():
    """Bucket-by-bucket all-reduce over gloo equals one all-reduce of the whole buffer, bit for bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, scale, same, nb in res:
        assert scale == 0.5 and same and nb > 1


def test_sync_gradients_single_process_is_identity():
    g = torch.ones(4)
    assert sync_gradients(g) == 1.0
    assert torch.equal(g, torch.ones(4))


def test_lr_schedule_matches_reference_scheduler():
    """KDLAET.yml train.scheduler: CosineAnnealingRestartCyclicLR values produced by the reference's
    own scheduler (tests/golden/lr_kdlaet.json, make_golden.py lr_goldens) at the lr BasicSR has in
    force at each iteration (scheduler stepped from iteration 2 on, base_model.py:183-193)."""
    import json
    import types

    from rethink_acoustic_image_enhancement_amd.train import CosineAnnealingRestartCyclicLR, KDLAETrainer
    from tests.util import GOLDEN

    with open(os.path.join(GOLDEN, "lr_kdlaet.json")) as f:
        g = json.load(f)
    sch = CosineAnnealingRestartCyclicLR(g["base_lr"], **g["scheduler"])
    fake = types.SimpleNamespace(scheduler=sch, init_lr=g["base_lr"], lr=g["base_lr"])
    for it, want in g["lr_at_iter"].items():
        got = KDLAETrainer.update_learning_rate(fake, int(it))
        assert abs(got - want) <= 1e-12 + 1e-9 * abs(want), (it, got, want)
    # linear warm-up (base_model.py:194-205) when warmup_iter > current_iter
    fake2 = types.SimpleNamespace(scheduler=None, init_lr=1e-4, lr=1e-4)
    assert abs(KDLAETrainer.update_learning_rate(fake2, 5, warmup_iter=10) - 5e-5) < 1e-15
