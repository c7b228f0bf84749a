"""Host-side §8f pieces: padded sizes, ASDQE statistics / CSV, checkpoint ingest (no GPU)."""
import csv
import os

import numpy as np
import pytest
import torch

from oracle.pipeline_oracle import calculate_statistics, notebook_pad
from rethink_acoustic_image_enhancement_amd.ASDQE_model import DenoiseRatePredictor
from rethink_acoustic_image_enhancement_amd.checkpoint import load_checkpoint, read_state_dict
from rethink_acoustic_image_enhancement_amd.hashweights import load_hash_weights
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_student, KDLAE_teacher
from rethink_acoustic_image_enhancement_amd.pipeline import padded_size, score_statistics, write_statistics_csv


@pytest.mark.parametrize("h,w", [(658, 438), (512, 512), (7, 9), (17, 8), (1, 16)])
def test_padded_size_matches_notebook(h, w):
    if h < 2 or w < 2:
        assert padded_size(h, w)[0] == (8 if h % 8 else h)
        return
    ref = notebook_pad(torch.zeros(1, 3, h, w)) if (h % 8 == 0 or (-h) % 8 < h) and (w % 8 == 0 or (-w) % 8 < w) else None
    H, W = padded_size(h, w)
    if ref is not None:
        assert (H, W) == tuple(ref.shape[2:])


def test_statistics_and_csv(tmp_path):
    rng = np.random.default_rng(0)
    vals = {m: rng.uniform(-1, 1, 37).astype(np.float32) for m in ("origin", "Teacher", "Student@0.05")}
    stats = {m: score_statistics(v) for m, v in vals.items()}
    for m, v in vals.items():
        ref = calculate_statistics(v)
        for k in ref:
            assert abs(stats[m][k] - float(ref[k])) <= 1e-6 * max(1.0, abs(float(ref[k])))
    p = tmp_path / "stats_transposed.csv"
    write_statistics_csv(stats, str(p))
    rows = list(csv.reader(open(p)))
    assert rows[0] == ["", "origin", "Teacher", "Student@0.05"]
    assert [r[0] for r in rows[1:]] == ["mean", "std", "min", "25%", "50%", "75%", "max"]
    assert rows[1][1] == f"{stats['origin']['mean']:.6f}"


def test_checkpoint_basicsr_layout(tmp_path):
    src = KDLAE_teacher(dim=16, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, LayerNorm_type="BiasFree")
    load_hash_weights(src)
    sd = src.state_dict()
    ema = {k: v + 1 for k, v in sd.items()}
    # save_network: {'params': sd, 'params_ema': ...} with 'module.' prefixes (DDP-wrapped nets)
    torch.save({"params": {"module." + k: v for k, v in sd.items()}, "params_ema": ema}, tmp_path / "net.pth")
    dst = KDLAE_teacher(dim=16, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, LayerNorm_type="BiasFree")
    assert load_checkpoint(dst, str(tmp_path / "net.pth")) == ([], [])
    assert all(torch.equal(dst.state_dict()[k], sd[k]) for k in sd)
    load_checkpoint(dst, str(tmp_path / "net.pth"), param_key="params_ema")
    assert all(torch.equal(dst.state_dict()[k], ema[k]) for k in sd)
    # static="train" checkpoint into static="no" fails strictly, as in the reference
    other = KDLAE_teacher(dim=16, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, LayerNorm_type="BiasFree",
                          static="no")
    with pytest.raises(RuntimeError):
        load_checkpoint(other, str(tmp_path / "net.pth"))
    miss, unexp = load_checkpoint(other, str(tmp_path / "net.pth"), strict=False)
    assert not miss and any(k.startswith("cen.") for k in unexp)


def test_checkpoint_raw_state_dicts(tmp_path):
    a = DenoiseRatePredictor()
    load_hash_weights(a)
    torch.save(a.state_dict(), tmp_path / "ASDQE.pth")           # raw sd (Train/ASDQE.py), strict=False load
    b = DenoiseRatePredictor()
    assert load_checkpoint(b, str(tmp_path / "ASDQE.pth"), strict=False) == ([], [])
    assert torch.equal(b.state_dict()["unet.up3.conv.double_conv.4.running_var"],
                       a.state_dict()["unet.up3.conv.double_conv.4.running_var"])
    s = KDLAE_student(residual=True)
    torch.save({"params": s.state_dict()}, tmp_path / "KDLAE-S.pth")
    assert set(read_state_dict(str(tmp_path / "KDLAE-S.pth"))) == set(s.state_dict())
    torch.save({"something": 3}, tmp_path / "bad.pth")
    with pytest.raises(RuntimeError):
        read_state_dict(str(tmp_path / "bad.pth"))


def test_frames_oracle_pinned_by_camus_fixture():
    """KDLAE-S.ipynb cell on the reference's own CAMUS frames (tests/golden/frames_camus7.npz): the
    oracle's load_consecutive_stack + pad-to-32 + student forward reproduces the reference module's
    output; COLOR_BGR2GRAY is the identity on these gray-as-BGRA frames (and on any R = G = B)."""
    from oracle.kdlae_oracle import StudentCfg, student_forward, student_param_shapes
    from oracle.pipeline_oracle import bgr2gray_u8, load_consecutive_stack, notebook_pad
    from tests.util import hash_sd_for, load_fixture

    d, kw = load_fixture("frames_camus7")
    frames = d["frames"]
    x = load_consecutive_stack(list(frames))
    assert torch.equal(x[0], torch.from_numpy(frames[..., 0].astype(np.float32) / 255.0))
    v = np.arange(256, dtype=np.uint8)
    assert np.array_equal(bgr2gray_u8(np.stack([v, v, v], -1)), v)
    xp = notebook_pad(x, 32)
    assert tuple(xp.shape) == (1, 7, 96, 64)
    cfg = StudentCfg(**kw)
    with torch.no_grad():
        y = student_forward(hash_sd_for(student_param_shapes(cfg)), xp, cfg)
    assert float((y - torch.from_numpy(d["restored"])).abs().max()) <= 1e-5


def test_asdqe_statistics_and_csv_match_the_script(tmp_path):
    """ASDQE_test.py calculate_statistics + visualize_comparison's CSV (pandas, float_format %.6f),
    from the fixture the script's own code path wrote (tests/golden/asdqe_scoring_mdd.npz)."""
    import json

    from oracle.asdqe_oracle import AsdqeCfg, asdqe_forward, asdqe_param_shapes
    from rethink_acoustic_image_enhancement_amd.pipeline import score_statistics, write_statistics_csv
    from tests.util import hash_sd_for, load_fixture

    d, kw = load_fixture("asdqe_scoring_mdd")
    methods = json.loads(bytes(d["methods"]).decode())
    stats = {m: score_statistics(d["pred_" + m]) for m in methods}
    write_statistics_csv(stats, str(tmp_path / "stats.csv"))
    assert (tmp_path / "stats.csv").read_text() == bytes(d["csv"]).decode()
    # the oracle reproduces the script's predictions from the same u8 pairs (ToTensor = /255)
    cfg = AsdqeCfg(**kw)
    sd = hash_sd_for(asdqe_param_shapes(cfg))
    t = lambda a: torch.from_numpy(a.astype(np.float32) / 255.0).permute(0, 3, 1, 2)  # noqa: E731
    with torch.no_grad():
        p = asdqe_forward(sd, t(d["lq"]), t(d["gt_Teacher"]), cfg).numpy().reshape(-1)
    assert np.abs(p - d["pred_Teacher"]).max() <= 1e-6
