"""GPU parity of the HIP KDLAE-T path (through the C ABI) against the oracle and the goldens.

Tolerance: 1e-3 fp32 max-abs on hq and sr (BASELINE.json north_star).  Every test here runs on
cuda:0 and calls KDLAE_teacher.forward -> libkdlae.so; there is no fallback path to hide behind.
"""
import glob
import json
import os

import numpy as np
import pytest
import torch

from oracle.kdlae_oracle import TeacherCfg, psnr, teacher_forward, teacher_param_shapes
from rethink_acoustic_image_enhancement_amd.hashweights import hash_images, load_hash_weights
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_teacher
from tests.util import GOLDEN, hash_sd_for, load_fixture, max_abs, mdd_input_tensor

pytestmark = pytest.mark.gpu
TOL = 1e-3
DEV = "cuda:0"

TEACHER = sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, "t_*.npz"))
                 if "_512" not in f)


def _model(kw):
    m = KDLAE_teacher(**kw)
    load_hash_weights(m)
    return m.to(DEV).eval()


def _run(m, img, rate):
    with torch.no_grad():
        out = m({"img": img.to(DEV), "denoise_rate": rate.to(DEV)})
    torch.cuda.synchronize()
    return {k: (v.cpu() if v is not None else None) for k, v in out.items()}


@pytest.mark.parametrize("name", TEACHER)
def test_golden_fixture(name):
    d, kw = load_fixture(name)
    out = _run(_model(kw), torch.from_numpy(d["img"]), torch.from_numpy(d["rate"]))
    e_hq = max_abs(out["hq"], torch.from_numpy(d["hq"]))
    print(f"{name}: hq max-abs {e_hq:.3e}")
    assert e_hq <= TOL, f"hq max-abs {e_hq}"
    if "sr" in d:
        e_sr = max_abs(out["sr"], torch.from_numpy(d["sr"]))
        assert e_sr <= TOL, f"sr max-abs {e_sr}"
    else:
        assert out["sr"] is None


def _run_512(name, img):
    d, kw = load_fixture(name)
    out = _run(_model(kw), img, torch.full((1, 1, 512, 512), 0.6))
    sub = {"hq": out["hq"][:, :, ::8, ::8], "sr": out["sr"][:, :, ::8, ::8],
           "hq_row": out["hq"][:, :, 257, :], "sr_row": out["sr"][:, :, 515, :]}
    return d, out, sub


def test_rand_512_full_size():
    """KDLAE-T at the benchmark resolution (1x3x512x512, hash-uniform image): 1e-3 vs the
    reference fp32 outputs (subsample, two full rows, channel sums)."""
    d, _ = load_fixture("t_rand_512")
    from rethink_acoustic_image_enhancement_amd.hashweights import hash_images as hi
    img = torch.from_numpy(hi("img:t_rand_512", (1, 3, 512, 512)))
    d, out, sub = _run_512("t_rand_512", img)
    for k, ref in (("hq", "hq_sub"), ("sr", "sr_sub"), ("hq_row", "hq_row257"), ("sr_row", "sr_row515")):
        e = max_abs(sub[k], torch.from_numpy(d[ref]))
        print(f"t_rand_512 {k}: max-abs {e:.3e}")
        assert e <= TOL, (k, e)
    np.testing.assert_allclose(out["hq"].double().sum(dim=(2, 3)).numpy(), d["hq_chsum"], rtol=1e-5)
    np.testing.assert_allclose(out["sr"].double().sum(dim=(2, 3)).numpy(), d["sr_chsum"], rtol=1e-5)


def test_mdd_512_config1():
    """Config 1 (MDD sonar sample 512x512, denoise_rate 0.6), judged against the reference's fp64 output.

    On this input the forward is ill-conditioned: every fp32 evaluation of it is a draw from a spread
    of errors.  The reference's own fp32 forward lands 3.1e-3 / 1.2e-3 / 7.5e-4 / 4.0e-3 (hq) from fp64
    at torch thread counts 8 / 4 / 2 / 1 (nothing else changed) and the other thread counts are 1.9e-3
    .. 8.6e-3 away from its default (8-thread) output (profiles/r04_config1_threads.txt); multiplying its
    LayerNorm outputs by (1 + u 2^-24), u ~ U[-1, 1], gives 1.0e-3 .. 2.4e-3 over 8 seeds
    (profiles/r04_config1_ensemble.txt).  The bar, per output (hq, sr) over every fixture sample (the
    [::8, ::8] subsample plus one full row), against the reference run the fixture holds (torch fp32,
    8 threads, its default):
      * ours is no farther from fp64 than the reference fp32 is, in max-abs and in mean-abs error;
      * PSNR >= 60 dB against the reference fp32.
    No bar is put on ours-vs-ref32 beyond the PSNR: a more accurate evaluation sits about as far from
    the reference fp32 output as that output is from fp64 (r06: one build of the opt-in fused MDTA
    kernel landed 4.7e-4 from fp64, 6.5x closer than the reference's own fp32 run, and 3.0e-3 from
    it).  r06 at the benched HEAD (profiles/r06_config1_mdd.txt): hq 2.71e-3 max / 1.82e-5 mean vs the
    reference's 3.07e-3 / 1.95e-5; sr 3.12e-3 / 1.66e-5 vs 3.40e-3 / 1.92e-5.  The 1e-3 bar against
    the reference fp32 holds on every well-conditioned input (all other fixtures, the 512^2 hash image
    included)."""
    d, _ = load_fixture("t_mdd_512")
    ens = json.load(open(os.path.join(GOLDEN, "t_mdd_512_ensemble.json")))
    thr = ens["ref32_threads"]
    d, out, sub = _run_512("t_mdd_512", mdd_input_tensor(d))
    for k, row, r32, r64, w32, w64 in (("hq", "hq_row", "hq_sub", "hq64_sub", "hq_row257", "hq64_row257"),
                                       ("sr", "sr_row", "sr_sub", "sr64_sub", "sr_row515", "sr64_row515")):
        ours = torch.cat([sub[k].double().flatten(), sub[row].double().flatten()])
        ref32 = torch.cat([torch.from_numpy(d[r32]).double().flatten(), torch.from_numpy(d[w32]).double().flatten()])
        ref64 = torch.cat([torch.from_numpy(d[r64]).double().flatten(), torch.from_numpy(d[w64]).double().flatten()])
        e_ours, e_ref = float((ours - ref64).abs().max()), float((ref32 - ref64).abs().max())
        m_ours, m_ref = float((ours - ref64).abs().mean()), float((ref32 - ref64).abs().mean())
        e_vs32 = float((ours - ref32).abs().max())
        print(f"t_mdd_512 {k}: ours-vs-fp64 max {e_ours:.3e} mean {m_ours:.3e}; ref32 (8 threads) max {e_ref:.3e} "
              f"mean {m_ref:.3e}; ref32 thread counts {thr['threads']}: {thr[k]}; perturbed-ref32 median "
              f"{ens[k + '_median']:.3e} (range {min(ens[k + '_max']):.3e} .. {max(ens[k + '_max']):.3e}); "
              f"ours-vs-ref32 max {e_vs32:.3e} (other ref32 thread counts vs 8 threads {thr[k + '_vs_8t'][1:]}); "
              f"PSNR vs ref32 {psnr(sub[k], torch.from_numpy(d[r32])):.1f} dB")
        assert e_ours <= e_ref, (k, e_ours, e_ref)
        assert m_ours <= m_ref, (k, m_ours, m_ref)
        assert psnr(sub[k], torch.from_numpy(d[r32])) >= 60.0


@pytest.mark.parametrize("kw,shape", [
    (dict(dim=48, LayerNorm_type="BiasFree", num_blocks=[1, 1, 1, 1], num_refinement_blocks=1), (3, 3, 64, 48)),
    (dict(dim=64, heads=[1, 1, 2, 4], num_blocks=[1, 1, 1, 1], num_refinement_blocks=1), (1, 3, 32, 40)),
    (dict(dim=32, heads=[1, 1, 2, 4], num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, bias=True), (2, 3, 40, 56)),
    (dict(dim=48, heads=[1, 2, 2, 4], num_blocks=[1, 1, 1, 2], num_refinement_blocks=2,
          LayerNorm_type="BiasFree", ffn_expansion_factor=2.0), (1, 3, 72, 32)),
    (dict(dim=32, heads=[1, 2, 4, 8], num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, params="mul",
          static="train"), (2, 3, 32, 32)),
    # dim 80: 5-tile patch_embed (a partial small-in tile group) and 160-wide output_param / cen (two
    # small-in passes of <= 128 outputs); C = 80 / 160 / 320 / 640 take the unfused FFN path
    (dict(dim=80, heads=[5, 5, 5, 5], num_blocks=[1, 1, 1, 1], num_refinement_blocks=1), (1, 3, 32, 32)),
])
def test_vs_oracle_random_configs(kw, shape):
    """Seeded hash weights/inputs at sizes the oracle finishes in seconds; every ctor branch."""
    cfg = TeacherCfg(**kw)
    sd = hash_sd_for(teacher_param_shapes(cfg))
    b, c, h, w = shape
    img = torch.from_numpy(hash_images(f"img{shape}", shape))
    rate = torch.from_numpy(hash_images(f"rate{shape}", (b, 1, h, w)))
    ref = teacher_forward(sd, img, rate, cfg)
    m = KDLAE_teacher(**kw)
    m.load_state_dict(sd)
    out = _run(m.to(DEV).eval(), img, rate)
    assert max_abs(out["hq"], ref["hq"]) <= TOL
    if ref["sr"] is not None:
        assert max_abs(out["sr"], ref["sr"]) <= TOL
        assert psnr(out["sr"], ref["sr"]) >= 60.0


def test_batch_invariance_and_determinism():
    """Size-independent properties: image i of a batch equals the same image alone, bit-exact,
    and two runs are bit-identical (fixed-order reductions, no float atomics)."""
    kw = dict(dim=48, LayerNorm_type="BiasFree", num_blocks=[2, 1, 1, 1], num_refinement_blocks=1)
    m = _model(kw)
    img = torch.from_numpy(hash_images("binv", (3, 3, 128, 96)))
    rate = torch.from_numpy(hash_images("binvr", (3, 1, 128, 96)))
    full = _run(m, img, rate)
    again = _run(m, img, rate)
    assert torch.equal(full["hq"], again["hq"]) and torch.equal(full["sr"], again["sr"])
    one = _run(m, img[1:2], rate[1:2])
    assert torch.equal(full["hq"][1:2], one["hq"]) and torch.equal(full["sr"][1:2], one["sr"])


@pytest.mark.parametrize("ln,split", [("BiasFree", False), ("WithBias", False), ("BiasFree", True), ("WithBias", True)])
def test_fused_attention_input_equals_unfused_bit_for_bit(ln, split, monkeypatch):
    """gemm_attn_in_kernel (x1 = x + M v, LN, project_in in one pass: the C = 48 blocks, and by default
    the C = 96 blocks' first project_in weight group) gives the same bits as the separate
    attention-output GEMM + LN/project_in GEMM it replaces (split=False: the C = 96 blocks unfused,
    KDLAE_DEBUG=no_attn_in_split)."""
    kw = dict(dim=48, LayerNorm_type=ln, num_blocks=[2, 1, 1, 1], num_refinement_blocks=1, bias=ln == "WithBias")
    img = torch.from_numpy(hash_images("fai", (2, 3, 64, 80)))
    rate = torch.from_numpy(hash_images("fair", (2, 1, 64, 80)))
    if not split:
        monkeypatch.setenv("KDLAE_DEBUG", "no_attn_in_split")
    fused = _run(_model(kw), img, rate)
    monkeypatch.setenv("KDLAE_DEBUG", "no_attn_in_fusion")  # read when a new handle builds its blocks
    unfused = _run(_model(kw), img, rate)
    assert torch.equal(fused["hq"], unfused["hq"]) and torch.equal(fused["sr"], unfused["sr"])


@pytest.mark.parametrize("ln,bias,shape", [
    ("BiasFree", False, (3, 3, 48, 64)),    # full tiles; 3 images per launch
    ("WithBias", True, (2, 3, 40, 56)),     # WithBias LN + conv biases; partial 16 x 8 tiles at the edges
    ("BiasFree", False, (1, 3, 72, 40)),    # ragged width (40 = 2.5 tiles) and height
])
def test_fused_ffn_equals_unfused_bit_for_bit(ln, bias, shape, monkeypatch):
    """ffn_fused_kernel (ffn.hip: LN + project_in recomputed on each tile's halo, dwconv + gate,
    project_out, residual; output to the other buffer of a ping-pong pair) gives the same bits as the
    unfused project_in GEMM + gdfn_out_kernel (KDLAE_DEBUG=no_ffn_fusion), for the C = 48 and C = 96
    stages (every stage here has an even block count, so all of them take the fused kernel)."""
    kw = dict(dim=48, LayerNorm_type=ln, num_blocks=[2, 2, 2, 2], num_refinement_blocks=2, bias=bias)
    img = torch.from_numpy(hash_images("ffnf", shape))
    rate = torch.from_numpy(hash_images("ffnfr", (shape[0], 1) + shape[2:]))
    fused = _run(_model(kw), img, rate)
    monkeypatch.setenv("KDLAE_DEBUG", "no_ffn_fusion")  # read when a new handle builds its blocks
    unfused = _run(_model(kw), img, rate)
    assert torch.equal(fused["hq"], unfused["hq"]) and torch.equal(fused["sr"], unfused["sr"])


@pytest.mark.parametrize("ln,bias,shape", [
    ("BiasFree", False, (2, 3, 64, 48)),    # whole 16 x 8 tiles, 2 images per launch
    ("WithBias", True, (1, 3, 72, 32)),     # WithBias LN + conv biases; 3 row segments of 24
])
def test_fused_mdta_matches_unfused(ln, bias, shape, monkeypatch):
    """mdta_fused_kernel (mdta_fused.hip, opt-in KDLAE_DEBUG=mdta_fusion: LN + qkv recomputed on each
    tile's halo, dwconv, Gram into the same slots) against the default qkv GEMM + Gram ring for the
    single-head C = 48 / 96 stages.  The Gram products run on split-bf16 MFMAs instead of the ring's
    f32 MFMA chain, so the two agree to fp32 rounding (1e-5 here), not bit for bit; both are held to
    the oracle at 1e-3 by the golden tests."""
    kw = dict(dim=48, LayerNorm_type=ln, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, bias=bias)
    img = torch.from_numpy(hash_images("mdf", shape))
    rate = torch.from_numpy(hash_images("mdfr", (shape[0], 1) + shape[2:]))
    unfused = _run(_model(kw), img, rate)
    monkeypatch.setenv("KDLAE_DEBUG", "mdta_fusion")  # read when a new handle builds its blocks
    fused = _run(_model(kw), img, rate)
    e_hq, e_sr = max_abs(fused["hq"], unfused["hq"]), max_abs(fused["sr"], unfused["sr"])
    print(f"fused vs unfused MDTA: hq {e_hq:.3e} sr {e_sr:.3e}")
    assert e_hq <= 1e-5 and e_sr <= 1e-5, (e_hq, e_sr)


def test_weight_reload_is_picked_up():
    kw = dict(dim=16, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1)
    m = _model(kw)
    img = torch.from_numpy(hash_images("wr", (1, 3, 16, 16)))
    rate = torch.full((1, 1, 16, 16), 0.5)
    a = _run(m, img, rate)["hq"]
    with torch.no_grad():
        m.output2.weight.mul_(2.0)
    b = _run(m, img, rate)["hq"]
    cfg = TeacherCfg(**kw)
    ref = teacher_forward({k: v.cpu() for k, v in m.state_dict().items()}, img, rate, cfg)
    assert not torch.equal(a, b)
    assert max_abs(b, ref["hq"]) <= TOL


def test_error_behaviour():
    m = _model(dict(dim=16, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1))
    with pytest.raises(RuntimeError):
        m({"img": torch.zeros(1, 3, 20, 24, device=DEV), "denoise_rate": torch.zeros(1, 1, 20, 24, device=DEV)})
    with pytest.raises(RuntimeError):
        m({"img": torch.zeros(1, 3, 16, 16), "denoise_rate": torch.zeros(1, 1, 16, 16)})
    with pytest.raises(KeyError):
        m({"img": torch.zeros(1, 3, 16, 16, device=DEV)})
    with pytest.raises(NotImplementedError):
        KDLAE_teacher(dim=16, dual_pixel_task=True).to(DEV)(
            {"img": torch.zeros(1, 3, 16, 16, device=DEV), "denoise_rate": torch.zeros(1, 1, 16, 16, device=DEV)})


def test_data_writes_bypassing_autograd_are_seen():
    """`.data` writes do not bump `_version`; BasicSR's model_ema (base_model.py:54-62)
    updates net_g_ema that way.  The HIP path repacks from the live parameters on every forward."""
    kw = dict(dim=16, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1)
    m = _model(kw)
    img = torch.from_numpy(hash_images("dw", (1, 3, 16, 24)))
    rate = torch.full((1, 1, 16, 24), 0.4)
    a = _run(m, img, rate)
    src = _model(kw)
    with torch.no_grad():
        for p in src.parameters():
            p.data.mul_(0.9)
        # model_ema(decay=0.5): net_g_ema.params.data.mul_(decay).add_(net_g.params.data, alpha=1 - decay)
        for pe, ps in zip(m.parameters(), src.parameters()):
            pe.data.mul_(0.5).add_(ps.data, alpha=0.5)
        m.output2.weight.data[0, 0, 1, 1] += 0.25
    b = _run(m, img, rate)
    assert not torch.equal(a["hq"], b["hq"])
    ref = teacher_forward({k: v.cpu() for k, v in m.state_dict().items()}, img, rate, TeacherCfg(**kw))
    assert max_abs(b["hq"], ref["hq"]) <= TOL and max_abs(b["sr"], ref["sr"]) <= TOL


def test_pack_device_rejects_wrong_size_and_host_commit_still_works():
    import ctypes

    from rethink_acoustic_image_enhancement_amd import _lib
    kw = dict(dim=16, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1)
    m = _model(kw)
    eng = m.engine(torch.device(DEV))
    L = _lib.lib()
    buf = torch.zeros(eng.numel + 1, device=DEV)
    assert L.kdlae_t_pack_device(eng.handle, ctypes.c_void_p(buf.data_ptr()), eng.numel + 1, None) == 4
    assert "expected" in _lib.last_error()
    # the host-staged path (set_param + commit) packs the same arena as the device path
    img = torch.from_numpy(hash_images("hc", (1, 3, 16, 16)))
    rate = torch.full((1, 1, 16, 16), 0.5)
    want = _run(m, img, rate)["hq"]
    for name, t in m.state_dict().items():
        host = t.detach().cpu().contiguous()
        _lib.check(L.kdlae_t_set_param(eng.handle, name.encode(), ctypes.c_void_p(host.data_ptr()), host.numel()), name)
    _lib.check(L.kdlae_t_commit_params(eng.handle, None), "commit")
    out = torch.empty(1, 3, 16, 16, device=DEV)
    sr = torch.empty(1, 3, 32, 32, device=DEV)
    ws = eng.workspace(L.kdlae_t_workspace_bytes(eng.handle, 1, 16, 16), torch.device(DEV))
    ic, rc = img.to(DEV).contiguous(), rate.to(DEV).contiguous()
    _lib.check(L.kdlae_t_forward(eng.handle, ctypes.c_void_p(ic.data_ptr()), ctypes.c_void_p(rc.data_ptr()), 1, 16, 16,
                                 ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(sr.data_ptr()),
                                 ctypes.c_void_p(ws.data_ptr()), ws.numel(), None), "forward")
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), want)
