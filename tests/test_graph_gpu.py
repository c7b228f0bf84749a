"""HIP-graph capture of the drop-in forward (torch.cuda.graph over the C-ABI launches).

Every launch of ``kdlae_t_forward`` (and of the per-forward weight pack program) goes on the caller's
stream with no host synchronisation, allocation or copy inside the forward, so a caller can capture
the module once and replay it: the replay must equal the eager forward bit for bit, follow new
contents of the static input buffers, and — because the pack program re-reads the live parameter
storages — follow in-place weight updates (BasicSR's ``model_ema`` style ``p.data`` writes) too.
KDLAE-S and ASDQE are captured the same way.
"""
import pytest
import torch

from oracle.kdlae_oracle import TeacherCfg, teacher_forward
from rethink_acoustic_image_enhancement_amd.ASDQE_model import DenoiseRatePredictor
from rethink_acoustic_image_enhancement_amd.hashweights import hash_images, load_hash_weights
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_student, KDLAE_teacher
from tests.util import max_abs

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _capture(fn, *static):
    """Warm up on a side stream (workspace and kernel attributes set outside capture), then capture."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.no_grad():
        for _ in range(2):
            fn(*static)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g), torch.no_grad():
        out = fn(*static)
    return g, out


def test_teacher_graph_replay_bit_exact_and_live():
    kw = dict(dim=48, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, LayerNorm_type="BiasFree")
    m = KDLAE_teacher(**kw)
    load_hash_weights(m)
    m = m.to(DEV).eval()
    img = torch.from_numpy(hash_images("graph_a", (2, 3, 64, 48))).to(DEV)
    rate = torch.full((2, 1, 64, 48), 0.6, device=DEV)
    s_img, s_rate = img.clone(), rate.clone()
    g, out = _capture(lambda a, b: m({"img": a, "denoise_rate": b}), s_img, s_rate)
    g.replay()
    torch.cuda.synchronize()
    with torch.no_grad():
        ref = m({"img": img, "denoise_rate": rate})
    assert torch.equal(out["hq"], ref["hq"]) and torch.equal(out["sr"], ref["sr"])
    # new input contents through the static buffers
    img2 = torch.from_numpy(hash_images("graph_b", (2, 3, 64, 48))).to(DEV)
    s_img.copy_(img2)
    s_rate.fill_(0.3)
    g.replay()
    torch.cuda.synchronize()
    with torch.no_grad():
        ref2 = m({"img": img2, "denoise_rate": torch.full_like(rate, 0.3)})
    assert torch.equal(out["hq"], ref2["hq"]) and torch.equal(out["sr"], ref2["sr"])
    # in-place weight update without a version bump: the replayed pack program sees it
    with torch.no_grad():
        for p in m.parameters():
            p.data.mul_(0.75)
    g.replay()
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    want = teacher_forward(sd, img2.cpu(), torch.full((2, 1, 64, 48), 0.3), TeacherCfg(**kw))
    e = max(max_abs(out["hq"].cpu(), want["hq"]), max_abs(out["sr"].cpu(), want["sr"]))
    print(f"graph replay after p.data.mul_: max-abs vs oracle {e:.3e}")
    assert e <= 1e-3


def test_student_and_asdqe_graph_replay():
    sm = KDLAE_student(residual=True, hidden_channels=[16, 32, 64])
    load_hash_weights(sm)
    sm = sm.to(DEV).eval()
    x = torch.from_numpy(hash_images("graph_s", (2, 4, 32, 32))).to(DEV)
    sx = x.clone()
    g, y = _capture(sm, sx)
    g.replay()
    torch.cuda.synchronize()
    with torch.no_grad():
        assert torch.equal(y, sm(x))
    am = DenoiseRatePredictor()
    load_hash_weights(am)
    am = am.to(DEV).eval()
    lq = torch.from_numpy(hash_images("graph_lq", (2, 3, 40, 40))).to(DEV)
    gt = torch.from_numpy(hash_images("graph_gt", (2, 3, 40, 40))).to(DEV)
    slq, sgt = lq.clone(), gt.clone()
    g2, score = _capture(am, slq, sgt)
    g2.replay()
    torch.cuda.synchronize()
    with torch.no_grad():
        assert torch.equal(score, am(lq, gt))


def test_module_replays_its_own_graph_for_repeated_shapes():
    """KDLAE_teacher.hip_graphs (default): the second call of a shape captures, later calls replay.
    Replayed outputs equal the launch-by-launch forward bit for bit, follow new inputs and in-place
    weight updates, are fresh tensors (no aliasing between calls), and survive a workspace regrowth
    (a larger shape reallocates the workspace: the stale graph must be re-captured, not replayed)."""
    kw = dict(dim=48, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, LayerNorm_type="BiasFree")
    m = KDLAE_teacher(**kw)
    load_hash_weights(m)
    m = m.to(DEV).eval()
    assert m.hip_graphs

    def run(img, rate, graphs=True):
        m.hip_graphs = graphs
        with torch.no_grad():
            out = m({"img": img, "denoise_rate": rate})
        m.hip_graphs = True
        return out

    img = torch.from_numpy(hash_images("mg_a", (1, 3, 64, 48))).to(DEV)
    rate = torch.full((1, 1, 64, 48), 0.6, device=DEV)
    ref = run(img, rate, graphs=False)
    outs = [run(img, rate) for _ in range(3)]  # eager, capture, replay
    assert len(m._graphs) == 1
    for o in outs:
        assert torch.equal(o["hq"], ref["hq"]) and torch.equal(o["sr"], ref["sr"])
    assert outs[1]["hq"].data_ptr() != outs[2]["hq"].data_ptr()
    img2 = torch.from_numpy(hash_images("mg_b", (1, 3, 64, 48))).to(DEV)
    o2 = run(img2, torch.full_like(rate, 0.3))
    assert torch.equal(o2["hq"], run(img2, torch.full_like(rate, 0.3), graphs=False)["hq"])
    assert torch.equal(outs[2]["hq"], ref["hq"])  # an earlier result is untouched by the replay
    with torch.no_grad():
        for p in m.parameters():
            p.data.mul_(0.9)
    o3 = run(img2, torch.full_like(rate, 0.3))
    assert torch.equal(o3["sr"], run(img2, torch.full_like(rate, 0.3), graphs=False)["sr"])
    # a larger shape regrows the workspace; the 64x48 graph must not replay into the freed buffer
    big = torch.from_numpy(hash_images("mg_c", (2, 3, 96, 96))).to(DEV)
    brate = torch.full((2, 1, 96, 96), 0.5, device=DEV)
    for _ in range(3):
        ob = run(big, brate)
    assert torch.equal(ob["hq"], run(big, brate, graphs=False)["hq"])
    o4 = run(img2, torch.full_like(rate, 0.3))
    assert torch.equal(o4["hq"], run(img2, torch.full_like(rate, 0.3), graphs=False)["hq"])


def test_implicit_capture_tolerates_other_threads():
    """The module's implicit capture (second call of a shape) uses thread-local capture mode: another
    thread of the process that allocates pinned host memory and copies it to the device meanwhile (a
    DataLoader pin_memory thread, an async checkpoint copy) must neither fail nor be captured."""
    import threading

    kw = dict(dim=48, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, LayerNorm_type="BiasFree")
    m = KDLAE_teacher(**kw)
    load_hash_weights(m)
    m = m.to(DEV).eval()
    img = torch.from_numpy(hash_images("mt_a", (1, 3, 64, 64))).to(DEV)
    rate = torch.full((1, 1, 64, 64), 0.6, device=DEV)
    with torch.no_grad():
        ref = m({"img": img, "denoise_rate": rate})  # eager: the next call of this shape captures
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    stop, errors, copies = threading.Event(), [], [0]

    def worker():
        n = 1 << 14
        try:
            while not stop.is_set():
                n = n + 4096 if n < (1 << 20) else 1 << 14  # new sizes: fresh pinned allocations
                h = torch.empty(n, pin_memory=True).fill_(1.0)
                with torch.cuda.stream(side):  # every device call of this thread on its own stream
                    d = h.to(DEV, non_blocking=True)
                    back = d[-1:].to("cpu", non_blocking=True)
                side.synchronize()
                assert float(back[0]) == 1.0
                copies[0] += 1
        except Exception as e:  # noqa: BLE001 (reported by the main thread)
            errors.append(repr(e))

    t = threading.Thread(target=worker)
    t.start()
    try:
        with torch.no_grad():
            outs = [m({"img": img, "denoise_rate": rate}) for _ in range(3)]  # capture, replay, replay
        torch.cuda.synchronize()
    finally:
        stop.set()
        t.join(timeout=60)
    assert not errors, errors
    assert copies[0] > 0
    assert len(m._graphs) == 1, "the shape should have been captured"
    for o in outs:
        assert torch.equal(o["hq"], ref["hq"]) and torch.equal(o["sr"], ref["sr"])
