"""The RCCL (torch "nccl" backend on ROCm) code paths of the multi-GPU build, executed on one GPU.

The GPU box has one MI355X, so these run a world of ONE rank: every collective is the identity, but
the calls are the ones an 8-GPU run makes ("the RCCL branches have never executed"):
* ``dist.init_process_group("nccl", device_id=...)`` as bench.py does for N > 1;
* ``shard.gather_outputs`` -> ``all_gather_into_tensor`` on device tensors (the §8e output gather),
  through ``sharded_forward`` on the real HIP module;
* ``train.allreduce_buckets_rccl``: the bucketed gradient all-reduce on the communication stream,
  each bucket enqueued behind its gradient-ready event (``kdlae_tt_mark_wait``) of a real marked
  backward; with one rank the SUM leaves every bucket unchanged, so the result must equal the
  unreduced gradient bit for bit.
The N-rank sharding / gather / reduction logic itself is covered by the gloo tests
(tests/test_shard.py, tests/test_train.py, tests/test_bench_launch.py).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist

from rethink_acoustic_image_enhancement_amd.hashweights import hash_images, load_hash_weights
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_teacher

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def rccl_world1():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(DEV)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=DEV)
    assert dist.get_backend() == "nccl"
    yield
    dist.destroy_process_group()


def test_rccl_output_gather_of_the_hip_module(rccl_world1):
    from rethink_acoustic_image_enhancement_amd.shard import gather_outputs, sharded_forward
    kw = dict(dim=48, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, LayerNorm_type="BiasFree")
    m = KDLAE_teacher(**kw)
    load_hash_weights(m)
    m = m.to(DEV).eval()
    img = torch.from_numpy(hash_images("rccl", (2, 3, 32, 48))).to(DEV)
    rate = torch.full((2, 1, 32, 48), 0.6, device=DEV)
    with torch.no_grad():
        ref = m({"img": img, "denoise_rate": rate})
        out = sharded_forward(m, {"img": img, "denoise_rate": rate}, gather=True)
    torch.cuda.synchronize()
    assert torch.equal(out["hq"], ref["hq"]) and torch.equal(out["sr"], ref["sr"])
    g = gather_outputs(ref["sr"])
    assert g.is_cuda and torch.equal(g, ref["sr"])


def test_rccl_overlapped_gather_of_the_hip_module(rccl_world1):
    """bench.py's N > 1 step on RCCL: each forward's hq / sr gather enqueued asynchronously on the
    collective stream while the next forward (HIP-graph replay) runs; after drain() every step's
    gathered output equals that step's local output bit for bit (world 1: the identity)."""
    from rethink_acoustic_image_enhancement_amd.shard import OverlappedGather
    kw = dict(dim=48, num_blocks=[1, 1, 1, 1], num_refinement_blocks=1, LayerNorm_type="BiasFree")
    m = KDLAE_teacher(**kw)
    load_hash_weights(m)
    m = m.to(DEV).eval()
    m.hip_graphs = True
    g = OverlappedGather(depth=2)
    outs, refs = [], []
    with torch.no_grad():
        for step in range(4):
            img = torch.from_numpy(hash_images(f"ovl{step}", (2, 3, 32, 48))).to(DEV)
            rate = torch.full((2, 1, 32, 48), 0.3 + 0.1 * step, device=DEV)
            o = m({"img": img, "denoise_rate": rate})
            refs.append({k: v.clone() for k, v in o.items()})
            outs.append(g(o))
            assert len(g.inflight) <= 2
        g.drain()
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        assert torch.equal(o["hq"], r["hq"]) and torch.equal(o["sr"], r["sr"])


def test_rccl_bucketed_allreduce_behind_gradient_events(rccl_world1):
    from rethink_acoustic_image_enhancement_amd.train import KDLAETrainer, allreduce_buckets_rccl
    m = KDLAE_teacher(LayerNorm_type="BiasFree")
    load_hash_weights(m)
    m = m.to(DEV)
    img = torch.from_numpy(hash_images("rccl_t", (2, 3, 64, 64))).to(DEV)
    rate = torch.full((2, 1, 64, 64), 0.6, device=DEV)
    gt = {"hq": img.clamp(0.2, 0.8), "sr": torch.nn.functional.interpolate(img, scale_factor=2).clamp(0.2, 0.8)}
    tr = KDLAETrainer(m)
    inp = {"img": img, "denoise_rate": rate}
    tr.forward_backward(inp, gt)
    want = tr.grad.clone()
    tr.forward_backward(inp, gt, marked=True)
    assert len(tr.buckets) >= 2 and tr.buckets[0][0] is not None
    allreduce_buckets_rccl(tr.grad, tr.buckets, tr.engine.handle)
    torch.cuda.synchronize()
    assert torch.equal(tr.grad, want)
