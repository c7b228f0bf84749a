"""bench.py --gpus N launches N rank processes itself.

Rehearsed on the CPU with the gloo backend and bench.py's stand-in forward (--cpu-standin): the
launcher, the contiguous rank shards of the synthetic T16 batch, the max-over-ranks timing and the
all-gather are the code the GPU run takes; only the forward and the backend differ.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_gpus_n_runs_n_ranks(n):
    steps, B = 3, 4
    p = _bench("--gpus", str(n), "--cpu-standin", "--steps", str(steps), "--warmup", "1", "--batch", str(B),
               "--size", "16")
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 alone prints
    res = json.loads(lines[0])
    assert res["n_gpus"] == n and res["config"]["global_batch"] == n * B
    ranks = sorted(res["standin"]["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == list(range(n))
    # disjoint contiguous shards covering images 0 .. n*B-1 in rank order
    covered = [i for r in ranks for i in range(r["first"], r["last"] + 1)]
    assert covered == list(range(n * B))
    # the all-gather reassembles the single-process batch
    assert res["standin"]["gather_equal"]
    # max over ranks: rank n-1 sleeps 0.01*(n-1) s per step, and the reported time covers it
    assert res["elapsed_s"] >= max(r["local_s"] for r in ranks) - 1e-6
    assert res["elapsed_s"] >= steps * 0.01 * (n - 1)
    assert abs(res["value"] - n * B * steps / res["elapsed_s"]) <= 1e-3 * res["value"] + 1e-3


def test_config5_width_under_torchrun():
    """Config 5's width (KDLAE-T bs=128 over 8 ranks, 16 per rank; Train/train.sh:5) launched the way the
    driver launches the scaling bench: torch.distributed.run --nproc-per-node 8, gloo stand-in.  The
    gather must reassemble images 0..127 in rank order."""
    n, B, steps = 8, 16, 2
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                        "--master-addr", "127.0.0.1", "--master-port", "29561", os.path.join(ROOT, "bench.py"),
                        "--gpus", str(n), "--cpu-standin", "--steps", str(steps), "--warmup", "1", "--batch", str(B),
                        "--size", "8"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == n and res["config"]["global_batch"] == 128 and res["config"]["per_gpu_batch"] == 16
    ranks = sorted(res["standin"]["ranks"], key=lambda r: r["rank"])
    assert [(r["first"], r["last"]) for r in ranks] == [(16 * i, 16 * i + 15) for i in range(n)]
    assert res["standin"]["gather_equal"]
    assert res["elapsed_s"] >= steps * 0.01 * (n - 1)


def test_gpus_n_fails_without_enough_devices():
    """No GPU here: --gpus 2 must exit non-zero instead of reporting n_gpus 1."""
    p = _bench("--gpus", "2", "--steps", "1", "--warmup", "0", timeout=120)
    assert p.returncode != 0
    assert "needs 2 visible GPUs" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_standin_single_rank_matches_contract():
    p = _bench("--cpu-standin", "--steps", "2", "--warmup", "0", "--batch", "3", "--size", "8")
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert res["n_gpus"] == 1 and res["config"]["global_batch"] == 3 and res["standin"]["gather_equal"]
