"""KDLAE-T forward throughput on MI355X (BASELINE.json configs[1] / configs[4]).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

`--gpus N` (N > 1) without a torchrun environment starts the N rank processes itself (one per GPU,
torch.distributed.run on 127.0.0.1, the reference's own launcher: Train/train.sh:5) before anything
touches the GPU, and exits non-zero when fewer than N devices are visible.

One step = one KDLAE-T forward (static="train": hq + sr, params="cat", BiasFree LN, fp32) of
16 synthetic 512x512 images per GPU (weak scaling: global batch 16*N, rank r owns images
[16r, 16r+16); for N > 1 the step ends with the RCCL all-gather of hq/sr).  Weights
are the deterministic hash recipe (random init of the real architecture), inputs are
hash-uniform images with per-image constant denoise_rate.

Printed JSON (rank 0): value = images/s over all ranks (max-over-ranks wall time of exactly K
steps between barriers + device syncs) of the module's default, un-instrumented forward (HIP-graph
replay); roofline of the dominant kernel class measured live with HIP events around each of its
launches in a separate probe pass of the same workload after the timed steps; cpu_baseline = the CPU oracle
(oracle/kdlae_oracle.py, test infrastructure) on one image of the same workload, 1 warm-up + the
median of 3 timed runs, whose output also gives the PSNR / max-abs of the GPU result
(rank 0, N=1 only).  The same line carries BASELINE configs[2] (KDLAE-S S8) and configs[3]
(ASDQE A64) under "s8" / "a64", each with its own value, roofline, cpu_baseline and parity.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from rethink_acoustic_image_enhancement_amd import _lib  # noqa: E402
from rethink_acoustic_image_enhancement_amd.hashweights import hash_images, hash_uniform, load_hash_weights  # noqa: E402
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_student, KDLAE_teacher  # noqa: E402
from rethink_acoustic_image_enhancement_amd.ASDQE_model import DenoiseRatePredictor  # noqa: E402
from rethink_acoustic_image_enhancement_amd.shard import OverlappedGather  # noqa: E402

METRIC = "images/sec KDLAE-T 1×512×512 fp32 at 1/2/4/8 MI355X; PSNR vs ref"
KW = dict(inp_channels=3, out_channels=3, dim=48, num_blocks=[4, 6, 6, 8], num_refinement_blocks=4,
          heads=[1, 2, 4, 8], ffn_expansion_factor=2.66, bias=False, LayerNorm_type="BiasFree",
          dual_pixel_task=False, static="train", params="cat")
PEAK_FP32_TFLOPS = 157.3   # MI355X dense FP32 (vector = MFMA f32), MI355X_MICROARCH.md
# r05: the inference GEMMs compute fp32 products on the bf16 matrix cores (csrc/mfma3.h: exact 3-way
# bf16 split, 6 MFMAs per 32-deep fp32 product block).  Their MFMA roof is the dense bf16 rate / 6:
# 1024 FLOP/clk/SIMD x 1024 SIMDs x 2.4 GHz = 2516.6 TF/s bf16 -> 419.4 TF/s of fp32 products.
PEAK_SPLIT_TFLOPS = 2516.6 / 6
PEAK_HBM_GBS = 8000.0      # HBM3E spec
# roofline definition versions: 1 (r01-r04) = the GEMM class (probe 1) against the 157.3 TF/s fp32 MFMA
# peak; 2 (r05-) = the dominant class by share of step (the feed-forward half, probe 3) against the
# 419.4 TF/s split-bf16 ceiling, the fp32-peak fraction kept as compute_view.frac_of_fp32_mfma_peak
ROOF_DEF_VERSION = 2
NESTED_TRAIN_STEPS, NESTED_TRAIN_WARMUP = 20, 5  # the training leg nested in the default T16 line
PROBE_CLASSES = {1: "conv_gemm (split-bf16 MFMA 1x1 / implicit-GEMM 3x3)", 2: "dwconv_gram (MDTA pass 1)",
                 3: "feed-forward half (fused FFN / GDFN tail)"}


def host_cores():
    """Host cores the CPU baseline may use: os.cpu_count() (BASELINE.md's plan), bounded by this
    process's CPU affinity and its cgroup CPU quota — on a shared GPU box os.cpu_count() reports the
    whole machine while the job is given a share of it.  Returns (threads, description)."""
    total = os.cpu_count() or 1
    n, why = total, [f"os.cpu_count()={total}"]
    try:
        aff = len(os.sched_getaffinity(0))
        why.append(f"affinity={aff}")
        n = min(n, aff)
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
            why.append(f"cgroup quota={quota}")
            n = min(n, quota)
    except (OSError, ValueError):
        pass
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        why.append(f"OMP_NUM_THREADS={env}")
        n = min(n, int(env))
    return max(1, n), ", ".join(why)


def make_inputs(first: int, n: int, H: int, W: int):
    """Images [first, first + n) of the global synthetic batch (keyed by global index, so every
    rank's shard is the matching slice of the single-process batch)."""
    imgs = np.stack([hash_images(f"img16:{first + i}", (3, H, W)) for i in range(n)])
    rates = (hash_uniform("rate16", first + n)[first:] + 1.0) * 0.5
    rate = np.broadcast_to(rates.astype(np.float32)[:, None, None, None], (n, 1, H, W)).copy()
    return torch.from_numpy(imgs), torch.from_numpy(rate)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv: list, need_gpus: bool = True) -> int:
    """Run this script as n rank processes under torch.distributed.run (one process per GPU,
    LOCAL_RANK -> device) and return its exit code.  Called before any GPU call; the parent only
    counts devices (torch.cuda.device_count() does not initialise HIP) and waits."""
    if need_gpus:
        visible = torch.cuda.device_count()
        if visible < n:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {visible}", file=sys.stderr, flush=True)
            return 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL)
    return subprocess.call(cmd, env=env)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def timed_steps(step, steps: int, distributed: bool, dev, drain=None):
    """Exactly `steps` calls of `step` bracketed by a barrier + device sync on both sides.
    `drain` (OverlappedGather.drain) runs inside the timed window, before the closing sync: every
    step's output gather is complete when the clock stops.
    Returns (max-over-ranks seconds, this rank's seconds, last output)."""
    _sync(dev)
    if distributed:
        dist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = step()
    if drain is not None:
        drain()
    _sync(dev)
    local = time.perf_counter() - t0
    elapsed = local
    if distributed:
        dist.barrier()
        t = torch.tensor([local], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, local, out


def cpu_timed(fn, runs: int = 3):
    """BASELINE.md CPU-baseline procedure: one untimed warm-up call, then the median of `runs`
    timed calls.  Returns (warm-up output, median seconds, sorted timings).  A progress line per
    call goes to stderr (the T16 sample is ~40 s a call: a silent 3-minute stretch reads as a hang
    to a watchdog)."""
    t0 = time.perf_counter()
    out = fn()
    print(f"[bench] cpu baseline warm-up: {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    ts = []
    for i in range(runs):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
        print(f"[bench] cpu baseline run {i + 1}/{runs}: {ts[-1]:.1f} s", file=sys.stderr, flush=True)
    ts.sort()
    return out, ts[len(ts) // 2], ts


def bench_standin(args, world, rank):
    """CPU rehearsal of the N-rank path (gloo, no GPU): the T16 sharding, timing and gather with a
    per-image stand-in for the forward.  Each rank sleeps rank-dependent time per step so the
    max-over-ranks timing is observable.  Used by tests/test_bench_launch.py."""
    dev = torch.device("cpu")
    B, H = args.batch or 16, args.size or 16
    img, rate = make_inputs(rank * B, B, H, H)
    delay = 0.01 * rank
    gather = OverlappedGather() if world > 1 else None

    def step():
        hq = img * 2 + rate
        time.sleep(delay)
        return gather({"hq": hq})["hq"] if gather else hq

    for _ in range(args.warmup):
        step()
    if gather:
        gather.drain()
    elapsed, local, full = timed_steps(step, args.steps, world > 1, dev, drain=gather.drain if gather else None)
    info = [{"rank": rank, "first": rank * B, "last": rank * B + B - 1, "local_s": local}]
    if world > 1:
        info = [None] * world
        dist.all_gather_object(info, {"rank": rank, "first": rank * B, "last": rank * B + B - 1, "local_s": local})
    if rank == 0:
        gimg, grate = make_inputs(0, world * B, H, H)
        res = {"metric": METRIC + " [CPU stand-in rehearsal]", "value": round(world * B * args.steps / elapsed, 3),
               "unit": "images/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(elapsed / args.steps * 1e3, 3), "elapsed_s": elapsed,
               "config": {"global_batch": world * B, "per_gpu_batch": B},
               "standin": {"ranks": info, "gather_equal": bool(torch.equal(full, gimg * 2 + grate))}}
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


S_KW = dict(inp_channels=1, out_channels=1, residual=True, hidden_channels=[16, 32, 64])  # KDLAE-S.ipynb:106
A_KW = dict(in_channels=3, dim=16)                                                          # ASDQE_test.py


def student_flops(hc, B, F, H, W):
    """Algorithmic FLOPs of one KDLAE-S forward (2 per MAC, un-padded channels)."""
    L, f, cin = len(hc) - 1, 0, 1
    for i in range(L):
        P = B * F * (H >> i) * (W >> i)
        f += 2 * P * 27 * (cin * hc[i] + hc[i] * hc[i])
        cin = hc[i]
    P = B * F * (H >> L) * (W >> L)
    f += 2 * P * 27 * (cin * hc[L] + hc[L] * hc[L])
    for i in range(L - 1, -1, -1):
        P = B * F * (H >> i) * (W >> i)
        cu = hc[L] if i == L - 1 else hc[i + 1]
        f += 2 * P * cu * hc[i] + 2 * P * 27 * 2 * hc[i] * hc[i]
    return f + 2 * B * F * H * W * hc[0]


def asdqe_flops(ci, d, B, H, W):
    """Algorithmic FLOPs of one ASDQE forward on the padded H' x W' grid (2 per MAC)."""
    Hp, Wp = -(-H // d) * d, -(-W // d) * d
    P = [B * (Hp >> i) * (Wp >> i) for i in range(4)]
    c = lambda p, a, b: 2 * p * 9 * (a * b + b * b)  # noqa: E731  DoubleConv
    f = 3 * c(P[0], ci, d) + c(P[0], 3 * d, 64) + c(P[1], 64, 128) + c(P[2], 128, 256) + c(P[3], 256, 256)
    f += c(P[2], 512, 128) + c(P[1], 256, 64) + c(P[0], 128, 64)
    return f


def bench_secondary(args, world, rank, dev, distributed, workload, batch=0, size=0, cpu=True):
    """S8 (KDLAE-S bs=8 4x512x512) and A64 (ASDQE bs=64 256x256): BASELINE.json configs[2], [3].
    Returns the result dict (rank 0 prints it, or nests it in the T16 line)."""
    if workload == "s8":
        B = batch or 8
        Fr, H, W = 4, size or 512, size or 512
        model = KDLAE_student(**S_KW)
        x = torch.from_numpy(np.stack([hash_images(f"s8:{rank * B + i}", (Fr, H, W)) for i in range(B)]))
        inputs = (x.to(dev),)
        flops = student_flops(S_KW["hidden_channels"], B, Fr, H, W)
        desc = f"KDLAE-S forward bs={B}/GPU {Fr}x{H}x{W} fp32 (hidden [16,32,64], residual)"
        metric = "samples/sec KDLAE-S 4-frame 512x512 fp32 (BASELINE configs[2])"
    else:
        B = batch or 64
        H = W = size or 256
        model = DenoiseRatePredictor(**A_KW)
        g = torch.from_numpy(np.stack([hash_images(f"a64gt:{rank * B + i}", (3, H, W)) for i in range(B)]))
        lq = (g + 0.1 * torch.from_numpy(hash_uniform("a64n", g.numel()).astype(np.float32)).view_as(g)).clamp(0, 1)
        inputs = (lq.to(dev), g.to(dev))
        flops = asdqe_flops(3, 16, B, H, W)
        desc = f"ASDQE forward bs={B}/GPU 3x{H}x{W} fp32 (dim 16, eval)"
        metric = "images/sec ASDQE 256x256 fp32 (BASELINE configs[3])"
    load_hash_weights(model)
    model = model.to(dev).eval()

    gather = distributed and not args.no_gather
    if gather:
        from rethink_acoustic_image_enhancement_amd.shard import gather_outputs

    def step():
        with torch.no_grad():
            o = model(*inputs)
            return gather_outputs(o) if gather else o

    for _ in range(args.warmup):
        step()
    # the whole forward runs on torch's current stream, so torch events bracket every launch
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed():
        ev0.record()
        for _ in range(args.steps):
            o = step()
        ev1.record()
        return o

    elapsed, _, out = timed_steps(timed, 1, distributed, dev)
    dev_ms = ev0.elapsed_time(ev1)
    if distributed:  # the gathered outputs: this rank's shard is rows [rank*B, rank*B + B)
        out = out[rank * B:(rank + 1) * B]
    ach = flops * args.steps / (dev_ms / 1e3) / 1e12
    # r05: the convs multiply on split-bf16 MFMAs (fp32-accurate products, ceiling 2516.6 / 6 TF/s);
    # the fraction of the fp32 MFMA peak the r01-r04 kernels were priced against is kept beside it
    roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": round(PEAK_SPLIT_TFLOPS, 1), "unit": "TFLOP/s",
            "frac": round(ach / PEAK_SPLIT_TFLOPS, 4), "frac_of_fp32_mfma_peak": round(ach / PEAK_FP32_TFLOPS, 4),
            "peak_definition": "fp32 products via split-bf16 MFMAs: dense bf16 2516.6 TF/s / 6",
            "traffic": None, "kernel": "whole forward (all launches)", "algorithmic_flops_per_step": flops}
    tr = pmc_workload_traffic(workload) if (B, H) == ((8, 512) if workload == "s8" else (64, 256)) else None
    if tr is not None:  # HBM bytes of one forward of this exact batch from a recorded PMC pass
        roof["traffic"], roof["traffic_source"], same = tr
        roof["traffic_unit"] = "bytes per forward (all launches)"
        roof["traffic_same_build"] = same  # the PMC pass profiled this exact libkdlae.so (sha256)
        if same:  # the rate those bytes imply at this run's step time (only for the profiled build)
            roof["traffic_rate_GBps"] = round(tr[0] * args.steps / (dev_ms / 1e3) / 1e9, 1)
            roof["traffic_frac_of_hbm"] = round(roof["traffic_rate_GBps"] / PEAK_HBM_GBS, 4)
    total = world * B * args.steps
    res = {"metric": metric, "value": round(total / elapsed, 3), "unit": "images/s" if workload == "a64"
           else "samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "fp32", "data": "synthetic (hash-uniform inputs, hash weights)",
           "config": {"workload": desc, "global_batch": world * B, "per_gpu_batch": B,
                      "parallelism": f"dp{world} (batch-sharded" + (", RCCL all-gather of outputs in every step)"
                                                                   if gather else ", no data-path collective)")},
           "roofline": roof}
    if rank == 0 and world == 1 and cpu:
        threads, tdesc = host_cores() if not args.cpu_threads else (args.cpu_threads, "--cpu-threads")
        torch.set_num_threads(threads)
        sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
        # bounded sample of the same workload (~2-3 s of CPU work per pass): the first n samples
        n = min(B, 4 if workload == "s8" else 32)
        if workload == "s8":
            from oracle.kdlae_oracle import StudentCfg, student_forward
            xs = inputs[0][:n].cpu()
            fn = lambda: student_forward(sd, xs, StudentCfg(**S_KW))  # noqa: E731
        else:
            from oracle.asdqe_oracle import AsdqeCfg, asdqe_forward
            lqs, gts = inputs[0][:n].cpu(), inputs[1][:n].cpu()
            fn = lambda: asdqe_forward(sd, lqs, gts, AsdqeCfg(**A_KW))  # noqa: E731
        with torch.no_grad():
            ref, med, ts = cpu_timed(fn)
        got = out[:n].cpu()
        res["cpu_baseline"] = {"value": round(n / med, 5), "unit": res["unit"], "cores": threads, "kind": "port",
                               "cores_from": tdesc,
                               "sample": f"first {n} samples of the workload batch in one call, torch-CPU oracle, "
                                         f"{threads} threads: 1 warm-up + median of 3 ({', '.join(f'{t:.2f}' for t in ts)} s)"}
        res["parity"] = {"vs": f"CPU oracle, samples 0..{n - 1}", "max_abs": float((got - ref).abs().max())}
    return res


def bench_train(args, world, rank, dev, distributed, nested=False):
    """KDLAE-T training iterations: ImageCleanModel.optimize_parameters with the
    KDLAET.yml fixed-patch setting (batch_size_per_gpu 6, gt_size 128, AdamW lr 1e-5 wd 5e-5 betas
    (0.2, 0.999), clip_grad_norm_ 0.01, L1LossSr); for N>1 every step all-reduces the flat gradient
    (107.5 MB) over RCCL, as DDP does.  One step = forward + loss + backward + all-reduce + clip + AdamW.
    nested: timed inside the default T16 run (its own steps / warm-up, no CPU baseline); returns the
    result instead of printing it."""
    from rethink_acoustic_image_enhancement_amd.train import KDLAETrainer

    B = 6 if nested else (args.batch or 6)
    H = W = 128 if nested else (args.size or 128)
    steps, warmup = (NESTED_TRAIN_STEPS, NESTED_TRAIN_WARMUP) if nested else (args.steps, args.warmup)
    model = KDLAE_teacher(**KW)
    load_hash_weights(model)
    model = model.to(dev)
    img, rate = make_inputs(1000 + rank * B, B, H, W)
    gt_hq = torch.from_numpy(np.stack([hash_images(f"train_gt:{rank * B + i}", (3, H, W)) for i in range(B)]))
    gt_sr = torch.from_numpy(np.stack([hash_images(f"train_gtsr:{rank * B + i}", (3, 2 * H, 2 * W))
                                       for i in range(B)]))
    batch = {"img": img.to(dev), "denoise_rate": rate.to(dev)}
    gt = {"hq": gt_hq.to(dev), "sr": gt_sr.to(dev)}
    # KDLAET.yml: mixing_augs {mixup: true, mixup_beta: 1.2, use_identity: true}; feed_train_data mixes
    trainer = KDLAETrainer(model, mixing_augs={"mixup": True, "mixup_beta": 1.2, "use_identity": True})
    import random
    random.seed(rank)
    torch.manual_seed(rank)

    def train_step():
        lq_m, gt_m = trainer.feed_train_data(batch, gt)
        return trainer.optimize_parameters(lq_m, gt_m)

    loss = None
    for _ in range(warmup):
        loss = train_step()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
        loss = train_step()
    ev1.record()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    dev_ms = ev0.elapsed_time(ev1)
    if distributed:
        dist.barrier()
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # SURVEY §8d forward FLOPs (1.9177 TFLOP per 512^2 image, linear in pixels) x 3 for fwd + dX + dW
    flops = 3 * 1.9177e12 * (H * W) / (512 * 512) * B
    ach = flops * steps / (dev_ms / 1e3) / 1e12
    total = world * B * steps
    res = {"metric": "images/sec KDLAE-T training step 128x128 patches fp32 (KDLAET.yml, SURVEY 8f rank 1)",
           "value": round(total / elapsed, 3), "unit": "images/s", "n_gpus": world, "steps": steps,
           "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 2), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
           "data": "synthetic (hash-uniform images and targets, hash weights of the real architecture)",
           "config": {"workload": f"KDLAE-T train step bs={B}/GPU {H}x{W} (+sr {2 * H}x{2 * W}), L1LossSr, "
                                  "clip_grad_norm_ 0.01, AdamW, mixup", "global_batch": world * B, "per_gpu_batch": B,
                      "parallelism": f"dp{world}" + (" (RCCL all-reduce of the flat gradient every step)"
                                                     if distributed else "")},
           "roofline": {"bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(ach / PEAK_FP32_TFLOPS, 4), "traffic": None,
                        "kernel": "whole training step (all launches, algorithmic 3x forward FLOPs)",
                        "algorithmic_flops_per_step": flops},
           "final_loss": float(loss)}
    if nested:
        return res
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.kdlae_oracle import TeacherCfg
        from oracle.train_oracle import TrainStep
        threads, tdesc = host_cores() if not args.cpu_threads else (args.cpu_threads, "--cpu-threads")
        torch.set_num_threads(threads)
        sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
        st = TrainStep(sd, TeacherCfg(**KW))
        t0 = time.perf_counter()
        st.step(batch["img"][:1].cpu(), batch["denoise_rate"][:1].cpu(),
                {"hq": gt["hq"][:1].cpu(), "sr": gt["sr"][:1].cpu()})
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(1.0 / dt, 5), "unit": "images/s", "cores": threads, "kind": "port",
                               "cores_from": tdesc,
                               "sample": f"1 image of the batch, one optimize_parameters step of the torch-CPU "
                                         f"training oracle, {threads} threads, {dt:.1f} s"}
        # parity of the trained weights' loss and gradients on image 0 (the oracle step above ran on the
        # same weights before its update; recompute its gradients without stepping)
        from oracle.train_oracle import loss_and_grads
        one = {"img": batch["img"][:1], "denoise_rate": batch["denoise_rate"][:1]}
        gt1 = {"hq": gt["hq"][:1], "sr": gt["sr"][:1]}
        l_gpu = float(trainer.forward_backward(one, gt1))
        g_gpu = trainer.engine.packed(trainer.grad.detach()).cpu()
        l_ref, g_ref = loss_and_grads(sd, one["img"].cpu(), one["denoise_rate"].cpu(),
                                      {k: v.cpu() for k, v in gt1.items()}, TeacherCfg(**KW))
        g_ref = torch.cat([g_ref[k].reshape(-1) for k, _ in model.named_parameters()])
        res["parity"] = {"vs": "torch-CPU training oracle, image 0, current weights",
                         "loss_rel_err": abs(l_gpu - float(l_ref)) / abs(float(l_ref)),
                         "grad_max_abs_err_rel_to_max": float((g_gpu - g_ref).abs().max() / g_ref.abs().max())}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if distributed:
        dist.destroy_process_group()


def bench_train_s(args, world, rank, dev, distributed):
    """KDLAE-S training iterations (KDLAES.yml: batch_size_per_gpu 4, num_pairs 7 frames, first progressive
    patch 128^2; L1LossForVideoFrames(0.9, mean, temporal 0.1); clip_grad_norm_ 0.01; AdamW lr 3e-4 wd 1e-4;
    mixup).  One step = forward + loss + backward + all-reduce (N > 1) + clip + AdamW."""
    from rethink_acoustic_image_enhancement_amd.train import KDLAESTrainer

    B = args.batch or 4
    H = W = args.size or 128
    Fr = 7
    model = KDLAE_student(**S_KW)
    load_hash_weights(model)
    model = model.to(dev)
    x = torch.from_numpy(np.stack([hash_images(f"trs_x:{rank * B + i}", (Fr, H, W)) for i in range(B)])).to(dev)
    gt = torch.from_numpy(np.stack([hash_images(f"trs_gt:{rank * B + i}", (Fr, H, W)) for i in range(B)])).to(dev)
    trainer = KDLAESTrainer(model, mixing_augs={"mixup": True, "mixup_beta": 1.2, "use_identity": True})
    import random
    random.seed(rank)
    torch.manual_seed(rank)

    def train_step():
        lq_m, gt_m = trainer.feed_train_data(x, gt)
        return trainer.optimize_parameters(lq_m, gt_m)

    loss = None
    for _ in range(args.warmup):
        loss = train_step()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed():
        ev0.record()
        out = None
        for _ in range(args.steps):
            out = train_step()
        ev1.record()
        return out

    elapsed, _, loss = timed_steps(timed, 1, distributed, dev)
    dev_ms = ev0.elapsed_time(ev1)
    flops = 3 * student_flops(S_KW["hidden_channels"], B, Fr, H, W)  # forward + dX + dW
    ach = flops * args.steps / (dev_ms / 1e3) / 1e12
    total = world * B * args.steps
    res = {"metric": "samples/sec KDLAE-S training step 7x128x128 fp32 (KDLAES.yml)",
           "value": round(total / elapsed, 3), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
           "data": "synthetic (hash-uniform frames and targets, hash weights of the real architecture)",
           "config": {"workload": f"KDLAE-S train step bs={B}/GPU {Fr}x{H}x{W}, L1LossForVideoFrames, "
                                  "clip_grad_norm_ 0.01, AdamW, mixup", "global_batch": world * B, "per_gpu_batch": B,
                      "parallelism": f"dp{world}" + (" (RCCL all-reduce of the flat gradient every step)"
                                                     if distributed else "")},
           "roofline": {"bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(ach / PEAK_FP32_TFLOPS, 4), "traffic": None,
                        "kernel": "whole training step (all launches, algorithmic 3x forward FLOPs)",
                        "algorithmic_flops_per_step": flops},
           "final_loss": float(loss)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.kdlae_oracle import StudentCfg
        from oracle.train_oracle import YML_S_LOSS, student_loss_and_grads
        threads, tdesc = host_cores() if not args.cpu_threads else (args.cpu_threads, "--cpu-threads")
        torch.set_num_threads(threads)
        sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
        t0 = time.perf_counter()
        l_ref, g_ref = student_loss_and_grads(sd, x[:1].cpu(), gt[:1].cpu(), StudentCfg(**S_KW), **YML_S_LOSS)
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(1.0 / dt, 5), "unit": "samples/s", "cores": threads, "kind": "port",
                               "cores_from": tdesc,
                               "sample": f"1 sample of the batch, forward + L1LossForVideoFrames + backward of the "
                                         f"torch-CPU oracle, {threads} threads, {dt:.1f} s"}
        trainer.forward_backward(x[:1], gt[:1])
        g = trainer.engine.packed(trainer.grad).cpu()
        gr = torch.cat([g_ref[k].reshape(-1) for k, _ in model.named_parameters()])
        res["parity"] = {"vs": "torch-CPU training oracle, sample 0, current weights",
                         "loss_rel_err": abs(float(trainer.loss) - float(l_ref)) / abs(float(l_ref)),
                         "grad_max_abs_err_rel_to_max": float((g - gr).abs().max() / gr.abs().max())}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if distributed:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["t16", "s8", "a64", "train", "train_s"], default="t16",
                    help="t16 = KDLAE-T bs16 512^2 (headline); s8 = KDLAE-S; a64 = ASDQE; train = KDLAE-T "
                         "training step (KDLAET.yml 6x128^2); train_s = KDLAE-S training step (KDLAES.yml 4x7x128^2)")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=0, help="images per GPU (0 = workload default)")
    ap.add_argument("--size", type=int, default=0, help="frame size (0 = workload default)")
    ap.add_argument("--probe", default="3,1",
                    help="kernel classes to probe, comma-separated; the first is the line's roofline (0 = off): "
                         "1 conv_gemm, 2 dwconv_gram, 3 feed-forward half")
    ap.add_argument("--probe-level", type=int, default=0, help="channel filter for the probe (0 = all)")
    ap.add_argument("--probe-steps", type=int, default=3,
                    help="steps of the separate probe pass after the timed steps (at most --steps)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true",
                    help="N>1: skip the RCCL all-gather of outputs (default: gathered inside each step, §8e)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0 = the host cores this process may use, see host_cores)")
    ap.add_argument("--no-bs1", action="store_true", help="t16: skip the single-image latency line")
    ap.add_argument("--no-secondary", action="store_true",
                    help="t16: skip the S8 / A64 lines (BASELINE configs[2], [3]) nested in the output")
    ap.add_argument("--no-train", action="store_true",
                    help="t16: skip the KDLAE-T training step (SURVEY 8f rank 1) nested in the output")
    ap.add_argument("--cpu-standin", action="store_true",
                    help="CPU rehearsal of the N-rank launch/shard/timing path (gloo, stand-in forward; tests)")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start the ranks before anything here touches the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], need_gpus=not args.cpu_standin))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr, flush=True)
        sys.exit(3)
    distributed = world > 1
    if args.cpu_standin:
        if distributed:
            dist.init_process_group("gloo")
        return bench_standin(args, world, rank)
    if distributed:
        if torch.cuda.device_count() < world:
            print(f"bench.py: WORLD_SIZE={world} but {torch.cuda.device_count()} visible GPUs", file=sys.stderr)
            sys.exit(3)
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    if args.workload == "train":
        return bench_train(args, world, rank, dev, distributed)
    if args.workload == "train_s":
        return bench_train_s(args, world, rank, dev, distributed)
    if args.workload != "t16":
        res = bench_secondary(args, world, rank, dev, distributed, args.workload, args.batch, args.size,
                              cpu=not args.no_cpu_baseline)
        if rank == 0:
            print(json.dumps(res), flush=True)
        if distributed:
            dist.destroy_process_group()
        return
    H = W = args.size or 512
    B = args.batch or 16

    model = KDLAE_teacher(**KW)
    load_hash_weights(model)
    model = model.to(dev).eval()
    img, rate = make_inputs(rank * B, B, H, W)
    batch = {"img": img.to(dev), "denoise_rate": rate.to(dev)}

    # the scaling metric runs to the end of the output all-gather.  Step i's gather
    # runs on RCCL's stream beside step i + 1's forward (the module returns fresh output tensors,
    # never the graph's buffers); timed_steps drains the last ones inside the timed window.
    gather = OverlappedGather() if distributed and not args.no_gather else None

    def step():
        with torch.no_grad():
            out = model(batch)
            return gather(out) if gather else out

    eng = model.engine(dev)
    L = _lib.lib()
    # The timed steps run the module's default forward, un-instrumented: probe disarmed and the
    # HIP-graph replay of a repeated shape (KDLAE_teacher.hip_graphs; the warmup's second call
    # captures).  The roofline comes from a separate probe pass AFTER the timed steps: the probe
    # brackets each launch of one kernel class with HIP events, so that pass runs launch by launch.
    model.hip_graphs = True
    drain = gather.drain if gather else None
    for _ in range(max(args.warmup, 2)):
        step()
    if drain:
        drain()
    torch.cuda.synchronize(dev)

    elapsed, _, out = timed_steps(step, args.steps, distributed, dev, drain=drain)
    if gather:  # this rank's own images of the gathered batch (for the parity leg)
        out = {k: (v[rank * B:(rank + 1) * B] if v is not None else None) for k, v in out.items()}

    def probe(cls):
        """Per-launch HIP-event probe of one kernel class over a separate launch-by-launch pass."""
        import ctypes
        import tempfile
        probe_steps = max(1, min(args.steps, args.probe_steps))
        model.hip_graphs = False
        L.kdlae_t_probe_arm(eng.handle, cls, args.probe_level)
        step()  # untimed: creates the probe's event pool outside the measured window
        if drain:
            drain()
        torch.cuda.synchronize(dev)
        L.kdlae_t_probe_arm(eng.handle, cls, args.probe_level)
        p_elapsed, _, _ = timed_steps(step, probe_steps, distributed, dev, drain=drain)
        model.hip_graphs = True
        ms, n, by, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
        dump = os.environ.get("KDLAE_PROBE_DUMP")
        own_dump = dump is None
        if own_dump:  # per-launch records for the class's per-shape roof (removed afterwards)
            fd, dump = tempfile.mkstemp(suffix=".csv")
            os.close(fd)
            os.environ["KDLAE_PROBE_DUMP"] = dump
        L.kdlae_t_probe_read(eng.handle, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(by), ctypes.byref(fl))
        launch_roof = per_launch_roof(dump)
        if own_dump:
            del os.environ["KDLAE_PROBE_DUMP"]
            os.unlink(dump)
        L.kdlae_t_probe_arm(eng.handle, 0, 0)
        if not n.value:
            return None
        sec = ms.value / 1e3
        # the class's bound: its algorithmic FLOPs at the split-bf16 ceiling vs its bytes at 8 TB/s
        if fl.value / (PEAK_SPLIT_TFLOPS * 1e12) > by.value / (PEAK_HBM_GBS * 1e9):
            ach = fl.value / sec / 1e12
            r = {"bound": "mfma", "achieved": round(ach, 2), "peak": round(PEAK_SPLIT_TFLOPS, 1),
                 "unit": "TFLOP/s", "frac": round(ach / PEAK_SPLIT_TFLOPS, 4), "traffic": None,
                 "peak_definition": "fp32 products via split-bf16 MFMAs: dense bf16 2516.6 TF/s / 6"}
        else:
            ach = by.value / sec / 1e9
            r = {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                 "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": None}
        r["definition_version"] = ROOF_DEF_VERSION
        if fl.value:  # the FLOP side of the same launches, against both fp32-product peaks
            tf = fl.value / sec / 1e12
            r["compute_view"] = {"achieved_tflops": round(tf, 2),
                                 "frac_of_split_bf16_peak": round(tf / PEAK_SPLIT_TFLOPS, 4),
                                 "frac_of_fp32_mfma_peak": round(tf / PEAK_FP32_TFLOPS, 4),
                                 "note": "fp32-accurate products; the split-bf16 peak (419.4) is the "
                                         "ceiling of this arithmetic, the fp32 MFMA peak (157.3) the "
                                         "ceiling of the r04 kernels"}
        tr = pmc_traffic(cls)
        if tr is not None:  # PMC HBM bytes per launch from a recorded pass; same_build: that pass
            r["traffic"], r["traffic_source"], r["traffic_same_build"] = tr  # profiled this exact .so
        if launch_roof is not None:
            r["per_shape_roof"] = launch_roof
        r.update({"kernel": PROBE_CLASSES[cls], "launches": int(n.value),
                  "avg_launch_us": round(ms.value * 1e3 / n.value, 2),
                  "probe_pass": {"steps": probe_steps, "ms_per_step": round(p_elapsed / probe_steps * 1e3, 2),
                                 "path": "launch by launch with HIP events around each probed launch, "
                                         "after the timed steps (which ran un-instrumented)"},
                  "share_of_step": round(ms.value / 1e3 / p_elapsed, 4),
                  "algorithmic_bytes_per_launch": by.value / n.value,
                  "algorithmic_flops_per_launch": fl.value / n.value})
        return r

    # the first listed class is the line's `roofline` (the dominant class, by its share of the step);
    # the others are reported under `roofline_classes`
    classes = [int(c) for c in str(args.probe).split(",") if c.strip() and int(c) != 0]
    roof, other = None, {}
    for i, cls in enumerate(classes):
        r = probe(cls)
        if i == 0:
            roof = r
        elif r is not None:
            other[PROBE_CLASSES[cls]] = r

    bs1 = None
    if not args.no_bs1 and B > 1 and world == 1:
        # the metric names 1x512x512: single-image latency of the drop-in module's forward on the same
        # GPU, each call synchronised (HIP events on the forward's stream), after the throughput run.
        # The module's default forward replays a HIP graph for a repeated shape (KDLAE_teacher.hip_graphs);
        # the launch-by-launch number is reported beside it.
        one = {"img": batch["img"][:1], "denoise_rate": batch["denoise_rate"][:1]}

        def latency(graphs):
            model.hip_graphs = graphs
            with torch.no_grad():
                for _ in range(3):
                    model(one)
                torch.cuda.synchronize(dev)
                ts = []
                for _ in range(10):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    o = model(one)
                    e1.record()
                    torch.cuda.synchronize(dev)
                    ts.append(e0.elapsed_time(e1))
            ts.sort()
            return ts, o

        gts, o_g = latency(True)
        ets, o_e = latency(False)
        med = gts[len(gts) // 2]
        bs1 = {"workload": f"KDLAE-T forward bs=1 1x3x{H}x{W} fp32 (same config), per GPU, module forward",
               "latency_ms_median": round(med, 3), "latency_ms_min": round(gts[0], 3),
               "images_per_s": round(1e3 / med, 3), "runs": len(gts),
               "forward_path": "HIP-graph replay of the whole forward (KDLAE_teacher.hip_graphs, default)",
               "launch_by_launch_latency_ms_median": round(ets[len(ets) // 2], 3),
               "graph_equals_launch_by_launch": bool(torch.equal(o_g["hq"], o_e["hq"]) and
                                                     torch.equal(o_g["sr"], o_e["sr"])),
               "hbm_roof_frac_survey_def": round(1e3 / med * 150.70e9 / 8.0e12, 4)}
        model.hip_graphs = True

    imgs_total = world * B * args.steps
    res = {
        "metric": METRIC, "value": round(imgs_total / elapsed, 3), "unit": "images/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (hash-uniform images, hash weights of the real architecture)",
        "config": {"workload": f"KDLAE-T forward bs={B}/GPU {H}x{W} fp32 (static=train, params=cat, BiasFree)",
                   "global_batch": world * B, "per_gpu_batch": B, "H": H, "W": W,
                   "timed_path": "the module's default forward (HIP-graph replay of the repeated shape), "
                                 "no probe armed",
                   "parallelism": f"dp{world} (batch-sharded" + (", RCCL all-gather of hq/sr in every step, "
                                                                 "overlapped with the next step's forward)"
                                                                if gather else ", no data-path collective)")},
        "roofline": roof,
    }
    if other:
        res["roofline_classes"] = other
    if bs1 is not None:
        res["bs1"] = bs1
    # algorithmic per-image figures of SURVEY.md §8d (KDLAE-T 512^2 static=train)
    if H == 512 and W == 512:
        ips = imgs_total / elapsed / world
        res["per_gpu"] = {"images_per_s": round(ips, 3),
                          "hbm_roof_frac_survey_def": round(ips * 150.70e9 / 8.0e12, 4),
                          "fp32_compute_frac": round(ips * 1.9177e12 / 157.3e12, 4),
                          # SURVEY §8d's per-op Σmax roof (41.8 img/s) prices every aten op's own HBM
                          # traffic; the fused kernels move less than that model, so >1 is possible
                          "vs_survey_unfused_sigma_max_roof": round(ips / 41.8, 4)}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"], res["parity"] = cpu_baseline(model, batch, out, args.cpu_threads)
    if not args.no_secondary and not args.batch and not args.size:
        # BASELINE configs[2] / [3] timed in the same run (their own weights, inputs and buffers)
        del model, batch, out, eng
        torch.cuda.empty_cache()
        for wl in ("s8", "a64"):
            sec = bench_secondary(args, world, rank, dev, distributed, wl, cpu=not args.no_cpu_baseline)
            keep = ("metric", "value", "unit", "ms_per_step", "config", "roofline", "cpu_baseline", "parity")
            res[wl] = {k: sec[k] for k in keep if k in sec}
            torch.cuda.empty_cache()
    if not args.no_train and not args.batch and not args.size:
        # SURVEY §8f rank 1, KDLAET.yml's 6 x 128^2 step, timed in the same run
        if "model" in locals():
            del model, batch, out, eng
        torch.cuda.empty_cache()
        tr = bench_train(args, world, rank, dev, distributed, nested=True)
        keep = ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "config", "roofline", "final_loss")
        res["train"] = {k: tr[k] for k in keep if k in tr}
        torch.cuda.empty_cache()
    if rank == 0:
        print(json.dumps(res), flush=True)
    if distributed:
        dist.destroy_process_group()


def per_launch_roof(path):
    """The class against each launch's own roof: sum over launches of max(FLOPs / MFMA peak,
    algorithmic bytes / HBM peak), divided by the summed measured time.  A class that mixes
    MFMA-bound and HBM-bound shapes (the 1x1 GEMMs at K = 48 are HBM-bound) cannot reach its MFMA
    fraction; this is the fraction of the time its launches would take at their own bound."""
    import csv
    try:
        rows = list(csv.DictReader(open(path)))
    except OSError:
        return None
    if not rows:
        return None
    t = sum(float(r["ms"]) for r in rows) / 1e3
    bound = sum(max(float(r["flops"]) / (PEAK_SPLIT_TFLOPS * 1e12), float(r["bytes"]) / (PEAK_HBM_GBS * 1e9))
                for r in rows)
    mfma_bound = sum(1 for r in rows
                     if float(r["flops"]) / (PEAK_SPLIT_TFLOPS * 1e12) >= float(r["bytes"]) / (PEAK_HBM_GBS * 1e9))
    return {"frac": round(bound / t, 4), "bound_ms": round(bound * 1e3, 2), "measured_ms": round(t * 1e3, 2),
            "launches_mfma_bound": mfma_bound, "launches_hbm_bound": len(rows) - mfma_bound,
            "definition": "sum_i max(flops_i / mfma_peak, bytes_i / hbm_peak) / sum_i t_i (HIP events); mfma_peak = "
                          "419.4 TF/s (split-bf16 fp32 products), hbm_peak = 8 TB/s"}


def lib_sha256():
    """sha256 of the libkdlae.so this process loaded (KDLAE_LIB or the in-tree build)."""
    import hashlib
    path = os.environ.get("KDLAE_LIB") or os.path.join(ROOT, "rethink_acoustic_image_enhancement_amd", "libkdlae.so")
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()
    except OSError:
        return None


def pmc_traffic(cls):
    """HBM bytes per launch of a kernel class from the committed rocprofv3 PMC summary
    (profiles/*pmc_traffic*.json, produced by tools/pmc_summary.py: FETCH_SIZE x2 + WRITE_SIZE)."""
    import glob
    def version(path):  # r02_pmc_traffic_v3.json -> (2, 3): numeric, round first, so r02 v3 > r01 v16
        m = re.search(r"r(\d+)_pmc_traffic_v(\d+)\.json$", path)
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic*.json")), key=version)
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    c = d.get("classes", {}).get(str(cls))
    if not c:
        return None
    return c["traffic_bytes_per_launch"], os.path.relpath(files[-1], ROOT), d.get("lib_sha256") == lib_sha256()


def pmc_workload_traffic(workload):
    """HBM bytes of one whole S8 / A64 forward from the committed PMC pass (profiles/rNN_pmc_<w>.json,
    tools/pmc_workload.py: FETCH_SIZE x2 + WRITE_SIZE, weight packing excluded); latest round wins."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{workload}.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    return d["traffic_bytes_per_forward"], os.path.relpath(files[-1], ROOT), d.get("lib_sha256") == lib_sha256()


def cpu_baseline(model, batch, out, threads):
    """Oracle (torch CPU restatement, test infrastructure) on image 0 of the workload."""
    from oracle.kdlae_oracle import TeacherCfg, psnr, teacher_forward

    threads, tdesc = host_cores() if not threads else (threads, "--cpu-threads")
    torch.set_num_threads(threads)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    img = batch["img"][:1].cpu()
    rate = batch["denoise_rate"][:1].cpu()
    with torch.no_grad():
        ref, med, ts = cpu_timed(lambda: teacher_forward(sd, img, rate, TeacherCfg(**KW)))
    hq, sr = out["hq"][:1].cpu(), out["sr"][:1].cpu()
    parity = {"vs": "CPU oracle, image 0", "hq_max_abs": float((hq - ref["hq"]).abs().max()),
              "sr_max_abs": float((sr - ref["sr"]).abs().max()),
              "hq_psnr_db": round(psnr(hq, ref["hq"]), 2), "sr_psnr_db": round(psnr(sr, ref["sr"]), 2)}
    base = {"value": round(1.0 / med, 5), "unit": "images/s", "cores": threads, "kind": "port",
            "cores_from": tdesc,
            "sample": f"1 image 1x3x{img.shape[-2]}x{img.shape[-1]} (image 0 of the bench batch), "
                      f"torch-CPU oracle, {threads} threads: 1 warm-up + median of 3 "
                      f"({', '.join(f'{t:.1f}' for t in ts)} s)"}
    return base, parity


if __name__ == "__main__":
    main()
