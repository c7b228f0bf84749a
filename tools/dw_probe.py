"""Timing probe of the 1x1 weight-gradient contractions of the KDLAE-T training step (6 x 128^2,
KDLAET.yml): dW = dY^T X over all pixels, through kdlae_debug_tgemm route 0 (the launch_tgemm
dispatch the training step uses: pixel-reduction kernel + fixed-order split-K reduce).  Prints one
line per shape: ms per launch, TF/s, GB/s of the operand bytes, and max |err| against torch fp64.
With `cold`, each timed launch reads a different copy of the operands (8 copies: past the 256 MB
Infinity Cache), as in the training step where they were written long before.
usage: python tools/dw_probe.py [reps] [cold]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rethink_acoustic_image_enhancement_amd import _lib  # noqa: E402
from tests.test_kernel_variants_gpu import TGemmDesc  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
copies = 8 if "cold" in sys.argv[2:] else 1
DEV = torch.device("cuda", 0)
# (label, M = Cout, N = Cin, P pixels, lda, ldb)
SHAPES = [
    ("enhance ffn.project_out", 48, 127, 393216, 48, 128),
    ("enhance ffn.project_in", 254, 48, 393216, 256, 48),
    ("enhance attn.project_out", 48, 48, 393216, 48, 48),
    ("level1 ffn.project_out", 96, 255, 98304, 96, 256),
    ("level1 ffn.project_in", 510, 96, 98304, 512, 96),
    ("level1 attn.project_out", 96, 96, 98304, 96, 96),
    ("level1 attn.qkv", 288, 96, 98304, 288, 96),
]
part = torch.empty(8 << 20, device=DEV)
for label, M, N, P, lda, ldb in SHAPES:
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    dY0 = (torch.rand(P, lda, generator=g) * 2 - 1).to(DEV)
    X0 = (torch.rand(P, ldb, generator=g) * 2 - 1).to(DEV)
    ops = [(dY0, X0)] + [(dY0.clone(), X0.clone()) for _ in range(copies - 1)]
    C = torch.zeros(M, N, device=DEV)
    d = TGemmDesc()
    d.nz1 = d.nz2 = 1
    d.dil = 1
    for k, v in dict(A=dY0.data_ptr(), sam=1, sak=lda, B=X0.data_ptr(), sbk=ldb, sbn=1, C=C.data_ptr(), scm=N, scn=1,
                     M=M, N=N, K=P, partial=part.data_ptr(), partial_floats=part.numel(), route=0).items():
        setattr(d, k, v)

    def run(i=0):
        d.A, d.B = ops[i % copies][0].data_ptr(), ops[i % copies][1].data_ptr()
        _lib.check(_lib.lib().kdlae_debug_tgemm(ctypes.byref(d), None), "kdlae_debug_tgemm")

    for i in range(3):
        run(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        run(i)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    run(0)
    ref = dY0[:, :M].double().T @ X0[:, :N].double()
    err = (C.double() - ref).abs().max().item() / (ref.abs().max().item() + 1e-30)
    flop = 2.0 * M * N * P
    byts = 4.0 * P * (M + N)
    print(f"{label:28s} M{M:4d} N{N:4d} P{P:7d}  {ms * 1e3:8.1f} us  {flop / ms / 1e9:6.1f} TF/s  "
          f"{byts / ms / 1e6:7.1f} GB/s  rel err {err:.1e}", flush=True)
    del dY0, X0, ops, C
