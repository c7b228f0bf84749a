"""fp32 GEMM rates of the training step's 1x1-conv shapes through torch.mm (hipBLASLt / rocBLAS)
on one MI355X, for comparison with the hand-written tgemm kernels (train.hip).

KDLAET.yml step: 6 images of 128^2 (+ the 256^2 sr branch).  Per level: P pixels, C in, N out.
Forms: fwd  Y[P,N] = X[P,C] W[N,C]^T;  dX  dX[P,C] = dY[P,N] W[N,C];  dW  dW[N,C] = dY[P,N]^T X[P,C].
"""
import json
import sys

import torch

dev = torch.device("cuda", 0)
torch.backends.cuda.matmul.allow_tf32 = False
B = 6
levels = [  # (P, C, hid) per TransformerBlock level of the released KDLAE-T at 128^2
    (B * 256 * 256, 48, 127),  # enhance (sr branch, 2H x 2W)
    (B * 128 * 128, 48, 127),  # encoder_level1
    (B * 128 * 128, 96, 255),  # decoder_level1 / refinement / refinement_out
    (B * 64 * 64, 96, 255),    # encoder/decoder level 2
    (B * 32 * 32, 192, 510),   # level 3
    (B * 16 * 16, 384, 1021),  # latent
]


def bench(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


rows = []
for P, C, hid in levels:
    for name, K, N in (("qkv", C, 3 * C), ("proj", C, C), ("pin", C, 2 * hid), ("pout", hid, C)):
        X = torch.randn(P, K, device=dev)
        W = torch.randn(N, K, device=dev)
        dY = torch.randn(P, N, device=dev)
        fl = 2.0 * P * K * N
        t_f = bench(lambda: torch.mm(X, W.t()))
        t_dx = bench(lambda: torch.mm(dY, W))
        t_dw = bench(lambda: torch.mm(dY.t(), X))
        r = {"P": P, "K": K, "N": N, "layer": name, "fwd_ms": round(t_f, 4), "dx_ms": round(t_dx, 4),
             "dw_ms": round(t_dw, 4), "fwd_tf": round(fl / t_f / 1e9, 1), "dx_tf": round(fl / t_dx / 1e9, 1),
             "dw_tf": round(fl / t_dw / 1e9, 1)}
        rows.append(r)
        print(json.dumps(r), flush=True)
tot = sum(r["fwd_ms"] + r["dx_ms"] + r["dw_ms"] for r in rows)
print(json.dumps({"sum_ms_one_block_per_level": round(tot, 3)}), file=sys.stderr)
