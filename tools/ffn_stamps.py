"""Where the fused FFN kernel's waves spend their cycles: one T16 forward on a KDLAE_FFN_STAMPS build.

usage: KDLAE_LIB=build_ab/libkdlae_stamps.so python tools/ffn_stamps.py [batch] [size]

The stamp build (csrc/ffn.hip, -DKDLAE_FFN_STAMPS) sums s_memtime differences per segment over every
wave of every launch; this prints each segment's share of the waves' total cycles for the C = 48 and
C = 96 kernels, P (project_in) and G (gate + project_out) roles separately.  The stamps fence the
schedule: shares, not lengths.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rethink_acoustic_image_enhancement_amd import _lib  # noqa: E402
from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_teacher  # noqa: E402
from rethink_acoustic_image_enhancement_amd.hashweights import load_hash_weights  # noqa: E402

SEGS = {0: ["dma issue (W-in)", "project_in MFMA + image write", "wait W-in DMA", "barrier", "-", "-",
            "tile prologue (LN, split, pin(0)) + rest", "total"],
        1: ["dma issue (W-out)", "gate (dwconv + GELU)", "project_out MFMA (odd chunks)", "barrier", "-",
            "W wait (even chunks)", "epilogue + rest", "total"]}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    fn = L.kdlae_debug_ffn_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    model = KDLAE_teacher(**bench.KW)
    load_hash_weights(model)
    model = model.to(dev).eval()
    model.hip_graphs = False
    img, rate = bench.make_inputs(0, B, H, H)
    batch = {"img": img.to(dev), "denoise_rate": rate.to(dev)}
    with torch.no_grad():
        model(batch)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 32)()
        assert fn(None, 1) == 0
        model(batch)
        torch.cuda.synchronize()
        assert fn(ctypes.cast(buf, ctypes.c_void_p), 0) == 0
    v = list(buf)
    for ci, C in enumerate((48, 96)):
        for role in (0, 1):
            seg = v[(ci * 2 + role) * 8:(ci * 2 + role + 1) * 8]
            tot = seg[7]
            if not tot:
                continue
            print(f"C{C} {'P' if role == 0 else 'G'} waves: total {tot / 1e9:.3f} G wave-cycles")
            for k in range(7):
                if SEGS[role][k] != "-":
                    print(f"   {SEGS[role][k]:40s} {seg[k] / tot:7.3f}")


if __name__ == "__main__":
    main()
