"""Config-1 (MDD sonar crop 512x512, denoise_rate 0.6) per-block error of the HIP path vs fp64.

ANALYSIS INFRASTRUCTURE (the cpu leg imports oracle/; nothing here is on the product path).

  gpu leg (GPU box):  python tools/config1_taps.py gpu --tag base [--out gpurun_out/c1]
      runs the drop-in module (the library KDLAE_LIB names, default the in-tree build) on the config-1
      input with kdlae_t_debug_taps armed and saves every stage input, block attention half and block output (subsampled to
      <= 65536 floats per block) plus hq / sr ([::2, ::2]) to <out>/taps_<tag>.npz.
  cpu leg (here):     python tools/config1_taps.py cpu [--out gpurun_out/c1] [--write profiles/...]
      runs the CPU oracle in fp64 and fp32 (and with the HIP path's Gram slot scheme) recording the same
      samples, then tabulates per block max-abs vs fp64 relative to the block's max |x| for every
      taps_*.npz found, so the block where the HIP error departs from the fp32 models shows up.
"""
import argparse
import glob
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BUDGET = 65536  # floats kept per block tap


def stride_for(h, w, c):
    s = 1
    while (h // s) * (w // s) * c > BUDGET and s < min(h, w):
        s *= 2
    return s


def setup():
    from tests.util import load_fixture, mdd_input_tensor
    d, kw = load_fixture("t_mdd_512")
    return kw, mdd_input_tensor(d), torch.full((1, 1, 512, 512), 0.6)


def gpu_leg(args):
    import ctypes

    from rethink_acoustic_image_enhancement_amd import _lib
    from rethink_acoustic_image_enhancement_amd.hashweights import load_hash_weights
    from rethink_acoustic_image_enhancement_amd.KDLAE_model import KDLAE_teacher

    kw, img, rate = setup()
    dev = torch.device("cuda:0")
    m = KDLAE_teacher(**kw)
    load_hash_weights(m)
    m = m.to(dev).eval()
    m.hip_graphs = False
    L = _lib.lib()
    eng = m.engine(dev)
    n = L.kdlae_t_debug_tap_count(eng.handle)
    H, W = img.shape[-2:]
    names, bufs = [], []
    for i in range(n):
        nm, C, num, den = ctypes.create_string_buffer(64), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(L.kdlae_t_debug_tap_info(eng.handle, i, nm, 64, ctypes.byref(C), ctypes.byref(num),
                                            ctypes.byref(den)), "tap_info")
        hi, wi = H * num.value // den.value, W * num.value // den.value
        names.append(nm.value.decode())
        bufs.append(torch.empty((1, hi, wi, C.value), device=dev))
    ptrs = (ctypes.c_void_p * n)(*[b.data_ptr() for b in bufs])
    _lib.check(L.kdlae_t_debug_taps(eng.handle, n, ptrs), "debug_taps")
    with torch.no_grad():
        out = m({"img": img.to(dev), "denoise_rate": rate.to(dev)})
    torch.cuda.synchronize()
    _lib.check(L.kdlae_t_debug_taps(eng.handle, 0, None), "debug_taps off")
    save = {"names": np.array(names), "hq": out["hq"][0, :, ::2, ::2].cpu().numpy(),
            "sr": out["sr"][0, :, ::2, ::2].cpu().numpy()}
    for nm, b in zip(names, bufs):
        _, hi, wi, c = b.shape
        s = stride_for(hi, wi, c)
        save["tap:" + nm] = b[0, ::s, ::s, :].permute(2, 0, 1).contiguous().cpu().numpy()  # [C, h, w]
    os.makedirs(args.out, exist_ok=True)
    path = os.path.join(args.out, f"taps_{args.tag}.npz")
    np.savez_compressed(path, **save)
    print(f"wrote {path}: {n} taps, lib {_lib.LIB_PATH}")


def oracle_run(cfg, sd, img, rate, mdta=None):
    """The oracle forward with the tap points recorded (same sampling as the taps): every stage's
    input, every block's attention half x1 = x + attn(norm1 x) and its output (KDLAE_model.py:159-163)."""
    import oracle.kdlae_oracle as O
    rec = {}
    orig = {n: getattr(O, n) for n in ("transformer_block", "stage", "mdta")}

    def keep(name, y):
        _, c, h, w = y.shape
        s = stride_for(h, w, c)
        rec[name] = y[0, :, ::s, ::s].double()

    def tb(x, sd_, p, heads, lt):
        x1 = x + O.mdta(O.layer_norm(x, sd_, p + ".norm1", lt), sd_, p + ".attn", heads)
        keep(p + ".attn", x1)
        y = x1 + O.gdfn(O.layer_norm(x1, sd_, p + ".norm2", lt), sd_, p + ".ffn")
        keep(p, y)
        return y

    def stage(x, sd_, name, n, heads, lt):
        if n > 0:
            keep(name + ".in", x)
        for i in range(n):
            x = tb(x, sd_, f"{name}.{i}", heads, lt)
        return x

    O.transformer_block, O.stage = tb, stage
    if mdta is not None:
        O.mdta = mdta
    try:
        with torch.no_grad():
            out = O.teacher_forward(sd, img, rate, cfg)
    finally:
        for n, f in orig.items():
            setattr(O, n, f)
    rec["hq"] = out["hq"][0, :, ::2, ::2].double()
    rec["sr"] = out["sr"][0, :, ::2, ::2].double()
    return rec


def cpu_leg(args):
    import oracle.kdlae_oracle as O
    from tests.util import hash_sd_for
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from config1_precision import mdta_slots  # the HIP Gram slot scheme on the oracle (r03 analysis)

    torch.set_num_threads(os.cpu_count() or 8)
    kw, img, rate = setup()
    cfg = O.TeacherCfg(**kw)
    sd32 = hash_sd_for(O.teacher_param_shapes(cfg))
    sd64 = {k: v.double() for k, v in sd32.items()}
    cache = os.path.join(args.out, "oracle_cache.pt")  # this script's own output (weights_only load)
    if os.path.exists(cache):
        c = torch.load(cache, weights_only=True)
        r64, cols = c["r64"], {"ref32": c["ref32"], "slots32": c["slots32"]}
    else:
        t = time.time()
        r64 = oracle_run(cfg, sd64, img.double(), rate.double())
        print(f"fp64 oracle {time.time() - t:.0f} s", flush=True)
        cols = {"ref32": oracle_run(cfg, sd32, img, rate),
                "slots32": oracle_run(cfg, sd32, img, rate, mdta=mdta_slots)}
        os.makedirs(args.out, exist_ok=True)
        torch.save({"r64": r64, **cols}, cache)
    for path in sorted(glob.glob(os.path.join(args.out, "taps_*.npz"))):
        d = np.load(path, allow_pickle=False)
        tag = os.path.basename(path)[5:-4]
        rec = {str(n): torch.from_numpy(d["tap:" + str(n)]).double() for n in d["names"]}
        rec["hq"] = torch.from_numpy(d["hq"]).double()
        rec["sr"] = torch.from_numpy(d["sr"]).double()
        cols["hip_" + tag] = rec
    keys = list(r64.keys())
    lines = [__doc__.strip(), "",
             "relative error per tap (stage input .in, attention half .attn, block output) = max-abs vs the fp64 oracle / max |x_fp64| over the",
             f"block's sample (<= {BUDGET} floats); hq / sr rows: absolute max-abs over [::2, ::2] and [::8, ::8].",
             "ref32 = the oracle in fp32 (= the reference's arithmetic); slots32 = ref32 with the HIP path's Gram",
             "scheme (fp32 sums over 1024-pixel slots, slots summed in fp64); hip_* = the HIP library builds.", "",
             f"{'block':<20}" + "".join(f"{c:>14}" for c in cols)]
    for k in keys:
        ref = r64[k]
        m = float(ref.abs().max())
        row = f"{k:<20}"
        for c, rec in cols.items():
            e = float((rec[k] - ref).abs().max())
            row += f"{(e if k in ('hq', 'sr') else e / max(m, 1e-30)):>14.3e}"
        lines.append(row)
    for k in ("hq", "sr"):
        row = f"{k + '[::8]':<20}"
        for c, rec in cols.items():
            row += f"{float((rec[k][:, ::4, ::4] - r64[k][:, ::4, ::4]).abs().max()):>14.3e}"
        lines.append(row)
    text = "\n".join(lines) + "\n"
    print(text)
    if args.write:
        with open(args.write, "w") as f:
            f.write(text)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("leg", choices=["gpu", "cpu"])
    ap.add_argument("--tag", default="base")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "c1"))
    ap.add_argument("--write", default="")
    args = ap.parse_args()
    (gpu_leg if args.leg == "gpu" else cpu_leg)(args)


if __name__ == "__main__":
    main()
