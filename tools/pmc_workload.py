"""HBM traffic of one whole forward of a secondary workload (S8 / A64) from two rocprofv3 --pmc passes.

Both passes run `bench.py --workload <w> --steps 1 --warmup 0 --no-cpu-baseline` (one forward).  The
one-time weight preparation (pack_* / split3 kernels, rocclr copies of the upload) is not part of a
forward and is left out; everything else is summed.  gfx950 correction (MI355X_MICROARCH.md §HBM):
fetched bytes = 2 x FETCH_SIZE x 1024, written bytes = WRITE_SIZE x 1024.

usage: python tools/pmc_workload.py <fetch csv> <write csv> <out.json> <workload> [forwards]
"""
import collections
import csv
import hashlib
import json
import os
import sys

SETUP = ("pack_", "split3_kernel", "__amd_rocclr")


def lib_sha256():
    """sha256 of the libkdlae.so the profiled run loaded (KDLAE_LIB or the in-tree build): bench.py
    reports the traffic as "this build's" only when its own library has the same hash."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.environ.get("KDLAE_LIB") or os.path.join(root, "rethink_acoustic_image_enhancement_amd", "libkdlae.so")
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()
    except OSError:
        return None


def load(path, counter):
    d = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("kdlae::", "")
        d[name][0] += 1
        d[name][1] += float(r["Counter_Value"]) * 1024.0
    return d


def main():
    fetch, write, out, workload = sys.argv[1:5]
    fwd = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    F, W = load(fetch, "FETCH_SIZE"), load(write, "WRITE_SIZE")
    kern = {}
    for k, (n, b) in F.items():
        if k.startswith(SETUP):
            continue
        w = W.get(k, [0, 0.0])[1]
        kern[k] = {"launches_per_forward": n / fwd, "fetch_bytes_corrected": 2.0 * b / fwd, "write_bytes": w / fwd,
                   "traffic_bytes": (2.0 * b + w) / fwd}
    tot = sum(v["traffic_bytes"] for v in kern.values())
    res = {"workload": workload, "forwards": fwd, "lib_sha256": lib_sha256(),
           "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py --workload "
                   f"{workload} --steps 1 --warmup 0; fetch doubled per the gfx950 rule; weight packing excluded",
           "traffic_bytes_per_forward": tot,
           "kernels": dict(sorted(kern.items(), key=lambda kv: -kv[1]["traffic_bytes"]))}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({"workload": workload, "traffic_bytes_per_forward": tot,
                      "top": {k: round(v["traffic_bytes"] / 1e9, 3) for k, v in list(res["kernels"].items())[:6]}},
                     indent=1))


if __name__ == "__main__":
    main()
