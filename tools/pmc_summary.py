"""Per-kernel-class HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide coalesced
streaming read, so fetched bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 is exact for 16-B/lane
stores.  Writes profiles/<out>.json with bytes per launch for each kernel class bench.py probes.

usage: python tools/pmc_summary.py <fetch run_counter_collection.csv> <write csv> <out.json> [forwards]
"""
import collections
import csv
import hashlib
import json
import os
import sys

CLASSES = {"conv_gemm_kernel": 1, "gemm_res_kernel": 1, "gemm_chunk_kernel": 1, "gemm_attn_in_kernel": 1, "dwconv_gram": 2,
           "dwconv_gate_kernel": 3, "ffn_fused_kernel": 3, "gdfn_out_kernel": 3, "gdfn2_kernel": 3}


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
    fetch, write, out = sys.argv[1:4]
    F, W = load(fetch, "FETCH_SIZE"), load(write, "WRITE_SIZE")
    cls = collections.defaultdict(lambda: {"launches": 0, "fetch_bytes_corrected": 0.0, "write_bytes": 0.0})
    for k, (n, b) in F.items():
        c = next((v for p, v in CLASSES.items() if k.startswith(p)), 0)
        cls[c]["launches"] += n
        cls[c]["fetch_bytes_corrected"] += 2.0 * b
        cls[c]["write_bytes"] += W.get(k, [0, 0.0])[1]
    res = {"note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; fetch doubled per gfx950 rule",
           "lib_sha256": lib_sha256(), "classes": {}}
    for c, v in sorted(cls.items()):
        t = v["fetch_bytes_corrected"] + v["write_bytes"]
        res["classes"][str(c)] = dict(v, traffic_bytes=t,
                                      traffic_bytes_per_launch=t / max(1, v["launches"]))
    tot = sum(v["fetch_bytes_corrected"] + v["write_bytes"] for v in cls.values())
    res["total_traffic_bytes"] = tot
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
