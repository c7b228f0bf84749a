"""Which of libkdlae.so's kernels a GPU test run launched.

    python tools/kernel_coverage.py <rocprofv3 output dir of `pytest -m gpu`> [lib] > profiles/...txt

The library's kernels are the __global__ host stubs in its symbol table (every template
instantiation the launch tables can reach); the launched ones are the kernel names in the
rocprofv3 --kernel-trace databases (.db) or --stats CSV(s).  Prints both lists and the difference.
"""
import csv
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def norm(name: str) -> str:
    """'void kdlae::gemm_res_kernel<8, 6, 2, 2, false, true>(kdlae::GemmParams)' -> 'gemm_res_kernel<8,6,2,2,false,true>'"""
    name = re.sub(r"^void\s+", "", name.strip()).replace("(anonymous namespace)::", "")
    depth, cut = 0, len(name)
    for i, ch in enumerate(name):  # drop the argument list: the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    name = name[:cut]
    lt = name.find("<")
    ident, targs = (name[:lt], name[lt:]) if lt >= 0 else (name, "")
    ident = ident.split("::")[-1].replace("__device_stub__", "")
    return ident + targs.replace(" ", "")


def library_kernels(lib):
    out = subprocess.run(["nm", "-C", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    ks = set()
    for line in out.splitlines():
        parts = line.split(" ", 2)
        if len(parts) < 3 or parts[1] not in ("T", "t", "W", "w", "V", "v"):
            continue
        sym = parts[2]
        if re.search(r"_kernel(<[^()]*>)?\(", sym) and "launch" not in sym.split("(")[0]:
            ks.add(norm(sym))
    return ks


def launched_kernels(prof_dir):
    import sqlite3
    ks = {}
    for f in glob.glob(os.path.join(prof_dir, "**", "*.db"), recursive=True):
        con = sqlite3.connect(f)
        if not con.execute("select name from sqlite_master where type in ('table', 'view') and name = 'kernels'").fetchall():
            continue  # a CSV run leaves an empty database beside its CSV files
        for (name, n) in con.execute("select name, count(*) from kernels group by name"):
            k = norm(name)
            ks[k] = ks.get(k, 0) + int(n)
    for f in glob.glob(os.path.join(prof_dir, "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            n = norm(row.get("Name") or row.get("KernelName") or "")
            if n:
                ks[n] = ks.get(n, 0) + int(float(row.get("Calls", 1) or 1))
    return ks


def main():
    prof = sys.argv[1]
    lib = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "rethink_acoustic_image_enhancement_amd", "libkdlae.so")
    have = library_kernels(lib)
    got = launched_kernels(prof)
    hit = sorted(k for k in have if k in got)
    miss = sorted(k for k in have if k not in got)
    print(f"kernels in {os.path.basename(lib)}: {len(have)}; launched by the run: {len(hit)}; never launched: {len(miss)}")
    print("\n# launched (calls)")
    for k in hit:
        print(f"{got[k]:>8}  {k}")
    print("\n# never launched")
    for k in miss:
        print(f"          {k}")
    return 0 if not miss else 1


if __name__ == "__main__":
    sys.exit(main())
