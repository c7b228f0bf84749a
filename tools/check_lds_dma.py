"""Guard for the LDS-DMA destination (M0) of every `buffer_load ... lds` in libkdlae.so.

Cause this guards against (r06, DESIGN §4 "LDS-DMA destinations and hipcc's switch lowering"): issuing
each G wave's project_out DMA pieces as a `switch` on the wave index made hipcc tail-merge the four
cases into one straight-line DMA block whose first piece takes M0 from an SGPR (`s_mov_b32 m0, s65`)
that only the wave 0 / 1 / 2 paths define: on the wave 3 path the register holds whatever an earlier
instruction left in it, so that wave's first 1 KiB piece lands at a stale LDS address and the
pair's project_out reads a stale plane (NaN / 0.1 max-abs on t_full_b1_48x80).

The check: per kernel, split the disassembly into basic blocks, run a forward "defined on every
path" data-flow over the SGPRs (a register counts as defined by any instruction that names it as a
destination; the user / system SGPRs the dispatch preloads count as defined at entry), and report
every M0 write that feeds an LDS DMA and reads an SGPR not defined on every path to it.

usage: python tools/check_lds_dma.py [libkdlae.so] [kernel-name-substring ...]
exit 0 = clean, 1 = findings (printed), 2 = tool error.
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ENTRY_SGPRS = 16  # kernarg pointer, dispatch ptr, workgroup ids, ... (preloaded user + system SGPRs)

INS = re.compile(r"^\s+([a-z_0-9]+)(?:\s+(.*?))?\s*//\s*([0-9A-F]+):")
TGT = re.compile(r"<(\S+)\+0x([0-9a-f]+)>")
SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")
NODEF = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_barrier", "s_nop", "s_endpgm",
         "s_setprio", "s_sleep", "s_dcache", "s_store", "s_buffer_store", "s_sendmsg", "s_trap", "s_setreg",
         "s_sethalt", "s_icache", "s_memtime", "s_memrealtime", "buffer_", "global_", "scratch_", "ds_",
         "flat_", "s_set_gpr_idx")


def sregs(text):
    out = set()
    for m in SREG.finditer(text or ""):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def operands(text):
    return [o.strip() for o in (text or "").split(",")]


def defs_of(op, args):
    """SGPRs an instruction writes (over-approximated for VALU ops with SGPR results)."""
    if op.startswith(NODEF):
        if op.startswith("s_memtime") or op.startswith("s_memrealtime"):
            return sregs(operands(args)[0])
        return set()
    ops = operands(args)
    if op.startswith("s_"):
        return sregs(ops[0]) if ops and ops[0] else set()
    if op.startswith("v_"):  # v_readfirstlane / v_readlane / v_cmp_*_e64 sdst / carry-out pairs
        d = set()
        for o in ops[:2]:
            d |= sregs(o)
        return d
    return set()


def kernels(dis):
    cur, name = None, None
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(\S+)>:", line)
        if m:
            if cur is not None:
                yield name, cur
            name, cur = m.group(2), []
            continue
        if cur is None:
            continue
        mi = INS.match(line)
        if mi:
            cur.append((int(mi.group(3), 16), mi.group(1), mi.group(2) or "", line))
    if cur is not None:
        yield name, cur


def check_kernel(name, ins):
    if not any(op.startswith("buffer_load") and "lds" in a.split()[-1:] for _, op, a, _ in ins):
        return []
    base = ins[0][0]
    addr_idx = {a: i for i, (a, _, _, _) in enumerate(ins)}
    # block leaders: entry, branch targets, instructions after a branch
    leaders = {0}
    succ_target = {}
    for i, (a, op, args, line) in enumerate(ins):
        if op.startswith("s_cbranch") or op == "s_branch":
            m = TGT.search(line)
            if m and m.group(1) == name:
                t = addr_idx.get(base + int(m.group(2), 16))
                if t is not None:
                    leaders.add(t)
                    succ_target[i] = t
            leaders.add(i + 1)
        elif op == "s_endpgm":
            leaders.add(i + 1)
    leaders = sorted(x for x in leaders if x < len(ins))
    blk_of = {}
    blocks = []
    for k, s in enumerate(leaders):
        e = leaders[k + 1] if k + 1 < len(leaders) else len(ins)
        blocks.append((s, e))
        for i in range(s, e):
            blk_of[i] = k
    succ = [set() for _ in blocks]
    for k, (s, e) in enumerate(blocks):
        last = e - 1
        op = ins[last][1]
        if last in succ_target:
            succ[k].add(blk_of[succ_target[last]])
        if op != "s_branch" and op != "s_endpgm" and e < len(ins):
            succ[k].add(k + 1)
    preds = [set() for _ in blocks]
    for k, ss in enumerate(succ):
        for t in ss:
            preds[t].add(k)
    gen = []
    for s, e in blocks:
        d = set()
        for i in range(s, e):
            d |= defs_of(ins[i][1], ins[i][2])
        gen.append(d)
    allregs = set(range(0, 106))
    IN = [set(allregs) for _ in blocks]
    OUT = [set(allregs) for _ in blocks]
    IN[0] = set(range(ENTRY_SGPRS))
    changed = True
    while changed:
        changed = False
        for k in range(len(blocks)):
            if k:
                new_in = set(allregs)
                for p in preds[k]:
                    new_in &= OUT[p]
                if not preds[k]:
                    new_in = set()
                IN[k] = new_in
            new_out = IN[k] | gen[k]
            if new_out != OUT[k]:
                OUT[k] = new_out
                changed = True
    findings = []
    for k, (s, e) in enumerate(blocks):
        live = set(IN[k])
        pending = None  # the last M0 write of this block and the SGPRs it read
        for i in range(s, e):
            a, op, args, line = ins[i]
            ops = operands(args)
            if ops and ops[0] == "m0" and op.startswith("s_"):
                read = set()
                for o in ops[1:]:
                    read |= sregs(o)
                pending = (i, read - live)
            if op.startswith("buffer_load") and args.split()[-1:] == ["lds"] and pending and pending[1]:
                j, undef = pending
                findings.append(f"{name}: LDS DMA at +0x{a - base:x} takes M0 from s{sorted(undef)} "
                                f"(written at +0x{ins[j][0] - base:x}: {ins[j][3].split('//')[0].strip()}), "
                                f"not defined on every path to it")
            live |= defs_of(op, args)
    return findings


def main():
    args = sys.argv[1:]
    lib = args[0] if args and args[0].endswith(".so") else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rethink_acoustic_image_enhancement_amd",
        "libkdlae.so")
    names = [a for a in args if not a.endswith(".so")]
    tmp = tempfile.mkdtemp(prefix="ldsdma_")
    try:
        so = os.path.join(tmp, "lib.so")
        shutil.copy(lib, so)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", so], cwd=tmp, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        objs = [os.path.join(tmp, f) for f in os.listdir(tmp) if f.endswith("gfx950")]
        if not objs:
            print("no gfx950 code objects found", file=sys.stderr)
            return 2
        findings, nk = [], 0
        for o in sorted(objs):
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", o],
                                 check=True, capture_output=True, text=True).stdout
            for name, ins in kernels(dis):
                if names and not any(n in name for n in names):
                    continue
                if any(op.startswith("buffer_load") and a.split()[-1:] == ["lds"] for _, op, a, _ in ins):
                    nk += 1
                findings += check_kernel(name, ins)
        for f in findings:
            print(f)
        print(f"check_lds_dma: {nk} kernels with LDS DMA checked, {len(findings)} finding(s)")
        return 1 if findings else 0
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())
