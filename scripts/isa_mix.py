#!/usr/bin/env python3
"""Static instruction mix of one kernel in a device assembly file (profiling aid, not product).

    hipcc --offload-arch=gfx950 <build.py flags> --offload-device-only -S -o k.s walker_hip.hip
    python scripts/isa_mix.py k.s 'walker_step_leanILb1ELi3E' [--dump out.s] [--blocks]

Counts the instructions of the kernel's body by class (VALU f64 / f32 / int / cvt / mov-cmp-sel / DPP, LDS,
VMEM, SALU, SMEM, branch) overall and per basic block, so a source change can be read as instructions before it
is timed on the box.  A static count: loop bodies count once (the dynamic mix comes from the PMC passes).
"""
import re
import sys
from collections import Counter, OrderedDict


def extract(path, pat):
    lines = open(path).read().splitlines()
    start = None
    for i, ln in enumerate(lines):
        if re.match(r"^_Z\S*" + pat + r"\S*:", ln):
            start = i
            break
    if start is None:
        raise SystemExit(f"no kernel matching {pat}")
    body = []
    for ln in lines[start + 1:]:
        if ln.startswith(".Lfunc_end") or "s_endpgm" in ln and False:
            break
        body.append(ln)
    return lines[start], body


def klass(op):
    if op.startswith("v_"):
        if "_dpp" in op or op.startswith("v_mov_b32_dpp"):
            return "valu_dpp"
        if op.startswith(("v_cvt_",)):
            return "valu_cvt"
        if op.endswith("_f64") or "_f64_" in op:
            return "valu_f64"
        if op.startswith(("v_mov", "v_cndmask", "v_cmp", "v_readlane", "v_readfirstlane", "v_writelane",
                          "v_accvgpr")):
            return "valu_mov_cmp_sel"
        if re.search(r"_(f32|f16|pk_f32)", op):
            return "valu_f32"
        return "valu_int"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_setprio", "s_sleep")):
        return "wait_nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    head, body = extract(path, pat)
    dump = None
    if "--dump" in sys.argv:
        dump = sys.argv[sys.argv.index("--dump") + 1]
    tot = Counter()
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = Counter()
    ops = Counter()
    for ln in body:
        s = ln.strip()
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            cur = m.group(1)
            blocks[cur] = Counter()
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        op = s.split()[0]
        k = klass(op)
        if k == "other":
            continue
        tot[k] += 1
        blocks[cur][k] += 1
        ops[op] += 1
    print(head.split(":")[0][:120])
    valu = sum(v for k, v in tot.items() if k.startswith("valu"))
    print(f"total VALU {valu}  " + "  ".join(f"{k} {v}" for k, v in sorted(tot.items())))
    if "--blocks" in sys.argv:
        for b, c in blocks.items():
            n = sum(c.values())
            if n:
                print(f"{b:22s} {n:5d}  " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
    if "--ops" in sys.argv:
        for op, n in ops.most_common(60):
            print(f"  {op:28s} {n}")
    if dump:
        open(dump, "w").write("\n".join([head] + body) + "\n")


if __name__ == "__main__":
    main()
