"""Per-basic-block instruction counts of one kernel in a gfx950 assembly listing (hipcc
--cuda-device-only -S): VALU (v_*), SALU (s_* minus branches/waits), LDS (ds_*), vector memory
(global_/buffer_/flat_), branches, with each block's successors, so a loop's VALU per iteration can
be attributed to its phases.  python tools/isa_blocks.py listing.s <symbol substring>"""

import re
import sys


def blocks(path, sym):
    lines = open(path).read().split("\n")
    start = next(k for k, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(sym) + r"\S*:", l))
    out, cur, name = [], [], lines[start].split(":")[0]
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            out.append((name, cur))
            name, cur = m.group(1), []
            continue
        t = l.split(";")[0].strip()
        if t and not t.startswith("."):
            cur.append(t)
    out.append((name, cur))
    return out


def kind(ins):
    op = ins.split()[0]
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "br"
    if op.startswith(("s_waitcnt", "s_nop", "s_setprio", "s_sleep")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    bl = blocks(path, sym)
    tot = {}
    for name, ins in bl:
        c = {}
        for x in ins:
            k = kind(x)
            c[k] = c.get(k, 0) + 1
            tot[k] = tot.get(k, 0) + 1
        succ = [x.split()[-1] for x in ins if x.startswith(("s_cbranch", "s_branch"))]
        print(f"{name:14s} n={len(ins):4d} valu={c.get('valu', 0):4d} salu={c.get('salu', 0):3d} lds={c.get('lds', 0):3d} "
              f"vmem={c.get('vmem', 0):3d} wait={c.get('wait', 0):3d} -> {' '.join(succ)}")
    print("total", tot)


if __name__ == "__main__":
    main()
