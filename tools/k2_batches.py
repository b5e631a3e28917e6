"""Copy-batch and dependency-level counts of C1-like streams: the streams are
compressed by the C oracle and their tokens walked here; for rounds of G consecutive tokens,
a batch runs from the first pending copy up to the first copy whose source reaches past that
copy's output position (copies whose source ends before the round, and zero regions, run in
any batch) -- the rule K2t and K2s use; levels are the dependency depth inside each round.
Usage: python tools/k2_batches.py [streams]"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import oracle as orc  # noqa: E402
from eazy_amd import synth  # noqa: E402


def tokens(c):
    """(is_copy, out_pos, L, D) of every literal and copy token (the forms C1's streams use)."""
    i, pos, out = 0, 0, []
    while i < len(c):
        t = c[i]
        if t == 0:
            i += 1
            continue
        if t == 0x80:  # header metas: magic, reset
            ml = c[i + 1] & 7
            i += 2 + (0 if ml == 7 else 1 << ml)
            continue
        l7, j = t & 0x7F, i + 1
        L = {124: lambda: 124 + c[j], 125: lambda: 380 + c[j] + 256 * c[j + 1]}.get(l7, lambda: l7)()
        j += {124: 1, 125: 2}.get(l7, 0)
        if t & 0x80:
            lng = c[j] == 0xFF
            j += lng
            o = c[j]
            j += 1
            D = {252: lambda: 252 + c[j], 253: lambda: 508 + c[j] + 256 * c[j + 1]}.get(o, lambda: o)()
            j += {252: 1, 253: 2}.get(o, 0)
            out.append((1, pos, L, D if lng else D + L))
        else:
            out.append((0, pos, L, 0))
            j += L
        pos += L
        i = j
    return out


def rounds(T, G):
    nb = nl = 0
    for r0 in range(0, len(T), G):
        R = T[r0 : r0 + G]
        start = R[0][1]
        pend, lv, depth = [], [], 0
        for cp, p, L, D in R:
            if not cp:
                continue
            cs = p - D
            need = cs + min(D, L)
            pend.append((p, need, D == 0 or need <= start))
            lvl = 1
            if D and need > start:
                lvl += max([lv_ for a, b, lv_ in lv if a < need and cs < b] or [0])
            lv.append((p, p + L, lvl))
            depth = max(depth, lvl)
        nl += depth
        while pend:
            oa, cut, rest = pend[0][0], False, []
            for k, (p, need, free) in enumerate(pend):
                if k == 0 or free or (not cut and need <= oa):
                    continue
                cut = True
                rest.append((p, need, free))
            pend = rest
            nb += 1
    return nb, nl


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    d = synth.logs(1, n * 4096)
    streams = [tokens(orc.compress(1 << 20, 1024, [bytes(d[s * 4096 : (s + 1) * 4096])])) for s in range(n)]
    print(f"{n} C1 streams: {sum(map(len, streams)) / n:.1f} tokens per stream")
    for G in (8, 16, 32, 64):
        b = l = 0
        for T in streams:
            x, y = rounds(T, G)
            b += x
            l += y
        print(f"rounds of {G:2d} tokens: {sum((len(T) + G - 1) // G for T in streams) / n:5.1f} rounds, "
              f"{b / n:5.1f} copy batches, {l / n:5.1f} dependency levels per stream")


if __name__ == "__main__":
    main()
