"""CPU model of k1_lean's window stepping at C1 (the round-4 review's item 1a).

Go's parse of each stream (writer.go:213-322, restated from tests/pyoracle.py's Writer.write with a
record of each action: the position x where a copy was taken and the position the parse resumes
at) drives the kernel's window stepping: a G-lane group judges positions i .. i+G-1 at once and
either takes the window's first action (i = the resume position) or moves on G positions.  Per
stream that gives the windows the group needs; streams run 64/G to a wave (one launch block), and
a wave iterates until its slowest stream is done, so the issue wasted on finished groups is
1 - sum(windows) / (streams per wave x max windows per wave).  Also reported: the visits per
window (Go's visited positions / windows) and the windows at G = 8.
python tools/k1_waste_model.py [--streams 2048]"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import pyoracle as po  # noqa: E402
from eazy_amd import synth  # noqa: E402


def actions(p: bytes, bs=1 << 20, hs=1024):
    """[(x, resume)] of Go's parse of one fresh single-Write stream, and the visits made."""
    w = po.Writer(bs, hs)
    acts, visits = [], 0
    done, i, n = 0, 0, len(p)
    start = w.pos
    blk = w.block
    while i + 4 <= n:
        visits += 1
        h = w._hash(p, i)
        pos = w.ht[h]
        w.ht[h] = (start + i) & 0xFFFFFFFF
        off = pos - w.pos
        if -off > w.bs:
            i += 1
            continue
        if off >= 0 and i > done + off:
            x = i
            d2, i2 = w._write_runlen(p, done, done + off, i)
            if d2 != done or i2 != x + 1:  # an action (a reject returns done, i + 1)
                acts.append((x, i2))
            done, i = d2, i2
            continue
        ist, st = i - 1, pos - 1
        while ist >= done and p[ist] == blk[st & w.mask]:
            ist -= 1
            st -= 1
        ist += 1
        st += 1
        iend, end = i, pos
        while iend < n and p[iend] == blk[end & w.mask]:
            iend += 1
            end += 1
        blit = w.pos - w.bs
        diff = (blit + (iend - done)) - st
        if diff > 0:
            end -= diff
            iend -= diff
        diff = (end - w.bs) - blit
        if diff > 0:
            end -= diff
            iend -= diff
        if end - st < po.MIN_COPY_CHUNK:
            i += 1
            continue
        if done < ist:
            w._literal(p, done, ist)
            w._copy_data(p, done, ist)
        w._copy(st, end)
        w._copy_data(p, ist, iend)
        if i + 1 + 4 <= n:
            w.ht[w._hash(p, i + 1)] = (start + i + 1) & 0xFFFFFFFF
        acts.append((i, iend))
        i = iend
        done = iend
    return acts, visits


def windows(acts, n, G):
    """Windows a G-lane group needs: from each resume position to the next action's window, then
    the trailing literal's windows (positions up to n - 4 are visited)."""
    w, cnt = 0, 0
    for x, nx in acts:
        cnt += (x - w) // G + 1
        w = nx
    if w + 4 <= n:
        cnt += (n - 3 - w + G - 1) // G
    return cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=2048)
    a = ap.parse_args()
    S = 4096
    data = synth.logs(1, a.streams * S).tobytes()
    w16, w8, vis = [], [], []
    for s in range(a.streams):
        p = data[s * S : (s + 1) * S]
        acts, v = actions(p)
        w16.append(windows(acts, S, 16))
        w8.append(windows(acts, S, 8))
        vis.append(v)
    w16, w8, vis = np.array(w16), np.array(w8), np.array(vis)
    for G, w in ((16, w16), (8, w8)):
        k = 64 // G
        m = w[: len(w) // k * k].reshape(-1, k)
        idle = 1.0 - m.sum() / (k * m.max(axis=1)).sum()
        print(f"G={G:2d}: windows per stream {w.mean():.1f} (min {w.min()}, max {w.max()}); "
              f"wave iterations per stream {m.max(axis=1).sum() / m.size:.1f}; idle-group waste {100 * idle:.2f} %; "
              f"Go's visits per window {vis.sum() / w.sum():.2f} of {G}")


if __name__ == "__main__":
    main()
