"""CPU models behind two K1 levers at C1, from Go's parse of C1 streams
(tools/k1_waste_model.py's actions, restated from tests/pyoracle.py):
  * two accepts per 16-lane window: the windows a group needs when, after the first acceptor's match
    ends inside the window, the next action is also taken in that window -- allowed when no position
    Go visits before it read a table entry written by a lane Go skipped (a skipped lane is the nearest
    earlier same-hash lane);
  * the forward cap: the fraction of accepts whose forward match reaches 24 / 32 / 40 / 48 bytes (a
    saturated count takes the cooperative extension gext).
python tools/k1_two_accept_model.py [--streams 512]"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]

import numpy as np  # noqa: E402

import pyoracle as po  # noqa: E402
from eazy_amd import synth  # noqa: E402
from k1_waste_model import actions, windows  # noqa: E402


def hashes(p, hs=1024):
    w = po.Writer(1 << 20, hs)
    return [w._hash(p, k) if k + 4 <= len(p) else -1 for k in range(len(p))]


def windows2(acts, n, G, H):
    """Windows with up to two actions per window (window matches assumed: the i+1 insert kept)."""
    w, cnt, two, k = 0, 0, 0, 0
    while True:
        if k >= len(acts):
            if w + 4 <= n:
                cnt += (n - 3 - w + G - 1) // G
            return cnt, two
        x1, nx1 = acts[k]
        if x1 >= w + G:
            cnt += 1
            w += G
            continue
        cnt += 1
        if k + 1 < len(acts):
            x2, nx2 = acts[k + 1]
            if x2 < w + G and nx1 >= x1 + 2 and x2 >= nx1:
                skipped = set(range(x1 + 2, nx1))  # (x1 + 1: the i+1 insert, kept)
                clean = True
                for q in range(nx1, x2 + 1):
                    r = next((t for t in range(q - 1, w - 1, -1) if H[t] == H[q]), None)
                    if r is not None and r in skipped:
                        clean = False
                        break
                if clean:
                    two += 1
                    k += 2
                    w = nx2
                    continue
        k += 1
        w = nx1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=512)
    a = ap.parse_args()
    S = 4096
    data = synth.logs(1, a.streams * S).tobytes()
    one = two = seconds = 0
    fwd = []
    for s in range(a.streams):
        p = data[s * S : (s + 1) * S]
        acts, _ = actions(p)
        fwd += [nx - x for x, nx in acts]
        one += windows(acts, S, 16)
        c, t = windows2(acts, S, 16, hashes(p))
        two += c
        seconds += t
    print(f"windows per stream: one accept {one / a.streams:.1f}, two accepts {two / a.streams:.1f} "
          f"({seconds / a.streams:.1f} second accepts per stream)")
    f = np.array(fwd)
    print("accepts whose forward match reaches the cap: " + ", ".join(f"{c}: {100 * (f >= c).mean():.2f} %" for c in (24, 32, 40, 48)))


if __name__ == "__main__":
    main()
