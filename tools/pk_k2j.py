"""Per-kernel timeline of K2j sequences from a rocprofv3 kernel trace (tools/k2j_small.py under
rocprofv3 --kernel-trace): for each sequence index given, the kernels' durations summed by name.
python tools/pk_k2j.py run_kernel_trace.csv [seq ...]"""

import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    seqs, cur = [], None
    for r in rows:
        n = r["Kernel_Name"].replace("ez::(anonymous namespace)::", "").split("(")[0]
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        s = int(r["Start_Timestamp"])
        if n == "kj_init":
            cur = []
            seqs.append(cur)
        if cur is not None:
            cur.append((n, d, s))
    for idx in [int(a) for a in sys.argv[2:]] or range(len(seqs)):
        q = seqs[idx]
        agg = collections.OrderedDict()
        for n, d, s in q:
            c, t = agg.get(n, (0, 0))
            agg[n] = (c + 1, t + d)
        span = (q[-1][2] + q[-1][1] - q[0][2]) / 1000
        print(f"sequence {idx}: span {span:.1f} us, {len(q)} kernels: " +
              ", ".join(f"{n} {t / 1000:.1f}" + (f" ({c}x)" if c > 1 else "") for n, (c, t) in agg.items()))


if __name__ == "__main__":
    main()
