"""Join the stream-size sweep of tools/gpurun/gpurun_hbm_sweep.sh into one table:
python tools/hbm_sweep.py gpurun_out/sweep 4096 16384 ...

Per size: compress / decompress GiB/s (device-resident), each stage's algorithmic
GB/s (n + c bytes per stream) against the 8 TB/s HBM peak, and its HBM
bytes per launch from the PMC passes (FETCH_SIZE x 2 + WRITE_SIZE, tools/traffic.py)
as a multiple of the algorithmic bytes."""

import json
import os
import sys

PEAK = 8000.0
# kx_: K1x rounds, kc_: K1c chunks, ke_: the wide token writer, kd_: deferred literals, kj_: K2j
STAGES = {"k1_compress": ("k1_", "kx_", "kc_", "ke_"), "k3_pack": ("k3_",), "k2_decompress": ("k2_", "kd_", "kj_")}


def main():
    root, sizes = sys.argv[1], [int(z) for z in sys.argv[2:]]
    rows = []
    for z in sizes:
        b = json.load(open(os.path.join(root, f"b_{z}.json")))
        t = json.load(open(os.path.join(root, f"t_{z}.json")))["kernels"]
        alg = b["roofline"]["algorithmic_bytes_per_launch"]
        row = {"stream_bytes": z, "streams": b["config"]["streams_per_gpu"], "ratio": round(b["ratio"], 3),
               "compress_GiBps": round(b["compress_GiBps"], 2), "decompress_GiBps": round(b["decompress_GiBps"], 2),
               "value": round(b["value"], 2), "kernel_ms": {k: round(v, 4) for k, v in b["kernel_ms"].items()}, "stages": {}}
        for st, pre in STAGES.items():
            ms = b["kernel_ms"][st]
            traffic = sum(v["traffic"] for k, v in t.items() if k.startswith(pre) and v.get("traffic"))
            kernels = sorted(k for k in t if k.startswith(pre))
            gbs = alg / (ms / 1e3) / 1e9
            row["stages"][st] = {"kernels": kernels, "achieved_GBps": round(gbs, 1), "frac": round(gbs / PEAK, 4),
                                 "traffic_B": int(traffic), "traffic_over_alg": round(traffic / alg, 2)}
        rows.append(row)
    print(json.dumps(rows, indent=1))
    print()
    print("| stream | streams | ratio | compress GiB/s | K1 GB/s (frac) | K1 traffic / alg | decompress GiB/s | K2 GB/s (frac) | K2 traffic / alg | K1 / K2 kernels |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        k1, k2 = r["stages"]["k1_compress"], r["stages"]["k2_decompress"]
        print(f"| {r['stream_bytes'] // 1024} KiB | {r['streams']} | {r['ratio']} | {r['compress_GiBps']} | "
              f"{k1['achieved_GBps']} ({k1['frac'] * 100:.1f} %) | {k1['traffic_over_alg']} | {r['decompress_GiBps']} | "
              f"{k2['achieved_GBps']} ({k2['frac'] * 100:.1f} %) | {k2['traffic_over_alg']} | "
              f"{'+'.join(k1['kernels'])} / {'+'.join(k2['kernels'])} |")


if __name__ == "__main__":
    main()
