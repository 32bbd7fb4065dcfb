"""Interleaved A/B of bench.py's step pipeline (chunks of the batch over two streams) on one box.

    python scripts/pipeline_ab.py [--workloads 1400,16k-aes128,16k] [--chunks 1,2,4] [--rounds 3] [--steps 20]

Each round measures every (workload, chunks) pair once with bench.measure (same pre-warm, warmup and timed
region as the bench line); prints one JSON line per measurement and a summary line of the medians."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="1400,16k-aes128,16k")
    ap.add_argument("--chunks", default="1,2,4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prewarm-ms", type=float, default=300.0)
    a = ap.parse_args()
    import numpy as np
    import torch

    import bench
    import rapido_amd as ra
    ra.require_gpu()
    dev = torch.device("cuda", 0)
    res = {}
    for rnd in range(a.rounds):
        for wl in a.workloads.split(","):
            for c in [int(x) for x in a.chunks.split(",")]:
                args = argparse.Namespace(pipeline=c, steps=a.steps, warmup=a.warmup, prewarm_ms=a.prewarm_ms)
                r, ex = bench.measure(ra, wl, args, dev, 0, 1, 16)
                ex["eng"].close()
                del ex
                torch.cuda.empty_cache()
                line = {"round": rnd, "workload": wl, "chunks": c, "value": r["value"],
                        "frac": r["roofline"]["frac"], "region_frac": r["roofline"]["region"]["frac"],
                        "seal_gibps": r["seal_gibps"], "open_gibps": r["open_gibps"],
                        "ms_per_step": r["ms_per_step"]}
                print(json.dumps(line), flush=True)
                res.setdefault((wl, c), []).append(r["value"])
    print(json.dumps({"summary": {f"{wl}/c{c}": round(float(np.median(v)), 2) for (wl, c), v in res.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
