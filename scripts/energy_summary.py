"""Summarises gpurun_out/<TAG> of scripts/gpu_energy_probe.sh into profiles/<label>_energy_probe.json.

    python scripts/energy_summary.py <TAG> <label>

Per (K, filler): the stream's HBM traffic (GB/s, read + write), socket power and mean gfx clock (amd-smi medians), and
the dynamic energy per byte of traffic, (socket W - idle W) / (GB/s), in pJ per byte."""
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from aes256_summary import sample, summarize  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag, label):
    src = os.path.join(ROOT, "gpurun_out", tag)
    idle = sample(os.path.join(src, "idle.json"))
    out = {"idle": idle, "configs": {}}
    for p in sorted(glob.glob(os.path.join(src, "probe_*.json"))):
        k, f = re.match(r"probe_(\d+)_(\d+)\.json", os.path.basename(p)).groups()
        lines = [json.loads(x) for x in open(p) if x.strip().startswith("{")]
        if not lines:
            continue
        r = lines[-1]
        pw = summarize(sorted(glob.glob(os.path.join(src, f"smi_{k}_{f}_*.json"))))
        ent = dict(r)
        if pw:
            ent.update({"socket_w": pw["socket_w_median"], "gfx_mhz": pw["gfx_mhz_median"], "samples": pw["samples"]})
            if idle:
                ent["dynamic_pj_per_byte"] = round((pw["socket_w_median"] - idle["socket_w"]) / (r["traffic_gbps"] * 1e9) * 1e12, 1)
        out["configs"][f"K{k}_filler{f}"] = ent
        print(f"K={k:>2} filler={f:>4}", json.dumps({x: ent.get(x) for x in ("traffic_gbps", "payload_gibps", "socket_w",
                                                                              "gfx_mhz", "dynamic_pj_per_byte")}))
    with open(os.path.join(ROOT, "profiles", f"{label}_energy_probe.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
