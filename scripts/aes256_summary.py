"""Summarises gpurun_out/<TAG> of scripts/aes256_study.sh into profiles/<label>_aes256_study.json.

    python scripts/aes256_summary.py <TAG> <label>

Power and clock: amd-smi `metric -p -c` samples (socket power; gfx clock averaged over the 8 XCDs) while the probe
(T-table only, and 8 T-table + 8 bitsliced waves) and the AES-256 batch kernels run; compute-only rates from the
probe logs; PMC of the AES-256 batch launches per 64-block wave step (SQ_* counters summed over the GPU)."""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def sample(path):
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    g = d["gpu_data"][0] if isinstance(d, dict) and "gpu_data" in d else d[0]
    p = g["power"]["socket_power"]["value"]
    clks = [v["clk"]["value"] for k, v in g["clock"].items() if k.startswith("gfx_") and isinstance(v, dict)]
    return {"socket_w": p, "gfx_mhz_mean": round(statistics.mean(clks), 1)}


def summarize(files):
    s = [x for x in map(sample, files) if x]
    if not s:
        return None
    return {"samples": len(s), "socket_w": [x["socket_w"] for x in s], "gfx_mhz_mean": [x["gfx_mhz_mean"] for x in s],
            "socket_w_median": statistics.median(x["socket_w"] for x in s),
            "gfx_mhz_median": statistics.median(x["gfx_mhz_mean"] for x in s)}


def rate(log):
    m = re.findall(r"T-table waves\s+(\d+):\s+[\d.]+ ms\s+([\d.]+) GB/s", open(log).read())
    return {int(a): float(b) for a, b in m}


def pmc(dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                if r["Kernel_Name"].startswith("mi355x_gcm_seal_aes256"):
                    agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: statistics.median(v) for c, v in d.items()} for k, d in agg.items()}


def main(tag, label):
    src = os.path.join(ROOT, "gpurun_out", tag)
    out = {"idle": summarize([os.path.join(src, "idle.json")])}
    out["probe_sweep_short"] = rate(os.path.join(src, "probe_sweep.log")) if os.path.exists(os.path.join(src, "probe_sweep.log")) else None
    for ntt in (16, 8):
        out[f"probe_{ntt}_ttable_waves"] = {"gbps_of_blocks": rate(os.path.join(src, f"probe_power_{ntt}.log")),
                                            "power": summarize(sorted(glob.glob(os.path.join(src, f"probe_{ntt}_*.json"))))}
    out["batch_aes256_16k"] = {"power": summarize(sorted(glob.glob(os.path.join(src, "bench_16k_*.json"))))}
    try:
        out["batch_aes256_16k"]["bench"] = json.loads(open(os.path.join(src, "bench_16k.json")).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        pass
    counters = pmc(sorted(glob.glob(os.path.join(src, "pmc_*"))))
    out["pmc_seal_aes256"] = counters
    for k, c in counters.items():
        steps = (1 << 18) * 1028 / 64.0 if "k4" in k else None  # wave steps of 256K x 16 KiB (257 steps x 4 lanes)
        if steps and "SQ_INSTS_VALU" in c:
            out.setdefault("per_wave_step", {})[k] = {
                x: round(c[x] / steps, 1) for x in
                ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM") if x in c}
        if "SQ_LDS_IDX_ACTIVE" in c and "GRBM_GUI_ACTIVE" in c:
            out.setdefault("lds_busy", {})[k] = round(c["SQ_LDS_IDX_ACTIVE"] / 256 / (c["GRBM_GUI_ACTIVE"] / 8), 3)
    path = os.path.join(ROOT, "profiles", f"{label}_aes256_study.json")
    json.dump(out, open(path, "w"), indent=1)
    print(path)
    print(json.dumps({k: v for k, v in out.items() if k not in ("pmc_seal_aes256",)}, indent=1)[:4000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
