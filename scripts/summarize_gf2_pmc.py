"""Summarise scripts/gpu_probe_gf2_pmc.sh (the MFMA-GHASH probe's resources per mode) into one JSON:

    python scripts/summarize_gf2_pmc.py gpurun_out/gf2pmc profiles/r03k_probe_gf2_resources.json

Per mode (AES-128): PMC per 64 blocks (LDS-array busy cycles, VALU / LDS wave-instructions, MFMA busy
cycles, wave cycles), the clock of the profiled dispatch (GRBM_GUI_ACTIVE / 8 over its duration), GB/s of the long
run, and socket power / gfx clock from amd-smi samples during that run."""
import collections
import csv
import glob
import json
import os
import re
import sys

MODES = {0: "aes_only", 1: "aes+mfma_ghash (v_perm pack, scaled)", 3: "aes+mfma_ghash (v_alignbit pack, unscaled)",
         2: "aes+nibble_ghash (shipped)"}
NCU = 256
BLOCKS_PER_DISPATCH = NCU * 16 * 48 * 2048  # probe_gf2.py defaults: 48 units per wave, 16 waves per CU, 2048 blocks a unit


def pmc(path, kernel):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].startswith(kernel):
            d = per[r["Dispatch_Id"]]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            d["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    if not per:
        return None
    last = per[sorted(per, key=int)[-1]]  # the second repetition (the first warms up)
    units = BLOCKS_PER_DISPATCH / 64  # 64-block groups (the counters sum over all CUs)
    out = {k + "_per_64_blocks": round(v / units, 1) for k, v in last.items()
           if not k.startswith("_") and k != "GRBM_GUI_ACTIVE"}
    out["clock_ghz_profiled"] = round(last["GRBM_GUI_ACTIVE"] / 8 / last["_ns"], 3)
    out["dispatch_ms_profiled"] = round(last["_ns"] / 1e6, 3)
    return out


def power(paths):
    watts, mhz = [], []
    for p in paths:
        try:
            g = json.load(open(p))["gpu_data"][0]
        except (ValueError, KeyError, IndexError):
            continue
        watts.append(g["power"]["socket_power"]["value"])
        clks = [v["clk"]["value"] for k, v in g["clock"].items() if k.startswith("gfx_") and isinstance(v, dict)]
        mhz.append(round(sum(clks) / len(clks)))
    return {"socket_power_w": watts, "gfx_mhz_mean_of_8_xcds": mhz}


def main(src, dst):
    res = {}
    for m, name in MODES.items():
        r = {"mode": name}
        p = os.path.join(src, f"pmc_{m}", "run_counter_collection.csv")
        if os.path.exists(p):
            r["pmc"] = pmc(p, f"probe_gf2_run_10_{m}")
        log = os.path.join(src, f"long_{m}.log")
        if os.path.exists(log):
            g = re.findall(r"AES-128 \S+\s*:\s*([\d.]+) ms\s+([\d.]+) GB/s", open(log).read())
            if g:
                r["long_run_ms_per_rep"], r["long_run_gbps_blocks"] = float(g[-1][0]), float(g[-1][1])
        r["power"] = power(sorted(glob.glob(os.path.join(src, f"power_{m}_*.json"))))
        res[MODES[m]] = r
    res["idle"] = power([os.path.join(src, "idle.json")])
    res["note"] = ("scripts/gpu_probe_gf2_pmc.sh: AES-128, 16 waves per CU, compute-only (no HBM). PMC from one "
                   "rocprofv3 --pmc pass per mode (the second of two dispatches), normalised per 64 blocks; "
                   "SQ_LDS_IDX_ACTIVE and SQ_VALU_MFMA_BUSY_CYCLES in cycles, SQ_WAVE_CYCLES / SQ_BUSY_CYCLES in "
                   "quad-cycles (MI355X_MICROARCH.md), SQ_INSTS_* in wave-instructions. Power: amd-smi metric -p -c, "
                   "1-s samples while the mode runs alone for about 20 s (PROBE_UNITS_PER_WAVE=480).")
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
