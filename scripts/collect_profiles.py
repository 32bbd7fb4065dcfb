"""Turns a gpurun_out/<TAG> measurement (scripts/gpu_round_bench.sh) into tracked files under profiles/.

    python scripts/collect_profiles.py <TAG> <round-label>

Writes
  profiles/<label>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of `bench.py` (default workload)
  profiles/<label>_bench.jsonl        the bench lines of that run (all workloads)
  profiles/<label>_pmc.json           PMC per kernel: FETCH_SIZE / WRITE_SIZE (separate passes) and SQ counters
  profiles/pmc_traffic.json           HBM bytes per launch for bench.py's roofline.traffic

HBM bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024: on gfx950 FETCH_SIZE reports half the bytes of
a wide (16 B/lane) streaming read and WRITE_SIZE is exact for 16 B/lane stores
(/opt/skills/guides/MI355X_MICROARCH.md, section HBM).
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        if "mi355x_" in r["Kernel_Name"]:
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main(tag, label):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{label}_kernel_stats.csv"))
    for w in ("16k", "16k-aes128", "ragged"):
        p = os.path.join(src, f"trace_{w}", "run_kernel_stats.csv")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, f"{label}_kernel_stats_{w}.csv"))
    with open(os.path.join(dst, f"{label}_bench.jsonl"), "w") as f:
        for name in ("bench_1400.json", "bench_other.jsonl"):
            p = os.path.join(src, name)
            if os.path.exists(p):
                for line in open(p):
                    if line.strip().startswith("{"):
                        f.write(line.strip() + "\n")
    fetch = counters(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = counters(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    sq = counters(os.path.join(src, "pmc_sq", "run_counter_collection.csv"))
    pmc = {}
    traffic = {}
    for k in fetch:
        if "setup" in k:
            continue
        fb = fetch[k]["FETCH_SIZE"] * 1024 * 2
        wb = write.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        pmc[k] = {"FETCH_SIZE_kB": fetch[k]["FETCH_SIZE"], "WRITE_SIZE_kB": write.get(k, {}).get("WRITE_SIZE"),
                  "hbm_bytes_per_launch": int(fb + wb), "sq": sq.get(k, {})}
        traffic[k] = {"hbm_bytes_per_launch": int(fb + wb), "source": f"profiles/{label}_pmc.json"}
    tpath = os.path.join(dst, "pmc_traffic.json")
    allt = json.load(open(tpath)) if os.path.exists(tpath) else {}
    allt["1400"] = traffic
    # other workloads: FETCH / WRITE passes only (scripts/gpu_round_bench.sh)
    others = {}
    for w in ("16k", "16k-aes128", "16k-max", "16k-max-aes128", "ragged"):
        fp = os.path.join(src, f"pmc_fetch_{w}", "run_counter_collection.csv")
        wp = os.path.join(src, f"pmc_write_{w}", "run_counter_collection.csv")
        if not (os.path.exists(fp) and os.path.exists(wp)):
            continue
        fw, ww = counters(fp), counters(wp)
        t = {}
        for k in fw:
            if "setup" in k or "mi355x_gcm_" not in k:
                continue
            b = int(fw[k]["FETCH_SIZE"] * 1024 * 2 + ww.get(k, {}).get("WRITE_SIZE", 0.0) * 1024)
            t[k] = {"hbm_bytes_per_launch": b, "source": f"profiles/{label}_pmc.json"}
            others.setdefault(w, {})[k] = {"FETCH_SIZE_kB": fw[k]["FETCH_SIZE"],
                                           "WRITE_SIZE_kB": ww.get(k, {}).get("WRITE_SIZE"), "hbm_bytes_per_launch": b}
        allt[w] = t
    sq16 = {}
    p16 = os.path.join(src, "pmc_sq_16k-aes128", "run_counter_collection.csv")
    if os.path.exists(p16):
        sq16 = {k: v for k, v in counters(p16).items() if "setup" not in k}
    with open(os.path.join(dst, f"{label}_pmc.json"), "w") as f:
        json.dump({"workload": "1400 (bench.py default)", "correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024",
                   "kernels": pmc, "other_workloads": others, "sq_16k-aes128": sq16}, f, indent=1)
    with open(tpath, "w") as f:
        json.dump(allt, f, indent=1)
    print(json.dumps(pmc, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
