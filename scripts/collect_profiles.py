"""Turns a gpurun_out/<TAG> measurement (scripts/gpu_round_bench.sh) into tracked files under profiles/.

    python scripts/collect_profiles.py <TAG> <round-label>

Writes
  profiles/<label>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of `bench.py` (default workload)
  profiles/<label>_bench.jsonl        the bench lines of that run (all workloads)
  profiles/<label>_pmc.json           PMC per kernel: FETCH_SIZE / WRITE_SIZE (separate passes) and SQ counters
  profiles/pmc_traffic.json           HBM bytes per launch for bench.py's roofline.traffic
  profiles/<label>_launches.json      per-dispatch durations of the engine kernels in every kernel-trace run, the
                                      warmup launches dropped: mean / median / min of the timed launches, and
                                      roofline.frac recomputed from them against the bench line's
  profiles/<label>_clocks.json        GPU-busy cycles (GRBM_GUI_ACTIVE / 8) and LDS busy per batch kernel and workload
  profiles/held_clock.json            the clock held under each kernel: those cycles over its un-profiled launch time
                                      (bench.py's lds_roofline)

    python scripts/collect_profiles.py --clocks-only <TAG> <label>   (scripts/gpu_held_clocks.sh: clocks only)

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
sys.path.insert(0, ROOT)
from bench import WORKLOADS  # noqa: E402  (bench.py imports nothing heavy at module level)


def counters(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        if "mi355x_" in r["Kernel_Name"]:
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def launches(trace_csv, timed):
    """kernel -> durations (ms) of its dispatches in order, from a rocprofv3 --kernel-trace CSV; the last `timed`
    dispatches of each kernel are the timed steps' (bench.py's pre-warm and warmup steps come first)"""
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        if r["Kernel_Name"].startswith("mi355x_"):
            d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    out = {}
    for k, v in d.items():
        t = sorted(v[-timed:]) if len(v) > timed else sorted(v)
        out[k] = {"dispatches": len(v), "warmup_dropped": len(v) - len(t), "timed_mean_ms": round(sum(t) / len(t), 4),
                  "timed_median_ms": round(t[len(t) // 2], 4), "timed_min_ms": round(t[0], 4),
                  "all_ms": [round(x, 4) for x in v]}
    return out


def held_cycles(counter_csv, warmup):
    """kernel -> (median GRBM_GUI_ACTIVE / 8 = GPU-busy cycles of one XCD per dispatch, median clock over the
    profiled dispatch time in GHz), timed dispatches"""
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(counter_csv)):
        if r["Kernel_Name"].startswith("mi355x_") and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            dt = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            d[r["Kernel_Name"]].append((float(r["Counter_Value"]) / 8.0, float(r["Counter_Value"]) / 8.0 / dt))
    out = {}
    for k, v in d.items():
        t = v[warmup:] or v
        out[k] = (sorted(x[0] for x in t)[len(t) // 2], sorted(x[1] for x in t)[len(t) // 2])
    return out


SIDE = ("16k", "16k-aes128", "16k-max", "16k-max-aes128", "ragged", "1400-mk64")


def bench_lines(src):
    lines = {}
    for name in ("bench_1400.json", "bench_other.jsonl"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            for line in open(p):
                if line.strip().startswith("{"):
                    b = json.loads(line)
                    lines[b["config"]["workload"]] = b
    return lines


def launches_all(src, tag, lines):
    """per-launch durations (warmups dropped) of every kernel-trace run, and roofline.frac recomputed from them
    against the bench lines"""
    name_of = {"1400": "trace", **{w: f"trace_{w}" for w in SIDE}}
    la = {}
    for w, d in name_of.items():
        p = os.path.join(src, d, "run_kernel_trace.csv")
        if not os.path.exists(p):
            continue
        ent = {"launches": launches(p, 20 if w == "1400" else 10), "trace": f"gpurun_out/{tag}/{d}"}
        line = lines.get(WORKLOADS[w]["name"])
        if line is not None:
            rf = line["roofline"]
            k = ent["launches"].get(rf["kernel"])
            if k is not None:
                ent["roofline_from_profile"] = {
                    "kernel": rf["kernel"], "algorithmic_bytes_per_launch": rf["algorithmic_bytes_per_launch"],
                    "frac_timed_mean": round(rf["algorithmic_bytes_per_launch"] / (k["timed_mean_ms"] * 1e-3) / 1e9 / rf["peak"], 4),
                    "frac_timed_median": round(rf["algorithmic_bytes_per_launch"] / (k["timed_median_ms"] * 1e-3) / 1e9 / rf["peak"], 4),
                    "bench_line_frac": rf["frac"], "bench_line_launch_ms": rf["launch_ms"]}
        la[w] = ent
    return la


def held_clocks(src, dst, label, lines, la):
    """profiles/<label>_clocks.json (GPU-busy cycles per dispatch of every PMC pass that has GRBM_GUI_ACTIVE) and
    profiles/held_clock.json updated with the clock of each batch kernel"""
    raw, hc = {}, {}
    for w, d in (("1400", "pmc_sq"), ("16k-aes128", "pmc_sq_16k-aes128"), *((w, f"pmc_clk_{w}") for w in SIDE)):
        p = os.path.join(src, d, "run_counter_collection.csv")
        if not os.path.exists(p) or w in hc:
            continue
        line = lines.get(WORKLOADS[w]["name"])
        lds = {k: v.get("SQ_LDS_IDX_ACTIVE") for k, v in counters(p).items()}
        hc[w], raw[w] = {}, {"pass": d}
        for k, (cyc, ghz_prof) in held_cycles(p, 1).items():
            if not k.startswith(("mi355x_gcm_seal_", "mi355x_gcm_open_")):
                continue  # microsecond kernels: GRBM_GUI_ACTIVE spans more than the dispatch, no clock to read
            # the kernel's busy cycles over its UN-profiled launch time (the bench line's HIP events): the clock
            # the chip holds in the benchmark itself; the profiled dispatches run slower (counter collection)
            kt = la.get(w, {}).get("launches", {}).get(k)
            if line is not None and line["roofline"]["kernel"] == k:
                ghz, how = cyc / (line["roofline"]["launch_ms"] * 1e6), "GRBM_GUI_ACTIVE / 8 / bench launch_ms"
            elif kt is not None:  # the other direction: its timed launches in the counter-free kernel trace
                ghz, how = cyc / (kt["timed_mean_ms"] * 1e6), "GRBM_GUI_ACTIVE / 8 / kernel-trace timed mean"
            else:
                ghz, how = ghz_prof, "GRBM_GUI_ACTIVE / 8 / profiled dispatch time"
            raw[w][k] = {"grbm_gui_active_per_xcd": round(cyc), "ghz_profiled_dispatch": round(ghz_prof, 3),
                         "lds_busy": round(lds[k] / 256.0 / cyc, 4) if lds.get(k) else None}
            hc[w][k] = {"ghz": round(ghz, 3), "ghz_profiled_dispatch": round(ghz_prof, 3),
                        "source": f"profiles/{label}_clocks.json ({how})"}
    if hc:
        with open(os.path.join(dst, f"{label}_clocks.json"), "w") as f:
            json.dump(raw, f, indent=1)
        hpath = os.path.join(dst, "held_clock.json")
        allh = json.load(open(hpath)) if os.path.exists(hpath) else {}
        allh.update(hc)
        with open(hpath, "w") as f:
            json.dump(allh, f, indent=1)
    return hc


def clocks_only(tag, label):
    """scripts/gpu_held_clocks.sh: bench lines, kernel traces and GRBM_GUI_ACTIVE passes of the side workloads only"""
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    lines = bench_lines(src)
    with open(os.path.join(dst, f"{label}_bench.jsonl"), "w") as f:
        for b in lines.values():
            f.write(json.dumps(b) + "\n")
    la = launches_all(src, tag, lines)
    with open(os.path.join(dst, f"{label}_launches.json"), "w") as f:
        json.dump(la, f, indent=1)
    print(json.dumps(held_clocks(src, dst, label, lines, la), indent=1))


def main(tag, label):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{label}_kernel_stats.csv"))
    for w in SIDE:
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
        if "setup" in k or "mi355x_gcm_" not in k:
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
    for w in SIDE:
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
    lines = bench_lines(src)
    la = launches_all(src, tag, lines)
    with open(os.path.join(dst, f"{label}_launches.json"), "w") as f:
        json.dump(la, f, indent=1)
    held_clocks(src, dst, label, lines, la)
    print(json.dumps(pmc, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "--clocks-only":
        clocks_only(sys.argv[2], sys.argv[3])
    else:
        main(sys.argv[1], sys.argv[2])
