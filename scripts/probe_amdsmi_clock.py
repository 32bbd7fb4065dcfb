"""What the amdsmi Python API reports while the batch kernels run (diagnostic for a live clock in bench.py; measurement
only).  The parent process never touches HIP: it samples amdsmi's GPU metrics every ~1 ms while a child runs bench.py
on the 16 KiB AES-128 workload for a few seconds, and reports the fields that carry the gfx clock, the socket power and
the activity, their update cadence, and their medians over the busy samples.

    python scripts/probe_amdsmi_clock.py      (GPU box)  -> one JSON line
"""
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    import amdsmi
    amdsmi.amdsmi_init()
    try:
        h = amdsmi.amdsmi_get_processor_handles()[0]
        first = amdsmi.amdsmi_get_gpu_metrics_info(h)
        keys = sorted(k for k in first if any(s in k for s in ("gfxclk", "power", "activity", "energy", "clock_counter")))
        out = {"keys": keys, "first": {k: first[k] for k in keys}}
        try:
            out["clock_info_gfx"] = amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX)
        except Exception as e:  # noqa: BLE001 -- reported
            out["clock_info_gfx"] = f"{type(e).__name__}: {e}"
        child = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "16k-aes128", "--steps",
                                  "400", "--warmup", "2", "--no-cpu-baseline", "--no-e2e", "--no-workloads"],
                                 stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
        samples = []
        t0 = time.time()
        while child.poll() is None and time.time() - t0 < 120:
            m = amdsmi.amdsmi_get_gpu_metrics_info(h)
            samples.append((time.time() - t0, {k: m[k] for k in keys}))
            time.sleep(0.001)
        line = child.communicate()[0].strip().splitlines()
        out["bench"] = json.loads(line[-1]) if line else None
        if out["bench"]:
            out["bench"] = {k: out["bench"][k] for k in ("value", "ms_per_step", "lds_roofline") if k in out["bench"]}
        out["n_samples"] = len(samples)

        def num(v):
            if isinstance(v, list):
                v = [x for x in v if isinstance(x, (int, float))]
                return statistics.mean(v) if v else None
            return v if isinstance(v, (int, float)) else None

        series = {k: [(t, num(s[k])) for t, s in samples] for k in keys}
        summary = {}
        for k, ser in series.items():
            vals = [v for _, v in ser if v is not None]
            changes = sum(1 for (_, a), (_, b) in zip(ser, ser[1:]) if a != b)
            summary[k] = {"median": statistics.median(vals) if vals else None, "min": min(vals) if vals else None,
                          "max": max(vals) if vals else None, "changes": changes}
        out["summary"] = summary
        act = "average_gfx_activity"
        if act in series:
            busy = [i for i, (_, v) in enumerate(series[act]) if v is not None and v >= 90]
            out["busy_samples"] = len(busy)
            out["busy_median"] = {k: statistics.median([series[k][i][1] for i in busy if series[k][i][1] is not None])
                                  for k in keys if busy and any(series[k][i][1] is not None for i in busy)}
        out["raw_head"] = [(round(t, 4), s) for t, s in samples[::max(1, len(samples) // 40)]][:40]
        print(json.dumps(out, default=str))
    finally:
        amdsmi.amdsmi_shut_down()


if __name__ == "__main__":
    main()
