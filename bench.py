"""Benchmark of the MI355X AES-GCM engine (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload 1400|16k|16k-aes128|ragged|...]
                    [--workloads LIST | --no-workloads] [--no-cpu-baseline] [--no-e2e]

One step = one pass of the hot path over one batch resident in HBM: seal every record
of the batch (ptls_mi355x_seal_batch), then open the sealed batch
(ptls_mi355x_open_batch).  `value` = payload bytes sealed + payload bytes opened by all
ranks / max-over-ranks wall time of the K timed steps, in GiB/s.

Default workload (N=1) is BASELINE.json configs[1]: AES-128-GCM seal+open of 1 M x 1400 B
TLS records (5-byte TLS header AAD, seq = record index, 256-B aligned records).  With
N > 1 (torchrun, one rank per GPU) every rank seals/opens its own 1 M-record shard --
configs[4], 8 M x 1400 B over 8 GPUs -- with no collective on the data path ("weak").

At N=1 the same run also measures, each on its own batch and clock, the other single-GPU configs
(`workloads`): the north-star config (AES-128-GCM, 256 K x 16 KiB), configs[2] (AES-256-GCM,
256 K x 16 KiB) and configs[3] (AES-128-GCM, 1 M records U{64..16384} B, sorted inside the step).

The JSON line also carries
  roofline      -- the dominant kernel's algorithmic HBM bytes per launch / its mean launch
                   time (HIP events on the launch stream) against the 8 TB/s HBM3E peak;
                   `traffic` = HBM bytes per launch from rocprofv3 PMC counters, measured at the end of
                   this run by two child passes of this script under rocprofv3 (FETCH_SIZE,
                   WRITE_SIZE; --no-live-pmc skips them and keeps profiles/pmc_traffic.json's figure);
  cpu_baseline  -- the reference engine (lib/fusion.c, built unmodified into oracle/_ref) with the
                   t/ptlsbench.c methodology: one pinned process per core, CLOCK_PROCESS_CPUTIME_ID,
                   1400 B and 16 KiB, AES-128 and AES-256, 1 core and all usable cores; measured
                   before the GPU is touched.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
DESC_BYTES = 40         # sizeof(ptls_mi355x_record_t): the engine's descriptor (src, dst, aad, seq u64; len, aadlen u32)
# SURVEY.md 8(d)'s algorithmic bytes count a 16-B descriptor plus the 8-B seq per record (2845 B per 1400-B seal); the
# engine's 40-B descriptor reads 16 B more per record, which the roofline does not credit (0.6 % at 1400 B)
SURVEY_DESC_BYTES = 16 + 8
LDS_CLOCK_GHZ = 2.4     # MI355X peak engine clock (the LDS roofline is priced at it, as HBM at its spec peak)
GIB = float(1 << 30)
METRIC = "device-resident AES-GCM GiB/s, 1.4 KB & 16 KiB record batches, 1/2/4/8 GPU"

WORKLOADS = {
    "1400": dict(name="AES-128-GCM seal+open, 1M x 1400 B TLS records", key=16, n=1 << 20, length=1400),
    "16k": dict(name="AES-256-GCM seal+open, 256K x 16 KiB TLS records", key=32, n=1 << 18, length=16384),
    "16k-aes128": dict(name="AES-128-GCM seal+open, 256K x 16 KiB TLS records", key=16, n=1 << 18, length=16384),
    # TLS-max inner plaintext: 16384 data bytes + the content-type byte (lib/picotls.c:636-639), SURVEY.md 8(d)
    "16k-max": dict(name="AES-256-GCM seal+open, 256K x 16385 B TLS-max records", key=32, n=1 << 18, length=16385),
    "16k-max-aes128": dict(name="AES-128-GCM seal+open, 256K x 16385 B TLS-max records", key=16, n=1 << 18,
                           length=16385),
    "ragged": dict(name="AES-128-GCM seal+open, 1M records U{64..16384} B", key=16, n=1 << 20, length=None),
    # multi-key batches (SURVEY.md 8(d) "K distinct keys with a per-record key index"): a server's 64 sessions, each
    # record of a random session, one launch each way (the launch's by-key sort inside the timed step)
    "1400-mk64": dict(name="AES-128-GCM seal+open, 1M x 1400 B TLS records of 64 sessions (per-record key index)",
                      key=16, n=1 << 20, length=1400, keys=64),
}
# the single-GPU configs measured beside `value` at N=1: the north-star config first
SIDE_WORKLOADS = "16k-aes128,16k,ragged,1400-mk64"

CPU_BENCH = os.path.join(ROOT, "oracle", "_ref", "ref_fusion_bench")
PTLSBENCH = os.path.join(ROOT, "oracle", "_ref", "ptlsbench")


def rank_shard(rank: int, world: int, n_per_rank: int):
    """Weak-scaling shard of rank `rank`: records [rank*n, (rank+1)*n) of the global batch (configs[4]:
    8 M x 1400 B over 8 GPUs = 1 M per GPU).  Returns (first global record index == first seq, count).
    Records are independent, so shards need no exchange."""
    if not 0 <= rank < world:
        raise ValueError("bad rank")
    return rank * n_per_rank, n_per_rank


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank float over the process group (the contract's max-over-ranks timing)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def check_device_map(dev_index: int, same_device_ok: bool, device_count: int):
    """Fail fast on a rank-to-GPU map that would measure the wrong thing: a device ordinal the node does not have, or two
    ranks of one host on one GPU (allowed only for the rehearsal, RAPIDO_BENCH_SAME_DEVICE=1).  Collective over the
    process group (all_gather_object); returns every rank's (host, device ordinal)."""
    import socket

    import torch.distributed as dist
    if not same_device_ok and not 0 <= dev_index < device_count:
        raise SystemExit(f"bench: device ordinal {dev_index} but torch.cuda.device_count() is {device_count}")
    world = dist.get_world_size()
    where = [None] * world
    dist.all_gather_object(where, (socket.gethostname(), dev_index))
    if not same_device_ok and len(set(where)) != world:
        raise SystemExit(f"bench: ranks share a GPU {where}; set RAPIDO_BENCH_SAME_DEVICE=1 for a same-device rehearsal")
    return where


RANK_KEYS = ("rank", "host", "device", "device_name", "rank_gibps", "rank_ms_per_step", "seal_gibps", "open_gibps",
             "launch_ms")
# optional per-rank figures carried when present: each GPU's own PCIe-inclusive rate (north_star: PCIe is per GPU), and
# the gfx clock and socket power sampled under its timed steps (ClockSampler: why one GPU of a node lags another)
RANK_OPTIONAL_KEYS = ("e2e_pcie", "gfx_mhz", "socket_power_w", "numa_node", "cpus", "pci_bus_id", "error")


def parse_cpulist(text: str) -> list:
    """The CPUs of a sysfs cpulist ("0-3,8,10-11")."""
    cpus = []
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.extend(range(int(lo), int(hi or lo) + 1))
    return cpus


def cpulist(cpus) -> str:
    """The compact cpulist form of a CPU set (the inverse of parse_cpulist)."""
    out, run = [], []
    for c in sorted(set(cpus)):
        if run and c == run[-1] + 1:
            run.append(c)
            continue
        if run:
            out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
        run = [c]
    if run:
        out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
    return ",".join(out)


def gpu_pci_bus_id(dev_index: int):
    """The GPU's PCI address ("0000:c1:00.0") from torch's device properties (the process's one HIP runtime), or
    None.  (A ctypes load of libamdhip64.so by name would bring in the system's HIP runtime beside torch's bundled
    one: two runtimes in one process.)"""
    try:
        import torch
        pr = torch.cuda.get_device_properties(dev_index)
        return f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
    except Exception:
        return None


def place_rank(dev_index: int, bus_id=None, sysfs: str = "/sys/bus/pci/devices") -> dict:
    """Puts this rank's host work on its GPU's NUMA node (north_star's per-GPU pinned hipMemcpyAsync
    rate): the node from the GPU's PCI address (sysfs numa_node), the process pinned to that node's CPUs (local_cpulist)
    within the CPUs it may use, and later allocations preferring the node's memory (set_mempolicy MPOL_PREFERRED), so the
    pinned staging and e2e_pcie buffers, touched first after this, are node-local.  Returns the fields every rank's line
    carries; a field that could not be had is None (never a guess)."""
    bus_id = bus_id if bus_id is not None else gpu_pci_bus_id(dev_index)
    out = {"pci_bus_id": bus_id, "numa_node": None, "cpus": None, "pinned": False, "mempolicy": None}
    if not bus_id:
        return out
    base = os.path.join(sysfs, bus_id)
    try:
        node = int(open(os.path.join(base, "numa_node")).read().strip())
    except (OSError, ValueError):
        return out
    out["numa_node"] = node if node >= 0 else None  # -1: the platform reports no node
    try:
        local = set(parse_cpulist(open(os.path.join(base, "local_cpulist")).read()))
    except OSError:
        local = set()
    allowed = os.sched_getaffinity(0)
    cpus = sorted(local & allowed)
    if cpus:
        os.sched_setaffinity(0, cpus)
        out["pinned"] = True
        out["cpus"] = cpulist(cpus)
    else:
        out["cpus"] = cpulist(allowed)  # the node's CPUs are not ours to use: left as it was, and said so
    if out["numa_node"] is not None:
        out["mempolicy"] = _prefer_node(out["numa_node"])
    return out


def _prefer_node(node: int) -> str:
    """set_mempolicy(MPOL_PREFERRED, {node}) for this process's later allocations (x86-64 syscall 238)."""
    import ctypes
    if node >= 64:
        return "node beyond the mask"
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        mask = ctypes.c_ulong(1 << node)
        rc = libc.syscall(238, 1, ctypes.byref(mask), 65)  # (MPOL_PREFERRED, nodemask, maxnode)
        return "preferred" if rc == 0 else f"errno {ctypes.get_errno()}"
    except OSError as e:  # pragma: no cover - libc is always there
        return str(e)


class RankFailure(Exception):
    """A rank's own verification failed: reported to every rank with the per-rank figures, then every rank exits."""


def fail_together(mine_error):
    """Every rank learns whether any rank failed (all_gather_object), so no rank waits in a later collective for one
    that has left: returns the per-rank errors (None where a rank passed)."""
    import torch.distributed as dist
    errs = [None] * dist.get_world_size()
    dist.all_gather_object(errs, mine_error)
    return errs


def gather_rank_stats(mine: dict):
    """Every rank's own figures (RANK_KEYS) gathered to every rank, in rank order (all_gather_object), so rank 0's line
    shows which rank lags.  `mine` must hold RANK_KEYS."""
    import torch.distributed as dist
    missing = [k for k in RANK_KEYS if k not in mine]
    if missing:
        raise ValueError(f"rank stats miss {missing}")
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, {k: mine[k] for k in RANK_KEYS + RANK_OPTIONAL_KEYS if k in mine})
    return out


def algorithmic_bytes(lengths_sum: int, n: int, aad_sum: int, seal: bool) -> int:
    """seal = read (L + aad + 8 seq + 16 descriptor) + write (L + 16 tag); open = read (L + 16 tag + aad
    + 8 + 16) + write (L + 4 status).  2845 B per 1400-B seal with the 5-B TLS AAD."""
    if seal:
        return lengths_sum + aad_sum + SURVEY_DESC_BYTES * n + lengths_sum + 16 * n
    return lengths_sum + 16 * n + aad_sum + SURVEY_DESC_BYTES * n + lengths_sum + 4 * n


# ------------------------------------------------------------------------------------------- CPU baseline ----
class ClockSampler:
    """The chip's gfx clock and socket power while a region runs, measured in THIS run: amdsmi's GPU metrics
    (`current_gfxclks`, one value per XCD, and `current_socket_power`; the same source as torch.cuda.clock_rate on
    ROCm) sampled every `period` seconds on a thread that never touches HIP.  The firmware refreshes them about every
    20-30 ms (scripts/probe_amdsmi_clock.py, profiles/r05zk_amdsmi_clock.json).  Off, with the reason, when amdsmi or
    the device's metrics are unavailable, or with RAPIDO_BENCH_NO_CLOCK=1."""

    _init = None  # amdsmi initialised once per process (None: not tried; else the error string or "")

    def __init__(self, dev, period: float = 0.004):
        import threading
        self.samples, self.err, self.h, self.period = [], None, None, period
        self._stop = threading.Event()
        self._thread = None
        try:
            if os.environ.get("RAPIDO_BENCH_NO_CLOCK") == "1":
                raise RuntimeError("disabled (RAPIDO_BENCH_NO_CLOCK=1)")
            import amdsmi
            import torch
            if ClockSampler._init is None:
                try:
                    amdsmi.amdsmi_init()
                    ClockSampler._init = ""
                except Exception as e:  # noqa: BLE001 -- reported in the line
                    ClockSampler._init = f"amdsmi_init: {type(e).__name__}: {e}"
            if ClockSampler._init:
                raise RuntimeError(ClockSampler._init)
            pr = torch.cuda.get_device_properties(dev)
            bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
            self.h = amdsmi.amdsmi_get_processor_handle_from_bdf(bdf)
            self._amdsmi = amdsmi
            self.read()  # fails here, not on the thread, if the metrics are unreadable
        except Exception as e:  # noqa: BLE001 -- reported in the line
            self.err = f"{type(e).__name__}: {e}"
            self.h = None

    def read(self):
        m = self._amdsmi.amdsmi_get_gpu_metrics_info(self.h)
        clks = [c for c in m.get("current_gfxclks") or [] if isinstance(c, (int, float))]
        if not clks and isinstance(m.get("current_gfxclk"), (int, float)):
            clks = [m["current_gfxclk"]]
        pw = m.get("current_socket_power")
        return (sum(clks) / len(clks) if clks else None, pw if isinstance(pw, (int, float)) else None)

    def _run(self):
        while not self._stop.is_set():
            try:
                mhz, w = self.read()
            except Exception:  # noqa: BLE001 -- a missed sample
                mhz, w = None, None
            self.samples.append((time.perf_counter(), mhz, w))
            self._stop.wait(self.period)

    def __enter__(self):
        import threading
        if self.h is not None:
            self._thread = threading.Thread(target=self._run, daemon=True)
            self._thread.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._thread is not None:
            self._thread.join()

    def summary(self, t_from: float, t_to: float) -> dict:
        """Medians over the samples taken in [t_from, t_to] (perf_counter seconds)."""
        import statistics
        if self.h is None:
            return {"source": None, "error": self.err}
        sel = [(c, w) for t, c, w in self.samples if t_from <= t <= t_to and c is not None]
        if not sel:
            return {"source": None, "error": "no sample in the window"}
        clk = [c for c, _ in sel]
        pw = [w for _, w in sel if w is not None]
        return {"gfx_mhz_median": round(statistics.median(clk), 1), "gfx_mhz_min": round(min(clk), 1),
                "gfx_mhz_max": round(max(clk), 1), "socket_power_w_median": statistics.median(pw) if pw else None,
                "samples": len(sel), "window_ms": round((t_to - t_from) * 1e3, 1),
                "source": "amdsmi current_gfxclks (mean of the XCDs) and current_socket_power, sampled in this run"}


def _cgroup_cpus():
    """CPUs' worth of the cgroup v2 quota (cpu.max), or None when unlimited."""
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else float(q) / float(period)
    except (OSError, ValueError):
        return None


def _physical_first(cpus):
    """The CPUs ordered so that distinct physical cores come first (SMT siblings last)."""
    seen, first, rest = set(), [], []
    for c in sorted(cpus):
        try:
            core = (open(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id").read().strip(),
                    open(f"/sys/devices/system/cpu/cpu{c}/topology/core_id").read().strip())
        except OSError:
            core = (c,)
        (rest if core in seen else first).append(c)
        seen.add(core)
    return first + rest, len(first)


def _run_workers(keylen, length, nrec, cpus):
    """One ref_fusion_bench process per CPU, all at once; -> (per-worker results, wall seconds)."""
    t0 = time.perf_counter()
    procs = [subprocess.Popen([CPU_BENCH, str(keylen), str(length), str(nrec), str(c)], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for c in cpus]
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=300)
        if p.returncode != 0:
            raise RuntimeError(f"ref_fusion_bench rc={p.returncode}: {o.strip()[-200:]} {e.strip()[-200:]}")
        outs.append(json.loads(o.strip().splitlines()[-1]))
    return outs, time.perf_counter() - t0


def cpu_baseline(main_key: int, main_length: int) -> dict:
    """The reference lib/fusion.c on this host's cores, t/ptlsbench.c methodology (t/ptlsbench.c:80-175):
    1 core and every usable core (one pinned process each), 1400 B and 16 KiB, AES-128 and AES-256.
    Per worker: CLOCK_PROCESS_CPUTIME_ID rates, as ptlsbench; all cores: the sum of those rates, and the
    wall-clock aggregate (total bytes / wall time of the whole run) beside it."""
    if not os.path.exists(CPU_BENCH):
        return {"value": None, "error": f"{CPU_BENCH} not built (oracle/Makefile needs /root/reference at build time)"}
    avail = sorted(os.sched_getaffinity(0))
    quota = _cgroup_cpus()
    ordered, physical = _physical_first(avail)
    usable = len(avail) if quota is None else max(1, min(len(avail), int(quota + 1e-6)))
    workers = ordered[:usable]
    cpu_model = open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(" :\t")
    configs = {}
    for keylen in (16, 32):
        for length in (1400, 16384):
            target = 1.5e9 if keylen == 16 else 1.0e9  # bytes per worker: ~0.3-0.6 s of CPU time each
            nrec = max(2000, int(target / length))
            one, w1 = _run_workers(keylen, length, nrec, workers[:1])
            alln, wall = _run_workers(keylen, length, nrec, workers)
            r1 = one[0]

            def so(r):  # seal+open bytes per CPU-second of one worker (each record sealed then opened)
                return 2.0 * r["len"] * r["n"] / ((r["encrypt_us"] + r["decrypt_us"]) * 1e-6) / GIB

            cput = sum(so(r) for r in alln)
            wall_agg = 2.0 * length * nrec * len(alln) / wall / GIB
            cpu_frac = sum((r["encrypt_us"] + r["decrypt_us"]) * 1e-6 for r in alln) / (wall * len(alln))
            configs[f"aes{8 * keylen}-{length}"] = {
                "seal_open_gibps_1core": round(so(r1), 3),
                "seal_gibps_1core": round(r1["seal_gibps"], 3), "open_gibps_1core": round(r1["open_gibps"], 3),
                "encrypt_mbps_1core": r1["encrypt_mbps"], "decrypt_mbps_1core": r1["decrypt_mbps"],
                "seal_open_gibps_all_cputime": round(cput, 3),
                "seal_open_gibps_all_wall": round(wall_agg, 3),
                "scaling_cputime": round(cput / so(r1), 2),
                "worker_cpu_time_per_wall": round(cpu_frac, 3),
                "records_per_worker": nrec}
    main = configs[f"aes{8 * main_key}-{main_length}"]
    siblings = len(workers) - min(len(workers), physical)
    note = (f"{len(avail)} CPUs in the affinity mask ({physical} physical cores), cgroup quota "
            f"{'none' if quota is None else f'{quota:g} CPUs'}: {len(workers)} pinned workers ({siblings} on SMT "
            f"siblings).  Per-worker rates use CLOCK_PROCESS_CPUTIME_ID as ptlsbench; the all-core value is their "
            f"sum, and the wall-clock aggregate is given beside it (equal when every worker owns its core: "
            f"worker_cpu_time_per_wall ~ 1).  The round-1 figure (6.4x on 16 threads) summed per-thread WALL "
            f"rates of 16 threads in ONE process, so cgroup throttling and SMT sharing cut it; here each worker "
            f"is its own process pinned to its own core.")
    out = {"value": main["seal_open_gibps_all_cputime"], "unit": "GiB/s", "cores": len(workers), "kind": "reference",
           "value_wall": main["seal_open_gibps_all_wall"], "value_1core": main["seal_open_gibps_1core"],
           "cores_available": len(avail), "physical_cores_available": physical, "cgroup_quota_cpus": quota,
           "cpu": cpu_model, "configs": configs, "scaling_note": note,
           "sample": f"lib/fusion.c (unmodified), t/ptlsbench.c methodology: 1000-record batches sealed then opened, "
                     f"32-B AAD = h[4] with seq, CLOCK_PROCESS_CPUTIME_ID; {len(workers)} pinned processes x "
                     f"~1-1.5 GB each per config; value = AES-{8 * main_key} {main_length} B seal+open, all workers"}
    # what the whole host would do (an extrapolation, not a measurement): every physical core at the measured 1-core
    # rate times the scaling efficiency measured on the cores this process may use (cgroup quota)
    eff = main["scaling_cputime"] / max(1, min(len(workers), physical))
    out["extrapolated_all_physical_cores"] = {
        "value": round(physical * main["seal_open_gibps_1core"] * eff, 1), "unit": "GiB/s", "cores": physical,
        "value_1core": main["seal_open_gibps_1core"], "scaling_efficiency_measured": round(eff, 3),
        "label": f"EXTRAPOLATION, not measured: {physical} physical cores x {main['seal_open_gibps_1core']} GiB/s x "
                 f"{eff:.3f} (the {len(workers)}-worker efficiency); all-core clocks under sustained VAES/VPCLMUL "
                 f"load may lower it further"}
    if os.path.exists(PTLSBENCH):  # configs[0]-style unmodified run (L = 1500, the reference's own CSV)
        try:
            r = subprocess.run([PTLSBENCH], capture_output=True, text=True, timeout=120)
            rows = [ln for ln in r.stdout.splitlines() if ", fusion," in ln]
            out["ptlsbench_unmodified"] = {"rows": rows, "note": "t/ptlsbench.c as shipped: N=1000, L=1500, "
                                                                 "AAD 32 B, 1 core, Mbps = 8 L N / us"}
        except (OSError, subprocess.SubprocessError) as e:
            out["ptlsbench_unmodified"] = {"error": str(e)}
    return out


# ------------------------------------------------------------------------------------------- GPU workload ----
def measure(ra, wl_key, args, dev, rank, world, check):
    """Times one workload: K steps (seal + open of the whole batch) after W warmups; -> result dict."""
    from rapido_amd.hostmem import to_cpu, to_gpu  # pinned copies (rapido_amd/hostmem.py)
    import numpy as np
    import torch
    import torch.distributed as dist
    from rapido_amd import records

    wl = WORKLOADS[wl_key]
    n = wl["n"]
    rng = np.random.default_rng(1 + rank)
    if wl["length"] is None:
        lengths = rng.integers(64, 16385, n).astype(np.uint64)
    else:
        lengths = np.full(n, wl["length"], dtype=np.uint64)
    recs, src_bytes, aad_bytes = records.layout(lengths, np.full(n, 5, dtype=np.uint64), align=256)
    first, n = rank_shard(rank, world, n)
    recs["seq"] = np.arange(n, dtype=np.uint64) + np.uint64(first)
    aad = np.zeros(aad_bytes, dtype=np.uint8)
    aad[: 5 * n] = records.tls_aad(lengths)

    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    d_src = torch.randint(0, 256, (src_bytes,), dtype=torch.uint8, device=dev, generator=gen)
    d_ct = torch.zeros_like(d_src)
    d_pt = torch.zeros_like(d_src)
    d_recs = to_gpu(recs.view(np.uint8), dev)
    d_aad = to_gpu(aad, dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    key = bytes(range(wl["key"]))
    iv = bytes(range(0xA0, 0xAC))
    eng = ra.Engine(key)
    mk = d_kidx = None
    if wl.get("keys"):  # one context and IV per session; every record of a random session
        nk = wl["keys"]
        mk_engines = [eng] + [ra.Engine(bytes((b + 7 * k) & 0xFF for b in range(wl["key"]))) for k in range(1, nk)]
        mk = ra.MultiKey(mk_engines, [bytes((b + k) & 0xFF for b in range(0xA0, 0xAC)) for k in range(nk)])
        d_kidx = to_gpu(rng.integers(0, nk, n).astype(np.int32), dev)
        if args.pipeline != 1:
            raise SystemExit("bench: the multi-key workload runs one launch each way (--pipeline 1)")
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    ragged = wl["length"] is None
    d_order = torch.zeros(n, dtype=torch.int32, device=dev)

    # The step's pipeline: the batch in `chunks` contiguous record ranges, chunk c sealed and then
    # opened on stream c % 2, each stream with its own engine context (work counters, sort scratch).  A persistent batch
    # kernel leaves CUs idle while its last record groups finish; the other stream's launch fills them.  Chunk c's bytes
    # are touched only by its stream, so consecutive steps need no synchronisation either.
    nchunk = max(1, int(args.pipeline))
    nstream = 1 if nchunk == 1 else 2
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(nstream - 1)]
    engs = [eng] + [ra.Engine(key) for _ in range(nstream - 1)]
    bounds = [min(n, (n * c // nchunk + 63) // 64 * 64) for c in range(nchunk)] + [n]
    chunks = [(c % nstream, bounds[c], bounds[c + 1]) for c in range(nchunk) if bounds[c + 1] > bounds[c]]

    def seal_chunk(e, s, r0, cnt):
        rp = d_recs.data_ptr() + r0 * DESC_BYTES
        if mk is not None:  # every session's records in one launch; the by-key device sort in the step, shared with open
            mk.order_by_key(d_kidx.data_ptr() + 4 * r0, cnt, d_order.data_ptr() + 4 * r0, s)
            mk.seal_batch_ordered(rp, d_kidx.data_ptr() + 4 * r0, d_order.data_ptr() + 4 * r0, cnt, d_src.data_ptr(),
                                  d_ct.data_ptr(), d_aad.data_ptr(), s)
        elif ragged:
            # length-binned, longest-first schedule; the device sort is inside the timed step
            e.order_by_length(rp, cnt, d_order.data_ptr() + 4 * r0, s)
            e.seal_batch_ordered(iv, rp, d_order.data_ptr() + 4 * r0, cnt, d_src.data_ptr(), d_ct.data_ptr(),
                                 d_aad.data_ptr(), s)
        else:
            e.seal_batch(iv, rp, cnt, d_src.data_ptr(), d_ct.data_ptr(), d_aad.data_ptr(), s)

    def open_chunk(e, s, r0, cnt):
        rp = d_recs.data_ptr() + r0 * DESC_BYTES
        if mk is not None:
            mk.open_batch_ordered(rp, d_kidx.data_ptr() + 4 * r0, d_order.data_ptr() + 4 * r0, cnt, d_ct.data_ptr(),
                                  d_pt.data_ptr(), d_aad.data_ptr(), d_st.data_ptr() + 4 * r0, s)
        elif ragged:
            e.open_batch_ordered(iv, rp, d_order.data_ptr() + 4 * r0, cnt, d_ct.data_ptr(), d_pt.data_ptr(),
                                 d_aad.data_ptr(), d_st.data_ptr() + 4 * r0, s)
        else:
            e.open_batch(iv, rp, cnt, d_ct.data_ptr(), d_pt.data_ptr(), d_aad.data_ptr(), d_st.data_ptr() + 4 * r0, s)

    def step(ev=None):
        if ev is not None:  # one chunk: HIP events around the step's two launches (the roofline's launch times)
            ev[0].record(stream)
        for si, r0, r1 in chunks:
            seal_chunk(engs[si], streams[si].cuda_stream, r0, r1 - r0)
        if ev is not None:
            ev[1].record(stream)
        for si, r0, r1 in chunks:
            open_chunk(engs[si], streams[si].cuda_stream, r0, r1 - r0)
        if ev is not None:
            ev[2].record(stream)

    def fork(ev):
        ev.record(streams[0])
        for s in streams[1:]:
            s.wait_event(ev)

    def join(ev_list):
        for s, ev in zip(streams[1:], ev_list):
            ev.record(s)
            streams[0].wait_event(ev)

    # untimed pre-warm: the power manager takes ~10-20 ms of load to raise the clock (the first launches of a run are
    # up to 35% slower, profiles/r03zc_launches.json), so steps run for prewarm_ms before the W warmup steps
    sampler = ClockSampler(dev)
    sampler.__enter__()
    t_pre, n_pre = time.perf_counter(), 0
    while (time.perf_counter() - t_pre) * 1e3 < args.prewarm_ms:
        step()
        torch.cuda.synchronize(dev)
        n_pre += 1
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ev_t0 = torch.cuda.Event(enable_timing=True)
    ev_t1 = torch.cuda.Event(enable_timing=True)
    ev_join = [torch.cuda.Event() for _ in streams[1:]]
    sev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)] if nchunk == 1 else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    fork(ev_t0)
    for i in range(args.steps):
        step(sev[i] if sev is not None else None)
    join(ev_join)
    ev_t1.record(streams[0])
    torch.cuda.synchronize(dev)
    t_end = time.perf_counter()
    sampler.__exit__(None, None, None)
    elapsed = t_end - t0
    elapsed_rank = elapsed
    # the clock under this load: the timed region, widened back into the steady pre-warm to hold several of the
    # firmware's 20-30 ms metric refreshes when the region is short
    live_clock = sampler.summary(max(t_pre + 0.2 * (t0 - t_pre), t0 - 0.25), t_end)
    if world > 1:
        dist.barrier()
        elapsed = max_over_ranks(elapsed, dev)
    region_ms = ev_t0.elapsed_time(ev_t1)  # the timed region on the GPU clock (HIP events)

    launches_note = "the timed steps' launches only (HIP events on the launch stream), warmups excluded"
    if sev is None:
        # chunks > 1: launches overlap at their ends, so a launch's own time is taken one launch at a time after the
        # timed region (the whole batch sealed, then opened, on one stream, HIP events around each launch)
        sev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(max(3, min(args.steps, 10)))]
        for ev in sev:
            ev[0].record(stream)
            seal_chunk(eng, sh, 0, n)
            ev[1].record(stream)
            open_chunk(eng, sh, 0, n)
            ev[2].record(stream)
        torch.cuda.synchronize(dev)
        launches_note = f"{len(sev)} launches of the whole batch one at a time after the timed region (HIP events)"
    seal_all = [e[0].elapsed_time(e[1]) for e in sev]
    open_all = [e[1].elapsed_time(e[2]) for e in sev]
    seal_ms, open_ms = float(np.mean(seal_all)), float(np.mean(open_all))

    # correctness after timing: every status verifies and sampled records open back to their plaintext (parity with
    # the reference engine is the test suite's job: tests/test_gpu_*.py against oracle/ and its pinned fixtures)
    st = to_cpu(d_st).view(np.uint32)
    if not (st == recs["len"]).all():
        raise SystemExit(f"bench: open status mismatch ({wl_key}) -- results invalid")
    if check and rank == 0:
        idx = rng.choice(n, size=min(check, n), replace=False)
        for r in recs[idx]:
            a, ln = int(r["src"]), int(r["len"])
            if not torch.equal(d_pt[a:a + ln], d_src[a:a + ln]) or torch.equal(d_ct[a:a + ln], d_src[a:a + ln]):
                raise SystemExit(f"bench: record did not round-trip ({wl_key}) -- results invalid")

    payload = float(lengths.sum())
    value = 2.0 * payload * world * args.steps / elapsed / GIB  # sealed + opened, all ranks
    seal_b = algorithmic_bytes(int(payload), n, 5 * n, True)
    open_b = algorithmic_bytes(int(payload), n, 5 * n, False)
    dom_is_seal = seal_ms >= open_ms
    dom_ms = seal_ms if dom_is_seal else open_ms
    dom_bytes = seal_b if dom_is_seal else open_b
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    # the whole timed region: every launch's algorithmic bytes over the region's HIP-event time (with chunks > 1 the
    # launches overlap at their ends)
    achieved_region = (seal_b + open_b) * args.steps / (region_ms * 1e-3) / 1e9
    kname_of = ra.kernel_name if mk is None else (lambda s_, k_, n_: ra.kernel_name_multikey(s_, k_, n_, False))
    kname = kname_of(dom_is_seal, wl["key"], n)
    chunk_kernels = sorted({kname_of(s, wl["key"], r1 - r0) for s in (True, False) for _, r0, r1 in chunks})

    # HBM bytes per launch from PMC counters: rocprofv3 cannot run inside this process, so this is the builder's
    # counter pass of the same workload and kernel (scripts/collect_profiles.py), labelled as such in the line
    traffic, traffic_source = None, None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            ent = json.load(open(pmc_path)).get(wl_key, {}).get(kname)
            if ent:
                traffic = ent["hbm_bytes_per_launch"]
                traffic_source = ("profiles/pmc_traffic.json: the builder's rocprofv3 PMC pass of this workload and "
                                  "kernel (2 x FETCH_SIZE + WRITE_SIZE), not measured in this run")
        except (ValueError, KeyError):
            traffic = None

    # the kernels' binding resource: LDS-array cycles of the T-table AES + table GHASH reads (16 ds_read_b128 per
    # block from the 8-bit latin tables at K = 4, 32 from the nibble tables)
    # (MI355X_MICROARCH.md LDS table: ds_read_b32 2 clk, ds_read_b128 4 clk per wave)
    b32_reads = 133 if wl["key"] == 16 else 197
    b128_reads = ra.batch_ghash_reads()
    lds_cycles_per_block = (2.0 * b32_reads + 4.0 * b128_reads) / 64.0
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    lds_nominal = ncu * LDS_CLOCK_GHZ * 1e9 / lds_cycles_per_block * 16 / 1e9  # payload GB/s
    dom_payload = payload / (dom_ms * 1e-3) / 1e9
    res = {
        "workload": wl["name"], "records_per_gpu": n, "steps": args.steps, "warmup": args.warmup,
        "prewarm": {"ms": args.prewarm_ms, "steps": n_pre},
        "value": round(value, 2), "unit": "GiB/s", "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "seal_gibps": round(payload / (seal_ms * 1e-3) / GIB, 2),
        "open_gibps": round(payload / (open_ms * 1e-3) / GIB, 2),
        "rank_gibps": round(2.0 * payload * args.steps / elapsed_rank / GIB, 2),
        "rank_ms_per_step": round(elapsed_rank / args.steps * 1e3, 4),
        "pipeline": {"chunks": len(chunks), "streams": nstream, "kernels": chunk_kernels,
                     "region_ms": round(region_ms, 4), "wall_ms": round(elapsed * 1e3, 4)},
        "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                     "traffic_source": traffic_source,
                     "algorithmic_bytes_per_launch": dom_bytes, "launch_ms": round(dom_ms, 4),
                     "algorithmic_bytes_def": "SURVEY.md 8(d): per record seal L + aad + 24 + L + 16, open L + 16 + aad "
                                              "+ 24 + L + 4 (16-B descriptor + 8-B seq); the engine's descriptors are "
                                              "40 B, 16 B per record not credited",
                     "launch_ms_median": round(float(np.median(seal_all if dom_is_seal else open_all)), 4),
                     "launches": launches_note,
                     "region": {"frac": round(achieved_region / HBM_PEAK_GBPS, 4), "achieved": round(achieved_region, 1),
                                "algorithmic_bytes_per_step": seal_b + open_b, "region_ms": round(region_ms, 4),
                                "note": "every launch of the timed region (seal + open, all chunks) over its HIP-event "
                                        "time"}},
        "lds_roofline": lds_roofline(kname, dom_payload, wl_key, wl["key"], b32_reads, b128_reads, lds_nominal, ncu,
                                     live_clock),
    }
    for e in engs[1:]:
        e.close()
    if mk is not None:
        res["sessions"] = {"keys": len(mk), "records_per_key": n // len(mk), "assignment": "uniform random per record",
                           "note": "one launch each way over every session's records (ptls_mi355x_*_batch_multikey_"
                                   "ordered); the by-key device sort (ptls_mi355x_order_by_key) runs once per step, "
                                   "in the timed step, as the ragged workload's length sort does"}
        for e in mk.engines[1:]:
            e.close()
    extra = dict(eng=eng, iv=iv, d_src=d_src, d_ct=d_ct, d_pt=d_pt, d_st=d_st, d_recs=d_recs, d_aad=d_aad, recs=recs,
                 n=n, src_bytes=src_bytes, payload=payload, stream=stream, key=wl["key"])
    return res, extra


def lds_roofline(kname, achieved, wl_key, key, b32_reads, b128_reads, nominal, ncu, live=None):
    """The LDS bound of the batch kernel.  The ceiling is the LDS array busy every cycle: b32_reads x 2 + b128_reads x 4
    array cycles per 64 blocks per CU (MI355X_MICROARCH.md LDS table), which the counters confirm exactly --
    SQ_LDS_IDX_ACTIVE per 64 blocks is 330.0 / 458.0 for the AES-128 / AES-256 read mix alone and 333 / 461 in the
    kernels (profiles/r05e_lds_ceiling.json).  Priced at the clock the chip holds under the kernel in THIS run (`live`:
    amdsmi, ClockSampler), beside the builder's counter-derived figure for the same workload (profiles/held_clock.json:
    GRBM_GUI_ACTIVE / 8 over the kernel's dispatch time) and the nominal 2.4 GHz."""
    cyc = 2.0 * b32_reads + 4.0 * b128_reads
    r = {"bound": "lds", "kernel": kname, "achieved": round(achieved, 1), "unit": "GB/s payload",
         "model": f"{b32_reads} ds_read_b32 + {b128_reads} ds_read_b128 per 16-B block: {cyc:.0f} LDS-array cycles per 64 "
                  f"blocks per CU",
         "ceiling_source": "the LDS array busy every cycle; SQ_LDS_IDX_ACTIVE per 64 blocks equals the model (probe "
                           "330.0 / 458.0, kernels 333 / 461: profiles/r05e_lds_ceiling.json)",
         "frac_meaning": "LDS-array BUSY fraction (achieved / the array busy every cycle at the clock held), not a fraction "
                         "of a demonstrated peak: the highest busy fraction any kernel or probe reached is 0.87-0.91 "
                         "(SQ_LDS_IDX_ACTIVE, profiles/r05e_lds_ceiling.json and the r05x counter pass), so 1.0 has not "
                         "been shown attainable (DESIGN.md section 3, ceiling table)",
         "peak_nominal_2p4ghz": round(nominal, 1), "frac_nominal_2p4ghz": round(achieved / nominal, 4)}
    held = None
    hpath = os.path.join(ROOT, "profiles", "held_clock.json")
    if os.path.exists(hpath):
        try:
            held = json.load(open(hpath)).get(wl_key, {}).get(kname)
        except ValueError:
            held = None
    def peak_at(ghz):
        return ncu * ghz * 1e9 / (cyc / 64.0) * 16 / 1e9

    if held:
        r["pmc_clock"] = {"ghz": held["ghz"], "peak": round(peak_at(held["ghz"]), 1),
                          "frac": round(achieved / peak_at(held["ghz"]), 4), "source": held["source"]}
    if live and live.get("gfx_mhz_median"):
        ghz = live["gfx_mhz_median"] / 1e3
        r.update({"peak": round(peak_at(ghz), 1), "frac": round(achieved / peak_at(ghz), 4),
                  "held_clock_ghz": round(ghz, 3), "held_clock_source": "live: measured in this run",
                  "live_clock": live})
    elif held:
        r.update({"peak": r["pmc_clock"]["peak"], "frac": r["pmc_clock"]["frac"], "held_clock_ghz": held["ghz"],
                  "held_clock_source": held["source"] + " (no live clock: " + str((live or {}).get("error")) + ")"})
    else:
        r.update({"peak": round(nominal, 1), "frac": round(achieved / nominal, 4),
                  "held_clock_source": "none for this kernel and workload: priced at 2.4 GHz"})
    return r


def window_latency(ra, extra, dev):
    """Latency side (not `value`): one rapido send window, 16 x 16 KiB records framed in one launch on the
    window kernels, device-resident, back-to-back launches timed with HIP events."""
    from rapido_amd.hostmem import to_gpu  # pinned copies (rapido_amd/hostmem.py)
    import numpy as np
    import torch
    WIN, FRAG = 16, 16384
    eng, iv, stream = extra["eng"], extra["iv"], extra["stream"]
    t = np.zeros(WIN, ra.TLS_RECORD_DTYPE)
    t["src"] = np.arange(WIN, dtype=np.uint64) * FRAG
    t["dst"] = np.arange(WIN, dtype=np.uint64) * (FRAG + 22)
    t["seq"] = np.arange(WIN, dtype=np.uint64)
    t["len"], t["type"] = FRAG, 23
    d_t = to_gpu(t.view(np.uint8), dev)
    d_wire = torch.zeros(WIN * (FRAG + 22), dtype=torch.uint8, device=dev)

    def window():
        eng.tls_seal_records(iv, d_t.data_ptr(), WIN, extra["d_src"].data_ptr(), d_wire.data_ptr(), stream.cuda_stream)

    for _ in range(5):
        window()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(stream)
    for _ in range(100):
        window()
    ev[1].record(stream)
    torch.cuda.synchronize(dev)
    return {"us_per_window": round(ev[0].elapsed_time(ev[1]) * 10.0, 2),
            "kernel": ra.kernel_name(True, extra["key"], WIN, framing=True),
            "window": f"{WIN} x {FRAG} B TLS records sealed in one launch (rapido send window), "
                      f"AES-{8 * extra['key']}, device-resident, 100 back-to-back launches"}


def e2e_pcie(ra, extra, dev, steps):
    """PCIe-inclusive: records start and end in pinned host memory (never `value`)."""
    import numpy as np
    import torch
    eng, iv, recs, n = extra["eng"], extra["iv"], extra["recs"], extra["n"]
    d_src, d_ct, d_recs, d_aad = extra["d_src"], extra["d_ct"], extra["d_recs"], extra["d_aad"]
    sh = extra["stream"].cuda_stream
    h_src = torch.empty(extra["src_bytes"], dtype=torch.uint8, pin_memory=True)
    h_dst = torch.empty(extra["src_bytes"], dtype=torch.uint8, pin_memory=True)
    h_src.copy_(d_src)  # device -> pinned: no pageable intermediate (rapido_amd/hostmem.py)
    torch.cuda.synchronize(dev)
    reps = max(2, steps // 4)
    t0 = time.perf_counter()
    for _ in range(reps):  # serial: one H2D, the seal, one D2H
        d_src.copy_(h_src, non_blocking=True)
        eng.seal_batch(iv, d_recs.data_ptr(), n, d_src.data_ptr(), d_ct.data_ptr(), d_aad.data_ptr(), sh)
        h_dst.copy_(d_ct, non_blocking=True)
    torch.cuda.synchronize(dev)
    serial = (time.perf_counter() - t0) / reps
    # pipelined: the batch in chunks over 3 streams, so the H2D of chunk i+1 and the D2H of chunk i-1
    # overlap the seal of chunk i (the copy engines run both directions at once)
    nchunk = 16
    bounds = np.linspace(0, n, nchunk + 1).astype(np.int64)
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    starts = recs["src"].astype(np.int64)
    ends = starts + recs["len"].astype(np.int64) + 16

    def pipelined():
        for c in range(nchunk):
            r0, r1 = int(bounds[c]), int(bounds[c + 1])
            a, b = int(starts[r0]), int(ends[r1 - 1])
            st = streams[c % 3]
            with torch.cuda.stream(st):
                d_src[a:b].copy_(h_src[a:b], non_blocking=True)
                eng.seal_batch(iv, d_recs.data_ptr() + r0 * DESC_BYTES, r1 - r0, d_src.data_ptr(), d_ct.data_ptr(),
                               d_aad.data_ptr(), st.cuda_stream)
                h_dst[a:b].copy_(d_ct[a:b], non_blocking=True)

    pipelined()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        pipelined()
    torch.cuda.synchronize(dev)
    piped = (time.perf_counter() - t0) / reps
    if not torch.equal(h_dst[: int(ends[-1])].to(dev), d_ct[: int(ends[-1])]):  # compared on the device (pinned H2D)
        raise SystemExit("bench: pipelined PCIe seal differs from the device-resident seal -- results invalid")
    # the receive side: the sealed records (h_dst) in, opened, plaintexts and statuses back into pinned host memory
    d_pt, d_st = extra["d_pt"], extra["d_st"]
    h_pt = torch.empty(extra["src_bytes"], dtype=torch.uint8, pin_memory=True)
    h_st = torch.empty(n, dtype=torch.int32, pin_memory=True)

    def pipelined_open():
        for c in range(nchunk):
            r0, r1 = int(bounds[c]), int(bounds[c + 1])
            a, b = int(starts[r0]), int(ends[r1 - 1])
            st = streams[c % 3]
            with torch.cuda.stream(st):
                d_ct[a:b].copy_(h_dst[a:b], non_blocking=True)
                eng.open_batch(iv, d_recs.data_ptr() + r0 * DESC_BYTES, r1 - r0, d_ct.data_ptr(), d_pt.data_ptr(),
                               d_aad.data_ptr(), d_st.data_ptr() + 4 * r0, st.cuda_stream)
                h_pt[a:b].copy_(d_pt[a:b], non_blocking=True)
                h_st[r0:r1].copy_(d_st[r0:r1], non_blocking=True)

    pipelined_open()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        pipelined_open()
    torch.cuda.synchronize(dev)
    piped_open = (time.perf_counter() - t0) / reps
    if not (h_st.numpy().view(np.uint32) == recs["len"]).all():
        raise SystemExit("bench: pipelined PCIe open did not verify every record -- results invalid")
    for i in np.linspace(0, n - 1, 64).astype(np.int64):  # plaintexts back in host memory
        a, ln = int(starts[i]), int(recs["len"][i])
        if not torch.equal(h_pt[a:a + ln], h_src[a:a + ln]):
            raise SystemExit("bench: pipelined PCIe open returned other plaintext -- results invalid")
    return {"seal_gibps_serial": round(extra["payload"] / serial / GIB, 2),
            "seal_gibps_pipelined": round(extra["payload"] / piped / GIB, 2),
            "open_gibps_pipelined": round(extra["payload"] / piped_open / GIB, 2),
            "note": "pinned host src -> H2D -> seal -> D2H -> pinned host dst; serial = one copy each way "
                    "around one launch; pipelined = 16 chunks over 3 streams; open: the sealed records in, "
                    "plaintexts and statuses out, pipelined the same way"}


def record_layer_stream(key_bytes: int = 16, nwin: int = 64, depth: int = 4, transport: str = "dma_in",
                        per_launch=(8, 1)):
    """Host-to-host side figure (never `value`): rapido send and receive windows (16 x 16 KiB records, lib/rapido.c
    :2115-2126) through the asynchronous record layer (include/ptls_mi355x.h section 5) on registered host buffers,
    `depth` launches in flight, each launch carrying the windows of `per_launch` connections of a session
    (record_layer_seal_submit / open_submit over that many layers, as rapido's loop keeps many connections' windows
    moving, lib/rapido.c:2176-2301).  dma_in (PTLS_MI355X_RECORD_LAYER_DMA_IN): the inputs reach device memory by
    DMA, the kernels write the wire records / the delivery kernel the plaintexts in place; direct: the kernels also
    read the inputs in place over PCIe.  Driven from C (scripts/rl_stream.c); timed on the host clock from the first
    submit to the last wait; every opened window is compared with its fragments.  *_sync: one launch at a time."""
    exe = os.path.join(ROOT, "scripts", "_build", "rl_stream")

    def run(tr, *extra, d=depth):
        r = subprocess.run([exe, str(nwin), str(d), str(key_bytes), tr, *map(str, extra)],
                           capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            raise SystemExit("bench: record-layer stream failed -- " + r.stderr.strip())
        return json.loads(r.stdout.strip().splitlines()[-1])

    res = run(transport, per_launch[0])
    # one connection: its consecutive windows, `per_launch[0]` of them per launch (the layer given that many times)
    res["one_connection"] = run(transport, per_launch[0], "one")
    res["one_window_per_launch"] = run(transport, per_launch[1])
    # one window per submit with more windows outstanding: the layer coalesces its queued windows (round 4)
    res["one_window_per_submit_coalesced"] = {f"depth_{d}": run(transport, 1, d=d) for d in (16, 32)}
    res["inputs_read_in_place"] = run("direct", per_launch[0])
    res["note"] = (f"{nwin} back-to-back windows of 16 x 16384 B records, AES-{8 * key_bytes}, host memory to host "
                   f"memory (registered buffers, {transport}), {per_launch[0]} connections' windows per launch, {depth} "
                   "launches in flight (record_layer_seal_submit / open_submit + wait), C driver scripts/rl_stream.c; "
                   f"*_sync: one launch at a time; one_connection: {per_launch[0]} consecutive windows of a single "
                   "connection per launch; one_window_per_launch: a single connection's windows, one per submit, 4 "
                   "outstanding (four single-window launches); one_window_per_submit_coalesced: one per submit with 16 / 32 "
                   "outstanding, coalesced by the layer into ceil(outstanding / 4)-window launches; "
                   "inputs_read_in_place: transport direct (kernels read the inputs over PCIe)")
    return res


_LIVE_PMC_FAILED = []  # the first failed pass: later workloads skip their passes (a bounded bench on any box)


def live_pmc_traffic(workload: str, timeout_s: float = 90.0) -> dict:
    """HBM bytes per launch of `workload`'s kernels measured on THIS box in THIS run: two child passes of this script
    under rocprofv3 (FETCH_SIZE, then WRITE_SIZE: their TCC counters do not fit one pass), 2 steps each, bytes =
    2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 per dispatch (gfx950: FETCH_SIZE reports half of a 16 B/lane streaming
    read; MI355X_MICROARCH.md, HBM section), averaged over the kernel's dispatches.  The children run after every
    timed region of this process.  -> {kernel: bytes} or {"error": ...}."""
    import csv
    import shutil
    import signal
    import tempfile
    if _LIVE_PMC_FAILED:
        return {"error": f"skipped after an earlier failed pass ({_LIVE_PMC_FAILED[0]})"}
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        _LIVE_PMC_FAILED.append("rocprofv3 not found")
        return {"error": "rocprofv3 not found"}
    tmp = tempfile.mkdtemp(prefix="rapido_pmc_")
    env = dict(os.environ, TMPDIR=tmp)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    per = {}
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(tmp, counter)
            cmd = [prof, "--pmc", counter, "--kernel-trace", "-d", out, "-o", "run", "--output-format", "csv", "--",
                   sys.executable, os.path.abspath(__file__), "--workload", workload, "--steps", "2", "--warmup", "1",
                   "--prewarm-ms", "0", "--check", "0", "--no-cpu-baseline", "--no-e2e", "--no-workloads",
                   "--no-live-pmc"]
            p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                 start_new_session=True)
            try:
                _, err = p.communicate(timeout=timeout_s)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)  # the child's own process group (rocprofv3 and the bench under it)
                p.wait()
                _LIVE_PMC_FAILED.append(f"{counter} pass of {workload} timed out")
                return {"error": f"{counter} pass timed out after {timeout_s:.0f} s"}
            path = os.path.join(out, "run_counter_collection.csv")
            if p.returncode != 0 or not os.path.exists(path):
                tail = (err or b"").decode(errors="replace").strip().splitlines()[-1:]
                _LIVE_PMC_FAILED.append(f"{counter} pass of {workload}: exit {p.returncode}")
                return {"error": f"{counter} pass: exit {p.returncode} {tail}"}
            vals = {}
            for r in csv.DictReader(open(path)):
                if r["Kernel_Name"].startswith("mi355x_") and r["Counter_Name"] == counter:
                    vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
            for k, v in vals.items():
                per.setdefault(k, {})[counter] = sum(v) / len(v)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return {k: int(2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024) for k, c in per.items()
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c}


def apply_live_traffic(res: dict, workload: str) -> None:
    """roofline.traffic of a result from live_pmc_traffic; the builder's committed figure stays beside it."""
    rf = res["roofline"]
    live = live_pmc_traffic(workload)
    if "error" in live or rf["kernel"] not in live:
        rf["traffic_live_error"] = live.get("error", f"no counters for {rf['kernel']}")
        return
    rf["traffic_builder"], rf["traffic_builder_source"] = rf["traffic"], rf["traffic_source"]
    rf["traffic"] = live[rf["kernel"]]
    rf["traffic_source"] = ("measured in this run on this GPU: rocprofv3 --pmc child passes of this workload "
                            "(FETCH_SIZE, WRITE_SIZE), 2 x FETCH_SIZE + WRITE_SIZE bytes per launch of the kernel")
    rf["traffic_over_algorithmic"] = round(rf["traffic"] / rf["algorithmic_bytes_per_launch"], 4)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--prewarm-ms", type=float, default=300.0,
                    help="untimed steps run for this long before the warmup steps (clock ramp)")
    ap.add_argument("--workload", default="1400", choices=sorted(WORKLOADS))
    ap.add_argument("--workloads", default=SIDE_WORKLOADS,
                    help="comma-separated side workloads measured at N=1 after the main one")
    ap.add_argument("--no-workloads", action="store_true", help="measure the main workload only")
    ap.add_argument("--side-steps", type=int, default=10, help="timed steps of each side workload")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="chunks of the batch per step, alternating over two streams (1: one stream, one launch each; "
                         "2 measured +0.1..1.9%%, profiles/r04a_pipeline_ab.jsonl)")
    ap.add_argument("--lanes", type=int, default=0, help="lanes per record (1/2/4/8); 0 = engine default")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e", action="store_true", help="(the default) time the PCIe-inclusive path, every rank")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive path")
    ap.add_argument("--check", type=int, default=64, help="records checked to round-trip after timing")
    ap.add_argument("--no-live-pmc", action="store_true",
                    help="at N=1, skip the rocprofv3 PMC child passes that measure roofline.traffic in this run")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    wl = WORKLOADS[args.workload]

    # the CPU baseline runs first: its worker processes start before this process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(wl["key"], wl["length"] or 8224)

    import torch
    import torch.distributed as dist

    import rapido_amd as ra

    # rehearsal only (a 1-GPU box): RAPIDO_BENCH_SAME_DEVICE=1 puts every rank on cuda:0 and
    # RAPIDO_BENCH_BACKEND=gloo replaces RCCL, which refuses two ranks on one GPU
    dev_index = 0 if os.environ.get("RAPIDO_BENCH_SAME_DEVICE") == "1" else local_rank
    if world > 1:
        torch.cuda.set_device(dev_index)
        backend = os.environ.get("RAPIDO_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
    device_count = torch.cuda.device_count()
    placement = None
    if world > 1:
        placement = check_device_map(dev_index, os.environ.get("RAPIDO_BENCH_SAME_DEVICE") == "1", device_count)
    dev = torch.device("cuda", dev_index if world > 1 else 0)
    torch.cuda.set_device(dev)
    ra.require_gpu()
    if args.lanes:
        ra.set_lanes_per_record(args.lanes)
    # this rank's host work on its GPU's NUMA node, before the measured path allocates and touches host buffers
    host_place = place_rank(dev.index if dev.index is not None else 0)

    # At N > 1 a rank whose own verification fails (SystemExit) does not leave alone: its error is gathered with every
    # other rank's (fail_together) before any later collective, and all ranks exit together.
    my_error = None
    try:
        res, extra = measure(ra, args.workload, args, dev, rank, world, args.check)
    except SystemExit as e:
        if world == 1:
            raise
        my_error, res, extra = str(e), None, None
    if world > 1:  # every rank, at the same point: learn whether any rank failed
        errs = fail_together(my_error)
        if any(errs):
            raise SystemExit(f"bench: rank(s) failed: {[(r, m) for r, m in enumerate(errs) if m]}")
    out = {
        "metric": METRIC,
        "value": res["value"],
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "prewarm": res["prewarm"],
        "ms_per_step": res["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-generated random payload, TLS 1.3 record headers as AAD)",
        "config": {"workload": wl["name"], "records_per_gpu": res["records_per_gpu"],
                   "record_bytes": wl["length"] if wl["length"] else "U{64..16384}",
                   "aad_bytes": 5, "key_bits": 8 * wl["key"], "lanes_per_record": ra.lib().ptls_mi355x_get_lanes_per_record(),
                   "parallelism": f"records sharded per GPU x{world}, no collective"},
        "seal_gibps": res["seal_gibps"],
        "open_gibps": res["open_gibps"],
        "roofline": res["roofline"],
        "lds_roofline": res["lds_roofline"],
        "pipeline": res["pipeline"],
        "build_id": ra.build_id(),
        "build_id_matches_sources": ra.build_id() == ra.source_build_id(),
    }
    out["device_count"] = device_count
    out["host_placement"] = host_place
    if world == 1 and not args.no_e2e:
        out["window_latency"] = window_latency(ra, extra, dev)
    e2e = None
    if not args.no_e2e:  # every rank at N > 1: each GPU's own link, all ranks at once (after the timed steps)
        try:
            e2e = e2e_pcie(ra, extra, dev, args.steps)
        except SystemExit as e:
            if world == 1:
                raise
            my_error = str(e)
        out["e2e_pcie"] = e2e
    if world > 1:
        errs = fail_together(my_error)
        if any(errs):
            raise SystemExit(f"bench: rank(s) failed: {[(r, m) for r, m in enumerate(errs) if m]}")
        import socket
        mine = {"rank": rank, "host": socket.gethostname(), "device": dev_index,
                "device_name": torch.cuda.get_device_name(dev), "rank_gibps": res["rank_gibps"],
                "rank_ms_per_step": res["rank_ms_per_step"], "seal_gibps": res["seal_gibps"],
                "open_gibps": res["open_gibps"], "launch_ms": res["roofline"]["launch_ms"],
                "gfx_mhz": res["lds_roofline"].get("live_clock", {}).get("gfx_mhz_median"),
                "socket_power_w": res["lds_roofline"].get("live_clock", {}).get("socket_power_w_median"),
                "numa_node": host_place["numa_node"], "cpus": host_place["cpus"],
                "pci_bus_id": host_place["pci_bus_id"]}
        if e2e is not None:
            mine["e2e_pcie"] = {k: e2e[k] for k in ("seal_gibps_serial", "seal_gibps_pipelined",
                                                     "open_gibps_pipelined")}
        out["ranks"] = gather_rank_stats(mine)
        out["placement"] = [list(p) for p in placement]
        if e2e is not None:
            out["e2e_pcie"] = dict(e2e, note=e2e["note"] + "; rank 0's figure here, every rank's in `ranks`, all ranks "
                                   "copying at once (each GPU on its own PCIe link, one host)")
    if world == 1 and not args.no_e2e:
        out["record_layer_stream"] = record_layer_stream(16)
    extra["eng"].close()
    del extra
    torch.cuda.empty_cache()

    if world == 1 and not args.no_workloads:
        side = {}
        sargs = argparse.Namespace(**vars(args))
        sargs.steps, sargs.warmup = args.side_steps, max(1, min(args.warmup, 2))
        for w in [x for x in args.workloads.split(",") if x and x != args.workload]:
            r, ex = measure(ra, w, sargs, dev, rank, world, min(args.check, 16))
            r["config_key"] = w
            side[w] = r
            ex["eng"].close()
            del ex
            torch.cuda.empty_cache()
        out["workloads"] = side

    # HBM traffic measured here, after every timed region: PMC child passes under rocprofv3 (N=1 only)
    if world == 1 and not args.no_live_pmc:
        apply_live_traffic(out, args.workload)
        for w, r in out.get("workloads", {}).items():
            apply_live_traffic(r, w)

    if cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
