"""bench.py's roofline bookkeeping on CPU: the committed held-clock and PMC-traffic files name real workloads and the
batch kernels those workloads run on, and lds_roofline prices the LDS model at the held clock (DESIGN.md section 3,
"The LDS ceiling, pinned with counters"; section 5)."""
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = re.compile(r"^mi355x_gcm_(seal|open)_aes(128|256)_k4(_mk)?$")  # _mk: the multi-key batch kernels


def _load(name):
    with open(os.path.join(ROOT, "profiles", name)) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["held_clock.json", "pmc_traffic.json"])
def test_profile_files_name_workloads_and_their_kernels(name):
    import bench
    d = _load(name)
    assert d
    for w, kernels in d.items():
        assert w in bench.WORKLOADS, w
        bits = "128" if bench.WORKLOADS[w]["key"] == 16 else "256"
        for k in kernels:
            m = KERNEL.match(k)
            assert m and m.group(2) == bits, (w, k)


def test_held_clocks_are_plausible_and_sourced():
    for w, kernels in _load("held_clock.json").items():
        for k, v in kernels.items():
            assert 1.0 < v["ghz"] <= 2.45, (w, k, v)
            src = v["source"].split(" ")[0]
            assert os.path.exists(os.path.join(ROOT, src)), (w, k, src)


def test_every_bench_workload_has_a_held_clock():
    import bench
    d = _load("held_clock.json")
    for w, wl in bench.WORKLOADS.items():
        bits = "128" if wl["key"] == 16 else "256"
        mk = "_mk" if wl.get("keys") else ""  # a multi-key workload runs the multi-key batch kernels
        assert {f"mi355x_gcm_seal_aes{bits}_k4{mk}", f"mi355x_gcm_open_aes{bits}_k4{mk}"} <= set(d.get(w, {})), w


def test_lds_roofline_prices_the_model_at_the_held_clock():
    import bench
    k = "mi355x_gcm_seal_aes128_k4"
    ghz = _load("held_clock.json")["16k-aes128"][k]["ghz"]
    nominal = 256 * 2.4 * 64 / 330 * 16  # GB/s of payload at 2.4 GHz: 330 LDS cycles per 64 blocks
    r = bench.lds_roofline(k, 1000.0, "16k-aes128", 16, 133, 16, nominal, 256)
    assert r["held_clock_ghz"] == ghz
    assert r["peak"] == pytest.approx(256 * ghz * 64 / 330 * 16, rel=1e-3)
    assert r["frac"] == pytest.approx(1000.0 / r["peak"], rel=1e-3)
    assert r["frac_nominal_2p4ghz"] == pytest.approx(1000.0 / nominal, rel=1e-3)
    none = bench.lds_roofline(k, 1000.0, "no-such-workload", 16, 133, 16, nominal, 256)
    assert none["peak"] == pytest.approx(nominal, rel=1e-3) and "2.4 GHz" in none["held_clock_source"]


def test_algorithmic_bytes_follow_survey_8d():
    import bench
    # 2845 B per 1400-B seal with a 5-B AAD (16-B descriptor + 8-B seq)
    assert bench.algorithmic_bytes(1400, 1, 5, True) == 2845
    assert bench.algorithmic_bytes(1400, 1, 5, False) == 1400 + 16 + 5 + 24 + 1400 + 4


def test_lds_roofline_prefers_the_live_clock():
    """A clock measured in the run (ClockSampler) prices the model; the builder's counter clock stays beside it."""
    import bench
    k = "mi355x_gcm_seal_aes128_k4"
    nominal = 256 * 2.4 * 64 / 330 * 16
    live = {"gfx_mhz_median": 1913.0, "samples": 40, "source": "amdsmi"}
    r = bench.lds_roofline(k, 1000.0, "16k-aes128", 16, 133, 16, nominal, 256, live)
    assert r["held_clock_ghz"] == pytest.approx(1.913)
    assert r["peak"] == pytest.approx(256 * 1.913 * 64 / 330 * 16, rel=1e-3)
    assert r["live_clock"] is live and r["held_clock_source"].startswith("live")
    assert r["pmc_clock"]["ghz"] == _load("held_clock.json")["16k-aes128"][k]["ghz"]
    off = bench.lds_roofline(k, 1000.0, "16k-aes128", 16, 133, 16, nominal, 256, {"error": "no amdsmi"})
    assert off["frac"] == off["pmc_clock"]["frac"] and "no amdsmi" in off["held_clock_source"]


def test_clock_sampler_reports_why_it_is_off():
    """Without a GPU the sampler never raises: it is off, says why, and its summary carries the reason."""
    import bench
    s = bench.ClockSampler(0)
    with s:
        pass
    summ = s.summary(0.0, 1e12)
    if s.h is None:
        assert s.err and summ["source"] is None and summ["error"]


FAKE_ROCPROF = """#!/usr/bin/env python3
import os, sys
a = sys.argv[1:]
counter, out = a[a.index("--pmc") + 1], a[a.index("-d") + 1]
if os.environ.get("FAKE_ROCPROF_FAIL") == counter:
    sys.exit(3)
os.makedirs(out, exist_ok=True)
v = {"FETCH_SIZE": (1000.0, 1002.0), "WRITE_SIZE": (500.0, 500.0)}[counter]
with open(os.path.join(out, "run_counter_collection.csv"), "w") as f:
    f.write("Kernel_Name,Counter_Name,Counter_Value\\n")
    for x in v:
        f.write(f"mi355x_gcm_seal_aes128_k4,{counter},{x}\\n")
    f.write(f"__amd_rocclr_fillBufferAligned,{counter},7\\n")
"""


def _fake_rocprof(tmp_path, monkeypatch):
    p = tmp_path / "rocprofv3"
    p.write_text(FAKE_ROCPROF)
    p.chmod(0o755)
    monkeypatch.setenv("PATH", f"{tmp_path}:{os.environ['PATH']}")


def test_live_pmc_traffic_from_two_child_passes(tmp_path, monkeypatch):
    """roofline.traffic measured in the run: a FETCH_SIZE and a WRITE_SIZE pass (rocprofv3 children), 2 x FETCH + WRITE
    in bytes per dispatch, averaged over the kernel's dispatches; the builder's committed figure kept beside it."""
    import bench
    _fake_rocprof(tmp_path, monkeypatch)
    monkeypatch.setattr(bench, "_LIVE_PMC_FAILED", [])
    live = bench.live_pmc_traffic("1400")
    assert live == {"mi355x_gcm_seal_aes128_k4": int(2 * 1001.0 * 1024 + 500.0 * 1024)}
    res = {"roofline": {"kernel": "mi355x_gcm_seal_aes128_k4", "traffic": 123, "traffic_source": "builder",
                        "algorithmic_bytes_per_launch": 2_000_000}}
    bench.apply_live_traffic(res, "1400")
    rf = res["roofline"]
    assert rf["traffic"] == live["mi355x_gcm_seal_aes128_k4"] and rf["traffic_builder"] == 123
    assert "measured in this run" in rf["traffic_source"] and rf["traffic_over_algorithmic"] > 1


def test_live_pmc_traffic_failure_keeps_the_builders_figure(tmp_path, monkeypatch):
    import bench
    _fake_rocprof(tmp_path, monkeypatch)
    monkeypatch.setattr(bench, "_LIVE_PMC_FAILED", [])
    monkeypatch.setenv("FAKE_ROCPROF_FAIL", "WRITE_SIZE")
    res = {"roofline": {"kernel": "mi355x_gcm_seal_aes128_k4", "traffic": 123, "traffic_source": "builder",
                        "algorithmic_bytes_per_launch": 2_000_000}}
    bench.apply_live_traffic(res, "1400")
    rf = res["roofline"]
    assert rf["traffic"] == 123 and rf["traffic_source"] == "builder" and "WRITE_SIZE pass" in rf["traffic_live_error"]


def test_live_pmc_traffic_stops_after_a_failed_pass(tmp_path, monkeypatch):
    """One failed pass ends the live passes for the run: the later workloads keep the builder's figure at once."""
    import bench
    _fake_rocprof(tmp_path, monkeypatch)
    monkeypatch.setattr(bench, "_LIVE_PMC_FAILED", [])
    monkeypatch.setenv("FAKE_ROCPROF_FAIL", "FETCH_SIZE")
    assert "FETCH_SIZE pass" in bench.live_pmc_traffic("1400")["error"]
    monkeypatch.delenv("FAKE_ROCPROF_FAIL")
    assert "skipped after an earlier failed pass" in bench.live_pmc_traffic("16k")["error"]
