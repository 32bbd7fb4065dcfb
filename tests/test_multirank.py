"""Multi-rank (N > 1) path of bench.py on CPU with gloo, world size 2: each rank owns a disjoint
1/N shard of the global record batch (no data-path collective) and the timing is max over ranks."""
import os
import socket

import pytest
import torch.multiprocessing as mp
from rapido_amd.hostmem import to_cpu, to_gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = bench.rank_shard(rank, world, 1000)
    spans = [None] * world
    dist.all_gather_object(spans, (first, n))
    t = bench.max_over_ranks(1.0 + rank)
    q.put((rank, spans, t))
    dist.destroy_process_group()


def test_shards_disjoint_and_max_time():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, spans, t in res:
        assert spans == [(0, 1000), (1000, 1000)]
        assert t == 2.0


def test_rank_shard_validates():
    import bench
    with pytest.raises(ValueError):
        bench.rank_shard(2, 2, 10)


def _ragged_worker(rank, world, port, q):
    """Rank `rank` seals its byte-balanced shard of one global ragged batch with the oracle (the CPU
    checker; the GPU ranks run the engine on the same shards) and reports its tags and work."""
    import hashlib

    import numpy as np
    import torch.distributed as dist
    import oracle
    from rapido_amd import records
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(11)
    lengths = rng.integers(0, 3000, 64).astype(np.uint64)
    key, iv = bytes(range(16)), bytes(range(0xA0, 0xAC))
    first, n = records.shard_by_bytes(lengths, np.full(64, 5, np.uint64), world)[rank]
    out = {}
    for i in range(first, first + n):
        pt = hashlib.sha256(b"rec%d" % i).digest() * (int(lengths[i]) // 32 + 1)
        pt = pt[: int(lengths[i])]
        out[i] = oracle.seal(key, oracle.build_iv(iv, i), bytes(records.tls_aad(lengths[i:i + 1])), pt)
    gathered = [None] * world
    dist.all_gather_object(gathered, out)
    q.put((rank, gathered))
    dist.destroy_process_group()


def test_ragged_byte_shards_cover_the_batch():
    import hashlib

    import numpy as np
    import oracle
    from rapido_amd import records
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ragged_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(11)
    lengths = rng.integers(0, 3000, 64).astype(np.uint64)
    key, iv = bytes(range(16)), bytes(range(0xA0, 0xAC))
    for _, gathered in res:
        merged = {}
        for part in gathered:
            assert not set(part) & set(merged)  # shards are disjoint
            merged.update(part)
        assert sorted(merged) == list(range(64))
        for i, sealed in merged.items():
            pt = (hashlib.sha256(b"rec%d" % i).digest() * (int(lengths[i]) // 32 + 1))[: int(lengths[i])]
            assert sealed == oracle.seal(key, oracle.build_iv(iv, i), bytes(records.tls_aad(lengths[i:i + 1])), pt)


def _line_worker(rank, world, port, q, dev_index, same_ok):
    """bench.py's N > 1 bookkeeping on gloo: the rank-to-GPU map check and the per-rank figures gathered for the line."""
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        placement = bench.check_device_map(dev_index(rank), same_ok, 2)
    except SystemExit as e:
        q.put((rank, "exit", str(e)))
        dist.destroy_process_group()
        return
    ranks = bench.gather_rank_stats({"rank": rank, "host": "h", "device": dev_index(rank), "device_name": "gfx950",
                                     "rank_gibps": 100.0 + rank, "rank_ms_per_step": 2.0 - rank, "seal_gibps": 1.0,
                                     "open_gibps": 2.0, "launch_ms": 1.5,
                                     "e2e_pcie": {"seal_gibps_serial": 20.0 + rank, "seal_gibps_pipelined": 30.0 + rank},
                                     "gfx_mhz": 2000.0 + rank, "socket_power_w": 1200 + rank})
    q.put((rank, placement, ranks))
    dist.destroy_process_group()


def _run_line(dev_index, same_ok):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_line_worker, args=(r, world, port, q, dev_index, same_ok)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _dev_per_rank(r):
    return r


def _dev_zero(r):
    return 0


def test_bench_line_per_rank_figures():
    """The N > 1 line carries every rank's own figures (device ordinal, rates, launch time) in rank order."""
    import bench
    for rank, placement, ranks in _run_line(_dev_per_rank, False):
        assert [p[1] for p in placement] == [0, 1]
        assert [r["rank"] for r in ranks] == [0, 1] and [r["device"] for r in ranks] == [0, 1]
        assert all(set(r) == set(bench.RANK_KEYS) | {"e2e_pcie", "gfx_mhz", "socket_power_w"} for r in ranks)
        assert [r["gfx_mhz"] for r in ranks] == [2000.0, 2001.0]  # each GPU's sampled clock rides with its rank
        assert [r["rank_gibps"] for r in ranks] == [100.0, 101.0]
        # each GPU's own PCIe-inclusive rate rides with its rank (north_star: PCIe is per GPU)
        assert [r["e2e_pcie"]["seal_gibps_pipelined"] for r in ranks] == [30.0, 31.0]


def test_bench_refuses_two_ranks_on_one_gpu():
    """Two ranks mapped to one device fail fast unless RAPIDO_BENCH_SAME_DEVICE (the rehearsal) allows it."""
    res = _run_line(_dev_zero, False)
    assert all(r[1] == "exit" and "share a GPU" in r[2] for r in res)
    for rank, placement, ranks in _run_line(_dev_zero, True):
        assert [p[1] for p in placement] == [0, 0] and len(ranks) == 2


@pytest.mark.parametrize("ordinal", [1, 7, -1])
def test_context_on_an_absent_device_fails_cleanly(engine_lib, ordinal):
    """A context asked for on a device ordinal this host does not have (ptls_mi355x_aesgcm_new_on: a rank mapped to
    GPU 7 of a smaller node) is refused with an error naming the ordinal -- never created silently on the current
    device.  Runs without a GPU (there every ordinal is absent)."""
    import rapido_amd as ra
    try:
        import torch
        have = torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        have = 0
    if 0 <= ordinal < have:
        pytest.skip(f"device {ordinal} is present here")
    with pytest.raises(RuntimeError, match=f"device ordinal {ordinal} is not present"):
        ra.Engine(bytes(16), device=ordinal)


@pytest.mark.gpu
def test_contexts_on_each_present_device(gpu):
    """ptls_mi355x_aesgcm_new_on: a context on every present ordinal lives there (seal of one record checked against
    the oracle), the caller's current device is unchanged, and the first absent ordinal is refused cleanly."""
    import numpy as np
    import torch

    import oracle
    import rapido_amd as ra
    n = torch.cuda.device_count()
    cur = torch.cuda.current_device()
    key, iv = bytes(range(16)), bytes(range(12))
    for d in range(n):
        eng = ra.Engine(key, device=d)
        assert eng.device == d and torch.cuda.current_device() == cur
        with torch.cuda.device(d):
            rec = np.zeros(1, ra.RECORD_DTYPE)
            rec[0] = (0, 0, 0, 5, 100, 0)
            src = torch.arange(100, dtype=torch.uint8, device=f"cuda:{d}")
            dst = torch.zeros(116, dtype=torch.uint8, device=f"cuda:{d}")
            d_rec = to_gpu(rec.view(np.uint8).copy(), f"cuda:{d}")
            eng.seal_batch(iv, d_rec.data_ptr(), 1, src.data_ptr(), dst.data_ptr(), src.data_ptr())
            torch.cuda.synchronize(d)
            assert to_cpu(dst).tobytes() == oracle.seal(key, oracle.build_iv(iv, 5), b"", bytes(range(100)))
        eng.close()
    with pytest.raises(RuntimeError, match=f"device ordinal {n} is not present"):
        ra.Engine(key, device=n)
    assert torch.cuda.current_device() == cur


def _place_worker(rank, world, port, q, sysfs):
    """bench.place_rank on gloo, world size 2: each rank's GPU (a fake PCI address per rank in a fake sysfs tree) on
    its own NUMA node; the rank pins itself to that node's CPUs and the fields ride in its line (gather_rank_stats)."""
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    place = bench.place_rank(rank, bus_id=f"0000:0{rank + 1}:00.0", sysfs=sysfs)
    mine = {"rank": rank, "host": "h", "device": rank, "device_name": "gfx950", "rank_gibps": 1.0,
            "rank_ms_per_step": 1.0, "seal_gibps": 1.0, "open_gibps": 1.0, "launch_ms": 1.0,
            "numa_node": place["numa_node"], "cpus": place["cpus"], "pci_bus_id": place["pci_bus_id"]}
    ranks = bench.gather_rank_stats(mine)
    errs = bench.fail_together("verification failed" if rank == 1 else None)
    q.put((rank, place, sorted(os.sched_getaffinity(0)), ranks, errs))
    dist.destroy_process_group()


def test_ranks_placed_on_their_gpus_numa_nodes(tmp_path):
    """every rank's host work sits on its GPU's NUMA node (PCI address -> numa_node ->
    local_cpulist), its line carries numa_node / cpus / pci_bus_id, and a rank's failure reaches every rank."""
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < 2:
        pytest.skip("needs two CPUs")
    half = len(allowed) // 2
    nodes = [allowed[:half], allowed[half:]]
    import bench
    for r in range(2):
        d = tmp_path / f"0000:0{r + 1}:00.0"
        d.mkdir()
        (d / "numa_node").write_text(f"{r}\n")
        (d / "local_cpulist").write_text(bench.cpulist(nodes[r]) + "\n")
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_place_worker, args=(r, world, port, q, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, place, affinity, ranks, errs in res:
        assert place["numa_node"] == rank and place["pinned"] and affinity == nodes[rank]
        assert place["cpus"] == bench.cpulist(nodes[rank])
        assert [r["numa_node"] for r in ranks] == [0, 1]
        assert [r["cpus"] for r in ranks] == [bench.cpulist(n) for n in nodes]
        assert [r["pci_bus_id"] for r in ranks] == ["0000:01:00.0", "0000:02:00.0"]
        assert errs == [None, "verification failed"]  # every rank learns that rank 1 failed


def test_placement_without_a_numa_node_is_reported_not_guessed(tmp_path):
    import bench
    d = tmp_path / "0000:09:00.0"
    d.mkdir()
    (d / "numa_node").write_text("-1\n")
    before = os.sched_getaffinity(0)
    place = bench.place_rank(0, bus_id="0000:09:00.0", sysfs=str(tmp_path))
    assert place["numa_node"] is None and not place["pinned"] and os.sched_getaffinity(0) == before
    assert bench.place_rank(0, bus_id="0000:0a:00.0", sysfs=str(tmp_path))["numa_node"] is None  # no such device
    assert bench.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert bench.cpulist([0, 1, 2, 3, 8, 10, 11]) == "0-3,8,10-11"
