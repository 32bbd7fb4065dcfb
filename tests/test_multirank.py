"""Multi-rank (N > 1) path of bench.py on CPU with gloo, world size 2: each rank owns a disjoint
1/N shard of the global record batch (no data-path collective) and the timing is max over ranks."""
import os
import socket

import pytest
import torch.multiprocessing as mp


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
