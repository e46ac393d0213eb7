"""world_size-2 gloo run of the multi-GPU exchange (lodestar_amd/dist.py) on
CPU: each rank's 576-byte Miller partial reaches every rank in rank order,
and the shard assignment covers every job exactly once."""
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
    import torch.distributed as dist
    from lodestar_amd.dist import allgather_partials, shard_jobs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    part = bytes([rank + 1]) * 576
    parts = allgather_partials(part, dist)
    shards = shard_jobs([98] * 10, world)
    q.put((rank, [p[0] for p in parts], [len(p) for p in parts], shards[rank]))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_allgather_partials_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=100) for _ in range(world))
    for p in ps:
        p.join(timeout=30)
    for rank, firsts, lens, shard in res:
        assert firsts == [1, 2]
        assert lens == [576, 576]
    assert sorted(res[0][3] + res[1][3]) == list(range(10))
