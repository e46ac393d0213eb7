"""world_size-2 gloo runs of the multi-GPU path (lodestar_amd/dist.py) on CPU:
the 576-byte Miller partials reach every rank in rank order, the shard
assignment covers every job exactly once, and the per-job verdicts of a node
batch are reassembled on every rank, both when the combined check passes and
when one shard holds a bad job (SURVEY §8e "Failure": the shards localise
with their own final exponentiations, then the verdicts are all-gathered).

The device is a stand-in with the bgv_partial / bgv_combine_final /
bgv_partial_finish contract (include/bgv.h); the arithmetic behind it is
covered by the GPU tests."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeShardDevice:
    """bgv_partial contract over known per-job outcomes: the partial encodes
    whether the shard's non-rejected jobs all verify; combine_final is the AND
    over the gathered partials; partial_finish reports the per-job outcomes."""

    def __init__(self, truth):
        self.truth = np.asarray(truth, np.int32)
        self.finished = 0

    def partial(self, arrays, on_device=False):
        t = self.truth[np.asarray(arrays["jobs"], np.int64)]
        ok_pairing = bool(((t == 1) | (t < 0)).all())
        part = bytes([1 if ok_pairing else 0]) * 576
        prov = np.where(t < 0, t, 1).astype(np.int32)
        self._t = t
        return part, np.zeros(0, np.int32), prov, bool((t >= 0).all())

    def combine_final(self, parts):
        return all(p[0] == 1 for p in parts)

    def partial_finish(self):
        self.finished += 1
        return self._t.copy()


# ten blocks: sets and pubkey references (with and without the 512-key sync
# aggregate, one near-empty block); shards are balanced by dist.job_work
JOB_SETS = [98, 98, 97, 98, 97, 98, 98, 97, 98, 2]
JOB_REFS = [95 * 128 + 514, 95 * 128 + 514, 95 * 128 + 2, 95 * 128 + 514, 95 * 64 + 2, 95 * 128 + 514,
            95 * 160 + 514, 95 * 128 + 2, 95 * 128 + 514, 2]


def _worker(rank, world, port, q, truth):
    import torch.distributed as dist
    from lodestar_amd.dist import allgather_partials, gather_job_results, job_work, shard_jobs, verify_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    part = bytes([rank + 1]) * 576
    parts = allgather_partials(part, dist)
    shards = shard_jobs(job_work(JOB_SETS, JOB_REFS), world)
    out = {"firsts": [p[0] for p in parts], "lens": [len(p) for p in parts], "shard": shards[rank]}
    for name, t in truth.items():
        dev = FakeShardDevice(t)
        valid, local = verify_sharded(dev, {"jobs": shards[rank]}, dist)
        full = gather_job_results(local, shards, len(t), dist)
        out[name] = (valid, full.tolist(), dev.finished)
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_sharded_verdicts_gloo_world2():
    world = 2
    truth = {
        "all_valid": [1] * 10,
        "one_false": [1, 1, 1, 1, 1, 1, 0, 1, 1, 1],       # a wrong-message block on one shard
        "rejected_and_false": [1, -3, 1, 1, 1, 1, 1, 1, 0, 1],  # a not-in-G2 block plus a false one
        "rejected_only": [1, 1, 1, 1, -8, 1, 1, 1, 1, 1],   # parse error: pairing check still passes
    }
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, truth)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=150) for _ in range(world))
    for p in ps:
        p.join(timeout=30)
    for rank in range(world):
        o = res[rank]
        assert o["firsts"] == [1, 2] and o["lens"] == [576, 576]
        for name, t in truth.items():
            valid, full, finished = o[name]
            assert full == t, (rank, name)
            want_valid = all(x == 1 or x < 0 for x in t)
            assert valid == want_valid
            assert finished == (0 if want_valid else 1)  # localisation only after a failed combined check
    assert sorted(res[0]["shard"] + res[1]["shard"]) == list(range(10))
    from lodestar_amd.dist import job_work
    w = job_work(JOB_SETS, JOB_REFS)
    loads = [sum(w[j] for j in res[r]["shard"]) for r in range(world)]
    assert max(loads) - min(loads) <= max(w)  # whole jobs: at most one job apart


class FakeStepDevice(FakeShardDevice):
    """one context of several in flight: the batch carries its own truth"""

    def __init__(self):
        super().__init__([])

    def partial(self, arrays, on_device=False):
        self.truth = np.asarray(arrays["truth"], np.int32)
        return super().partial(arrays, on_device)


STEP_TRUTHS = [
    [1] * 10,
    [1, 1, 1, 1, 1, 1, 0, 1, 1, 1],
    [1, -3, 1, 1, 1, 1, 1, 1, 0, 1],
    [1] * 10,
    [1, 1, 1, 1, -8, 1, 1, 1, 1, 1],
    [0] + [1] * 9,
    [1] * 10,
]


def _worker_in_flight(rank, world, port, q, depth):
    """dist.run_in_flight: `depth` contexts per rank, the device work on worker
    threads, the exchanges of every step on the main thread in step order"""
    from concurrent.futures import ThreadPoolExecutor

    import torch.distributed as dist
    from lodestar_amd.dist import combine_sharded, gather_job_results, job_work, run_in_flight, shard_jobs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shards = shard_jobs(job_work(JOB_SETS, JOB_REFS), world)
    devs = [FakeStepDevice() for _ in range(depth)]
    got, submitted, finished = {}, [], []
    ex = ThreadPoolExecutor(max_workers=depth)

    def submit(k):
        submitted.append(k)
        assert k - len(finished) <= depth  # never more than `depth` outstanding
        return ex.submit(devs[k % depth].partial, {"jobs": shards[rank], "truth": STEP_TRUTHS[k]})

    def finish(k, res):
        finished.append(k)
        valid, local = combine_sharded(devs[k % depth], res, dist)
        got[k] = (valid, gather_job_results(local, shards, 10, dist).tolist())
        return valid

    ok = run_in_flight(submit, finish, len(STEP_TRUTHS), depth)
    ex.shutdown()
    q.put((rank, {"ok": ok, "got": got, "order": finished, "submitted": submitted}))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("depth", [1, 3])
def test_in_flight_sharded_steps_gloo_world2(depth):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_in_flight, args=(r, world, port, q, depth)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=150) for _ in range(world))
    for p in ps:
        p.join(timeout=30)
    for rank in range(world):
        o = res[rank]
        assert o["order"] == list(range(len(STEP_TRUTHS)))  # finished in step order
        assert o["submitted"] == list(range(len(STEP_TRUTHS)))
        for k, t in enumerate(STEP_TRUTHS):
            valid, full = o["got"][k]
            assert full == t, (rank, k)
            assert valid == all(x == 1 or x < 0 for x in t)
        assert o["ok"] == all(all(x == 1 or x < 0 for x in t) for t in STEP_TRUTHS)


def test_run_in_flight_order_and_depth():
    """single process: at most `depth` outstanding, finishes in order, AND of the finishes"""
    from concurrent.futures import Future

    from lodestar_amd.dist import run_in_flight
    live, peak, done = set(), [0], []

    def submit(k):
        live.add(k)
        peak[0] = max(peak[0], len(live))
        f = Future()
        f.set_result(k * k)
        return f

    def finish(k, r):
        live.discard(k)
        done.append((k, r))
        return k != 4

    assert run_in_flight(submit, finish, 9, 3) is False
    assert done == [(k, k * k) for k in range(9)] and peak[0] == 3
    done.clear()
    assert run_in_flight(submit, lambda k, r: done.append(k) or True, 0, 2) is True and done == []


def test_select_jobs_rebases_offsets():
    from lodestar_amd.dist import select_jobs
    arrays = {"n_sets": 5, "n_jobs": 3, "job_offsets": np.array([0, 2, 3, 5], np.uint32),
              "pk_offsets": np.array([0, 2, 3, 6, 7, 9], np.uint32),
              "pk_indices": np.arange(9, dtype=np.uint32) + 100,
              "msgs": np.arange(5 * 32, dtype=np.uint8).reshape(5, 32),
              "sigs": np.zeros((5, 192), np.uint8), "sig_len": np.full(5, 96, np.uint32), "n_raw": 0}
    sub = select_jobs(arrays, [0, 2])
    assert sub["n_sets"] == 4 and sub["n_jobs"] == 2
    assert sub["job_offsets"].tolist() == [0, 2, 4]
    assert sub["pk_offsets"].tolist() == [0, 2, 3, 4, 6]
    assert sub["pk_indices"].tolist() == [100, 101, 102, 106, 107, 108]
    assert (sub["msgs"] == arrays["msgs"][[0, 1, 3, 4]]).all()
