"""Faulted batches at the sizes an 8-GPU node actually runs, at their DEFAULT
pipeline layouts (no bgv_cfg overrides), through both device paths:

  * the per-GPU shard of the 32-epoch segment, C4/8 = 128 blocks = 12,544 sets
    (four-lane Miller loop, three-lane cofactor clearing, digit MSM, deferred
    subgroup checks at the time of writing), and
  * the one-epoch slice, 32 blocks = 3,136 sets (the batch range sync issues,
    sync/constants.ts:41; two-pair view Miller loop on 18 lanes, nine-lane
    view clearing), and the two other view-Miller ranges: 16 blocks = 1,568
    sets (18 lanes per two pairs) and 64 blocks = 6,272 sets (9 lanes),
  * the layouts of the larger shards (fewer GPUs, or one GPU taking a bigger
    share): 256 blocks = 25,088 sets = C4/4 (two-lane Miller loop, digit MSM),
    352 blocks = 34,496 sets (one-lane Miller loop and (job, window) MSM in
    latency mode, from 32,000 sets) and 608 blocks = 59,584 sets (bulk hash,
    one pair per Miller item, from 59,000 sets),

each with 1 % faults of the four C5 kinds (bench.inject_faults: wrong message,
swapped pubkey, cleared compression flag, on-curve point outside G2):

  1. bgv_verify: per-block verdicts and per-set codes equal the construction;
  2. bgv_partial -> bgv_combine_final -> bgv_partial_finish, the multi-GPU path
     (SURVEY 8e), on the whole batch and split into two work-balanced shards:
     the combined check fails, and the shards' localisation gives the same
     verdicts (multithread/worker.ts:74-96: per-job retry after a failed
     batch; verifyBlocksSignatures.ts:56-59: the first bad block is named);
  3. 8 sampled blocks (faulted and clean) re-verified by the C restatement
     (oracle/bls_ref.c) on the same keys, messages and signatures;

and the real partial path over two ranks: two processes, one context each
(both on GPU 0), gloo all-gathers of the 576-byte partials and of the per-job
verdicts (lodestar_amd/dist.py verify_sharded / gather_job_results); and the
same path over an RCCL ("nccl") process group of world size 1 with cuda:0
tensors, the collective code bench.py takes on the 8-GPU node.
"""
import os
import socket

import numpy as np
import pytest

import bench
from tests.test_gpu_configs import N_TABLE, SEED, _cref_block_check

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from lodestar_amd import native
    d = native.Device(0)
    d.gen_keys(0, N_TABLE, SEED)
    yield d
    d.close()


# blocks -> the layout prepare() picks by default at that size (bgv_api.hip)
SIZES = {128: "c4_over_8", 64: "view_miller_9_lanes", 32: "epoch_slice", 16: "view_miller_18_lanes",
         256: "c4_over_4", 352: "one_lane_miller_latency_hash", 608: "bulk_one_pair_per_item"}
# the layout fields prepare() must pick at the larger sizes (bgv_api.hip thresholds)
LAYOUT = {256: {"split": 1, "miller_lanes": 2, "msm": 4, "clear_lanes": 1},
          352: {"split": 1, "miller_lanes": 1, "msm": 2, "clear_lanes": 1},
          608: {"split": 0, "miller_lanes": 1, "pairs_per_item": 1, "msm": 2}}


def test_faulted_shard_on_reserved_bulk_context():
    """the C4/8 shard (128 blocks, 1 % faults of the four C5 kinds) on a bulk
    context that leaves 32 CUs to a priority context (bgv_cfg.cu_split = -32,
    device 0 of the pools when CUs are reserved), beside a priority context
    (cu_split = +32) verifying a faulted one-block batch at the same time:
    every verdict and set code as constructed on both"""
    import threading

    from lodestar_amd import native
    bulk = native.Device(0, cu_split=-32)
    prio = native.Device(0, cu_split=32)
    try:
        for d in (bulk, prio):
            d.gen_keys(0, N_TABLE, SEED)
        a = bench.build_segment(list(range(128)), seed=SEED + 7500)
        fa, expect, code = bench.inject_faults(bulk, a, 0.01, SEED + 7600, with_codes=True)
        one = bench.build_segment([0], seed=SEED + 7700)
        fo, expect1, code1 = bench.inject_faults(prio, one, 0.05, SEED + 7800, with_codes=True)
        out = {}

        def run_prio():
            out["prio"] = prio.verify(fo)

        t = threading.Thread(target=run_prio)
        t.start()
        jr, sc = bulk.verify(fa)
        t.join()
        assert jr.tolist() == expect.tolist() and sc.tolist() == code.tolist()
        assert bulk.last_stats.batch_retries == 1
        jr1, sc1 = out["prio"]
        assert jr1.tolist() == expect1.tolist() and sc1.tolist() == code1.tolist()
    finally:
        bulk.close()
        prio.close()


@pytest.mark.parametrize("blocks", sorted(SIZES))
def test_faulted_shard_default_layout(dev, blocks):
    from lodestar_amd.dist import batch_job_work, select_jobs, shard_jobs
    a = bench.build_segment(list(range(blocks)), seed=SEED + 7000 + blocks)
    fa, expect, code = bench.inject_faults(dev, a, 0.01, SEED + 7100 + blocks, with_codes=True)
    n = a["n_sets"]
    assert n == 98 * blocks
    assert (expect == 0).any() and (expect < 0).any() and (expect == 1).any()

    # 1. bgv_verify at the default layout of this size
    jr, sc = dev.verify(fa)
    layout = dev.last_stats.layout()
    assert jr.tolist() == expect.tolist()
    assert sc.tolist() == code.tolist()
    assert dev.last_stats.batch_retries == 1
    print(f"{n} sets, default layout {layout}")
    for k, v in LAYOUT.get(blocks, {}).items():
        assert layout[k] == v, (k, layout)

    # 2a. the whole batch as one shard: partial -> combined check -> localisation
    part, sc2, prov, ok = dev.partial(fa)
    assert sc2.tolist() == code.tolist()
    assert prov.tolist() == [e if e < 0 else 1 for e in expect.tolist()]
    assert not ok  # rejected jobs are known before the pairing check
    assert dev.last_stats.layout() == layout
    assert not dev.combine_final([part])
    assert dev.partial_finish().tolist() == expect.tolist()

    # 2b. two work-balanced shards (the node path with world = 2)
    shards = shard_jobs(batch_job_work(fa), 2)
    subs = [select_jobs(fa, s) for s in shards]
    parts = [dev.partial(s)[0] for s in subs]
    assert not dev.combine_final(parts)
    got = np.zeros(blocks, np.int32)
    for ids, s in zip(shards, subs):
        dev.partial(s)  # the pending partial is per context: re-run this shard's
        got[np.asarray(ids)] = dev.partial_finish()
    assert got.tolist() == expect.tolist()
    # a clean shard combines to a valid batch
    clean = [j for j in range(blocks) if expect[j] == 1]
    cp, _, cjr, cok = dev.partial(select_jobs(fa, clean))
    assert cok and (cjr == 1).all() and dev.combine_final([cp])

    # 3. the C restatement on 8 sampled blocks
    rng = np.random.default_rng(blocks)
    bad = np.nonzero(expect != 1)[0]
    good = np.nonzero(expect == 1)[0]
    sample = sorted(rng.choice(bad, size=min(4, len(bad)), replace=False).tolist()
                    + rng.choice(good, size=8 - min(4, len(bad)), replace=False).tolist())
    _cref_block_check(dev, fa, sample, expect)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


BLOCKS_2R = 64


def _rank(rank, world, port, q):
    try:
        import torch.distributed as dist

        from lodestar_amd import native
        from lodestar_amd.dist import batch_job_work, gather_job_results, select_jobs, shard_jobs, verify_sharded
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        d = native.Device(0)
        d.gen_keys(0, N_TABLE, SEED)
        a = bench.build_segment(list(range(BLOCKS_2R)), seed=SEED + 7500)
        fa, expect = bench.inject_faults(d, a, 0.01, SEED + 7600)
        shards = shard_jobs(batch_job_work(fa), world)
        out = {"expect": expect.tolist(), "shard": shards[rank]}
        for name, arr in (("faulted", fa), ("clean", bench.signed(d, a))):
            valid, local = verify_sharded(d, select_jobs(arr, shards[rank]), dist)
            full = gather_job_results(local, shards, BLOCKS_2R, dist)
            out[name] = (bool(valid), full.tolist(), d.last_stats.layout())
        d.close()
        dist.destroy_process_group()
        q.put((rank, out))
    except BaseException as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))


@pytest.mark.timeout(240)
def test_two_rank_partial_path_gloo():
    """dist.verify_sharded over two processes with real devices: every rank
    ends with every job's verdict, faulted and clean"""
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = dict(q.get(timeout=200) for _ in range(world))
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert isinstance(res[r], dict), res[r]
    expect = res[0]["expect"]
    assert sorted(res[0]["shard"] + res[1]["shard"]) == list(range(BLOCKS_2R))
    for r in range(world):
        valid, full, _ = res[r]["faulted"]
        assert not valid and full == expect
        valid, full, _ = res[r]["clean"]
        assert valid and full == [1] * BLOCKS_2R


def _rccl_rank(port, q):
    """one rank of an RCCL group (world size 1) on GPU 0: dist.verify_sharded
    and dist.gather_job_results with device tensors, faulted and clean"""
    try:
        import torch
        import torch.distributed as dist

        from lodestar_amd import native
        from lodestar_amd.dist import batch_job_work, gather_job_results, select_jobs, shard_jobs, verify_sharded
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        assert dist.get_backend() == "nccl"
        dev = torch.device("cuda:0")
        d = native.Device(0)
        d.gen_keys(0, N_TABLE, SEED)
        a = bench.build_segment(list(range(BLOCKS_RCCL)), seed=SEED + 7700)
        fa, expect = bench.inject_faults(d, a, 0.01, SEED + 7800)
        shards = shard_jobs(batch_job_work(fa), 1)
        out = {"expect": expect.tolist(), "shard": shards[0]}
        for name, arr in (("faulted", fa), ("clean", bench.signed(d, a))):
            jr, _ = d.verify(arr)
            valid, local = verify_sharded(d, select_jobs(arr, shards[0]), dist, device=dev)
            full = gather_job_results(local, shards, BLOCKS_RCCL, dist, device=dev)
            out[name] = (bool(valid), full.tolist(), jr.tolist())
        d.close()
        dist.destroy_process_group()
        q.put(out)
    except BaseException as e:  # report instead of hanging the parent
        q.put(repr(e))


BLOCKS_RCCL = 32


@pytest.mark.timeout(240)
def test_rccl_world1_partial_path():
    """the RCCL leg of dist.py (all-gathers of the partial and of the verdicts
    through cuda:0 tensors) gives bgv_verify's verdicts, faulted and clean"""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_rank, args=(_free_port(), q))
    p.start()
    try:
        res = q.get(timeout=200)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert isinstance(res, dict), res
    expect = res["expect"]
    assert res["shard"] == list(range(BLOCKS_RCCL))
    valid, full, jr = res["faulted"]
    assert (not valid) and full == expect and jr == expect
    assert any(e != 1 for e in expect)
    valid, full, jr = res["clean"]
    assert valid and full == [1] * BLOCKS_RCCL and jr == full
