"""Host logic of the IBlsVerifier mirror (no GPU): chunking, batch encoding,
error strings, block-level verdict ordering and job sharding."""
import asyncio
import os

import numpy as np
import pytest

from lodestar_amd import verifier as V
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

from lodestar_amd.dist import batch_job_work, job_work, shard_balance, shard_jobs


def test_chunkify_matches_reference_unit_test():
    # packages/beacon-node/test/unit/chain/bls/utils.test.ts (minPerChunk = 3)
    expected = [
        [[0]], [[0, 1]], [[0, 1, 2]], [[0, 1, 2, 3]], [[0, 1, 2, 3, 4]],
        [[0, 1, 2], [3, 4, 5]], [[0, 1, 2, 3], [4, 5, 6]], [[0, 1, 2, 3], [4, 5, 6, 7]],
    ]
    for i, exp in enumerate(expected):
        assert V.chunkify_maximize_chunk_size(list(range(i + 1)), 3) == exp
    assert V.chunkify_maximize_chunk_size([], 128) == [[]]


def test_chunkify_pool_sizes():
    for n in (1, 127, 128, 255, 256, 257, 1000, 8000):
        chunks = V.chunkify_maximize_chunk_size(list(range(n)), 128)
        assert [x for c in chunks for x in c] == list(range(n))
        if n >= 256:  # floor(n / 128) chunks of ceil(n / count) (the last one may be shorter)
            assert len(chunks) == n // 128 or len(chunks) == -(-n // -(-n // (n // 128)))
            assert max(len(c) for c in chunks) == -(-n // (n // 128))


def _set(idxs, root=b"\x01" * 32, sig=b"\xaa" * 96):
    pks = [V.PublicKey(index=i) for i in idxs]
    if len(pks) == 1:
        return V.create_single_signature_set_from_components(pks[0], root, sig)
    return V.create_aggregate_signature_set_from_components(pks, root, sig)


def test_encode_jobs_layout():
    raw = V.PublicKey.from_bytes(b"\x11" * 96)
    jobs = [[_set([5]), _set([1, 2, 3])], [V.create_single_signature_set_from_components(raw, b"\x02" * 32, b"\x00" * 32)]]
    a = V.encode_jobs(jobs)
    assert a["n_sets"] == 3 and a["n_jobs"] == 2
    assert a["job_offsets"].tolist() == [0, 2, 3]
    assert a["pk_offsets"].tolist() == [0, 1, 4, 5]
    assert a["pk_indices"].tolist() == [5, 1, 2, 3, 0x80000000]
    assert a["n_raw"] == 1 and a["raw_pks"].tobytes() == b"\x11" * 96
    assert a["sig_len"].tolist() == [96, 96, 32]
    assert (a["sigs"][2] == 0).all()  # a 32-byte signature travels as its length only


def test_empty_aggregate_rejects():
    with pytest.raises(V.BlsError, match="EMPTY_AGGREGATE_ARRAY"):
        V.encode_jobs([[V.create_aggregate_signature_set_from_components([], bytes(32), bytes(96))]])


def test_error_strings_match_reference_tests():
    assert "BLST_INVALID_SIZE" in str(V.error_for_code(8))          # multithread.test.ts:97
    assert "BLST_ERROR" in str(V.error_for_code(3))                  # spec/general/bls.ts:37
    assert str(V.error_for_code(10)) == "Empty signature set"        # maybeBatch.ts:30
    with pytest.raises(V.BlsError, match="BLST_INVALID_SIZE"):
        V.PublicKey.from_bytes(b"\x00" * 10)


def test_reject_first_invalid_resolve_all_valid():
    # test/unit/chain/blocks/rejectFirstInvalidResolveAllValid.test.ts
    async def run():
        loop = asyncio.get_running_loop()
        futs = [loop.create_future() for _ in range(3)]
        task = asyncio.ensure_future(V.reject_first_invalid_resolve_all_valid(futs))
        await asyncio.sleep(0)
        futs[2].set_result(True)
        await asyncio.sleep(0)
        futs[1].set_result(False)
        res = await task
        assert res == {"allValid": False, "index": 1}
        futs2 = [loop.create_future() for _ in range(3)]
        task2 = asyncio.ensure_future(V.reject_first_invalid_resolve_all_valid(futs2))
        for f in futs2:
            f.set_result(True)
        assert await task2 == {"allValid": True}
    asyncio.run(run())


def test_shard_jobs_balanced_and_complete():
    sizes = [98] * 1024 + [1, 5, 128]
    for world in (1, 2, 4, 8):
        shards = shard_jobs(sizes, world)
        flat = sorted(j for s in shards for j in s)
        assert flat == list(range(len(sizes)))
        loads = [sum(sizes[j] for j in s) for s in shards]
        assert max(loads) - min(loads) <= 128


def mixed_segment_jobs(n_blocks=256, seed=7):
    """(sets, pubkey refs) per block of a mixed range-sync segment: full blocks
    with the 512-key sync aggregate, full blocks without it, blocks of fewer
    and smaller attestations, and near-empty blocks (proposer + randao)"""
    import random
    rnd = random.Random(seed)
    out = []
    for _ in range(n_blocks):
        kind = rnd.random()
        if kind < 0.1:  # near-empty: proposer + randao
            out.append((2, 2))
        else:
            n_att = rnd.randint(8, 95) if kind < 0.35 else 95
            k = [rnd.choice((64, 96, 128, 160)) for _ in range(n_att)]
            sync = kind < 0.7  # with or without the sync aggregate
            out.append((n_att + 2 + sync, sum(k) + 2 + 512 * sync))
    return out


def test_shard_jobs_balance_work_on_a_mixed_segment():
    """shards balanced by sum W(k) (sets + pubkey references), not
    by set count; within 5% max/mean over 8 shards on a mixed segment"""
    jobs = mixed_segment_jobs()
    work = job_work([s for s, _ in jobs], [k for _, k in jobs])
    for world in (2, 4, 8):
        shards = shard_jobs(work, world)
        assert sorted(j for s in shards for j in s) == list(range(len(jobs)))
        assert shard_balance(work, shards) <= 1.05, world
    # a 512-key sync job outweighs a 1-key single, so they no longer count the same
    a, b = job_work([1, 1], [512, 1])
    assert a > b


def test_shard_jobs_weights_a_reserved_device():
    """a device whose bulk context leaves CUs to the priority context runs at
    RESERVED_CAP: it gets a proportionally smaller shard, so the shards finish
    together (load / cap within 5% max/mean)"""
    from lodestar_amd.dist import RESERVED_CAP
    jobs = mixed_segment_jobs()
    work = job_work([s for s, _ in jobs], [k for _, k in jobs])
    for world in (2, 4, 8):
        caps = [RESERVED_CAP] + [1.0] * (world - 1)
        shards = shard_jobs(work, world, caps)
        assert sorted(j for s in shards for j in s) == list(range(len(jobs)))
        t = [sum(work[j] for j in sh) / c for sh, c in zip(shards, caps)]
        assert max(t) / (sum(t) / world) <= 1.05, world
        assert sum(work[j] for j in shards[0]) < min(sum(work[j] for j in sh) for sh in shards[1:])
    assert shard_jobs(work, 4, [1.0] * 4) == shard_jobs(work, 4)


def test_batch_job_work_matches_job_work():
    jo = np.array([0, 2, 5, 5, 6], np.uint32)
    po = np.array([0, 1, 513, 641, 642, 643, 771], np.uint32)
    assert batch_job_work({"job_offsets": jo, "pk_offsets": po}) == job_work([2, 3, 0, 1], [513, 130, 0, 128])


def test_node_shard_jobs_is_the_python_assignment():
    import json
    import shutil
    import subprocess
    from tools import build
    if not shutil.which("node") or not build.build_addon():
        pytest.skip("node or its headers are absent")
    jobs = mixed_segment_jobs(64, seed=3)
    sets = [[{"type": "aggregate", "pubkeys": [0] * (k // s)} for _ in range(s)] for s, k in jobs]
    # give every job exactly k references: the first set takes the remainder
    for (s, k), js in zip(jobs, sets):
        js[0]["pubkeys"] = [0] * (k - (k // s) * (s - 1))
    script = ("const m = require(%r); const jobs = JSON.parse(require('fs').readFileSync(0, 'utf8'));"
              "const caps = (w) => [m.RESERVED_CAP].concat(new Array(w - 1).fill(1));"
              "console.log(JSON.stringify([8, 4, 2].map((w) => m.shardJobs(jobs.map(m.jobWork), w))"
              ".concat([8, 4, 2].map((w) => m.shardJobs(jobs.map(m.jobWork), w, caps(w))))));") % os.path.join(
                  ROOT, "lodestar_amd", "napi", "index.js")
    out = json.loads(subprocess.check_output(["node", "-e", script], input=json.dumps(sets).encode()))
    work = job_work([s for s, _ in jobs], [k for _, k in jobs])
    from lodestar_amd.dist import RESERVED_CAP
    assert out == [shard_jobs(work, w) for w in (8, 4, 2)] + [shard_jobs(work, w, [RESERVED_CAP] + [1.0] * (w - 1))
                                                              for w in (8, 4, 2)]
