"""GPU parity at every BASELINE.json config shape:

  C1  128 single-pubkey sets in one job (BlsSingleThreadVerifier path,
      verifySignatureSetsMaybeBatch, singleThread.ts:14-35)
  C2  64 aggregate sets x k=128 from a 2^20-validator table, one batchable
      call through the IBlsVerifier mirror (multithread/index.ts:151-191)
  C3  blocks of 128 x k=128 attestations + the k=512 sync aggregate + 2
      singles, through verifyBlocksSignatures with and without coalescing;
      a faulted block resolves {allValid: false, index: b}
      (verifyBlocksSignatures.ts:56-59)
  C4  the 32-epoch range-sync segment: 1,024 blocks x 98 sets = 100,352 sets,
      12.98 M pubkey references into a 2^20 table, clean and with 1 % of the
      sets faulted (C5: a quarter each wrong message, swapped pubkey index,
      cleared compression flag, on-curve point outside G2), expected verdicts
      by construction, 16 sampled blocks re-verified by the C restatement
      (oracle/bls_ref.c) on the same keys, messages and signatures.

Keys are sk_i = SHA256("bgv-sk" || LE64(seed) || LE32(i)) mod r generated on
the device (pinned against the oracle in test_gpu_parity); signatures are
device-signed and spot-checked against the C restatement here.
"""
import asyncio

import numpy as np
import pytest

import bench
from tests import gpu_util as G

pytestmark = pytest.mark.gpu

N_TABLE = 1 << 20
SEED = bench.SEED


@pytest.fixture(scope="module")
def big():
    """one context with the 2^20-key table (C2, C4)"""
    from lodestar_amd import native
    d = native.Device(0)
    d.gen_keys(0, N_TABLE, SEED)
    yield d
    d.close()


def _sign(d, arrays):
    sigs = np.zeros((arrays["n_sets"], 192), np.uint8)
    d.gen_sign(arrays, sigs)
    return dict(arrays, sigs=sigs, sig_len=np.full(arrays["n_sets"], 96, np.uint32))


def _cref_block_check(d, arrays, jobs, expect):
    """re-verify the given jobs with the C restatement: aggregated keys from
    the device table rows, the batch's messages and signatures"""
    from oracle import cref
    jo, po, idx = arrays["job_offsets"], arrays["pk_offsets"], arrays["pk_indices"]
    table = np.frombuffer(d.pubkeys_get(0, d.pubkeys_count()), np.uint8).reshape(-1, 96)
    for j in jobs:
        pks, msgs, sigs = [], [], []
        for i in range(int(jo[j]), int(jo[j + 1])):
            rows = idx[po[i]:po[i + 1]]
            pks.append(cref.aggregate([table[int(r)].tobytes() for r in rows]))
            msgs.append(arrays["msgs"][i].tobytes())
            sigs.append(arrays["sigs"][i, : int(arrays["sig_len"][i])].tobytes())
        assert cref.verify_job(pks, msgs, sigs) == int(expect[j]), j


def test_device_keys_and_signatures_match_c_restatement(big):
    """a few table rows and device signatures against oracle/bls_ref.c"""
    from oracle import cref
    for i in (0, 1, 12345, N_TABLE - 1):
        assert big.pubkeys_get(i, 1) == cref.sk_to_pk(cref.device_sk(SEED, i)), i
    a = bench.singles(4, 77)
    a["pk_indices"] = np.array([3, 9, 70000, N_TABLE - 2], np.uint32)
    a = _sign(big, a)
    for k in range(4):
        sk = cref.device_sk(SEED, int(a["pk_indices"][k]))
        assert a["sigs"][k, :96].tobytes() == cref.sign(sk, a["msgs"][k].tobytes()), k


def test_c1_single_sets_maybe_batch():
    """C1: 128 single sets, one job, the BlsSingleThreadVerifier path"""
    from lodestar_amd import verifier as V
    pool = V.BlsGpuVerifier(devices=(0,))
    try:
        d = pool.devices[0]
        d.gen_keys(0, 4096, SEED)
        a = bench.singles(128, SEED + 3000)
        a["pk_indices"] = (a["pk_indices"] % 4096).astype(np.uint32)
        a = _sign(d, a)
        sets = G.sets_from_arrays(a)[0]
        assert len(sets) == 128 and all(s.type == V.SignatureSetType.single for s in sets)
        assert pool.verify_signature_sets_maybe_batch(sets)
        assert pool.metrics["batch_retries"] == 0
        bad = list(sets)
        bad[77] = V.create_single_signature_set_from_components(sets[78].pubkey, sets[77].signingRoot, sets[77].signature)
        assert not pool.verify_signature_sets_maybe_batch(bad)
        _cref_block_check(d, a, [0], [1])
    finally:
        asyncio.run(pool.close())


def test_c2_gossip_batch(big):
    """C2: 64 x k=128 aggregates, one batchable call; a concurrent call with
    one bad set resolves false without touching the good call"""
    from lodestar_amd import verifier as V
    g = bench.build_segment([0], seed=SEED + 1000)
    n2, k2 = 64, bench.ATT_K
    a = {"n_sets": n2, "n_jobs": 1, "job_offsets": np.array([0, n2], np.uint32),
         "pk_offsets": (np.arange(n2 + 1) * k2).astype(np.uint32),
         "pk_indices": g["pk_indices"][: n2 * k2].copy(), "msgs": g["msgs"][:n2].copy(), "n_raw": 0}
    a = _sign(big, a)
    jr, sc = big.verify(a)
    assert jr.tolist() == [1] and (sc == 0).all()
    _cref_block_check(big, a, [0], [1])
    # the bad call's job (set 5 signed over set 6's message) fails in the C restatement too
    wrong = dict(a, msgs=a["msgs"].copy())
    wrong["msgs"][5] = a["msgs"][6]
    _cref_block_check(big, wrong, [0], [0])
    sets = G.sets_from_arrays(a)[0]

    async def run(pool):
        opts = V.VerifySignatureOpts(batchable=True)
        bad = list(sets)
        bad[5] = V.create_aggregate_signature_set_from_components(sets[5].pubkeys, sets[6].signingRoot, sets[5].signature)
        return await asyncio.gather(pool.verify_signature_sets(sets, opts), pool.verify_signature_sets(bad, opts))

    pool = V.BlsGpuVerifier(devices=(0,))
    try:
        for c in pool._contexts():  # every context's table replica (batches in flight go to any of them)
            c.gen_keys(0, N_TABLE, SEED)
        assert asyncio.run(run(pool)) == [True, False]
        assert pool.metrics["aggregated_pubkeys_total"] == 2 * n2 * k2
    finally:
        asyncio.run(pool.close())


@pytest.mark.parametrize("coalesce,att_k", [(False, 128), (True, 128), (True, 440)])
def test_c3_blocks_first_invalid(coalesce, att_k):
    """C3: verifyBlocksSignatures over 3 blocks of 131 sets (128 x k=att_k +
    sync k=512 + 2 singles; k = 440 is ~90% of a 488-member committee at 1M
    validators); block 1 has one wrong-message attestation"""
    from lodestar_amd import verifier as V
    pool = V.BlsGpuVerifier(devices=(0,))
    try:
        d = pool.devices[0]
        for c in pool._contexts():  # every context's table replica
            c.gen_keys(0, N_TABLE, SEED)
        blocks, arrays = [], []
        for b in range(3):
            a = bench.build_segment([b], seed=SEED + 2000, att_per_block=128, att_k=att_k)
            assert a["n_sets"] == 131 and int(a["pk_offsets"][-1]) == 128 * att_k + 512 + 2
            sign_msgs = a["msgs"].copy()
            if b == 1:
                sign_msgs[40, 0] ^= 1
            s = _sign(d, dict(a, msgs=sign_msgs))
            s["msgs"] = a["msgs"]
            blocks.append(G.sets_from_arrays(s)[0])
            arrays.append(s)

        async def run(bl):
            return await V.verify_blocks_signatures(pool, bl, coalesce=coalesce)

        assert asyncio.run(run(blocks)) == {"allValid": False, "index": 1}
        assert asyncio.run(run([blocks[0], blocks[2]])) == {"allValid": True}
        for b, s in enumerate(arrays):  # each block re-verified by the C restatement
            _cref_block_check(d, s, [0], [0 if b == 1 else 1])
    finally:
        asyncio.run(pool.close())


def test_c4_segment_clean_on_device(big):
    """C4: the whole 100,352-set segment, inputs resident in HBM: every block valid
    in ONE batch check (no retry), and six sampled blocks valid under the C
    restatement (oracle/bls_ref.c) too"""
    import torch
    a = bench.build_segment(list(range(1024)))
    assert a["n_sets"] == 100352 and int(a["pk_offsets"][-1]) == 12978176
    dev = torch.device("cuda", 0)
    da = bench.to_device(a, torch, dev)
    sigs = torch.zeros((a["n_sets"], 192), dtype=torch.uint8, device=dev)
    big.gen_sign(da, sigs, on_device=True)
    da["sigs"] = sigs
    da["sig_len"] = torch.full((a["n_sets"],), 96, dtype=torch.int32, device=dev)
    da["scalars"] = None
    jr, _ = big.verify(da, on_device=True, want_set_codes=False)
    assert (jr == 1).all()
    st = big.last_stats
    assert st.batch_retries == 0 and st.batch_sigs_success == 100352 and st.pubkeys_aggregated == 12978176
    # sampled blocks (first, middle, last, and three more) re-verified by the C
    # restatement on the same keys, messages and device signatures
    host = dict(a, sigs=sigs.cpu().numpy(), sig_len=np.full(a["n_sets"], 96, np.uint32))
    pick = [0, 511, 1023] + [int(x) for x in np.random.default_rng(SEED).choice(np.arange(1, 1023), 3, replace=False)]
    _cref_block_check(big, host, pick, np.ones(1024, np.int32))


def test_c5_faulted_segment_host_resident(big):
    """C4 with 1 % faulted sets (C5), host-resident inputs through the pinned
    staging path: per-block verdicts and per-set codes as constructed, every
    faulted block named; 16 sampled blocks (faulted and clean) re-verified by
    the C restatement.  At this size the bulk path runs the Miller loop over
    fixed-argument lines and defers the subgroup checks of the second half of
    the sets (bgv_api.hip prepare): signatures outside G2 sit in both halves."""
    a = bench.build_segment(list(range(1024)))
    fa, expect = bench.inject_faults(big, a, 0.01, SEED + 4000)
    jr, sc = big.verify(fa)
    assert jr.tolist() == expect.tolist()
    assert big.last_stats.batch_retries == 1
    assert set(np.unique(sc).tolist()) == {0, 1, 3}
    not_in_g2 = np.nonzero(sc == 3)[0]
    assert (not_in_g2 < a["n_sets"] // 2).any() and (not_in_g2 >= a["n_sets"] // 2).any()
    assert (expect == 0).sum() > 0 and (expect < 0).sum() > 0
    rng = np.random.default_rng(3)
    faulted = np.nonzero(expect != 1)[0]
    clean = np.nonzero(expect == 1)[0]
    sample = sorted(rng.choice(faulted, size=8, replace=False).tolist() + rng.choice(clean, size=8, replace=False).tolist())
    _cref_block_check(big, fa, sample, expect)


def test_c5_half_segment_deferred_subgroup_checks(big):
    """C4/2 (512 blocks, 50,176 sets: one pair per Miller item, so the bulk
    path defers the G2 subgroup checks beside the Miller loops) with 2 %
    faults of the four kinds: job verdicts and set codes as constructed,
    including a subgroup failure ahead of a later decode failure in one job
    (first failing code in set order)"""
    a = bench.build_segment(list(range(512)))
    fa, expect = bench.inject_faults(big, a, 0.02, SEED + 5000)
    jr, sc = big.verify(fa)
    assert jr.tolist() == expect.tolist()
    assert set(np.unique(sc).tolist()) == {0, 1, 3}
    jo = a["job_offsets"]
    mixed = [j for j in range(512) if 3 in sc[jo[j]:jo[j + 1]].tolist() and 1 in sc[jo[j]:jo[j + 1]].tolist()]
    assert any(expect[j] == -3 for j in mixed) and any(expect[j] == -1 for j in mixed)


def test_pool_batches_in_flight_on_one_device():
    """contexts_per_device (default 3): block calls that arrive while a device
    batch runs go to another context of the same GPU at once, and every
    verdict is that block's (one wrong-message block among eight)"""
    from lodestar_amd import verifier as V
    pool = V.BlsGpuVerifier(devices=(0,))
    try:
        assert len(pool.devices) == V.CONTEXTS_PER_DEVICE
        for c in pool._contexts():
            c.gen_keys(0, N_TABLE, SEED)
        a = _sign(pool.devices[0], bench.build_segment(list(range(8)), seed=SEED + 6000))
        blocks = G.sets_from_arrays(a)
        bad = list(blocks[5])
        bad[7] = V.create_aggregate_signature_set_from_components(bad[7].pubkeys, bad[8].signingRoot, bad[7].signature)
        blocks[5] = bad

        async def run():
            futs = []
            for k, b in enumerate(blocks):
                futs.append(asyncio.ensure_future(pool.verify_signature_sets(b)))
                await asyncio.sleep(0.002)  # the next block arrives while this one runs
            return await asyncio.gather(*futs)

        assert asyncio.run(run()) == [k != 5 for k in range(8)]
        assert pool.peak_busy >= 2, pool.peak_busy
    finally:
        asyncio.run(pool.close())
