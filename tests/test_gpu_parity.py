"""GPU parity tests: the HIP path (through the C ABI) against the oracle's
golden vectors and against oracle-computed values.  Run on an MI355X:

    python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
"""
import asyncio
import hashlib

import numpy as np
import pytest

from oracle import bls12_381 as B
from tests import gpu_util as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from lodestar_amd import native
    d = native.Device(0)
    G.load_golden_table(d)
    yield d
    d.close()


def test_table_decompression_matches_oracle(dev):
    """bgv_pubkeys_set(compressed) == oracle g1_decompress for all 100 interop keys."""
    pks = G.interop_pubkeys48()
    got = dev.pubkeys_get(0, 100)
    for i in range(100):
        code, pt = B.g1_decompress(pks[48 * i : 48 * i + 48])
        assert code == 0
        assert got[96 * i : 96 * i + 96] == B.g1_serialize(pt), i


def test_golden_batch_all_jobs(dev):
    arrays, expected, codes = G.golden_arrays()
    jr, sc = dev.verify(arrays)
    assert jr.tolist() == expected
    assert sc.tolist() == codes
    st = dev.last_stats
    assert st.batch_retries == 1  # the batch holds invalid jobs


@pytest.mark.parametrize("job", list(range(len(G.batch_vectors()["jobs"]))))
def test_golden_each_job_alone(dev, job):
    arrays, expected, codes = G.golden_arrays([job])
    jr, sc = dev.verify(arrays)
    assert jr.tolist() == expected
    assert sc.tolist() == codes


@pytest.mark.parametrize("cu_split", [32, -32, 8])
def test_golden_batch_on_partitioned_cus(cu_split):
    """the priority context (cu_split > 0: streams on reserved CUs) and the
    bulk context beside it (< 0) give the golden verdicts and set codes"""
    from lodestar_amd import native
    d = native.Device(0, cu_split=cu_split)
    try:
        G.load_golden_table(d)
        arrays, expected, codes = G.golden_arrays()
        jr, sc = d.verify(arrays)
        assert jr.tolist() == expected
        assert sc.tolist() == codes
        valid, _, _ = G.golden_arrays([0, 1, 9])
        assert d.verify(valid)[0].tolist() == [1, 1, 1]
    finally:
        d.close()


def test_golden_valid_jobs_single_batch_check(dev):
    valid = [0, 1, 9, 11, 12, 13]
    arrays, expected, _ = G.golden_arrays(valid)
    jr, _ = dev.verify(arrays)
    assert jr.tolist() == [1] * len(valid) == expected
    assert dev.last_stats.batch_retries == 0
    assert dev.last_stats.batch_sigs_success == arrays["n_sets"]


def test_verdict_independent_of_scalars(dev):
    for seed in (1, 2, 3):
        arrays, expected, _ = G.golden_arrays(scalars_seed=seed)
        jr, _ = dev.verify(arrays)
        assert jr.tolist() == expected
    arrays, expected, _ = G.golden_arrays()
    arrays["scalars"] = None  # drawn inside the library (device ChaCha20 keyed by getrandom)
    jr, _ = dev.verify(arrays)
    assert jr.tolist() == expected


def test_partial_combine_matches_verify(dev):
    valid = [0, 1, 9, 11]
    a0, _, _ = G.golden_arrays(valid[:2])
    a1, _, _ = G.golden_arrays(valid[2:])
    p0, _, _, ok0 = dev.partial(a0)
    p1, _, _, ok1 = dev.partial(a1)
    assert ok0 and ok1
    assert dev.combine_final([p0, p1])
    bad, _, _ = G.golden_arrays([2])  # wrong-message job
    p2, _, _, ok2 = dev.partial(bad)
    assert ok2
    assert not dev.combine_final([p0, p1, p2])


def test_sharded_localisation_matches_verify(dev):
    """SURVEY §8e "Failure": the golden batch split into 3 shards of whole
    jobs; partial -> combined check -> (on failure) bgv_partial_finish per
    shard gives exactly bgv_verify's per-job verdicts, and a shard whose own
    check passes does not retry per job."""
    from lodestar_amd.dist import select_jobs, shard_jobs
    arrays, expected, _ = G.golden_arrays()
    jo = arrays["job_offsets"]
    shards = shard_jobs([int(jo[j + 1] - jo[j]) for j in range(arrays["n_jobs"])], 3)
    parts, provisional = [], []
    for ids in shards:
        p, _, jr, _ = dev.partial(select_jobs(arrays, ids))
        parts.append(p)
        provisional.append(jr)
    assert not dev.combine_final(parts)  # the golden batch holds false jobs
    got = np.zeros(arrays["n_jobs"], np.int32)
    for ids, prov in zip(shards, provisional):
        sub = select_jobs(arrays, ids)
        dev.partial(sub)
        local = dev.partial_finish()
        want = [expected[j] for j in ids]
        assert local.tolist() == want
        assert [int(x) if x < 0 else 1 for x in prov] == [w if w < 0 else 1 for w in want]
        assert dev.last_stats.batch_retries == (1 if 0 in want else 0)
        got[np.asarray(ids)] = local
    assert got.tolist() == expected
    # finish without a partial before it is refused
    from lodestar_amd import native
    dev.verify(G.golden_arrays([0])[0])
    with pytest.raises(native.BgvNativeError) as e:
        dev.partial_finish()
    assert e.value.status == native.BGV_E_STATE


def test_gen_keys_and_sign_match_oracle(dev):
    from lodestar_amd import native
    d = native.Device(0)
    seed = 0x4C4F4445
    d.gen_keys(0, 8, seed)
    got = d.pubkeys_get(0, 8)
    for i in range(8):
        h = hashlib.sha256(b"bgv-sk" + seed.to_bytes(8, "little") + i.to_bytes(4, "little")).digest()
        sk = int.from_bytes(h, "big") % B.R
        assert got[96 * i : 96 * i + 96] == B.g1_serialize(B.sk_to_pk(sk)), i
    # one aggregate set over keys 1, 3, 5 signed on the device
    m = hashlib.sha256(b"m").digest()
    arrays = {"n_sets": 1, "n_jobs": 1, "job_offsets": np.array([0, 1], np.uint32),
              "pk_offsets": np.array([0, 3], np.uint32), "pk_indices": np.array([1, 3, 5], np.uint32),
              "msgs": np.frombuffer(m, np.uint8).copy()}
    out = np.zeros(192, np.uint8)
    d.gen_sign(arrays, out)
    sks = [int.from_bytes(hashlib.sha256(b"bgv-sk" + seed.to_bytes(8, "little") + i.to_bytes(4, "little")).digest(), "big") % B.R for i in (1, 3, 5)]
    assert out[:96].tobytes() == B.g2_compress(B.sign(sum(sks) % B.R, m))
    d.close()


def _synthetic(dev_, n_sets, k, n_keys, seed, fault_every=0):
    """device-generated keys + signatures; every fault_every-th set signs the wrong message"""
    rng = np.random.default_rng(seed)
    idx = np.concatenate([rng.choice(n_keys, size=k, replace=False) for _ in range(n_sets)]).astype(np.uint32)
    msgs = rng.integers(0, 256, size=(n_sets, 32), dtype=np.uint8)
    arrays = {"n_sets": n_sets, "n_jobs": n_sets, "job_offsets": np.arange(n_sets + 1, dtype=np.uint32),
              "pk_offsets": (np.arange(n_sets + 1) * k).astype(np.uint32), "pk_indices": idx, "msgs": msgs}
    sigs = np.zeros((n_sets, 192), np.uint8)
    sign_msgs = msgs.copy()
    bad = np.zeros(n_sets, bool)
    if fault_every:
        bad[::fault_every] = True
        sign_msgs[bad, 0] ^= 1
    dev_.gen_sign(dict(arrays, msgs=sign_msgs), sigs)
    arrays["sigs"] = sigs
    arrays["sig_len"] = np.full(n_sets, 96, np.uint32)
    arrays["scalars"] = rng.integers(1, 2**63, size=n_sets, dtype=np.uint64)
    return arrays, bad


def test_synthetic_batch_with_faults():
    from lodestar_amd import native
    d = native.Device(0)
    d.gen_keys(0, 512, 99)
    arrays, bad = _synthetic(d, 300, 16, 512, 5, fault_every=37)
    jr, sc = d.verify(arrays)
    assert (jr == np.where(bad, 0, 1)).all()
    assert (sc == 0).all()
    # the same sets grouped as 3 jobs of 100: a job is valid iff it has no fault
    arrays["n_jobs"] = 3
    arrays["job_offsets"] = np.array([0, 100, 200, 300], np.uint32)
    jr, _ = d.verify(arrays)
    assert jr.tolist() == [int(not bad[i * 100 : (i + 1) * 100].any()) for i in range(3)]
    d.close()


def test_async_verifier_like_reference_e2e():
    """packages/beacon-node/test/e2e/chain/bls/multithread.test.ts:8-104 on the GPU:
    three valid single sets (sk = 0x0101.., 0x0202.., 0x0303.., msg = same bytes)
    resolve true whether submitted sync / async / batchable; a 32-byte signature
    in a batchable job rejects with BLST_INVALID_SIZE while 8 others resolve true."""
    from lodestar_amd import verifier as V
    v = G.batch_vectors()
    sets = []
    for k in range(3):
        s = v["jobs"][0]["sets"][k]
        pk = V.PublicKey.from_bytes(bytes.fromhex(v["raw_pubkeys"][k]))
        sets.append(V.create_single_signature_set_from_components(pk, bytes.fromhex(s["msg"]), bytes.fromhex(s["sig"])))

    async def run():
        pool = V.BlsGpuVerifier(devices=(0,))
        try:
            assert not pool.prio_reserved  # one device: no CU reservation by default
            assert await pool.verify_signature_sets(sets)
            assert await pool.verify_signature_sets(sets, V.VerifySignatureOpts(batchable=True))
            assert await pool.verify_signature_sets(sets, V.VerifySignatureOpts(verifyOnMainThread=True))
            assert pool.metrics["main_thread_calls"] == 1  # mainThreadDurationInThreadPool
            # a call that throws is timed too (the reference's finally, multithread/index.ts:156-167)
            short = V.create_single_signature_set_from_components(sets[0].pubkey, sets[0].signingRoot, bytes(32))
            with pytest.raises(V.BlsError, match="BLST_INVALID_SIZE"):
                await pool.verify_signature_sets([short], V.VerifySignatureOpts(verifyOnMainThread=True))
            assert pool.metrics["main_thread_calls"] == 2
            good = [pool.verify_signature_sets(sets, V.VerifySignatureOpts(batchable=True)) for _ in range(8)]
            bad_set = V.create_single_signature_set_from_components(sets[0].pubkey, sets[0].signingRoot, bytes(32))
            bad = pool.verify_signature_sets([bad_set], V.VerifySignatureOpts(batchable=True))
            res = await asyncio.gather(*good, bad, return_exceptions=True)
            assert res[:8] == [True] * 8
            assert isinstance(res[8], V.BlsError) and "BLST_INVALID_SIZE" in str(res[8])
            with pytest.raises(V.BlsError, match="Empty signature set"):
                await pool.verify_signature_sets([])
            with pytest.raises(V.BlsError, match="EMPTY_AGGREGATE_ARRAY"):
                await pool.verify_signature_sets([V.create_aggregate_signature_set_from_components([], bytes(32), bytes(96))])
        finally:
            await pool.close()
        with pytest.raises(V.QueueError):
            await pool.verify_signature_sets(sets)
        # BlsSingleThreadVerifier (blsVerifyAllMainThread, chain.ts:200-202)
        single = V.BlsGpuSingleThreadVerifier(0)
        try:
            assert single.can_accept_work()
            assert await single.verify_signature_sets(sets)
            wrong = [V.create_single_signature_set_from_components(sets[0].pubkey, sets[1].signingRoot, sets[0].signature)]
            assert not await single.verify_signature_sets(wrong)
            with pytest.raises(V.BlsError, match="Empty signature set"):
                await single.verify_signature_sets([])
            assert single.metrics["main_thread_calls"] == 2
        finally:
            await single.close()
        with pytest.raises(V.QueueError):
            await single.verify_signature_sets(sets)
        # blsVerifyAllMultiThread (chain/options.ts:14): verifyOnMainThread joins the queue
        pool = V.BlsGpuVerifier(devices=(0,), bls_verify_all_multi_thread=True)
        try:
            jobs0 = pool.metrics["jobs_started"]
            assert await pool.verify_signature_sets(sets, V.VerifySignatureOpts(verifyOnMainThread=True))
            assert pool.metrics["jobs_started"] > jobs0
            assert not pool.prio_reserved and pool.prio is None  # no priority context is opened
        finally:
            await pool.close()

    asyncio.run(run())


def test_microbench_runs(dev):
    assert dev.bench_fpmul(256 * 64, 64) > 0
    assert dev.bench_mad(256 * 64, 64) > 0


def test_cooperative_miller_bit_identical_to_serial():
    """The cooperative Miller loop (miller_coop.h) in its three layouts (36,
    6 and 18 lanes per pair), the two- and four-lane loops (miller_duo.h,
    miller_quad.h) and the
    one-lane loop (pairing.h, bgv_cfg.miller = 1)
    produce the same Fp12 batch partial, byte for byte, and the same verdicts."""
    from lodestar_amd import native
    outs = {}
    for mode in ("serial", "coop", "6", "18", "duo", "quad"):
        d = native.Device(0, miller={"serial": 1, "coop": 36, "6": 6, "18": 18, "duo": 2, "quad": 4}[mode])
        try:
            G.load_golden_table(d)
            a, expected, _ = G.golden_arrays([0, 1, 9, 11, 12, 13], scalars_seed=3)
            part, _, _, ok = d.partial(a)
            jr, _ = d.verify(G.golden_arrays(scalars_seed=3)[0])
            first = d.pubkeys_count()
            d.gen_keys(first, 256, 5)
            syn, bad = _synthetic_on(d, 200, 8, first, 256, 9, fault_every=17)
            jr2, _ = d.verify(syn)
            outs[mode] = (part, ok, jr.tolist(), jr2.tolist(), bad)
        finally:
            d.close()
    for mode in ("coop", "6", "18", "duo", "quad"):  # 36, 6, 18, 2 and 4 lanes per pair
        assert outs["serial"][0] == outs[mode][0], mode
        assert outs["serial"][1:4] == outs[mode][1:4], mode
    assert outs["coop"][2] == G.golden_arrays()[1]
    assert outs["coop"][3] == np.where(outs["coop"][4], 0, 1).tolist()


def _synthetic_on(dev_, n_sets, k, first, n_keys, seed, fault_every=0):
    rng = np.random.default_rng(seed)
    idx = (first + np.concatenate([rng.choice(n_keys, size=k, replace=False) for _ in range(n_sets)])).astype(np.uint32)
    msgs = rng.integers(0, 256, size=(n_sets, 32), dtype=np.uint8)
    arrays = {"n_sets": n_sets, "n_jobs": n_sets, "job_offsets": np.arange(n_sets + 1, dtype=np.uint32),
              "pk_offsets": (np.arange(n_sets + 1) * k).astype(np.uint32), "pk_indices": idx, "msgs": msgs}
    sign_msgs = msgs.copy()
    bad = np.zeros(n_sets, bool)
    if fault_every:
        bad[::fault_every] = True
        sign_msgs[bad, 0] ^= 1
    sigs = np.zeros((n_sets, 192), np.uint8)
    dev_.gen_sign(dict(arrays, msgs=sign_msgs), sigs)
    arrays.update(sigs=sigs, sig_len=np.full(n_sets, 96, np.uint32),
                  scalars=rng.integers(1, 2**63, size=n_sets, dtype=np.uint64))
    return arrays, bad


def _oracle_pk_code(b: bytes) -> int:
    """PublicKey.fromBytes(b, affine, validate=true) per the oracle: decode
    code, then infinity -> 6 (BLST_PK_IS_INFINITY), [r]P != O -> 3."""
    code, pt = B.g1_decompress(b)
    if code:
        return code
    if pt is None:
        return 6
    return 0 if B.g1_in_subgroup(pt) else 3


def test_pubkey_validation_matches_oracle(dev):
    """bgv_pubkeys_validate == the oracle on the 100 interop keys, their
    negations, and every rejection class (processDeposit.ts:57-66)."""
    pks = G.interop_pubkeys48()
    keys = [pks[48 * i : 48 * i + 48] for i in range(100)]
    keys += [bytes([k[0] ^ 0x20]) + k[1:] for k in keys[:4]]           # -P: still in G1
    keys.append(bytes([0xC0]) + bytes(47))                               # infinity
    keys.append(bytes([keys[0][0] & 0x7F]) + keys[0][1:])                # compression flag cleared
    keys.append(bytes([0xE0]) + bytes(47))                               # infinity flag with sign bit
    pb = bytearray(B.P.to_bytes(48, "big"))
    pb[0] |= 0x80
    keys.append(bytes(pb))                                               # x = p
    rng = np.random.default_rng(17)
    off_curve = in_e1_not_g1 = 0
    while off_curve < 3 or in_e1_not_g1 < 3:
        x = int.from_bytes(rng.bytes(48), "big") % B.P
        y = B.fp_sqrt((x * x * x + B.B1) % B.P)
        if y is None and off_curve < 3:
            xb = bytearray(x.to_bytes(48, "big"))
            xb[0] |= 0x80
            keys.append(bytes(xb))
            off_curve += 1
        elif y is not None and in_e1_not_g1 < 3 and not B.g1_in_subgroup((x, y)):
            keys.append(B.g1_compress((x, y)))
            in_e1_not_g1 += 1
    got = dev.pubkeys_validate(b"".join(keys)).tolist()
    want = [_oracle_pk_code(k) for k in keys]
    assert got == want
    assert set(want) == {0, 1, 2, 3, 6}


def test_single_set_and_light_client_aggregate():
    """verifySignatureSet (util/signatureSets.ts:24-38) and the light client's
    isValidBlsAggregate (light-client/src/validation.ts:152-175) on the device,
    with oracle-made keys and signatures (sk = 0x0101.., 0x0202.., 0x0303..)."""
    from lodestar_amd import verifier as V
    sks = [int.from_bytes(bytes([k]) * 32, "big") % B.R for k in (1, 2, 3)]
    pks = [V.PublicKey.from_bytes(B.g1_serialize(B.sk_to_pk(sk))) for sk in sks]
    msg = bytes(range(32))
    agg_sig = B.g2_compress(B.sign(sum(sks) % B.R, msg))
    one_sig = B.g2_compress(B.sign(sks[0], msg))
    pool = V.BlsGpuVerifier(devices=(0,))
    try:
        assert pool.is_valid_bls_aggregate(pks, msg, agg_sig)
        assert not pool.is_valid_bls_aggregate(pks[:2], msg, agg_sig)
        assert not pool.is_valid_bls_aggregate(pks, bytes(32), agg_sig)
        with pytest.raises(V.BlsError, match="Error aggregating pubkeys"):
            pool.is_valid_bls_aggregate([], msg, agg_sig)
        with pytest.raises(V.BlsError, match="Error deserializing signature: BLST_ERROR: BLST_INVALID_SIZE"):
            pool.is_valid_bls_aggregate(pks, msg, agg_sig[:32])
        single = V.create_single_signature_set_from_components
        aggregate = V.create_aggregate_signature_set_from_components
        assert pool.verify_signature_set(single(pks[0], msg, one_sig))
        assert not pool.verify_signature_set(single(pks[1], msg, one_sig))
        assert pool.verify_signature_set(aggregate(pks, msg, agg_sig))
        assert not pool.verify_signature_set(aggregate(pks[1:], msg, agg_sig))
    finally:
        asyncio.run(pool.close())


def test_signature_msm_bit_identical_to_per_set_scaling():
    """sum_j r_i sigma_i by the per-job bucket MSM (k_msm_*, default for
    large batches) and by per-set [r_i] sigma_i + tree give the same S_job:
    the batch partial (which holds the (-G1, S_job) Miller values) is
    byte-identical, and the golden verdicts hold in both modes."""
    from lodestar_amd import native
    outs = {}
    for mode in ("0", "1", "2", "3", "4"):  # 3: one-lane scaling, checks deferred, in latency mode
        d = native.Device(0, msm=int(mode), **({"split": 1} if mode in ("3", "4") else {}))
        try:
            G.load_golden_table(d)
            a, _, _ = G.golden_arrays([0, 1, 9, 10, 11, 12, 13], scalars_seed=5)
            part, _, _, ok = d.partial(a)
            arrays, expected, codes = G.golden_arrays(scalars_seed=5)
            jr, sc = d.verify(arrays)
            assert jr.tolist() == expected and sc.tolist() == codes
            first = d.pubkeys_count()
            d.gen_keys(first, 256, 5)
            syn, bad = _synthetic_on(d, 300, 8, first, 256, 4, fault_every=23)
            syn["n_jobs"] = 3
            syn["job_offsets"] = np.array([0, 100, 200, 300], np.uint32)
            syn_part, _, _, _ = d.partial(syn)
            jr2, _ = d.verify(syn)
            assert jr2.tolist() == [int(not bad[i * 100:(i + 1) * 100].any()) for i in range(3)]
            outs[mode] = (part, ok, syn_part)
        finally:
            d.close()
    assert outs["0"] == outs["1"] == outs["2"] == outs["3"] == outs["4"]


def test_signature_tree_large_jobs_bit_identical():
    """Jobs of 300 and 200 sets (a nine-level S_job tree, past the 256-set span
    of the MSM defaults) summed by the nine-lane tree levels (msm 0 below
    16,384 sets, k_s_level_coop) and by the (job, window) MSM: same batch
    partial, byte for byte, and the verdicts of a clean and a faulted job."""
    from lodestar_amd import native
    outs = {}
    for mode in (0, 2):
        d = native.Device(0, msm=mode)
        try:
            G.load_golden_table(d)
            first = d.pubkeys_count()
            d.gen_keys(first, 256, 7)
            syn, bad = _synthetic_on(d, 500, 4, first, 256, 9, fault_every=0)
            syn["n_jobs"] = 2
            syn["job_offsets"] = np.array([0, 300, 500], np.uint32)
            part, _, _, ok = d.partial(syn)
            jr, _ = d.verify(syn)
            assert jr.tolist() == [1, 1] and ok
            faulted, _ = _synthetic_on(d, 500, 4, first, 256, 9, fault_every=211)
            faulted["n_jobs"] = 2
            faulted["job_offsets"] = np.array([0, 300, 500], np.uint32)
            jr2, _ = d.verify(faulted)
            assert jr2.tolist() == [0, 0]  # sets 0 and 211 (job 0), 422 (job 1)
            outs[mode] = part
        finally:
            d.close()
    assert outs[0] == outs[2]


@pytest.mark.gpu
def test_latency_split_mode_bit_identical():
    """Latency mode (bgv_cfg.split = 1, default below 59,000 sets: two map lanes
    per message, subgroup check beside [r_i] sigma_i) and the one-lane-per-set
    kernels (split = 0) give the same batch partial, byte for byte, and the
    same per-job verdicts and set codes on the golden jobs (which include
    off-curve and out-of-subgroup signatures)."""
    from lodestar_amd import native
    outs = {}
    for mode in ("0", "1", "1c3", "1c1"):  # cofactor clearing on 9 / 3 / 1 lanes per point
        d = native.Device(0, split=int(mode[0]), **({"clear_lanes": int(mode[2])} if len(mode) > 1 else {}))
        try:
            G.load_golden_table(d)
            a, expected, codes = G.golden_arrays([0, 1, 9, 11, 12, 13], scalars_seed=3)
            part, _, _, ok = d.partial(a)
            ga, gexp, gcodes = G.golden_arrays(scalars_seed=3)
            jr, sc = d.verify(ga)
            first = d.pubkeys_count()
            d.gen_keys(first, 256, 5)
            syn, bad = _synthetic_on(d, 200, 8, first, 256, 9, fault_every=17)
            jr2, _ = d.verify(syn)
            outs[mode] = (part, ok, jr.tolist(), sc.tolist(), jr2.tolist(), bad)
        finally:
            d.close()
    assert outs["0"][0] == outs["1"][0] == outs["1c3"][0] == outs["1c1"][0]
    assert outs["0"][1:5] == outs["1"][1:5] == outs["1c3"][1:5] == outs["1c1"][1:5]
    assert outs["1"][2] == gexp and outs["1"][3] == gcodes
    assert outs["1"][4] == np.where(outs["1"][5], 0, 1).tolist()


@pytest.mark.gpu
def test_two_level_job_fold_bit_identical():
    """The two-level per-job fold (k_job_prefold, default for <= 256 jobs of
    >= 64 sets: groups of ~sqrt(span) sets fold side by side, then the job
    folds the group values) and the one-level fold (bgv_cfg.prefold = 0) give the
    same batch partial, byte for byte, on ragged jobs (64, 100, 3, 1 and 132
    sets), the same per-job verdicts when the batch check fails and every job
    takes its own final exponentiation, and a passing batch when no set is
    faulted."""
    from lodestar_amd import native
    offs = [0, 64, 164, 167, 168, 300]
    outs = {}
    for mode in ("0", "1"):
        d = native.Device(0, prefold=int(mode))
        try:
            first = d.pubkeys_count()
            d.gen_keys(first, 256, 5)
            res = []
            for fault_every in (0, 150):  # 150: faults at sets 0 and 150 (jobs 0 and 1)
                syn, bad = _synthetic_on(d, 300, 8, first, 256, 21, fault_every=fault_every)
                syn["n_jobs"] = len(offs) - 1
                syn["job_offsets"] = np.array(offs, np.uint32)
                part, _, _, ok = d.partial(syn)
                jr, _ = d.verify(syn)
                want = [int(not bad[offs[j]:offs[j + 1]].any()) for j in range(len(offs) - 1)]
                assert jr.tolist() == want
                assert d.combine_final([part]) == (not bad.any())
                res.append((part, ok, jr.tolist()))
            outs[mode] = res
        finally:
            d.close()
    assert outs["0"] == outs["1"]


def test_multi_device_verifier_partial_combine():
    """BlsGpuVerifier over two contexts (both on GPU 0 here: the code path of
    one process owning several GPUs): a device batch split by job,
    one partial Miller product per context (bgv_partial), ONE combined final
    exponentiation (bgv_combine_final) and, when it fails, per-shard
    localisation (bgv_partial_finish).  Verdicts equal a one-context
    bgv_verify of the same jobs, clean and with faulted shards; the golden
    jobs (rejections of every kind) give their golden verdicts."""
    from lodestar_amd import native
    from lodestar_amd import verifier as V
    pool = V.BlsGpuVerifier(devices=(0, 0), shard_min_sets=1)
    single = native.Device(0)
    try:
        for d in pool.devices + [single]:
            G.load_golden_table(d)
            first = d.pubkeys_count()
            d.gen_keys(first, 256, 5)
        syn, bad = _synthetic_on(single, 240, 8, first, 256, 11, fault_every=29)
        syn["n_jobs"] = 12
        syn["job_offsets"] = (np.arange(13) * 20).astype(np.uint32)
        jobs = G.sets_from_arrays(syn)
        want = [not bad[k * 20:(k + 1) * 20].any() for k in range(12)]
        jr1, _ = single.verify(syn)
        assert jr1.tolist() == [int(w) for w in want]
        retries = pool.metrics["batch_retries"]
        got = pool._run_device_batch(jobs)  # split over both contexts
        assert got == want
        assert pool.metrics["batch_retries"] == retries + 1
        clean = [j for j, w in zip(jobs, want) if w]
        assert pool._run_device_batch(clean) == [True] * len(clean)
        assert pool.metrics["batch_retries"] == retries + 1
        # golden jobs: rejected jobs stay rejected with their codes
        ga, gexp, _ = G.golden_arrays(scalars_seed=9)
        raw = ga["raw_pks"].reshape(-1, 96)
        gjobs = [[V.ISignatureSet(V.SignatureSetType.aggregate, s.signingRoot, s.signature,
                                  pubkeys=[V.PublicKey(raw=raw[p.index & 0x7FFFFFFF].tobytes()) if p.index & 0x80000000 else p
                                           for p in ([s.pubkey] if s.pubkey else s.pubkeys)])
                  for s in job] for job in G.sets_from_arrays(dict(ga, sigs=ga["sigs"].reshape(-1, 192),
                                                                   msgs=ga["msgs"].reshape(-1, 32)))]
        res = pool._run_device_batch(gjobs)
        assert [1 if r is True else 0 if r is False else -r.code for r in res] == gexp

        async def run():  # through the queue: block-sized calls split over both contexts
            return await asyncio.gather(*[pool.verify_signature_sets(j) for j in jobs])

        assert asyncio.run(run()) == want
    finally:
        single.close()
        asyncio.run(pool.close())
