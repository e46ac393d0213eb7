"""The HBM index2pubkey table's lifecycle on the GPU (pubkeyCache.ts:56-77
syncPubkeys, epochContext.ts:701-704 addPubkey) and the index error class:

* growth then verify: a set naming a row not yet synced is rejected per set
  (BGV_INDEX_RANGE) while a co-batched job verifies; after the sync it verifies;
* a write past the end (a gap) or past 2^31 - 1 rows fails and changes nothing;
* a key that does not deserialize fails the whole write (PublicKey.fromBytes
  throws) and leaves the table as it was;
* addPubkey rewrites a row in place; the identity key aggregates as nothing;
* the Python PubkeyTable mirror raises BlsError the way the reference throws.
Keys are the reference's interop keys; signatures come from the C restatement
(oracle/bls_ref.c), pinned to the Python oracle in test_cref."""
import numpy as np
import pytest

from oracle import bls12_381 as B
from tests import gpu_util as G

pytestmark = pytest.mark.gpu


def _keys():
    pks = G.interop_pubkeys48()
    return [pks[48 * i: 48 * i + 48] for i in range(100)]


def _job_arrays(sets):
    """sets: [(indices, msg, sig96)] -> one job per set"""
    n = len(sets)
    idx = [i for s in sets for i in s[0]]
    return {"n_sets": n, "n_jobs": n, "job_offsets": np.arange(n + 1, dtype=np.uint32),
            "pk_offsets": np.concatenate([[0], np.cumsum([len(s[0]) for s in sets])]).astype(np.uint32),
            "pk_indices": np.array(idx, np.uint32),
            "msgs": np.frombuffer(b"".join(s[1] for s in sets), np.uint8).reshape(n, 32).copy(),
            "sigs": np.frombuffer(b"".join(s[2].ljust(192, b"\0") for s in sets), np.uint8).reshape(n, 192).copy(),
            "sig_len": np.full(n, 96, np.uint32), "scalars": np.arange(1, n + 1, dtype=np.uint64), "n_raw": 0}


def _signed(indices, tag):
    from oracle import cref
    m = bytes([tag]) * 32
    sk = sum(B.interop_secret_key(i) for i in indices) % B.R
    return (indices, m, cref.sign(sk, m))


def test_table_growth_gap_bad_key_and_rewrite():
    from lodestar_amd import native
    keys = _keys()
    d = native.Device(0)
    try:
        d.pubkeys_set(0, b"".join(keys[:50]), native.PK_COMPRESSED_48)
        assert d.pubkeys_count() == 50
        early, late = _signed([3, 7], 1), _signed([60, 2], 2)
        jr, sc = d.verify(_job_arrays([early, late]))
        assert jr.tolist() == [1, -9] and sc.tolist() == [0, 9]  # row 60 not synced yet
        # a gap is refused, and so is a row count past 2^31 - 1
        with pytest.raises(native.BgvNativeError) as e:
            d.pubkeys_set(60, keys[60], native.PK_COMPRESSED_48)
        assert e.value.status == native.BGV_E_TABLE_RANGE
        with pytest.raises(native.BgvNativeError) as e:
            d.pubkeys_set(0xFFFFFFF0, b"".join(keys[:32]), native.PK_COMPRESSED_48)
        assert e.value.status == native.BGV_E_TABLE_RANGE
        # a key that does not deserialize fails the whole write, nothing stored
        bad = bytes([keys[55][0] & 0x7F]) + keys[55][1:]  # compression flag cleared
        with pytest.raises(native.BgvNativeError) as e:
            d.pubkeys_set(50, b"".join(keys[50:55]) + bad, native.PK_COMPRESSED_48)
        assert e.value.status == native.BGV_E_BAD_PUBKEY and "BLST_BAD_ENCODING" in str(e.value)
        assert d.pubkeys_count() == 50
        # not on the curve (uncompressed import)
        x = bytearray(B.g1_serialize(B.g1_decompress(keys[1])[1]))
        x[95] ^= 1
        with pytest.raises(native.BgvNativeError) as e:
            d.pubkeys_set(50, bytes(x), native.PK_UNCOMPRESSED_96)
        assert "BLST_POINT_NOT_ON_CURVE" in str(e.value) and d.pubkeys_count() == 50
        # sync the rest: the pending set now verifies
        d.pubkeys_set(50, b"".join(keys[50:]), native.PK_COMPRESSED_48)
        assert d.pubkeys_count() == 100
        jr, _ = d.verify(_job_arrays([early, late]))
        assert jr.tolist() == [1, 1]
        # addPubkey rewrites row 10 with key 11: a set naming row 10 now needs sk_11
        d.pubkeys_set(10, keys[11], native.PK_COMPRESSED_48)
        assert d.pubkeys_count() == 100
        by10, by11 = _signed([10], 3), _signed([11], 3)
        jr, _ = d.verify(_job_arrays([([10], by10[1], by10[2]), ([10], by11[1], by11[2])]))
        assert jr.tolist() == [0, 1]
        d.pubkeys_set(10, keys[10], native.PK_COMPRESSED_48)
        # the identity key (compressed 0xc0..) is stored and aggregates as nothing
        d.pubkeys_set(100, bytes([0xC0]) + bytes(47), native.PK_COMPRESSED_48)
        s = _signed([5], 4)
        jr, sc = d.verify(_job_arrays([([5, 100], s[1], s[2]), ([100], s[1], s[2])]))
        assert jr.tolist() == [1, -6] and sc.tolist() == [0, 6]
    finally:
        d.close()


def test_pubkey_table_mirror_errors():
    import asyncio

    from lodestar_amd import verifier as V
    keys = _keys()
    pool = V.BlsGpuVerifier(devices=(0,))
    try:
        pool.table.sync_pubkeys(keys[:20])
        assert len(pool.table) == 20 and pool.table.pubkey2index[keys[19]] == 19
        pool.table.sync_pubkeys(keys[:40])  # appends 20..39 only
        assert len(pool.table) == 40
        bad = bytes([0x9F]) + b"\xff" * 47  # x >= p
        with pytest.raises(V.BlsError, match="BLST_BAD_ENCODING"):
            pool.table.sync_pubkeys(keys[:40] + [bad])
        assert len(pool.table) == 40
        pool.table.add_pubkey(40, keys[40])
        assert len(pool.table) == 41
        s = _signed([40, 1], 9)
        sets = [V.create_aggregate_signature_set_from_components([pool.table[40], pool.table[1]], s[1], s[2])]
        assert pool.verify_signature_sets_maybe_batch(sets)
        out = [V.create_single_signature_set_from_components(pool.table[4000], s[1], s[2])]
        with pytest.raises(V.BlsError, match="BGV_INDEX_RANGE"):
            pool.verify_signature_sets_maybe_batch(out)
    finally:
        asyncio.run(pool.close())
