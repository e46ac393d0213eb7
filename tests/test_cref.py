"""The C restatement (oracle/bls_ref.c) against the pinned Python oracle and
the golden vectors.  CPU only."""
import json
import os
import subprocess

import pytest

from oracle import bls12_381 as B
from tests import gpu_util as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def C():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    from oracle import cref
    return cref


def test_sk_to_pk_matches_interop_kat(C):
    """all 100 keys of the reference's test-cache/interop-pubkeys.json =
    compress(sk_i G1), sk_i from interop.ts:19-23"""
    pks = json.load(open(os.path.join(G.GOLDEN, "interop-pubkeys.json")))
    assert len(pks) == 100
    for i in range(100):
        sk = B.interop_secret_key(i)
        pt = B.g1_decompress(bytes.fromhex(pks[i][2:]))[1]
        assert C.sk_to_pk(sk) == B.g1_serialize(pt)


def test_hash_and_sign_match_python_oracle(C):
    for m in (bytes(32), bytes(range(32)), b"\xff" * 32):
        assert C.hash_to_g2(m) == B.g2_serialize(B.hash_to_g2(m))
    assert C.sign(12345, bytes(range(32))) == B.g2_compress(B.sign(12345, bytes(range(32))))


def test_deposit_kat(C):
    from tests.test_oracle_kat import deposit0_signing_root, DEPOSIT0_SIG
    sk, _, root = deposit0_signing_root()
    assert C.sign(sk, root).hex() == DEPOSIT0_SIG


def test_golden_jobs(C):
    v = G.batch_vectors()
    pks48 = G.interop_pubkeys48()
    raw = [bytes.fromhex(p) for p in v["raw_pubkeys"]]
    base, extra = v["extra_table_base"], [bytes.fromhex(p) for p in v["extra_table"]]

    def row(i):
        return extra[i - base] if i >= base else B.g1_serialize(B.g1_decompress(pks48[48 * i : 48 * i + 48])[1])

    checked = 0
    for jid, job in enumerate(v["jobs"]):
        pks, msgs, sigs = [], [], []
        if any(s["raw"] is None and max(s["pk"]) >= base + len(extra) for s in job["sets"]):
            assert job["expected"] == -9  # index past the table: rejected by construction
            continue
        for s in job["sets"]:
            if s["raw"] is not None:
                pks.append(raw[s["raw"]])
            else:
                pks.append(C.aggregate([row(i) for i in s["pk"]]))
            msgs.append(bytes.fromhex(s["msg"]))
            sigs.append(bytes.fromhex(s["sig"]))
        assert C.verify_job(pks, msgs, sigs) == job["expected"], jid
        checked += 1
    assert checked == len(v["jobs"]) - 1


def test_aggregate_matches_python(C):
    sks = [3, 5, 7, 11]
    pts = [B.sk_to_pk(s) for s in sks]
    assert C.aggregate([B.g1_serialize(p) for p in pts]) == B.g1_serialize(B.aggregate_pubkeys(pts))
    # P + P (doubling inside aggregation) and P + (-P) (infinity)
    p = B.sk_to_pk(9)
    assert C.aggregate([B.g1_serialize(p)] * 2) == B.g1_serialize(B.E1.add(p, p))
    assert C.aggregate([B.g1_serialize(p), B.g1_serialize(B.E1.neg(p))]) == B.g1_serialize(None)


def test_mulx_header_is_generated():
    """oracle/bls_ref_mulx.h is the output of tools/gen_cref_mulx.py"""
    import os
    from tools import gen_cref_mulx
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    assert open(os.path.join(root, "oracle", "bls_ref_mulx.h")).read() == gen_cref_mulx.gen()
