"""GPU parity of the signature decode (Signature.fromBytes(sig, affine, true),
maybeBatch.ts:23,36) on waves that mix lanes taking different arms of the
Fp2 square root and of the ZCash sign choice (verdict r05 item 5).

A point of E2 with Im(x^3) = -4 has x^3 + 4(1 + i) in Fp, so its y is real
(y.c1 = 0: fp2_sqrt's Fp arm, and fp2_lex_largest decides on y.c0) or purely
imaginary (y.c0 = 0: the Fp arm's non-residue case).  Such points sit in
shuffled waves beside ordinary points, valid G2 signatures, the uncompressed
form of the same points, the identity and rejected encodings.  Every decoded
point and code, read back through the test-only entry bgv_debug_g2_decode, is
compared with the oracle's g2_decompress / g2_deserialize.  The same
encodings then go through bgv_verify as single-set jobs: the set codes are the
oracle's Signature.fromBytes codes (the special points are off the G2
subgroup: BLST_POINT_NOT_IN_GROUP), and the valid signatures verify.

gfx950 once miscompiled the early-return form of the sign choice under a
divergent exec mask (one signature in 66,640 decoded to -y);
fp2_lex_largest and fp2_sqrt have one exit since r06."""
import random

import numpy as np
import pytest

from oracle import bls12_381 as B
from tests import gpu_util as G
from tests.hostcheck import g2_b

P = B.P


def special_points(rnd: random.Random, want: int):
    """on-curve points with y.c1 = 0 and with y.c0 = 0 (each ~half)"""
    real, imag = [], []
    while len(real) < want or len(imag) < want:
        b = rnd.randrange(1, P)
        a2 = (pow(b, 3, P) - 4) * pow(3 * b, P - 2, P) % P
        a = B.fp_sqrt(a2)
        if a is None:
            continue
        if rnd.getrandbits(1):
            a = (-a) % P
        x = (a, b)
        rhs = B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B2)
        assert rhs[1] == 0
        t = rhs[0]
        r = B.fp_sqrt(t)
        if r is not None:
            if len(real) < want:
                real.append((x, (r, 0)))
        else:
            s = B.fp_sqrt((-t) % P)
            if len(imag) < want:
                imag.append((x, (0, s)))
    return real, imag


def ordinary_points(rnd: random.Random, n: int):
    out = []
    while len(out) < n:
        x = (rnd.randrange(P), rnd.randrange(P))
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B2))
        if y is not None and y[0] and y[1]:
            out.append((x, y))
    return out


def compress(pt, large: bool) -> bytes:
    """96-byte ZCash encoding of x with a chosen sign flag"""
    x, _ = pt
    out = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
    out[0] |= 0x80 | (0x20 if large else 0)
    return bytes(out)


def encodings(seed: int = 20261018):
    rnd = random.Random(seed)
    real, imag = special_points(rnd, 72)
    ordinary = ordinary_points(rnd, 96)
    encs = []
    for pt in real + imag + ordinary:
        encs.append(compress(pt, bool(rnd.getrandbits(1))))
    for pt in real[:12] + imag[:12]:  # uncompressed forms of the special points
        encs.append(B.g2_serialize(pt))
    v = G.batch_vectors()
    valid = [bytes.fromhex(s["sig"]) for j in v["jobs"] if j["expected"] == 1 for s in j["sets"]]
    encs += [s for s in valid if len(s) == 96][:16]
    # rejected and identity encodings
    x = (rnd.randrange(P), rnd.randrange(P))
    while B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B2)) is not None:
        x = (rnd.randrange(P), rnd.randrange(P))
    for _ in range(4):
        encs.append(compress((x, None), bool(rnd.getrandbits(1))))  # not on the curve
    encs.append(bytes([0xC0]) + bytes(95))                          # identity
    bad = bytearray(compress(real[0], True))
    bad[0] &= 0x7F                                                  # compression flag cleared
    encs.append(bytes(bad))
    big = bytearray((P + 5).to_bytes(48, "big") + bytes(48))        # x.c1 >= p
    big[0] |= 0x80
    encs.append(bytes(big))
    order = list(range(len(encs)))
    rnd.shuffle(order)
    encs = [encs[k] for k in order]
    # one wave of special points only, with alternating sign flags
    encs += [compress(pt, k % 2 == 0) for k, pt in enumerate((real[12:44] + imag[12:44]))]
    return encs


def oracle_decode(enc: bytes):
    code, pt = B.g2_decompress(enc) if len(enc) == 96 else B.g2_deserialize(enc)
    if code != B.BLST_SUCCESS or pt is None:
        return code, bytes(192)
    return code, g2_b(pt)


def test_special_points_generator():
    """the generator's points are on E2 with a zero y component"""
    rnd = random.Random(7)
    real, imag = special_points(rnd, 4)
    for x, y in real + imag:
        assert B.E2.on_curve((x, y))
        assert not B.g2_in_subgroup((x, y))
    assert all(y[1] == 0 for _, y in real) and all(y[0] == 0 for _, y in imag)
    encs = encodings()
    assert len(encs) >= 256


@pytest.mark.gpu
def test_decode_mixed_waves_match_oracle():
    from lodestar_amd import native
    encs = encodings()
    n = len(encs)
    sigs = np.zeros((n, 192), np.uint8)
    lens = np.zeros(n, np.uint32)
    for i, e in enumerate(encs):
        sigs[i, :len(e)] = np.frombuffer(e, np.uint8)
        lens[i] = len(e)
    d = native.Device(0)
    try:
        out, codes = d.debug_g2_decode(sigs, lens)
    finally:
        d.close()
    for i, e in enumerate(encs):
        code, want = oracle_decode(e)
        assert int(codes[i]) == code, ("code", i)
        assert out[i].tobytes() == want, ("point", i)


@pytest.mark.gpu
def test_verify_mixed_waves_set_codes():
    """the same encodings as single-set jobs through bgv_verify: set codes are
    the oracle's Signature.fromBytes codes, the golden valid signatures verify"""
    from lodestar_amd import native
    v = G.batch_vectors()
    valid = {}
    for j in v["jobs"]:
        if j["expected"] == 1:
            for s in j["sets"]:
                valid.setdefault(bytes.fromhex(s["sig"]), s)
    encs = encodings()
    n = len(encs)
    d = native.Device(0)
    try:
        G.load_golden_table(d)
        msgs, idx, want_codes, want_jobs = [], [], [], []
        for e in encs:
            s = valid.get(e)
            if s is not None and s["raw"] is None:
                msgs.append(bytes.fromhex(s["msg"]))
                idx.append(list(s["pk"]))
            else:
                msgs.append(bytes(32))
                idx.append([0])
            try:
                B.signature_from_bytes(e, True)
                code = 0
            except B.BlstError as err:
                code = err.code
            want_codes.append(code)
            want_jobs.append(-code if code else None)
        pk_off = np.cumsum([0] + [len(k) for k in idx]).astype(np.uint32)
        sigs = np.zeros((n, 192), np.uint8)
        for i, e in enumerate(encs):
            sigs[i, :len(e)] = np.frombuffer(e, np.uint8)
        arrays = {
            "n_sets": n, "n_jobs": n,
            "job_offsets": np.arange(n + 1, dtype=np.uint32),
            "pk_offsets": pk_off,
            "pk_indices": np.array([k for ks in idx for k in ks], np.uint32),
            "raw_pks": np.zeros(1, np.uint8), "n_raw": 0,
            "msgs": np.frombuffer(b"".join(msgs), np.uint8).copy(),
            "sigs": sigs.reshape(-1).copy(),
            "sig_len": np.array([len(e) for e in encs], np.uint32),
            "scalars": np.random.default_rng(5).integers(1, 2**63, size=n, dtype=np.uint64),
        }
        out = d.debug_stages(arrays)
    finally:
        d.close()
    assert out["set_code"].tolist() == want_codes
    res = out["job_result"].tolist()
    for i, e in enumerate(encs):
        if want_jobs[i] is not None:
            assert res[i] == want_jobs[i], ("job", i)
        elif e in valid and valid[e]["raw"] is None:
            assert res[i] == 1, ("valid", i)
        elif B.signature_from_bytes(e, True) is None:
            assert res[i] == 0, ("identity", i)
