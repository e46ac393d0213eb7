"""Generate tests/golden/batch_vectors.json with the Python oracle.

Run in the build container (the oracle is test infrastructure; only the
JSON travels to the GPU box).  Pubkeys come from the reference's own
interop table (tests/golden/interop-pubkeys.json = packages/state-transition/
test-cache/interop-pubkeys.json) plus the three raw keys of
packages/beacon-node/test/e2e/chain/bls/multithread.test.ts:25-38
(sk = 0x0101..01 / 0x0202..02 / 0x0303..03, msg = the same 32 bytes).
Expected verdicts / errors are computed by oracle.verify_job, i.e. the
reference's maybeBatch semantics restated.

    python tools/gen_golden.py
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12_381 as B  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "batch_vectors.json")
DEPOSIT0_SIG = (
    "a95af8ff0f8c06af4d29aef05ce865f85f82df42b606008ec5b1bcb42b17ae47f4b78cdce1db31ce32d18f42a6b296b4"
    "014a2164981780e56b5a40d7723c27b8423173e58fa36f075078b177634f66351412b867c103f532aedd50bcd9b98446"
)


def msg(i):
    return hashlib.sha256(b"golden-msg" + i.to_bytes(4, "little")).digest()


def agg_sig(sks, m):
    return B.g2_compress(B.sign(sum(sks) % B.R, m))


def not_on_curve_sig():
    x0 = 1
    while True:
        x = (x0, 1)
        if B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B2)) is None:
            out = bytearray(B._tobe(x[1]) + B._tobe(x[0]))
            out[0] |= 0x80
            return bytes(out)
        x0 += 1


def not_in_group_sig():
    x0 = 3
    while True:
        x = (x0, 7)
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B2))
        if y is not None and not B.g2_in_subgroup((x, y)):
            return B.g2_compress((x, y))
        x0 += 1


def main():
    interop = json.load(open(os.path.join(ROOT, "tests", "golden", "interop-pubkeys.json")))
    sks = [B.interop_secret_key(i) for i in range(len(interop))]
    pts = {}

    def pk_point(idxs):
        acc = None
        for i in idxs:
            if i not in pts:
                pts[i] = B.g1_decompress(bytes.fromhex(interop[i][2:]))[1]
            acc = B.E1.add(acc, pts[i])
        return acc

    # raw keys of multithread.test.ts:25-38
    raw_sks = [int.from_bytes(bytes([k + 1]) * 32, "big") % B.R for k in range(3)]
    raw_pks = [B.g1_serialize(B.sk_to_pk(s)) for s in raw_sks]

    jobs = []  # list of list of set dicts

    def S(pk_idx=None, raw=None, m=None, sig=None):
        return {"pk": pk_idx or [], "raw": raw, "msg": m, "sig": sig}

    # J0: multithread.test.ts valid single sets (raw pubkeys, msg = sk bytes)
    jobs.append([S(raw=k, m=bytes([k + 1]) * 32, sig=B.g2_compress(B.sign(raw_sks[k], bytes([k + 1]) * 32))) for k in range(3)])
    # J1: aggregate (k=5) + single, valid
    jobs.append([S([1, 2, 3, 4, 5], m=msg(1), sig=agg_sig([sks[i] for i in [1, 2, 3, 4, 5]], msg(1))),
                 S([7], m=msg(2), sig=agg_sig([sks[7]], msg(2)))])
    # J2: wrong message (valid point) -> false
    jobs.append([S([8], m=msg(3), sig=agg_sig([sks[8]], msg(3))),
                 S([9], m=msg(4), sig=agg_sig([sks[9]], msg(99)))])
    # J3: 32-byte signature -> BLST_INVALID_SIZE (multithread.test.ts:86-103)
    jobs.append([S([10], m=msg(5), sig=bytes(32))])
    # J4: compression flag cleared -> BAD_ENCODING
    good = bytearray(agg_sig([sks[11]], msg(6)))
    bad = bytearray(good)
    bad[0] &= 0x7F
    jobs.append([S([11], m=msg(6), sig=bytes(good)), S([11], m=msg(6), sig=bytes(bad))])
    # J5: x1 >= p -> BAD_ENCODING
    xp = bytearray(B._tobe(B.P) + bytes(48))
    xp[0] |= 0x80
    jobs.append([S([12], m=msg(7), sig=bytes(xp))])
    # J6: not on curve
    jobs.append([S([13], m=msg(8), sig=not_on_curve_sig()), S([13], m=msg(8), sig=agg_sig([sks[13]], msg(8)))])
    # J7: on curve, not in G2
    jobs.append([S([14], m=msg(9), sig=agg_sig([sks[14]], msg(9))), S([14], m=msg(9), sig=not_in_group_sig())])
    # J8: infinity signature, single set -> false
    jobs.append([S([15], m=msg(10), sig=bytes([0xC0]) + bytes(95))])
    # J9: uncompressed 192-byte signature, valid
    jobs.append([S([16, 17], m=msg(11), sig=B.g2_serialize(B.sign((sks[16] + sks[17]) % B.R, msg(11))))])
    # J10: swapped pubkey (sig by 18, pubkey 19) -> false
    jobs.append([S([19], m=msg(12), sig=agg_sig([sks[18]], msg(12))), S([20], m=msg(13), sig=agg_sig([sks[20]], msg(13)))])
    # J11: deposit #0 KAT (genesisState.test.ts:50-55), valid
    from tests.test_oracle_kat import deposit0_signing_root
    _, _, root = deposit0_signing_root()
    jobs.append([S([0], m=root, sig=bytes.fromhex(DEPOSIT0_SIG))])
    # J12: a 40-pubkey aggregate + 3 singles, valid
    agg = list(range(40, 80))
    jobs.append([S(agg, m=msg(14), sig=agg_sig([sks[i] for i in agg], msg(14)))] +
                [S([80 + k], m=msg(15 + k), sig=agg_sig([sks[80 + k]], msg(15 + k))) for k in range(3)])
    # J13: duplicate pubkey in an aggregate (P + P doubling path), valid
    jobs.append([S([21, 21, 22], m=msg(20), sig=agg_sig([sks[21], sks[21], sks[22]], msg(20)))])
    # J14: signature uncompressed 192 bytes but flag 0x80 set -> BAD_ENCODING
    u = bytearray(B.g2_serialize(B.sign(sks[23], msg(21))))
    u[0] |= 0x80
    jobs.append([S([23], m=msg(21), sig=bytes(u))])
    # J15: empty job (chunkify of [] = [[]]) -> "Empty signature set"
    jobs.append([])

    out_jobs = []
    for jid, job in enumerate(jobs):
        sets = []
        for s in job:
            pkp = pk_point(s["pk"]) if s["raw"] is None else B.sk_to_pk(raw_sks[s["raw"]])
            sets.append((pkp, s["msg"], s["sig"]))
        try:
            verdict = 1 if B.verify_job(sets) else 0
        except B.BlstError as e:
            verdict = -e.code
        except ValueError:
            verdict = -10
        codes = []
        for s in job:
            try:
                B.signature_from_bytes(s["sig"], True)
                codes.append(0)
            except B.BlstError as e:
                codes.append(e.code)
        out_jobs.append({
            "expected": verdict,
            "sets": [{"pk": s["pk"], "raw": s["raw"], "msg": s["msg"].hex(), "sig": s["sig"].hex(), "code": c}
                     for s, c in zip(job, codes)],
        })
        print(jid, verdict, codes, flush=True)
    json.dump({"generator": "tools/gen_golden.py (oracle/bls12_381.py)",
               "raw_pubkeys": [p.hex() for p in raw_pks], "jobs": out_jobs}, open(OUT, "w"), indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
