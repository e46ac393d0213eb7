"""Generate tests/golden/batch_vectors.json with the Python oracle.

Run in the build container (the oracle is test infrastructure; only the
JSON travels to the GPU box).  Pubkeys come from the reference's own
interop table (tests/golden/interop-pubkeys.json = packages/state-transition/
test-cache/interop-pubkeys.json) plus the three raw keys of
packages/beacon-node/test/e2e/chain/bls/multithread.test.ts:25-38
(sk = 0x0101..01 / 0x0202..02 / 0x0303..03, msg = the same 32 bytes).
Expected verdicts / errors are computed by oracle.verify_job, i.e. the
reference's maybeBatch semantics restated.

Every set also carries its batch scalar and the canonical per-stage values
the device must reproduce (SURVEY §8c golden plan; compared on the GPU by
tests/test_gpu_stages.py through bgv_debug_stages): the decoded signature,
H(m), the aggregated pubkey, r * pubkey, and the GT value of its Miller pair;
every job its S_job = sum r_i sigma_i and the GT value of its product.  GT
values are e(P, Q)^3 (the device's final exponentiation computes the cube of
the textbook value, include/bgv.h bgv_debug) as 12 flat coefficients of
oracle.f12 (Fp[w]/(w^12 - 2 w^6 + 2)).  Points: G1 x || y, G2 x.c0 || x.c1
|| y.c0 || y.c1, 48-byte big-endian, all-zero for the identity / rejected.

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


TABLE_BASE = 100  # extra_table rows follow the 100 interop keys
INDEX_RANGE = 9   # include/bgv.h BGV_SET_INDEX_RANGE: index2pubkey[i] undefined on the caller's side


def scalar(i):
    """batch scalar of golden set i (64-bit, non-zero)"""
    return int.from_bytes(hashlib.sha256(b"golden-scalar" + i.to_bytes(4, "little")).digest()[:8], "little") | 1


def fp_b(v):
    return (v % B.P).to_bytes(48, "big")


def g1_b(pt):
    return bytes(96) if pt is None else fp_b(pt[0]) + fp_b(pt[1])


def g2_b(pt):
    return bytes(192) if pt is None else b"".join(fp_b(c) for c in (pt[0][0], pt[0][1], pt[1][0], pt[1][1]))


def gt_hex(f):
    return "".join(fp_b(c).hex() for c in f)


def cube(f):
    return B.f12_mul(B.f12_mul(f, f), f)


def main():
    interop = json.load(open(os.path.join(ROOT, "tests", "golden", "interop-pubkeys.json")))
    sks = [B.interop_secret_key(i) for i in range(len(interop))]
    pts = {}
    # rows appended after the interop keys (uncompressed 96 B): -P_24, the identity
    neg24 = B.E1.neg(B.g1_decompress(bytes.fromhex(interop[24][2:]))[1])
    extra_table = [B.g1_serialize(neg24), bytes([0x40]) + bytes(95)]
    extra_pts = {TABLE_BASE: neg24, TABLE_BASE + 1: None}

    def pk_point(idxs):
        acc = None
        for i in idxs:
            if i >= TABLE_BASE:
                acc = B.E1.add(acc, extra_pts[i])
                continue
            if i not in pts:
                pts[i] = B.g1_decompress(bytes.fromhex(interop[i][2:]))[1]
            acc = B.E1.add(acc, pts[i])
        return acc

    # raw keys of multithread.test.ts:25-38, then the uncompressed identity (raw key 3)
    raw_sks = [int.from_bytes(bytes([k + 1]) * 32, "big") % B.R for k in range(3)]
    raw_pks = [B.g1_serialize(B.sk_to_pk(s)) for s in raw_sks] + [bytes([0x40]) + bytes(95)]
    raw_pts = [B.sk_to_pk(s) for s in raw_sks] + [None]

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
    # J16: P + (-P) aggregates to the identity -> BLST_PK_IS_INFINITY (blst
    # Pairing.mul_n_aggregate); the signature is the identity (sk sum 0)
    jobs.append([S([25], m=msg(30), sig=agg_sig([sks[25]], msg(30))),
                 S([24, TABLE_BASE], m=msg(31), sig=bytes([0xC0]) + bytes(95))])
    # J17: a valid set, then a set whose only (raw) key is the identity -> BLST_PK_IS_INFINITY
    jobs.append([S([26], m=msg(32), sig=agg_sig([sks[26]], msg(32))),
                 S(raw=3, m=msg(33), sig=agg_sig([sks[27]], msg(33)))])
    # J18: a pubkey index past the table -> rejected per set (BGV_INDEX_RANGE); the
    # reference's index2pubkey[i] is undefined and the caller throws
    jobs.append([S([28], m=msg(34), sig=agg_sig([sks[28]], msg(34))),
                 S([29, 5000], m=msg(35), sig=agg_sig([sks[29]], msg(35)))])
    # J19: 192-byte signature with the sign flag (0x20) -> BAD_ENCODING
    u = bytearray(B.g2_serialize(B.sign(sks[30], msg(36))))
    u[0] |= 0x20
    jobs.append([S([30], m=msg(36), sig=bytes(u))])
    # J20: precedence: set 0's pubkeys sum to the identity, set 1's signature
    # does not decode -> every signature is parsed first (maybeBatch.ts:20-24):
    # BAD_ENCODING, not PK_IS_INFINITY
    jobs.append([S([24, TABLE_BASE], m=msg(37), sig=bytes([0xC0]) + bytes(95)),
                 S([31], m=msg(38), sig=bytes(xp))])
    # J21: two valid sets on the appended rows' neighbours, one key repeated
    # across sets (a 2-set batch, non-trivial S_job)
    jobs.append([S([32, 33, 34], m=msg(39), sig=agg_sig([sks[32], sks[33], sks[34]], msg(39))),
                 S([34], m=msg(40), sig=agg_sig([sks[34]], msg(40)))])

    out_jobs = []
    set_no = 0
    batch_gt = B.F12_ONE
    neg_g1 = B.E1.neg(B.G1)
    for jid, job in enumerate(jobs):
        sets, inter = [], []
        range_err = False
        for s in job:
            if s["raw"] is not None:
                pkp = raw_pts[s["raw"]]
            elif any(i >= TABLE_BASE + len(extra_table) for i in s["pk"]):
                pkp, range_err = None, True
            else:
                pkp = pk_point(s["pk"])
            sets.append((pkp, s["msg"], s["sig"]))
        codes, sig_pts = [], []
        for s in job:
            try:
                sig_pts.append(B.signature_from_bytes(s["sig"], True))
                codes.append(0)
            except B.BlstError as e:
                sig_pts.append(None)
                codes.append(e.code)
        for k, s in enumerate(job):  # device set code: signature code, else pubkey code
            if codes[k] == 0:
                if s["raw"] is None and any(i >= TABLE_BASE + len(extra_table) for i in s["pk"]):
                    codes[k] = INDEX_RANGE
                elif sets[k][0] is None:
                    codes[k] = B.BLST_PK_IS_INFINITY
        sig_codes = [c if c not in (INDEX_RANGE, B.BLST_PK_IS_INFINITY) else 0 for c in codes]
        if range_err and not any(sig_codes):
            verdict = -INDEX_RANGE
        else:
            try:
                verdict = 1 if B.verify_job(sets) else 0
            except B.BlstError as e:
                verdict = -e.code
            except ValueError:
                verdict = -10
        job_ok = verdict >= 0
        s_acc = None
        job_gt = B.F12_ONE
        for k, s in enumerate(job):
            r = scalar(set_no + k)
            pkp = sets[k][0]
            h = B.hash_to_g2(s["msg"])
            rpk = B.E1.mul(pkp, r) if pkp is not None else None
            pair = cube(B.pairing(rpk, h)) if rpk is not None else B.F12_ONE
            inter.append({"scalar": str(r), "sig_aff": g2_b(sig_pts[k]).hex(), "h_aff": g2_b(h).hex(),
                          "pk_agg": g1_b(pkp).hex(), "rpk_aff": g1_b(rpk).hex(), "pair_gt": gt_hex(pair)})
            if job_ok:
                if sig_pts[k] is not None:
                    s_acc = B.E2.add(s_acc, B.E2.mul(sig_pts[k], r))
                job_gt = B.f12_mul(job_gt, pair)
        job_pair = B.F12_ONE
        if job_ok and s_acc is not None:
            job_pair = cube(B.pairing(neg_g1, s_acc))
            job_gt = B.f12_mul(job_gt, job_pair)
        if not job_ok:
            s_acc = None
            job_gt = B.F12_ONE
        batch_gt = B.f12_mul(batch_gt, job_gt)
        assert (verdict == 1) == (job_ok and B.f12_eq(job_gt, B.F12_ONE)) or verdict < 0
        set_no += len(job)
        out_jobs.append({
            "expected": verdict,
            "s_aff": g2_b(s_acc).hex(),
            "job_pair_gt": gt_hex(job_pair),
            "job_gt": gt_hex(job_gt),
            "sets": [dict({"pk": s["pk"], "raw": s["raw"], "msg": s["msg"].hex(), "sig": s["sig"].hex(), "code": c}, **it)
                     for s, c, it in zip(job, codes, inter)],
        })
        print(jid, verdict, codes, flush=True)
    json.dump({"generator": "tools/gen_golden.py (oracle/bls12_381.py)",
               "gt_note": "GT values are e(P, Q)^3 as 12 flat coefficients of oracle.f12 (Fp[w]/(w^12 - 2 w^6 + 2))",
               "raw_pubkeys": [p.hex() for p in raw_pks], "extra_table_base": TABLE_BASE,
               "extra_table": [p.hex() for p in extra_table], "batch_gt": gt_hex(batch_gt),
               "jobs": out_jobs}, open(OUT, "w"), indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
