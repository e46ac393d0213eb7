"""Shared helpers for the GPU parity tests: load the golden vectors into
bgv_batch arrays.  TEST ONLY."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def interop_pubkeys48() -> bytes:
    pks = json.load(open(os.path.join(GOLDEN, "interop-pubkeys.json")))
    return b"".join(bytes.fromhex(p[2:]) for p in pks)


_VECTORS = None


def batch_vectors():
    global _VECTORS
    if _VECTORS is None:
        _VECTORS = json.load(open(os.path.join(GOLDEN, "batch_vectors.json")))
    return _VECTORS


def load_golden_table(dev):
    """the device table the golden jobs index: the 100 interop keys, then the
    generator's extra rows (uncompressed: -P_24, the identity)"""
    from lodestar_amd import native
    v = batch_vectors()
    dev.pubkeys_set(0, interop_pubkeys48(), native.PK_COMPRESSED_48)
    dev.pubkeys_set(v["extra_table_base"], b"".join(bytes.fromhex(x) for x in v["extra_table"]), native.PK_UNCOMPRESSED_96)


def golden_arrays(jobs_sel=None, scalars_seed=None):
    """bgv_batch arrays for the golden jobs (all, or the ids in jobs_sel).
    scalars_seed=None: the generator's batch scalars (the ones its per-stage
    values were computed with); an int: fresh random scalars."""
    v = batch_vectors()
    raw = [bytes.fromhex(p) for p in v["raw_pubkeys"]]
    jobs = [v["jobs"][k] for k in (jobs_sel if jobs_sel is not None else range(len(v["jobs"])))]
    job_off, pk_off, idx, msgs, sigs, lens, exp_codes, scal = [0], [0], [], [], [], [], [], []
    for j in jobs:
        for s in j["sets"]:
            scal.append(int(s["scalar"]))
            if s["raw"] is not None:
                idx.append(0x80000000 | s["raw"])
            else:
                idx.extend(s["pk"])
            pk_off.append(len(idx))
            msgs.append(bytes.fromhex(s["msg"]))
            sig = bytes.fromhex(s["sig"])
            lens.append(len(sig))
            sigs.append(sig[:192].ljust(192, b"\0") if len(sig) in (96, 192) else bytes(192))
            exp_codes.append(s["code"])
        job_off.append(len(msgs))
    n = len(msgs)
    if scalars_seed is None:
        scalars = np.array(scal or [1], np.uint64)
    else:
        scalars = np.random.default_rng(scalars_seed).integers(1, 2**63, size=max(n, 1), dtype=np.uint64)
    arrays = {
        "n_sets": n,
        "n_jobs": len(jobs),
        "job_offsets": np.array(job_off, np.uint32),
        "pk_offsets": np.array(pk_off, np.uint32),
        "pk_indices": np.array(idx or [0], np.uint32),
        "raw_pks": np.frombuffer(b"".join(raw), np.uint8).copy(),
        "n_raw": len(raw),
        "msgs": np.frombuffer(b"".join(msgs) or bytes(32), np.uint8).copy(),
        "sigs": np.frombuffer(b"".join(sigs) or bytes(192), np.uint8).copy(),
        "sig_len": np.array(lens or [0], np.uint32),
        "scalars": scalars,
    }
    expected = [j["expected"] for j in jobs]
    return arrays, expected, exp_codes


def sets_from_arrays(arrays):
    """bgv_batch host arrays -> jobs of ISignatureSet (lodestar_amd.verifier)
    with table-index pubkeys: single for one key, aggregate otherwise"""
    from lodestar_amd import verifier as V
    jo, po, idx = arrays["job_offsets"], arrays["pk_offsets"], arrays["pk_indices"]
    jobs = []
    for j in range(arrays["n_jobs"]):
        sets = []
        for i in range(int(jo[j]), int(jo[j + 1])):
            keys = [V.PublicKey(index=int(x)) for x in idx[po[i]:po[i + 1]]]
            sig = arrays["sigs"][i, : int(arrays["sig_len"][i])].tobytes()
            root = arrays["msgs"][i].tobytes()
            if len(keys) == 1:
                sets.append(V.create_single_signature_set_from_components(keys[0], root, sig))
            else:
                sets.append(V.create_aggregate_signature_set_from_components(keys, root, sig))
        jobs.append(sets)
    return jobs
