"""Shared helpers for the GPU parity tests: load the golden vectors into
bgv_batch arrays.  TEST ONLY."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def interop_pubkeys48() -> bytes:
    pks = json.load(open(os.path.join(GOLDEN, "interop-pubkeys.json")))
    return b"".join(bytes.fromhex(p[2:]) for p in pks)


def batch_vectors():
    return json.load(open(os.path.join(GOLDEN, "batch_vectors.json")))


def golden_arrays(jobs_sel=None, scalars_seed=7):
    """bgv_batch arrays for the golden jobs (all, or the ids in jobs_sel)."""
    v = batch_vectors()
    raw = [bytes.fromhex(p) for p in v["raw_pubkeys"]]
    jobs = [v["jobs"][k] for k in (jobs_sel if jobs_sel is not None else range(len(v["jobs"])))]
    job_off, pk_off, idx, msgs, sigs, lens, exp_codes = [0], [0], [], [], [], [], []
    for j in jobs:
        for s in j["sets"]:
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
    rng = np.random.default_rng(scalars_seed)
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
        "scalars": rng.integers(1, 2**63, size=max(n, 1), dtype=np.uint64),
    }
    expected = [j["expected"] for j in jobs]
    return arrays, expected, exp_codes
