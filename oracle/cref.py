"""ctypes view of oracle/libbls_ref.so (the C restatement, oracle/bls_ref.c).

TEST INFRASTRUCTURE: used by tests/ as a checker and by bench.py's
cpu_baseline leg.  Never imported by lodestar_amd/.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libbls_ref.so")
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} not built (make -C oracle)")
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        L.bref_init.restype = None
        L.bref_verify_job.argtypes = [P, P, P, P, ctypes.c_int, P]
        L.bref_verify_job.restype = ctypes.c_int
        L.bref_aggregate.argtypes = [P, ctypes.c_int, P]
        L.bref_sk_to_pk.argtypes = [P, P]
        L.bref_sign.argtypes = [P, P, P]
        L.bref_hash_to_g2.argtypes = [P, ctypes.c_int, P]
        L.bref_bench_jobs.argtypes = [P, ctypes.c_int, P, P, P, P, P, P, ctypes.c_int, P]
        L.bref_bench_jobs.restype = ctypes.c_double
        L.bref_init()
        _lib = L
    return _lib


def _buf(b: bytes):
    return ctypes.create_string_buffer(bytes(b), len(b))


def sk_to_pk(sk: int) -> bytes:
    out = ctypes.create_string_buffer(96)
    lib().bref_sk_to_pk(_buf(sk.to_bytes(32, "big")), out)
    return out.raw


def sign(sk: int, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(96)
    lib().bref_sign(_buf((sk % R).to_bytes(32, "big")), _buf(msg), out)
    return out.raw


def hash_to_g2(msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(192)
    lib().bref_hash_to_g2(_buf(msg), len(msg), out)
    return out.raw


def aggregate(pks96: list[bytes]) -> bytes:
    out = ctypes.create_string_buffer(96)
    lib().bref_aggregate(_buf(b"".join(pks96)), len(pks96), out)
    return out.raw


def verify_job(pks96: list[bytes], msgs: list[bytes], sigs: list[bytes], scalars=None) -> int:
    """maybeBatch semantics for one job; 1 / 0 / -blst_code (-10 = empty job)."""
    n = len(msgs)
    sb = b"".join(s[:192].ljust(192, b"\0") if len(s) in (96, 192) else bytes(192) for s in sigs)
    lens = np.array([len(s) for s in sigs] or [0], np.uint32)
    sc = np.array(scalars if scalars is not None else [i + 1 for i in range(max(n, 1))], np.uint64)
    return lib().bref_verify_job(_buf(b"".join(pks96) or bytes(96)), _buf(b"".join(msgs) or bytes(32)),
                                 _buf(sb or bytes(192)), lens.ctypes.data, n, sc.ctypes.data)


def device_sk(seed: int, i: int) -> int:
    """the synthetic key rule of bgv_gen_keys (include/bgv.h)"""
    h = hashlib.sha256(b"bgv-sk" + seed.to_bytes(8, "little") + i.to_bytes(4, "little")).digest()
    return int.from_bytes(h, "big") % R


def bench_segment_sample(budget_s: float = 15.0, seed: int = 0x4C4F4445, threads: int | None = None,
                         table: int = 4096, blocks: int | None = None) -> dict:
    """Time the reference pool's work on a bounded sample of the C4 workload
    (blocks of 95 x k=128 + 1 x k=512 + 2 singles, one job per block, one job
    per worker at a time) on `threads` host cores.  The table is `table`
    keys (aggregation cost depends on k, not on the table size)."""
    L = lib()
    threads = threads or min(16, os.cpu_count() or 1)
    rng = np.random.default_rng(seed)
    sks = [device_sk(seed, i) for i in range(table)]
    with ThreadPoolExecutor(threads) as ex:  # ctypes releases the GIL
        pks = list(ex.map(sk_to_pk, sks))
    table96 = np.frombuffer(b"".join(pks), np.uint8).copy()

    def block_sets(b):
        sets = []
        for a in range(95):
            sets.append(rng.choice(table, size=128, replace=False))
        sets.append(rng.choice(table, size=512, replace=False))
        sets.extend([rng.integers(0, table, size=1), rng.integers(0, table, size=1)])
        return sets

    # calibrate: one block per thread first, then as many as fit in the budget
    def run(nb):
        all_sets, msgs = [], []
        job_off, pk_off, idx = [0], [0], []
        for b in range(nb):
            for k, s in enumerate(block_sets(b)):
                all_sets.append(s)
                idx.extend(int(v) for v in s)
                pk_off.append(len(idx))
                msgs.append(hashlib.sha256(b"bgv-cpu" + seed.to_bytes(8, "little") + (b * 98 + k).to_bytes(4, "little")).digest())
            job_off.append(len(all_sets))
        with ThreadPoolExecutor(threads) as ex:
            sigs = list(ex.map(lambda t: sign(sum(sks[int(v)] for v in t[0]) % R, t[1]), zip(all_sets, msgs)))
        n = len(all_sets)
        res = np.zeros(nb, np.int32)
        sig_arr = np.frombuffer(b"".join(s.ljust(192, b"\0") for s in sigs), np.uint8).copy()
        # keep every array alive across the call (ctypes gets raw addresses)
        a_job = np.array(job_off, np.uint32)
        a_pk = np.array(pk_off, np.uint32)
        a_idx = np.array(idx, np.uint32)
        a_msg = np.frombuffer(b"".join(msgs), np.uint8).copy()
        a_len = np.full(n, 96, np.uint32)
        wall = L.bref_bench_jobs(a_job.ctypes.data, nb, a_pk.ctypes.data, a_idx.ctypes.data, table96.ctypes.data,
                                 a_msg.ctypes.data, sig_arr.ctypes.data, a_len.ctypes.data, threads, res.ctypes.data)
        assert (res == 1).all(), res
        return n, wall

    if blocks is None:
        n, wall = run(threads)
        per_block = wall / 1.0  # one block per thread ran in parallel
        extra = int(max(0, budget_s - wall) / max(per_block, 1e-3)) * threads
        if extra >= threads:
            n2, wall2 = run(extra)
            n, wall = n2, wall2
    else:
        n, wall = run(blocks)
    return {"value": round(n / wall, 1), "unit": "sets/s", "cores": threads, "kind": "port",
            "sample": f"{n} sets = {n // 98} C4 blocks (95 x k=128, 1 x k=512, 2 singles; one job per block), "
                      f"{table}-key table, oracle/bls_ref.c (6x64-bit limbs, x86-64-v3) on {threads} threads, "
                      f"aggregation inside the workers; wall {wall:.2f} s",
            "per_set_core_ms": round(wall * threads / n * 1e3, 3)}
