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


class _Workload:
    """A keyed table plus signed sets for the CPU pool benchmarks: `table`
    synthetic keys (the bgv_gen_keys rule), sets signed by the C restatement."""

    def __init__(self, threads: int, seed: int, table: int):
        self.threads, self.seed, self.table = threads, seed, table
        self.rng = np.random.default_rng(seed)
        self.sks = [device_sk(seed, i) for i in range(table)]
        with ThreadPoolExecutor(threads) as ex:  # ctypes releases the GIL
            pks = list(ex.map(sk_to_pk, self.sks))
        self.table96 = np.frombuffer(b"".join(pks), np.uint8).copy()
        self.msg_ctr = 0

    def jobs(self, shapes: list[list[int]], fault_rate: float = 0.0):
        """shapes: per job, the pubkey count of every set.  Returns the
        bref_bench_jobs arrays and the expected verdict of every job (a faulted
        set signs a different message: the job resolves false)."""
        all_sets, msgs, sign_msgs = [], [], []
        job_off, pk_off, idx = [0], [0], []
        expected = []
        for shape in shapes:
            bad = False
            for k in shape:
                s = self.rng.choice(self.table, size=k, replace=False) if k > 1 else self.rng.integers(0, self.table, size=1)
                all_sets.append(s)
                idx.extend(int(v) for v in s)
                pk_off.append(len(idx))
                m = hashlib.sha256(b"bgv-cpu" + self.seed.to_bytes(8, "little") + self.msg_ctr.to_bytes(4, "little")).digest()
                self.msg_ctr += 1
                msgs.append(m)
                f = fault_rate > 0 and self.rng.random() < fault_rate
                bad |= f
                sign_msgs.append(bytes([m[0] ^ 1]) + m[1:] if f else m)
            job_off.append(len(all_sets))
            expected.append(0 if bad else 1)
        with ThreadPoolExecutor(self.threads) as ex:
            sigs = list(ex.map(lambda t: sign(sum(self.sks[int(v)] for v in t[0]) % R, t[1]), zip(all_sets, sign_msgs)))
        n = len(all_sets)
        return {"job": np.array(job_off, np.uint32), "pk": np.array(pk_off, np.uint32),
                "idx": np.array(idx, np.uint32), "msg": np.frombuffer(b"".join(msgs), np.uint8).copy(),
                "sig": np.frombuffer(b"".join(x.ljust(192, b"\0") for x in sigs), np.uint8).copy(),
                "len": np.full(n, 96, np.uint32), "n_sets": n, "n_jobs": len(shapes),
                "expected": np.array(expected, np.int32)}

    def run(self, a: dict, threads: int) -> float:
        """bref_bench_jobs: whole jobs to `threads` workers (a job is one worker
        message, multithread/index.ts:405-420), aggregation + maybeBatch
        verification in the worker; asserts the verdicts; wall seconds"""
        res = np.zeros(a["n_jobs"], np.int32)
        wall = lib().bref_bench_jobs(a["job"].ctypes.data, a["n_jobs"], a["pk"].ctypes.data, a["idx"].ctypes.data,
                                     self.table96.ctypes.data, a["msg"].ctypes.data, a["sig"].ctypes.data,
                                     a["len"].ctypes.data, threads, res.ctypes.data)
        assert (res == a["expected"]).all(), (res, a["expected"])
        return wall


C4_BLOCK = [128] * 95 + [512, 1, 1]  # 95 attestations (k=128), sync aggregate (k=512), randao + proposer


def bench_segment_sample(budget_s: float = 15.0, seed: int = 0x4C4F4445, threads: int | None = None,
                         table: int = 4096, blocks: int | None = None, fault_rate: float = 0.0,
                         work: _Workload | None = None) -> dict:
    """Time the reference pool's work on a bounded sample of the C4 workload
    (blocks of 95 x k=128 + 1 x k=512 + 2 singles, one non-batchable job per
    block, verifyBlocksSignatures.ts:30-47, one job per worker at a time) on
    `threads` host cores.  A faulted block resolves false after its one batch
    check (non-batchable jobs are not retried, worker.ts:87-94), so C5 costs
    what C4 costs.  The table is `table` keys (aggregation cost depends on k,
    not on the table size)."""
    threads = threads or min(16, os.cpu_count() or 1)
    w = work or _Workload(threads, seed, table)
    if blocks is None:  # calibrate: one block per thread, then as many as fit in the budget
        a = w.jobs([C4_BLOCK] * threads, fault_rate)
        wall = w.run(a, threads)
        extra = int(max(0, budget_s - wall) / max(wall, 1e-3)) * threads
        if extra >= threads:
            a = w.jobs([C4_BLOCK] * extra, fault_rate)
            wall = w.run(a, threads)
    else:
        a = w.jobs([C4_BLOCK] * blocks, fault_rate)
        wall = w.run(a, threads)
    n = a["n_sets"]
    return {"value": round(n / wall, 1), "unit": "sets/s", "cores": threads, "kind": "port",
            "sample": f"{n} sets = {n // 98} C4 blocks (95 x k=128, 1 x k=512, 2 singles; one job per block)"
                      + (f", {fault_rate:.0%} of the sets faulted" if fault_rate else "")
                      + f", {w.table}-key table, oracle/bls_ref.c (6x64-bit mulx/adx Montgomery) on {threads} threads, "
                        f"aggregation inside the workers; wall {wall:.2f} s",
            "per_set_core_ms": round(wall * threads / n * 1e3, 3),
            "jobs_false": int((a["expected"] == 0).sum())}


def bench_job_latency(w: _Workload, shape: list[int], reps: int = 5) -> dict:
    """p50 wall time of ONE job of the given set shape on one worker thread
    (aggregation + maybeBatch verification): the reference pool sends a job of
    <= 128 sets (or one verifyOnMainThread call) to a single thread"""
    a = w.jobs([shape])
    t = sorted(w.run(a, 1) for _ in range(reps))
    return {"p50": round(t[len(t) // 2] * 1e3, 3), "sets": len(shape), "pubkey_refs": int(sum(shape)), "threads": 1}


def bench_configs(threads: int, budget_s: float = 12.0, seed: int = 0x4C4F4445, table: int = 4096) -> dict:
    """CPU baseline for every BASELINE config with the reference pool's
    semantics (multithread/index.ts:39,405-420): one set (verifyOnMainThread,
    chain/validation/block.ts:146) and 3 / 8 / 32-set batches, C1 (128 singles, one job,
    BlsSingleThreadVerifier on one thread), C2 (64 x k=128 batchable gossip
    sets, one job on one worker), C3 (a block: 128 x k=128 + sync k=512 + 2
    singles, one job), C4 sets/s over `threads` workers, C5 = C4 with 1% of
    the sets faulted."""
    w = _Workload(threads, seed, table)
    out = {"single_set_latency_ms": bench_job_latency(w, [1], reps=9),
           # verifyMultipleSignatures of 3 / 8 / 32 sets (test/perf/bls/bls.test.ts:43-53)
           "small_batch_latency_ms": {str(k): bench_job_latency(w, [1] * k)["p50"] for k in (3, 8, 32)},
           "c1_singles_latency_ms": bench_job_latency(w, [1] * 128),
           "c2_gossip_latency_ms": bench_job_latency(w, [128] * 64),
           "c3_block_latency_ms": bench_job_latency(w, [128] * 128 + [512, 1, 1], reps=3)}
    out["c4"] = bench_segment_sample(budget_s=budget_s, threads=threads, work=w)
    out["c5_faulted"] = bench_segment_sample(budget_s=budget_s / 3, threads=threads, fault_rate=0.01, work=w)
    return out
