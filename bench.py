"""Benchmark: BLS signature sets verified per second on MI355X.

Workload (BASELINE.json configs[3], "C4"): a 32-epoch range-sync chain
segment = 1024 blocks x 98 signature sets (95 attestation aggregates of 128
pubkeys + 1 sync aggregate of 512 + randao + proposer singles) = 100,352
sets, 12.98 M pubkey references into a 1,048,576-validator index2pubkey
table resident in HBM.  One block = one verifySignatureSets call = one job
(verifyBlocksSignatures.ts:30-47; non-batchable, <= 128 sets per job).

A step = one pass of the hot path over the whole segment: every set's
signature decoded + subgroup-checked, every message hashed to G2, every
pubkey set gathered and aggregated from the table, 64-bit random scalars
drawn (device ChaCha20 keyed by getrandom) and applied, one Miller loop per
set, per-block products,
and the final exponentiation (one for the segment; per-block ones only if
it fails).  Inputs (indices, messages, signatures) are resident in HBM
before the timed region.  --inflight D batches are in flight per GPU (auto:
3, or 4 when a GPU's batch is under 32,000 sets, i.e. the strong-scaling
shards of N >= 4), one context each, as a pool with D contexts per device
runs them: the next batches' phase 1 fills the SIMDs a batch's Miller phase
leaves idle.  Multi-GPU (default, strong scaling): ONE segment split by job
over the ranks (dist.shard_jobs); each rank reduces its shard to one Fp12
Miller product, the 576-byte partials are all-gathered over RCCL and ONE
final exponentiation runs on their product, then the per-block verdicts are
all-gathered.  --weak: every rank verifies its own segment.
A second measurement times the gossip batch (BASELINE configs[1], "C2":
64 aggregate sets x 128 pubkeys, batchable, one job) for the p50 latency.

Synthetic data: keys sk_i = SHA256("bgv-sk"||LE64(seed)||LE32(i)) mod r and
signatures are generated on the device (bgv_gen_keys / bgv_gen_sign).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--blocks B]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_VALIDATORS = 1 << 20
SETS_PER_BLOCK = 98
ATT_PER_BLOCK = 95
ATT_K = 128
SYNC_K = 512
SEED = 0x4C4F4445
# batches in flight per GPU (one context each): the next batches' hash, pubkey
# and decode kernels fill the SIMDs a batch's one-wave Miller phase leaves idle
# (profiles/r06b_overlap_sizes.txt: C4 36.7 -> 34.2 / 33.1 ms per batch with
# 2 / 3 in flight, 34.0 with 4; C4/8 9.65 -> 8.35 / 7.59 ms with 3 / 4): three
# for batches of >= 32,000 sets per GPU, four below (the shards of N >= 4)
INFLIGHT = 3
INFLIGHT_SMALL = 4
INFLIGHT_SMALL_BELOW = 32000


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def build_segment(blocks: list[int], seed: int = SEED, att_per_block: int = ATT_PER_BLOCK, att_k: int = ATT_K):
    """Host arrays for the given block ids of the segment (deterministic per
    block): att_per_block attestation aggregates of att_k pubkeys, the sync
    aggregate (512) and two singles per block."""
    job_off, pk_off, idx, msgs = [0], [0], [], []
    per_block = att_per_block + SETS_PER_BLOCK - ATT_PER_BLOCK
    perm = np.random.default_rng(seed).permutation(N_VALIDATORS).astype(np.uint32)
    n = 0
    for b in blocks:
        rng = np.random.default_rng([seed, b])
        # attesters of the block: disjoint committees (a slice of a shuffling)
        start = int(rng.integers(0, N_VALIDATORS))
        att = np.take(perm, np.arange(start, start + att_per_block * att_k) % N_VALIDATORS)
        sync = rng.choice(N_VALIDATORS, size=SYNC_K, replace=False).astype(np.uint32)
        singles = rng.integers(0, N_VALIDATORS, size=2).astype(np.uint32)
        for a in range(att_per_block):
            idx.append(att[a * att_k : (a + 1) * att_k])
            pk_off.append(pk_off[-1] + att_k)
        idx.append(sync)
        pk_off.append(pk_off[-1] + SYNC_K)
        for s in singles:
            idx.append(np.array([s], np.uint32))
            pk_off.append(pk_off[-1] + 1)
        for k in range(per_block):
            msgs.append(hashlib.sha256(b"bgv-msg" + seed.to_bytes(8, "little") + (b * per_block + k).to_bytes(4, "little")).digest())
        n += per_block
        job_off.append(n)
    return {
        "n_sets": n,
        "n_jobs": len(blocks),
        "job_offsets": np.array(job_off, np.uint32),
        "pk_offsets": np.array(pk_off, np.uint32),
        "pk_indices": np.concatenate(idx).astype(np.uint32),
        "msgs": np.frombuffer(b"".join(msgs), np.uint8).reshape(n, 32).copy(),
        "n_raw": 0,
    }


def to_device(arrays: dict, torch, dev):
    out = dict(arrays)
    for k, v in arrays.items():
        if isinstance(v, np.ndarray):
            t = torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else v.view(np.int64) if v.dtype == np.uint64 else v)
            out[k] = t.to(dev)
    return out


def fpmul_counts():
    p = os.path.join(ROOT, "tools", "fpmul_counts.json")  # tools/opcount.cpp
    return json.load(open(p)) if os.path.exists(p) else None


# stage -> its main kernel (rocprofv3 name) for the PMC traffic lookup
STAGE_KERNEL = {"sig_decode_subgroup": "k_sig", "hash_to_g2": "k_hash", "pk_gather": "k_pk_chunk",
                "pk_aggregate_scale": "k_pk", "sig_scale": "k_msm_bucket", "sig_sum_tree": "k_msm_job",
                "miller_loop": "k_miller", "miller_loop_jobs": "k_miller_coop", "miller_product_tree": "k_job_fold",
                "batch_final_exp": "k_batch_final"}


def pmc_traffic(stage: str):
    """HBM-side bytes per launch of the stage's main kernel from the committed
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.json)."""
    p = os.path.join(ROOT, "tools", "pmc_traffic.json")
    if not os.path.exists(p):
        return None, None
    t = json.load(open(p))
    k = t["kernels"].get(STAGE_KERNEL.get(stage, ""), None)
    if not k:
        return None, None
    return k["fetch_bytes"] + k["write_bytes"], t["source"]


def cpu_baseline(budget_s: float = 12.0):
    """oracle C restatement (oracle/libbls_ref.so: mulx/adx Montgomery, multi-pair
    Miller loop with a shared squaring) timed on the threads this host's cgroup
    grants, on bounded samples of every config with the reference pool's
    semantics (oracle/cref.py bench_configs); None when not built."""
    try:
        from oracle import cref
    except Exception as e:  # noqa: BLE001
        log("cpu_baseline unavailable:", e)
        return None
    affinity = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    threads = min(affinity, quota) if quota else affinity
    per = cref.bench_configs(threads=threads, budget_s=budget_s, seed=SEED)
    out = dict(per["c4"])  # the metric's config (C4) at the top level
    out["per_config"] = {k: v for k, v in per.items() if k != "c4"}
    phys = physical_cores()
    out["cores_affinity"] = affinity
    out["cgroup_cpu_quota"] = quota
    out["cores_physical_machine"] = phys
    per_core = out["value"] / threads
    out["per_core_sets_per_s"] = round(per_core, 1)
    out["blst_reference_ms_per_set"] = 0.9  # "Time per sig ~0.9ms on good machines" (metrics/metrics/lodestar.ts:426-428)
    if phys and phys > threads:  # labelled extrapolation, not a measurement
        out["extrapolated_all_physical_cores_sets_per_s"] = round(per_core * phys, 1)
    return out


def cgroup_cpu_quota():
    """CPUs granted by the cgroup (cpu.max quota / period), None if unlimited"""
    for p in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(p).read().split()[:2]
            if q != "max":
                return max(1, int(-(-int(q) // int(per))))
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, -(-q // per))
    except (OSError, ValueError):
        pass
    return None


def physical_cores():
    """distinct (physical id, core id) pairs in /proc/cpuinfo"""
    try:
        seen, phys = set(), None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":")[1].strip()
            elif line.startswith("core id"):
                seen.add((phys, line.split(":")[1].strip()))
        return len(seen) or None
    except OSError:
        return None


def singles(n: int, seed: int):
    """C1: n single-pubkey sets in one job"""
    rng = np.random.default_rng(seed)
    msgs = [hashlib.sha256(b"bgv-msg-c1" + seed.to_bytes(8, "little") + i.to_bytes(4, "little")).digest() for i in range(n)]
    return {"n_sets": n, "n_jobs": 1, "job_offsets": np.array([0, n], np.uint32),
            "pk_offsets": np.arange(n + 1, dtype=np.uint32),
            "pk_indices": rng.integers(0, N_VALIDATORS, size=n).astype(np.uint32),
            "msgs": np.frombuffer(b"".join(msgs), np.uint8).reshape(n, 32).copy(), "n_raw": 0}


def golden_fault_sigs():
    """96-byte signatures the oracle rejects, from the committed golden vectors
    (tests/golden/batch_vectors.json, generated by tools/gen_golden.py):
    on-curve-not-in-G2 (BLST_POINT_NOT_IN_GROUP)."""
    v = json.load(open(os.path.join(ROOT, "tests", "golden", "batch_vectors.json")))
    for j in v["jobs"]:
        for st in j["sets"]:
            if st.get("code") == 3 and len(st["sig"]) == 192:
                return bytes.fromhex(st["sig"])
    raise RuntimeError("no not-in-G2 vector in the golden file")


def inject_faults(d, arrays: dict, rate: float, seed: int, with_codes: bool = False):
    """C5: `rate` of the sets faulted, a quarter each of wrong-message
    signature (-> false), swapped pubkey index (-> false), cleared compression flag
    (-> reject BLST_BAD_ENCODING) and an on-curve point outside G2 (-> reject
    BLST_POINT_NOT_IN_GROUP).  Returns (arrays with sigs, expected per-job results)
    and, with_codes, the expected per-set codes."""
    n, nj = arrays["n_sets"], arrays["n_jobs"]
    rng = np.random.default_rng(seed)
    pick = np.sort(rng.choice(n, size=max(4, int(n * rate)), replace=False))
    kind = rng.permutation(np.arange(len(pick)) % 4)
    sign_msgs = arrays["msgs"].copy()
    sign_msgs[pick[kind == 0], 0] ^= 1
    sigs = np.zeros((n, 192), np.uint8)
    d.gen_sign(dict(arrays, msgs=sign_msgs), sigs)
    out = dict(arrays, pk_indices=arrays["pk_indices"].copy())
    for i in pick[kind == 1]:
        o = int(arrays["pk_offsets"][i])
        out["pk_indices"][o] = (int(out["pk_indices"][o]) + 1) % N_VALIDATORS
    sigs[pick[kind == 2], 0] &= 0x7F
    bad_g2 = np.frombuffer(golden_fault_sigs(), np.uint8)
    sigs[pick[kind == 3], :96] = bad_g2
    out["sigs"] = sigs
    out["sig_len"] = np.full(n, 96, np.uint32)
    code = np.zeros(n, np.int32)
    code[pick[kind == 2]] = 1
    code[pick[kind == 3]] = 3
    false_set = np.zeros(n, bool)
    false_set[pick[(kind == 0) | (kind == 1)]] = True
    expect = []
    jo = arrays["job_offsets"]
    for j in range(nj):
        c = code[jo[j]:jo[j + 1]]
        nz = np.nonzero(c)[0]
        expect.append(-int(c[nz[0]]) if len(nz) else (0 if false_set[jo[j]:jo[j + 1]].any() else 1))
    if with_codes:
        return out, np.array(expect, np.int32), code
    return out, np.array(expect, np.int32)


def p50_latency(d, arrays: dict, reps: int = 7, on_device: bool = False):
    lat = []
    for _ in range(reps):
        t1 = time.perf_counter()
        jr, _ = d.verify(arrays, on_device=on_device, want_set_codes=False)
        lat.append((time.perf_counter() - t1) * 1e3)
        assert (jr == 1).all()
    return round(float(np.median(lat[1:])), 3)


def signed(d, arrays: dict) -> dict:
    s = np.zeros((arrays["n_sets"], 192), np.uint8)
    d.gen_sign(arrays, s)
    return dict(arrays, sigs=s, sig_len=np.full(arrays["n_sets"], 96, np.uint32))


def small_configs(d, torch, dev, arrays):
    """C1, C2, C3, single-set and C5 legs (rank 0): host -> device -> verdict"""
    out = {}
    g = build_segment([0], seed=SEED + 1000)
    n2, k2 = 64, ATT_K
    c2a = signed(d, {"n_sets": n2, "n_jobs": 1, "job_offsets": np.array([0, n2], np.uint32),
                     "pk_offsets": (np.arange(n2 + 1) * k2).astype(np.uint32),
                     "pk_indices": g["pk_indices"][: n2 * k2].copy(), "msgs": g["msgs"][:n2].copy(), "n_raw": 0})
    out["c2_gossip_latency_ms"] = {"p50": p50_latency(d, c2a), "sets": n2, "pubkeys_per_set": k2}
    # C3: one block = 128 attestation aggregates (k=128) + sync (k=512) + 2 singles, one job
    c3a = signed(d, build_segment([0], seed=SEED + 2000, att_per_block=128))
    out["c3_block_latency_ms"] = {"p50": p50_latency(d, c3a), "sets": c3a["n_sets"], "pubkey_refs": int(c3a["pk_offsets"][-1])}
    # C3 at 1M validators: attestations carry ~90% of a 488-member committee (k = 440)
    c3b = signed(d, build_segment([0], seed=SEED + 2500, att_per_block=128, att_k=440))
    out["c3_block_k440_latency_ms"] = {"p50": p50_latency(d, c3b), "sets": c3b["n_sets"], "pubkey_refs": int(c3b["pk_offsets"][-1])}
    # C1: 128 single sets, one job
    out["c1_singles_latency_ms"] = {"p50": p50_latency(d, signed(d, singles(128, SEED + 3000))), "sets": 128}
    # one set (verifyOnMainThread gossip block proposer, chain/validation/block.ts:146)
    out["single_set_latency_ms"] = {"p50": p50_latency(d, signed(d, singles(1, SEED + 3500))), "sets": 1}
    # verifyMultipleSignatures of 3 / 8 / 32 single sets (test/perf/bls/bls.test.ts:43-53)
    out["small_batch_latency_ms"] = {str(k): p50_latency(d, signed(d, singles(k, SEED + 3600 + k))) for k in (3, 8, 32)}
    # C5: the C4 segment with 1% faults; the batch check fails, so every block takes
    # the per-job final exponentiation (worker retry, multithread/worker.ts:74-85)
    c5a, c5_expect = inject_faults(d, arrays, 0.01, SEED + 4000)
    c5d = to_device(c5a, torch, dev)
    c5d["scalars"] = None
    jr5, _ = d.verify(c5d, on_device=True, want_set_codes=False)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    reps5, ok5 = 3, bool((jr5.astype(np.int32) == c5_expect).all())
    for _ in range(reps5):
        jr5, _ = d.verify(c5d, on_device=True, want_set_codes=False)
        ok5 &= bool((jr5.astype(np.int32) == c5_expect).all())
    torch.cuda.synchronize()
    t5 = (time.perf_counter() - t1) / reps5
    out["c5_faulted_c4"] = {"sets_per_s": round(c5a["n_sets"] / t5, 1), "ms_per_step": round(t5 * 1e3, 3), "fault_rate": 0.01,
                            "faulted_sets": int(max(4, int(c5a["n_sets"] * 0.01))), "jobs_true": int((c5_expect == 1).sum()),
                            "jobs_false": int((c5_expect == 0).sum()), "jobs_rejected": int((c5_expect < 0).sum()),
                            "verdicts_match_expected": ok5, "batch_retries": int(d.last_stats.batch_retries)}
    return out


def mixed_sizes(d, darr, reps: int = 4):
    """A node alternating gossip batches with range-sync segments:
    C2 (64 sets, host-resident, no fixed-argument lines) then the device-resident
    C4 segment (lines), `reps` times.  The line buffer stays allocated across the
    small batches (bgv_api.hip LINES_KEEP), so the C4 calls of the mixed
    sequence take what the plain ones do."""
    g = build_segment([0], seed=SEED + 1000)
    n2, k2 = 64, ATT_K
    c2a = signed(d, {"n_sets": n2, "n_jobs": 1, "job_offsets": np.array([0, n2], np.uint32),
                     "pk_offsets": (np.arange(n2 + 1) * k2).astype(np.uint32),
                     "pk_indices": g["pk_indices"][: n2 * k2].copy(), "msgs": g["msgs"][:n2].copy(), "n_raw": 0})
    c2_ms, c4_ms = [], []
    for _ in range(reps):
        t1 = time.perf_counter()
        jr, _ = d.verify(c2a, want_set_codes=False)
        c2_ms.append((time.perf_counter() - t1) * 1e3)
        assert (jr == 1).all()
        t1 = time.perf_counter()
        jr, _ = d.verify(darr, on_device=True, want_set_codes=False)
        c4_ms.append((time.perf_counter() - t1) * 1e3)
        assert (jr == 1).all()
    return {"c2_ms_p50": round(float(np.median(c2_ms)), 3), "c4_ms_p50": round(float(np.median(c4_ms)), 3),
            "reps": reps, "note": "C2 and C4 batches alternated on one context"}


def epoch_slice(d, torch, dev, arrays_host: dict, sigs, blocks: int = 32, reps: int = 7, ds=None):
    """One epoch of the segment (32 blocks = 3,136 sets): the batch a range
    sync hands the verifier per epoch (sync/constants.ts:41), on device, p50;
    with `ds`, also the pace of a stream of such batches with len(ds) in flight
    (the pool's contexts per device)"""
    from concurrent.futures import ThreadPoolExecutor

    from lodestar_amd.dist import run_in_flight, select_jobs
    sub = select_jobs(dict(arrays_host, sigs=sigs), list(range(blocks)))
    da = to_device(sub, torch, dev)
    da.update(sig_len=torch.full((sub["n_sets"],), 96, dtype=torch.int32, device=dev), scalars=None)
    p50 = p50_latency(d, da, reps=reps, on_device=True)
    out = {"sets": int(sub["n_sets"]), "blocks": blocks, "p50_ms": p50, "sets_per_s": round(sub["n_sets"] / p50 * 1e3, 1),
           "layout": d.last_stats.layout()}
    if ds and len(ds) > 1:
        ex = ThreadPoolExecutor(max_workers=len(ds))

        def submit(k):
            return ex.submit(ds[k % len(ds)].verify, da, on_device=True, want_set_codes=False)

        def finish(k, res):
            return bool((res[0] == 1).all())

        n = 8 * len(ds)
        assert run_in_flight(submit, finish, len(ds), len(ds))
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        assert run_in_flight(submit, finish, n, len(ds))
        ms = (time.perf_counter() - t1) / n * 1e3
        ex.shutdown()
        out.update(ms_per_batch_in_flight=round(ms, 3), inflight=len(ds),
                   sets_per_s_in_flight=round(sub["n_sets"] / ms * 1e3, 1))
    return out


def host_resident_c4(d, arrays_host: dict, reps: int = 3, ds=None):
    """C4 with every input in host memory: the pinned staging copy and the
    PCIe transfer are inside the timed region (the path a Node caller takes);
    with `ds`, also len(ds) such batches in flight (the Node pool's contexts
    per device: each stages and copies its own batch)"""
    d.verify(arrays_host, want_set_codes=False)
    t = []
    for _ in range(reps):
        t1 = time.perf_counter()
        jr, _ = d.verify(arrays_host, want_set_codes=False)
        t.append(time.perf_counter() - t1)
        assert (jr == 1).all()
    ms = float(np.median(t)) * 1e3
    out = {"ms_per_step": round(ms, 3), "sets_per_s": round(arrays_host["n_sets"] / ms * 1e3, 1),
           "h2d_bytes": int(arrays_host["n_sets"] * (32 + 192 + 4) + arrays_host["pk_indices"].nbytes
                            + arrays_host["pk_offsets"].nbytes + arrays_host["job_offsets"].nbytes)}
    if ds and len(ds) > 1:
        from concurrent.futures import ThreadPoolExecutor

        from lodestar_amd.dist import run_in_flight
        ex = ThreadPoolExecutor(max_workers=len(ds))

        def submit(k):
            return ex.submit(ds[k % len(ds)].verify, arrays_host, want_set_codes=False)

        def finish(k, res):
            return bool((res[0] == 1).all())

        n = 3 * len(ds)
        assert run_in_flight(submit, finish, len(ds), len(ds))
        t1 = time.perf_counter()
        assert run_in_flight(submit, finish, n, len(ds))
        mi = (time.perf_counter() - t1) / n * 1e3
        ex.shutdown()
        out.update(ms_per_batch_in_flight=round(mi, 3), inflight=len(ds),
                   sets_per_s_in_flight=round(arrays_host["n_sets"] / mi * 1e3, 1))
    return out


def shard_projection(d, torch, dev, arrays_host: dict, ds=None, worlds=(2, 4, 8), reps: int = 5):
    """Strong sharding of ONE C4 segment measured on one GPU: each rank's
    shard (dist.shard_jobs) through bgv_partial, plus the node's combination of
    `world` partials (bgv_combine_final).  ms = median partial + combine; the
    RCCL all-gather of 576 B per rank is not included (latency-bound, ~tens of
    us over xGMI).  projected_sets_per_s = 100,352 / ms.  With `ds` (the
    contexts of the batches in flight), ms_in_flight = the shard's time per
    segment with len(ds) segments in flight (dist.run_in_flight: partials on
    worker threads, combinations in order on this thread), the per-GPU pace of
    a node verifying a stream of segments (an N-rank run of this bench takes
    shards under INFLIGHT_SMALL_BELOW sets INFLIGHT_SMALL deep)."""
    from concurrent.futures import ThreadPoolExecutor

    from lodestar_amd.dist import batch_job_work, run_in_flight, select_jobs, shard_balance, shard_jobs
    work = batch_job_work(arrays_host)
    out = {}
    ex = ThreadPoolExecutor(max_workers=len(ds)) if ds and len(ds) > 1 else None
    for world in worlds:
        shards = shard_jobs(work, world)
        # the heaviest shard sets the node's time
        ids = max(shards, key=lambda s: sum(work[j] for j in s))
        sub = to_device(select_jobs(arrays_host, ids), torch, dev)
        sub["scalars"] = None
        part, _, jr, ok = d.partial(sub, on_device=True)
        assert ok
        t = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            part, _, jr, ok = d.partial(sub, on_device=True)
            valid = d.combine_final([part] * world)
            t.append(time.perf_counter() - t1)
        ms = float(np.median(t)) * 1e3
        e = {"sets_per_rank": int(sub["n_sets"]), "ms": round(ms, 3),
             "work_max_over_mean": round(shard_balance(work, shards), 4),
             "projected_sets_per_s": round(arrays_host["n_sets"] / ms * 1e3, 1)}
        if ex is not None:
            dd = ds

            def submit(k):
                return ex.submit(dd[k % len(dd)].partial, sub, on_device=True)

            def finish(k, res):
                return dd[k % len(dd)].combine_final([res[0]] * world) and res[3]

            n = 4 * len(dd)
            assert run_in_flight(submit, finish, len(dd), len(dd))
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            assert run_in_flight(submit, finish, n, len(dd))
            mi = (time.perf_counter() - t1) / n * 1e3
            e.update(ms_in_flight=round(mi, 3), inflight=len(dd),
                     projected_sets_per_s_in_flight=round(arrays_host["n_sets"] / mi * 1e3, 1))
        out[f"c4_over_{world}"] = e
    if ex is not None:
        ex.shutdown()
    return out


def reserved_device(d, gpu, torch, dev, darr, arrays_host: dict, reps: int = 5):
    """The bulk pace of a device whose bulk context leaves 32 CUs to a
    verifyOnMainThread priority context (bgv_cfg.cu_split = -32; the pools'
    device 0 on a multi-device node, and on one device when asked): C4 and the
    heaviest C4/8 shard (bgv_partial) on a reserved context against the same
    batches on the unreserved one, medians of `reps`.  cap_at_shard is the
    RESERVED_CAP the shard weighting should use (lodestar_amd/napi/reserved_cap.json)."""
    from lodestar_amd import native
    from lodestar_amd.dist import RESERVED_CAP, batch_job_work, select_jobs, shard_jobs
    work = batch_job_work(arrays_host)
    ids = max(shard_jobs(work, 8), key=lambda s: sum(work[j] for j in s))
    sub = to_device(select_jobs(arrays_host, ids), torch, dev)
    sub["scalars"] = None

    def med(ctx):
        c4, sh = [], []
        for k in range(reps + 1):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            jr, _ = ctx.verify(darr, on_device=True, want_set_codes=False)
            t2 = time.perf_counter()
            _, _, _, ok = ctx.partial(sub, on_device=True)
            t3 = time.perf_counter()
            assert (jr == 1).all() and ok
            if k:
                c4.append((t2 - t1) * 1e3)
                sh.append((t3 - t2) * 1e3)
        return float(np.median(c4)), float(np.median(sh))

    dr = native.Device(gpu, cu_split=-32)
    try:
        dr.gen_keys(0, N_VALIDATORS, SEED)
        free_c4, free_sh = med(d)
        res_c4, res_sh = med(dr)
    finally:
        dr.close()
    return {"cu_split": -32, "c4_ms": round(res_c4, 3), "c4_unreserved_ms": round(free_c4, 3),
            "c4_over_8_ms": round(res_sh, 3), "c4_over_8_unreserved_ms": round(free_sh, 3),
            "sets_per_s": round(arrays_host["n_sets"] / res_c4 * 1e3, 1),
            "cap_at_c4": round(free_c4 / res_c4, 4), "cap_at_shard": round(free_sh / res_sh, 4),
            "reserved_cap_in_use": RESERVED_CAP,
            "note": "pool default: reserved only with >= 2 devices (device 0); a one-device pool reserves nothing unless priorityCus asks"}


def one_in_flight(d, darr, torch, reps: int = 5):
    """C4 verified back to back on one context: ms per batch (median) and the
    per-stage HIP-event times of those batches (the isolated kernel durations)"""
    from lodestar_amd import native
    t, st = [], np.zeros(native.N_STAGES)
    for k in range(reps + 1):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        jr, _ = d.verify(darr, on_device=True, want_set_codes=False)
        assert (jr == 1).all()
        if k:
            t.append((time.perf_counter() - t1) * 1e3)
            st += np.array(list(d.last_stats.stage_ms))
    ms = float(np.median(t))
    stage = {d.stage_name(i): float(st[i] / reps) for i in range(native.N_STAGES) if d.stage_name(i) != "unknown"}
    return {"ms_p50": round(ms, 3), "sets_per_s": round(darr["n_sets"] / ms * 1e3, 1), "reps": reps}, stage


def weak_leg(ds, torch, dev, dist, coll_dev, rank, world, args):
    """N > 1 extra: every rank verifies its OWN whole segment (seeded per rank),
    one 576-B partial per rank all-gathered, ONE final exponentiation; the
    node's sets/s over all ranks (weak scaling, not BASELINE configs[3]),
    len(ds) segments in flight per GPU like the main measurement."""
    from concurrent.futures import ThreadPoolExecutor

    from lodestar_amd.dist import combine_sharded, run_in_flight
    seg = build_segment(list(range(args.blocks)), seed=SEED + 7919 * (rank + 1))
    da = to_device(seg, torch, dev)
    sigs = torch.zeros((seg["n_sets"], 192), dtype=torch.uint8, device=dev)
    ds[0].gen_sign(da, sigs, on_device=True)
    da.update(sigs=sigs, sig_len=torch.full((seg["n_sets"],), 96, dtype=torch.int32, device=dev), scalars=None)
    ex = ThreadPoolExecutor(max_workers=len(ds))

    def submit(k):
        return ex.submit(ds[k % len(ds)].partial, da, on_device=True)

    def finish(k, res):
        valid, jr = combine_sharded(ds[k % len(ds)], res, dist, device=coll_dev)
        return valid and bool((jr == 1).all())

    assert run_in_flight(submit, finish, len(ds) + max(args.warmup, 1), len(ds)), "weak-leg warm-up did not verify"
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ok = run_in_flight(submit, finish, args.steps, len(ds))
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=coll_dev if coll_dev is not None else "cpu", dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ex.shutdown()
    return {"sets_per_s": round(seg["n_sets"] * world * args.steps / elapsed, 1), "sets_per_rank": seg["n_sets"],
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "verified": ok, "inflight": len(ds),
            "note": "every rank its own 32-epoch segment; one partial per rank all-gathered, one final exponentiation"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--blocks", type=int, default=1024, help="blocks in the segment (1024 = 32 epochs)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-c2", action="store_true", help="skip the C1/C2/C3/C5, host-resident and shard legs (profiling runs)")
    ap.add_argument("--weak", action="store_true",
                    help="N > 1: every rank verifies its own segment (default: ONE segment split across the ranks, BASELINE configs[3])")
    ap.add_argument("--no-weak-leg", action="store_true", help="N > 1: skip the extra weak-scaling measurement")
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches in flight per GPU: contexts on the GPU, one worker thread each (dist.run_in_flight); "
                         "0 = auto (3, or 4 for batches under 32,000 sets per GPU)")
    ap.add_argument("--input-sync", choices=("once", "per-call"), default="once",
                    help="device inputs of the timed steps: synchronised once before them (default), or torch's "
                         "stream waited for on every call")
    ap.add_argument("--cfg", action="append", default=[], metavar="KEY=VAL",
                    help="bgv_cfg override for every context (A/B runs only, e.g. pairs=4)")
    args = ap.parse_args()
    assert args.inflight >= 0
    cfg = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in args.cfg}

    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BGV_BENCH_REHEARSE=1: every rank on GPU 0 with gloo collectives, to
    # rehearse the N > 1 path on a one-GPU box (RCCL refuses two ranks on one
    # device); the driver's multi-GPU runs never set it
    rehearse = os.environ.get("BGV_BENCH_REHEARSE") == "1"
    gpu = 0 if rehearse else local
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811

        torch.cuda.set_device(gpu)
        dist.init_process_group("gloo" if rehearse else "nccl")
    dev = torch.device("cuda", gpu)
    coll_dev = None if rehearse else dev  # where the collectives' tensors live

    shard = world > 1 and not args.weak
    from lodestar_amd import native
    from lodestar_amd.dist import batch_job_work, gather_job_results, select_jobs, shard_jobs, verify_sharded

    # per-stage timing events are automatic from 65,536 sets; below that they
    # add ~5 us of queue time per event on the critical path (C4/8 shard 9.65 ->
    # 9.75 ms, profiles/r04g_sweep_timed.txt), so the timed steps of N > 1 run
    # without them and one extra step on a timed context gives the breakdown
    d = native.Device(gpu, **cfg)
    t0 = time.time()
    d.gen_keys(0, N_VALIDATORS, SEED)
    log(f"[bench] {N_VALIDATORS} keys generated in {time.time() - t0:.1f}s")
    # the other contexts of the batches in flight: each holds its own table
    # replica (as every context of the pools does) and its own streams
    if not args.inflight:
        per_gpu = args.blocks * SETS_PER_BLOCK // (world if (world > 1 and not args.weak) else 1)
        args.inflight = INFLIGHT_SMALL if per_gpu < INFLIGHT_SMALL_BELOW else INFLIGHT
    ds = [d]
    for _ in range(args.inflight - 1):
        x = native.Device(gpu, **cfg)
        x.gen_keys(0, N_VALIDATORS, SEED)
        ds.append(x)

    seg = build_segment(list(range(args.blocks)), seed=SEED + (0 if shard else rank))
    jo = seg["job_offsets"]
    shards = shard_jobs(batch_job_work(seg), world) if shard else None
    arrays = select_jobs(seg, shards[rank]) if shard else seg
    darr = to_device(arrays, torch, dev)
    n_sets = arrays["n_sets"]
    sigs = torch.zeros((n_sets, 192), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t0 = time.time()
    d.gen_sign(darr, sigs, on_device=True)
    darr["sigs"] = sigs
    darr["sig_len"] = torch.full((n_sets,), 96, dtype=torch.int32, device=dev)
    darr["scalars"] = None  # drawn by the library per call (device ChaCha20 keyed by getrandom)
    log(f"[bench] rank {rank}: {n_sets} sets signed in {time.time() - t0:.1f}s")

    # a step = one batch: bgv_verify (N = 1) or this rank's shard through
    # bgv_partial, then (in step order, on this thread) the all-gather of the
    # partials, the combined final check and the per-block verdicts.  Steps
    # go round-robin to the contexts, args.inflight of them outstanding; the
    # batches read the same device-resident inputs (read-only) and draw their
    # own scalars
    from concurrent.futures import ThreadPoolExecutor

    from lodestar_amd.dist import combine_sharded, run_in_flight
    ex = ThreadPoolExecutor(max_workers=args.inflight)
    stage_sum = np.zeros(native.N_STAGES)
    t_sub, lat = {}, []

    # the inputs are written once above and only read by the steps: one
    # synchronisation here instead of a wait for torch's stream on every call
    # (--input-sync per-call restores it)
    torch.cuda.synchronize()
    per_call = args.input_sync == "per-call"

    def submit(k):
        c = ds[k % len(ds)]
        t_sub[k] = time.perf_counter()
        if world == 1:
            return ex.submit(c.verify, darr, on_device=True, want_set_codes=False, sync_inputs=per_call)
        return ex.submit(c.partial, darr, on_device=True, sync_inputs=per_call)

    def finish(k, res):
        c = ds[k % len(ds)]
        if world == 1:
            ok = bool((res[0] == 1).all())
        else:
            valid, local_jr = combine_sharded(c, res, dist, device=coll_dev)
            if shard:  # every rank ends with the whole segment's per-block verdicts
                full = gather_job_results(local_jr, shards, seg["n_jobs"], dist, device=coll_dev)
                ok = valid and bool((full == 1).all())
            else:
                ok = valid and bool((local_jr == 1).all())
        lat.append((time.perf_counter() - t_sub.pop(k)) * 1e3)
        stage_sum[:] += np.array(list(c.last_stats.stage_ms))
        return ok

    # every context verifies one batch first (its buffers sized), then W warm-up steps
    assert run_in_flight(submit, finish, len(ds), len(ds)), "context priming batch did not verify"
    assert run_in_flight(submit, finish, args.warmup, len(ds)), "warm-up batch did not verify"
    stage_sum[:] = 0
    lat.clear()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    all_ok = run_in_flight(submit, finish, args.steps, len(ds))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    step_ms = list(lat)
    if dist:
        t = torch.tensor([elapsed], device=coll_dev if coll_dev is not None else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        okt = torch.tensor([1 if all_ok else 0], device=coll_dev if coll_dev is not None else "cpu")
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        all_ok = bool(okt.item())
    total_sets = seg["n_sets"] * (1 if shard else world)
    ms_per_step = elapsed / args.steps * 1e3
    value = total_sets * args.steps / elapsed

    timed_layout = d.last_stats.layout()  # the variant the timed batches ran with (bgv_stats), before the extra legs
    if not stage_sum.any():  # untimed shard steps: one step of the same shard on a timed context, after the timed region
        dt = native.Device(gpu, timing=1)
        dt.gen_keys(0, N_VALIDATORS, SEED)
        dt.partial(darr, on_device=True)
        stage_sum = np.array(list(dt.last_stats.stage_ms)) * args.steps
        dt.close()
    stage_ms = {d.stage_name(i): float(stage_sum[i] / args.steps) for i in range(native.N_STAGES) if d.stage_name(i) != "unknown"}

    legs = {}
    iso_stage_ms = None
    if rank == 0 and world == 1:
        # the same batch with ONE in flight (the r01-r05 step): its latency and
        # the kernels' durations without other batches beside them
        legs["one_in_flight"], iso_stage_ms = one_in_flight(d, darr, torch)
    if shard and not args.no_weak_leg:
        legs["weak_scaling"] = weak_leg(ds, torch, dev, dist, coll_dev, rank, world, args)
    if rank == 0 and world == 1 and not args.no_c2:
        legs.update(small_configs(d, torch, dev, arrays))
        host = dict(arrays)
        host["sigs"] = sigs.cpu().numpy()
        host["sig_len"] = np.full(n_sets, 96, np.uint32)
        host["scalars"] = None
        legs["c4_host_resident"] = host_resident_c4(d, host, ds=ds)
        # (the legs below run len(ds) deep; an N-rank run takes its shards
        # INFLIGHT_SMALL deep, profiles/r06o_depth_streams/: a fourth context
        # here, open beside the reserved leg's CU-masked queues, coincided with
        # queue scratch failures there)
        legs["c4_epoch_slice"] = epoch_slice(d, torch, dev, arrays, host["sigs"], ds=ds)
        legs["mixed_sizes"] = mixed_sizes(d, darr)
        if world == 1:
            legs["strong_shard_projection"] = shard_projection(d, torch, dev, host, ds)

    # roofline (INT32 VALU): algorithmic Fp-mul per set x sets / the stage's
    # HIP-event time in the timed steps, for every stage; the dominant kernel
    # is the stage with the largest time (stages overlap on three streams)
    roof = None
    counts = fpmul_counts()
    if rank == 0:
        mad_ms = d.bench_mad(256 * 256 * 8, 4096)
        mad_rate = 256 * 256 * 8 * 4096 * 8 / (mad_ms * 1e-3)  # lane-ops/s
        peak_fpmul = mad_rate / 288.0 / 1e9
        fpm_ms = d.bench_fpmul(256 * 256 * 8, 2048)
        fpm_rate = 256 * 256 * 8 * 2048 / (fpm_ms * 1e-3) / 1e9
        per_stage = {}
        stage_counts = dict(counts["per_set"]) if counts else {}
        lay = timed_layout
        if counts and lay["lines"] and "per_set_lines" in counts:
            stage_counts["miller_loop"] = counts["per_set_lines"]["miller_loop"]
        if counts and lay["lines"] and lay["pairs_per_item"] == 4 and "per_set_lines4" in counts:
            stage_counts["miller_loop"] = counts["per_set_lines4"]["miller_loop"]
            stage_counts["miller_product_tree"] = counts["per_set_lines4"]["miller_product_tree"]
        share = (n_sets - min(lay["defer_from"], n_sets)) / max(n_sets, 1)
        check_c = None
        if counts and "g2_decompress_only" in counts:
            check_c = counts["per_set"]["sig_decode_subgroup"] - counts["g2_decompress_only"]
            stage_counts["sig_decode_subgroup"] = counts["g2_decompress_only"] + (1.0 - share) * check_c
        for k, ms in stage_ms.items():
            if ms <= 0:
                continue
            e = {"ms": round(ms, 3), "share_of_step": round(ms / ms_per_step, 3)}
            if k in stage_counts:
                ach = stage_counts[k] * n_sets / (ms * 1e-3) / 1e9
                e.update(fpmul_per_set=stage_counts[k], achieved_G_fpmul_per_s=round(ach, 3),
                         frac=round(ach / peak_fpmul, 4))
            per_stage[k] = e
        pk_refs = int(arrays["pk_offsets"][-1])
        gather = None
        if stage_ms.get("pk_gather", 0) > 0:
            gb = pk_refs * (96 + 4) / (stage_ms["pk_gather"] * 1e-3) / 1e9
            gather = {"kernel": "k_pk_chunk", "algorithmic_bytes": pk_refs * (96 + 4), "ms": round(stage_ms["pk_gather"], 3),
                      "GB_per_s": round(gb, 1), "hbm_peak_GB_per_s": 8000, "frac_hbm": round(gb / 8000, 4),
                      "note": "96-B table row + 4-B index per pubkey reference; compute-bound (one G1 mixed addition per row)"}
        step_total = None
        if counts:
            step_total = counts["per_set_total"]
            if lay["lines"] and lay["pairs_per_item"] == 4 and "per_set_total_lines4" in counts:
                step_total = counts["per_set_total_lines4"]
        dom = max(stage_ms, key=stage_ms.get)
        e = per_stage.get(dom, {})
        iso = None
        if iso_stage_ms and dom in stage_counts and iso_stage_ms.get(dom, 0) > 0:
            ach_i = stage_counts[dom] * n_sets / (iso_stage_ms[dom] * 1e-3) / 1e9
            iso = {"kernel_ms": round(iso_stage_ms[dom], 3), "achieved": round(ach_i, 3), "frac": round(ach_i / peak_fpmul, 4),
                   "stage_ms": {k: round(v, 3) for k, v in iso_stage_ms.items() if v > 0},
                   "note": "the same kernel with ONE batch in flight (one_in_flight leg): no other batch shares the chip"}
        traffic, tsrc = pmc_traffic(dom)
        roof = {"bound": "valu-int32", "kernel": dom, "kernel_name": STAGE_KERNEL.get(dom),
                "achieved": e.get("achieved_G_fpmul_per_s"), "peak": round(peak_fpmul, 3), "unit": "G Fp-mul/s",
                "frac": e.get("frac"), "traffic": traffic,
                "traffic_unit": "bytes per launch (FETCH_SIZE + WRITE_SIZE, raw)", "traffic_source": tsrc,
                "per_set_fpmul": e.get("fpmul_per_set"), "sets_per_launch": n_sets, "kernel_ms": e.get("ms"),
                "peak_def": "measured v_mad_u64_u32 lane-ops/s / 288 (12x32-bit CIOS product count)",
                "mad_u64_lane_ops_per_s": mad_rate, "peak_fpmul28_G_per_s": round(mad_rate / 393 / 1e9, 3),
                "fpmul_microbench_G_per_s": round(fpm_rate, 3),
                "per_stage": per_stage, "pubkey_gather": gather, "isolated": iso,
                "timing_note": ("kernel_ms: the stage's HIP-event time inside the timed region, where %d batches are in flight "
                                "and share the chip" % args.inflight),
                "miller_lines": ({"active": True, "kernel_name": "k_lines", "fpmul_per_set": counts["per_set_lines"]["miller_lines"],
                                  "note": "untimed step on the hash stream between hash_to_g2 and miller_loop"}
                                 if counts and lay["lines"] and "per_set_lines" in counts else {"active": False}),
                "pipeline_variant": lay,
                "deferred_subgroup_checks": {"share_of_sets": share, "kernel_name": "k_sig_split",
                                             "fpmul_per_set": round(share * check_c, 1) if check_c is not None else None,
                                             "note": "untimed: beside the Miller loops, before the fold"},
                "step_fpmul_per_set": step_total,
                "step_fpmul_G_per_s": round(step_total * n_sets / (ms_per_step * 1e-3) / 1e9, 3) if counts else None}

    # the reserved-device leg runs last, after every other GPU measurement: its
    # CU-masked streams each take a hardware queue of its own, and on some boxes
    # a queue's scratch allocation failed there (HSA_STATUS_ERROR_OUT_OF_RESOURCES
    # with the other contexts' queues holding theirs), so a failure is recorded
    # in the leg instead of ending the run
    if rank == 0 and world == 1 and not args.no_c2:
        for c in ds[1:]:
            c.close()
        try:
            legs["reserved_device"] = reserved_device(d, gpu, torch, dev, darr, host)
        except Exception as e:  # noqa: BLE001
            legs["reserved_device"] = {"error": f"{type(e).__name__}: {e}"[:400]}

    if rank == 0:
        cpu = None if (args.no_cpu or world > 1) else cpu_baseline()
        par = (f"one segment sharded by job over {world} GPUs (shard_jobs), RCCL all-gather of Miller partials + per-job verdicts"
               if shard else f"one segment per GPU x{world}, RCCL all-gather of Miller partials")
        par += f"; {args.inflight} batches in flight per GPU (contexts, dist.run_in_flight)"
        out = {
            "metric": "BLS signature sets verified/sec (node)",
            "value": round(value, 1),
            "unit": "sets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (device-generated keys/signatures, seeded)",
            "config": {"workload": "C4 range-sync segment: 32 epochs = %d blocks x 98 sets (95 att k=128, sync k=512, 2 singles), 1M-validator table in HBM" % args.blocks,
                       "sets": total_sets, "pubkey_refs": int(args.blocks * (ATT_PER_BLOCK * ATT_K + SYNC_K + 2)) * (1 if shard else world),
                       "table_validators": N_VALIDATORS, "jobs": args.blocks * (1 if shard else world), "parallelism": par,
                       "inflight": args.inflight, **({"cfg_overrides": cfg} if cfg else {})},
            "c4_step_ms_p50": round(float(np.median(step_ms)), 3),
            "c4_step_ms_note": "submit -> verdict of one batch with the others in flight; one_in_flight has the lone batch",
            **legs,
            "verified": all_ok,
            "stage_ms": {k: round(v, 3) for k, v in stage_ms.items()},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    ex.shutdown()
    for c in ds:
        c.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
