"""Multi-GPU glue for the batch verifier.

Signature sets shard by job across ranks (one process per GPU; a job is
never split: its verdict is the AND of its sets).  Every rank reduces its
shard to one Fp12 Miller product (576 B, bgv_partial); the partials are
all-gathered (RCCL over xGMI on the GPU node, gloo in the CPU tests) and
multiplied before ONE final exponentiation (bgv_combine_final).  At 576 B
per rank the exchange is latency-bound, so a single all-gather is the whole
collective on the success path.

Failure path (SURVEY §8e "Failure"; the reference always resolves per job,
multithread/index.ts:356-372, and verifyBlocksSignatures names the first bad
block, verifyBlocksSignatures.ts:56-59): when the combined check fails, each
rank runs the final exponentiation of its OWN shard on the intermediates
bgv_partial left on the device and, only if that fails too, one per job
(bgv_partial_finish, the worker's per-job retry).  The per-job int32
verdicts are then all-gathered so every rank holds the whole batch's.
"""
from __future__ import annotations

import json
import os

import numpy as np

PARTIAL_BYTES = 576


# Work model for balancing shards (SURVEY 8e "balancing by sum W(k)"): the
# device cost of a set in Montgomery Fp products, from the instrumented host
# build of the kernels' headers (tools/opcount.cpp -> tools/fpmul_counts.json):
# every set pays its signature decode + checks, hash_to_G2, [r]PK, its Miller
# loop and its share of the signature sum and folds (per_set_total minus the
# gather, 15,201.7 - 1,411.6); every pubkey reference one G1 mixed addition of
# the gather (11).  So a 512-key sync aggregate weighs 1.4 single sets and a
# 98-set block of 128-key aggregates ~109 sets.
WORK_PER_SET = 13790.0
WORK_PER_PUBKEY = 11.0


def job_work(job_sets, job_refs) -> list[float]:
    """W(job) = sets * WORK_PER_SET + pubkey references * WORK_PER_PUBKEY"""
    return [s * WORK_PER_SET + k * WORK_PER_PUBKEY for s, k in zip(job_sets, job_refs)]


def batch_job_work(arrays: dict) -> list[float]:
    """job_work of every job of a bgv_batch (host numpy arrays)"""
    jo = np.asarray(arrays["job_offsets"], np.int64)
    po = np.asarray(arrays["pk_offsets"], np.int64)
    sets = jo[1:] - jo[:-1]
    refs = po[jo[1:]] - po[jo[:-1]]
    return job_work(sets.tolist(), refs.tolist())


def shard_jobs(job_weights, world: int, caps=None) -> list[list[int]]:
    """Whole jobs to ranks, greedy by work (largest first, each to the least
    loaded rank), job order kept inside a shard.  A job is never split (its
    verdict is an AND of its sets).  job_weights: batch_job_work / job_work,
    or set counts.  caps: relative speed of each rank (default all 1); load is
    compared as load / cap, so a device whose bulk context leaves CUs to a
    priority context (RESERVED_CAP) gets a proportionally smaller shard."""
    shards: list[list[int]] = [[] for _ in range(world)]
    load = [0.0] * world
    cap = [1.0] * world if caps is None else [float(c) for c in caps]
    w = [float(x) for x in job_weights]
    floor = min((x for x in w if x > 0), default=1.0)  # an empty job still costs a slot
    for j in sorted(range(len(w)), key=lambda j: (-w[j], j)):
        r = min(range(world), key=lambda k: (load[k] / cap[k], k))
        shards[r].append(j)
        load[r] += max(w[j], floor)
    return [sorted(s) for s in shards]


# throughput of a device whose bulk context reserves CUs for a priority context
# (bgv_cfg.cu_split < 0), relative to an unreserved one, at the 8-GPU shard
# size: workgroups go round-robin over the shader engines, so the bulk context
# runs at the pace of an engine that lost a CU, and the mid-size chains pay more
# than C4 (12,544 sets 9.55 -> 11.73 ms; C4 36.8 -> 41.7 ms).
# One value for both bindings: napi/reserved_cap.json (index.js reads it too).
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "napi", "reserved_cap.json")) as _f:
    RESERVED_CAP = float(json.load(_f)["RESERVED_CAP"])


def shard_balance(job_weights, shards) -> float:
    """max over shards of the shard's work / mean shard work (1.0 = even)"""
    loads = [sum(float(job_weights[j]) for j in s) for s in shards]
    mean = sum(loads) / max(len(loads), 1)
    return max(loads) / mean if mean else 1.0


def select_jobs(arrays: dict, jobs: list[int]) -> dict:
    """The bgv_batch arrays (host, numpy) of a subset of a batch's jobs, with
    job and pubkey offsets rebased; per-set arrays are sliced, the raw-key
    table is shared."""
    jo = np.asarray(arrays["job_offsets"], np.int64)
    po = np.asarray(arrays["pk_offsets"], np.int64)
    sets = np.concatenate([np.arange(jo[j], jo[j + 1]) for j in jobs]) if jobs else np.zeros(0, np.int64)
    sizes = np.array([jo[j + 1] - jo[j] for j in jobs], np.int64)
    k = po[sets + 1] - po[sets]
    idx = (np.concatenate([np.arange(po[i], po[i + 1]) for i in sets]) if len(sets) else np.zeros(0, np.int64))
    out = dict(arrays)
    out["n_sets"] = int(len(sets))
    out["n_jobs"] = len(jobs)
    out["job_offsets"] = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    out["pk_offsets"] = np.concatenate([[0], np.cumsum(k)]).astype(np.uint32)
    out["pk_indices"] = np.asarray(arrays["pk_indices"])[idx].astype(np.uint32) if len(idx) else np.zeros(1, np.uint32)
    n = int(arrays["n_sets"])
    for key, width in (("msgs", 32), ("sigs", 192), ("sig_len", 1), ("scalars", 1)):
        v = arrays.get(key)
        if v is not None:  # flat byte arrays and (n, width) arrays alike
            rows = np.asarray(v)[: max(n, 1) * width].reshape(max(n, 1), width) if width > 1 else np.asarray(v)
            out[key] = rows[sets].copy() if len(sets) else rows[:1].copy()
    return out


def allgather_partials(partial: bytes, dist, device=None) -> list[bytes]:
    """All-gather one 576-byte partial per rank; returns them in rank order."""
    import torch

    assert len(partial) == PARTIAL_BYTES
    t = torch.frombuffer(bytearray(partial), dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [p.cpu().numpy().tobytes() for p in parts]


def combine_sharded(dev, partial_result, dist, device=None):
    """The exchange half of verify_sharded: this rank's bgv_partial result
    (as dev.partial returns it) -> all-gather -> combined final check on
    `dev` (the context that made the partial), and the per-shard
    localisation when it fails.  Returns (node_batch_valid, local_job_results)."""
    part, _, jobs, _ = partial_result
    parts = allgather_partials(part, dist, device)
    if dev.combine_final(parts):
        return True, np.asarray(jobs, np.int32)
    return False, np.asarray(dev.partial_finish(), np.int32)


def verify_sharded(dev, arrays: dict, dist, device=None, on_device: bool = False):
    """This rank's shard -> partial -> all-gather -> combined final check, and
    the per-shard localisation when it fails.

    Returns (node_batch_valid, local_job_results): local_job_results[j] is
    this shard's job j as bgv_verify reports it (1 valid, 0 invalid, -code
    rejected).  Every rank takes the same branch (the combined verdict is
    computed from the same all-gathered partials)."""
    return combine_sharded(dev, dev.partial(arrays, on_device=on_device), dist, device)


def run_in_flight(submit, finish, steps: int, depth: int) -> bool:
    """Several batches in flight on one GPU.  Step k's device work goes to
    context k % depth through submit(k) -> concurrent.futures.Future (a worker
    thread: the library's calls release the GIL, and every context has its
    own streams), while the calling thread finishes the steps IN ORDER with
    finish(k, result) -> bool: the collectives of a sharded step (so every
    rank issues its all-gathers in the same order from one thread) and the
    verdict checks.  At most `depth` steps are outstanding, so context
    k % depth has been finished when step k is submitted to it.  The next
    batch's hash, pubkey and decode kernels then fill the SIMDs that a
    batch's Miller phase leaves idle (C4: 36.7 -> 33.1 ms per batch with
    three in flight, profiles/r06b_overlap_sizes.txt).  Returns the AND of
    the finishes."""
    from collections import deque

    pending: deque = deque()
    ok = True
    for k in range(steps):
        if len(pending) == depth:
            j, fut = pending.popleft()
            ok &= bool(finish(j, fut.result()))
        pending.append((k, submit(k)))
    while pending:
        j, fut = pending.popleft()
        ok &= bool(finish(j, fut.result()))
    return ok


def gather_job_results(local: np.ndarray, shards: list[list[int]], n_jobs: int, dist, device=None) -> np.ndarray:
    """All-gather every rank's per-job verdicts (padded to the largest shard)
    and place them at their batch job ids: the int32 verdict of every job of
    the node batch, on every rank."""
    import torch

    width = max(1, max(len(s) for s in shards))
    buf = np.zeros(width, np.int32)
    buf[: len(local)] = local
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    out = np.zeros(n_jobs, np.int32)
    for r, ids in enumerate(shards):
        vals = parts[r].cpu().numpy()
        out[np.asarray(ids, np.int64)] = vals[: len(ids)]
    return out
