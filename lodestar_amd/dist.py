"""Multi-GPU glue for the batch verifier.

Signature sets shard by job across ranks (one process per GPU).  Every rank
reduces its shard to one Fp12 Miller product (576 B, bgv_partial); the
partials are all-gathered (RCCL over xGMI on the GPU node, gloo in the CPU
tests) and multiplied before ONE final exponentiation (bgv_combine_final).
At 576 B per rank the exchange is latency-bound, so a single all-gather is
the whole collective; there is no other data-path communication.
"""
from __future__ import annotations

PARTIAL_BYTES = 576


def shard_jobs(job_sizes: list[int], world: int) -> list[list[int]]:
    """Whole jobs to ranks, greedy by set count (largest first), job order kept
    inside a shard.  A job is never split (its verdict is an AND of its sets)."""
    shards: list[list[int]] = [[] for _ in range(world)]
    load = [0] * world
    for j in sorted(range(len(job_sizes)), key=lambda j: (-job_sizes[j], j)):
        r = load.index(min(load))
        shards[r].append(j)
        load[r] += max(job_sizes[j], 1)
    return [sorted(s) for s in shards]


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


def verify_sharded(dev, arrays: dict, dist, device=None, on_device: bool = False) -> tuple[bool, bool]:
    """This rank's shard -> partial -> all-gather -> combined final check.
    Returns (node_batch_valid, this_shard_parsed_ok)."""
    part, _, ok = dev.partial(arrays, on_device=on_device)
    parts = allgather_partials(part, dist, device)
    return dev.combine_final(parts), ok
