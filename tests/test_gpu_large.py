"""Large-batch GPU parity: >= 65,536 sets switches the Miller stage to two
pairs per work item (shared accumulator).  Device-generated keys and
signatures (checked against the oracle in test_gpu_parity), faults injected
by signing a different message; expected per-job verdicts follow from which
sets were faulted (the oracle's verdict for a wrong-message set is False,
golden job 2)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_two_pair_items_batch_with_faults():
    from lodestar_amd import native
    d = native.Device(0)
    try:
        d.gen_keys(0, 4096, 7)
        rng = np.random.default_rng(11)
        n, k, per_job = 66640, 4, 98  # 680 jobs of 98 sets
        idx = rng.integers(0, 4096, size=n * k).astype(np.uint32)
        msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        arrays = {"n_sets": n, "n_jobs": n // per_job,
                  "job_offsets": (np.arange(n // per_job + 1) * per_job).astype(np.uint32),
                  "pk_offsets": (np.arange(n + 1) * k).astype(np.uint32), "pk_indices": idx, "msgs": msgs}
        bad = np.zeros(n, bool)
        bad[rng.choice(n, size=40, replace=False)] = True
        sign_msgs = msgs.copy()
        sign_msgs[bad, 5] ^= 0x80
        sigs = np.zeros((n, 192), np.uint8)
        d.gen_sign(dict(arrays, msgs=sign_msgs), sigs)
        arrays.update(sigs=sigs, sig_len=np.full(n, 96, np.uint32),
                      scalars=rng.integers(1, 2**63, size=n, dtype=np.uint64))
        jr, sc = d.verify(arrays)
        want = [0 if bad[j * per_job:(j + 1) * per_job].any() else 1 for j in range(n // per_job)]
        assert jr.tolist() == want
        assert (sc == 0).all()
        assert d.last_stats.batch_retries == 1
        # an odd job size leaves single-pair items inside 2-pair batches
        arrays2 = dict(arrays)
        arrays2["job_offsets"] = np.array([0, 1, 100, 30001, n], np.uint32)
        arrays2["n_jobs"] = 4
        jr2, _ = d.verify(arrays2)
        bounds = [0, 1, 100, 30001, n]
        assert jr2.tolist() == [0 if bad[bounds[i]:bounds[i + 1]].any() else 1 for i in range(4)]
    finally:
        d.close()


@pytest.mark.parametrize("pairs", [4])
def test_four_pair_items_ragged_jobs_with_faults(pairs):
    """pairs_per_item = 4 (miller_loop_lines4 over precomputed lines): jobs of
    every size mod 4 leave items of 1, 2 and 3 live pairs, whose dead pairs'
    lines are forced to 1; faulted sets in items at every position; verdicts
    and the retry count equal the two-pair default's"""
    from lodestar_amd import native
    d4 = native.Device(0, pairs=pairs, lines=1)
    d2 = native.Device(0)
    try:
        for d in (d4, d2):
            d.gen_keys(0, 4096, 7)
        rng = np.random.default_rng(13)
        sizes = [98, 97, 1, 2, 3, 5, 6, 7, 99, 100, 128, 4, 9, 13, 98, 98]
        sizes += [98] * ((70000 - sum(sizes)) // 98)
        n = sum(sizes)
        k = 4
        idx = rng.integers(0, 4096, size=n * k).astype(np.uint32)
        msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        jo = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
        arrays = {"n_sets": n, "n_jobs": len(sizes), "job_offsets": jo,
                  "pk_offsets": (np.arange(n + 1) * k).astype(np.uint32), "pk_indices": idx, "msgs": msgs}
        bad = np.zeros(n, bool)
        for j in (2, 4, 5, 7, 11, 13):  # a fault in a short job / at each item position
            bad[jo[j] + (j % int(sizes[j]))] = True
        bad[rng.choice(n, size=24, replace=False)] = True
        sign_msgs = msgs.copy()
        sign_msgs[bad, 5] ^= 0x80
        sigs = np.zeros((n, 192), np.uint8)
        d2.gen_sign(dict(arrays, msgs=sign_msgs), sigs)
        arrays.update(sigs=sigs, sig_len=np.full(n, 96, np.uint32),
                      scalars=rng.integers(1, 2**63, size=n, dtype=np.uint64))
        want = [0 if bad[jo[j]:jo[j + 1]].any() else 1 for j in range(len(sizes))]
        jr4, sc4 = d4.verify(arrays)
        assert d4.last_stats.layout()["pairs_per_item"] == pairs and d4.last_stats.layout()["lines"] == 1
        assert jr4.tolist() == want and (sc4 == 0).all()
        assert d4.last_stats.batch_retries == 1
        jr2, _ = d2.verify(arrays)
        assert jr2.tolist() == want
        # the clean batch passes the batch check with no retry
        clean = dict(arrays, msgs=sign_msgs)
        jr4c, _ = d4.verify(clean)
        assert jr4c.tolist() == [1] * len(sizes) and d4.last_stats.batch_retries == 0
    finally:
        d4.close()
        d2.close()


def test_many_jobs_batch_fold_and_fold_boundary():
    """2,100 single-set jobs: the batch product folds by 32 three times
    (2100 -> 66 -> 3 -> 1, ping-ponging f_batch and f_tmp); a job of exactly
    256 sets is the largest that folds in one workgroup (bgv_tail.hip)."""
    from lodestar_amd import native
    d = native.Device(0)
    try:
        d.gen_keys(0, 512, 3)
        rng = np.random.default_rng(5)
        n, k = 2100, 2
        idx = rng.integers(0, 512, size=n * k).astype(np.uint32)
        msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        arrays = {"n_sets": n, "n_jobs": n, "job_offsets": np.arange(n + 1, dtype=np.uint32),
                  "pk_offsets": (np.arange(n + 1) * k).astype(np.uint32), "pk_indices": idx, "msgs": msgs}
        sigs = np.zeros((n, 192), np.uint8)
        d.gen_sign(arrays, sigs)
        arrays.update(sigs=sigs, sig_len=np.full(n, 96, np.uint32),
                      scalars=rng.integers(1, 2**63, size=n, dtype=np.uint64))
        jr, _ = d.verify(arrays)
        assert jr.tolist() == [1] * n and d.last_stats.batch_retries == 0
        good = sigs.copy()
        bad = [7, 1500, 2099]
        for i in bad:
            arrays["sigs"][i] = good[(i + 1) % n]  # a valid signature of another set
        jr, _ = d.verify(arrays)
        assert jr.tolist() == [0 if i in bad else 1 for i in range(n)]
        assert d.last_stats.batch_retries == 1
        # 256-set job (fold path) + 1844 singles; then a 257-set job (tree path)
        for first in (256, 257):
            a2 = dict(arrays, sigs=good.copy())
            a2["job_offsets"] = np.concatenate([[0], np.arange(first, n + 1)]).astype(np.uint32)
            a2["n_jobs"] = len(a2["job_offsets"]) - 1
            jr2, _ = d.verify(a2)
            assert jr2.tolist() == [1] * a2["n_jobs"]
            a2["sigs"][first // 2] = good[0]
            jr2, _ = d.verify(a2)
            assert jr2.tolist() == [0] + [1] * (a2["n_jobs"] - 1)
    finally:
        d.close()
