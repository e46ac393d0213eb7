"""Four processes verifying on GPU 0 at once (the shape of the N>1 bench
rehearsal, and of several Lodestar processes sharing a card): each builds its
work-balanced shard of a C4 segment with torch (to_device copies, torch.zeros
signature buffer, torch.full signature lengths -- all on torch's stream), signs
it and verifies it at once.  The library runs on its own streams, so the
FIRST call only sees complete inputs because native.py waits for the
producing torch stream (_sync_producers; include/bgv.h bgv_batch).  Before
that wait, other processes' kernels delayed torch's fills enough for the first
verify of most ranks to report 23-106 bad jobs (r04, tools/diag_concurrent.py).
Every call of every rank must verify, through bgv_verify and through
bgv_partial + bgv_combine_final."""
import multiprocessing as mp
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 4
BLOCKS = 1024


def _rank(rank, q):
    try:
        sys.path.insert(0, ROOT)
        import torch

        import bench
        from lodestar_amd import native
        from lodestar_amd.dist import batch_job_work, select_jobs, shard_jobs
        dev = torch.device("cuda", 0)
        seg = bench.build_segment(list(range(BLOCKS)), seed=bench.SEED)
        shards = shard_jobs(batch_job_work(seg), WORLD)
        d = native.Device(0)
        d.gen_keys(0, bench.N_VALIDATORS, bench.SEED)
        a = select_jobs(seg, shards[rank])
        da = bench.to_device(a, torch, dev)
        sigs = torch.zeros((a["n_sets"], 192), dtype=torch.uint8, device=dev)
        d.gen_sign(da, sigs, on_device=True)
        da.update(sigs=sigs, sig_len=torch.full((a["n_sets"],), 96, dtype=torch.int32, device=dev), scalars=None)
        runs = []
        for _ in range(2):
            jr, _ = d.verify(da, on_device=True, want_set_codes=False)
            part, _, _, pok = d.partial(da, on_device=True)
            runs.append((int((jr != 1).sum()), bool(pok), bool(d.combine_final([part]))))
        d.close()
        q.put((rank, runs))
    except BaseException as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))


@pytest.mark.timeout(240)
def test_ranks_sharing_one_gpu_verify_from_the_first_call():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, q)) for r in range(WORLD)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=200) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in range(WORLD):
        assert not isinstance(out[r], str), out[r]
        for bad_jobs, pok, combined in out[r]:
            assert bad_jobs == 0 and pok and combined, (r, out[r])
