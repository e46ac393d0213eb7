"""GPU parity of the per-stage intermediates (SURVEY §8c golden plan): every
stage of the HIP pipeline, read back through the test-only ABI entry
bgv_debug_stages, is byte-identical to the oracle's value in
tests/golden/batch_vectors.json (tools/gen_golden.py):

  decoded signature, H(m), aggregated pubkey, r_i * pubkey   (affine points)
  GT value of every set pair and every (-G1, S_job) pair    (FE of the Miller value)
  S_job = sum r_i sigma_i, GT value of every job product and of the batch

Miller values themselves are not canonical (projective line scalings differ
by factors the final exponentiation kills), so pairs are compared after it.
The device FE computes the cube of the textbook value, and the golden values
are e(P, Q)^3.  Each pipeline variant a batch can take is compared:
latency mode (two-lane hash maps, cooperative G2 and Miller), the bulk
one-lane kernels, the bulk Miller kernel with one and with two pairs per work
item, and the per-job Pippenger MSM for S_job.
"""
import numpy as np
import pytest

from oracle import bls12_381 as B
from tests import gpu_util as G
from tests.hostcheck import b_tower

pytestmark = pytest.mark.gpu

MODES = {
    "latency": {},
    "coop6_jobs18": {"miller": 6, "job_lanes": 18},
    "duo_msm_fused_clear3": {"miller": 2, "msm": 1, "clear_lanes": 3},
    "quad_msm0_clear3": {"miller": 4, "msm": 0, "clear_lanes": 3},
    "quad_split_msm4": {"miller": 4, "msm": 4, "split": 1, "clear_lanes": 3},
    "quad_split_msm3": {"miller": 4, "msm": 3, "split": 1, "clear_lanes": 3},
    "split_one_lane_miller_msm2": {"split": 1, "miller": 1, "msm": 2, "clear_lanes": 1},
    "duo_clear1_msm4": {"split": 1, "miller": 2, "msm": 4, "clear_lanes": 1},
    "bulk": {"split": 0},
    "bulk_serial_msm": {"split": 0, "miller": 1, "msm": 1, "pairs": 1},
    "c4_path": {"split": 0, "miller": 1, "msm": 2, "pairs": 2},
    # four pairs per item over precomputed lines (miller_loop_lines4); the golden
    # jobs' sizes leave items of 1-3 live pairs (dummy lines forced to 1)
    "c4_path_pairs4": {"split": 0, "miller": 1, "msm": 2, "pairs": 4, "lines": 1},
    "bulk_msm4": {"split": 0, "miller": 1, "msm": 4, "pairs": 1},
    # two-pair Miller loop in Karatsuba views (miller_kv.h), 9 and 18 lanes per two pairs
    "kv3_clear3_msm4": {"split": 1, "miller_kv": 3, "msm": 4, "clear_lanes": 3},
    "kv6_clear9": {"split": 1, "miller_kv": 6, "clear_lanes": 9},
    "kv9_clear9": {"split": 1, "miller_kv": 9, "clear_lanes": 9},
    "kv2_clear3_msm4": {"split": 1, "miller_kv": 2, "msm": 4, "clear_lanes": 3},
}


def _flat(gt_bytes: bytes):
    return B.tower_to_f12(b_tower(gt_bytes))


def _golden_gt(hexstr: str):
    return tuple(int(hexstr[96 * k: 96 * k + 96], 16) for k in range(12))


@pytest.fixture(scope="module")
def golden():
    v = G.batch_vectors()
    sets = [s for j in v["jobs"] for s in j["sets"]]
    return v, sets


@pytest.mark.parametrize("mode", list(MODES))
def test_stage_values_match_oracle(golden, mode):
    from lodestar_amd import native
    v, sets = golden
    d = native.Device(0, **MODES[mode])
    try:
        G.load_golden_table(d)
        arrays, expected, codes = G.golden_arrays()
        out = d.debug_stages(arrays)
    finally:
        d.close()
    n, J = arrays["n_sets"], arrays["n_jobs"]
    assert out["job_result"].tolist() == expected
    assert out["set_code"].tolist() == codes
    for i, s in enumerate(sets):
        assert out["sig_aff"][i].tobytes().hex() == s["sig_aff"], ("sig_aff", i)
        assert out["h_aff"][i].tobytes().hex() == s["h_aff"], ("h_aff", i)
        assert out["pk_agg"][i].tobytes().hex() == s["pk_agg"], ("pk_agg", i)
        assert out["rpk_aff"][i].tobytes().hex() == s["rpk_aff"], ("rpk_aff", i)
    for j, job in enumerate(v["jobs"]):
        assert out["s_aff"][j].tobytes().hex() == job["s_aff"], ("s_aff", j)
        assert B.f12_eq(_flat(out["job_fe"][j].tobytes()), _golden_gt(job["job_gt"])), ("job_gt", j)
        assert B.f12_eq(_flat(out["pair_fe"][n + j].tobytes()), _golden_gt(job["job_pair_gt"])), ("job_pair", j)
    assert B.f12_eq(_flat(out["batch_fe"].tobytes()), _golden_gt(v["batch_gt"]))
    # set pairs: one Miller value per set, or (two pairs per work item) the
    # item's product at its first set and the identity at its second; an item
    # with a rejected pubkey contributes the identity
    step = 2 if MODES[mode].get("miller_kv", 0) > 0 else MODES[mode].get("pairs", 1)
    jo = arrays["job_offsets"]
    for j in range(J):
        beg, end = int(jo[j]), int(jo[j + 1])
        for i in range(beg, end, step):
            grp = list(range(i, min(i + step, end)))
            want = B.F12_ONE
            if all(sets[k]["pk_agg"] != "00" * 96 for k in grp):  # no rejected pubkey in the item
                for k in grp:
                    want = B.f12_mul(want, _golden_gt(sets[k]["pair_gt"]))
            assert B.f12_eq(_flat(out["pair_fe"][i].tobytes()), want), ("pair", i)
            for k in grp[1:]:
                assert B.f12_eq(_flat(out["pair_fe"][k].tobytes()), B.F12_ONE), ("pair2", k)


def test_stage_values_independent_of_batching(golden):
    """the same job alone and inside the full batch: identical stage values
    (each set's values depend only on its own inputs and scalar)"""
    from lodestar_amd import native
    v, sets = golden
    d = native.Device(0)
    try:
        G.load_golden_table(d)
        full = d.debug_stages(G.golden_arrays()[0])
        first = 0
        for j, job in enumerate(v["jobs"]):
            one = d.debug_stages(G.golden_arrays([j])[0])
            k = len(job["sets"])
            for key in ("sig_aff", "h_aff", "pk_agg", "rpk_aff"):
                assert (one[key][:k] == full[key][first:first + k]).all(), (key, j)
            assert (one["s_aff"][0] == full["s_aff"][j]).all() if v["jobs"][j]["sets"] else True
            first += k
    finally:
        d.close()


def test_debug_pair_values_before_the_product_tree():
    """bgv_debug_stages' pair values are every pair's own Miller value even when
    the two-level job fold (k_job_prefold, default for <= 256 jobs of 64-256
    sets, e.g. one C2 gossip batch) folds groups of them in place: identical
    with the fold on and off, and their product is the job's value (1 for a
    valid job)."""
    from lodestar_amd import native
    from tests.test_gpu_parity import _synthetic_on
    outs = {}
    for prefold in (0, 1):
        d = native.Device(0, prefold=prefold)
        try:
            d.gen_keys(0, 512, 5)
            a, bad = _synthetic_on(d, 64, 8, 0, 512, 21)
            a["n_jobs"] = 1
            a["job_offsets"] = np.array([0, 64], np.uint32)
            out = d.debug_stages(a)
            assert out["job_result"].tolist() == [1]
            assert d.last_stats.layout() is not None
            outs[prefold] = out
        finally:
            d.close()
    assert (outs[0]["pair_fe"] == outs[1]["pair_fe"]).all()
    prod = B.F12_ONE
    for k in range(65):  # 64 set pairs and the job's (-G1, S_job) pair
        prod = B.f12_mul(prod, _flat(outs[1]["pair_fe"][k].tobytes()))
    assert B.f12_eq(prod, _flat(outs[1]["job_fe"][0].tobytes()))
    assert B.f12_eq(prod, B.F12_ONE)
