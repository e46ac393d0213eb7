"""Repeat bgv_debug_stages on the golden batch in one bgv_cfg mode and report
which stage values differ from the golden ones (BGV_LIB selects the library)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from lodestar_amd import native
    from tests import gpu_util as G
    from tests.test_gpu_stages import MODES
    mode, reps = sys.argv[1], int(sys.argv[2])
    v = G.batch_vectors()
    sets = [s for j in v["jobs"] for s in j["sets"]]
    bad_runs = 0
    for r in range(reps):
        d = native.Device(0, **MODES[mode])
        G.load_golden_table(d)
        arrays, expected, codes = G.golden_arrays()
        out = d.debug_stages(arrays)
        d.close()
        diff = {}
        if out["job_result"].tolist() != expected:
            diff["job_result"] = [j for j, (a, b) in enumerate(zip(out["job_result"].tolist(), expected)) if a != b]
        for key in ("sig_aff", "h_aff", "pk_agg", "rpk_aff"):
            bad = [i for i, s in enumerate(sets) if out[key][i].tobytes().hex() != s[key]]
            if bad:
                diff[key] = bad[:8]
        bad = [j for j, job in enumerate(v["jobs"]) if out["s_aff"][j].tobytes().hex() != job["s_aff"]]
        if bad:
            diff["s_aff"] = bad[:8]
        if diff:
            bad_runs += 1
            print(json.dumps({"rep": r, "diff": diff}), flush=True)
    print(json.dumps({"mode": mode, "lib": os.environ.get("BGV_LIB", "default"), "reps": reps, "bad_runs": bad_runs}))


if __name__ == "__main__":
    main()
