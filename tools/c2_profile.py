"""C2 latency probe for profiling runs: the bench's gossip batch (64 sets x
128 pubkeys, one job, host arrays) verified REPS times, with the per-call
host-to-verdict latency and the library's stage times printed.  Run under
`rocprofv3 --kernel-trace` to get the C2 kernel timeline (tools/c2_timeline.py)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from lodestar_amd import native  # noqa: E402

REPS = int(os.environ.get("REPS", "20"))

d = native.Device(0)
d.gen_keys(0, bench.N_VALIDATORS, bench.SEED)
g = bench.build_segment([0], seed=bench.SEED + 1000)
n2, k2 = 64, bench.ATT_K
a = {"n_sets": n2, "n_jobs": 1, "job_offsets": np.array([0, n2], np.uint32),
     "pk_offsets": (np.arange(n2 + 1) * k2).astype(np.uint32),
     "pk_indices": g["pk_indices"][: n2 * k2].copy(), "msgs": g["msgs"][:n2].copy(), "n_raw": 0}
s2 = np.zeros((n2, 192), np.uint8)
d.gen_sign(a, s2)
a.update(sigs=s2, sig_len=np.full(n2, 96, np.uint32))
lat = []
for _ in range(REPS):
    t1 = time.perf_counter()
    jr, _ = d.verify(a, want_set_codes=False)
    lat.append((time.perf_counter() - t1) * 1e3)
    assert jr.tolist() == [1]
st = d.last_stats
print("p50 ms", round(float(np.median(lat[1:])), 3), "device total ms", round(st.total_ms, 3))
print({d.stage_name(i): round(float(st.stage_ms[i]), 3) for i in range(native.N_STAGES) if d.stage_name(i) != "unknown"})
