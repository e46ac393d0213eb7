#!/bin/bash
# r06: bench with batches in flight (default 3), then 2 and 4, then the N = 2 rehearsal on one GPU (gloo)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 20 > gpurun_out/bench_if3.json 2> gpurun_out/bench_if3.log &&
timeout -k 10 300 python -u bench.py --steps 20 --no-c2 --no-cpu --inflight 4 > gpurun_out/bench_if4.json 2> gpurun_out/bench_if4.log &&
timeout -k 10 300 python -u bench.py --steps 20 --no-c2 --no-cpu --inflight 2 > gpurun_out/bench_if2.json 2> gpurun_out/bench_if2.log &&
BGV_BENCH_REHEARSE=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 6 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.log
rc=$?
for f in bench_if3 bench_if4 bench_if2 rehearse2; do python - "$f" <<'PY'
import json, sys
f = sys.argv[1]
try:
    j = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
except Exception as e:
    print(f, "no line", e); sys.exit(0)
print(f, j["value"], j["ms_per_step"], j.get("c4_step_ms_p50"), j.get("one_in_flight"), j["verified"],
      (j.get("strong_shard_projection") or {}).get("c4_over_8"), (j.get("roofline") or {}).get("frac"),
      ((j.get("roofline") or {}).get("isolated") or {}).get("frac"), j.get("weak_scaling"))
PY
done
exit $rc
