#!/bin/bash
# r06: reserved-context faulted shard test, then an alternating same-box A/B of in-flight
# defaults: A = 3 in flight, B = 3 + pairs 4, C = 4 + pairs 4 + 16 HW queues, D = 4 + 16 HW queues
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab6
timeout -k 10 300 python -u -m pytest tests/test_gpu_shards.py -k reserved -x -v --timeout 200 --timeout-method thread > gpurun_out/ab6/test.log 2>&1 || { tail -30 gpurun_out/ab6/test.log; exit 1; }
grep -E "passed|failed" gpurun_out/ab6/test.log | tail -1
run() {
  local tag=$1; shift
  env $ENVS timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 24 "$@" > gpurun_out/ab6/$tag.json 2> gpurun_out/ab6/$tag.log || return $?
  python -c "import json; j=json.loads(open('gpurun_out/ab6/$tag.json').read().strip().splitlines()[-1]); print('$tag', j['value'], j['ms_per_step'], j['one_in_flight']['ms_p50'], (j['strong_shard_projection'] if 'strong_shard_projection' in j else ''))"
}
for r in 1 2 3; do
  ENVS="X=1" run A$r --inflight 3 &&
  ENVS="X=1" run B$r --inflight 3 --cfg pairs=4 &&
  ENVS="GPU_MAX_HW_QUEUES=16" run C$r --inflight 4 --cfg pairs=4 &&
  ENVS="GPU_MAX_HW_QUEUES=16" run D$r --inflight 4 || exit $?
done
