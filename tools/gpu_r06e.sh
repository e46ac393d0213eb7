#!/bin/bash
# r06: four pairs per Miller item: stage + large tests, then C4 A/B (pairs 2 default vs 4), same box
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/p4
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_large.py -x -v --timeout 300 --timeout-method thread > gpurun_out/p4/tests.log 2>&1 || { tail -30 gpurun_out/p4/tests.log; exit 1; }
tail -3 gpurun_out/p4/tests.log
run() {
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 20 "$@" > gpurun_out/p4/$tag.json 2> gpurun_out/p4/$tag.log || return $?
  python -c "import json; j=json.loads(open('gpurun_out/p4/$tag.json').read().strip().splitlines()[-1]); r=j['roofline']; print('$tag', j['value'], j['ms_per_step'], j['one_in_flight']['ms_p50'], j['stage_ms']['miller_loop'], r['isolated']['stage_ms'].get('miller_loop'), j['roofline']['pipeline_variant']['pairs_per_item'])"
}
run a1 && run b1 --cfg pairs=4 && run a2 && run b2 --cfg pairs=4 && run b1if4 --cfg pairs=4 --inflight 4
