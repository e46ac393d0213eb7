#!/bin/bash
# r06: GPU suite, then same-box A/B: 50% deferred checks against the default 75%, and four in flight against three
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab7
TEST_TIMEOUT=800 NO_BENCH=1 bash tools/gpu_round.sh || exit $?
run() {
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 30 "$@" > gpurun_out/ab7/$tag.json 2> gpurun_out/ab7/$tag.log || return $?
  python -c "import json; j=json.loads(open('gpurun_out/ab7/$tag.json').read().strip().splitlines()[-1]); print('$tag', j['value'], j['ms_per_step'], j['one_in_flight']['ms_p50'])"
}
for r in 1 2 3; do run def$r && run d50_$r --cfg defer_pct=50 && run if4_$r --inflight 4 || exit $?; done
