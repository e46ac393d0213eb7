#!/bin/bash
# r06: the timed steps' device inputs synchronised once (default) against torch's
# stream waited for on every call (--input-sync per-call), three in flight, alternating
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06ad
run() {
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 30 "$@" > gpurun_out/r06ad/$tag.json 2> gpurun_out/r06ad/$tag.log || return $?
  python -c "import json; j=json.loads(open('gpurun_out/r06ad/$tag.json').read().strip().splitlines()[-1]); print('$tag', j['value'], j['ms_per_step'], j['c4_step_ms_p50'], j['one_in_flight']['ms_p50'])" | tee -a gpurun_out/r06ad/summary.txt
}
for r in 1 2 3; do run once_$r && run percall_$r --input-sync per-call || exit $?; done
