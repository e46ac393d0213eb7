#!/bin/bash
# r06: four pairs per Miller item (--cfg pairs=4) against the default two, three in flight, alternating
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06ac
run() {
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 30 "$@" > gpurun_out/r06ac/$tag.json 2> gpurun_out/r06ac/$tag.log || return $?
  python -c "import json; j=json.loads(open('gpurun_out/r06ac/$tag.json').read().strip().splitlines()[-1]); print('$tag', j['value'], j['ms_per_step'], j['one_in_flight']['ms_p50'])" | tee -a gpurun_out/r06ac/summary.txt
}
for r in 1 2 3; do run p2_$r && run p4_$r --cfg pairs=4 || exit $?; done
