#!/bin/bash
# r06: pairs = 4 against the default two pairs, three in flight, alternating three times (same box)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/p4b
run() {
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 30 "$@" > gpurun_out/p4b/$tag.json 2> gpurun_out/p4b/$tag.log || return $?
  python -c "import json; j=json.loads(open('gpurun_out/p4b/$tag.json').read().strip().splitlines()[-1]); print('$tag', j['value'], j['ms_per_step'], j['one_in_flight']['ms_p50'])"
}
for r in 1 2 3; do run A$r && run B$r --cfg pairs=4 || exit $?; done
