#!/bin/bash
# r06: pipeline knobs re-swept with three batches in flight (same box, alternating):
# default, no precomputed lines, 50% / 100% / 0% deferred checks, digit MSM
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/knobs
run() {
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 24 "$@" > gpurun_out/knobs/$tag.json 2> gpurun_out/knobs/$tag.log || return $?
  python -c "import json; j=json.loads(open('gpurun_out/knobs/$tag.json').read().strip().splitlines()[-1]); print('$tag', j['value'], j['ms_per_step'], j['one_in_flight']['ms_p50'])"
}
for r in 1 2; do
  run def$r && run nolines$r --cfg lines=0 && run defer50_$r --cfg defer_pct=50 && run defer100_$r --cfg defer_pct=100 && run defer0_$r --cfg defer_pct=0 && run msm4_$r --cfg msm=4 || exit $?
done
