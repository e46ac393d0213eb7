#!/bin/bash
# r06: batches in flight x hardware queues (same box): C4 bench lines without the side legs
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/hwq
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 20 ${BARGS} > gpurun_out/hwq/$tag.json 2> gpurun_out/hwq/$tag.log || return $?
  python -c "import json,sys; j=json.loads(open('gpurun_out/hwq/$tag.json').read().strip().splitlines()[-1]); print('$tag', j['value'], j['ms_per_step'], j['one_in_flight']['ms_p50'])"
}
BARGS="--inflight 3" run if3_q4 X=1 &&
BARGS="--inflight 3" run if3_q16 GPU_MAX_HW_QUEUES=16 &&
BARGS="--inflight 4" run if4_q16 GPU_MAX_HW_QUEUES=16 &&
BARGS="--inflight 6" run if6_q24 GPU_MAX_HW_QUEUES=24 &&
BARGS="--inflight 3" run if3_q4b X=1
