#!/bin/bash
# r06: one wave per SIMD (512 registers, no scratch spills) for the bulk hash /
# signature / pubkey kernels, with batches in flight: default bench C4 leg
# alternating with libbgv_hw1 / _sw1 / _pw1 (BGV_HASH_WAVES / BGV_SIG_WAVES /
# BGV_PK_WAVES = 1)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06s
run() {
  local tag=$1 lib=$2; shift 2
  BGV_LIB=$PWD/lodestar_amd/$lib timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 30 "$@" > gpurun_out/r06s/$tag.json 2> gpurun_out/r06s/$tag.log || return $?
  python -c "import json; j=json.loads(open('gpurun_out/r06s/$tag.json').read().strip().splitlines()[-1]); print('$tag', j['value'], j['ms_per_step'], j['one_in_flight']['ms_p50'], j['roofline']['frac'], j.get('c4_over_8', {}))" | tee -a gpurun_out/r06s/summary.txt
}
for r in 1 2; do run def$r libbgv.so && run hw1_$r libbgv_hw1.so && run sw1_$r libbgv_sw1.so && run pw1_$r libbgv_pw1.so || exit $?; done
