#!/bin/bash
# r06: pubkey gather with the index prefetched two ahead (BGV_PKC_IDX2 1,
# default) against one ahead (libbgv_pk1.so): tests, then alternating bench C4
# legs (in flight + the lone batch's gather stage time)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06ab/tests.log 2>&1 || { tail -20 gpurun_out/r06ab/tests.log; exit 1; }
tail -1 gpurun_out/r06ab/tests.log
run() {
  local tag=$1 lib=$2
  BGV_LIB=$PWD/lodestar_amd/$lib timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 30 > gpurun_out/r06ab/$tag.json 2> gpurun_out/r06ab/$tag.log || return $?
  python -c "import json; j=json.loads(open('gpurun_out/r06ab/$tag.json').read().strip().splitlines()[-1]); r=j['roofline']; print('$tag', j['value'], j['ms_per_step'], j['one_in_flight']['ms_p50'], 'gather', r['per_stage']['pk_gather']['ms'], 'iso', r['isolated']['stage_ms']['pk_gather'])" | tee -a gpurun_out/r06ab/summary.txt
}
for r in 1 2 3; do run idx2_$r libbgv.so && run idx1_$r libbgv_pk1.so || exit $?; done
