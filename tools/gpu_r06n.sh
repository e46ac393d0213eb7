#!/bin/bash
# r06: the register-only MSM (k_msm_scan) — stage and parity tests, then a
# same-box alternating A/B of the default bench against the two-kernel form
# (libbgv_msmold.so = tools/build.py --variant msmold BGV_MSM_SCAN=0)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab8
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/ab8/tests.log 2>&1 || { tail -20 gpurun_out/ab8/tests.log; exit 1; }
tail -3 gpurun_out/ab8/tests.log
run() {
  local tag=$1 lib=$2; shift 2
  BGV_LIB=$PWD/lodestar_amd/$lib timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 30 "$@" > gpurun_out/ab8/$tag.json 2> gpurun_out/ab8/$tag.log || return $?
  python -c "import json; j=json.loads(open('gpurun_out/ab8/$tag.json').read().strip().splitlines()[-1]); print('$tag', j['value'], j['ms_per_step'], j['one_in_flight']['ms_p50'], j['roofline']['frac'])"
}
for r in 1 2 3; do run scan$r libbgv.so && run old$r libbgv_msmold.so || exit $?; done
