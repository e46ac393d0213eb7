#!/bin/bash
# r06: the Fp2 sum-of-products leaf: microbenchmark, stage/parity tests on the default
# library (leaf in every calling unit), then an alternating C4 A/B of three builds:
#   K = libbgv_kara.so (Karatsuba everywhere), L = libbgv.so (leaf everywhere),
#   M = libbgv_kernkara.so (leaf in the Miller / latency units, Karatsuba in bgv_kernels.hip)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/fp2
timeout -k 10 120 ./tools/ubench_fp2 > gpurun_out/fp2/ubench.json 2>&1 || exit $?
cat gpurun_out/fp2/ubench.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_parity.py tests/test_gpu_decode_mixed.py tests/test_gpu_fp_ops.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fp2/tests.log 2>&1 || { tail -30 gpurun_out/fp2/tests.log; exit 1; }
tail -2 gpurun_out/fp2/tests.log
run() {
  local tag=$1 lib=$2; shift 2
  BGV_LIB=$PWD/lodestar_amd/$lib timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 24 "$@" > gpurun_out/fp2/$tag.json 2> gpurun_out/fp2/$tag.log || return $?
  python -c "import json; j=json.loads(open('gpurun_out/fp2/$tag.json').read().strip().splitlines()[-1]); s=j['roofline']['isolated']['stage_ms']; print('$tag', j['value'], j['ms_per_step'], j['one_in_flight']['ms_p50'], {k: s.get(k) for k in ('hash_to_g2','miller_loop','sig_decode_subgroup','pk_aggregate_scale')})"
}
for r in 1 2; do
  run K$r libbgv_kara.so && run L$r libbgv.so && run M$r libbgv_kernkara.so || exit $?
done
