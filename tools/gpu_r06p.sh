#!/bin/bash
# r06: streams per context (libbgv_s1.so: one stream, libbgv_s2.so: two) against
# the four-stream default, with batches in flight: parity first, then probes
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06p
for v in s1 s2; do
  BGV_LIB=$PWD/lodestar_amd/libbgv_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06p/tests_$v.log 2>&1 || { tail -20 gpurun_out/r06p/tests_$v.log; exit 1; }
  tail -1 gpurun_out/r06p/tests_$v.log
done
probe() {
  local v=$1 b=$2 c=$3
  echo "lib=$v blocks=$b ctx=$c" >> gpurun_out/r06p/probe.txt
  BGV_LIB=$PWD/lodestar_amd/$v timeout -k 10 240 python -u tools/overlap_probe.py --blocks $b --ctx $c --steps 12 >> gpurun_out/r06p/probe.txt 2>&1
}
for r in 1 2; do
  for v in libbgv.so libbgv_s1.so libbgv_s2.so; do
    probe $v 128 4 && probe $v 1024 3 && probe $v 32 4 || { echo "probe failed"; tail -5 gpurun_out/r06p/probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/r06p/probe.txt
