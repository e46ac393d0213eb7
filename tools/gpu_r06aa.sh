#!/bin/bash
# r06: quad Miller line-round operand plans in registers and the X^2 select in round 3 only
# (BGV_QUAD_PLAN 1, default) against the per-round table load and select (libbgv_qp0.so):
# same-box alternating sweeps at 12,544 sets, alone and four in flight
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06aa
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r06aa/tests.log 2>&1 || { tail -20 gpurun_out/r06aa/tests.log; exit 1; }
tail -1 gpurun_out/r06aa/tests.log
BGV_LIB=$PWD/lodestar_amd/libbgv_qp0.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q -k quad --timeout 200 --timeout-method thread > gpurun_out/r06aa/tests_qold.log 2>&1 || { tail -20 gpurun_out/r06aa/tests_qold.log; exit 1; }
tail -1 gpurun_out/r06aa/tests_qold.log
for r in 1 2 3; do
  for lib in libbgv.so libbgv_qp0.so; do
    BGV_LIB=$PWD/lodestar_amd/$lib timeout -k 10 200 python -u tools/sweep_modes.py --sizes 12544 --modes default --reps 9 | sed "s|^|$lib |" >> gpurun_out/r06aa/sweep.txt || exit 1
    echo "$lib" >> gpurun_out/r06aa/probe.txt
    BGV_LIB=$PWD/lodestar_amd/$lib timeout -k 10 200 python -u tools/overlap_probe.py --blocks 128 --ctx 4 --steps 12 2>/dev/null | grep contexts >> gpurun_out/r06aa/probe.txt || exit 1
  done
done
cat gpurun_out/r06aa/sweep.txt gpurun_out/r06aa/probe.txt
