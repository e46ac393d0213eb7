#!/bin/bash
# r06: quad Miller operand selects through an LDS zero slot (BGV_QUAD_ZSLOT 1,
# default) against value selects (libbgv_qold.so): stage/parity tests, then
# same-box alternating sweeps at 12,544 sets, alone and four in flight
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06u
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r06u/tests.log 2>&1 || { tail -20 gpurun_out/r06u/tests.log; exit 1; }
tail -1 gpurun_out/r06u/tests.log
BGV_LIB=$PWD/lodestar_amd/libbgv_qold.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q -k quad --timeout 200 --timeout-method thread > gpurun_out/r06u/tests_qold.log 2>&1 || { tail -20 gpurun_out/r06u/tests_qold.log; exit 1; }
tail -1 gpurun_out/r06u/tests_qold.log
for r in 1 2 3; do
  for lib in libbgv.so libbgv_qold.so; do
    BGV_LIB=$PWD/lodestar_amd/$lib timeout -k 10 200 python -u tools/sweep_modes.py --sizes 12544 --modes default --reps 9 | sed "s|^|$lib |" >> gpurun_out/r06u/sweep.txt || exit 1
    echo "$lib" >> gpurun_out/r06u/probe.txt
    BGV_LIB=$PWD/lodestar_amd/$lib timeout -k 10 200 python -u tools/overlap_probe.py --blocks 128 --ctx 4 --steps 12 2>/dev/null | grep contexts >> gpurun_out/r06u/probe.txt || exit 1
  done
done
cat gpurun_out/r06u/sweep.txt gpurun_out/r06u/probe.txt
