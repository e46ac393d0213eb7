#!/bin/bash
# stage tests, C4 A/B of the one-wave hash kernel variants, view-Miller
# boundary sweep at mid sizes
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TESTS="tests/test_gpu_stages.py" LIBS="libbgv.so libbgv_pkc0.so libbgv_hw1.so libbgv_hw1ci.so" SIZES=100352 bash tools/gpu_ab.sh
timeout -k 10 400 python -u tools/sweep_modes.py --sizes 2048,3136,4704,6272,9408,10976 --modes default,kv0,kv3,kv6 --reps 7 > gpurun_out/sweep_kvb.txt 2>&1
cat gpurun_out/sweep_kvb.txt
