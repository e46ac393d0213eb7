#!/bin/bash
# r06: GPU suite + default bench (tools/gpu_round.sh), then the two-batches-in-flight
# probe with the default hardware queues and with 8.  Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TEST_TIMEOUT=700 bash tools/gpu_round.sh || exit $?
timeout -k 10 200 python -u tools/overlap_probe.py > gpurun_out/overlap_q4.txt 2>&1 &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/overlap_probe.py > gpurun_out/overlap_q8.txt 2>&1
rc=$?
cat gpurun_out/overlap_q4.txt gpurun_out/overlap_q8.txt | grep mode
exit $rc
