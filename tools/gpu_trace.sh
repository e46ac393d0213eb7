#!/bin/bash
# Kernel timelines of the current library at chosen sizes (run from the repo
# root via gpurun):  SIZES=3136,12544 TAG=r05 bash tools/gpu_trace.sh
# -> gpurun_out/timeline_$TAG.txt
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-cur}
rm -rf gpurun_out/trace_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_$TAG -o run --output-format csv -- python3 tools/size_trace.py --sizes ${SIZES:-3136,12544} > gpurun_out/trace_$TAG.log 2>&1
python3 tools/size_trace.py --analyze $(find gpurun_out/trace_$TAG -name "*kernel_trace.csv" | head -1) > gpurun_out/timeline_$TAG.txt
rm -rf gpurun_out/trace_$TAG
