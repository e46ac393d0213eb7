#!/bin/bash
# Kernel timelines of the default library and a variant at chosen sizes
# (run from the repo root via gpurun):
#   VARIANT=lodestar_amd/libbgv_x.so SIZES=12544 bash tools/trace_ab.sh
# -> gpurun_out/timeline_ab_a.txt, gpurun_out/timeline_ab_b.txt
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VARIANT=${VARIANT:-lodestar_amd/libbgv_x.so}
for L in a b; do
  rm -rf gpurun_out/trace_ab_$L
  if [ $L = b ]; then export BGV_LIB=$VARIANT; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_ab_$L -o run --output-format csv -- python3 tools/size_trace.py --sizes ${SIZES:-12544} > gpurun_out/trace_ab_$L.log 2>&1
  python3 tools/size_trace.py --analyze $(find gpurun_out/trace_ab_$L -name "*kernel_trace.csv" | head -1) > gpurun_out/timeline_ab_$L.txt
  rm -rf gpurun_out/trace_ab_$L
done
