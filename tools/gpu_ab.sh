#!/bin/bash
# One GPU call: a test subset, then an A/B of variant libraries at mid sizes,
# then kernel timelines of the default library.  Every GPU step has its own
# limit; the chain stops at the first failure.
#   TESTS="tests/test_gpu_stages.py" LIBS="libbgv_r03.so libbgv.so" SIZES=3136,12544 bash tools/gpu_ab.sh
set -e
cd "${GRAFT_REPO_ROOT:-.}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab.txt
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_ab.log 2>&1 || { tail -30 gpurun_out/gputest_ab.log; exit 1; }
  tail -3 gpurun_out/gputest_ab.log
fi
if [ -n "$LIBS" ]; then
  for rep in 1 2; do
    LIBS="$LIBS" SIZES=${SIZES:-3136,12544} bash tools/ab_lib.sh
  done
  cat gpurun_out/ab.txt
fi
if [ -n "$TRACE" ]; then
  rm -rf gpurun_out/trace_ab
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_ab -o run --output-format csv -- python3 tools/size_trace.py --sizes $TRACE > gpurun_out/trace_ab.log 2>&1
  python3 tools/size_trace.py --analyze $(find gpurun_out/trace_ab -name "*kernel_trace.csv" | head -1) > gpurun_out/timeline_ab.txt
  cat gpurun_out/timeline_ab.txt | cut -c1-100
fi
