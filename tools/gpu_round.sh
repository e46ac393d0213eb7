#!/bin/bash
# One GPU-box session: the -m gpu suite, then (unless it crashed) the default
# bench line.  Each GPU step has its own time limit; a crash / timeout stops
# the script before the next GPU step.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gputest.log 2>&1
rc=$?
tail -5 gpurun_out/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.log
brc=$?
tail -3 gpurun_out/bench.log
cat gpurun_out/bench.json | head -c 3000
exit $(( rc > brc ? rc : brc ))
