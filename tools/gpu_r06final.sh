#!/bin/bash
# r06 round-end set of the final tree: GPU suite, smoke, then the round profile
# (tools/profile_r06.sh: default bench line, kernel trace + stats of the
# C4-only command, PMC passes) and the timed-region agreement / in-flight views
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TEST_TIMEOUT=700 NO_BENCH=1 bash tools/gpu_round.sh || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
TAG=r06fin bash tools/profile_r06.sh || exit $?
T=$(find gpurun_out/prof_r06fin/trace_c4 -name "*kernel_trace.csv" | head -1)
python3 tools/timed_region_check.py $T gpurun_out/prof_r06fin/bench_c4_traced.json > gpurun_out/prof_r06fin/timed_region_check.txt
python3 tools/inflight_trace.py $T > gpurun_out/prof_r06fin/inflight_timeline.txt
cat gpurun_out/prof_r06fin/timed_region_check.txt
