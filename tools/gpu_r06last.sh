#!/bin/bash
# r06 last check of the final tree: GPU suite, smoke, default bench line
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06last
TEST_TIMEOUT=700 NO_BENCH=1 bash tools/gpu_round.sh || exit $?
cp gpurun_out/gputest.log gpurun_out/r06last/gputest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06last/smoke.log 2>&1 || { cat gpurun_out/r06last/smoke.log; exit 1; }
tail -1 gpurun_out/r06last/smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/r06last/bench_default.json 2> gpurun_out/r06last/bench_default.log || { tail -5 gpurun_out/r06last/bench_default.log; exit 1; }
head -c 700 gpurun_out/r06last/bench_default.json; echo
