#!/bin/bash
# r06 round-end set on one box: GPU suite, smoke, then the round profile (tools/profile_r06.sh:
# default bench line, kernel trace + stats of the C4-only command, PMC passes).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TEST_TIMEOUT=700 NO_BENCH=1 bash tools/gpu_round.sh || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
TAG=${TAG:-r06z} bash tools/profile_r06.sh
