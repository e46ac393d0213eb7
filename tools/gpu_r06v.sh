#!/bin/bash
# r06 final set on one box: GPU suite, smoke, default bench line, and the
# kernel timelines of one set / one epoch / the C4/8 shard (tools/size_trace.py)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06v
TEST_TIMEOUT=700 NO_BENCH=1 bash tools/gpu_round.sh || exit $?
cp gpurun_out/gputest.log gpurun_out/r06v/gputest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06v/smoke.log 2>&1 || { cat gpurun_out/r06v/smoke.log; exit 1; }
tail -1 gpurun_out/r06v/smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/r06v/bench_default.json 2> gpurun_out/r06v/bench_default.log || { tail -5 gpurun_out/r06v/bench_default.log; exit 1; }
head -c 1500 gpurun_out/r06v/bench_default.json; echo
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06v/trace_sizes -o run --output-format csv -- python3 tools/size_trace.py --sizes 98,3136,12544 > gpurun_out/r06v/size_trace.log 2>&1 || { tail -5 gpurun_out/r06v/size_trace.log; exit 1; }
python3 tools/size_trace.py --analyze $(find gpurun_out/r06v/trace_sizes -name "*kernel_trace.csv" | head -1) > gpurun_out/r06v/timelines_98_3136_12544.txt
grep "==" gpurun_out/r06v/timelines_98_3136_12544.txt
