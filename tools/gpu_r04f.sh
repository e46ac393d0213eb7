#!/bin/bash
# hash maps launched before the host set-up: full GPU suite, latency sweep, single-set trace
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_f.log 2>&1 || { tail -30 gpurun_out/gputest_f.log; exit 1; }
tail -2 gpurun_out/gputest_f.log
timeout -k 10 300 python -u tools/sweep_modes.py --sizes 98,1568,3136,6272,12544 --modes default --reps 9 > gpurun_out/sweep_f.txt 2>&1
cut -c1-80 gpurun_out/sweep_f.txt
rm -rf gpurun_out/trace_f
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/trace_f -o run --output-format csv -- python3 tools/size_trace.py --sizes 3136,12544 --single 5 > gpurun_out/trace_f.log 2>&1
python3 tools/size_trace.py --analyze $(find gpurun_out/trace_f -name "*kernel_trace.csv" | head -1) > gpurun_out/timeline_f.txt
grep ms_p50 gpurun_out/trace_f.log
grep -E "sets:|hash_map|copyBuffer|gen_scalars" gpurun_out/timeline_f.txt | cut -c1-90
