#!/bin/bash
# cyclotomic view squaring in the final exponentiation: stage + parity tests,
# A/B against the c_mul squaring at latency sizes, small-size view-Miller sweep
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TESTS="tests/test_gpu_stages.py tests/test_gpu_parity.py" LIBS="libbgv.so libbgv_fec0.so" SIZES=98,3136,12544 bash tools/gpu_ab.sh
timeout -k 10 300 python -u tools/sweep_modes.py --sizes 98,490,980,1960 --modes default,kv6 --reps 9 > gpurun_out/sweep_small_kv.txt 2>&1
cut -c1-200 gpurun_out/sweep_small_kv.txt
rm -rf gpurun_out/trace_lat
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/trace_lat -o run --output-format csv -- python3 tools/size_trace.py --sizes 98,3136,12544 --single 5 > gpurun_out/trace_lat.log 2>&1
python3 tools/size_trace.py --analyze $(find gpurun_out/trace_lat -name "*kernel_trace.csv" | head -1) > gpurun_out/timeline_lat.txt
grep ms_p50 gpurun_out/trace_lat.log
