#!/bin/bash
# thresholds at 32,000 / 60,000 sets: full GPU suite, default sweep over the moved cliffs, default bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_h.log 2>&1 || { tail -30 gpurun_out/gputest_h.log; exit 1; }
tail -2 gpurun_out/gputest_h.log
timeout -k 10 400 python -u tools/sweep_modes.py --modes default --reps 7 \
  --sizes 28224,29792,31360,32928,34496,36064,37632,50176,53312,56448,59584,62720,65856 > gpurun_out/sweep_h.txt 2>&1
cut -c1-100 gpurun_out/sweep_h.txt
timeout -k 10 400 python -u bench.py > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err
tail -c 600 gpurun_out/bench_h.json
