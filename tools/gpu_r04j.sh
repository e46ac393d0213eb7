#!/bin/bash
# split threshold at 59,000 sets: full GPU suite, sweep at the edge, default bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_j.log 2>&1 || { tail -30 gpurun_out/gputest_j.log; exit 1; }
tail -2 gpurun_out/gputest_j.log
timeout -k 10 400 python -u tools/sweep_modes.py --modes default --reps 7 \
  --sizes 56448,58016,59584,61152,62720 > gpurun_out/sweep_j.txt 2>&1
cut -c1-100 gpurun_out/sweep_j.txt
timeout -k 10 400 python -u bench.py > gpurun_out/bench_j.json 2> gpurun_out/bench_j.err
tail -c 600 gpurun_out/bench_j.json
