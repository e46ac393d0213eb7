#!/bin/bash
# r06 round profile on the GPU box (run from the repo root via gpurun):
#   default bench line; rocprofv3 kernel trace + stats of the C4-only command
#   (every k_* dispatch belongs to a C4 batch, 3 in flight, so the per-kernel
#   averages compare with the bench's in-flight stage times); PMC passes
#   (FETCH_SIZE, WRITE_SIZE, SQ) over one C4 batch with one in flight (rocprofv3
#   serialises dispatches under --pmc, so the per-launch bytes do not depend on it).
# Every GPU step has its own time limit and the steps are chained with &&.
set -e
TAG=${TAG:-r06}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 python3 bench.py --steps 20 > $OUT/bench_default.json 2> $OUT/bench_default.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_c4 -o run --output-format csv -- python3 bench.py --no-c2 --no-cpu --steps 20 > $OUT/bench_c4_traced.json 2> $OUT/bench_traced_c4.log
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-c2 --no-cpu --inflight 1 > $OUT/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-c2 --no-cpu --inflight 1 > $OUT/write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $OUT/sq -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-c2 --no-cpu --inflight 1 > $OUT/sq.log 2>&1
find $OUT -name "*.csv" | sort
head -c 600 $OUT/bench_default.json
