# Round profile collection on the GPU box (run from the repo root via gpurun):
#   default bench line; rocprofv3 kernel trace + stats of the default command
#   and of the C4-only command (every k_* dispatch is a C4 step, so the
#   per-kernel averages compare with the bench's stage times); PMC passes
#   (FETCH_SIZE, WRITE_SIZE, SQ utilisation) over one C4 step.
# Every GPU step has its own time limit and the steps are chained with &&.
set -e
TAG=${TAG:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py > $OUT/bench_traced.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_c4 -o run --output-format csv -- python3 bench.py --no-c2 --no-cpu > $OUT/bench_traced_c4.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-c2 --no-cpu > $OUT/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-c2 --no-cpu > $OUT/write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $OUT/sq -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-c2 --no-cpu > $OUT/sq.log 2>&1
find $OUT -name "*.csv" | sort
cat $OUT/bench_default.json
