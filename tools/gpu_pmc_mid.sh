#!/bin/bash
# SQ counters per kernel of mid-size batches (tools/size_trace.py) in one
# rocprofv3 --pmc pass; the summary lands in gpurun_out/pmc_mid_summary.txt
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_mid
rm -rf $OUT && mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $OUT -o run --output-format csv -- python3 tools/size_trace.py --sizes ${SIZES:-12544} --reps 1 > $OUT/run.log 2>&1
python3 tools/pmc_table.py $(find $OUT -name "*counter_collection.csv" | head -1) > gpurun_out/pmc_mid_summary.txt || true
cat gpurun_out/pmc_mid_summary.txt
