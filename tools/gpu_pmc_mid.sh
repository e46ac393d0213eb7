#!/bin/bash
# Per-kernel counters of mid-size batches (tools/size_trace.py): one SQ pass,
# then FETCH_SIZE and WRITE_SIZE passes, each its own rocprofv3 run.
# Summaries land in gpurun_out/pmc_mid_*.txt
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_mid
rm -rf $OUT && mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $OUT/sq -o run --output-format csv -- python3 tools/size_trace.py --sizes ${SIZES:-12544} --reps 1 > $OUT/sq.log 2>&1
python3 tools/pmc_table.py $(find $OUT/sq -name "*counter_collection.csv" | head -1) > gpurun_out/pmc_mid_summary.txt || true
if [ "${TRAFFIC:-0}" = 1 ]; then
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/size_trace.py --sizes ${SIZES:-12544} --reps 1 > $OUT/fetch.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 tools/size_trace.py --sizes ${SIZES:-12544} --reps 1 > $OUT/write.log 2>&1
  python3 tools/pmc_table.py $(find $OUT/fetch -name "*counter_collection.csv" | head -1) > gpurun_out/pmc_mid_fetch.txt || true
  python3 tools/pmc_table.py $(find $OUT/write -name "*counter_collection.csv" | head -1) > gpurun_out/pmc_mid_write.txt || true
fi
cat gpurun_out/pmc_mid_summary.txt
