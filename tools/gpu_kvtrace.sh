set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/trace_kv gpurun_out/pmc_kv
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/trace_kv -o run --output-format csv -- python3 tools/size_trace.py --sizes 3136,12544 --cfg '{"miller_kv": 3}' > gpurun_out/trace_kv.log 2>&1
python3 tools/size_trace.py --analyze $(find gpurun_out/trace_kv -name "*kernel_trace.csv" | head -1) > gpurun_out/timeline_kv.txt
grep -E "sets:|miller|hash_clear|k_pk|batch_final" gpurun_out/timeline_kv.txt | cut -c1-110
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY -d gpurun_out/pmc_kv -o run --output-format csv -- python3 tools/size_trace.py --sizes 12544 --reps 1 --cfg '{"miller_kv": 3}' > gpurun_out/pmc_kv.log 2>&1
python3 tools/pmc_table.py $(find gpurun_out/pmc_kv -name "*counter_collection.csv" | head -1) --kernels=k_miller_kv,k_miller_quad > gpurun_out/pmc_kv.txt
cat gpurun_out/pmc_kv.txt
