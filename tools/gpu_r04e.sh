#!/bin/bash
# shard fault tests at the view-Miller sizes; 4-rank strong-shard rehearsal of the N>1 bench on one GPU
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_concurrent.py 4 3 1 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_shards.log 2>&1 || { tail -30 gpurun_out/gputest_shards.log; exit 1; }
tail -8 gpurun_out/gputest_shards.log
BGV_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --steps 3 --warmup 1 > gpurun_out/rehearse4.json 2> gpurun_out/rehearse4.log || { tail -30 gpurun_out/rehearse4.log; exit 1; }
cut -c1-1500 gpurun_out/rehearse4.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_stages_kv9.log 2>&1 || { tail -30 gpurun_out/gputest_stages_kv9.log; exit 1; }
tail -2 gpurun_out/gputest_stages_kv9.log
timeout -k 10 400 python -u tools/sweep_modes.py --sizes 1176,1960,3136,4704 --modes default,kv9 --reps 9 > gpurun_out/sweep_kv9.txt 2>&1
cut -c1-120 gpurun_out/sweep_kv9.txt
