#!/bin/bash
# r06: GPU suite + default bench (tools/gpu_round.sh), then the N = 4 strong-shard
# rehearsal on one GPU (gloo, 4 batches in flight per rank)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TEST_TIMEOUT=700 BENCH_ARGS="--steps 20" bash tools/gpu_round.sh || exit $?
BGV_BENCH_REHEARSE=1 timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 8 > gpurun_out/rehearse4.json 2> gpurun_out/rehearse4.log
rc=$?
tail -c 600 gpurun_out/rehearse4.json
exit $rc
