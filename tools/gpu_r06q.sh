#!/bin/bash
# r06: pipeline variants of the C4/8 shard (12,544 sets) with four batches in
# flight (the N = 8 strong-scaling shard): the size-picked default was swept
# for a lone batch; in flight another variant may fill the chip better
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06q
probe() {
  local tag=$1; shift
  echo "variant=$tag" >> gpurun_out/r06q/probe.txt
  timeout -k 10 240 python -u tools/overlap_probe.py --blocks 128 --ctx 4 --steps 12 "$@" >> gpurun_out/r06q/probe.txt 2>&1
}
for r in 1 2; do
  probe default && probe duo --cfg miller=2 && probe kv3 --cfg miller_kv=3 && probe clear1 --cfg clear_lanes=1 \
  && probe msm2 --cfg msm=2 && probe bulkhash --cfg split=0 && probe c4pipe --cfg split=0 --cfg miller=1 --cfg pairs=2 --cfg msm=2 \
  && probe kv6 --cfg miller_kv=6 || { echo "probe failed"; tail -5 gpurun_out/r06q/probe.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r06q/probe.txt
