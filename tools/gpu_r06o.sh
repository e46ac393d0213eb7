#!/bin/bash
# r06: deeper in-flight pools for the strong-scaling shards (C4/8 = 128 blocks,
# C4/32 = 32 blocks): 4 / 5 / 6 / 8 contexts on one GPU (tools/overlap_probe.py)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06o
for spec in 128:4 128:6 128:8 128:5 32:6 32:8 256:4 256:6; do
  b=${spec%%:*}; c=${spec#*:}
  echo "blocks=$b ctx=$c" >> gpurun_out/r06o/probe.txt
  timeout -k 10 240 python -u tools/overlap_probe.py --blocks $b --ctx $c --steps 12 >> gpurun_out/r06o/probe.txt 2>&1 || { echo "probe $spec failed rc=$?"; tail -5 gpurun_out/r06o/probe.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r06o/probe.txt
