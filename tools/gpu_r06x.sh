#!/bin/bash
# r06: the priority call's latency (one set, and one 98-set block) beside 0-3
# bulk contexts verifying C4 batches at once, with (cu 32) and without (cu 0)
# the CU split (tools/reserved_pool_probe.py)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06x
rm -f gpurun_out/r06x/probe3.txt
for spec in 1:32:1 2:32:1 3:32:1 1:0:1 3:0:1 3:32:98; do
  IFS=: read c u k <<< "$spec"
  timeout -k 10 300 python -u tools/reserved_pool_probe.py --ctx $c --cu $u --prio-sets $k --steps 6 >> gpurun_out/r06x/probe3.txt 2>> gpurun_out/r06x/probe3.log || { echo "failed $spec"; grep -v amdgpu.ids gpurun_out/r06x/probe3.log | tail -5; exit 1; }
done
cat gpurun_out/r06x/probe3.txt
