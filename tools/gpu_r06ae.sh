#!/bin/bash
# r06: the multi-device pools' device 0 (three cu_split -32 bulk contexts + a +32
# priority context) under load, three separate processes: any queue-scratch failure?
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06ae
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/reserved_pool_probe.py --ctx 3 --cu 32 --steps 8 --gap-ms 20 >> gpurun_out/r06ae/probe.txt 2>> gpurun_out/r06ae/probe.log
  echo "run $r exit $?" >> gpurun_out/r06ae/probe.txt
done
grep -c OUT_OF_RESOURCES gpurun_out/r06ae/probe.log || true
cat gpurun_out/r06ae/probe.txt
