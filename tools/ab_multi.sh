#!/bin/bash
# C4 bench line of the default library and several variants, in rounds
# (run from the repo root via gpurun):
#   VARIANTS="lodestar_amd/libbgv_v1.so lodestar_amd/libbgv_v2.so" ROUNDS=2 bash tools/ab_multi.sh
# -> gpurun_out/abm/<round>_<name>.json
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abm
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 200 python3 bench.py --no-c2 --no-cpu --steps 10 > gpurun_out/abm/${r}_default.json 2> gpurun_out/abm/${r}_default.log
  for v in $VARIANTS; do
    n=$(basename $v .so)
    BGV_LIB=$v timeout -k 10 200 python3 bench.py --no-c2 --no-cpu --steps 10 > gpurun_out/abm/${r}_$n.json 2> gpurun_out/abm/${r}_$n.log
  done
done
