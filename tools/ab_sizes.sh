#!/bin/bash
# On-device bgv_verify medians of the default library and a variant at chosen
# sizes, alternating (run from the repo root via gpurun):
#   VARIANT=lodestar_amd/libbgv_x.so SIZES=12544 ROUNDS=3 bash tools/ab_sizes.sh
# -> gpurun_out/ab_sizes.jsonl ({"lib": ..., "row": sweep_modes row})
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab_sizes.jsonl
for r in $(seq 1 ${ROUNDS:-3}); do
  timeout -k 10 300 python3 -u tools/sweep_modes.py --sizes ${SIZES:-12544} --modes ${MODES:-default} --reps 7 | sed 's/^/{"lib": "default", "row": /; s/$/}/' >> gpurun_out/ab_sizes.jsonl
  BGV_LIB=${VARIANT:-lodestar_amd/libbgv_x.so} timeout -k 10 300 python3 -u tools/sweep_modes.py --sizes ${SIZES:-12544} --modes ${MODES:-default} --reps 7 | sed 's/^/{"lib": "variant", "row": /; s/$/}/' >> gpurun_out/ab_sizes.jsonl
done
