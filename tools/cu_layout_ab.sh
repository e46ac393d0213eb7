#!/bin/bash
# Bulk (cu_split -8) and priority (cu_split 8) contexts under the reserved-CU
# layouts of variant libraries, against the full chip (r05: the BGV_CU_RESERVE_LAYOUT
# knob these were built with is gone; tools/cu_mask_probe.hip showed why its
# spread layouts were wrong: they put every reserved CU on one XCC).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/cu_layout.jsonl
timeout -k 10 300 python3 -u tools/sweep_modes.py --sizes ${SIZES:-98,12544,100352} --modes default,bulk_cu8,prio_cu8 --reps 5 | sed 's/^/{"lib": "default", "row": /; s/$/}/' >> gpurun_out/cu_layout.jsonl
for L in ${LIBS:-libbgv_l1.so libbgv_l2.so}; do
  BGV_LIB=lodestar_amd/$L timeout -k 10 300 python3 -u tools/sweep_modes.py --sizes ${SIZES:-98,12544,100352} --modes bulk_cu8,prio_cu8 --reps 5 | sed "s/^/{\"lib\": \"$L\", \"row\": /; s/\$/}/" >> gpurun_out/cu_layout.jsonl
done
