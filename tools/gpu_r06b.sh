#!/bin/bash
# r06: batches in flight per GPU (tools/overlap_probe.py) at C4, C4/8 and one epoch, 2 and 3 contexts
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
out=gpurun_out/overlap_sizes.txt
: > $out
for spec in "1024 2" "1024 3" "128 2" "128 3" "128 4" "32 2" "32 4"; do
  set -- $spec
  echo "blocks=$1 ctx=$2" >> $out
  timeout -k 10 200 python -u tools/overlap_probe.py --blocks $1 --ctx $2 --steps 8 >> $out 2>&1 || exit $?
done
grep -v "^\[" $out
