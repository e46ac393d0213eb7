#!/bin/bash
# r06: batches in flight from one vs two / three processes on one GPU (each
# process has its own four HIP hardware queues), tools/proc_probe.py
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06t
p() { timeout -k 10 300 python -u tools/proc_probe.py "$@" >> gpurun_out/r06t/probe.txt 2>> gpurun_out/r06t/err.txt; }
for r in 1 2; do
  p --procs 1 --ctx 4 --blocks 128 && p --procs 2 --ctx 2 --blocks 128 && p --procs 2 --ctx 3 --blocks 128 \
  && p --procs 2 --ctx 4 --blocks 128 && p --procs 4 --ctx 1 --blocks 128 \
  && p --procs 1 --ctx 3 --blocks 1024 --steps 8 && p --procs 2 --ctx 2 --blocks 1024 --steps 8 || { echo failed; tail -20 gpurun_out/r06t/err.txt; exit 1; }
done
cat gpurun_out/r06t/probe.txt
