#!/bin/bash
# r06: verifyOnMainThread single sets on a one-GPU pool (no CU split) beside
# three bulk contexts in flight, one priority call every 50 ms:
#   libbgv.so      streams as shipped (bulk hash/pubkey streams high, priority context = a bulk context)
#   libbgv_xprio   bulk streams all normal, the priority context's streams all high
#   libbgv_xprio2  bulk streams as shipped, the priority context's streams all high
# plus the bulk C4 bench leg of each build (no priority calls)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06y
rm -f gpurun_out/r06y/probe2.txt
for r in 1 2; do
  for lib in libbgv.so libbgv_xprio.so libbgv_xprio2.so; do
    echo -n "$lib " >> gpurun_out/r06y/probe2.txt
    BGV_LIB=$PWD/lodestar_amd/$lib timeout -k 10 300 python -u tools/reserved_pool_probe.py --ctx 3 --cu 0 --prio-sets 1 --steps 8 --gap-ms 50 >> gpurun_out/r06y/probe2.txt 2>> gpurun_out/r06y/probe2.log || { echo "failed"; grep -v amdgpu.ids gpurun_out/r06y/probe2.log | tail -5; exit 1; }
    BGV_LIB=$PWD/lodestar_amd/$lib timeout -k 10 300 python -u bench.py --no-c2 --no-cpu --steps 30 > gpurun_out/r06y/bench_${lib}_$r.json 2> gpurun_out/r06y/bench.log || exit 1
    python -c "import json; j=json.loads(open('gpurun_out/r06y/bench_${lib}_$r.json').read().strip().splitlines()[-1]); print('$lib bench', j['value'], j['ms_per_step'])" >> gpurun_out/r06y/probe2.txt
  done
done
cat gpurun_out/r06y/probe2.txt
