#!/bin/bash
# r06: in-flight-aware pipeline choice (bulk pipeline from 32,000 sets when other
# batches of the process are in flight on the device): tests, the C4/2 probe,
# the default bench line
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06ah
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_large.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r06ah/tests.log 2>&1 || { tail -20 gpurun_out/r06ah/tests.log; exit 1; }
tail -1 gpurun_out/r06ah/tests.log
for b in 512 384; do
  echo "blocks=$b" >> gpurun_out/r06ah/probe.txt
  timeout -k 10 240 python -u tools/overlap_probe.py --blocks $b --ctx 3 --steps 8 2>/dev/null | grep mode >> gpurun_out/r06ah/probe.txt || exit 1
done
cat gpurun_out/r06ah/probe.txt
timeout -k 10 500 python -u bench.py > gpurun_out/r06ah/bench_default.json 2> gpurun_out/r06ah/bench_default.log || { tail -5 gpurun_out/r06ah/bench_default.log; exit 1; }
python -c "import json; j=json.loads(open('gpurun_out/r06ah/bench_default.json').read().strip().splitlines()[-1]); print(j['value'], j['ms_per_step'], j['verified']); print(json.dumps(j['strong_shard_projection'])); print(j['reserved_device'])"
