mkdir -p gpurun_out
for s in 0 1 2 4 5 0; do
  BGV_SCHED=$s timeout -k 10 120 python bench.py --no-c2 --no-cpu > gpurun_out/sched_$s.log 2>&1 || exit 1
  echo "sched=$s $(python -c "import json,sys;d=json.loads(open('gpurun_out/sched_$s.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['stage_ms'])")"
done
