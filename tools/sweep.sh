# A/B sweep on the GPU box: each argument is "label ENV=VAL ..." ; runs bench.py (C4 only)
mkdir -p gpurun_out
for spec in "$@"; do
  set -- $spec; label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-c2 --no-cpu > gpurun_out/ab_$label.log 2>&1 || { echo "$label FAILED"; tail -5 gpurun_out/ab_$label.log; exit 1; }
  echo "$label $(python -c "import json;d=json.loads(open('gpurun_out/ab_$label.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],{k:v for k,v in d['stage_ms'].items() if v>0.5})")"
done
