#!/bin/bash
# r06: in-flight variants around the C4/8 shard: two-lane Miller and one-lane
# clearing together, at 64 / 96 / 128 / 160 blocks, four batches in flight
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06r
probe() {
  local b=$1 tag=$2; shift 2
  echo "blocks=$b variant=$tag" >> gpurun_out/r06r/probe.txt
  timeout -k 10 240 python -u tools/overlap_probe.py --blocks $b --ctx 4 --steps 12 "$@" >> gpurun_out/r06r/probe.txt 2>&1
}
for r in 1 2; do
  for b in 128 64 96 160; do
    probe $b default && probe $b duo --cfg miller=2 && probe $b clear1 --cfg clear_lanes=1 \
    && probe $b duo_clear1 --cfg miller=2 --cfg clear_lanes=1 || { echo "probe failed"; tail -5 gpurun_out/r06r/probe.txt; exit 1; }
  done
done
python - <<'PY'
import json, collections
rows = collections.defaultdict(list); cur = None
for line in open("gpurun_out/r06r/probe.txt"):
    if line.startswith("blocks="): cur = line.strip(); continue
    if line.startswith("{"):
        j = json.loads(line)
        rows[cur].append(j["ms_per_batch"])
for k, v in rows.items(): print(k, "seq", v[0::2], "inflight", v[1::2])
PY
