#!/bin/bash
# r06: the C4/2 shard (50,176 sets, N = 2) and its neighbours, three in flight:
# the size-picked latency-mode pipeline against the bulk one (split=0, two pairs
# per item over lines, as C4)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06ag
probe() {
  local b=$1 tag=$2; shift 2
  echo "blocks=$b variant=$tag" >> gpurun_out/r06ag/probe.txt
  timeout -k 10 240 python -u tools/overlap_probe.py --blocks $b --ctx 3 --steps 8 "$@" 2>/dev/null | grep mode >> gpurun_out/r06ag/probe.txt
}
for r in 1 2; do
  for b in 512 384; do
    probe $b default && probe $b bulk2 --cfg split=0 --cfg pairs=2 && probe $b bulk1 --cfg split=0 || { echo failed; exit 1; }
  done
done
python - <<'PY'
import json, collections
rows = collections.defaultdict(list); cur = None
for line in open("gpurun_out/r06ag/probe.txt"):
    if line.startswith("blocks="): cur = line.strip(); continue
    if line.startswith("{"): rows[cur].append(json.loads(line)["ms_per_batch"])
for k, v in rows.items(): print(k, "seq", v[0::2], "inflight", v[1::2])
PY
