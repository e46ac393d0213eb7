#!/bin/bash
# three rounds of a C4 A/B of LIBS (tools/ab_lib.sh)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out; rm -f gpurun_out/ab.txt
for rep in ${ROUNDS:-1 2 3}; do LIBS="$LIBS" SIZES=${SIZES:-100352} bash tools/ab_lib.sh; done
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
for line in open("gpurun_out/ab.txt"):
    lib, js = line.split(" ", 1)
    d = json.loads(js)
    r[(lib, d["sets"])].append(d["ms"])
for k, v in sorted(r.items()):
    print(k, [round(x, 2) for x in v], "median", sorted(v)[len(v) // 2])
PY
