#!/bin/bash
# r06: full bench legs (latency configs, shard projection) with the Fp2 leaf in the Miller
# and latency units (default libbgv.so) against Karatsuba everywhere (libbgv_kara.so)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/fp2b
run() {
  local tag=$1 lib=$2; shift 2
  BGV_LIB=$PWD/lodestar_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu --steps 20 "$@" > gpurun_out/fp2b/$tag.json 2> gpurun_out/fp2b/$tag.log || return $?
  python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
j = json.loads(open(f"gpurun_out/fp2b/{t}.json").read().strip().splitlines()[-1])
sp = j["strong_shard_projection"]
print(t, j["value"], j["ms_per_step"], "one", j["one_in_flight"]["ms_p50"], "c2", j["c2_gossip_latency_ms"]["p50"], "single", j["single_set_latency_ms"]["p50"],
      "epoch", j["c4_epoch_slice"]["p50_ms"], j["c4_epoch_slice"].get("ms_per_batch_in_flight"), "c4/8", sp["c4_over_8"]["ms"], sp["c4_over_8"].get("ms_in_flight"),
      "c4/4", sp["c4_over_4"]["ms"], "c4/2", sp["c4_over_2"]["ms"])
PY
}
run M1 libbgv.so && run K1 libbgv_kara.so && run M2 libbgv.so && run K2 libbgv_kara.so
