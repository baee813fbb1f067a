#!/bin/bash
# k_map ablation timings (measurement only): WCG_MAP_ABLATE = 0 full, 1 tokenize only,
# 2 + key extraction/hash, 3 + LDS lookups (misses dropped)
for A in ${ABLATIONS:-0 1 2 3}; do
  WCG_MAP_ABLATE=$A python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-verify --no-end-to-end "$@" > /tmp/abl_$A.json || exit $?
  python3 - "$A" <<'PY'
import json, sys
d = json.loads(open(f"/tmp/abl_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], d["phase_ms_avg"], d.get("stats"))
PY
done
