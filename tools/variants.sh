#!/bin/bash
# Bench the default libwcg and variant builds (build/libwcg_*.so, via WCG_LIB) back to back.
# Usage: tools/variants.sh OUT_PREFIX [lib ...]; extra bench args in $BENCH_ARGS
OUT=$1; shift
for L in "" "$@"; do
  tag=$(basename "${L:-default}" .so)
  extra=$BENCH_ARGS; case "$tag" in *nowait*|*diag*) extra="$extra --no-verify";; esac
  WCG_LIB=$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end $extra \
    > "${OUT}_${tag}.jsonl" 2> "${OUT}_${tag}.err" || { echo "variant $tag rc=$?"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['phase_ms_avg'], d['verified_vs_oracle'])" "${OUT}_${tag}.jsonl" "$tag"
done
