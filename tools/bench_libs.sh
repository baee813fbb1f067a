#!/bin/bash
# One bench line per library (WCG_LIB), C2 by default: tools/bench_libs.sh OUTDIR [bench args --] lib...
OUT=$1; shift
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end"
if [ "$1" == "--args" ]; then ARGS=$2; shift 2; fi
mkdir -p "$OUT"
for L in "$@"; do
  tag=$(basename "${L:-default}" .so)
  WCG_LIB=$L timeout -k 10 180 python3 bench.py $ARGS > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
  python3 -c "
import json,sys
d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1])
print('$tag', d['value'], d['unit'], 'ms/step', d['ms_per_step'], d['phase_ms_avg'], 'ok', d.get('verified_vs_oracle'))"
done
