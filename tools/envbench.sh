#!/bin/bash
# tools-style: one bench line with extra env: envbench.sh OUT TAG LIB [VAR=VAL ...]
OUT=$1; TAG=$2; L=$3; shift 3
mkdir -p $OUT
env WCG_LIB=$L "$@" timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end > $OUT/$TAG.json 2> $OUT/$TAG.err || exit $?
python3 -c "
import json
d=json.loads(open('$OUT/$TAG.json').read().strip().splitlines()[-1]); s=d['stats']
print('$TAG', d['value'], 'ms/step', d['ms_per_step'], d['phase_ms_avg'], 'hit', round(s['lds_hits']/s['tokens'],4), 'ok', d.get('verified_vs_oracle'))"
