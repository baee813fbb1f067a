#!/bin/bash
for spec in "default|" "evict2|build/libwcg_evict.so|2" "evict4|build/libwcg_evict.so|4" "evict8|build/libwcg_evict.so|8"; do
  IFS='|' read tag lib em <<< "$spec"
  WCG_LIB=$lib WCG_EVICT_MIN=${em:-2} timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end > gpurun_out/ev_$tag.json 2>gpurun_out/ev_$tag.err || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['phase_ms_avg'], d['verified_vs_oracle'], d['stats']['lds_hits']/d['stats']['tokens'])" gpurun_out/ev_$tag.json $tag
done
