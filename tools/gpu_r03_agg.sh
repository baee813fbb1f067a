#!/bin/bash
# round 3: k_agg probe-group variants (C2, C4 1 GiB), k_map phase stamps and ablation levels at HEAD
export TMPDIR=/tmp
A="--steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end --no-verify"
tools/gpu_steps.sh \
 "250|tools/bench_libs.sh gpurun_out/agg build/var/libwcg_agg2.so build/var/libwcg_agg4.so build/var/libwcg_agg2.so build/var/libwcg_agg4.so > gpurun_out/agg_c2.txt 2>&1" \
 "300|tools/bench_libs.sh gpurun_out/aggc4 --args '--steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end --workload c4_utf8_zipf_64gib --bytes 1073741824' build/var/libwcg_agg2.so build/var/libwcg_agg4.so > gpurun_out/agg_c4.txt 2>&1" \
 "120|WCG_LIB=build/var/libwcg_stamps.so python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end --no-verify > gpurun_out/stamps.json 2> gpurun_out/stamps.err" \
 "400|for L in 5 4 1 2 3 0; do WCG_MAP_ABLATE=\$L python3 bench.py $A > gpurun_out/abl_\$L.json 2>/dev/null || exit 1; python3 -c \"import json;d=json.loads(open('gpurun_out/abl_\$L.json').read().strip().splitlines()[-1]);print('ablate', \$L, d['phase_ms_avg'])\" >> gpurun_out/ablate.txt; done"
