#!/bin/bash
# round 3: k_rp occupancy experiment on C4 1 GiB (LDS buffer 96 vs 48 units, slices 4/8/16), C2 check
export TMPDIR=/tmp
C4="--steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end --workload c4_utf8_zipf_64gib --bytes 1073741824"
one() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['value'], d['ms_per_step'], d['phase_ms_avg'], d.get('verified_vs_oracle'))" "$1" "$2"; }
export -f one
tools/gpu_steps.sh \
 "100|python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-end-to-end > gpurun_out/c2.json 2>/dev/null && one gpurun_out/c2.json c2 >> gpurun_out/rp.txt" \
 "500|for v in 'd 4' 'd 8' 'q48 4' 'q48 8' 'q48 16'; do set -- \$v; L=; [ \$1 = q48 ] && L=build/var/libwcg_rpqb48.so; WCG_LIB=\$L WCG_RP_SLICES=\$2 python3 bench.py $C4 > gpurun_out/c4_\$1_\$2.json 2>/dev/null || exit 1; one gpurun_out/c4_\$1_\$2.json \"c4 \$1 slices \$2\" >> gpurun_out/rp.txt; done"
