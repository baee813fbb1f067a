#!/bin/bash
# round 3: GPU suite, C2 bench (k_map timed by hipExtLaunchKernel events), k_agg flush ablation
# (wrong counts: unverified), C4 1 GiB bench
export TMPDIR=/tmp
one() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['phase_ms_avg'], d.get('verified_vs_oracle'))" "$1" "$2"; }
export -f one
tools/gpu_steps.sh \
 "400|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1" \
 "300|for r in 1 2; do for v in default aggab3; do L=; [ \$v = aggab3 ] && L=build/var/libwcg_aggab3.so; X=; [ \$v = aggab3 ] && X=--no-verify; WCG_LIB=\$L python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-end-to-end \$X > gpurun_out/c2_\$v.json 2>/dev/null || exit 1; one gpurun_out/c2_\$v.json \$v >> gpurun_out/next.txt; done; done" \
 "200|python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end --workload c4_utf8_zipf_64gib --bytes 1073741824 > gpurun_out/c4.json 2>/dev/null && one gpurun_out/c4.json c4 >> gpurun_out/next.txt"
