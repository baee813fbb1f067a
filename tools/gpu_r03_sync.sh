#!/bin/bash
# round 3: GPU suite at the working tree; C2 step: device-sized reduce vs exact, spin vs blocking
# sync, k_map wait-first variant; C2 kernel trace
export TMPDIR=/tmp
A="--steps 30 --warmup 5 --no-cpu-baseline --no-end-to-end"
one() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['value'], d['ms_per_step'], d['phase_ms_avg'], d.get('verified_vs_oracle'))" "$1" "$2"; }
export -f one
tools/gpu_steps.sh \
 "400|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1" \
 "300|for r in 1 2; do for v in default spin exact; do e=; [ \$v = spin ] && e=WCG_SPIN_SYNC=1; [ \$v = exact ] && e=WCG_EXACT_REDUCE=1; env \$e python3 bench.py $A > gpurun_out/b_\$v.json 2>/dev/null || exit 1; one gpurun_out/b_\$v.json \$v >> gpurun_out/sync.txt; done; done" \
 "200|tools/bench_libs.sh gpurun_out/wf build/var/libwcg_waitfirst.so '' build/var/libwcg_waitfirst.so '' > gpurun_out/waitfirst.txt 2>&1" \
 "150|tools/prof_trace.sh gpurun_out/trace_c2 > gpurun_out/trace_c2.log 2>&1"
