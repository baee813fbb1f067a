#!/bin/bash
# round 3: AGG_DIRECT one-pass aggregation (256 buckets, records emitted) - GPU suite, C2 A/B against
# the round-2 design (WCG_AGG_DIRECT=0), C4 1 GiB
export TMPDIR=/tmp
one() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['phase_ms_avg'], d['stats']['global_ops'], d['stats']['emitted'], d.get('verified_vs_oracle'))" "$1" "$2"; }
export -f one
tools/gpu_steps.sh \
 "400|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1" \
 "300|for r in 1 2; do for v in 1 0; do WCG_AGG_DIRECT=\$v python3 bench.py --steps 30 --warmup 15 --no-cpu-baseline --no-end-to-end > gpurun_out/c2_d\$v.json 2>gpurun_out/c2_d\$v.err || exit 1; one gpurun_out/c2_d\$v.json direct\$v >> gpurun_out/direct.txt; done; done" \
 "200|python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end --workload c4_utf8_zipf_64gib --bytes 1073741824 > gpurun_out/c4.json 2>/dev/null && one gpurun_out/c4.json c4 >> gpurun_out/direct.txt" \
 "150|tools/prof_trace.sh gpurun_out/trace_c2 > gpurun_out/trace_c2.log 2>&1"
