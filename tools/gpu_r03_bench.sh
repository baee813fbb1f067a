#!/bin/bash
# round 3: GPU suite + C2 bench lines (timing mode 3) + C4 1 GiB + C2 kernel trace
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "400|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1" \
 "200|for r in 1 2 3; do python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-end-to-end > gpurun_out/bench_c2_\$r.json 2> gpurun_out/bench_c2_\$r.err || exit 1; done" \
 "200|python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end --workload c4_utf8_zipf_64gib --bytes 1073741824 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err" \
 "150|tools/prof_trace.sh gpurun_out/trace_c2 > gpurun_out/trace_c2.log 2>&1"
