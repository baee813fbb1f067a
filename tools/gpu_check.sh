#!/bin/bash
# Standard GPU round trip: parity tests, one bench line, k_map ablation timings, and a bench line
# per variant library given as arguments (built under build/var/ by the caller).
# Usage (on the GPU box, via gpurun): tools/gpu_check.sh [variant.so ...]
specs=(
  "300|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1"
  "120|python bench.py --no-cpu-baseline > gpurun_out/bench.json 2>gpurun_out/bench.err"
)
[ -n "$ABLATIONS" ] && specs+=("200|ABLATIONS=\"$ABLATIONS\" tools/ablate.sh > gpurun_out/ablate.log 2>&1")
for v in "$@"; do
  specs+=("120|WCG_LIB=$v python bench.py --no-cpu-baseline > gpurun_out/bench_$(basename $v .so).json 2>&1")
done
tools/gpu_steps.sh "${specs[@]}"
