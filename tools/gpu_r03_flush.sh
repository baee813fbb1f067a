#!/bin/bash
# round 3: k_agg flush with its first global probes batched (default build) vs the previous build
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300|tools/bench_libs.sh gpurun_out/fl --args '--steps 30 --warmup 15 --no-cpu-baseline --no-end-to-end' build/var/libwcg_kr4.so '' build/var/libwcg_kr4.so '' > gpurun_out/flush.txt 2>&1" \
 "400|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1"
