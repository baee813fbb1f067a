#!/bin/bash
# kernel trace of the default C2 bench line (30 timed steps after 15 warm-up: the trace's timed
# launches compare directly with the line's HIP-event average), then C4 at full size (64 GiB, one job)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "240|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_c2_default -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end > gpurun_out/bench_traced.json 2> gpurun_out/bench_traced.err" \
  "900|python -u tools/c4_full.py --jobs 2 --out gpurun_out/c4_full.json > gpurun_out/c4_full.log 2>&1"
