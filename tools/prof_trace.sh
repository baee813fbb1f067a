#!/bin/bash
# kernel-trace + stats of a short bench run; summary copied to profiles/ by the caller
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_trace}
shift
rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-verify --no-end-to-end "$@"
