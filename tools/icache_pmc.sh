#!/bin/bash
# Instruction-cache counters of k_map for the default build and a variant library (WCG_LIB).
# Usage: tools/icache_pmc.sh OUTDIR [variant.so ...]
export TMPDIR=/tmp
OUT=$1; shift
i=0
for L in "" "$@"; do
  i=$((i+1))
  WCG_LIB=$L timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --kernel-include-regex k_map --output-format csv -d "$OUT/v$i" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-end-to-end > /dev/null || exit $?
done
