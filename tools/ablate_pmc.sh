#!/bin/bash
# Instruction mix of k_map per ablation level (WCG_MAP_ABLATE, see wcg_map.h): one PMC pass each.
# Usage: tools/ablate_pmc.sh OUTDIR
export TMPDIR=/tmp
OUT=$1
for A in ${ABLATIONS:-5 4 1 2 3 0}; do
  WCG_MAP_ABLATE=$A rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    --kernel-include-regex k_map --output-format csv -d "$OUT/abl$A" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify || exit $?
done
