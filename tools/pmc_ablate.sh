#!/bin/bash
# VALU/SALU/LDS instruction counts of k_map per ablation level (WCG_MAP_ABLATE: 5 loads only,
# 4 + letter masks, 1 + start list, 0 full) for one library.  Usage: tools/pmc_ablate.sh OUTDIR [lib]
export TMPDIR=/tmp
OUT=$1; L=$2
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH"
for A in 5 4 1 0; do
  WCG_LIB=$L WCG_MAP_ABLATE=$A timeout -s KILL 60 rocprofv3 --pmc $P1 --kernel-include-regex k_map --output-format csv -d "$OUT/abl$A" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-end-to-end > "$OUT/abl$A.log" 2>&1 || exit $?
  echo "== ablate $A"; python3 tools/pmc_summary.py "$OUT/abl$A" | grep -E "INSTS|WAVE_CYCLES"
done
