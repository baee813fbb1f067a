#!/bin/bash
# PMC passes (each its own run, --pmc only with kernel filtering; no sys/runtime trace) over a
# short bench run (the last pass: MFMA instruction and busy counters, expected 0 on every kernel
# of this path).  Usage: tools/prof_pmc.sh OUTDIR KERNEL_REGEX [bench args...]
export TMPDIR=/tmp
OUT=$1; KRE=$2; shift 2
passes=(
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE"
 "FETCH_SIZE"
 "WRITE_SIZE"
 "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU SQ_WAVES"
)
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p --kernel-include-regex "$KRE" --output-format csv -d "$OUT/pass$i" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-end-to-end "$@" || exit $?
done
