#!/bin/bash
# Instruction mix / stall counters of k_map per ablation level (WCG_MAP_ABLATE, see wcg_map.h):
# two PMC passes each.  Usage: tools/ablate_pmc.sh OUTDIR
export TMPDIR=/tmp
OUT=$1
for A in ${ABLATIONS:-5 4 1 2 3 0}; do
  WCG_MAP_ABLATE=$A timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    --kernel-include-regex k_map --output-format csv -d "$OUT/abl$A/p1" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-end-to-end > /dev/null || exit $?
  WCG_MAP_ABLATE=$A timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE \
    --kernel-include-regex k_map --output-format csv -d "$OUT/abl$A/p2" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-end-to-end > /dev/null || exit $?
done
