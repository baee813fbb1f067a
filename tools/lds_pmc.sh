#!/bin/bash
# LDS / wait counters of k_map (one PMC pass).  Usage: tools/lds_pmc.sh OUTDIR [variant.so]
export TMPDIR=/tmp
OUT=$1; L=$2
WCG_LIB=$L timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU \
  --kernel-include-regex k_map --output-format csv -d "$OUT/p1" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify > /dev/null || exit $?
WCG_LIB=$L timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_WR \
  --kernel-include-regex k_map --output-format csv -d "$OUT/p2" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify > /dev/null || exit $?
