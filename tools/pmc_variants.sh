#!/bin/bash
# Two SQ counter passes on k_map for each library given (""=default build), then a bench line per
# library.  Usage: [BENCH_ARGS='--workload ...'] tools/pmc_variants.sh OUTDIR lib...
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE"
for L in "$@"; do
  tag=$(basename "${L:-default}" .so)
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    WCG_LIB=$L timeout -s KILL 60 rocprofv3 --pmc $P --kernel-include-regex k_map --output-format csv -d "$OUT/$tag/p$i" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-end-to-end $BENCH_ARGS > "$OUT/$tag.p$i.log" 2>&1 || exit $?
  done
  WCG_LIB=$L timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end $BENCH_ARGS > "$OUT/$tag.bench.json" 2> "$OUT/$tag.bench.err" || exit $?
  python3 tools/pmc_summary.py "$OUT/$tag" > "$OUT/$tag.pmc.txt"
done
