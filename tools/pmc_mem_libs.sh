#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (each its own run) of the kernels matching KRE, per library:
# tools/pmc_mem_libs.sh OUTDIR KRE lib...  (then tools/pmc_summary.py OUTDIR/<lib>)
export TMPDIR=/tmp
OUT=$1; KRE=$2; shift 2
mkdir -p "$OUT"
for L in "$@"; do
  tag=$(basename "$L" .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    WCG_LIB=$L timeout -s KILL 60 rocprofv3 --pmc $c --kernel-include-regex "$KRE" --output-format csv -d "$OUT/$tag/$c" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-end-to-end > "$OUT/$tag.$c.log" 2>&1 || exit $?
  done
  python3 tools/pmc_summary.py "$OUT/$tag" > "$OUT/$tag.txt"
  cat "$OUT/$tag.txt"
done
