#!/bin/bash
# kernel trace + stats of a short C4 1 GiB bench per library: tools/prof_libs.sh OUTDIR lib...
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$OUT"
for L in "$@"; do
  tag=$(basename "$L" .so)
  WCG_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$tag" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-verify --no-end-to-end \
    --workload c4_utf8_zipf_64gib --bytes 1073741824 > "$OUT/$tag.log" 2>&1 || exit $?
done
