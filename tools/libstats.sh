#!/bin/bash
# per-library kernel averages (us) and bench phases from a prof_libs.sh output directory
for d in "$1"/*/; do echo "$d"; python3 - "$d" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] + 'run_kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv) > 2 else 14]:
    print('  %-44s %6s %9.1f' % (r['Name'][:44], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
for f in "$1"/*.log; do python3 - "$f" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['phase_ms_avg'])
PY
done
