#!/usr/bin/env python3
"""Per-kernel mean duration (us) from a rocprofv3 kernel-trace CSV directory."""
import csv
import glob
import sys
from collections import defaultdict

d = defaultdict(list)
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items(), key=lambda x: -sum(x[1])):
    print(f"{k:70s} n={len(v):4d} avg_us={sum(v) / len(v):9.2f} total_us={sum(v):10.1f}")
