#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (tools/prof_pmc.sh output): per kernel, mean per dispatch.
Dispatches are keyed by (pass file, dispatch id): every pass is its own run with its own ids, so a
counter collected in two passes (SQ_INSTS_VALU, SQ_WAVES) is averaged over both, not summed."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "?")
        acc[k][row["Counter_Name"]].append(((f, row.get("Dispatch_Id")), float(row["Counter_Value"])))
for k, cs in acc.items():
    print(k[:90])
    for c, vals in sorted(cs.items()):
        per = defaultdict(float)
        for d, v in vals:
            per[d] += v
        xs = list(per.values())
        print(f"   {c:28s} {sum(xs) / len(xs):16.4e}  (dispatches {len(xs)})")
