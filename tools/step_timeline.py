#!/usr/bin/env python3
"""One step's kernels from a rocprofv3 kernel-trace CSV directory: start offset, duration and the
gap before each kernel, from a k_map launch to the next (the second-to-last step by default), plus
the k_map launch statistics.  Usage: step_timeline.py <trace dir> [steps back from the end]."""
import csv
import glob
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
maps = [i for i, r in enumerate(rows) if "k_map<" in r[2]]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
if len(maps) < back + 1:
    sys.exit("not enough k_map launches in the trace")
d = [(rows[i][1] - rows[i][0]) / 1e3 for i in maps]
print(f"k_map launches: {len(maps)}, mean {sum(d) / len(d):.1f} us, min {min(d):.1f}, max {max(d):.1f}")
a, b = maps[-back - 1], maps[-back]
t0 = rows[a][0]
prev_end = t0
print(f"one step's kernels (k_map launch {len(maps) - back} of {len(maps)}):")
for s, e, n in rows[a:b]:
    print(f"  {(s - t0) / 1e3:9.1f} us {(e - s) / 1e3:8.1f} us  gap {max(0, s - prev_end) / 1e3:6.1f}  {n[:80]}")
    prev_end = max(prev_end, e)
print(f"step (k_map start to next k_map start): {(rows[b][0] - t0) / 1e3:.1f} us")
