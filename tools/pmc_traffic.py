#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from tools/prof_pmc.sh passes -> profiles/traffic_latest.json
(read by bench.py for roofline.traffic).

bytes = FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024: rocprofv3 reports both in KiB, and on gfx950
FETCH_SIZE counts half the bytes of wide streaming reads (MI355X_MICROARCH.md, HBM/rocprofv3
section).  WRITE_SIZE is exact for 16-byte-per-lane streaming stores; k_map's miss-log stores are
8 bytes per lane, so its write figure is the L2's memory-side count, not a byte-exact one.

Usage: pmc_traffic.py PMC_DIR KERNEL_SUBSTRING WORKLOAD BYTES_PER_GPU [OUT_JSON]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(root, kernel):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel in row.get("Kernel_Name", ""):
                vals[row["Counter_Name"]][(f, row.get("Dispatch_Id"))] += float(row["Counter_Value"])
    return {c: sum(d.values()) / len(d) for c, d in vals.items() if d}


def main():
    root, kernel, workload, nbytes = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "traffic_latest.json")
    c = per_dispatch(root, kernel)
    fetch = c["FETCH_SIZE"] * 1024 * 2
    write = c["WRITE_SIZE"] * 1024
    res = {"kernel": kernel, "workload": workload, "bytes_per_gpu": nbytes,
           "hbm_bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch), "write_bytes": round(write),
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({root}), mean per dispatch; "
                     "FETCH_SIZE x2 gfx950 correction"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
