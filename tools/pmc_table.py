#!/usr/bin/env python3
"""Per-variant table of the k_map SQ counters and bench line written by tools/pmc_variants.sh."""
import csv, glob, json, os, sys
from collections import defaultdict
base = sys.argv[1]
for d in sorted(glob.glob(f"{base}/*/")):
    t = os.path.basename(d.rstrip("/"))
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    v = {c: sum(x.values()) / len(x) for c, x in vals.items()}
    try:
        b = json.loads(open(f"{base}/{t}.bench.json").read().strip().splitlines()[-1])
        bl = f"{b['value']:8.1f} GB/s map {b['phase_ms_avg']['map']:.4f} agg {b['phase_ms_avg']['agg']:.4f} hit {b['stats']['lds_hits'] / b['stats']['tokens']:.3f} ok {b['verified_vs_oracle']}"
    except Exception as e:
        bl = f"bench: {e}"
    print(f"{t:22s} {bl}")
    if "SQ_WAVE_CYCLES" in v:
        W = v["SQ_WAVE_CYCLES"]
        print(f"    VALU {v.get('SQ_INSTS_VALU', 0):.3e} SALU {v.get('SQ_INSTS_SALU', 0):.3e} LDS {v.get('SQ_INSTS_LDS', 0):.3e} "
              f"BR {v.get('SQ_INSTS_BRANCH', 0):.3e} | wait {v['SQ_WAIT_ANY'] / W:.2f} stall {v['SQ_WAIT_INST_ANY'] / W:.2f} "
              f"active {v['SQ_ACTIVE_INST_ANY'] / W:.2f} | LDS conflicts {v.get('SQ_LDS_BANK_CONFLICT', 0) / max(v.get('SQ_LDS_IDX_ACTIVE', 1), 1):.2f}")
