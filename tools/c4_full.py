#!/usr/bin/env python3
"""BASELINE config 4 at full size on one MI355X: 64 GiB of mixed-script UTF-8 (Zipf s = 0.9 over
a 5e7-word vocabulary, seed 44), resident in HBM, counted as ONE word-count job - 8 DoMap calls
(wcg_map_device, 8 GiB each; --call-gib 1: 64 calls; generator blocks end in '\\n', so every call
is a whole split) into one context sized for 5e7 keys, then DoReduce + Merge (wcg_reduce) - and the merged file checked
exactly against the input by the oracle's verifier (oracle/wc_oracle.c wco_verify_merged: every
input token decrements its line's count; all counts must end at 0, keys strictly ascending).

  python tools/c4_full.py [--gib 64] [--jobs 2] [--out gpurun_out/c4_full.json]

Prints progress lines while it generates (the 5e7-word generator takes ~1 min to build, the text
~3 min on 16 threads) and while it verifies.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mit-6.824-2015_amd"))
sys.path.insert(0, ROOT)


def log(*a):
    print(f"[c4_full {time.strftime('%H:%M:%S')}]", *a, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=64)
    ap.add_argument("--call-gib", type=int, default=8)
    ap.add_argument("--jobs", type=int, default=2, help="timed jobs (after one untimed)")
    ap.add_argument("--max-keys", type=int, default=50_000_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "c4_full.json"))
    ap.add_argument("--no-verify", action="store_true", help="diagnostics: skip the oracle's check")
    args = ap.parse_args()

    import numpy as np
    import torch
    import wcg
    from wcg.corpus import Generator, CONFIGS, BLOCK
    from tests import oracle_bridge as ob

    cfg = CONFIGS["c4_utf8_zipf_64gib"]
    n = args.gib << 30
    call = args.call_gib << 30
    assert call % BLOCK == 0 and n % call == 0
    log(f"building the {cfg['vocab']:.0e}-word generator")
    gen = Generator(cfg["mode"], cfg["vocab"], cfg["zipf_s"], cfg["seed"])
    host = np.empty(n, dtype=np.uint8)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    t0 = time.perf_counter()
    for g in range(n >> 30):
        a = g << 30
        gen.fill_ptr(host.ctypes.data + a, 1 << 30, first_block=a // BLOCK, threads=args.threads)
        dev[a:a + (1 << 30)].copy_(torch.from_numpy(host[a:a + (1 << 30)]))
        if g % 4 == 3 or g == (n >> 30) - 1:
            log(f"generated + copied {g + 1} GiB ({time.perf_counter() - t0:.0f} s)")
    torch.cuda.synchronize()

    eng = wcg.Engine(device=0, max_input_bytes=0, max_keys=args.max_keys)
    eng.enable_timing(True)

    def job():
        eng.reset()
        for c in range(n // call):
            eng.map_device(dev.data_ptr() + c * call, call)
        nk, nb = eng.reduce()
        eng.sync()
        return nk, nb

    times = []
    for j in range(1 + args.jobs):
        t = time.perf_counter()
        nk, nb = job()
        dt = time.perf_counter() - t
        log(f"job {j} ({'untimed' if j == 0 else 'timed'}): {dt * 1e3:.1f} ms, {nk} keys, {nb} bytes")
        if j:
            times.append(dt)
    ph, _ = eng.timings()
    st = eng.stats()
    merged = eng.result()
    eng.close()
    del dev
    if args.no_verify:
        log(f"merged file {len(merged)} bytes; not verified (--no-verify)")
        print(json.dumps({"job_ms": [round(t * 1e3, 2) for t in times], "verified_vs_oracle": None,
                          "phase_ms_last_job": {k: round(v, 3) for k, v in ph.items()}, "stats": st}), flush=True)
        return
    log(f"merged file {len(merged)} bytes; verifying against the input on {args.threads} threads")

    res = {}
    th = threading.Thread(target=lambda: res.update(
        v=ob.verify_merged(host.ctypes.data, n, merged, args.threads)), daemon=True)
    tv = time.perf_counter()
    th.start()
    while th.is_alive():
        th.join(30)
        if th.is_alive():
            log(f"verifying ({time.perf_counter() - tv:.0f} s)")
    ok, msg, ntok, nkeys = res["v"]
    log(f"verify: ok={ok} {msg!r} tokens={ntok} keys={nkeys} ({time.perf_counter() - tv:.0f} s)")

    best = min(times)
    out = {
        "workload": "c4_utf8_zipf_64gib", "total_bytes": n, "map_calls": n // call, "call_bytes": call,
        "max_keys": args.max_keys, "jobs_timed": len(times),
        "job_ms": [round(t * 1e3, 2) for t in times],
        "value": round(n / best / 1e9, 3), "unit": "GB/s (best job, device-resident input)",
        "hbm_roofline_frac_whole_job": round(n / best / 1e9 / 8000.0, 4),
        "phase_ms_last_job": {k: round(v, 3) for k, v in ph.items()},
        "stats": st, "verified_vs_oracle": ok, "verify_msg": msg,
        "oracle_tokens": ntok, "oracle_keys": nkeys,
        "tokens_match": st.get("tokens") == ntok,
    }
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        f.write(json.dumps(out) + "\n")
    print(json.dumps(out), flush=True)
    sys.exit(0 if ok and out["tokens_match"] else 3)


if __name__ == "__main__":
    main()
