#!/usr/bin/env python3
"""Ingest timeline probe: wcg_map_file on a 1 GiB C2 file in tmpfs, timed
per job, for a rocprofv3 --kernel-trace --memory-copy-trace run.  Also times each leg alone (host
read into pinned memory, pinned H2D) like bench.py's ingest_ceilings.

  rocprofv3 --kernel-trace --memory-copy-trace --stats -d OUT -o run -- python3 tools/ingest_probe.py
"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mit-6.824-2015_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import wcg
    from wcg.corpus import Generator, CONFIGS
    import bench
    n = int(os.environ.get("PROBE_BYTES", str(1 << 30)))
    cfg = CONFIGS["c2_ascii_zipf_1gib"]
    d = tempfile.mkdtemp(prefix="wcg-probe-", dir="/dev/shm")
    path = os.path.join(d, "input.txt")
    try:
        host = torch.empty(n, dtype=torch.uint8)
        Generator(cfg["mode"], cfg["vocab"], cfg["zipf_s"], cfg["seed"]).fill_ptr(host.data_ptr(), n)
        host.numpy().tofile(path)
        del host
        with wcg.Engine(device=0, max_input_bytes=0, max_keys=1 << 18) as eng:
            for rep in range(4):
                t0 = time.perf_counter()
                eng.reset()
                mapped, size = eng.map_file(path)
                t1 = time.perf_counter()
                eng.reduce()
                out = eng.result()
                t2 = time.perf_counter()
                print(f"job {rep}: map_file {1e3 * (t1 - t0):.2f} ms (host side returns), reduce+result "
                      f"{1e3 * (t2 - t1):.2f} ms, total {1e3 * (t2 - t0):.2f} ms = {n / (t2 - t0) / 1e9:.2f} GB/s, "
                      f"{len(out)} bytes out", flush=True)
        print("legs alone:", bench.ingest_ceilings(path, n), flush=True)
    finally:
        for f in os.listdir(d):
            os.unlink(os.path.join(d, f))
        os.rmdir(d)


if __name__ == "__main__":
    main()
