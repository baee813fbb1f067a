#!/usr/bin/env python3
"""Measurement (r06): C2 jobs on ONE engine back to back (the bench's pipelined loop) against jobs
alternating between TWO engines on two streams, so that one job's map can start on the CUs the
other job's aggregation tail and reduce leave idle.  Every job runs in full; the last job of each
engine is checked against the oracle.  Usage: tools/exp_two_ctx.py [steps] [streams-first|bench] [contexts]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mit-6.824-2015_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402  (before libwcg: one HIP runtime)
import wcg  # noqa: E402
from wcg.corpus import Generator, CONFIGS  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
cfg = CONFIGS["c2_ascii_zipf_1gib"]
n = cfg["nbytes"]
host = torch.empty(n, dtype=torch.uint8).pin_memory()
Generator(cfg["mode"], cfg["vocab"], cfg["zipf_s"], cfg["seed"]).fill_ptr(host.data_ptr(), n)
dev = host.to("cuda:0")
torch.cuda.synchronize()
keys_cap = max(min(2 * cfg["vocab"], n // 32), 1 << 18)
order = sys.argv[2] if len(sys.argv) > 2 else "streams-first"
nctx = int(sys.argv[3]) if len(sys.argv) > 3 else 2
engs = []
if order == "streams-first":          # the streams, then the engines
    streams = [torch.cuda.Stream() for _ in range(nctx)]
    for s in streams:
        e = wcg.Engine(device=0, max_input_bytes=0, max_keys=keys_cap)
        e.set_stream(s.cuda_stream)
        engs.append(e)
else:                                 # bench.py's order: a current stream, its engine, then the second
    streams = [torch.cuda.Stream()]
    torch.cuda.set_stream(streams[0])
    e = wcg.Engine(device=0, max_input_bytes=0, max_keys=keys_cap)
    e.set_stream(streams[0].cuda_stream)
    e.enable_timing(3)
    engs.append(e)
    streams.append(torch.cuda.Stream())
    e = wcg.Engine(device=0, max_input_bytes=0, max_keys=keys_cap)
    e.set_stream(streams[1].cuda_stream)
    engs.append(e)
print("order", order, flush=True)


def job(e):
    e.reset()
    e.map_device(dev.data_ptr(), n)
    e.reduce_async()


def run(neng, k):
    pend = [False] * neng
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        j = i % neng
        if pend[j]:
            engs[j].reduce_wait()
        job(engs[j])
        pend[j] = True
    for j in range(neng):
        if pend[j]:
            engs[j].reduce_wait()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


for rep in range(2):
    for neng in range(1, nctx + 1):
        run(neng, 10)                               # warm-up
        ms = run(neng, steps)
        print(f"engines {neng}: {ms:.4f} ms/job = {n / ms / 1e6:.1f} GB/s", flush=True)
from tests import oracle_bridge as ob  # noqa: E402
want = ob.merged(host.numpy().tobytes(), 16)
print("verified", [e.result() == want for e in engs], flush=True)

if order == "bench":
    # bench.py's sequence: W warm-up pipelined jobs on engine 0, a K-job pipelined loop, a K-job
    # synced loop, W warm-up two-engine jobs, the K-job two-engine loop
    W, K = 5, 20

    def pipelined(k):
        for _ in range(k):
            job(engs[0])
        engs[0].reduce_wait()

    for _ in range(3):
        pipelined(W)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pipelined(K)
        torch.cuda.synchronize()
        tp = (time.perf_counter() - t0) / K * 1e3
        t0 = time.perf_counter()
        for _ in range(K):
            engs[0].reset()
            engs[0].map_device(dev.data_ptr(), n)
            engs[0].reduce()
        torch.cuda.synchronize()
        ts = (time.perf_counter() - t0) / K * 1e3
        engs[0].enable_timing(0)
        run(2, W)
        t2 = run(2, K)
        engs[0].enable_timing(3)
        print(f"bench sequence: pipelined {tp:.4f} synced {ts:.4f} two {t2:.4f} ms/job", flush=True)
