"""The N > 1 orchestration (wcg/distributed.py) driving the real GPU engine.

Two ranks share the one MI355X of the test box and talk over gloo with host-staged record
buffers (RCCL needs one GPU per rank; the driver's 8-GPU run covers that path).  Each rank maps
a line-aligned range, the ihash shuffle moves every key to its owner, the owners' results hold
only their partitions, and the merged file on rank 0 must equal the oracle's - twice in a row, so
the engines' reset between jobs is covered too.
"""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mit-6.824-2015_amd")


def _corpus():
    from wcg.corpus import Generator
    d = Generator(0, 30_000, 1.0, 21).bytes(6 << 20)
    return d + b"\n" + b"longkeylongkeylongkey" * 2 + b" " + "ǅ".encode() * 20 + b" zebra\n"


def _worker(rank, world, port, q):
    try:
        for p in (ROOT, PKG):
            if p not in sys.path:
                sys.path.insert(0, p)
        import torch
        import torch.distributed as dist
        import wcg
        from wcg import distributed as wd
        from tests import oracle_bridge as ob
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        data = _corpus()
        lo, hi = wd.line_aligned_ranges(len(data), world, lambda i: data[i])[rank]
        R = 64
        with wcg.Engine(0, max(hi - lo, 1), 1 << 19) as eng:
            te = wd.TorchEngine(eng, host_staging=True)
            want = ob.merged(data) if rank == 0 else None
            for rep in range(2):
                eng.reset()
                eng.map_host(data[lo:hi])
                wd.shuffle_reduce(te, R)
                owned = eng.result().splitlines()
                owner_ok = all((wcg.ihash(l.rsplit(b": ", 1)[0]) % R) % world == rank for l in owned)
                merged = wd.gather_merge(te)          # rank 0 merges the owners' sorted runs
                q.put((rank, rep, owner_ok, len(owned), merged == want if rank == 0 else None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, "err", repr(e), 0, None))
        raise


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_one_gpu_gloo(built):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(100)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not q.empty():
        msgs.append(q.get(timeout=5))
    assert all(p.exitcode == 0 for p in procs), (msgs, [p.exitcode for p in procs])
    assert len(msgs) == 2 * world, msgs
    for rank, rep, owner_ok, nowned, merged_ok in msgs:
        assert owner_ok and nowned > 0, (rank, rep)
        if rank == 0:
            assert merged_ok, rep
