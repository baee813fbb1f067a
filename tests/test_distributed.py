"""CPU test of the N > 1 path (wcg/distributed.py) with the gloo backend, world_size 2 and 3.

The GPU engine cannot run here, so each rank drives the orchestration with an oracle-backed
stand-in that speaks libwcg's 32-byte record-unit wire format (include/wcg.h, WCG_RECORD_BYTES).
This checks the range partitioning, the owner rule (ihash % nReduce) % world, the count +
payload all-to-all-v, the owner-side reduce (each owner's sorted run) and the k-way merge of the
runs on rank 0 against the oracle.
"""
import os
import socket
import struct

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.oracle_bridge import wc_ref

LONG_FLAG = 1 << 63
CONT_MARK = 1 << 62


def encode(key: bytes, cnt: int) -> bytes:
    """libwcg record units (csrc/wcg_reduce.h: k_export_write)."""
    if len(key) <= 15:
        pad = key + b"\0" * (16 - len(key))
        hi, lo = struct.unpack(">QQ", pad)
        return struct.pack("<QQQQ", hi, lo, cnt, len(key))
    hi, lo = struct.unpack(">QQ", key[:16])
    out = struct.pack("<QQQQ", hi, lo, cnt, LONG_FLAG | (len(key) << 40))
    for i in range(0, len(key), 24):
        chunk = key[i:i + 24].ljust(24, b"\0")
        out += chunk + struct.pack("<Q", CONT_MARK)
    return out


def decode(buf: bytes):
    i, n = 0, len(buf) // 32
    while i < n:
        hi, lo, cnt, ref = struct.unpack_from("<QQQQ", buf, 32 * i)
        assert ref != CONT_MARK, "continuation unit without header"
        if ref & LONG_FLAG:
            ln = (ref >> 40) & ((1 << 23) - 1)
            nu = (ln + 23) // 24
            raw = b"".join(buf[32 * (i + 1 + k): 32 * (i + 1 + k) + 24] for k in range(nu))
            yield raw[:ln], cnt
            i += 1 + nu
        else:
            key = struct.pack(">QQ", hi, lo)[:ref]
            yield key, cnt
            i += 1


class OracleEngine:
    def __init__(self):
        self.counts = {}

    def reset(self):
        self.counts = {}

    def map_bytes(self, data):
        for k, v in wc_ref.word_count(data).items():
            self.counts[k] = self.counts.get(k, 0) + v

    def export_tensor(self, nreduce, nranks):
        buckets = [[] for _ in range(nranks)]
        for k, c in self.counts.items():
            buckets[(wc_ref.ihash(k) % nreduce) % nranks].append(encode(k, c))
        parts = [b"".join(b) for b in buckets]
        blob = b"".join(parts) or b"\0" * 32
        return torch.frombuffer(bytearray(blob), dtype=torch.uint8), [len(p) // 32 for p in parts]

    def import_tensor(self, t, nunits):
        for k, c in decode(t[: nunits * 32].numpy().tobytes()):
            self.counts[k] = self.counts.get(k, 0) + c

    def reduce(self):
        return len(self.counts), len(self.result())

    def result(self):
        return wc_ref.merged_output(self.counts)

    def result_tensor(self):
        out = self.result()
        return torch.frombuffer(bytearray(out or b"\0"), dtype=torch.uint8), len(out)

    def merge_runs_tensor(self, t, run_bytes):
        """k-way merge of sorted "key: count" runs (the owners' disjoint outputs) by key bytes."""
        import heapq
        raw, runs, off = t.numpy().tobytes(), [], 0
        for n in run_bytes:
            runs.append(raw[off:off + n].splitlines(keepends=True))
            off += n
        for run in runs:
            keys = [l.rsplit(b": ", 1)[0] for l in run]
            assert keys == sorted(keys), "a run is not sorted"
        merged = list(heapq.merge(*runs, key=lambda l: l.rsplit(b": ", 1)[0]))
        self.counts = {l.rsplit(b": ", 1)[0]: int(l.rsplit(b": ", 1)[1]) for l in merged}
        assert b"".join(merged) == self.result()
        return len(merged), len(self.result())


def corpus():
    from wcg.corpus import Generator
    d = Generator(1, 5_000, 1.0, 17).bytes(400_000)
    return d + b"\n" + b"abcdefghijklmnopqrstuvwxyz" * 3 + b" " + "ǅ".encode() * 20 + b"\n"


def _worker(rank, world, port, q):
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        from wcg import distributed as wd
        data = corpus()
        lo, hi = wd.line_aligned_ranges(len(data), world, lambda i: data[i])[rank]
        eng = OracleEngine()
        eng.map_bytes(data[lo:hi])
        R = 64
        wd.shuffle_reduce(eng, R)
        owned = set(eng.counts)
        assert all((wc_ref.ihash(k) % R) % world == rank for k in owned)
        merged = wd.gather_merge(eng)
        if rank == 0:
            q.put(("ok", merged == wc_ref.merged_output(wc_ref.word_count(data))))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("err", repr(e)))
        raise


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_shuffle_and_merge(built, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    status, ok = q.get(timeout=5)
    assert status == "ok" and ok


def test_wire_format_roundtrip():
    keys = [b"a", b"abcdefghijklmno", b"abcdefghijklmnop", "中文".encode() * 9, b"z" * 100]
    blob = b"".join(encode(k, i + 1) for i, k in enumerate(keys))
    assert list(decode(blob)) == [(k, i + 1) for i, k in enumerate(keys)]


def test_line_aligned_ranges():
    from wcg import distributed as wd
    data = b"ab cd\nef gh\nij\nkl mn op\n"
    rs = wd.line_aligned_ranges(len(data), 3, lambda i: data[i])
    assert rs[0][0] == 0 and rs[-1][1] == len(data)
    for (a, b), (c, d) in zip(rs, rs[1:]):
        assert b == c and (b == 0 or data[b - 1] == 0x0A)


# ---------------------------------------------------------------- the rank launcher of bench.py
def _launch(nprocs, extra, timeout=120):
    import io
    from wcg.launch import launch_ranks
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "standin_rank.py")
    buf = io.StringIO()
    rc = launch_ranks(script, extra, nprocs, timeout, out=buf)
    return rc, buf.getvalue()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_launcher_runs_every_rank(world):
    """`bench.py --gpus N` without an external launcher: the parent starts N ranks (before any GPU
    call), relays rank 0's one JSON line and exits 0."""
    import json
    rc, out = _launch(world, [])
    assert rc == 0, out
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == world and rec["verified_vs_oracle"] is True


def test_launcher_reports_a_failed_rank():
    rc, out = _launch(2, ["--fail-rank", "1"])
    assert rc != 0
    assert not [l for l in out.splitlines() if l.startswith("{")]


def test_launcher_bounds_a_hung_rank():
    import time
    t0 = time.time()
    rc, out = _launch(2, ["--hang-rank", "1"], timeout=20)
    assert rc != 0
    assert time.time() - t0 < 60


def test_launcher_kills_a_rank_that_ignores_sigterm(tmp_path):
    """torch.distributed.run starts every rank in a session of its own, so a signal to
    the launcher's process group alone does not reach them; a rank that ignores SIGTERM (stuck in
    a driver call, or handling the signal) must still be gone when launch_ranks returns."""
    import time
    from wcg.launch import _alive
    t0 = time.time()
    rc, out = _launch(2, ["--ignore-term-rank", "1", "--pid-dir", str(tmp_path)], timeout=15)
    assert rc != 0
    assert time.time() - t0 < 90
    pids = [int(open(os.path.join(tmp_path, f)).read()) for f in os.listdir(tmp_path)]
    assert len(pids) == 2, pids
    assert not [p for p in pids if _alive(p)], "a rank outlived the launcher"


def test_bench_self_launches_before_any_gpu_call():
    """bench.py hands `--gpus N` without WORLD_SIZE to the launcher before importing torch."""
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")).read()
    main = src[src.index("def main():"):]
    assert main.index("launch_ranks(") < main.index("import torch")
