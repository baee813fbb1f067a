"""Config 5: master + workers over UNIX-socket RPC (wcg/mr.py), modelled on the reference's
test_test.go (TestBasic / TestOneFailure / TestManyFailures, test_test.go:136-191).

The CPU tests run the workers with a stand-in engine that speaks libwcg's record-unit format
(the oracle's counts behind it). The `gpu` test runs the same master and workers on the real
HIP engine. Every test checks:
  * the merged file against the oracle, byte for byte;
  * every -res-<r> file against the reference's DoReduce output;
  * that CleanupFiles finds exactly the reference's file names.
"""
import os
import threading
import time

import pytest

from tests.oracle_bridge import wc_ref
from tests.test_distributed import decode, encode


class StandInEngine:
    """wcg.Engine's job interface over the oracle (CPU tests only)."""

    def __init__(self):
        self.counts = {}

    def reset(self):
        self.counts = {}

    def map_host(self, data):
        for k, v in wc_ref.word_count(data).items():
            self.counts[k] = self.counts.get(k, 0) + v

    def export_host(self, nreduce, nranks):
        buckets = [[] for _ in range(nranks)]
        for k, c in self.counts.items():
            buckets[(wc_ref.ihash(k) % nreduce) % nranks].append(encode(k, c))
        parts = [b"".join(b) for b in buckets]
        return b"".join(parts), [len(p) // 32 for p in parts]

    def import_host(self, recs):
        for k, c in decode(recs):
            self.counts[k] = self.counts.get(k, 0) + c

    def reduce(self):
        return len(self.counts), 0

    def partition(self, nreduce, r):
        return wc_ref.res_file(self.counts, nreduce, r)

    def partitions(self, nreduce):
        return [self.partition(nreduce, r) for r in range(nreduce)]

    def result(self):
        return wc_ref.merged_output(self.counts)

    def map_json(self, data, nreduce):
        return wc_ref.map_files(data, nreduce)


def _input(tmp_path, nbytes=300_000):
    from wcg.corpus import Generator
    data = Generator(1, 20_000, 1.0, 31).bytes(nbytes)
    data += b"carriage\r\nreturn lines\r\n" + "ǅungla ĳssel".encode() + b" tail-without-newline"
    path = tmp_path / "824-mrinput.txt"
    path.write_bytes(data)
    return str(path), data


def _expected(data):
    # the parity input for the file path: Split's line handling (CR dropped, final \n added)
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    text = b"".join((l[:-1] if l.endswith(b"\r") else l) + b"\n" for l in lines)
    return wc_ref.word_count(text)


def _run(tmp_path, factory, nmap, nreduce, schedule, timeout=240):
    """schedule(master_addr, start_worker) starts workers (possibly over time)."""
    from wcg import mr
    path, data = _input(tmp_path)
    sock = tmp_path / "sock"
    sock.mkdir()
    master = str(sock / "mr-master")
    job = mr.MapReduce(nmap, nreduce, path, master, str(tmp_path))
    workers = []

    def start(nrpc):
        w = mr.Worker(master, str(sock / f"mr-worker{len(workers)}"), factory, str(tmp_path), nrpc).start()
        workers.append(w)
        return w

    stop = threading.Event()
    t = threading.Thread(target=schedule, args=(start, stop), daemon=True)
    t.start()
    merged = job.wait(timeout)
    stop.set()
    t.join(10)
    counts = _expected(data)
    assert merged == wc_ref.merged_output(counts)
    for r in range(nreduce):
        with open(os.path.join(str(tmp_path), mr.merge_name(job.file, r)), "rb") as f:
            assert f.read() == wc_ref.res_file(counts, nreduce, r)
    job.cleanup_files()                     # every reference file name exists (else raises)
    left = [f for f in os.listdir(tmp_path) if f.startswith("mrtmp.")]
    assert left == [], left
    return job, workers


def _basic(start, stop):
    start(-1)
    start(-1)


def _one_failure(start, stop):
    start(10)                               # dies after 10 RPCs (worker.go:80-89)
    start(-1)


def _many_failures(start, stop):
    while not stop.is_set():                # test_test.go:167-191: new 10-RPC workers keep coming
        start(10)
        start(10)
        time.sleep(0.3)


@pytest.mark.parametrize("name,schedule", [("basic", _basic), ("one_failure", _one_failure),
                                           ("many_failures", _many_failures)])
def test_master_workers_cpu_standin(tmp_path, name, schedule):
    job, workers = _run(tmp_path, StandInEngine, nmap=20, nreduce=10, schedule=schedule)
    if name == "basic":                     # checkWorker: every worker did at least one job
        assert len(job.stats) == 2 and all(n > 0 for n in job.stats), job.stats
        # worker.go:40-43: each worker's Njobs counts its DoJob connections plus the Shutdown RPC's
        assert sum(job.stats) == 20 + 10 + 2, job.stats


def test_split_matches_reference_rules(tmp_path):
    from wcg import mr
    p = tmp_path / "in.txt"
    p.write_bytes(b"ab cd\r\nef\n\ngh ij kl\nlast")
    n = mr.split(str(p), 3, str(tmp_path), "in.txt")
    parts = [(tmp_path / mr.map_name("in.txt", k)).read_bytes() for k in range(n)]
    assert b"".join(parts) == b"ab cd\nef\n\ngh ij kl\nlast\n"
    # size 25, nchunk = 25 // 3 + 1 = 9: a new split starts once more than 9 * m bytes were written
    assert parts == [b"ab cd\nef\n\n", b"gh ij kl\n", b"last\n"]


def test_split_p1_line_limit(tmp_path):
    """Quirk P1 (bufio.Scanner, mapreduce.go:164-176): a line of 65,535 bytes is split like any
    other; one of 65,536 bytes (with or without its '\n') ends the scan silently - the lines
    before it are the whole input, as in the oracle's restatement."""
    from wcg import mr
    for L, stops in ((65535, False), (65536, True), (70000, True)):
        for tail in (b"\nafter line\n", b""):
            data = b"first line\n" + b"y" * L + tail
            p = tmp_path / f"in{L}{len(tail)}.txt"
            p.write_bytes(data)
            n = mr.split(str(p), 1, str(tmp_path), p.name)
            got = b"".join((tmp_path / mr.map_name(p.name, k)).read_bytes() for k in range(n))
            assert got == b"".join(wc_ref.split(data, 1)), (L, tail)
            assert (got == b"first line\n") == stops


def test_json_intermediates_cpu_standin(tmp_path):
    """json_intermediates: DoMap writes the reference's per-occurrence JSON lines and DoReduce
    reads them back (the file formats and names the CPU DoReduce / CleanupFiles expect)."""
    from wcg import mr
    path, data = _input(tmp_path, 100_000)
    fname = os.path.basename(path)
    nmap, nreduce = 4, 3
    n = mr.split(path, nmap, str(tmp_path), fname)
    eng = StandInEngine()
    for m in range(n):
        mr.do_map(eng, m, str(tmp_path), fname, nreduce, json_intermediates=True)
        split = (tmp_path / mr.map_name(fname, m)).read_bytes()
        want = wc_ref.map_files(split, nreduce)
        for r in range(nreduce):
            assert (tmp_path / mr.reduce_name(fname, m, r)).read_bytes() == want[r]
    counts = _expected(data)
    for r in range(nreduce):
        mr.do_reduce(eng, r, str(tmp_path), fname, n)
        assert (tmp_path / mr.merge_name(fname, r)).read_bytes() == wc_ref.res_file(counts, nreduce, r)


@pytest.mark.gpu
def test_master_workers_gpu(tmp_path, built):
    import wcg
    _run(tmp_path, lambda: wcg.Engine(0, 1 << 20, 1 << 18), nmap=8, nreduce=5, schedule=_one_failure)


@pytest.mark.gpu
def test_run_single_gpu(tmp_path, built):
    """RunSingle (mapreduce.go:344-356) on the GPU: -res-<r> files and the merged file."""
    import wcg
    from wcg import mr
    path, data = _input(tmp_path)
    with wcg.Engine(0, 1 << 20, 1 << 18) as e:
        merged = mr.run_single(5, 3, path, e, str(tmp_path))
    counts = _expected(data)
    assert merged == wc_ref.merged_output(counts)
    for r in range(3):
        assert (tmp_path / mr.merge_name(os.path.basename(path), r)).read_bytes() == wc_ref.res_file(counts, 3, r)


def _p2_input(nbytes):
    """Lines of letters whose tokens straddle the read cap in the middle of a word and of a
    2-byte rune (the P2 cut lands wherever the split's byte count says)."""
    unit = "wörd ".encode() * 700 + b"tailtoken\n"     # ~4 KiB lines: Split stays quick at 1 GiB
    return (unit * (nbytes // len(unit) + 1))[:nbytes] + b"end\n"


@pytest.mark.parametrize("cap", [4096, 4097, 4099, 10000])
def test_run_single_p2_read_cap_cpu_standin(tmp_path, monkeypatch, cap):
    """Quirk P2 (mapreduce.go:205-207): DoMap's single Read returns at most READ_CAP bytes (1 GiB
    in Go 1.16-1.20); a larger split is mapped as its prefix.  With the cap lowered, RunSingle's
    merged and -res-<r> files equal the oracle's restatement (wc_ref.run_single(read_cap=...)),
    and differ from the uncapped counts - the emulation is exercised, not bypassed."""
    from wcg import mr
    monkeypatch.setattr(mr, "READ_CAP", cap)
    data = _p2_input(40_000)
    path = tmp_path / "p2.txt"
    path.write_bytes(data)
    merged = mr.run_single(3, 4, str(path), StandInEngine(), str(tmp_path))
    ref = wc_ref.run_single(data, 3, 4, read_cap=cap)
    assert merged == ref["merged"]
    for r in range(4):
        assert (tmp_path / mr.merge_name("p2.txt", r)).read_bytes() == ref["res"][r]
    assert merged != wc_ref.run_single(data, 3, 4)["merged"]


def test_do_reduce_mixed_intermediate_formats(tmp_path):
    """Workers of one job may write different intermediate formats (record units / the
    reference's JSON lines); DoReduce reads each file in its own format and loses nothing."""
    from wcg import mr
    path, data = _input(tmp_path, 60_000)
    fname = os.path.basename(path)
    nmap, nreduce = 4, 3
    n = mr.split(path, nmap, str(tmp_path), fname)
    eng = StandInEngine()
    for m in range(n):
        mr.do_map(eng, m, str(tmp_path), fname, nreduce, json_intermediates=(m % 2 == 0))
    counts = _expected(data)
    for r in range(nreduce):
        mr.do_reduce(eng, r, str(tmp_path), fname, n)
        assert (tmp_path / mr.merge_name(fname, r)).read_bytes() == wc_ref.res_file(counts, nreduce, r)


@pytest.mark.gpu
def test_run_single_p2_split_over_1gib_gpu(tmp_path, built):
    """A real split larger than 1 GiB (nMap = 1, 1 GiB + 5 MiB): the GPU RunSingle maps exactly
    DoMap's first 1 GiB (P2), checked against the C oracle on that prefix."""
    import wcg
    from wcg import mr
    from tests import oracle_bridge as ob
    n = (1 << 30) + (5 << 20)
    data = _p2_input(n)
    path = tmp_path / "big.txt"
    path.write_bytes(data)
    split = wc_ref.split(data, 1)
    assert len(split) == 1 and len(split[0]) > mr.READ_CAP
    want = ob.merged(split[0][:mr.READ_CAP], 16)
    with wcg.Engine(0, 0, 1 << 18) as e:
        merged = mr.run_single(1, 3, str(path), e, str(tmp_path))
    ob.assert_same(merged, want)
