"""GPU: the data formats and the ingest either side of the hot path, bit-exact.

  * wcg_map_file (Split + DoMap from a file through the pinned double-buffered ingest): several
    64 MiB chunks, CRLF lines, and quirk P1 (a 64 KiB line ends the input) at a chunk edge;
  * wcg_map (host split) streamed in chunks cut after ASCII non-letters, including a split with
    no such byte for longer than a chunk (keys stay short: inside the parity domain a key is at
    most one 64 KiB line);
  * wcg_partition_all: every -res-<r> file in one pass, against the oracle (R = 1, 3, 64, 1000);
  * wcg_map_json: DoMap's per-occurrence JSON intermediates, byte-exact, consumed by the CPU
    DoReduce port (oracle/mr_port.c) to the reference's -res-<r> bytes;
  * RunSingle from the wc.go CLI with the P1 boundary lines (65,535 / 65,536 bytes);
  * dense long tokens (every token 16 letters): the long-token log fills and k_map counts the
    rest inline.
"""
import os
import random

import pytest

from tests import oracle_bridge as ob
from tests.oracle_bridge import wc_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(built):
    import wcg
    e = wcg.Engine(device=0, max_input_bytes=0, max_keys=1 << 21)
    yield e
    e.close()


def _split_text(data):
    """The bytes Split feeds to the map phase (P1 cut, CR before LF dropped, final LF added)."""
    return b"".join(wc_ref.split(data, 1))


def test_map_file_multi_chunk(eng, tmp_path):
    from wcg.corpus import Generator
    data = Generator(1, 50_000, 1.0, 23).bytes(150 << 20)            # 3 chunks of 64 MiB
    data = data.replace(b"\n", b"\r\n", 1000)
    p = tmp_path / "in.txt"
    p.write_bytes(data)
    eng.reset()
    mapped, size = eng.map_file(str(p))
    assert size == len(data) and mapped == len(data)
    eng.reduce()
    ob.assert_same(eng.result(), ob.merged(data))


@pytest.mark.parametrize("where", ["start", "middle", "chunk_edge", "end_no_newline"])
def test_map_file_p1_truncation(eng, tmp_path, where):
    from wcg.corpus import Generator
    base = Generator(0, 20_000, 1.0, 29).bytes(70 << 20)
    bad = b"z" * 65536
    if where == "start":
        data = bad + b"\n" + base
    elif where == "middle":
        cut = base.index(b"\n", 10 << 20) + 1
        data = base[:cut] + bad + b"\n" + base[cut:]
    elif where == "chunk_edge":                                       # the long line spans 64 MiB
        cut = base.index(b"\n", (64 << 20) - 30000) + 1
        data = base[:cut] + bad + b"\n" + base[cut:]
    else:
        data = base + bad
    p = tmp_path / f"p1_{where}.txt"
    p.write_bytes(data)
    eng.reset()
    mapped, size = eng.map_file(str(p))
    want_text = _split_text(data)
    eng.reduce()
    ob.assert_same(eng.result(), ob.merged(want_text))
    assert mapped < size
    # 65,535 bytes + '\n' still fits: nothing is cut
    ok = data.replace(bad, b"z" * 65535)
    p.write_bytes(ok)
    eng.reset()
    mapped, size = eng.map_file(str(p))
    eng.reduce()
    assert mapped == size and eng.result() == ob.merged(ok)


def test_map_host_streamed_chunks(eng):
    from wcg.corpus import Generator
    data = Generator(1, 30_000, 1.0, 31).bytes(140 << 20)
    # 80 MB without one ASCII byte (short tokens split by U+3000, a non-ASCII separator), so a
    # 64 MiB chunk has no safe cut inside it, then more text
    blob = data[: 5 << 20] + "éé\u3000中".encode() * (8 << 20) + b" " + data[5 << 20:]
    for d in (data, blob):
        eng.reset()
        eng.map_host(d)
        eng.reduce()
        ob.assert_same(eng.result(), ob.merged(d))


@pytest.mark.parametrize("R", [1, 3, 64, 1000])
def test_partition_all(eng, R):
    from wcg.corpus import Generator
    data = Generator(1, 40_000, 1.0, 37).bytes(16 << 20)
    data += b" " + b"longkeylongkeylongkey" * 3 + b" " + "ǅ".encode() * 20 + b"\n"
    eng.reset()
    eng.map_host(data)
    eng.reduce()
    r = ob.Result(data)
    parts = eng.partitions(R)
    assert len(parts) == R
    for i in (0, R // 2, R - 1):
        assert eng.partition(R, i) == parts[i]
    assert parts == [r.res(R, i) for i in range(R)]


def test_map_json_feeds_cpu_do_reduce(eng, tmp_path):
    from wcg.corpus import Generator
    splits = [Generator(1, 3_000, 1.0, 41 + m).bytes(1 << 20) for m in range(3)]
    splits[1] += b" " + b"x" * 70 + " ǅungla".encode() + b"\n"
    nreduce, fname = 5, "in.txt"
    for m, s in enumerate(splits):
        parts = eng.map_json(s, nreduce)
        assert parts == wc_ref.map_files(s, nreduce), m
        for r in range(nreduce):
            (tmp_path / f"mrtmp.{fname}-{m}-{r}").write_bytes(parts[r])
    counts = wc_ref.word_count(b"".join(splits))
    for r in range(nreduce):
        ob.do_reduce_files(str(tmp_path), fname, r, len(splits))
        assert (tmp_path / f"mrtmp.{fname}-res-{r}").read_bytes() == wc_ref.res_file(counts, nreduce, r)
    assert eng.map_json(b"", 3) == [b"", b"", b""]


def test_run_single_cli_p1_lines(built, tmp_path):
    """wc.go's sequential mode (RunSingle(5, 3)) through the CLI entry, with lines at the P1
    boundary: 65,535 bytes (kept) and 65,536 bytes (the scan ends there)."""
    from wcg import wc, mr
    from wcg.corpus import Generator
    base = Generator(0, 5_000, 1.0, 43).bytes(2 << 20)
    cut = base.index(b"\n", (19 << 20) // 10) + 1                    # late: Split still makes 5 files (P3)
    for L in (65535, 65536):
        data = base[:cut] + b"q" * L + b"\n" + base[cut:]
        d = tmp_path / str(L)
        d.mkdir()
        p = d / "kjv.txt"
        p.write_bytes(data)
        merged = wc.run_single(str(p))
        want = ob.merged(_split_text(data))
        assert merged == want and (d / "mrtmp.kjv.txt").read_bytes() == want
        counts = wc_ref.word_count(_split_text(data))
        for r in range(3):
            assert (d / mr.merge_name("kjv.txt", r)).read_bytes() == wc_ref.res_file(counts, 3, r)


def test_dense_long_tokens_fill_the_log(eng):
    """~4.1 MB of 16-letter tokens separated by single spaces: 58 long tokens per 992-byte step,
    far above the log's average sizing, so most are counted inline (exact either way)."""
    rng = random.Random(5)
    words = [bytes(rng.choice(b"abcdefgh") for _ in range(16)) for _ in range(2000)]
    toks = [rng.choice(words) for _ in range(4_100_000 // 17)]
    data = b" ".join(toks) + b"\n"
    eng.reset()
    eng.map_host(data)
    eng.reduce()
    ob.assert_same(eng.result(), ob.merged(data))
    st = eng.stats()
    assert st["overflow"] == 0 and st["long_tokens"] == len(toks)


def test_free_releases_result_and_export_buffers(built):
    """wcg_free: the formatted output and the export records are library-owned
    until freed; after the free the result calls report WCG_ESTATE, the next job works as usual,
    and a pointer the context did not hand out is rejected."""
    import wcg
    from tests import oracle_bridge as ob
    data = b"the cat and the hat\nand the bat\n" * 50
    with wcg.Engine(0, 0, 1 << 16) as e:
        e.reset()
        e.map_host(data)
        e.reduce()
        ptr, nb = e.result_device()
        assert nb == len(ob.merged(data))
        e.free(ptr)
        with pytest.raises(wcg.WcgError):
            e.result()
        dev, counts = e.export(3, 2)
        assert sum(counts) > 0
        e.free(dev)
        with pytest.raises(wcg.WcgError):
            e.free(12345)
        e.reset()
        e.map_host(data)
        e.reduce()
        assert e.result() == ob.merged(data)
