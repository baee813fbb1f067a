"""Device-sized reduce (round 3): after its first job a context runs compaction, sort and
formatting of one-pass jobs on the record count held in device memory (no host read between
compaction and the sort; the one read-back is the formatted size at the end of wcg_reduce).

The sort is then planned for the previous job's count, so these tests run one engine through
jobs whose key counts jump up and down (more keys than the plan: oversized buckets; 0 and 1 key;
long-key ties), then use the partition / export paths that need the exact count on the host, and a
job that overflows the tables (the error must surface, and the next job must be right again).
Everything is compared byte for byte with the C oracle.
"""
import random

import pytest

from tests import oracle_bridge as ob

pytestmark = pytest.mark.gpu


def corpus(nkeys, ntok, seed, long_every=0):
    rnd = random.Random(seed)
    words = []
    for i in range(nkeys):
        n = 1 + rnd.randrange(14)
        words.append("".join(rnd.choice("abcdefghijklmnopqrstuvwxyzABC") for _ in range(n)) + f"q{i:x}")
    out = []
    for t in range(ntok):
        w = words[rnd.randrange(nkeys)] if t < ntok - nkeys else words[t - (ntok - nkeys)]
        if long_every and t % long_every == 0:
            w = "Z" * 20 + w          # long keys sharing a 16-byte prefix: the tie sort
        out.append(w)
        out.append(" " if rnd.randrange(9) else "\n")
    return "".join(out).encode()


def job(eng, data):
    eng.reset()
    eng.map_host(data)
    nk, nb = eng.reduce()
    out = eng.result()
    assert len(out) == nb
    return nk, out


@pytest.fixture(scope="module")
def eng(built):
    import wcg
    e = wcg.Engine(device=0, max_input_bytes=64 << 20, max_keys=1 << 19)
    yield e
    e.close()


@pytest.mark.parametrize("seq", [
    [(20000, 200000), (3, 50), (300000, 600000), (0, 0), (1, 7), (50000, 300000), (2, 2)],
])
def test_key_counts_jump(eng, seq):
    for i, (nkeys, ntok) in enumerate(seq):
        data = corpus(nkeys, ntok, 100 + i, long_every=97) if nkeys else b"...\n  \n"
        nk, got = job(eng, data)
        want = ob.merged(data)
        ob.assert_same(got, want)
        assert nk == want.count(b"\n")


def test_partitions_and_export_after_device_sized_reduce(eng):
    job(eng, corpus(5000, 40000, 7))                  # the hint for the next job
    data = corpus(30000, 120000, 8, long_every=53)
    nk, got = job(eng, data)                          # device-sized
    ob.assert_same(got, ob.merged(data))
    ref = ob.Result(data)
    for r in (0, 5, 63):
        assert eng.partition(64, r) == ref.res(64, r)
    counts = eng.export_count(64, 3)            # units per owner rank (long keys take several)
    import wcg
    fresh = wcg.Engine(device=0, max_input_bytes=64 << 20, max_keys=1 << 19)
    try:
        job(fresh, data)                          # a first job: the exact (read-back) path
        assert fresh.export_count(64, 3) == counts
    finally:
        fresh.close()
    assert sum(counts) >= nk


def test_overflow_surfaces_then_recovers(built):
    import wcg
    e = wcg.Engine(device=0, max_input_bytes=8 << 20, max_keys=1024)
    try:
        small = corpus(300, 3000, 11)
        job(e, small)                                 # exact path; sets the hint
        with pytest.raises(wcg.WcgError):
            job(e, corpus(20000, 40000, 12))          # device-sized: the table overflows
        nk, got = job(e, small)
        ob.assert_same(got, ob.merged(small))
    finally:
        e.close()
