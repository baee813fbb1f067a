"""One-launch reduce of small one-pass jobs (r05, csrc/wcg_fused.h): compaction, sample sort, tie
order and formatting of up to 2^17 keys in one persistent kernel.  Every job is compared byte for
byte with the C oracle, the path taken is checked with wcg_reduce_path, and the rare paths are
forced: buckets past their region (the spill list and the workgroup's global merge sort, through a
huge WCG_FUSED_TARGET), buckets of a few records (a tiny target: hundreds of buckets, many sample
runs), long keys sharing a 16-byte prefix in small runs and in runs of thousands, 0 / 1 / 2 keys,
and many launches in a row (the control block's epoch and counter reset)."""
import os
import random

import pytest

from tests import oracle_bridge as ob

pytestmark = pytest.mark.gpu


def corpus(nkeys, ntok, seed, tie_every=0, tie_prefix="Z" * 20, tie_keys=0):
    rnd = random.Random(seed)
    words = []
    for i in range(nkeys):
        n = 1 + rnd.randrange(14)
        words.append("".join(rnd.choice("abcdefghijklmnopqrstuvwxyzABC") for _ in range(n)) + f"q{i:x}")
    ties = [tie_prefix + "".join(rnd.choice("abcdefghij") for _ in range(1 + rnd.randrange(30))) + f"r{i:x}"
            for i in range(tie_keys)]
    out = []
    for t in range(ntok):
        w = words[rnd.randrange(nkeys)] if t < ntok - nkeys else words[t - (ntok - nkeys)]
        if tie_every and t % tie_every == 0:
            w = tie_prefix + w              # long keys sharing a 16-byte prefix
        out.append(w)
        out.append(" " if rnd.randrange(9) else "\n")
    out.extend(w + "\n" for w in ties)
    return "".join(out).encode()


@pytest.fixture(scope="module")
def eng(built):
    import wcg
    e = wcg.Engine(device=0, max_input_bytes=64 << 20, max_keys=1 << 18)
    yield e
    e.close()


@pytest.fixture
def target():
    old = os.environ.get("WCG_FUSED_TARGET")

    def set_(v):
        if v is None:
            os.environ.pop("WCG_FUSED_TARGET", None)
        else:
            os.environ["WCG_FUSED_TARGET"] = str(v)
    yield set_
    set_(old)


def job(eng, data):
    eng.reset()
    eng.map_host(data)
    nk, nb = eng.reduce()
    out = eng.result()
    assert len(out) == nb
    return nk, out


def check(eng, data, fused=True):
    nk, got = job(eng, data)
    want = ob.merged(data)
    ob.assert_same(got, want)
    assert nk == want.count(b"\n")
    assert eng.reduce_path() == (1 if fused else 0)
    return nk


def test_first_job_takes_the_general_path(built):
    import wcg
    with wcg.Engine(device=0, max_input_bytes=8 << 20, max_keys=1 << 16) as e:
        data = corpus(500, 4000, 1)
        check(e, data, fused=False)          # no hint yet: the exact multi-launch path
        check(e, data, fused=True)


@pytest.mark.parametrize("nkeys,ntok,tie_every", [
    (1, 5, 0), (2, 9, 0), (300, 3000, 0), (5000, 40000, 17), (100000, 400000, 0), (60000, 300000, 41),
])
def test_sizes(eng, nkeys, ntok, tie_every):
    job(eng, corpus(2000, 8000, 2))          # a hint within the one-launch range
    check(eng, corpus(nkeys, ntok, 10 + nkeys, tie_every=tie_every))


def test_empty_and_letterless(eng):
    """jobs of no key (after a job of 0 keys the hint is 0: the next job takes the general path)"""
    job(eng, corpus(100, 500, 4))
    check(eng, b"")
    check(eng, corpus(100, 500, 5), fused=False)
    check(eng, b"... 123 !!\n")
    job(eng, corpus(100, 500, 6))
    check(eng, corpus(1, 1, 7))


def test_tiny_buckets_many_runs(eng, target):
    """target 3: ~1000 buckets capped at 512, 2048 samples in 4 runs; every bucket sorts as E = 1"""
    job(eng, corpus(2000, 8000, 6))
    target(3)
    check(eng, corpus(1500, 12000, 7, tie_every=5))
    check(eng, corpus(30000, 90000, 8))


def test_oversized_buckets_spill(eng, target):
    """one bucket of every record (target past n): the region holds 2048, the rest spills, and
    the workgroup merge-sorts the bucket in global memory (3 windows of formatting)"""
    job(eng, corpus(2000, 8000, 9))
    target(1 << 30)
    check(eng, corpus(5000, 30000, 11, tie_every=13))
    target(1500)                             # buckets near and past the region size
    check(eng, corpus(40000, 200000, 12, tie_every=29))


def test_long_tie_runs(eng, target):
    """3000 long keys sharing a 16-byte prefix: one bucket-sized run (LDS path, counted ranks) and,
    with one bucket, a run across the global sort's chunks"""
    job(eng, corpus(2000, 8000, 13))
    check(eng, corpus(2000, 10000, 14, tie_keys=3000))
    target(1 << 30)
    check(eng, corpus(200, 1000, 15, tie_keys=3000))


def test_many_launches(eng):
    """50 jobs in a row on one context: the epoch and counter reset of every launch"""
    job(eng, corpus(3000, 9000, 16))
    for i in range(50):
        nk = 1 + (i * 7919) % 4000
        check(eng, corpus(nk, 3 * nk, 100 + i, tie_every=7 if i % 3 == 0 else 0))


def test_partitions_after_fused_reduce(eng):
    job(eng, corpus(3000, 9000, 17))
    data = corpus(20000, 80000, 18, tie_every=23)
    check(eng, data)
    ref = ob.Result(data)
    for r in (0, 3, 63):
        assert eng.partition(64, r) == ref.res(64, r)
    counts = eng.export_count(64, 4)
    assert sum(counts) >= 20000


# ---------------------------------------------------------------- wcg_reduce_async
def test_async_back_to_back(eng):
    """jobs queued behind each other without a host wait: the last one's result is exact, the
    earlier ones were dropped by the next reset"""
    datas = [corpus(500 + 97 * i, 4000, 200 + i, tie_every=11 if i % 2 else 0) for i in range(12)]
    job(eng, datas[0])
    for d in datas:
        eng.reset()
        eng.map_host(d)
        eng.reduce_async()
    nk, nb = eng.reduce_wait()
    want = ob.merged(datas[-1])
    assert nb == len(want) and nk == want.count(b"\n")
    ob.assert_same(eng.result(), want)
    assert eng.reduce_path() == 1


def test_async_result_calls_wait(eng):
    data = corpus(3000, 20000, 300, tie_every=19)
    job(eng, corpus(1000, 5000, 301))
    eng.reset()
    eng.map_host(data)
    eng.reduce_async()
    ob.assert_same(eng.result(), ob.merged(data))          # no reduce_wait: result() waits
    eng.reset()
    eng.map_host(data)
    eng.reduce_async()
    ref = ob.Result(data)
    assert eng.partition(64, 7) == ref.res(64, 7)          # so does the partition path
    assert eng.stats()["keys"] == ref.merged().count(b"\n")


def test_async_first_job_is_synchronous(built):
    import wcg
    with wcg.Engine(device=0, max_input_bytes=8 << 20, max_keys=1 << 16) as e:
        data = corpus(400, 3000, 302)
        e.reset()
        e.map_host(data)
        e.reduce_async()                                   # no hint: the multi-launch path, at once
        assert e.reduce_path() == 0
        ob.assert_same(e.result(), ob.merged(data))


def test_async_error_surfaces_at_wait(built):
    """a table that fills in an async job: reduce_async returns, reduce_wait reports WCG_EFULL,
    and the next job is exact again"""
    import wcg
    from wcg._lib import WcgError, WCG_EFULL
    with wcg.Engine(device=0, max_input_bytes=8 << 20, max_keys=1024) as e:
        small = corpus(300, 2000, 303)
        job(e, small)
        e.reset()
        e.map_host(corpus(6000, 12000, 304))               # 6000 keys in a 2048-slot table
        e.reduce_async()
        with pytest.raises(WcgError) as ex:
            e.reduce_wait()
        assert ex.value.status == WCG_EFULL
        nk, got = job(e, small)
        ob.assert_same(got, ob.merged(small))


def test_two_contexts_fused_concurrently(built):
    """Two contexts' one-launch reduces queued at once on their own streams run side by side on
    the GPU, so neither launch has all its workgroups resident: work must be handed out without a
    residency assumption (a fixed first item per workgroup deadlocked when another process's
    launch held half the CUs: the N = 2 rehearsal on one GPU)."""
    import wcg
    engines = [wcg.Engine(device=0, max_input_bytes=64 << 20, max_keys=1 << 18) for _ in range(2)]
    datas = [corpus(30_000, 300_000, seed=s) for s in (3, 4)]
    wants = [ob.merged(d) for d in datas]
    try:
        for rep in range(4):
            for e, d in zip(engines, datas):
                e.reset()
                e.map_host(d)
            for e in engines:
                e.reduce_async()
            for e, want in zip(engines, wants):
                e.reduce_wait()
                ob.assert_same(e.result(), want)
                assert e.reduce_path() == (1 if rep else 0)
    finally:
        for e in engines:
            e.close()
