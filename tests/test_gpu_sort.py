"""GPU: the reduce-side sort (csrc/wcg_sort.h) and the Merge of sorted runs, bit-exact.

  * the sample sort at several bucket counts, including the oversized-bucket path (forced with
    WCG_SORT_TARGET) and a single bucket;
  * tie groups: long keys sharing a 16-byte prefix - a group of 1e5 keys (the global bitonic
    path), many small groups, and keys that also share bytes 16-31 (the full-compare path);
  * wcg_merge_runs: the owners' sorted runs merged on one GPU (k = 1..9 runs, empty runs,
    long-key ties across runs).
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


def gpu_wc(eng, data):
    eng.reset()
    eng.map_host(data)
    eng.reduce()
    return eng.result()


def _vocab_text(rng, nkeys, long_frac=0.1):
    ks = set()
    while len(ks) < nkeys:
        L = rng.randrange(16, 60) if rng.random() < long_frac else rng.randrange(1, 16)
        ks.add(bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyzXYZ") for _ in range(L)))
    ks = list(ks)
    rng.shuffle(ks)
    words = ks + [rng.choice(ks) for _ in range(nkeys)]
    rng.shuffle(words)
    return b" ".join(words) + b"\n"


@pytest.mark.parametrize("target", [None, "64", "3000", "1000000"])
def test_sample_sort_bucket_paths(eng, target):
    """Default buckets; tiny buckets (many, through the sample merge sort); buckets of ~3000 (the
    512-thread class of 2049-4096 records, r04); one bucket larger than the LDS sort (the
    in-workgroup global merge path)."""
    data = _vocab_text(random.Random(2), 150_000)
    old = os.environ.get("WCG_SORT_TARGET")
    try:
        if target:
            os.environ["WCG_SORT_TARGET"] = target
        ob.assert_same(gpu_wc(eng, data), ob.merged(data))
    finally:
        if old is None:
            os.environ.pop("WCG_SORT_TARGET", None)
        else:
            os.environ["WCG_SORT_TARGET"] = old


@pytest.mark.parametrize("nkeys,target", [(60_000, "1"), (150_000, "8"), (400_000, "16")])
def test_two_pass_scatter(built, nkeys, target):
    """The large-B scatter's two passes (coarse buckets, then buckets; wcg_sort.h k_ss_sx): ~2
    records per bucket over 32768 buckets, so pass 2's tiles of 4096 records span more than 1024
    buckets (the per-record reservation path); 8 per bucket (tiles spanning ~4 coarse ranges,
    ranked); 16 per bucket over 400k keys.  A fresh
    context each: its first job takes the sample sort whatever its key count (the one-launch
    reduce needs a previous job's count)."""
    import wcg
    data = _vocab_text(random.Random(nkeys), nkeys)
    old = os.environ.get("WCG_SORT_TARGET")
    try:
        os.environ["WCG_SORT_TARGET"] = target
        with wcg.Engine(device=0, max_input_bytes=0, max_keys=1 << 21) as e:
            ob.assert_same(gpu_wc(e, data), ob.merged(data))
            assert e.reduce_path() != 1
    finally:
        if old is None:
            os.environ.pop("WCG_SORT_TARGET", None)
        else:
            os.environ["WCG_SORT_TARGET"] = old


@pytest.mark.parametrize("n", [1, 2, 3, 100, 4095, 4096, 4097, 20_000])
def test_sort_small_counts(eng, n):
    rng = random.Random(n)
    data = _vocab_text(rng, n, long_frac=0.3)
    ob.assert_same(gpu_wc(eng, data), ob.merged(data))


@pytest.mark.parametrize("tail", [1, 2])
def test_bucket_compressed_word_runs(eng, tail):
    """The bucket networks sort one word per record: hi minus the bucket's least hi, then as many
    top bits of lo as fit.  Keys differing in byte 4 (a wide hi range per bucket) and again only in
    bytes 13-14 (below the kept lo bits) tie in that word: runs of 26 are insertion-sorted by the
    full (hi, lo); runs of 676 take the (hi, lo) network again."""
    rng = random.Random(tail)
    al = b"abcdefghijklmnopqrstuvwxyz"
    ks = []
    for c1 in al:
        for t in range(26 ** tail):
            suf = bytes([al[t % 26]]) if tail == 1 else bytes([al[t // 26], al[t % 26]])
            ks.append(b"abcd" + bytes([c1]) + b"efghijkl" + suf)
    words = ks + [rng.choice(ks) for _ in range(len(ks))]
    rng.shuffle(words)
    data = b" ".join(words) + b"\n"
    ob.assert_same(gpu_wc(eng, data), ob.merged(data))
    assert eng.stats()["keys"] == len(ks)


def test_tie_group_of_1e5_long_keys(eng):
    """1e5 distinct keys sharing one 16-byte prefix: one tie group far above the LDS group size,
    sorted by a workgroup-wide bitonic network over scratch (not one lane)."""
    rng = random.Random(7)
    pre = b"sharedprefixabcd"
    ks = set()
    while len(ks) < 100_000:
        ks.add(pre + bytes(rng.choice(b"abcdefghij") for _ in range(rng.randrange(0, 12))))
    words = list(ks) * 2
    rng.shuffle(words)
    data = b" ".join(words) + b"\n"
    out = gpu_wc(eng, data)
    assert out == ob.merged(data)
    assert eng.stats()["keys"] == len(ks)


def test_tie_groups_many_and_deep(eng):
    """Many small groups, and groups whose keys also share bytes 16-31 (and beyond): the cached
    second 16 bytes tie too, so the full-byte comparison decides."""
    rng = random.Random(11)
    words = []
    for g in range(3000):
        p = bytes(rng.choice(b"klmnop") for _ in range(16))
        for _ in range(rng.randrange(2, 6)):
            words.append(p + bytes(rng.choice(b"xy") for _ in range(rng.randrange(0, 4))))
    deep = b"q" * 40
    for _ in range(500):
        words.append(deep + bytes(rng.choice(b"ab") for _ in range(rng.randrange(0, 10))))
    words += [b"r" * L for L in range(14, 40)]               # prefixes of each other
    rng.shuffle(words)
    data = b" ".join(words) + b"\n"
    ob.assert_same(gpu_wc(eng, data), ob.merged(data))


def _runs(counts, k, rng):
    """k disjoint sorted runs of "key: count" lines (keys dealt at random)."""
    parts = [dict() for _ in range(k)]
    for key, c in counts.items():
        parts[rng.randrange(k)][key] = c
    return [wc_ref.merged_output(p) for p in parts]


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8, 9])
def test_merge_runs(built, k):
    import torch
    import wcg
    rng = random.Random(k)
    data = _vocab_text(rng, 40_000, long_frac=0.2)
    pre = b"commonprefix0123"
    data += b" ".join(pre + bytes(rng.choice(b"abc") for _ in range(rng.randrange(0, 8))) for _ in range(3000))
    data += b"\n"
    counts = wc_ref.word_count(data)
    runs = _runs(counts, k, rng)
    if k > 2:
        runs[1] = b""                                         # an owner with no keys
        counts = {}
        for r in runs:
            for line in r.splitlines():
                key, c = line.rsplit(b": ", 1)
                counts[key] = int(c)
    blob = b"".join(runs)
    t = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to("cuda")
    torch.cuda.synchronize()
    with wcg.Engine(0, 0, 1 << 12) as e:                      # small tables: records grow on demand
        nk, nb = e.merge_runs(t.data_ptr(), [len(r) for r in runs])
        ob.assert_same(e.result(), wc_ref.merged_output(counts))
        assert nk == len(counts) and nb == len(blob)
