"""GPU parity: the HIP path (through the C ABI) against the oracle, bit-exact.

Small inputs: committed golden fixtures (tests/golden) + edge cases; medium inputs: the C oracle
on seeded corpora; full-size (1 GiB) inputs: oracle too (multi-threaded C, seconds) plus
size-independent properties (token count, sum of counts, sortedness).
"""
import base64
import glob
import json
import os
import random

import pytest

from tests import oracle_bridge as ob
from tests.oracle_bridge import wc_ref

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def eng(built):
    import wcg
    e = wcg.Engine(device=0, max_input_bytes=64 << 20, max_keys=1 << 20)
    yield e
    e.close()


def gpu_wc(eng, data, splits=1):
    eng.reset()
    if splits <= 1:
        eng.map_host(data)
    else:   # cut after '\n' like Split does
        pos = 0
        for k in range(splits):
            end = len(data) if k == splits - 1 else data.find(b"\n", (len(data) * (k + 1)) // splits)
            end = len(data) if end < 0 else end + 1
            if end > pos:
                eng.map_host(data[pos:end])
            pos = max(pos, end)
    nk, nb = eng.reduce()
    out = eng.result()
    assert len(out) == nb
    return out


def golden():
    for p in sorted(glob.glob(os.path.join(GOLDEN, "*.json"))):
        if p.endswith("fnv1a32_kat.json"):
            continue
        yield os.path.basename(p)[:-5], json.load(open(p))


@pytest.mark.parametrize("name", [n for n, _ in golden()])
def test_golden(eng, name):
    d = json.load(open(os.path.join(GOLDEN, name + ".json")))
    data = base64.b64decode(d["input_b64"])
    assert gpu_wc(eng, data) == base64.b64decode(d["merged_b64"])
    for R, files in d["res"].items():
        for r, f in enumerate(files):
            assert eng.partition(int(R), r) == base64.b64decode(f), (name, R, r)
    st = eng.stats()
    assert st["tokens"] == d["ntokens"] and st["keys"] == d["nkeys"]


def test_tile_boundaries(eng):
    # tokens that start/end exactly at 16-byte chunk and 8 KiB tile boundaries, and long keys
    rng = random.Random(5)
    parts = []
    for L in list(range(1, 40)) + [63, 64, 65, 127, 128, 129, 8191, 8192, 8193]:
        parts.append(b"w" * L)
        parts.append(b" " * rng.randrange(1, 3))
    data = b"".join(parts) * 3
    for shift in range(0, 20):
        d = b"x" * shift + b" " + data
        assert gpu_wc(eng, d) == ob.merged(d), shift


def test_utf8_at_tile_boundaries(eng):
    # multi-byte runes straddling every 16-byte chunk and tile position
    for shift in range(0, 17):
        d = (b"a" * shift + "é中𠀀ab中 ".encode() * 3000 + b"\x80\xe4\xb8" * 50 + "ǅ ".encode() * 2000)
        assert gpu_wc(eng, d) == ob.merged(d), shift


def test_random_bytes(eng):
    rng = random.Random(99)
    pool = [b"a", b"Zq", b" ", b"\n", b"\x80", b"\xc3\xa9", b"\xe4\xb8\xad", b"\xf0\xa0\x80\x80", b"\xed\xa0\x80",
            b"\xc0", b"\xff", b"\xe0\xa0", b"\xcc\x81", b"\xc3", b"\x00", b"abcdefghijklmnopq"]
    for _ in range(30):
        n = rng.randrange(1, 50_000)
        out = bytearray()
        while len(out) < n:
            out += rng.choice(pool) if rng.random() < 0.8 else bytes([rng.randrange(256)])
        d = bytes(out)
        ob.assert_same(gpu_wc(eng, d), ob.merged(d))


def test_many_distinct_keys_force_global_path(eng):
    # > LDS slots per workgroup: exercises the global-table miss path and the flush
    keys = [("k%x" % i).translate(str.maketrans("0123456789", "ghijklmnop")).encode() for i in range(300_000)]
    random.Random(3).shuffle(keys)
    d = b" ".join(keys) + b"\n"
    ob.assert_same(gpu_wc(eng, d), ob.merged(d))
    st = eng.stats()
    assert st["global_ops"] > 0


def test_single_hot_key_counts(eng):
    d = b"the " * 2_000_000
    assert gpu_wc(eng, d) == b"the: 2000000\n"


def test_long_keys_and_prefix_ties(eng):
    rng = random.Random(8)
    words = []
    for i in range(4000):
        p = b"commonprefixabcd"                           # 16 bytes shared by all long keys
        tail = bytes(rng.choice(b"xyzXYZ") for _ in range(rng.randrange(0, 30)))
        words.append(p + tail)
    words += [b"q" * rng.randrange(1, 300) for _ in range(500)]
    d = b" ".join(words) + b"\n"
    ob.assert_same(gpu_wc(eng, d), ob.merged(d))


def test_long_keys_hot_cached_and_cell_sizes(eng):
    """k_long: hot long keys counted through the workgroup LDS cache over many rounds, keys at
    the arena cell boundaries (16, 32 bytes in a slot cell; 33+ on the heap) that differ only in
    their last byte, UTF-8 long keys, and the same keys again in a second map call (cells and
    slots kept, cache rebuilt per launch)."""
    rng = random.Random(17)
    base = {L: b"k" * (L - 1) for L in (16, 17, 31, 32, 33, 47, 48, 49, 200)}
    vocab = [b + bytes([c]) for b in base.values() for c in b"abcXYZ"]
    vocab += [("λέξη" * 3 + "中文字符" + "한국어" + s).encode() for s in ("a", "b", "ab", "")]
    hot = vocab[:3]
    words = []
    for _ in range(400_000):
        words.append(rng.choice(hot) if rng.random() < 0.6 else rng.choice(vocab))
    d = b" ".join(words) + b"\n"
    want = ob.merged(d)
    ob.assert_same(gpu_wc(eng, d), want)
    ob.assert_same(gpu_wc(eng, d, splits=3), want)
    st = eng.stats()
    assert st["long_tokens"] == 400_000 and st["overflow"] == 0 and st["spin_fail"] == 0


@pytest.mark.parametrize("mode", [0, 1])
def test_corpus_multi_split(eng, mode):
    from wcg.corpus import Generator
    d = Generator(mode, 50_000, 1.0, 21).bytes(24 << 20)
    want = ob.merged(d)
    ob.assert_same(gpu_wc(eng, d), want)
    assert gpu_wc(eng, d, splits=5) == want        # DoMap per split accumulates (RunSingle M=5)
    st = eng.stats()
    assert st["overflow"] == 0 and st["spin_fail"] == 0


def test_partition_files_match_oracle(eng):
    from wcg.corpus import Generator
    d = Generator(1, 20_000, 1.0, 4).bytes(4 << 20)
    gpu_wc(eng, d)
    r = ob.Result(d)
    for R in (3, 64):
        parts = [eng.partition(R, i) for i in range(R)]
        assert parts == [r.res(R, i) for i in range(R)]
        assert wc_ref.merge_res_files(parts) == r.merged()


def test_export_import_roundtrip(built):
    """the shuffle: export from 2 'ranks', route records by owner, import, merge = oracle"""
    import wcg
    from wcg.corpus import Generator
    d = Generator(0, 30_000, 1.0, 6).bytes(8 << 20)
    d += b" " + b"longkeylongkeylongkey" * 3 + b" " + b"x" * 100 + b"\n"
    cut = d.find(b"\n", len(d) // 2) + 1
    halves = [d[:cut], d[cut:]]
    nranks, R = 2, 64
    senders = [wcg.Engine(0, 16 << 20, 1 << 19) for _ in range(nranks)]
    recvs = [wcg.Engine(0, 0, 1 << 19) for _ in range(nranks)]
    for e, h in zip(senders, halves):
        e.reset(); e.map_host(h)
    for rcv in recvs:
        rcv.reset()
    for e in senders:
        ptr, counts = e.export(R, nranks)
        off = 0
        for dst, c in enumerate(counts):
            if c:   # same process, same device: import straight from the exporter's buffer
                recvs[dst].import_records(ptr + off * wcg.RECORD_BYTES, c)
            off += c
    outs = []
    for i, rcv in enumerate(recvs):
        rcv.reduce()
        outs.append(rcv.result())
    want = ob.merged(d)
    merged_lines = sorted(b"".join(outs).splitlines(keepends=True))
    assert b"".join(merged_lines) == want
    for r in range(nranks):   # each receiver holds exactly the keys it owns
        for line in outs[r].splitlines():
            key = line.rsplit(b": ", 1)[0]
            assert (wcg.ihash(key) % R) % nranks == r


@pytest.mark.slow
def test_full_size_c2(built):
    """BASELINE config 2 at full size (1 GiB ASCII Zipf, V=1e5, s=1.0, seed 42) from device memory."""
    import torch
    import wcg
    from wcg.corpus import Generator, CONFIGS
    cfg = CONFIGS["c2_ascii_zipf_1gib"]
    n = cfg["nbytes"]
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    Generator(cfg["mode"], cfg["vocab"], cfg["zipf_s"], cfg["seed"]).fill_ptr(host.data_ptr(), n)
    dev = host.to("cuda")
    with wcg.Engine(0, 0, 1 << 20) as e:
        e.reset()
        e.map_device(dev.data_ptr(), n)
        nk, nb = e.reduce()
        got = e.result()
        st = e.stats()
    data = host.numpy().tobytes()
    r = ob.Result(data, 16)
    ob.assert_same(got, r.merged())
    assert st["tokens"] == r.ntokens and nk == r.nkeys


@pytest.mark.slow
def test_full_size_c2_second_job_fused(built):
    """The headline's reduce path at full size: C2 run as two jobs on one engine,
    as bench.py's timed steps run it.  The first job takes the multi-launch reduce (no hint yet);
    the second, with the first job's key count as its hint, takes the one-launch k_fused_reduce
    (1e5 keys, 1.8e8 tokens) - both merged files byte for byte against the oracle."""
    import torch
    import wcg
    from wcg.corpus import Generator, CONFIGS
    cfg = CONFIGS["c2_ascii_zipf_1gib"]
    n = cfg["nbytes"]
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    Generator(cfg["mode"], cfg["vocab"], cfg["zipf_s"], cfg["seed"]).fill_ptr(host.data_ptr(), n)
    dev = host.to("cuda")
    data = host.numpy().tobytes()
    r = ob.Result(data, 16)
    want = r.merged()
    with wcg.Engine(0, 0, 1 << 20) as e:
        for job, path in ((0, 0), (1, 1)):
            e.reset()
            e.map_device(dev.data_ptr(), n)
            nk, nb = e.reduce()
            assert e.reduce_path() == path, f"job {job}: reduce path {e.reduce_path()}, expected {path}"
            ob.assert_same(e.result(), want)
            assert nk == r.nkeys and e.stats()["tokens"] == r.ntokens


@pytest.mark.parametrize("shape", ["mixed_16_50", "exactly_16", "runs_100_300"])
def test_long_token_lengths(built, shape):
    """Inputs made only of long tokens (every step logs dozens): each logged length must be the
    token's (a spilled prefetch register once gave whole steps stale letter masks, so lengths of
    1-5 bytes), repeats fold in k_long_hash's cache, partitions aggregate in k_long_agg."""
    import wcg
    rng = random.Random({"mixed_16_50": 1, "exactly_16": 2, "runs_100_300": 3}[shape])
    if shape == "mixed_16_50":
        words = [bytes(rng.choice(b"abcdefgh") for _ in range(rng.randrange(16, 50))) for _ in range(3000)]
        data = b" ".join(rng.choice(words) for _ in range(100_000)) + b"\n"
    elif shape == "exactly_16":
        words = [bytes(rng.choice(b"abcdefgh") for _ in range(16)) for _ in range(3000)]
        data = b" ".join(rng.choice(words) for _ in range(100_000)) + b" " + b" ".join(words) + b"\n"
    else:                                   # runs past the 1 KiB window: walked by k_long_hash
        words = [bytes(rng.choice(b"abcdefgh") for _ in range(rng.randrange(100, 300))) for _ in range(300)]
        data = b" ".join(rng.choice(words) for _ in range(20_000)) + b"\n"
    with wcg.Engine(0, 0, 1 << 20) as e:
        e.reset()
        e.map_host(data)
        e.reduce()
        ob.assert_same(e.result(), ob.merged(data))
        assert e.stats()["overflow"] == 0


@pytest.mark.parametrize("calls", [1, 2])
def test_high_cardinality_spill_and_record_log(built, calls):
    """~3M distinct inline keys (one map call, or two that share a third of them): k_agg's pass-1
    tables overflow, entries and table flushes spill to k_rp's sub-buckets, pass 2 emits each key
    as a record; one call emits every key once (no merge, no global-table scan), two calls emit
    shared keys twice and the records are merged after the sort."""
    import wcg
    rng = random.Random(9)
    alpha = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJ"
    keys = list({bytes(rng.choice(alpha) for _ in range(rng.randrange(3, 16))) for _ in range(3_100_000)})
    third = len(keys) // 3
    d1 = b" ".join(keys[: 2 * third] + keys[:50_000]) + b"\n"
    d2 = b" ".join(keys[third:] + keys[:50_000]) + b"\n"
    with wcg.Engine(0, 0, 8_000_000) as e:        # > 4M keys: the two-pass aggregation
        e.reset()
        e.map_host(d1)
        if calls == 2:
            e.map_host(d2)
        e.reduce()
        data = d1 + d2 if calls == 2 else d1
        ob.assert_same(e.result(), ob.merged(data))
        st = e.stats()
        assert st["keys"] == (len(keys) if calls == 2 else 2 * third) and st["emitted"] > 0
