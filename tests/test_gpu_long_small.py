"""GPU: k_long_small (r05, csrc/wcg_map.h) - the long-key work of a one-pass map call in one
workgroup, taken when the context's previous job logged at most 4096 long tokens.  Every job runs
on one context after a priming job with a few long tokens, so the small path is the one taken, and
is compared byte for byte with the C oracle:
  * hot and cold long keys, keys sharing a 16-byte prefix, UTF-8 long keys, 16..300-byte keys;
  * runs whose length k_map leaves open (they reach a window's look-ahead chunk: walked here),
    including ones that end up 15 bytes or shorter (counted as inline keys);
  * more distinct long keys than the LDS slot table holds (fenced fallback inserts);
  * tens of thousands of long tokens (many rounds), after which the hint sends the next job back
    to k_long_hash + k_long_agg, and the small path again after a job with few."""
import random

import pytest

from tests import oracle_bridge as ob

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(built):
    import wcg
    e = wcg.Engine(device=0, max_input_bytes=64 << 20, max_keys=1 << 18)
    yield e
    e.close()


def run(eng, data):
    eng.reset()
    eng.map_host(data)
    eng.reduce()
    st = eng.stats()
    ob.assert_same(eng.result(), ob.merged(data))
    assert st["overflow"] == 0 and st["spin_fail"] == 0
    return st


def prime(eng):
    st = run(eng, b"short words only and one loooooooooooooooooooooooong token\n" * 3)
    assert 0 < st["long_tokens"] <= 4096


def nlong(data):
    return sum(1 for t in ob.tokens(data) if len(t) > 15)


def filler(rnd, n):
    return " ".join("".join(rnd.choice("abcdefgh") for _ in range(1 + rnd.randrange(7))) for _ in range(n))


def test_mixed_long_keys(eng):
    rnd = random.Random(5)
    prime(eng)
    pre = "sharedprefixabcd"                                   # 16 bytes
    keys = [pre + "".join(rnd.choice("xyz") for _ in range(1 + rnd.randrange(12))) for _ in range(40)]
    keys += ["".join(rnd.choice("klmnop") for _ in range(16 + rnd.randrange(284))) for _ in range(60)]
    keys += ["λόγος" * (4 + rnd.randrange(6)) for _ in range(5)] + ["Straße" * 4, "日本語テキスト" * 3]
    parts = []
    for i in range(3000):
        parts.append(filler(rnd, 3))
        k = keys[0] if i % 3 == 0 else keys[rnd.randrange(len(keys))]     # one hot long key
        parts.append(k)
    data = (" ".join(parts) + "\n").encode()
    st = run(eng, data)
    assert st["long_tokens"] == nlong(data) == 3000


def test_open_length_runs_at_window_ends(eng):
    """Tokens placed across every offset near the 992-byte step edges: some reach the look-ahead
    chunk with their length open (walked by the kernel), long or 15 bytes and shorter."""
    rnd = random.Random(6)
    prime(eng)
    out = bytearray()
    for k in range(400):
        step_end = (len(out) // 992 + 1) * 992
        gap = step_end - len(out) - rnd.randrange(1, 40)
        out += b" " * max(1, gap)
        n = rnd.choice([3, 9, 14, 15, 16, 17, 31, 64, 200, 1100])
        out += "".join(rnd.choice("abcdefghijklmnopqrstuvwxyzé") for _ in range(n)).encode()
        out += b" " + filler(rnd, 5).encode()
    out += b"\n"
    run(eng, bytes(out))


def test_more_distinct_long_keys_than_slots(eng):
    rnd = random.Random(7)
    prime(eng)
    keys = ["longdistinctkey" + "".join(rnd.choice("abcdefghijklmnop") for _ in range(12)) for _ in range(3500)]
    data = (" ".join(keys + keys[:500]) + "\n").encode()
    st = run(eng, data)
    assert st["long_tokens"] == nlong(data) == 4000


def test_many_long_tokens_then_few(eng):
    rnd = random.Random(8)
    prime(eng)
    keys = ["manyroundslongkey" + "".join(chr(97 + (i >> (4 * k)) % 16) for k in range(3)) for i in range(300)]
    big = (" ".join(keys[rnd.randrange(300)] for _ in range(50_000)) + "\n").encode()
    st = run(eng, big)                                          # small path, ~49 rounds
    assert st["long_tokens"] == 50_000
    run(eng, big)                                               # hint > 4096: the partitioned kernels
    run(eng, b"few long tokens: abcdefghijklmnopqrstuvwxyz abcdefghijklmnopqrstuvwxyz\n")
    run(eng, big[: len(big) // 3].rsplit(b" ", 1)[0] + b"\n")   # hint 2: small again


def test_large_context_jobs_do_not_leak_long_keys(built):
    """a large context (max_keys > 4M: two-pass aggregation, and wcg_reset clears
    only the listed table claims) runs jobs with different long-key sets, two map calls each, with
    a reset between them; every job's output must be its own input's, exactly (a claim missing
    from the list would leave an earlier job's key behind)."""
    import wcg
    rnd = random.Random(11)
    with wcg.Engine(device=0, max_input_bytes=16 << 20, max_keys=5_000_000) as e:
        for job in range(3):
            keys = [f"job{'abc'[job]}longkey" + "".join(rnd.choice("defghijkl") for _ in range(8 + job * 5))
                    for _ in range(400)]
            calls = [(" ".join(rnd.choice(keys) for _ in range(3000)) + " " + filler(rnd, 500) + "\n").encode()
                     for _ in range(2)]
            e.reset()
            for c in calls:
                e.map_host(c)
            e.reduce()
            ob.assert_same(e.result(), ob.merged(b"".join(calls)))
