"""GPU: parity at the configs' scale and over the whole Unicode range, bit-exact.

  * every Unicode scalar value 0x80-0x10FFFF through the kernel's UTF-8 decoder and letter
    table, one per token and in runs that straddle 16-byte chunks, against the C oracle;
  * C4's key cardinality: the first GiB of the C4 generator (2.4e7 distinct keys) through
    several wcg_map_device calls into one context sized for 5e7 keys;
  * the 64 GiB job's call size: 16 GiB of C4 in two 8 GiB calls, verified exactly;
  * a C3-shaped job: 2 GiB of the C3 generator, nReduce = 64, all 64 -res-<r> files;
  * C3 at its full size: 16 GiB in one wcg_map_device call, verified exactly (r06).
"""
import pytest

from tests import oracle_bridge as ob

pytestmark = pytest.mark.gpu


def _scalars():
    return [cp for cp in range(0x80, 0x110000) if not (0xD800 <= cp <= 0xDFFF)]


@pytest.mark.parametrize("layout", ["separated", "runs"])
def test_every_unicode_scalar(built, layout):
    import wcg
    cps = _scalars()
    if layout == "separated":
        data = b" ".join(chr(cp).encode() for cp in cps) + b"\n"
    else:
        # runs of 1..7 code points with 0..15 ASCII letters in front, so runs start at every
        # byte offset of a 16-byte chunk and straddle chunk edges
        parts, i, k = [], 0, 0
        while i < len(cps):
            n = 1 + k % 7
            parts.append(b"a" * (k % 16) + "".join(chr(c) for c in cps[i:i + n]).encode() + b"\x80" * (k % 2) + b" ")
            i += n
            k += 1
        data = b"".join(parts) + b"\n"
    with wcg.Engine(0, 0, 1 << 21) as e:
        e.reset()
        e.map_host(data)
        e.reduce()
        ob.assert_same(e.result(), ob.merged(data))


@pytest.fixture(scope="module")
def c4_gen(built):
    from wcg.corpus import Generator, CONFIGS
    cfg = CONFIGS["c4_utf8_zipf_64gib"]
    print("c4: building the 5e7-word generator", flush=True)
    return Generator(cfg["mode"], cfg["vocab"], cfg["zipf_s"], cfg["seed"])


@pytest.fixture(scope="module")
def c4_gib(c4_gen):
    import torch
    n = 1 << 30
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    c4_gen.fill_ptr(host.data_ptr(), n)
    print("c4: 1 GiB generated", flush=True)
    return host


@pytest.mark.timeout(600)
def test_c4_gib_5e7_key_table_multi_call(c4_gib):
    import torch
    import wcg
    host = c4_gib
    n = host.numel()
    data = host.numpy().tobytes()
    dev = host.to("cuda")
    torch.cuda.synchronize()
    q = n // 4                                               # 1 MiB generator blocks end in '\n'
    with wcg.Engine(0, 0, 50_000_000) as e:
        e.reset()
        for k in range(4):                                   # four DoMap calls into one table
            e.map_device(dev.data_ptr() + k * q, q)
        nk, nb = e.reduce()
        got = e.result()
        st = e.stats()
    print(f"c4: GPU done, {nk} keys; oracle counting", flush=True)
    r = ob.Result(data, 16)
    assert nk == r.nkeys and nk > 20_000_000
    assert st["tokens"] == r.ntokens and st["overflow"] == 0
    ob.assert_same(got, r.merged())


@pytest.mark.timeout(600)
def test_c4_4gib_sixteen_calls_record_log_overflow(c4_gen):
    """Many DoMap calls into one two-pass job: 16 calls of 256 MiB emit ~1.3e8 pass-2 records,
    more than the record log holds (max_keys), so later calls fall back to global-table inserts
    and the reduce merges log and table.  Checked exactly by the oracle's verifier (the 64 GiB
    run of tools/c4_full.py uses the same check)."""
    import numpy as np
    import torch
    import wcg
    n, q = 4 << 30, 256 << 20
    host = np.empty(n, dtype=np.uint8)
    c4_gen.fill_ptr(host.ctypes.data, n)
    dev = torch.from_numpy(host).to("cuda")
    torch.cuda.synchronize()
    with wcg.Engine(0, 0, 50_000_000) as e:
        e.reset()
        for k in range(n // q):
            e.map_device(dev.data_ptr() + k * q, q)
        nk, _ = e.reduce()
        got = e.result()
        st = e.stats()
    del dev
    assert st["emitted"] > 50_000_000 + 65536 and st["global_ops"] > 0 and st["overflow"] == 0
    print(f"c4 4 GiB: {nk} keys, {st['emitted']} records emitted; verifying", flush=True)
    ok, msg, ntok, nkeys = ob.verify_merged(host.ctypes.data, n, got, 16)
    assert ok, msg
    assert ntok == st["tokens"] and nkeys == nk


@pytest.mark.timeout(600)
def test_c4_16gib_two_8gib_calls(c4_gen):
    """The 64 GiB job's call size (tools/c4_full.py: 8 GiB per wcg_map_device) at a quarter of its
    length: 16 GiB of the C4 generator in two 8 GiB calls into one 5e7-key context.  Each call's
    pass 2 emits more records than the record log holds, so the second call's records go to the
    global table and the reduce merges log and table.  Checked exactly by the oracle's verifier
    (every input token decrements its line's count; keys strictly ascending).  ~2 minutes: 25 s
    to generate, a few s on the GPU, ~70 s to verify on 16 threads."""
    import threading
    import time
    import numpy as np
    import torch
    import wcg
    from wcg.corpus import BLOCK
    n, q, gib = 16 << 30, 8 << 30, 1 << 30
    host = np.empty(n, dtype=np.uint8)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    for g in range(n // gib):
        a = g * gib
        c4_gen.fill_ptr(host.ctypes.data + a, gib, first_block=a // BLOCK, threads=16)
        dev[a:a + gib].copy_(torch.from_numpy(host[a:a + gib]))
    torch.cuda.synchronize()
    print("c4 16 GiB: generated", flush=True)
    with wcg.Engine(0, 0, 50_000_000) as e:
        e.reset()
        for k in range(n // q):
            e.map_device(dev.data_ptr() + k * q, q)
        nk, _ = e.reduce()
        got = e.result()
        st = e.stats()
    del dev
    assert st["emitted"] > 50_000_000 and st["global_ops"] > 0 and st["overflow"] == 0 and nk > 20_000_000
    print(f"c4 16 GiB: {nk} keys, {st['emitted']} records emitted; verifying", flush=True)
    res = {}
    th = threading.Thread(target=lambda: res.update(v=ob.verify_merged(host.ctypes.data, n, got, 16)), daemon=True)
    t0 = time.perf_counter()
    th.start()
    while th.is_alive():
        th.join(20)
        print(f"c4 16 GiB: verifying ({time.perf_counter() - t0:.0f} s)", flush=True)
    ok, msg, ntok, nkeys = res["v"]
    assert ok, msg
    assert ntok == st["tokens"] and nkeys == nk


@pytest.mark.timeout(600)
def test_c3_shaped_2gib_nreduce_64(built):
    import torch
    import wcg
    from wcg.corpus import Generator, CONFIGS
    cfg = CONFIGS["c3_ascii_zipf_16gib"]
    n = 2 << 30
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    Generator(cfg["mode"], cfg["vocab"], cfg["zipf_s"], cfg["seed"]).fill_ptr(host.data_ptr(), n)
    dev = host.to("cuda")
    torch.cuda.synchronize()
    with wcg.Engine(0, 0, 1 << 20) as e:
        e.reset()
        e.map_device(dev.data_ptr(), n)
        e.reduce()
        parts = e.partitions(64)
        merged = e.result()
    del dev
    r = ob.Result(host.numpy().tobytes(), 16)
    ob.assert_same(merged, r.merged())
    assert parts == [r.res(64, i) for i in range(64)]


@pytest.mark.timeout(600)
def test_c3_full_16gib_one_call(built):
    """BASELINE config 3 at its full size on one GPU, as bench.py maps it: 16 GiB of the C3 generator
    in ONE wcg_map_device call (the miss log, region sizes and 32-bit unit offsets at their largest
    one-pass extent), then DoReduce + Merge; checked exactly by the oracle's verifier (every input
    token decrements its line's count; keys strictly ascending).  ~1-2 minutes."""
    import threading
    import time
    import numpy as np
    import torch
    import wcg
    from wcg.corpus import Generator, CONFIGS, BLOCK
    cfg = CONFIGS["c3_ascii_zipf_16gib"]
    gen = Generator(cfg["mode"], cfg["vocab"], cfg["zipf_s"], cfg["seed"])
    n, gib = 16 << 30, 1 << 30
    host = np.empty(n, dtype=np.uint8)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    for g in range(n // gib):
        a = g * gib
        gen.fill_ptr(host.ctypes.data + a, gib, first_block=a // BLOCK, threads=16)
        dev[a:a + gib].copy_(torch.from_numpy(host[a:a + gib]))
    torch.cuda.synchronize()
    print("c3 16 GiB: generated", flush=True)
    keys_cap = max(min(2 * cfg["vocab"], n // 32), 1 << 18)     # as bench.py sizes it
    with wcg.Engine(0, 0, keys_cap) as e:
        e.reset()
        e.map_device(dev.data_ptr(), n)
        nk, _ = e.reduce()
        got = e.result()
        st = e.stats()
    del dev
    assert st["overflow"] == 0 and nk == cfg["vocab"]
    res = {}
    th = threading.Thread(target=lambda: res.update(v=ob.verify_merged(host.ctypes.data, n, got, 16)), daemon=True)
    t0 = time.perf_counter()
    th.start()
    while th.is_alive():
        th.join(20)
        print(f"c3 16 GiB: verifying ({time.perf_counter() - t0:.0f} s)", flush=True)
    ok, msg, ntok, nkeys = res["v"]
    assert ok, msg
    assert ntok == st["tokens"] and nkeys == nk
