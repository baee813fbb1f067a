"""Diagnostics: long-key counting on small inputs, GPU vs oracle, printing differences."""
import os, sys, random
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mit-6.824-2015_amd")]
import torch  # noqa: F401  (one HIP runtime: torch first)
import wcg
from tests import oracle_bridge as ob

def run(name, data):
    with wcg.Engine(0, 0, 1 << 16) as e:
        e.reset(); e.map_host(data); e.reduce()
        got = e.result(); st = e.stats()
    want = ob.merged(data)
    if got == want:
        print(name, "OK", st, flush=True); return
    g = dict(l.rsplit(b": ", 1) for l in got.splitlines())
    w = dict(l.rsplit(b": ", 1) for l in want.splitlines())
    bad = [(k, g.get(k), w.get(k)) for k in set(g) | set(w) if g.get(k) != w.get(k)]
    print(name, "DIFF", len(bad), st, flush=True)
    for k, a, b in sorted(bad)[:12]:
        print("   ", k[:60], "gpu", a, "oracle", b, flush=True)

rng = random.Random(1)
run("one42", b"longkeylongkeylongkey" * 2 + b"\n")
run("two42", (b"longkeylongkeylongkey" * 2 + b" ") * 2 + b"\n")
run("one20", b"abcdefghijklmnopqrst\n")
run("mix", b"abcdefghijklmnopqrst zebra " + b"abcdefghijklmnopqrst " * 3 + "ǅ".encode() * 20 + b"\n")
words = [bytes(rng.choice(b"abcdefgh") for _ in range(rng.randrange(16, 50))) for _ in range(3000)]
run("many", b" ".join(rng.choice(words) for _ in range(100000)) + b"\n")
w16 = [bytes(rng.choice(b"abcdefgh") for _ in range(16)) for _ in range(3000)]
run("w16", b" ".join(rng.choice(w16) for _ in range(100000)) + b"\n")
run("w16distinct", b" ".join(w16) + b"\n")
wl = [bytes(rng.choice(b"abcdefgh") for _ in range(rng.randrange(100, 300))) for _ in range(300)]
run("walks", b" ".join(rng.choice(wl) for _ in range(20000)) + b"\n")
