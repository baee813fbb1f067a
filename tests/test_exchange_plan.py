"""The host-side plan of the multi-GPU shuffle and of Merge's gather (wcg_exchange_plan /
wcg_gather_plan in libwcg.so: the arithmetic wcg_exchange and wcg_gather_merge run between their
count all-gather and their RCCL sends / receives), checked on the CPU for worlds 2..8 against a
plain Python model, with empty peers, one-sided traffic and root != 0.

Reference semantics: DoMap writes partition r = ihash(key) % nReduce (mapreduce.go:214-230) and
DoReduce r reads partition r of every map job in map-job order (mapreduce.go:242-263); here rank d
receives from every rank s in rank order, so the units from s land after those of ranks < s.
"""
import random

import pytest


def model_exchange(counts, rank):
    W = len(counts)
    send_cnt = list(counts[rank])
    send_off = [sum(send_cnt[:d]) for d in range(W)]
    recv_cnt = [counts[s][rank] for s in range(W)]
    recv_off = [sum(recv_cnt[:s]) for s in range(W)]
    return {"send_off": send_off, "send_cnt": send_cnt, "recv_off": recv_off, "recv_cnt": recv_cnt,
            "sent": sum(send_cnt), "received": sum(recv_cnt)}


def matrices(W, rng):
    yield [[0] * W for _ in range(W)]                                  # nothing moves
    yield [[rng.randrange(1, 1000) for _ in range(W)] for _ in range(W)]   # dense
    m = [[rng.choice([0, 0, rng.randrange(1, 10 ** 7)]) for _ in range(W)] for _ in range(W)]
    yield m                                                            # sparse: empty peers
    yield [[(7 if s == 0 else 0) for d in range(W)] for s in range(W)]   # only rank 0 sends
    yield [[(5 if d == W - 1 else 0) for d in range(W)] for s in range(W)]   # all to the last rank
    yield [[(2 ** 40 + s * W + d) for d in range(W)] for s in range(W)]  # 64-bit counts


@pytest.mark.parametrize("W", range(1, 9))
def test_exchange_plan_matches_model(built, W):
    import wcg
    rng = random.Random(W)
    for m in matrices(W, rng):
        for rank in range(W):
            assert wcg.exchange_plan(m, rank) == model_exchange(m, rank), (W, rank, m)


@pytest.mark.parametrize("W", range(2, 9))
def test_exchange_plan_is_consistent_between_peers(built, W):
    """What s sends to d (its send slice for d) has exactly the size d reserves for s, and every
    receive buffer is covered once, in source order, with no gaps or overlaps."""
    import wcg
    rng = random.Random(100 + W)
    for m in matrices(W, rng):
        plans = [wcg.exchange_plan(m, r) for r in range(W)]
        for s in range(W):
            for d in range(W):
                assert plans[s]["send_cnt"][d] == plans[d]["recv_cnt"][s]
        for d in range(W):
            p = plans[d]
            end = 0
            for s in range(W):
                assert p["recv_off"][s] == end
                end += p["recv_cnt"][s]
            assert end == p["received"]
        assert sum(p["sent"] for p in plans) == sum(p["received"] for p in plans)


@pytest.mark.parametrize("W", range(1, 9))
def test_gather_plan_root_placement(built, W):
    import wcg
    rng = random.Random(7 * W)
    for _ in range(5):
        sizes = [rng.choice([0, rng.randrange(1, 10 ** 9)]) for _ in range(W)]
        for root in range(W):
            off, total = wcg.gather_plan(sizes, root)
            assert total == sum(sizes)
            assert off == [sum(sizes[:p]) for p in range(W)]
            # root's own run goes to off[root]: the runs are back to back in rank order whatever the root
            assert off[root] + sizes[root] == (off[root + 1] if root + 1 < W else total)


def test_plans_refuse_bad_arguments(built):
    import wcg
    from wcg._lib import WcgError
    with pytest.raises(WcgError):
        wcg.exchange_plan([[1, 2], [3, 4]], 2)          # rank outside the world
    with pytest.raises(WcgError):
        wcg.gather_plan([1, 2, 3], 3)                   # root outside the world
    with pytest.raises(WcgError):
        wcg.gather_plan([], 0)
