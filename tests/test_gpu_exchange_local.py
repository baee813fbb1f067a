"""The multi-GPU shuffle and Merge for worlds 2..8 on one MI355X: W contexts stand in for the W
ranks of a node, and wcg_exchange_local / wcg_gather_merge_local run the code of wcg_exchange /
wcg_gather_merge (the count matrix, the plan of wcg_exchange_plan / wcg_gather_plan, the export,
import, DoReduce and merge kernels) with device copies in place of the RCCL sends and receives
(one GPU cannot host several RCCL ranks).  Checked byte for byte against the oracle:
  * after the exchange, context p holds exactly the partitions r with r % W == p, and each of
    its -res-<r> files equals the reference's DoReduce output for r (mapreduce.go:242-280);
  * the merged file at root (root = 0 and root != 0) equals Merge's (mapreduce.go:284-321).
What this leaves to the 8-GPU node: only ncclSend/ncclRecv pairing of the same plan.
"""
import pytest

pytestmark = pytest.mark.gpu


def _corpus(seed, size=3 << 20):
    from wcg.corpus import Generator, ASCII, UTF8
    a = Generator(ASCII, 30_000, 1.0, seed).bytes(size)
    u = Generator(UTF8, 10_000, 1.0, seed + 1).bytes(size // 4)
    tail = (b"\n" + b"longkeylongkeylongkey" * 3 + b" " + "ǅ".encode() * 25 + b" zebra "
            + b"abcdefghijklmnopqrstuvwxyz0abcdefghijklmnopqrstuvwxyzA\n")
    return a + u + tail


def _ranges(data, W):
    from wcg.distributed import line_aligned_ranges
    return line_aligned_ranges(len(data), W, lambda i: data[i])


@pytest.mark.parametrize("W,root,nreduce", [(2, 1, 64), (3, 2, 7), (4, 0, 64), (5, 3, 3), (8, 5, 64), (8, 0, 1)])
def test_exchange_gather_local(built, W, root, nreduce):
    import wcg
    from tests import oracle_bridge as ob
    data = _corpus(seed=40 + W)
    ref = ob.Result(data)
    want = ref.merged()
    engines = [wcg.Engine(device=0, max_keys=1 << 18) for _ in range(W)]
    try:
        for rep in range(2):                           # buffers are reused on the second job
            for e, (a, b) in zip(engines, _ranges(data, W)):
                e.reset()
                e.map_host(data[a:b])
            sent, received = wcg.exchange_local(engines, nreduce)
            assert sum(sent) == sum(received)
            paths = []
            for p, e in enumerate(engines):
                e.reduce()
                paths.append(e.reduce_path())
                if nreduce >= W:
                    parts = e.partitions(nreduce)
                    for r in range(nreduce):
                        if r % W == p:
                            ob.assert_same(parts[r], ref.res(nreduce, r))
                        else:
                            assert parts[r] == b"", (p, r)
                    e.reduce()                         # partitions() reordered the records: sort again
            # the owners' reduce of the second job (imported keys) takes the one-launch reduce
            # wherever the first job left a key count
            assert (1 in paths) == (rep == 1), paths
            nk, nb = wcg.gather_merge_local(engines, root)
            assert nk == ref.nkeys and nb == len(want)
            ob.assert_same(engines[root].result(), want)
    finally:
        for e in engines:
            e.close()


def test_exchange_local_empty_ranks(built):
    """Ranks with no input and a rank that owns nothing (nreduce < world)."""
    import wcg
    from tests import oracle_bridge as ob
    data = b"alpha beta gamma\nalpha delta\n" * 1000
    W = 4
    engines = [wcg.Engine(device=0, max_keys=1 << 16) for _ in range(W)]
    try:
        for e in engines:
            e.reset()
        engines[2].map_host(data)                      # only rank 2 has input
        sent, received = wcg.exchange_local(engines, 2)   # partitions 0, 1: ranks 2 and 3 own nothing
        assert sent[0] == sent[1] == sent[3] == 0
        assert received[2] == received[3] == 0
        for e in engines:
            e.reduce()
        assert engines[3].result() == b""
        nk, nb = wcg.gather_merge_local(engines, 3)
        ob.assert_same(engines[3].result(), ob.merged(data))
    finally:
        for e in engines:
            e.close()


def test_reduce_twice_and_after_free(built):
    """a second wcg_reduce with no map in between, and wcg_free of the output
    followed by wcg_reduce, on a context whose previous job set the device-sized plan."""
    import wcg
    from tests import oracle_bridge as ob
    data = _corpus(seed=77, size=1 << 20)
    want = ob.merged(data)
    with wcg.Engine(device=0, max_keys=1 << 18) as e:
        for _ in range(2):                             # the second job runs device-sized
            e.reset()
            e.map_host(data)
            e.reduce()
            ob.assert_same(e.result(), want)
        for _ in range(3):
            nk, nb = e.reduce()
            assert nb == len(want)
            ob.assert_same(e.result(), want)
        ptr, _ = e.result_device()
        e.free(ptr)
        e.reduce()
        ob.assert_same(e.result(), want)
        e.partitions(5)                                # partition, then reduce again
        e.reduce()
        ob.assert_same(e.result(), want)


def test_exchange_local_full_table_fails_every_context(built):
    """the status agreement of wcg_exchange, driven through
    wcg_exchange_local.  One context's table overflows (max_keys far below the keys of its range):
    the exchange fails on every context with that status, the others' errors name the failed
    rank, no data moves, and the healthy context still reduces its own range exactly."""
    import wcg
    from tests import oracle_bridge as ob
    data = _corpus(seed=91, size=1 << 20)
    (a0, b0), (a1, b1) = _ranges(data, 2)
    engines = [wcg.Engine(device=0, max_keys=1 << 18), wcg.Engine(device=0, max_keys=1 << 7)]
    try:
        for e, (a, b) in zip(engines, [(a0, b0), (a1, b1)]):
            e.reset()
            e.map_host(data[a:b])
        with pytest.raises(wcg.WcgError) as ei:
            wcg.exchange_local(engines, 4)
        from wcg._lib import WCG_EFULL
        assert ei.value.status == WCG_EFULL
        assert "rank 1 failed" in str(ei.value)              # context 0's error names the rank
        engines[0].reduce()
        ob.assert_same(engines[0].result(), ob.merged(data[a0:b0]))
    finally:
        for e in engines:
            e.close()
