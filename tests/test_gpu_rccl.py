"""The shuffle and the final Merge inside libwcg over RCCL (wcg_comm_init / wcg_exchange /
wcg_gather_merge), on the device with no host staging.

The box has one MI355X, and RCCL allows one rank per GPU, so the communicator here has world 1:
every kernel, every ncclAllToAll / ncclSend / ncclRecv / ncclAllGather call and the one host read
of the counts run exactly as on a node (the unit counts, send and receive offsets and the import
are those of rank 0 of a world of 1; the per-peer arithmetic for world > 1 is the same loop).
The chain is export -> exchange -> import -> DoReduce -> gather -> merge of the runs, byte for
byte against the oracle (mapreduce.go:214-230 partitioning, :242-263 DoReduce, :284-321 Merge).
"""
import os

import pytest

pytestmark = pytest.mark.gpu


def _corpus(seed=31, size=8 << 20):
    from wcg.corpus import Generator, ASCII, UTF8
    a = Generator(ASCII, 40_000, 1.0, seed).bytes(size)
    u = Generator(UTF8, 20_000, 1.0, seed + 1).bytes(size // 4)
    tail = (b"\n" + b"longkeylongkeylongkey" * 3 + b" " + "ǅ".encode() * 25 + b" zebra "
            + b"abcdefghijklmnopqrstuvwxyz0abcdefghijklmnopqrstuvwxyzA\n")
    return a + u + tail


@pytest.fixture(scope="module")
def engine(built):
    import torch
    import wcg
    with wcg.Engine(device=0, max_input_bytes=0, max_keys=1 << 19) as eng:
        eng.comm_init(wcg.Engine.comm_id(), 0, 1)
        # the bench's arrangement: the engine on a torch stream (set_stream orders the streams)
        s = torch.cuda.Stream()
        eng.set_stream(s.cuda_stream)
        yield eng


def test_exchange_reduce_gather_merge_world1(engine):
    from tests import oracle_bridge as ob
    import torch
    data = _corpus()
    dev = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
    torch.cuda.synchronize()
    want = ob.merged(data)
    engine.enable_timing(2)
    for rep in range(3):                       # reset between jobs is covered too
        engine.reset()
        engine.map_device(dev.data_ptr(), len(data))
        sent, received = engine.exchange(64)
        assert sent == received > 0            # world 1: every unit comes back to this rank
        nk, nb = engine.reduce()               # DoReduce of the owned partitions (all of them)
        run = engine.result()
        ob.assert_same(run, want)
        mk, mb = engine.gather_merge(0)        # Merge of the runs at root
        assert (mk, mb) == (nk, nb)
        ob.assert_same(engine.result(), want)
    ph, launches = engine.timings()
    assert launches == 3
    for k in ("export", "exchange", "import", "gather", "merge"):
        assert ph[k] > 0, (k, ph)
    engine.enable_timing(0)


def test_exchange_empty_input(engine):
    engine.reset()
    assert engine.exchange(3) == (0, 0)
    assert engine.reduce() == (0, 0)
    assert engine.gather_merge(0) == (0, 0)
    assert engine.result() == b""


def test_exchange_then_partitions(engine):
    """After the exchange the engine holds its partitions as DoReduce would: every -res-<r> file
    equals the oracle's (world 1 owns all of them)."""
    from tests import oracle_bridge as ob
    data = _corpus(seed=5, size=2 << 20)
    engine.reset()
    engine.map_host(data)
    engine.exchange(7)
    engine.reduce()
    got = engine.partitions(7)
    ref = ob.Result(data)
    for r in range(7):
        ob.assert_same(got[r], ref.res(7, r))


def test_calls_out_of_order(built):
    import wcg
    from wcg._lib import WcgError, WCG_ESTATE
    with wcg.Engine(device=0, max_keys=1 << 16) as eng:
        eng.map_host(b"alpha beta\n")
        with pytest.raises(WcgError) as ei:
            eng.exchange(3)                    # no communicator yet
        assert ei.value.status == WCG_ESTATE
        eng.comm_init(wcg.Engine.comm_id(), 0, 1)
        with pytest.raises(WcgError) as ei:
            eng.gather_merge(0)                # no reduce result yet
        assert ei.value.status == WCG_ESTATE
        eng.reduce()
        eng.gather_merge(0)
        # the merged result is line records, not keys: partitions and export refuse
        with pytest.raises(WcgError) as ei:
            eng.partitions(3)
        assert ei.value.status == WCG_ESTATE
        with pytest.raises(WcgError) as ei:
            eng.export_count(3, 1)
        assert ei.value.status == WCG_ESTATE
        assert eng.result() == b"alpha: 1\nbeta: 1\n"
