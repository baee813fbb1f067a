"""GPU: a stream of jobs dealt in turn to two contexts, each on its own HIP stream (r06, bench.py's
multi-context loop).  One job's k_map then runs beside the other context's k_agg,
one-launch reduce and clear; the contexts share nothing but the read-only input.  Every job's
merged file is compared byte for byte with the C oracle when its context is reused (after
wcg_reduce_wait), so a job whose tables another job's kernels touched would show up here."""
import pytest

from tests import oracle_bridge as ob

pytestmark = pytest.mark.gpu


def _touch(torch, streams):
    # HIP deals hardware queues at a stream's first use: give both their first work in turn
    for s in streams:
        with torch.cuda.stream(s):
            torch.zeros(1, device="cuda:0")
    torch.cuda.synchronize()


# C2's corpus (one-pass jobs: split miss buckets, the one-launch reduce from a context's second job
# on) and C4-like mixed UTF-8 text in a context sized for 8 Mi keys (two-pass jobs: k_rp, pass 2,
# the forked long-key kernels and the multi-launch sort)
@pytest.mark.parametrize("mode,vocab,zipf,nbytes,keys", [(0, 100_000, 1.0, 64 << 20, 1 << 18),
                                                         (1, 1_000_000, 0.9, 32 << 20, 8 << 20)])
def test_jobs_dealt_to_two_contexts(built, mode, vocab, zipf, nbytes, keys):
    import torch
    import wcg
    from wcg.corpus import Generator
    gen = Generator(mode, vocab, zipf, 45)
    # three different inputs (generator blocks 0, 40, 80), resident in HBM
    datas = [gen.bytes(nbytes, first_block=k * 40) for k in range(3)]
    wants = [ob.merged(d, 16) for d in datas]
    devs = [torch.frombuffer(bytearray(d), dtype=torch.uint8).to("cuda:0") for d in datas]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    _touch(torch, streams)
    engs = []
    try:
        for s in streams:
            e = wcg.Engine(device=0, max_input_bytes=0, max_keys=keys)
            e.set_stream(s.cuda_stream)
            engs.append(e)
        last = [None, None]                      # the job each context ran last
        checked = 0
        for i in range(10):
            j = i % 2
            e = engs[j]
            if last[j] is not None:
                e.reduce_wait()
                ob.assert_same(e.result(), wants[last[j]])
                checked += 1
            e.reset()
            e.map_device(devs[i % 3].data_ptr(), nbytes)
            e.reduce_async()
            last[j] = i % 3
        for j in range(2):
            engs[j].reduce_wait()
            ob.assert_same(engs[j].result(), wants[last[j]])
            checked += 1
        assert checked == 10
    finally:
        for e in engs:
            e.close()
