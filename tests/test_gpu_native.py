"""A C caller of the boundary: tests/native/run_single_gpu.c replays
INTEGRATION.md's cgo runSingleGPU (RunSingle, mapreduce.go:344-356) call for call through
libwcg.so - Split into nMap files (P1), one read of at most 1 GiB per split (P2), wcg_map per
split, wcg_reduce, the wcg_partition size query then copy for every -res-<r>, wcg_result_copy,
wcg_result_device + wcg_free - then the same job through wcg_reduce_async / wcg_reduce_wait, and
the world-1 RCCL sequence (wcg_comm_id / wcg_comm_init / wcg_exchange / wcg_reduce /
wcg_gather_merge).  Every file it writes is diffed against the oracle."""
import os
import subprocess

import pytest

from tests import oracle_bridge as ob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "bin", "run_single_gpu")


def test_harness_built_and_linked(built):
    """(CPU) the harness links against libwcg.so and refuses a bad command line"""
    assert os.path.exists(EXE)
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("nmap,nreduce", [(5, 3), (7, 64)])
def test_run_single_gpu_c_harness(built, tmp_path, nmap, nreduce):
    from wcg.corpus import Generator, ASCII
    data = Generator(ASCII, 100_000, 1.0, 42).bytes(24 << 20)     # a C2 slice
    fname = "c2.txt"
    (tmp_path / fname).write_bytes(data)
    r = subprocess.run([EXE, str(tmp_path), fname, str(nmap), str(nreduce)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    # the reference's progress lines, in order
    assert r.stdout.startswith(f"Split {fname}\n")
    for m in range(nmap):
        assert f"DoMap: read split mrtmp.{fname}-{m} " in r.stdout
    # Split: the splits concatenate back to the input (short lines, no CR)
    splits = b"".join((tmp_path / f"mrtmp.{fname}-{m}").read_bytes() for m in range(nmap))
    assert splits == data
    want = ob.merged(data)
    ob.assert_same((tmp_path / f"mrtmp.{fname}").read_bytes(), want)
    ob.assert_same((tmp_path / f"mrtmp.{fname}.async").read_bytes(), want)
    ob.assert_same((tmp_path / f"mrtmp.{fname}.comm").read_bytes(), want)
    ref = ob.Result(data)
    for q in range(nreduce):
        assert (tmp_path / f"mrtmp.{fname}-res-{q}").read_bytes() == ref.res(nreduce, q), q
    nl = want.count(b"\n")
    assert f"keys {nl} bytes {len(want)}" in r.stdout
    assert "path 1" in r.stdout               # the second job took the one-launch reduce
