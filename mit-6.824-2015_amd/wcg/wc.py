"""Command line of src/main/wc.go (wc.go:40-58) over the GPU word count:

  python -m wcg.wc master <file> sequential          RunSingle(5, 3, ...) on the GPU
  python -m wcg.wc master <file> <master-socket>     MakeMapReduce(5, 3, ...), waits for workers
  python -m wcg.wc worker <master-socket> <me>       RunWorker(..., nRPC = 100) on the GPU

nMap = 5, nReduce = 3 and nRPC = 100 are wc.go's constants (wc.go:49,51,56).  Environment knobs a
harness may set without changing that interface: WCG_DEVICE (HIP device of this process, default
0), WCG_NRPC (the worker's RPC budget, the failure-injection knob of worker.go:80-89),
WCG_JSON_INTERMEDIATES=1 (DoMap writes the reference's per-occurrence JSON -m-r files).

Device tables are sized from the input: a distinct key needs at least two input bytes (a letter
and a separator), so a job is first run with room for one key per 16 input bytes and, if the
aggregation table fills (WCG_EFULL), run again with room for every key the input could hold.
"""
from __future__ import annotations

import os
import sys

from . import mr

NMAP, NREDUCE, NRPC = 5, 3, 100           # wc.go:49, 51, 56
MAX_SPLIT = 1 << 30                       # parity domain P2: DoMap reads a split with one Read


def _device() -> int:
    return int(os.environ.get("WCG_DEVICE", "0"))


def _keys_for(nbytes: int, dense: bool) -> int:
    return max(1 << 18, nbytes // (2 if dense else 16) + 1024)


def engine_for(nbytes: int, dense: bool = False):
    """An engine whose tables hold the distinct keys of `nbytes` of input (dense: the worst case,
    one key per 2 bytes; else one per 16 bytes)."""
    from ._lib import Engine
    return Engine(device=_device(), max_input_bytes=min(max(nbytes, 1), MAX_SPLIT) + (64 << 10),
                  max_keys=_keys_for(nbytes, dense))


class SizedEngine:
    """Engine proxy for long-lived workers: ensure(nbytes, dense) re-opens the device context when
    a job needs larger tables or a larger staging buffer than the current one has (mr.py calls it
    before every job and again, dense, when a job's table filled)."""

    def __init__(self):
        self._e = None
        self._keys = self._staging = 0

    def ensure(self, nbytes: int, dense: bool = False) -> None:
        keys, staging = _keys_for(nbytes, dense), min(max(nbytes, 1 << 20), MAX_SPLIT)
        if self._e is None or keys > self._keys or staging > self._staging:
            if self._e is not None:
                self._e.close()
            from ._lib import Engine
            self._keys, self._staging = max(keys, self._keys), max(staging, self._staging)
            self._e = Engine(device=_device(), max_input_bytes=self._staging + (64 << 10), max_keys=self._keys)

    def __getattr__(self, name):
        if self._e is None:
            self.ensure(1 << 20)
        return getattr(self._e, name)

    def close(self):
        if self._e is not None:
            self._e.close()
            self._e = None


def run_single(path: str, nmap: int = NMAP, nreduce: int = NREDUCE) -> bytes:
    """RunSingle (mapreduce.go:344-356) on the GPU with tables sized from the input."""
    from ._lib import WcgError, WCG_EFULL
    workdir = os.path.dirname(os.path.abspath(path))
    size = os.path.getsize(path)
    for dense in (False, True):
        with engine_for(size, dense) as e:
            try:
                return mr.run_single(nmap, nreduce, path, e, workdir)
            except WcgError as err:
                if err.status != WCG_EFULL or dense:
                    raise
    raise AssertionError("unreachable")


def main(argv) -> int:
    if len(argv) != 4:                    # wc.go:45-46: a note, exit status 0
        print(f"{argv[0]}: see usage comments in file")
        return 0
    if argv[1] == "master":
        workdir = os.path.dirname(os.path.abspath(argv[2]))
        if argv[3] == "sequential":
            run_single(argv[2])
        else:
            mr.MapReduce(NMAP, NREDUCE, argv[2], argv[3], workdir).wait()
    else:
        nrpc = int(os.environ.get("WCG_NRPC", str(NRPC)))
        w = mr.Worker(argv[2], argv[3], SizedEngine, os.getcwd(), nrpc,
                      json_intermediates=os.environ.get("WCG_JSON_INTERMEDIATES") == "1").start()
        w.join()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
