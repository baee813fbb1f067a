"""Command line of src/main/wc.go (wc.go:40-58) over the GPU word count:

  python -m wcg.wc master <file> sequential          RunSingle(5, 3, ...) on GPU 0
  python -m wcg.wc master <file> <master-socket>     MakeMapReduce(5, 3, ...), waits for workers
  python -m wcg.wc worker <master-socket> <me>       RunWorker(..., nRPC = 100) on GPU 0
"""
from __future__ import annotations

import os
import sys

from . import mr


def _engine():
    from ._lib import Engine
    return Engine(device=int(os.environ.get("WCG_DEVICE", "0")), max_input_bytes=1 << 30, max_keys=1 << 22)


def main(argv) -> int:
    if len(argv) != 4:
        print("Usage: python -m wcg.wc master <file> sequential|<socket>  |  worker <master> <me>")
        return 2
    if argv[1] == "master":
        workdir = os.path.dirname(os.path.abspath(argv[2]))
        if argv[3] == "sequential":
            with _engine() as e:
                mr.run_single(5, 3, argv[2], e, workdir)
        else:
            mr.MapReduce(5, 3, argv[2], argv[3], workdir).wait()
    else:
        w = mr.Worker(argv[2], argv[3], _engine, os.getcwd(), 100).start()
        w.join()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
