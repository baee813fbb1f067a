"""A config-5 worker process for the CPU tests: wcg/mr.py's Worker (worker.go:60-92) serving
DoJob with the oracle-backed stand-in engine of tests/test_mr_workers.py (test infrastructure; the
product worker is `python -m wcg.wc worker <master> <me>`, which binds one GPU).

  python tests/standin_worker.py <master-socket> <me> <nrpc> <workdir>
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mit-6.824-2015_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from tests.test_mr_workers import StandInEngine  # noqa: E402
from wcg import mr  # noqa: E402

if __name__ == "__main__":
    master, me, nrpc, workdir = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    mr.Worker(master, me, StandInEngine, workdir, nrpc).start().join()
