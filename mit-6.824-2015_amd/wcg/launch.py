"""Start the N rank processes of a one-node job (one per GPU) from a plain `--gpus N` run.

The reference starts its distributed word count as one master plus W worker processes
(mapreduce.go:358-380 MakeMapReduce/Run, master.go:57-82 RunMaster dispatching to the registered
workers).  Here the ranks of the multi-GPU job are started by torch.distributed.run as children
of the calling process, which itself never touches a GPU (so nothing is exec'd from a process that
has initialised one).  The children's stdout is relayed line by line (only rank 0 prints the
result line); a rank that fails ends the job (torch.distributed.run stops the others), and a job
that outlives `timeout` is killed as a whole process group, so a stalled collective ends the run
with a non-zero status instead of hanging it.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import List, Optional, TextIO

TIMEOUT_STATUS = 124


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(script: str, argv: List[str], nprocs: int, timeout: float,
                 extra_env: Optional[dict] = None, out: Optional[TextIO] = None) -> int:
    """Run `script argv` as `nprocs` ranks under torch.distributed.run (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT set for each).  Returns the job's exit status:
    0 when every rank succeeded, the launcher's status when one failed, 124 after a timeout."""
    out = out or sys.stdout
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nprocs}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", script, *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    env.update(extra_env or {})
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, start_new_session=True, text=True, bufsize=1)

    def relay():
        for line in proc.stdout:
            out.write(line)
            out.flush()

    t = threading.Thread(target=relay, daemon=True)
    t.start()
    try:
        rc = proc.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        sys.stderr.write(f"launch: the {nprocs}-rank job exceeded {timeout:.0f} s; stopping it\n")
        for sig, grace in ((signal.SIGTERM, 15), (signal.SIGKILL, 10)):
            try:
                os.killpg(proc.pid, sig)
            except ProcessLookupError:
                break
            try:
                proc.wait(timeout=grace)
                break
            except subprocess.TimeoutExpired:
                continue
        rc = TIMEOUT_STATUS
    t.join(timeout=5)
    if rc != 0:
        sys.stderr.write(f"launch: the {nprocs}-rank job ended with status {rc}\n")
    return rc if rc >= 0 else 128 - rc
