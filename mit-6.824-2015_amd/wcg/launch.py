"""Start the N rank processes of a one-node job (one per GPU) from a plain `--gpus N` run.

The reference starts its distributed word count as one master plus W worker processes
(mapreduce.go:358-380 MakeMapReduce/Run, master.go:57-82 RunMaster dispatching to the registered
workers).  Here the ranks of the multi-GPU job are started by torch.distributed.run as children
of the calling process, which itself never touches a GPU (so nothing is exec'd from a process that
has initialised one).  The children's stdout is relayed line by line (only rank 0 prints the
result line); a rank that fails ends the job (torch.distributed.run stops the others), and a job
that outlives `timeout` is stopped: SIGTERM to the launcher's process group AND to every
descendant process (torch.distributed.run starts each rank in a session of its own, so the group
signal alone does not reach them), then SIGKILL to every descendant still alive after the grace
period.  A stalled collective therefore ends the run with a non-zero status, and no rank is left
holding its GPU after launch_ranks returns.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import List, Optional, Set, TextIO

TIMEOUT_STATUS = 124
TERM_GRACE_S = 10.0        # after SIGTERM, before SIGKILL of every descendant still alive


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def descendants(pid: int) -> Set[int]:
    """Every live descendant of `pid` (children of all its threads, recursively, from /proc)."""
    seen: Set[int] = set()
    todo = [pid]
    while todo:
        p = todo.pop()
        try:
            tasks = os.listdir(f"/proc/{p}/task")
        except OSError:
            continue
        for t in tasks:
            try:
                with open(f"/proc/{p}/task/{t}/children") as f:
                    kids = [int(x) for x in f.read().split()]
            except (OSError, ValueError):
                continue
            for k in kids:
                if k not in seen:
                    seen.add(k)
                    todo.append(k)
    return seen


def _alive(pid: int) -> bool:
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(") ")[-1][:1] not in ("Z", "X")   # a zombie has exited
    except OSError:
        return False


def _signal_all(pids: Set[int], sig: int) -> None:
    for p in pids:
        try:
            os.kill(p, sig)
        except (ProcessLookupError, PermissionError):
            pass


def stop_job(proc: subprocess.Popen, grace: float = TERM_GRACE_S) -> None:
    """SIGTERM the launcher's group and all its descendants; after `grace` seconds SIGKILL every
    one of them still alive (the descendants are collected again, so late children count too)."""
    tree = descendants(proc.pid)
    try:
        os.killpg(proc.pid, signal.SIGTERM)
    except ProcessLookupError:
        pass
    _signal_all(tree, signal.SIGTERM)
    deadline = time.time() + grace
    while time.time() < deadline:
        tree |= descendants(proc.pid)
        if proc.poll() is not None and not any(_alive(p) for p in tree):
            break
        time.sleep(0.2)
    tree |= descendants(proc.pid)
    try:
        os.killpg(proc.pid, signal.SIGKILL)
    except ProcessLookupError:
        pass
    _signal_all({p for p in tree if _alive(p)}, signal.SIGKILL)
    try:
        proc.wait(timeout=10)
    except subprocess.TimeoutExpired:
        pass
    t_end = time.time() + 5
    while time.time() < t_end and any(_alive(p) for p in tree):
        time.sleep(0.1)


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
        sys.stderr.write(f"launch: the {nprocs}-rank job exceeded {timeout:.0f} s; stopping it "
                         f"(each rank's stack is dumped to stderr on SIGTERM)\n")
        stop_job(proc)
        rc = TIMEOUT_STATUS
    t.join(timeout=5)
    if rc != 0:
        sys.stderr.write(f"launch: the {nprocs}-rank job ended with status {rc}\n")
    return rc if rc >= 0 else 128 - rc
