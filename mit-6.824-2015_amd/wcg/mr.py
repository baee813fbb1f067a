"""Config 5: the Lab 1 master/worker MapReduce with GPU-bound word-count workers.

This mirrors the reference's src/mapreduce control flow, restricted to the wc job (SURVEY.md
§3.2, §8(f) rank 1). Paths are relative to /root/reference.

Reference pieces mirrored here:
  * names: MapName / ReduceName / MergeName (mapreduce.go:136-138, 181-183, 233-235);
  * Split (mapreduce.go:141-179): bufio.Scanner lines, a trailing "\\r" dropped, "\\n" appended,
    a new split once more than size/nMap + 1 bytes have been written;
  * the master (master.go:29-88): a dispatcher hands jobs to registered or idle workers, and a
    failed Worker.DoJob RPC puts the job back for another worker (re-execution);
  * the registration server and Run (mapreduce.go:84-133, 358-380);
  * the worker (worker.go:22-92): Register, then serve at most nRPC connections (failure
    injection), DoJob and Shutdown;
  * Merge (mapreduce.go:284-321) on the host, from the -res-<r> JSON files.

Where the GPU changes the data plane:
  * DoMap runs the split through one wcg engine (tokenize + aggregate on the GPU). It writes its
    nReduce intermediate files mrtmp.<f>-<m>-<r> as pre-aggregated 32-byte record units
    (include/wcg.h, WCG_RECORD_BYTES) partitioned by ihash(key) % nReduce, not per-occurrence
    JSON. The file names are the reference's, so CleanupFiles is unchanged.
  * DoReduce imports partition r from every map job's file and writes mrtmp.<f>-res-<r> in the
    reference's JSON lines, byte-identical, so the unmodified CPU Merge consumes it.

RPC: one JSON request line and one JSON reply line per UNIX-socket connection. This stands in
for net/rpc + gob (common.go:59-74); the method names and argument fields are the reference's.
A worker process binds one GPU: set HIP_VISIBLE_DEVICES per process, or pass `device`.
"""
from __future__ import annotations

import json
import os
import sys
import queue
import socket
import threading
from typing import Callable, Dict, List, Optional

MAP, REDUCE = "Map", "Reduce"          # common.go:6-9
MAX_LINE = 64 * 1024                   # bufio.Scanner's default token limit (parity domain P1)


# ---------------------------------------------------------------- file names
def map_name(f: str, m: int) -> str:
    return f"mrtmp.{f}-{m}"


def reduce_name(f: str, m: int, r: int) -> str:
    return f"{map_name(f, m)}-{r}"


def merge_name(f: str, r: int) -> str:
    return f"mrtmp.{f}-res-{r}"


# ---------------------------------------------------------------- RPC (common.go:59-74)
def call(srv: str, method: str, args: dict, timeout: float = 600.0) -> Optional[dict]:
    """Send one RPC; returns the reply dict, or None when the server could not be reached or
    the call failed (the reference's call() returning false)."""
    try:
        with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as s:
            s.settimeout(timeout)
            s.connect(srv)
            s.sendall(json.dumps({"method": method, "args": args}).encode() + b"\n")
            buf = b""
            while not buf.endswith(b"\n"):
                chunk = s.recv(65536)
                if not chunk:
                    return None
                buf += chunk
        rep = json.loads(buf)
        return rep.get("reply") if rep.get("ok") else None
    except (OSError, ValueError):
        return None


def _serve_conn(conn: socket.socket, handlers: Dict[str, Callable[[dict], dict]]) -> None:
    with conn:
        buf = b""
        while not buf.endswith(b"\n"):
            chunk = conn.recv(65536)
            if not chunk:
                return
            buf += chunk
        req = json.loads(buf)
        fn = handlers.get(req.get("method"))
        try:
            rep = {"ok": True, "reply": fn(req.get("args", {}))} if fn else {"ok": False}
        except Exception as e:  # an RPC handler error is the caller's failed call
            rep = {"ok": False, "error": repr(e)}
        conn.sendall(json.dumps(rep).encode() + b"\n")


def _listen(addr: str) -> socket.socket:
    if os.path.exists(addr):
        os.remove(addr)             # only needed for "unix" (mapreduce.go:111, worker.go:72)
    l = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    l.bind(addr)
    l.listen(64)
    return l


# ---------------------------------------------------------------- Split / Merge (host)
def _atomic_write(path: str, data: bytes) -> None:
    """Write a job's output file as temp-then-rename: a worker killed mid-write never leaves a
    truncated file under the reference's name, and a re-executed job replaces it whole (the
    reference truncates in place with os.Create, mapreduce.go:215,270)."""
    d, base = os.path.split(path)          # a dot name: never taken for a reference file
    tmp = os.path.join(d, f".{base}.tmp{os.getpid()}.{threading.get_ident()}")
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)


def split(path: str, nmap: int, workdir: str, fname: str) -> int:
    """Split (mapreduce.go:141-179); returns the number of split files written.

    Quirk P1 is kept: bufio.Scanner's buffer holds at most 64 KiB, so a line that does not fit
    with its '\n' (65,536 bytes or more before the '\n', or at the end of the input) stops the
    scan silently, and the rest of the input is never split (the reference checks no scanner
    error after its loop, mapreduce.go:164-176)."""
    print(f"Split {fname}", flush=True)
    data = open(path, "rb").read()
    nchunk = len(data) // nmap + 1
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()                 # the scanner yields no empty token after a final "\n"
    outs, cur, m, i = [], [], 1, 0
    for line in lines:
        if len(line) >= MAX_LINE:
            break                   # ErrTooLong ends Scan(); the loop just stops (P1)
        if i > nchunk * m:
            outs.append(b"".join(cur))
            cur, m = [], m + 1
        if line.endswith(b"\r"):
            line = line[:-1]        # bufio.ScanLines drops one trailing carriage return
        cur.append(line + b"\n")
        i += len(line) + 1
    outs.append(b"".join(cur))
    for k, b in enumerate(outs):
        _atomic_write(os.path.join(workdir, map_name(fname, k)), b)
    return len(outs)


def merge(workdir: str, fname: str, nreduce: int) -> bytes:
    """Merge (mapreduce.go:284-321): later files win on equal keys, sort.Strings order (bytes),
    "%s: %s\\n"; writes mrtmp.<f> and returns its bytes."""
    kvs: Dict[bytes, bytes] = {}
    for r in range(nreduce):
        print(f"Merge: read {merge_name(fname, r)}", flush=True)
        with open(os.path.join(workdir, merge_name(fname, r)), "rb") as f:
            for line in f:
                try:
                    kv = json.loads(line)
                except ValueError:
                    break           # a decode error ends the file, as the reference's loop does
                kvs[kv["Key"].encode()] = kv["Value"].encode()
    out = b"".join(k + b": " + kvs[k] + b"\n" for k in sorted(kvs))
    _atomic_write(os.path.join(workdir, "mrtmp." + fname), out)
    return out


# ---------------------------------------------------------------- GPU DoMap / DoReduce
EFULL = 4                              # WCG_EFULL (include/wcg.h): aggregation table full

# Quirk P2: DoMap reads its split with ONE file.Read of the split's size
# (mapreduce.go:205-207), and Go's os.File.Read on Linux moves at most 1 GiB per call
# (internal/poll maxRW; Go 1.16-1.20, the versions whose unicode tables are Unicode 13 like ours),
# returning a nil error for the short read.  A split over 1 GiB is therefore mapped as its first
# 1 GiB followed by zero bytes - the tokens of the first 1 GiB alone, since NUL separates.  The
# GPU DoMap emulates exactly that (oracle/wc_ref.py domap_read restates it).
READ_CAP = 1 << 30


def read_split(path: str) -> bytes:
    """The bytes DoMap's single Read of a split file returns (P2: at most READ_CAP)."""
    size = os.path.getsize(path)
    with open(path, "rb") as f:
        b = f.read(READ_CAP)
    if size > READ_CAP:
        print(f"P2: split {os.path.basename(path)} is {size} bytes; DoMap's single Read maps its first "
              f"{READ_CAP} (the reference's behaviour, emulated)", file=sys.stderr, flush=True)
    return b


def _sized_job(engine, nbytes: int, job):
    """Run job() on an engine sized for nbytes of input when the engine can be re-sized
    (wc.SizedEngine.ensure); once more with worst-case tables if its table filled."""
    ensure = getattr(engine, "ensure", None)
    if ensure is None:
        return job()
    ensure(nbytes)
    try:
        return job()
    except Exception as e:   # WcgError(WCG_EFULL): rerun the whole job with room for every key
        if getattr(e, "status", None) != EFULL:
            raise
    ensure(nbytes, True)
    return job()


def do_map(engine, job: int, workdir: str, fname: str, nreduce: int, json_intermediates: bool = False) -> None:
    """DoMap (mapreduce.go:193-231) on the GPU: one split -> nReduce intermediate files.

    Default: pre-aggregated 32-byte record units partitioned by ihash % nReduce (what a GPU
    DoReduce imports).  json_intermediates=True writes the reference's own per-occurrence JSON
    lines instead ({"Key":"tok","Value":"1"}\n for every token, in input order,
    mapreduce.go:214-230), byte for byte, so an unmodified CPU DoReduce can consume them."""
    name = map_name(fname, job)
    path = os.path.join(workdir, name)
    print(f"DoMap: read split {name} {os.path.getsize(path)}", flush=True)
    b = read_split(path)
    if json_intermediates:
        parts = _sized_job(engine, len(b), lambda: engine.map_json(b, nreduce))
        for r in range(nreduce):
            _atomic_write(os.path.join(workdir, reduce_name(fname, job, r)), parts[r])
        return

    def run():
        engine.reset()
        if b:
            engine.map_host(b)
        return engine.export_host(nreduce, nreduce)
    recs, counts = _sized_job(engine, len(b), run)
    off = 0
    for r in range(nreduce):
        _atomic_write(os.path.join(workdir, reduce_name(fname, job, r)), recs[off * 32:(off + counts[r]) * 32])
        off += counts[r]


def do_reduce(engine, job: int, workdir: str, fname: str, nmap: int) -> None:
    """DoReduce (mapreduce.go:239-280) on the GPU: partition `job` of every map job -> the
    reference's -res-<job> JSON lines (every imported key belongs to this partition)."""
    files = []
    for m in range(nmap):
        name = reduce_name(fname, m, job)
        print(f"DoReduce: read {name}", flush=True)
        with open(os.path.join(workdir, name), "rb") as f:
            files.append(f.read())
    # each file by its own format: a GPU DoMap's record units, or the reference's JSON lines (a
    # CPU DoMap, or a GPU worker with json_intermediates) - workers of one job may differ.  A record
    # unit never starts with '{' (its first byte is a key byte or zero padding; '{' is no letter).
    is_json = [f[:1] == b"{" for f in files]

    def run():
        engine.reset()
        for data, js in zip(files, is_json):
            if js:
                # decode on the host as DoReduce's json.Decoder does (mapreduce.go:249-261), one
                # key per line, and count the keys on the GPU
                keys = _json_keys(data)
                if keys:
                    engine.map_host(keys)
            else:
                engine.import_host(data)
        engine.reduce()
        return engine.partition(1, 0)
    # one distinct key per record unit (or per JSON line) at most
    nunits = sum(f.count(b"\n") if js else len(f) // 32 for f, js in zip(files, is_json))
    _atomic_write(os.path.join(workdir, merge_name(fname, job)), _sized_job(engine, 16 * nunits, run))


def _json_keys(data: bytes) -> bytes:
    """Keys of {"Key":"k","Value":"1"} lines, newline-separated (the decoder stops at the first
    line that is not such an object, as the reference's loop ends on a decode error)."""
    out = []
    for line in data.split(b"\n"):
        if not (line.startswith(b'{"Key":"') and line.endswith(b'","Value":"1"}')):
            break
        out.append(line[8:-14])
    return b"\n".join(out) + b"\n" if out else b""


# ---------------------------------------------------------------- worker (worker.go)
class Worker:
    """RunWorker (worker.go:60-92): register with the master, then serve at most nrpc
    connections (nrpc < 0: unlimited).  Each DoJob runs on this worker's GPU engine."""

    def __init__(self, master: str, me: str, engine_factory: Callable[[], object], workdir: str,
                 nrpc: int = -1, json_intermediates: bool = False):
        self.master, self.me, self.workdir = master, me, workdir
        self.nrpc, self.njobs = nrpc, 0
        self.json_intermediates = json_intermediates
        self.engine = engine_factory()
        self.lock = threading.Lock()            # one job at a time on the engine
        self.l = _listen(me)
        self.thread = threading.Thread(target=self._serve, daemon=True)

    def start(self) -> "Worker":
        if call(self.master, "MapReduce.Register", {"Worker": self.me}) is None:
            print(f"Register: RPC {self.master} register error")
        self.thread.start()
        return self

    def DoJob(self, a: dict) -> dict:                       # worker.go:22-34
        print(f"Dojob {self.me} job {a['JobNumber']} file {a['File']} operation {a['Operation']} "
              f"N {a['NumOtherPhase']}", flush=True)
        with self.lock:
            if a["Operation"] == MAP:
                do_map(self.engine, a["JobNumber"], self.workdir, a["File"], a["NumOtherPhase"],
                       self.json_intermediates)
            else:
                do_reduce(self.engine, a["JobNumber"], self.workdir, a["File"], a["NumOtherPhase"])
        return {"OK": True}

    def Shutdown(self, a: dict) -> dict:                    # worker.go:36-44
        self.nrpc = 0                       # stop accepting (closing the listener ends accept())
        self.l.close()
        # worker.go:40-43: the reply carries nJobs as it stands - the Shutdown RPC's own
        # connection included - and only then is that connection uncounted (wk.nJobs--), so
        # KillWorkers' list holds jobs + 1 per worker, as the reference's does
        njobs = self.njobs
        self.njobs -= 1
        return {"Njobs": njobs, "OK": True}

    def _serve(self) -> None:
        handlers = {"Worker.DoJob": self.DoJob, "Worker.Shutdown": self.Shutdown}
        while self.nrpc != 0:
            try:
                conn, _ = self.l.accept()
            except OSError:
                break
            self.nrpc -= 1
            self.njobs += 1
            threading.Thread(target=_serve_conn, args=(conn, handlers), daemon=True).start()
        self.l.close()

    def join(self, timeout: Optional[float] = None) -> None:
        self.thread.join(timeout)


# ---------------------------------------------------------------- master (master.go, mapreduce.go)
class MapReduce:
    """MakeMapReduce + Run (mapreduce.go:84-90, 369-380): split, dispatch map then reduce jobs to
    registered workers with re-execution on RPC failure, merge, shut the workers down."""

    def __init__(self, nmap: int, nreduce: int, path: str, master: str, workdir: str):
        self.nmap, self.nreduce, self.path, self.addr, self.workdir = nmap, nreduce, path, master, workdir
        self.file = os.path.basename(path)
        self.register_q: "queue.Queue[str]" = queue.Queue()
        self.workers: Dict[str, dict] = {}
        self.done = threading.Event()
        self.stats: List[int] = []
        self.merged: Optional[bytes] = None
        self.error: Optional[BaseException] = None
        self.alive = True
        self.l = _listen(master)
        threading.Thread(target=self._registration_server, daemon=True).start()
        threading.Thread(target=self._run, daemon=True).start()

    # registration server (mapreduce.go:92-133)
    def _registration_server(self) -> None:
        handlers = {"MapReduce.Register": self._register, "MapReduce.Shutdown": self._shutdown}
        while self.alive:
            try:
                conn, _ = self.l.accept()
            except OSError:
                break
            threading.Thread(target=_serve_conn, args=(conn, handlers), daemon=True).start()

    def _register(self, a: dict) -> dict:
        self.register_q.put(a["Worker"])
        return {"OK": True}

    def _shutdown(self, a: dict) -> dict:
        self.alive = False
        self.l.close()
        return {}

    def _run(self) -> None:                                 # mapreduce.go:369-380
        try:
            print(f"Run mapreduce job {self.addr} {self.file}", flush=True)
            self.nsplits = split(self.path, self.nmap, self.workdir, self.file)
            self.stats = self.run_master()
            self.merged = merge(self.workdir, self.file, self.nreduce)
            if call(self.addr, "MapReduce.Shutdown", {}) is None:
                print(f"Cleanup: RPC {self.addr} error", flush=True)
            print(f"{self.addr}: MapReduce done", flush=True)
        except BaseException as e:   # reported through wait()
            self.error = e
        finally:
            self.done.set()

    def run_master(self) -> List[int]:                      # master.go:29-88
        idle: "queue.Queue[str]" = queue.Queue()
        jobs: "queue.Queue[Optional[dict]]" = queue.Queue()
        donec: "queue.Queue[int]" = queue.Queue()

        def next_worker() -> str:
            while True:                     # select { registerChannel, idleWorkerChannel }
                try:
                    w = self.register_q.get_nowait()
                    self.workers[w] = {"address": w}
                    return w
                except queue.Empty:
                    pass
                try:
                    return idle.get(timeout=0.05)
                except queue.Empty:
                    pass

        def do_job(worker: str, job: dict) -> None:
            if call(worker, "Worker.DoJob", job) is not None:
                donec.put(1)
                idle.put(worker)
            else:
                print(f"RunMaster: RPC {worker} Worker.DoJob error")
                jobs.put(job)               # re-execute on another worker

        def dispatcher() -> None:
            while True:
                job = jobs.get()
                if job is None:
                    return
                w = next_worker()
                threading.Thread(target=do_job, args=(w, job), daemon=True).start()

        threading.Thread(target=dispatcher, daemon=True).start()
        for i in range(self.nmap):
            jobs.put({"File": self.file, "Operation": MAP, "JobNumber": i, "NumOtherPhase": self.nreduce})
        for _ in range(self.nmap):
            donec.get()
        for i in range(self.nreduce):
            jobs.put({"File": self.file, "Operation": REDUCE, "JobNumber": i, "NumOtherPhase": self.nmap})
        for _ in range(self.nreduce):
            donec.get()
        jobs.put(None)                      # close(jobChannel)
        return self.kill_workers()

    def kill_workers(self) -> List[int]:                    # master.go:13-27
        out = []
        for w in list(self.workers):
            rep = call(w, "Worker.Shutdown", {})
            if rep is None:
                print(f"DoWork: RPC {w} shutdown error")
            else:
                out.append(rep["Njobs"])
        return out

    def wait(self, timeout: Optional[float] = None) -> bytes:
        """<-mr.DoneChannel; returns the merged file's bytes."""
        if not self.done.wait(timeout):
            raise TimeoutError("MapReduce did not finish")
        if self.error:
            raise self.error
        return self.merged

    def cleanup_files(self) -> None:                        # mapreduce.go:330-341
        for i in range(self.nmap):
            os.remove(os.path.join(self.workdir, map_name(self.file, i)))
            for j in range(self.nreduce):
                os.remove(os.path.join(self.workdir, reduce_name(self.file, i, j)))
        for i in range(self.nreduce):
            os.remove(os.path.join(self.workdir, merge_name(self.file, i)))
        os.remove(os.path.join(self.workdir, "mrtmp." + self.file))


# ---------------------------------------------------------------- RunSingle (mapreduce.go:344-356)
def run_single(nmap: int, nreduce: int, path: str, engine, workdir: str) -> bytes:
    """RunSingle with the wc UDFs on one GPU: Split as the reference does, every split mapped
    into one engine, the nReduce -res-<r> files and the merged mrtmp.<f> written from it."""
    fname = os.path.basename(path)
    split(path, nmap, workdir, fname)
    engine.reset()
    for m in range(nmap):       # fewer split files than nMap (P3): open fails, as DoMap's does
        name = map_name(fname, m)
        print(f"DoMap: read split {name} {os.path.getsize(os.path.join(workdir, name))}", flush=True)
        b = read_split(os.path.join(workdir, name))
        if b:
            engine.map_host(b)
    engine.reduce()
    parts = engine.partitions(nreduce)          # every -res-<r> in one formatting pass
    for r in range(nreduce):
        _atomic_write(os.path.join(workdir, merge_name(fname, r)), parts[r])
    out = engine.result()
    for r in range(nreduce):
        print(f"Merge: read {merge_name(fname, r)}", flush=True)
    _atomic_write(os.path.join(workdir, "mrtmp." + fname), out)
    return out
