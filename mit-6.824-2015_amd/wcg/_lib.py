"""ctypes binding of libwcg.so (C ABI declared in include/wcg.h).

The product path has no CPU fallback: if libwcg.so is missing or no GPU is visible, opening an
engine raises.  Build the library with `python -c "import __graft_entry__ as g; g.build()"`.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))
# WCG_LIB: an alternative build of the same library (measurement variants only)
LIB_PATH = os.environ.get("WCG_LIB") or os.path.join(_HERE, "libwcg.so")

WCG_OK, WCG_EINVAL, WCG_ENOMEM, WCG_EHIP, WCG_EFULL, WCG_ESTATE = range(6)
RECORD_BYTES = 32

_lib: Optional[ctypes.CDLL] = None

# every symbol include/wcg.h declares (tests check the library exports them all)
EXPORTED = [
    "wcg_open", "wcg_close", "wcg_last_error", "wcg_set_stream", "wcg_reset", "wcg_map",
    "wcg_map_device", "wcg_reduce", "wcg_result_device", "wcg_result_copy", "wcg_partition",
    "wcg_export", "wcg_import", "wcg_timings", "wcg_enable_timing", "wcg_stats", "wcg_ihash",
    "wcg_version", "wcg_map_file", "wcg_partition_all", "wcg_map_json", "wcg_export_count",
    "wcg_export_write", "wcg_merge_runs", "wcg_result_copy_device", "wcg_sync", "wcg_free",
    "wcg_comm_id", "wcg_comm_init", "wcg_exchange", "wcg_gather_merge", "wcg_exchange_plan",
    "wcg_gather_plan", "wcg_exchange_local", "wcg_gather_merge_local", "wcg_reduce_path",
    "wcg_reduce_async", "wcg_reduce_wait", "wcg_ingest_stats",
]
COMM_ID_BYTES = 128


class WcgError(RuntimeError):
    """Non-zero status from libwcg (the reference would log.Fatal at this point)."""

    def __init__(self, status: int, msg: str):
        super().__init__(f"wcg status {status}: {msg}")
        self.status = status


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run __graft_entry__.build() (hipcc gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    P, U64, U32, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    PU64 = ctypes.POINTER(ctypes.c_uint64)
    sig = {
        "wcg_open": (I, [I, U64, U64, ctypes.POINTER(P)]),
        "wcg_close": (I, [P]),
        "wcg_last_error": (ctypes.c_char_p, [P]),
        "wcg_set_stream": (I, [P, P]),
        "wcg_reset": (I, [P]),
        "wcg_map": (I, [P, ctypes.c_char_p, U64]),
        "wcg_map_device": (I, [P, P, U64]),
        "wcg_reduce": (I, [P, PU64, PU64]),
        "wcg_result_device": (I, [P, ctypes.POINTER(P), PU64]),
        "wcg_result_copy": (I, [P, P, U64]),
        "wcg_partition": (I, [P, U32, U32, P, U64, PU64]),
        "wcg_export": (I, [P, U32, U32, ctypes.POINTER(P), PU64]),
        "wcg_import": (I, [P, P, U64]),
        "wcg_timings": (I, [P, ctypes.POINTER(ctypes.c_double), I, PU64]),
        "wcg_enable_timing": (I, [P, I]),
        "wcg_stats": (I, [P, PU64]),
        "wcg_ihash": (U32, [ctypes.c_char_p, U64]),
        "wcg_version": (ctypes.c_char_p, []),
        "wcg_map_file": (I, [P, ctypes.c_char_p, PU64, PU64]),
        "wcg_partition_all": (I, [P, U32, P, U64, PU64]),
        "wcg_map_json": (I, [P, ctypes.c_char_p, U64, U32, P, U64, PU64]),
        "wcg_export_count": (I, [P, U32, U32, PU64]),
        "wcg_export_write": (I, [P, P]),
        "wcg_merge_runs": (I, [P, P, PU64, U32, PU64, PU64]),
        "wcg_result_copy_device": (I, [P, P]),
        "wcg_sync": (I, [P]),
        "wcg_free": (I, [P, P]),
        "wcg_comm_id": (I, [P]),
        "wcg_comm_init": (I, [P, P, I, I]),
        "wcg_exchange": (I, [P, U32, PU64, PU64]),
        "wcg_gather_merge": (I, [P, I, PU64, PU64]),
        "wcg_exchange_plan": (I, [PU64, U32, U32, PU64, PU64, PU64, PU64, PU64]),
        "wcg_gather_plan": (I, [PU64, U32, U32, PU64, PU64]),
        "wcg_exchange_local": (I, [ctypes.POINTER(P), U32, U32, PU64, PU64]),
        "wcg_gather_merge_local": (I, [ctypes.POINTER(P), U32, U32, PU64, PU64]),
        "wcg_reduce_path": (I, [P, ctypes.POINTER(I)]),
        "wcg_reduce_async": (I, [P]),
        "wcg_reduce_wait": (I, [P, PU64, PU64]),
        "wcg_ingest_stats": (I, [P, ctypes.POINTER(ctypes.c_double), I]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


_hiprt = None


def _hip() -> ctypes.CDLL:
    """The HIP runtime (plain copies between host buffers and libwcg's device buffers)."""
    global _hiprt
    if _hiprt is None:
        for name in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
            try:
                h = ctypes.CDLL(name)
                break
            except OSError:
                continue
        else:
            raise ImportError("libamdhip64.so not found")
        h.hipMemcpy.restype = ctypes.c_int
        h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        h.hipMalloc.restype = ctypes.c_int
        h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        h.hipFree.restype = ctypes.c_int
        h.hipFree.argtypes = [ctypes.c_void_p]
        h.hipDeviceSynchronize.restype = ctypes.c_int
        _hiprt = h
    return _hiprt


def _hip_check(rc: int, what: str) -> None:
    if rc != 0:
        raise WcgError(WCG_EHIP, f"{what} failed: hipError {rc}")


def ihash(key: bytes) -> int:
    """FNV-1a 32 (mapreduce.go:185-189) via the library's host helper."""
    return load().wcg_ihash(key, len(key))


class Engine:
    """One GPU's word-count context (wraps wcg_ctx).

    Phase methods mirror the reference data plane: map_* = DoMap+Map over a split,
    reduce() = DoReduce x R + Merge, partition() = one DoReduce output file."""

    def __init__(self, device: int = 0, max_input_bytes: int = 0, max_keys: int = 1 << 20):
        self._lib = load()
        self._ctx = ctypes.c_void_p()
        rc = self._lib.wcg_open(device, max_input_bytes, max_keys, ctypes.byref(self._ctx))
        if rc != WCG_OK:
            msg = self._lib.wcg_last_error(self._ctx).decode() if self._ctx else "open failed"
            if self._ctx:
                self._lib.wcg_close(self._ctx)
                self._ctx = ctypes.c_void_p()
            raise WcgError(rc, msg)
        self.device = device

    # -- plumbing
    def _chk(self, rc: int) -> None:
        if rc != WCG_OK:
            raise WcgError(rc, self._lib.wcg_last_error(self._ctx).decode())

    def close(self) -> None:
        if self._ctx:
            self._lib.wcg_close(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr: int) -> None:
        self._chk(self._lib.wcg_set_stream(self._ctx, ctypes.c_void_p(stream_ptr)))

    def enable_timing(self, on=True) -> None:
        """on = True/1: phase times of the last job; 2: summed over every job from now on (no
        timings() call, hence no host round trip, needed between jobs); 3: as 2, the map kernel
        only (each event is a ~5 us bubble between kernels); False/0: off."""
        mode = on if on in (2, 3) and on is not True else (1 if on else 0)
        self._chk(self._lib.wcg_enable_timing(self._ctx, mode))

    # -- phases
    def reset(self) -> None:
        self._chk(self._lib.wcg_reset(self._ctx))

    def map_host(self, data: bytes) -> None:
        self._chk(self._lib.wcg_map(self._ctx, data, len(data)))

    def map_device(self, dev_ptr: int, n: int) -> None:
        self._chk(self._lib.wcg_map_device(self._ctx, ctypes.c_void_p(dev_ptr), n))

    def map_file(self, path: str) -> Tuple[int, int]:
        """Split + DoMap of a whole file through the pinned double-buffered ingest; returns
        (bytes mapped, file size) - fewer bytes mapped when a 64 KiB+ line ended the scan (P1)."""
        mapped, size = ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(self._lib.wcg_map_file(self._ctx, os.fsencode(path), ctypes.byref(mapped), ctypes.byref(size)))
        return mapped.value, size.value

    def map_json(self, data: bytes, nreduce: int) -> List[bytes]:
        """DoMap's reference-exact JSON intermediate files (one per partition) for one split."""
        sizes = (ctypes.c_uint64 * nreduce)()
        self._chk(self._lib.wcg_map_json(self._ctx, data, len(data), nreduce, None, 0, sizes))
        total = sum(sizes)
        buf = ctypes.create_string_buffer(max(total, 1))
        self._chk(self._lib.wcg_map_json(self._ctx, data, len(data), nreduce, buf, total, sizes))
        return _slices(buf.raw, list(sizes))

    def reduce(self) -> Tuple[int, int]:
        nk, nb = ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(self._lib.wcg_reduce(self._ctx, ctypes.byref(nk), ctypes.byref(nb)))
        return nk.value, nb.value

    def reduce_async(self) -> None:
        """wcg_reduce_async: queue the reduce (no host wait); reduce_wait() or any result call
        waits for it, the next reset()/map_*() drops it."""
        self._chk(self._lib.wcg_reduce_async(self._ctx))

    def reduce_wait(self) -> Tuple[int, int]:
        nk, nb = ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(self._lib.wcg_reduce_wait(self._ctx, ctypes.byref(nk), ctypes.byref(nb)))
        return nk.value, nb.value

    def result_device(self) -> Tuple[int, int]:
        p, nb = ctypes.c_void_p(), ctypes.c_uint64()
        self._chk(self._lib.wcg_result_device(self._ctx, ctypes.byref(p), ctypes.byref(nb)))
        return p.value or 0, nb.value

    def result_copy_device(self, dev_ptr: int) -> None:
        """Async device copy of the formatted output into a caller's buffer (context stream)."""
        self._chk(self._lib.wcg_result_copy_device(self._ctx, ctypes.c_void_p(dev_ptr)))

    def sync(self) -> None:
        self._chk(self._lib.wcg_sync(self._ctx))

    def free(self, dev_ptr: int) -> None:
        """wcg_free: release the device buffer of result_device() or export() early."""
        self._chk(self._lib.wcg_free(self._ctx, dev_ptr))

    def result(self) -> bytes:
        _, nb = self.result_device()
        buf = ctypes.create_string_buffer(max(nb, 1))
        self._chk(self._lib.wcg_result_copy(self._ctx, buf, nb))
        return buf.raw[:nb]

    def partitions(self, nreduce: int) -> List[bytes]:
        """Every -res-<r> file of the last reduce (one device formatting pass for all)."""
        sizes = (ctypes.c_uint64 * nreduce)()
        self._chk(self._lib.wcg_partition_all(self._ctx, nreduce, None, 0, sizes))
        total = sum(sizes)
        buf = ctypes.create_string_buffer(max(total, 1))
        self._chk(self._lib.wcg_partition_all(self._ctx, nreduce, buf, total, sizes))
        return _slices(buf.raw, list(sizes))

    def partition(self, nreduce: int, r: int) -> bytes:
        nb = ctypes.c_uint64()
        self._chk(self._lib.wcg_partition(self._ctx, nreduce, r, None, 0, ctypes.byref(nb)))
        buf = ctypes.create_string_buffer(max(nb.value, 1))
        self._chk(self._lib.wcg_partition(self._ctx, nreduce, r, buf, nb.value, ctypes.byref(nb)))
        return buf.raw[:nb.value]

    def export(self, nreduce: int, nranks: int) -> Tuple[int, List[int]]:
        """Bucket the local aggregate by owner rank; returns (device ptr, units per rank)."""
        p = ctypes.c_void_p()
        counts = (ctypes.c_uint64 * nranks)()
        self._chk(self._lib.wcg_export(self._ctx, nreduce, nranks, ctypes.byref(p), counts))
        return p.value or 0, list(counts)

    def export_count(self, nreduce: int, nranks: int) -> List[int]:
        """Units per destination rank of the local aggregate (one host synchronisation)."""
        counts = (ctypes.c_uint64 * nranks)()
        self._chk(self._lib.wcg_export_count(self._ctx, nreduce, nranks, counts))
        return list(counts)

    def export_write(self, dev_ptr: int) -> None:
        """Write the units counted by export_count into a caller's device buffer (async)."""
        self._chk(self._lib.wcg_export_write(self._ctx, ctypes.c_void_p(dev_ptr)))

    def import_records(self, dev_ptr: int, nunits: int) -> None:
        self._chk(self._lib.wcg_import(self._ctx, ctypes.c_void_p(dev_ptr), nunits))

    def merge_runs(self, dev_ptr: int, run_bytes: List[int]) -> Tuple[int, int]:
        """Merge sorted "key: count\n" runs held back to back at dev_ptr into this context's
        result (Merge, mapreduce.go:284-321); returns (keys, bytes)."""
        rb = (ctypes.c_uint64 * max(len(run_bytes), 1))(*run_bytes)
        nk, nb = ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(self._lib.wcg_merge_runs(self._ctx, ctypes.c_void_p(dev_ptr), rb, len(run_bytes),
                                           ctypes.byref(nk), ctypes.byref(nb)))
        return nk.value, nb.value

    # -- the shuffle and the final Merge over RCCL, inside the library
    @staticmethod
    def comm_id() -> bytes:
        """ncclGetUniqueId (made once, on rank 0, and handed to every rank by the host)."""
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        rc = load().wcg_comm_id(buf)
        if rc != WCG_OK:
            raise WcgError(rc, "wcg_comm_id: ncclGetUniqueId failed")
        return buf.raw

    def comm_init(self, comm_id: bytes, rank: int, world: int) -> None:
        """ncclCommInitRank for this engine (collective: every rank calls it)."""
        if len(comm_id) != COMM_ID_BYTES:
            raise WcgError(WCG_EINVAL, "comm_init: the id is 128 bytes")
        self._chk(self._lib.wcg_comm_init(self._ctx, comm_id, rank, world))

    def exchange(self, nreduce: int) -> Tuple[int, int]:
        """The ihash % nreduce shuffle (collective): afterwards this engine holds exactly the keys
        of the partitions its rank owns.  Returns (units sent, units received)."""
        snt, rcv = ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(self._lib.wcg_exchange(self._ctx, nreduce, ctypes.byref(snt), ctypes.byref(rcv)))
        return snt.value, rcv.value

    def gather_merge(self, root: int = 0) -> Tuple[int, int]:
        """Merge of every rank's sorted run at root (collective, after reduce()); (keys, bytes) of
        the merged file on root, (0, 0) elsewhere."""
        nk, nb = ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(self._lib.wcg_gather_merge(self._ctx, root, ctypes.byref(nk), ctypes.byref(nb)))
        return nk.value, nb.value

    # -- host copies of the record units (the file-based shuffle of the config-5 workers)
    def export_host(self, nreduce: int, nranks: int) -> Tuple[bytes, List[int]]:
        """export() copied to host memory: (record units, units per rank)."""
        ptr, counts = self.export(nreduce, nranks)
        n = sum(counts) * RECORD_BYTES
        buf = ctypes.create_string_buffer(max(n, 1))
        if n:
            _hip_check(_hip().hipMemcpy(buf, ctypes.c_void_p(ptr), n, 2), "hipMemcpy D2H")
        return buf.raw[:n], counts

    def import_host(self, records: bytes) -> None:
        """import_records() from host memory (staged through a temporary device buffer)."""
        if len(records) % RECORD_BYTES:
            raise WcgError(WCG_EINVAL, "import_host: not a whole number of record units")
        n = len(records) // RECORD_BYTES
        if n == 0:
            return
        hip = _hip()
        dev = ctypes.c_void_p()
        _hip_check(hip.hipMalloc(ctypes.byref(dev), len(records)), "hipMalloc")
        try:
            _hip_check(hip.hipMemcpy(dev, records, len(records), 1), "hipMemcpy H2D")
            self.import_records(dev.value, n)
            _hip_check(hip.hipDeviceSynchronize(), "hipDeviceSynchronize")
        finally:
            hip.hipFree(dev)

    # -- diagnostics
    PHASES = ("map", "agg", "compact", "sort", "format", "export", "exchange", "import", "gather", "merge")

    def timings(self) -> Tuple[dict, int]:
        """Device ms per phase of the last job (needs enable_timing) and map launch count."""
        ms = (ctypes.c_double * 10)()
        nl = ctypes.c_uint64()
        self._chk(self._lib.wcg_timings(self._ctx, ms, 10, ctypes.byref(nl)))
        return dict(zip(self.PHASES, list(ms))), nl.value

    def reduce_path(self) -> int:
        """1 if the last reduce() ran the one-launch reduce (wcg_fused.h), 0 for the multi-launch one."""
        v = ctypes.c_int()
        self._chk(self._lib.wcg_reduce_path(self._ctx, ctypes.byref(v)))
        return v.value

    INGEST_STATS = ["host_issue_ms", "read_ms", "slot_wait_ms", "copy_ms", "copy_span_ms",
                    "copy_engine_idle_frac", "map_ms", "device_span_ms", "chunks"]

    def ingest_stats(self) -> dict:
        """The last map_file / map_host ingest's breakdown (wcg_ingest_stats): host reading and
        slot waits, the chunks' H2D copies and the copy engine's idle share of its span, the
        chunks' map kernels, and the device span from the first copy to the last map."""
        v = (ctypes.c_double * len(self.INGEST_STATS))()
        self._chk(self._lib.wcg_ingest_stats(self._ctx, v, len(self.INGEST_STATS)))
        return dict(zip(self.INGEST_STATS, list(v)))

    def stats(self) -> dict:
        s = (ctypes.c_uint64 * 9)()
        self._chk(self._lib.wcg_stats(self._ctx, s))
        keys = ["tokens", "keys", "lds_hits", "global_ops", "long_tokens", "arena_bytes", "overflow",
                "spin_fail", "emitted"]
        return dict(zip(keys, list(s)))


def _slices(raw: bytes, sizes: List[int]) -> List[bytes]:
    out, off = [], 0
    for n in sizes:
        out.append(raw[off:off + n])
        off += n
    return out


def exchange_plan(counts: List[List[int]], rank: int) -> dict:
    """wcg_exchange_plan: counts[s][d] = units rank s sends to rank d -> this rank's send / receive
    offsets and counts (host arithmetic, no GPU)."""
    W = len(counts)
    flat = (ctypes.c_uint64 * (W * W))(*[int(x) for row in counts for x in row])
    so, sc, ro, rc = [(ctypes.c_uint64 * W)() for _ in range(4)]
    tot = (ctypes.c_uint64 * 2)()
    st = load().wcg_exchange_plan(flat, W, rank, so, sc, ro, rc, tot)
    if st != WCG_OK:
        raise WcgError(st, "wcg_exchange_plan: bad arguments")
    return {"send_off": list(so), "send_cnt": list(sc), "recv_off": list(ro), "recv_cnt": list(rc),
            "sent": tot[0], "received": tot[1]}


def gather_plan(sizes: List[int], root: int) -> Tuple[List[int], int]:
    """wcg_gather_plan: where each rank's run lands in root's receive buffer, and the total."""
    W = len(sizes)
    sz = (ctypes.c_uint64 * max(W, 1))(*sizes)
    off = (ctypes.c_uint64 * max(W, 1))()
    tot = ctypes.c_uint64()
    st = load().wcg_gather_plan(sz, W, root, off, ctypes.byref(tot))
    if st != WCG_OK:
        raise WcgError(st, "wcg_gather_plan: bad arguments")
    return list(off)[:W], tot.value


def _ctx_array(engines: List["Engine"]):
    return (ctypes.c_void_p * len(engines))(*[e._ctx.value for e in engines])


def exchange_local(engines: List["Engine"], nreduce: int) -> Tuple[List[int], List[int]]:
    """wcg_exchange_local: the shuffle across engines of this process (a world of len(engines)
    ranks, device copies for transport).  Returns (units sent, units received) per engine."""
    W = len(engines)
    snt, rcv = (ctypes.c_uint64 * W)(), (ctypes.c_uint64 * W)()
    st = load().wcg_exchange_local(_ctx_array(engines), W, nreduce, snt, rcv)
    if st != WCG_OK:
        msgs = "; ".join(load().wcg_last_error(e._ctx).decode() for e in engines)
        raise WcgError(st, f"wcg_exchange_local: {msgs}")
    return list(snt), list(rcv)


def gather_merge_local(engines: List["Engine"], root: int) -> Tuple[int, int]:
    """wcg_gather_merge_local: every engine's sorted run merged into engines[root]'s result."""
    nk, nb = ctypes.c_uint64(), ctypes.c_uint64()
    st = load().wcg_gather_merge_local(_ctx_array(engines), len(engines), root, ctypes.byref(nk), ctypes.byref(nb))
    if st != WCG_OK:
        msgs = "; ".join(load().wcg_last_error(e._ctx).decode() for e in engines)
        raise WcgError(st, f"wcg_gather_merge_local: {msgs}")
    return nk.value, nb.value


def version() -> str:
    return load().wcg_version().decode()
