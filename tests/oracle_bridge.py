"""Test-side access to the oracle (oracle/liboracle.so and oracle/wc_ref.py).

Only tests/, __graft_entry__.smoke() and bench.py (its cpu_baseline leg, and the result check
after the timed region) use this module, always as the checker; the product never does.
"""
from __future__ import annotations

import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")
if ORACLE_DIR not in sys.path:
    sys.path.insert(0, ORACLE_DIR)

import wc_ref  # noqa: E402,F401  (pure-Python restatement)

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        L = ctypes.CDLL(LIB_PATH)
        P, U64, U32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
        L.wco_count.restype = P
        L.wco_count.argtypes = [ctypes.c_char_p, U64, ctypes.c_int]
        L.wco_merged.restype = U64
        L.wco_merged.argtypes = [P, P]
        L.wco_res.restype = U64
        L.wco_res.argtypes = [P, U32, U32, P]
        L.wco_nkeys.restype = U64
        L.wco_nkeys.argtypes = [P]
        L.wco_ntokens.restype = U64
        L.wco_ntokens.argtypes = [P]
        L.wco_free.argtypes = [P]
        L.wco_ihash.restype = U32
        L.wco_ihash.argtypes = [ctypes.c_char_p, U64]
        L.wco_is_letter.restype = ctypes.c_int
        L.wco_is_letter.argtypes = [U32]
        L.wco_unicode_version.restype = ctypes.c_char_p
        L.wco_tokens.restype = U64
        L.wco_tokens.argtypes = [ctypes.c_char_p, U64, ctypes.POINTER(U64), ctypes.POINTER(U32), U64]
        L.mrp_run_single.restype = ctypes.c_int
        L.mrp_run_single.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.mrp_run_parallel.restype = ctypes.c_int
        L.mrp_run_parallel.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.mrp_do_reduce.restype = None
        L.mrp_do_reduce.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.wco_verify_merged.restype = ctypes.c_int
        L.wco_verify_merged.argtypes = [P, U64, P, U64, ctypes.c_int, ctypes.POINTER(U64), ctypes.POINTER(U64),
                                        ctypes.c_char_p, U64]
        _lib = L
    return _lib


class Result:
    def __init__(self, data: bytes, nthreads: int = 8):
        self._data = data           # keep alive: keys alias it
        self.h = lib().wco_count(data, len(data), nthreads)

    def merged(self) -> bytes:
        n = lib().wco_merged(self.h, None)
        buf = ctypes.create_string_buffer(max(n, 1))
        lib().wco_merged(self.h, buf)
        return buf.raw[:n]

    def res(self, nreduce: int, r: int) -> bytes:
        n = lib().wco_res(self.h, nreduce, r, None)
        buf = ctypes.create_string_buffer(max(n, 1))
        lib().wco_res(self.h, nreduce, r, buf)
        return buf.raw[:n]

    @property
    def nkeys(self) -> int:
        return lib().wco_nkeys(self.h)

    @property
    def ntokens(self) -> int:
        return lib().wco_ntokens(self.h)

    def __del__(self):
        try:
            lib().wco_free(self.h)
        except Exception:
            pass


def merged(data: bytes, nthreads: int = 8) -> bytes:
    return Result(data, nthreads).merged()


def verify_merged(data_ptr: int, n: int, merged: bytes, nthreads: int = 16):
    """Exact check of a merged file against n input bytes at host address data_ptr, without
    building the oracle's sorted result (wco_verify_merged: every input token decrements its
    line's count; all must end at 0, keys strictly ascending).  For inputs too large for
    Result (C4 at 64 GiB).  Returns (ok, message, ntokens, nkeys)."""
    msg = ctypes.create_string_buffer(512)
    nt, nk = ctypes.c_uint64(0), ctypes.c_uint64(0)
    mbuf = ctypes.create_string_buffer(merged, len(merged)) if merged else ctypes.create_string_buffer(1)
    rc = lib().wco_verify_merged(data_ptr, n, ctypes.addressof(mbuf), len(merged), nthreads,
                                 ctypes.byref(nt), ctypes.byref(nk), msg, 512)
    return rc == 0, msg.value.decode(errors="replace"), nt.value, nk.value


def tokens(data: bytes):
    n = len(data)
    cap = n // 2 + 1
    st = (ctypes.c_uint64 * cap)()
    ln = (ctypes.c_uint32 * cap)()
    nt = lib().wco_tokens(data, n, st, ln, cap)
    return [data[st[i]:st[i] + ln[i]] for i in range(nt)]


def run_single_files(directory: str, file: str, nmap: int, nreduce: int) -> int:
    return lib().mrp_run_single(directory.encode(), file.encode(), nmap, nreduce)


def run_parallel_files(directory: str, file: str, nmap: int, nreduce: int, nworkers: int) -> int:
    """The master/worker path's work with nworkers worker threads (oracle/mr_port.c)."""
    return lib().mrp_run_parallel(directory.encode(), file.encode(), nmap, nreduce, nworkers)


def do_reduce_files(directory: str, file: str, job: int, nmap: int) -> None:
    """The CPU DoReduce (mapreduce.go:239-280) over mrtmp.<file>-<m>-<job> files in directory."""
    lib().mrp_do_reduce(directory.encode(), file.encode(), job, nmap)


def first_diff(got: bytes, want: bytes) -> str:
    """A short description of where two merged files first differ (pytest's own diff of
    multi-megabyte byte strings takes minutes)."""
    if got == want:
        return "equal"
    g, w = got.splitlines(keepends=True), want.splitlines(keepends=True)
    for i, (a, b) in enumerate(zip(g, w)):
        if a != b:
            return f"line {i}: got {a[:80]!r} want {b[:80]!r} ({len(g)} vs {len(w)} lines)"
    return f"prefix equal, {len(g)} vs {len(w)} lines, {len(got)} vs {len(want)} bytes"


def assert_same(got: bytes, want: bytes) -> None:
    if got != want:
        raise AssertionError(first_diff(got, want))
