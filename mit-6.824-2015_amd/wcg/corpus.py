"""Synthetic corpora for the benchmark configs; binding of libgencorpus.so.

The reference's own corpus (src/main/kjv12.txt) is absent (.MISSING_LARGE_BLOBS:2), so every
throughput number is measured on these deterministic generators (see csrc/gencorpus.c).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgencorpus.so")
BLOCK = 1 << 20
_lib = None

ASCII, UTF8 = 0, 1

# named configs of BASELINE.json
CONFIGS = {
    "c2_ascii_zipf_1gib": dict(mode=ASCII, vocab=100_000, zipf_s=1.0, seed=42, nbytes=1 << 30),
    "c3_ascii_zipf_16gib": dict(mode=ASCII, vocab=100_000, zipf_s=1.0, seed=43, nbytes=16 << 30),
    "c4_utf8_zipf_64gib": dict(mode=UTF8, vocab=50_000_000, zipf_s=0.9, seed=44, nbytes=64 << 30),
}


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run __graft_entry__.build()")
        lib = ctypes.CDLL(LIB_PATH)
        lib.wcgen_create.restype = ctypes.c_void_p
        lib.wcgen_create.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_double, ctypes.c_uint64]
        lib.wcgen_destroy.argtypes = [ctypes.c_void_p]
        lib.wcgen_fill.restype = ctypes.c_int
        lib.wcgen_fill.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                   ctypes.c_int]
        _lib = lib
    return _lib


class Generator:
    def __init__(self, mode: int = ASCII, vocab: int = 100_000, zipf_s: float = 1.0, seed: int = 42):
        self._lib = _load()
        self._h = self._lib.wcgen_create(mode, vocab, zipf_s, seed)

    def fill_ptr(self, ptr: int, nbytes: int, first_block: int = 0, threads: int = 0) -> None:
        """Write nbytes of corpus starting at block `first_block` into host memory at ptr."""
        if threads <= 0:
            threads = min(16, os.cpu_count() or 1)
        self._lib.wcgen_fill(self._h, ctypes.c_void_p(ptr), nbytes, first_block, threads)

    def bytes(self, nbytes: int, first_block: int = 0) -> bytes:
        buf = ctypes.create_string_buffer(max(nbytes, 1))
        self.fill_ptr(ctypes.addressof(buf), nbytes, first_block)
        return buf.raw[:nbytes]

    def close(self):
        if self._h:
            self._lib.wcgen_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
