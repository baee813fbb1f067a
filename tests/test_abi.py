"""CPU tests of the drop-in boundary: libwcg.so loads and exports every symbol include/wcg.h
declares (no compute calls: there is no GPU in the build container)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "wcg.h")).read()
    return sorted(set(re.findall(r"^WCG_API\s+[\w\s\*]+?\b(wcg_\w+)\(", src, flags=re.M)))


def test_header_declares_the_abi():
    syms = header_symbols()
    for s in ("wcg_open", "wcg_map", "wcg_map_device", "wcg_reduce", "wcg_partition", "wcg_export",
              "wcg_import", "wcg_close", "wcg_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol(built):
    import wcg
    lib = ctypes.CDLL(wcg._lib.LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert missing == []
    assert sorted(header_symbols()) == sorted(wcg.EXPORTED)


def test_host_helpers_without_gpu(built):
    import wcg
    assert wcg.ihash(b"the") == 0xB40EB21C and wcg.ihash(b"") == 0x811C9DC5
    assert "gfx950" in wcg.version() and "13.0.0" in wcg.version()


def test_kernels_are_gfx950_code_objects(built):
    import wcg
    blob = open(wcg._lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
