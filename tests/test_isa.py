"""Static checks on the gfx950 code of k_map (CPU only: hipcc cross-compiles).

k_map's input stream uses inline-asm loads with hand-counted waits; the compiler must not copy
those registers between a load and its wait.  tools/check_inflight.py verifies that from the
generated assembly (tagged loads/waits must all use the same registers), and the kernel must not
spill to scratch (a scratch reload inside the loop would force a vmcnt(0) that drains the
prefetch)."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "mit-6.824-2015_amd", "csrc", "wcg_api.hip")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_inflight  # noqa: E402

# k_map<0, SPLIT>: one-pass jobs log short and medium keys to separate miss buckets (SPLIT), two-pass
# jobs to one set; both instances carry the same discipline
KMAPS = ["_ZN3wcg5k_mapILi0ELb1EEEvNS_7MapArgsE", "_ZN3wcg5k_mapILi0ELb0EEEvNS_7MapArgsE"]


@pytest.fixture(scope="module")
def device_asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "wcg_api.s"
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--cuda-device-only",
                        "-S", SRC, "-o", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return out.read_text()


@pytest.mark.parametrize("kmap", KMAPS)
def test_map_asm_loads_not_copied_before_wait(device_asm, kmap):
    errors, loads, waits = check_inflight.check(device_asm, kmap)
    assert not errors, errors
    sets = "ABCD"
    assert set(loads) == {s + "0" for s in sets}
    # every set: a counted wait in each unrolled step and the drain after the loop
    assert sorted({w[0] for w in waits}) == list(sets) and len(waits) >= 2 * len(sets)


@pytest.mark.parametrize("kmap", KMAPS)
def test_map_unit_stores_unconditional(device_asm, kmap):
    """The prefetch accounting counts 1 miss-log unit store per short-key iteration, 2 per medium
    iteration and 2 after a step's last medium iteration (r06: carried tokens): they must be the
    inline-asm stores issued by the whole wave, 5 per inlined copy of the step (four register
    sets and the tail), plus the 4 of the drain of the carried tokens after the last step."""
    lines = check_inflight.kernel_lines(device_asm, kmap)
    stores = [l for l in lines if "wcg-store" in l]
    assert stores and all("buffer_store_dwordx2" in l for l in stores)
    assert len(stores) == 5 * 5 + 4, len(stores)


@pytest.mark.parametrize("kmap", KMAPS)
def test_map_no_scratch(device_asm, kmap):
    lines = check_inflight.kernel_lines(device_asm, kmap)
    assert not any(re.search(r"\bscratch_(load|store)", l) for l in lines)
