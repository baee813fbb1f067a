import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mit-6.824-2015_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

# One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same soname as
# /opt/rocm's).  Loading torch first makes libwcg bind to the runtime torch uses; loading libwcg
# first would put the system runtime under torch, which then finds no GPU.
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: larger CPU-side cases")


@pytest.fixture(scope="session")
def built():
    """Build every native artefact once (hipcc cross-compiles without a GPU)."""
    import __graft_entry__ as g
    g.build()
    return True
