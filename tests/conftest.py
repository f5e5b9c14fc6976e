import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_PY = os.path.join(ROOT, "open-source-search-engine_amd", "python")
for p in (PKG_PY, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C ABI on the device)")


def _ensure_built():
    lib = os.path.join(ROOT, "open-source-search-engine_amd", "lib", "libgbgpu.so")
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "open-source-search-engine_amd"), "-j8"])
    if not os.path.exists(orc):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])


_ensure_built()


@pytest.fixture(scope="session")
def engine():
    import gbgpu
    # torch (device tensors in some tests) brings its own HIP runtime, which
    # must initialise before the library's on the GPU box
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except ImportError:
        pass
    e = gbgpu.Engine(0)
    yield e
    e.close()
