import os
import subprocess
import sys

import pytest

# torch bundles its own HIP runtime and links it by the unversioned name "libamdhip64.so": if libspeq_scan.so
# (which binds libamdhip64.so.7) loaded first, torch would load a second HIP runtime that then sees no GPU.
# Importing torch first makes libspeq_scan.so bind to torch's runtime (same SONAME), one runtime per process.
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def _built() -> bool:
    return all(os.path.exists(os.path.join(ROOT, p)) for p in
               ("speq_amd/libspeq_scan.so", "bin/speq", "oracle/build/libkmer_oracle.so"))


@pytest.fixture(scope="session", autouse=True)
def built_artifacts():
    """Builds the library/CLI/oracle once if a previous build() did not (hipcc cross-compiles without a GPU)."""
    if not _built():
        subprocess.run(["make", "-C", ROOT, "-j", str(min(16, os.cpu_count() or 4)), "all"], check=True)
    yield


def gpu_available() -> bool:
    from speq_amd import lib
    return lib().speq_device_count() > 0
