import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libalbedo_als.so")


@pytest.fixture(scope="session")
def gpu_lib():
    """The engine library on a box with a gfx950 device.  A gpu-marked test never falls back:
    missing library or device is a failure, not a skip."""
    from albedo_amd import _lib
    lib = _lib.load()
    n = _lib.device_count()
    assert n > 0, "no gfx950 device visible to libalbedo_als.so"
    return lib


@pytest.fixture(autouse=True)
def _isolated_data_dir(tmp_path, monkeypatch):
    """albedo's date-keyed caches (settings.data_dir) live in the test's own directory."""
    monkeypatch.setenv("ALBEDO_DATA_DIR", str(tmp_path / "spark-data"))
