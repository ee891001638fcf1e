import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU cases")


@pytest.fixture(scope="session")
def goldens():
    from tests.golden_io import load_goldens
    return load_goldens()


LIB_SWITCHES = ("VA_F32_SPLIT", "VA_CONV3H", "VA_CONV3T", "VA_CONV3Q", "VA_SPLITK", "VA_SPLITK_KS", "VA_CONV_PATCH",
                "VA_CONV4", "VA_PW", "VA_CT_RUNS", "VA_CT_WGP")


@pytest.fixture
def switch(monkeypatch):
    """switch(name, value) sets one of the library's A/B switches (va355.h va_switches_reload: read once per process)
    for this test and makes the library re-read them; value None unsets it.  Restored after the test."""
    from vision_assist_amd import _lib

    def set_(name: str, value: str | None = None) -> None:
        assert name in LIB_SWITCHES, name
        if value is None:
            monkeypatch.delenv(name, raising=False)
        else:
            monkeypatch.setenv(name, value)
        _lib.load()
        _lib.reload_switches()
    return set_


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_teardown(item):
    yield  # the fixtures (monkeypatch's environment) are restored by now: the library re-reads its switches
    lib = sys.modules.get("vision_assist_amd._lib")
    if lib is not None and getattr(lib, "_LIB", None) is not None:
        lib.reload_switches()
