import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")
SCENES = os.path.join(GOLD, "scenes")
REF_ROOT = "/root/reference/RTBase"
ASSETS = os.path.join(ROOT, "assets")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through librtg.so)")


@pytest.fixture(scope="session", autouse=True)
def native_build():
    """Compile the native libraries (host, HIP, oracle, _ref when available) once per session."""
    from raytracingrenderer_amd import build
    build.build_host()
    build.build_oracle()
    if os.path.exists(build.HIPCC):
        build.build_device()
    build.build_ref()
    yield


def scene_path(name):
    """Scene directory: committed fixture, staged asset, or the reference tree (build container)."""
    for base in (SCENES, ASSETS, REF_ROOT):
        p = os.path.join(base, name)
        if os.path.isdir(p):
            return p
    return None


def has_gpu():
    try:
        from raytracingrenderer_amd import _native as N
        import ctypes as C
        n = C.c_int(0)
        N.rtg().rtg_device_count(C.byref(n))
        return n.value > 0
    except Exception:
        return False
