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
    config.addinivalue_line("markers", "host_glibc: compares with the host's C library transcendentals, which "
                                       "are the reference platform's only on glibc 2.35 with its FMA build")


_LIBM_REASON = []


def reference_libm_mismatch():
    """None when the host C library's sinf / cosf / acosf / atan2f are the reference platform's:
    glibc 2.35, whose FMA build x86-64 selects by ifunc on CPUs with FMA and AVX2 (what
    include/rtg_math.h restates and profiles/r03_libm_exhaustive.txt checked on all 2^32 inputs).
    Otherwise the reason, for a skip: tests that compare with the host's libm (libref.so, the
    oracle's libm flavour) would then compare with a different libm."""
    if not _LIBM_REASON:
        import ctypes
        why = None
        try:
            f = ctypes.CDLL("libc.so.6").gnu_get_libc_version
            f.restype = ctypes.c_char_p
            ver = f().decode()
        except Exception as e:  # pragma: no cover
            ver = "unknown (%s)" % e
        flags = set()
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("flags"):
                    flags = set(line.split(":", 1)[1].split())
                    break
        except OSError:
            pass
        if ver != "2.35":
            why = "host glibc %s, not 2.35 (include/rtg_math.h restates glibc 2.35's float functions)" % ver
        elif not {"fma", "avx2"} <= flags:
            why = "host CPU lacks FMA/AVX2: glibc 2.35 runs its non-FMA sinf/cosf build here"
        _LIBM_REASON.append(why)
    return _LIBM_REASON[0]


def require_reference_libm():
    why = reference_libm_mismatch()
    if why:
        pytest.skip("host libm is not the reference platform's: " + why)


def pytest_runtest_setup(item):
    if item.get_closest_marker("host_glibc"):
        require_reference_libm()


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
