"""In-tree native build for the MI355X path tracer.

Outputs (git-ignored, shipped to the GPU box with the source snapshot):
  raytracingrenderer_amd/lib/librth.so       host front-end (C++17, g++)         include/rth.h
  raytracingrenderer_amd/lib/librtg.so       HIP kernels + C-ABI (hipcc gfx950)  include/rtg.h
  raytracingrenderer_amd/lib/rtg_render      headless CLI (-scene -SPP -outputFilename)
  raytracingrenderer_amd/lib/debug/librtg.so diagnostic build (RTG_DEBUG=1: per-wave clocks, fetch
                                             capture + replay; tools/roof_replay.py, tools/wavetime.py)
  oracle/_build/liboracle_rtm.so             test-only CPU restatement, shared math
  oracle/_build/liboracle_libm.so            test-only CPU restatement, C-library math
  oracle/_build/libm_check                   test-only: include/rtg_math.h vs the host glibc
  oracle/_build/div_rewrites                 test-only: k_shade's reciprocal products vs the divisions
Every float-producing unit is compiled with -ffp-contract=off (bit-faithful arithmetic).
"""
import os
import shutil
import subprocess
import tempfile
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "raytracingrenderer_amd")
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib")
ORACLE = os.path.join(ROOT, "oracle")
ORACLE_BUILD = os.path.join(ORACLE, "_build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RTG_ARCH", "gfx950")

HOST_SRC = ["host/image_io.cpp", "host/jpeg_decode.cpp", "host/gem_json.cpp", "host/scene_front.cpp"]
DEVICE_SRC = ["device/rtg_kernels.hip", "device/rtg_shade.hip", "device/rtg_light.hip", "device/rtg_multi.hip",
              "device/rtg_bvh.hip"]
# per-unit compile flags: k_shade's translation unit takes LLVM's max-ilp scheduler, which its
# latency-bound body prefers, while the traversal keeps the default; the traversal's
# unit is built without SLP vectorisation, whose packed FP32 pairs in the triangle test held k_trace at
# 80 VGPRs (6 waves per SIMD); without them it needs 64 and runs at 7 (C3 +4 %). k_shade
# without it too: 62 instead of 68 VGPRs, fewer pair moves (C5 shading -4 %)
DEVICE_FLAGS = {"device/rtg_shade.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp", "-fno-slp-vectorize"],
                "device/rtg_kernels.hip": ["-fno-slp-vectorize"]}


def _newer(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


HOST_CXXFLAGS = ["-std=c++17", "-O2", "-ffp-contract=off", "-fPIC", "-shared", "-Wall"]
DEVICE_CXXFLAGS = ["-O3", "-ffp-contract=off", "-std=c++17", "-fPIC"]
DEVICE_LDFLAGS = ["-ldl", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"]


def source_hash(which, debug=False):
    """Build id of a library: sha256 (16 hex digits) over its sources, every header it can include
    (include/, csrc/<host|device>/*.h) and its compile flags. Embedded in the library
    (rtg_build_id / rth_build_id); smoke() and the GPU tests check it against the tree they run in,
    and the build rebuilds whenever the embedded id differs (not by file times)."""
    import hashlib
    hsh = hashlib.sha256()
    if which == "device":
        src = DEVICE_SRC
        flags = [ARCH] + DEVICE_CXXFLAGS + DEVICE_LDFLAGS + sum((DEVICE_FLAGS.get(r, []) for r in DEVICE_SRC), [])
        flags += ["-DRTG_DEBUG=1"] if debug else []
    else:
        src = HOST_SRC
        flags = HOST_CXXFLAGS
    files = [os.path.join(CSRC, r) for r in src] + sorted(_deps([]))
    for f in files:
        hsh.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            hsh.update(fh.read())
    hsh.update(" ".join(flags).encode())
    return hsh.hexdigest()[:16]


def embedded_id(path, tag):
    """The build id a built library carries (the `tag` + 16 hex digits string), or None."""
    try:
        data = open(path, "rb").read()
    except OSError:
        return None
    i = data.find(tag.encode())
    if i < 0:
        return None
    return data[i + len(tag):i + len(tag) + 16].decode("ascii", "replace")


def _stale(out, which, tag, debug=False):
    return not os.path.exists(out) or embedded_id(out, tag) != source_hash(which, debug)


def _deps(paths):
    extra = [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))]
    for sub in ("host", "device"):
        d = os.path.join(CSRC, sub)
        extra += [os.path.join(d, f) for f in os.listdir(d) if f.endswith(".h")]
    return list(paths) + extra


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build failed: " + " ".join(cmd))
    return r


def build_host(force=False):
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, "librth.so")
    src = [os.path.join(CSRC, s) for s in HOST_SRC]
    if force or _stale(out, "host", "rth-build-id:"):
        _run(["g++"] + HOST_CXXFLAGS + ['-DRTH_BUILD_ID="%s"' % source_hash("host"), "-o", out] + src +
             ["-lz", "-lpthread"])
    return out


def build_device(force=False, debug=False):
    d = os.path.join(LIB, "debug") if debug else LIB
    os.makedirs(d, exist_ok=True)
    out = os.path.join(d, "librtg.so")
    src = [os.path.join(CSRC, s) for s in DEVICE_SRC]
    if force or _stale(out, "device", "rtg-build-id:", debug):
        bid = source_hash("device", debug)
        # one object per unit (each with its own flags, compiled in parallel), then one link
        with tempfile.TemporaryDirectory() as tmp:
            objs, procs = [], []
            for rel, path in zip(DEVICE_SRC, src):
                obj = os.path.join(tmp, os.path.basename(rel) + ".o")
                cmd = ([HIPCC, "--offload-arch=" + ARCH] + DEVICE_CXXFLAGS + ['-DRTG_BUILD_ID="%s"' % bid] +
                       (["-DRTG_DEBUG=1"] if debug else []) + DEVICE_FLAGS.get(rel, []) + ["-c", "-o", obj, path])
                procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
                objs.append(obj)
            for cmd, pr in procs:
                log = pr.communicate()[0]
                if pr.returncode != 0:
                    sys.stderr.write(log)
                    raise RuntimeError("build failed: " + " ".join(cmd))
            _run([HIPCC, "--offload-arch=" + ARCH, "-fPIC", "-shared", "-o", out] + objs + DEVICE_LDFLAGS)
    return out


def build_variant(name, extra_flags):
    """A/B variant of librtg (tools/mkab.sh): the product's units and flags plus `extra_flags`
    (e.g. -DRTG_FOO=1), into lib/ab/<name>.so; loaded through RTG_LIB by tools/ab*.sh. A flag written
    `unit:flag` (e.g. `rtg_kernels:-fslp-vectorize`) goes to that unit only; extra flags come after the
    product's, so they override them."""
    d = os.path.join(LIB, "ab")
    os.makedirs(d, exist_ok=True)
    out = os.path.join(d, name + ".so")
    src = [os.path.join(CSRC, s) for s in DEVICE_SRC]
    with tempfile.TemporaryDirectory() as tmp:
        objs, procs = [], []
        for rel, path in zip(DEVICE_SRC, src):
            obj = os.path.join(tmp, os.path.basename(rel) + ".o")
            unit = os.path.splitext(os.path.basename(rel))[0]
            flags = [f.split(":", 1)[1] if ":" in f else f for f in extra_flags
                     if ":" not in f or f.split(":", 1)[0] == unit]
            cmd = ([HIPCC, "--offload-arch=" + ARCH] + DEVICE_CXXFLAGS + ['-DRTG_BUILD_ID="ab-%s"' % name] +
                   DEVICE_FLAGS.get(rel, []) + flags + ["-c", "-o", obj, path])
            procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
            objs.append(obj)
        for cmd, pr in procs:
            log = pr.communicate()[0]
            if pr.returncode != 0:
                sys.stderr.write(log)
                raise RuntimeError("build failed: " + " ".join(cmd))
        _run([HIPCC, "--offload-arch=" + ARCH, "-fPIC", "-shared", "-o", out] + objs + DEVICE_LDFLAGS)
    return out


def build_cli(force=False):
    out = os.path.join(LIB, "rtg_render")
    src = [os.path.join(CSRC, "host", "cli.cpp")]
    if not os.path.exists(src[0]):
        return None
    if force or _newer(out, _deps(src) + [os.path.join(LIB, "librth.so")]):
        _run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-o", out] + src +
             ["-L" + LIB, "-lrth", "-lrtg", "-Wl,-rpath,$ORIGIN", "-ldl"])
    return out


def build_oracle(force=False):
    """Test infrastructure: the C restatement (checker / cpu_baseline only)."""
    os.makedirs(ORACLE_BUILD, exist_ok=True)
    src = os.path.join(ORACLE, "rt_oracle.c")
    outs = []
    for flavour, libm in (("rtm", "0"), ("libm", "1")):
        out = os.path.join(ORACLE_BUILD, "liboracle_%s.so" % flavour)
        if force or _newer(out, _deps([src])):
            _run(["gcc", "-std=c11", "-O2", "-ffp-contract=off", "-fPIC", "-shared", "-D_GNU_SOURCE",
                  "-DORACLE_LIBM=" + libm, "-o", out, src, "-lm", "-lpthread"])
        outs.append(out)
    chk = os.path.join(ORACLE_BUILD, "libm_check")
    chk_src = os.path.join(ORACLE, "libm_check.c")
    if force or _newer(chk, _deps([chk_src])):
        _run(["gcc", "-std=c11", "-O2", "-ffp-contract=off", "-fno-builtin", "-pthread", "-o", chk, chk_src, "-lm"])
    outs.append(chk)
    # the divisions by pi that k_shade computes as products with a reciprocal, checked exhaustively
    dv = os.path.join(ORACLE_BUILD, "div_rewrites")
    dv_src = os.path.join(ORACLE, "div_rewrites.c")
    if force or _newer(dv, [dv_src]):
        _run(["gcc", "-std=c11", "-O2", "-ffp-contract=off", "-D_GNU_SOURCE", "-pthread", "-o", dv, dv_src, "-lm"])
    outs.append(dv)
    return outs


SAN_FLAGS = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
             "-ffp-contract=off"]


def build_sanitized(force=False):
    """Test infrastructure: the host front-end's sources (librth) and the C oracle built with
    AddressSanitizer + UBSan into one driver, tests/native/_build/host_sanitize
    (tests/native/host_sanitize.cpp: scenes, textures and corrupted copies of every input file;
    tests/test_sanitize.py runs it). CPU only; nothing on the GPU is sanitized."""
    nat = os.path.join(ROOT, "tests", "native")
    out_dir = os.path.join(nat, "_build")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "host_sanitize")
    drv = os.path.join(nat, "host_sanitize.cpp")
    orc = os.path.join(ORACLE, "rt_oracle.c")
    src = [os.path.join(CSRC, s) for s in HOST_SRC]
    if force or _newer(out, _deps(src + [drv, orc])):
        obj = os.path.join(out_dir, "rt_oracle_san.o")
        _run(["gcc", "-std=c11", "-D_GNU_SOURCE", "-DORACLE_LIBM=0", "-c", "-o", obj, orc] + SAN_FLAGS)
        _run(["g++", "-std=c++17", "-o", out, drv] + src + [obj] + SAN_FLAGS + ["-lz", "-lpthread", "-lm"])
    return out


def build_sbvh_check(force=False):
    """Test infrastructure: tests/native/sbvh_check (rtg_bvh.hip's host code + librth, no GPU code
    run) into tests/native/_build/; tests/test_bvh.py runs it."""
    nat = os.path.join(ROOT, "tests", "native")
    out_dir = os.path.join(nat, "_build")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "sbvh_check")
    src = [os.path.join(nat, "sbvh_check.cpp"), os.path.join(CSRC, "device", "rtg_bvh.hip")]
    if force or _newer(out, _deps(src) + [os.path.join(LIB, "librth.so")]):
        _run([HIPCC, "-O2", "-std=c++17", "-ffp-contract=off", "-o", out] + src +
             ["-L" + LIB, "-lrth", "-Wl,-rpath," + LIB])
    return out


def build_ref(force=False):
    """oracle/_ref: the reference's own compilable headers, only when /root/reference exists."""
    mk = os.path.join(ORACLE, "ref", "Makefile")
    if not os.path.isdir("/root/reference/RTBase") or not os.path.exists(mk):
        return None
    _run(["make", "-s", "-C", os.path.join(ORACLE, "ref")] + (["-B"] if force else []))
    return os.path.join(ORACLE, "_ref", "libref.so")


def stage_assets():
    """Copy reference scene data (not code) used by tests/bench into assets/ (git-ignored, travels
    to the GPU box): coffee (config C5), bathroom (C4), materialball (the env-lit scene) and GI.hdr.
    Only when /root/reference is present."""
    src = "/root/reference/RTBase"
    dst = os.path.join(ROOT, "assets")
    if not os.path.isdir(src):
        return
    os.makedirs(dst, exist_ok=True)
    for name in ("coffee", "bathroom", "materialball"):
        if os.path.isdir(os.path.join(src, name)) and not os.path.isdir(os.path.join(dst, name)):
            shutil.copytree(os.path.join(src, name), os.path.join(dst, name))
    for f, into in (("GI.hdr", ""), ("GI.hdr", "coffee")):  # C5 = coffee_f + "envmap": "GI.hdr"
        d = os.path.join(dst, into, f)
        if os.path.exists(os.path.join(src, f)) and os.path.isdir(os.path.dirname(d)) and not os.path.exists(d):
            shutil.copy(os.path.join(src, f), d)


def build_all(force=False, device=True):
    stage_assets()
    build_host(force)
    if device:
        build_device(force)
        build_device(force, debug=True)
    build_cli(force)
    build_oracle(force)
    build_ref(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, device="--no-device" not in sys.argv)
    print("ok")
