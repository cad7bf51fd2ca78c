"""Register budget of the hot kernels (compiled here for gfx950, no GPU needed): a change that
makes the traversal or shading kernel spill in its loop costs ~15 % (a scratch reload per node
step is a vector-memory request in a request-bound loop), so the spill counts are pinned."""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEVICE = os.path.join(ROOT, "raytracingrenderer_amd", "csrc", "device")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    from raytracingrenderer_amd.build import DEVICE_FLAGS  # each unit with the flags the build uses
    res = {"_asm": {}}
    for rel in ("device/rtg_kernels.hip", "device/rtg_shade.hip"):
        with tempfile.TemporaryDirectory() as d:
            out = os.path.join(d, "k.s")
            subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17"] +
                           DEVICE_FLAGS.get(rel, []) + ["--cuda-device-only", "-S", "-o", out,
                                                        os.path.join(DEVICE, os.path.basename(rel))],
                           check=True, capture_output=True)
            s = open(out).read()
        res["_asm"][rel] = s
        md = s[s.index("amdhsa.kernels"):]
        for blk in md.split("  - .agpr_count")[1:]:
            name = re.search(r"\.name:\s+(\S+)", blk).group(1)
            res[name] = {k: int(re.search(r"\." + k + r":\s+(\d+)", blk).group(1))
                         for k in ("vgpr_count", "vgpr_spill_count", "sgpr_count", "sgpr_spill_count",
                                   "private_segment_fixed_size", "group_segment_fixed_size")}
    return res


def _find(kernels, prefix):
    names = [k for k in kernels if k.startswith(prefix) and k != "_asm"]
    assert names, prefix
    return kernels[names[0]]


def test_traversal_fits_seven_waves_without_spills(kernels):
    """k_trace (global-memory walk) at 7 waves per SIMD: VGPRs <= 72 (512 / 7, granule 8), SGPRs
    <= 96 (800 / (ceil(n / 16) * 16 + 16) >= 7, MI355X_MICROARCH.md 'Residency'), no VGPR spills, and
    a one-wave block's LDS (the 16-entry stack) small enough for 28 blocks per CU."""
    k = _find(kernels, "_Z7k_traceILb0ELb0E")
    assert k["vgpr_count"] <= 72, k
    assert k["sgpr_count"] <= 96, k
    assert k["vgpr_spill_count"] == 0 and k["private_segment_fixed_size"] == 0, k
    assert 28 * k["group_segment_fixed_size"] <= 160 * 1024 and k["group_segment_fixed_size"] <= 4608, k
    # the small-scene variant (scene image + 7-entry stack in LDS) at the same 7 blocks per SIMD
    ks = _find(kernels, "_Z7k_traceILb0ELb1E")
    assert ks["vgpr_count"] <= 72 and ks["sgpr_count"] <= 96 and ks["vgpr_spill_count"] == 0, ks
    assert ks["group_segment_fixed_size"] <= 5120, ks


def test_shading_kernel_does_not_spill(kernels):
    k = _find(kernels, "_Z7k_shadeILb0E")
    assert k["vgpr_spill_count"] == 0 and k["private_segment_fixed_size"] == 0, k


def test_shade_tables_are_waited_for_before_the_barrier(kernels):
    """k_shade<.., TAB = true> fills its material / light tables with global_load_lds, which
    completes on vmcnt; other waves read them after the block barrier. The instruction before that
    first s_barrier must be an s_waitcnt with vmcnt(0) (rtg_shade.hip issues it explicitly)."""
    s = kernels["_asm"]["device/rtg_shade.hip"]
    for name in ("_Z7k_shadeILb0ELb1E", "_Z7k_shadeILb1ELb1E"):
        body = s[s.index(name + "Ev"):]
        body = body[body.index("global_load_lds_dwordx4"):]
        pre = body[:body.index("s_barrier")].strip().splitlines()
        waits = [l.strip() for l in pre if l.strip().startswith("s_waitcnt")]
        assert waits and "vmcnt(0)" in waits[-1], (name, waits[-3:])
