#!/usr/bin/env python3
"""VGPR / spill / LDS of the device kernels for gfx950 (no GPU needed), each translation unit with the
flags the build gives it (build.py DEVICE_FLAGS): python tools/kres.py [-D...]"""
import os, re, subprocess, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raytracingrenderer_amd.build import CSRC, DEVICE_FLAGS, DEVICE_SRC  # noqa: E402

for rel in DEVICE_SRC:
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
                        "--cuda-device-only", "-S", "-o", out, os.path.join(CSRC, rel)] + DEVICE_FLAGS.get(rel, []) +
                       sys.argv[1:], check=True)
        s = open(out).read()
    if "amdhsa.kernels" not in s:
        continue
    md = s[s.index("amdhsa.kernels"):]
    print("==", rel)
    for blk in md.split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        f = {k: int(re.search(r"\." + k + r":\s+(\d+)", blk).group(1))
             for k in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "group_segment_fixed_size")}
        print("%-40s vgpr %3d sgpr %3d spill v%d s%d lds %d" % (name[:40], f["vgpr_count"], f["sgpr_count"],
              f["vgpr_spill_count"], f["sgpr_spill_count"], f["group_segment_fixed_size"]))
