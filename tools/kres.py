#!/usr/bin/env python3
"""VGPR / spill / LDS of the kernels in rtg_kernels.hip for gfx950 (no GPU needed):
python tools/kres.py [-D...]"""
import os, re, subprocess, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "raytracingrenderer_amd", "csrc", "device", "rtg_kernels.hip")
with tempfile.TemporaryDirectory() as d:
    out = os.path.join(d, "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
                    "--cuda-device-only", "-S", "-o", out, SRC] + sys.argv[1:], check=True)
    s = open(out).read()
md = s[s.index("amdhsa.kernels"):]
for blk in md.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    f = {k: int(re.search(r"\." + k + r":\s+(\d+)", blk).group(1))
         for k in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "group_segment_fixed_size")}
    print("%-40s vgpr %3d sgpr %3d spill v%d s%d lds %d" % (name[:40], f["vgpr_count"], f["sgpr_count"],
          f["vgpr_spill_count"], f["sgpr_spill_count"], f["group_segment_fixed_size"]))
