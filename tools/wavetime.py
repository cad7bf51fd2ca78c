#!/usr/bin/env python3
"""Per-launch wave start / drain / end percentiles of k_trace (drain tails).

  python tools/wavetime.py [--shard-of N] [--lib raytracingrenderer_amd/lib/debug/librtg.so]

Renders the C3 workload (rank 0's tiles of an N-way split) once with the diagnostic build's
RTG_OPT_WAVETIME: the library prints one [wavetime] line per trace launch on stderr (clock of each
wave's start, the first wave to find the work counters dry, each wave's end)."""
import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(a):
    from raytracingrenderer_amd import RayTracer, loadScene, write_synthetic_scene
    from raytracingrenderer_amd import _native as N
    from raytracingrenderer_amd.distributed import tiles_for_rank
    d = tempfile.mkdtemp(prefix="rtg_wt_")
    write_synthetic_scene(d, n_tris=a.tris, seed=20251015, width=a.width, height=a.height)
    rt = RayTracer(loadScene(d), max_depth=a.max_depth, seed=1234)
    tl = tiles_for_rank(a.width, a.height, 0, a.shard_of) if a.shard_of > 1 else None
    rt.set_options(flags=N.RTG_OPT_CULL)
    rt.render(a.spp, tiles=tl, first_sample=0)  # warm-up
    rt.set_options(flags=N.RTG_OPT_CULL | N.RTG_OPT_WAVETIME)
    rt.render(a.spp, tiles=tl, first_sample=0)
    rt.synchronize()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=os.path.join(ROOT, "raytracingrenderer_amd", "lib", "debug", "librtg.so"))
    p.add_argument("--shard-of", type=int, default=1)
    p.add_argument("--tris", type=int, default=1_000_000)
    p.add_argument("--width", type=int, default=1024)
    p.add_argument("--height", type=int, default=1024)
    p.add_argument("--spp", type=int, default=64)
    p.add_argument("--max-depth", type=int, default=4)
    p.add_argument("--child", action="store_true")
    a = p.parse_args()
    if a.child:
        return run(a)
    env = dict(os.environ, RTG_LIB=a.lib)
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"] + sys.argv[1:], env=env,
                       capture_output=True, text=True, timeout=600)
    sys.stdout.write("".join(l + "\n" for l in r.stderr.splitlines() if "[wavetime]" in l))
    if r.returncode:
        sys.stderr.write(r.stderr[-3000:])
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
