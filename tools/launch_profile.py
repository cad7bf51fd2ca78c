"""Per trace launch of one waited-for render: device ms (RTG_OPT_TIMING events) and the rays it walked
(rtg_launch_rays), for the tail analysis of DESIGN.md §7. usage: python tools/launch_profile.py [--shard-of N]
[--config C3]; prints one JSON line."""
import argparse
import ctypes as C
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--shard-of", type=int, default=1)
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    from raytracingrenderer_amd import RayTracer, loadScene, write_synthetic_scene
    from raytracingrenderer_amd import _native as N
    from raytracingrenderer_amd.distributed import tiles_for_rank
    work = tempfile.mkdtemp(prefix="rtg_lp_")
    write_synthetic_scene(work, n_tris=1_000_000, seed=20251015, width=1024, height=1024)
    s = loadScene(work)
    rt = RayTracer(s, max_depth=4, seed=1234)
    tiles = tiles_for_rank(1024, 1024, 0, a.shard_of) if a.shard_of > 1 else None
    rt.set_options(flags=N.RTG_OPT_CULL | N.RTG_OPT_TIMING)
    rt.render(64, tiles=tiles, first_sample=0)  # warm-up
    best = None
    for _ in range(a.reps):
        rt.clear()
        rt.render(64, tiles=tiles, first_sample=0)
        n = C.c_uint32()
        ms = (C.c_double * 64)()
        N.rtg().rtg_launch_times(rt.handle, ms, 64, C.byref(n))
        t = [round(ms[i], 4) for i in range(n.value)]
        rays = (C.c_uint64 * 64)()
        N.rtg().rtg_launch_rays(rt.handle, rays, 64, C.byref(n))
        r = [int(rays[i]) for i in range(n.value)]
        if best is None or sum(t) < sum(best[0]):
            best = (t, r)
    t, r = best
    print(json.dumps({"shard_of": a.shard_of, "trace_ms": t, "rays": r, "total_ms": round(sum(t), 3),
                      "mrays_per_ms": [round(x / 1e6 / max(y, 1e-9), 2) for x, y in zip(r, t)]}))


if __name__ == "__main__":
    main()
