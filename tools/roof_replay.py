#!/usr/bin/env python3
"""Locality-matched roofline of k_trace: replay every trace launch's own record
fetches and compare k_trace's time with the replay's.

  python tools/roof_replay.py --lib raytracingrenderer_amd/lib/debug/librtg.so [bench-like args]

Runs in two processes: (1) the product library (raytracingrenderer_amd/lib/librtg.so) renders the
C3 workload once with RTG_OPT_TIMING for the per-launch k_trace times, and once in counting mode
for the fetches per launch; (2) the diagnostic build (RTG_DEBUG=1) captures, launch by launch, the
record fetches of every ray (rtg_debug_capture) and replays them on the device (rtg_debug_replay).
Per launch: achieved = fetches / k_trace time; ceiling = replayed fetches / replay time. Writes one
JSON line per launch and a total line (stdout)."""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def scene(a):
    from raytracingrenderer_amd import loadScene, write_synthetic_scene
    if a.config != "C3":
        from bench import CONFIGS, scene_dir
        c = CONFIGS[a.config]
        return loadScene(scene_dir(c["scene"]), width=a.width, height=a.height,
                         skip_missing=c.get("skip_missing", False), envmap=c.get("envmap"))
    d = tempfile.mkdtemp(prefix="rtg_roof_")
    write_synthetic_scene(d, n_tris=a.tris, seed=20251015, width=a.width, height=a.height)
    return loadScene(d)


def tiles(a):
    """rank 0's tiles of a frame split over --shard-of ranks (None: the whole frame)."""
    if a.shard_of <= 1:
        return None
    from raytracingrenderer_amd.distributed import tiles_for_rank
    return tiles_for_rank(a.width, a.height, 0, a.shard_of)


def product(a):
    """k_trace ms per launch (timed) and the fetch count of the whole render (counting pass)."""
    from raytracingrenderer_amd import RayTracer
    from raytracingrenderer_amd import _native as N
    s = scene(a)
    tl = tiles(a)
    rt = RayTracer(s, max_depth=a.max_depth, seed=1234)
    rt.set_options(flags=N.RTG_OPT_CULL)
    rt.render(a.spp, tiles=tl, first_sample=0)  # warm-up
    best = None
    for _ in range(a.reps):
        rt.clear()
        rt.set_options(flags=N.RTG_OPT_CULL | N.RTG_OPT_TIMING)
        rt.render(a.spp, tiles=tl, first_sample=0)
        n = C.c_uint32()
        ms = (C.c_double * 64)()
        N.rtg().rtg_launch_times(rt._h, ms, 64, C.byref(n))
        t = list(ms[:n.value])
        best = t if best is None else [min(x, y) for x, y in zip(best, t)]
    rt.clear()
    rt.set_options(flags=N.RTG_OPT_CULL | N.RTG_OPT_COUNT)
    rt.render(a.spp, tiles=tl, first_sample=0)
    st = rt.stats()
    fetches = st["node_lane_steps"] + st["tri_tests"] + st["shadow_tri_tests"] + st["leafbox_tests"]
    print(json.dumps({"launch_ms": best, "count_fetches": fetches, "chunk_spp": st["chunk_samples"],
                      "rays": st["extension_rays"] + st["shadow_rays"]}), flush=True)


def replay(a):
    from raytracingrenderer_amd import RayTracer
    from raytracingrenderer_amd import _native as N
    s = scene(a)
    tl = tiles(a)
    rt = RayTracer(s, max_depth=a.max_depth, seed=1234)
    rt.set_options(flags=N.RTG_OPT_CULL)
    L = N.rtg()
    for b in range(a.max_depth + 3):
        rt.clear()
        assert L.rtg_debug_capture(rt._h, b) == 0, L.rtg_last_error()
        rt.render(a.spp, tiles=tl, first_sample=0)
        out = (C.c_double * 4)()
        assert L.rtg_debug_replay(rt._h, out) == 0, L.rtg_last_error()
        print(json.dumps({"launch": b, "replay_ms": out[0], "replayed_fetches": out[1],
                          "ext_rays": out[2], "shadow_rays": out[3]}), flush=True)
    L.rtg_debug_capture(rt._h, -1)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=os.path.join(ROOT, "raytracingrenderer_amd", "lib", "debug", "librtg.so"))
    p.add_argument("--mode", default="all", choices=["all", "product", "replay"])
    p.add_argument("--config", default="C3", help="a bench.py config (scene, size, spp, depth)")
    p.add_argument("--tris", type=int, default=1_000_000)
    p.add_argument("--width", type=int, default=0)
    p.add_argument("--height", type=int, default=0)
    p.add_argument("--spp", type=int, default=0)
    p.add_argument("--max-depth", type=int, default=0)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--shard-of", type=int, default=1, help="rank 0's tiles of an N-way split (bench --shard-of)")
    a = p.parse_args()
    from bench import CONFIGS
    c = CONFIGS[a.config]
    a.width = a.width or c["width"]
    a.height = a.height or c["height"]
    a.spp = a.spp or c["spp"]
    a.max_depth = a.max_depth or c["depth"]
    if a.mode == "product":
        return product(a)
    if a.mode == "replay":
        return replay(a)
    base = [sys.executable, os.path.abspath(__file__), "--config", a.config, "--tris", str(a.tris), "--width", str(a.width), "--height",
            str(a.height), "--spp", str(a.spp), "--max-depth", str(a.max_depth), "--reps", str(a.reps), "--shard-of", str(a.shard_of)]
    env = dict(os.environ)
    env.pop("RTG_LIB", None)
    prod = subprocess.run(base + ["--mode", "product"], capture_output=True, text=True, env=env, timeout=900)
    if prod.returncode:
        sys.stderr.write(prod.stderr)
        sys.exit(prod.returncode)
    pr = json.loads(prod.stdout.strip().splitlines()[-1])
    env["RTG_LIB"] = a.lib
    rep = subprocess.run(base + ["--mode", "replay"], capture_output=True, text=True, env=env, timeout=900)
    if rep.returncode:
        sys.stderr.write(rep.stderr)
        sys.exit(rep.returncode)
    rows = [json.loads(l) for l in rep.stdout.splitlines() if l.startswith("{")]
    tot_replayed = tot_replay_ms = tot_ms = 0.0
    for r in rows:
        b = r["launch"]
        r["k_trace_ms"] = pr["launch_ms"][b] if b < len(pr["launch_ms"]) else None
        r["ceiling_g_fetches_per_s"] = r["replayed_fetches"] / r["replay_ms"] / 1e6 if r["replay_ms"] > 0 else None
        tot_replayed += r["replayed_fetches"]
        tot_replay_ms += r["replay_ms"]
        tot_ms += r["k_trace_ms"] or 0.0
        print(json.dumps(r))
    ceiling = tot_replayed / tot_replay_ms / 1e6
    achieved = pr["count_fetches"] / tot_ms / 1e6
    n_launch = len(rows)
    if len(pr["launch_ms"]) != n_launch:
        sys.stderr.write("the render ran %d trace launches, the capture %d: more than one chunk, so the replay "
                         "would not cover the timed launches; use --spp of one chunk\n" % (len(pr["launch_ms"]), n_launch))
        sys.exit(3)
    print(json.dumps({"total": True, "config": a.config, "spp": a.spp, "chunk_spp": pr.get("chunk_spp"),
                      "shard_of": a.shard_of, "count_fetches": pr["count_fetches"], "replayed_fetches": tot_replayed,
                      "k_trace_ms": tot_ms, "replay_ms": tot_replay_ms,
                      "achieved_g_fetches_per_s": achieved, "ceiling_g_fetches_per_s": ceiling,
                      "frac": achieved / ceiling,
                      "note": "ceiling = the launches' own fetch streams replayed (same addresses, per-ray order, "
                              "ray grouping, occupancy, slice work distribution; 8 dependent VALU/step, round 4: 64); "
                              "achieved = counted fetches / k_trace time of the product library"}))


if __name__ == "__main__":
    main()
