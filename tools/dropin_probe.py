#!/usr/bin/env python3
"""Drop-in frame loop probe: C3 (synth-1M, 1024^2, MAX_DEPTH 4) rendered as F
one-sample render calls, queued (rtg_render_async) or synchronous, with the host time of every call.
Run it under `rocprofv3 --kernel-trace` and feed the trace to tools/overlap.py to see whether the
frames' kernels overlap on the GPU.

  python tools/dropin_probe.py [--frames 64] [--policy queued|sync] [--tris N]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from raytracingrenderer_amd import RayTracer, loadScene, write_synthetic_scene  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=64)
    p.add_argument("--policy", default="queued", choices=["queued", "sync"])
    p.add_argument("--tris", type=int, default=1_000_000)
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--no-coalesce", action="store_true", help="RTG_OPT_NO_COALESCE: every queued call issued at once")
    a = p.parse_args()
    d = tempfile.mkdtemp(prefix="rtg_probe_")
    write_synthetic_scene(d, n_tris=a.tris, seed=20251015, width=1024, height=1024)
    rt = RayTracer(loadScene(d), max_depth=4, seed=1234)
    if a.no_coalesce:
        from raytracingrenderer_amd import _native as N
        rt.set_options(flags=rt.flags | N.RTG_OPT_NO_COALESCE)
    for f in range(4):  # warm: every slot's buffers
        rt.render(1, first_sample=f, sync=False)
    rt.synchronize()
    for rep in range(a.reps):
        rt.clear()
        calls = []
        t0 = time.perf_counter()
        for f in range(a.frames):
            c0 = time.perf_counter()
            rt.render(1, first_sample=f, sync=(a.policy == "sync"))
            calls.append(time.perf_counter() - c0)
        t1 = time.perf_counter()
        rt.synchronize()
        t2 = time.perf_counter()
        c = np.array(calls) * 1e3
        print(json.dumps({"rep": rep, "policy": a.policy + ("_each" if a.no_coalesce else ""), "frames": a.frames, "wall_ms_per_frame": round((t2 - t0) * 1e3 / a.frames, 4),
                          "enqueue_ms_total": round((t1 - t0) * 1e3, 2), "drain_ms": round((t2 - t1) * 1e3, 2),
                          "call_ms": {"p10": round(float(np.percentile(c, 10)), 4), "p50": round(float(np.median(c)), 4),
                                      "p90": round(float(np.percentile(c, 90)), 4), "max": round(float(c.max()), 4),
                                      "first4": [round(float(x), 4) for x in c[:4]]}}), flush=True)


if __name__ == "__main__":
    main()
