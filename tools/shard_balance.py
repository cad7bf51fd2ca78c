"""Per-rank load of the tile partition at N ranks (one GPU): time and rays of each rank's tiles,
and the job rate they project (film reduce not included).
usage: python tools/shard_balance.py N scheme   (scheme: mod | diag)"""
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raytracingrenderer_amd import RayTracer, loadScene, write_synthetic_scene  # noqa: E402

N = int(sys.argv[1])
scheme = sys.argv[2]
d = tempfile.mkdtemp()
write_synthetic_scene(d, n_tris=1_000_000, seed=20251015)
s = loadScene(d)
rt = RayTracer(s)
tx, ty = 32, 32
t = np.arange(tx * ty, dtype=np.uint32)
x, y = t % tx, t // tx
owner = (t % N) if scheme == "mod" else ((x + y) % N)
res = []
for r in list(range(N)) + list(range(N)):  # two passes; the second is reported
    tiles = t[owner == r]
    rt.clear()
    rt.render(8, tiles=tiles, first_sample=0)  # warm
    rt.clear()
    t0 = time.perf_counter()
    rt.render(64, tiles=tiles, first_sample=0)
    dt = time.perf_counter() - t0
    st = rt.stats()
    res.append((dt * 1e3, (st["extension_rays"] + st["shadow_rays"]) / 1e6))
res = res[N:]
ms = [a for a, _ in res]
print(scheme, N, "ms per rank:", [round(a, 1) for a in ms], "max/mean %.3f" % (max(ms) / np.mean(ms)),
      "Mrays:", [round(b, 1) for _, b in res],
      "projected job Mray/s (all rays / slowest rank): %.0f" % (sum(b for _, b in res) / (max(ms) / 1e3)))
