"""Ad-hoc GPU bring-up check: GPU film vs oracle on cornell + synthetic, query API, quick timing."""
import hashlib, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raytracingrenderer_amd import loadScene, RayTracer, write_synthetic_scene
from oracle.pyoracle import Oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
def cmp(name, a, b):
    same = np.array_equal(a.view(np.uint32), b.view(np.uint32))
    diff = np.abs(a - b); rel = diff / np.maximum(np.abs(b), 1e-30)
    print("%-28s bitexact=%s maxabs=%.3g frac>1e-4=%.5f" % (name, same, np.nanmax(diff), float(np.mean(rel > 1e-4))), flush=True)
    return same

s = loadScene(os.path.join(ROOT, "tests/golden/scenes/cornell-box"), width=256, height=256)
o = Oracle(s, 4, "rtm")
ref, _ = o.render(4, seed=1234, threads=8)
for cull in (True, False):
    rt = RayTracer(s, seed=1234, cull=cull)
    rt.render(4)
    f, spp = rt.film()
    cmp("cornell256x4 cull=%d" % cull, f, ref)
    print(" md5(film/4)", hashlib.md5((f / 4.0).astype(np.float32).tobytes()).hexdigest(), rt.stats(), flush=True)
# query API
rng = np.random.default_rng(1)
n = 20000
orig = rng.uniform(-1.5, 1.5, (n, 3)).astype(np.float32) + np.array([0, 1, 0], np.float32)
d = rng.normal(size=(n, 3)).astype(np.float32); d /= np.linalg.norm(d, axis=1, keepdims=True)
rays = np.zeros((n, 8), np.float32); rays[:, :3] = orig; rays[:, 4:7] = d; rays[:, 3] = rng.uniform(0.1, 3, n)
rt = RayTracer(s, seed=1234)
cmp("closest query", rt.trace_closest(rays), o.trace_closest(rays))
print("visible query equal:", np.array_equal(rt.trace_visible(rays), o.trace_visible(rays)), flush=True)
# synthetic
sd = "/tmp/synth10k"
write_synthetic_scene(sd, n_tris=10000, seed=7, width=64, height=64)
s2 = loadScene(sd)
o2 = Oracle(s2, 4, "rtm")
ref2, _ = o2.render(4, seed=99, threads=8)
rt2 = RayTracer(s2, seed=99)
rt2.render(4)
cmp("synth10k 64x64x4", rt2.film()[0], ref2)
# timing on synth 1M
sd = "/tmp/synth1m"
t = time.time(); write_synthetic_scene(sd, n_tris=1000000, seed=20251015); print("gen %.1fs" % (time.time() - t), flush=True)
t = time.time(); s3 = loadScene(sd); print("load+bvh %.1fs" % (time.time() - t), s3.info.load_ms, s3.info.bvh_ms, s3.info.bvh_depth, flush=True)
rt3 = RayTracer(s3, seed=5)
rt3.render(1); rt3.synchronize()
for flags in (1, 1 | 4):
    rt3.set_options(flags=flags)
    t = time.time(); rt3.render(8); dt = time.time() - t
    st = rt3.stats()
    print("synth1m 1024^2 x8: %.1f ms  render_ms=%.1f" % (dt * 1e3, st["render_ms"]), st, flush=True)
rt3.set_options(flags=1 | 2)
rt3.clear(); rt3.render(1)
st = rt3.stats()
print("counts", st, flush=True)
