"""Create / render / destroy many handles in one process (the GPU test suite's pattern), eager and
queued renders, to find a hang in handle teardown. Prints progress every 10 handles."""
import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from raytracingrenderer_amd import RayTracer, loadScene
from raytracingrenderer_amd import _native as N
root = os.environ.get("GRAFT_REPO_ROOT", ".")
s = loadScene(os.path.join(root, "tests/golden/scenes/cornell-mat"), width=64, height=35)
t0 = time.time()
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 200):
    rt = RayTracer(s, seed=7, max_depth=8, max_paths=(300 if i % 3 == 0 else 0))
    if i % 2:
        rt.set_options(flags=rt.flags | N.RTG_OPT_SERIAL)
    rt.render(2, first_sample=0)
    rt.render(1, first_sample=2, sync=False)
    f, n = rt.film()
    del rt
    if i % 10 == 0:
        print(i, round(time.time() - t0, 2), flush=True)
print("done", round(time.time() - t0, 2), flush=True)
