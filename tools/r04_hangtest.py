import os, sys, time
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "tests"))
import numpy as np
from raytracingrenderer_amd import RayTracer, loadScene
s = loadScene(os.path.join(os.environ["GRAFT_REPO_ROOT"], "tests/golden/scenes/cornell-box"), width=32, height=32)
for spp, mp in ((4, 0), (64, 0), (65, 0), (130, 0), (130, 1024)):
    t0 = time.time()
    rt = RayTracer(s, seed=1234, max_paths=mp)
    rt.render(spp, first_sample=0)
    f, n = rt.film()
    print(spp, mp, "ok", round(time.time() - t0, 3), float(f.mean()), flush=True)
