import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import os, numpy as np
from raytracingrenderer_amd import RayTracer, loadScene
s = loadScene(os.path.join("tests", "golden", "scenes", "cornell-box"), width=64, height=64)
rt = RayTracer(s, seed=1)
rt.render(1)
print("render done", rt.film()[1])
