"""The own tree's spatial splits (rtg_bvh.hip build_sbvh), checked on the CPU:
every child box lies inside its parent's, every triangle has a leaf slot, and every triangle's
vertices and random points lie in one of its fragments' boxes (the coverage the exactness argument
needs). The GPU tests (test_gpu_parity.py wide-walk, grazing and adversarial rays) check the walk."""
import os
import subprocess

import pytest

from conftest import SCENES


@pytest.fixture(scope="module")
def check():
    from raytracingrenderer_amd import build
    if not os.path.exists(build.HIPCC):
        pytest.skip("hipcc not available")
    build.build_host()
    return build.build_sbvh_check()


@pytest.mark.parametrize("args", [["cornell-box"], ["cornell-mat"], ["x", "synth", "20000"], ["x", "synth", "200000"]])
def test_sbvh_tree_contains_and_covers(check, args):
    a = [os.path.join(SCENES, args[0])] + args[1:] if len(args) == 1 else args
    r = subprocess.run([check] + a, capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    f = r.stdout.split()
    assert f[f.index("boxes") + 1] == "0," and f[f.index("tris", 3) + 1] == "0," and f[f.index("points") + 1] == "0"
