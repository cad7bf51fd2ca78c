"""The north_star parity criterion (BASELINE.json): the GPU film against the
reference CPU render on a fixed seed, within 1e-4 relative per pixel.

"The reference CPU render" is RTBase's own compiled classes (oracle/_ref/libref.so: Scene::traverse /
visible, calculateShadingData, the BSDFs, lights, camera and Film::splat built from
/root/reference, with pathTrace / computeDirect / the tile pool restated on top, and the C library's
acosf / sinf / cosf / atan2f, as RTBase gets them on Linux). libref.so reproduces the survey's C1
known-answer md5 of the reference itself (tests/test_oracle.py).

The device's transcendentals restate glibc's (include/rtg_math.h, checked on every float input), so
the criterion holds with margin: every pixel of every scene is bit-identical, on all five scenes of
BASELINE.json's configs (C1 cornell, C2's cornell at depth 8 with glass / mirror / environment,
C3's synthetic triangles, C4's bathroom_f at depth 16, C5's coffee_f + GI.hdr), and on the one
reference scene whose environment map is a light (materialball_f with envmap.hdr as lights[0]).
The statistics the survey asks for (identical non-finite masks, fraction within 1e-4, image-mean
relative error) are printed as well."""
import os
import tempfile

import numpy as np
import pytest

from conftest import SCENES, scene_path
from oracle.pyoracle import Oracle
from raytracingrenderer_amd import RayTracer, loadScene, write_synthetic_scene

TOL = 1e-4  # relative, per pixel and channel (north_star)


def compare(got_sum, want_sum, spp):
    """Per-pixel statistics of the normalised films (Film::save divides the sum by SPP)."""
    a = got_sum / np.float32(spp)
    b = want_sum / np.float32(spp)
    fa, fb = np.isfinite(a), np.isfinite(b)
    rel = np.where(a == b, 0.0, np.abs(a.astype(np.float64) - b) / np.maximum(np.abs(b.astype(np.float64)), 1e-30))
    ok = (rel <= TOL).all(axis=2) & fa.all(axis=2) & fb.all(axis=2)
    ma, mb = a[fa].astype(np.float64).mean(), b[fb].astype(np.float64).mean()
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    return {"masks_equal": bool(np.array_equal(fa, fb)), "frac_within": float(ok.mean()),
            "mean_rel": float(abs(ma - mb) / max(abs(mb), 1e-30)), "bit_exact_frac": float(same.all(axis=2).mean()),
            "divergent": np.argwhere(~ok)}


def _scene(case):
    """(scene dir, loadScene kwargs, depth, spp) of the five north-star cases."""
    if case == "synth20k":
        d = tempfile.mkdtemp(prefix="rtg_ns_")
        write_synthetic_scene(d, n_tris=20000, seed=3, width=256, height=256)
        return d, dict(width=256, height=256), 4, 4
    if case == "C1":
        return os.path.join(SCENES, "cornell-box"), dict(width=256, height=256), 4, 4
    if case == "cornell-mat":
        return os.path.join(SCENES, "cornell-mat"), dict(width=160, height=120), 8, 8
    name = {"coffee+GI": "coffee", "bathroom": "bathroom", "materialball-d4": "materialball",
            "materialball-d8": "materialball"}[case]
    p = scene_path(name)
    if p is None:
        pytest.fail("%s assets missing (raytracingrenderer_amd.build.stage_assets)" % name)
    if case == "coffee+GI":
        return p, dict(width=200, height=250, skip_missing=True, envmap="GI.hdr"), 4, 4
    if case.startswith("materialball"):  # envmap.hdr is lights[0]: NEE samples the sphere
        return p, dict(width=160, height=90, skip_missing=True), int(case[-1]), 4
    return p, dict(width=192, height=108, skip_missing=True), 16, 4


CASES = ["C1", "synth20k", "cornell-mat", "coffee+GI", "bathroom", "materialball-d4", "materialball-d8"]


@pytest.mark.gpu
@pytest.mark.host_glibc
@pytest.mark.parametrize("case", CASES)
def test_north_star_vs_reference_cpu_render(case):
    """GPU film vs libref.so (RTBase's classes, glibc math): every pixel within 1e-4, bit-identical."""
    from oracle import pyref
    if not pyref.available():
        pytest.fail("oracle/_ref/libref.so missing: build it where /root/reference exists")
    path, kw, depth, spp = _scene(case)
    s = loadScene(path, **kw)
    rt = RayTracer(s, seed=1234, max_depth=depth)
    rt.render(spp, first_sample=0)
    film, n = rt.film()
    assert n == spp
    r = pyref.RefScene(path, kw["width"], kw["height"], kw.get("skip_missing", False), kw.get("envmap"),
                       flavour="libm")
    ref, _ = r.render(spp, seed=1234, max_depth=depth, threads=8)
    st = compare(film, ref, spp)
    print("%s vs the reference CPU render (glibc): %.4f %% of pixels within 1e-4, mean rel %.2e, bit-exact %.4f %%"
          % (case, 100 * st["frac_within"], st["mean_rel"], 100 * st["bit_exact_frac"]))
    assert st["masks_equal"]
    assert st["frac_within"] == 1.0, st["divergent"][:8]
    assert st["mean_rel"] <= 1e-4
    assert st["bit_exact_frac"] == 1.0


@pytest.mark.host_glibc
@pytest.mark.parametrize("case", ["cornell-mat", "bathroom"])
def test_oracle_math_flavours_render_identical_films(case):
    """CPU (oracle builds only): the C oracle with include/rtg_math.h and with the C library's
    transcendentals render the same film bit for bit on the glossy scenes where a 1-ulp
    transcendental difference changes paths (round 2 measured 98.4 % within 1e-4 on bathroom_f
    depth 16 with correctly-rounded functions in place of glibc's)."""
    path, kw, depth, spp = _scene(case)
    if case == "bathroom":
        kw, spp = dict(width=96, height=54, skip_missing=True), 2
    s = loadScene(path, **kw)
    a, ca = Oracle(s, depth, "rtm").render(spp, seed=1234, threads=8)
    b, cb = Oracle(s, depth, "libm").render(spp, seed=1234, threads=8)
    st = compare(a, b, spp)
    assert st["masks_equal"] and st["bit_exact_frac"] == 1.0 and ca.tolist() == cb.tolist()
