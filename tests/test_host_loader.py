"""Host front-end (librth) vs the reference's own loader/BVH/texture code (golden fixtures made by
tests/golden/make_golden.py from oracle/_ref, i.e. RTBase compiled from /root/reference)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLD, REF_ROOT, SCENES, scene_path
from raytracingrenderer_amd import loadScene, read_hdr, save_hdr, write_synthetic_scene

ARRAYS = ("positions", "normals", "uvs", "material", "node_bounds", "node_links", "lights", "camera")
DIGESTS = json.load(open(os.path.join(GOLD, "scene_digests.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def scene_arrays(s):
    c = s.camera
    cam = np.concatenate([c["inv_proj"].ravel(), c["camera"].ravel(), c["origin"],
                          np.array([c["width"], c["height"]], np.float32)]).astype(np.float32)
    return {"positions": s.positions, "normals": s.normals, "uvs": s.uvs, "material": s.material_index,
            "node_bounds": s.node_bounds, "node_links": s.node_links, "lights": s.lights, "camera": cam}


def test_cornell_bit_exact_vs_reference_loader():
    g = np.load(os.path.join(GOLD, "cornell256_rays.npz"))
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=256, height=256)
    mine = scene_arrays(s)
    for k in ARRAYS:
        assert mine[k].shape == g[k].shape, k
        assert np.array_equal(np.ascontiguousarray(mine[k]).view(np.uint32), g[k].view(np.uint32)), k
    # light triangles sit at post-sort indices 25, 26
    assert list(s.lights) == [25, 26]
    assert s.info.bvh_depth == 9 and s.desc.n_nodes == 45


def _check_digests(name, s):
    d = DIGESTS[name]
    mine = scene_arrays(s)
    assert s.desc.n_tris == d["n_tris"] and s.desc.n_nodes == d["n_nodes"] and s.desc.n_lights == d["n_lights"]
    for k in ARRAYS:
        assert sha(mine[k]) == d[k], "%s: %s differs from the reference loader" % (name, k)
    mi = np.array([[m.kind, m.two_sided] for m in s.materials], np.int32)
    mf = np.array([[m.int_ior, m.ext_ior, m.emission[0], m.emission[1], m.emission[2]] for m in s.materials], np.float32)
    assert sha(mi) == d["mat_info"] and sha(mf) == d["mat_f"]


def test_synthetic_scene_matches_reference_loader(tmp_path):
    write_synthetic_scene(str(tmp_path), n_tris=20000, seed=3, width=128, height=96)
    _check_digests("synth20k", loadScene(str(tmp_path)))


@pytest.mark.parametrize("name,dirname,w,h", [("coffee_f", "coffee", 400, 500), ("bathroom_f", "bathroom", 480, 270),
                                             ("materialball_f", "materialball", 320, 180)])
def test_filtered_scenes_match_reference_loader(name, dirname, w, h):
    p = scene_path(dirname)
    if p is None:
        pytest.skip("scene assets not available here")
    s = loadScene(p, width=w, height=h, skip_missing=True)
    _check_digests(name, s)
    assert s.info.dropped_instances == {"coffee_f": 3, "bathroom_f": 4, "materialball_f": 1}[name]
    if name == "materialball_f":  # the environment is the scene's only light (lights[0] = env: -1)
        assert s.info.env_in_lights == 1 and list(s.lights) == [-1]


def test_synthetic_generator_deterministic(tmp_path):
    a, b, c = (str(tmp_path / x) for x in "abc")
    write_synthetic_scene(a, n_tris=500, seed=11, width=32, height=32)
    write_synthetic_scene(b, n_tris=500, seed=11, width=32, height=32)
    write_synthetic_scene(c, n_tris=500, seed=12, width=32, height=32)
    ha, hb, hc = (sha(loadScene(x).positions) for x in (a, b, c))
    assert ha == hb != hc


@pytest.mark.parametrize("fn", ["bathroom/floor_tiles.png", "bathroom/rug_mask.png", "GI.hdr", "materialball/envmap.hdr",
                                "bathroom/marble.jpg", "bathroom/picture1.jpg", "bathroom/wallpaper-1.jpg",
                                "bathroom/wallpaper-2.jpg", "bathroom/wood.jpg", "bathroom/wood2.jpg"])
def test_texture_decode_matches_stb(fn):
    kat = json.load(open(os.path.join(GOLD, "texture_decode_kat.json")))
    path = os.path.join(REF_ROOT, fn)
    if fn not in kat or not os.path.exists(path):
        pytest.skip("texture not available here")
    if fn.endswith(".hdr"):
        t = read_hdr(path)
    else:
        import ctypes as C
        from raytracingrenderer_amd import _native as N
        w, h, ch = C.c_int32(), C.c_int32(), C.c_int32()
        p = C.POINTER(C.c_uint8)()
        assert N.rth().rth_read_ldr(path.encode(), C.byref(w), C.byref(h), C.byref(ch), C.byref(p)) == 0
        raw = np.ctypeslib.as_array(p, shape=(h.value * w.value * ch.value,)).copy()
        N.rth().rth_free(C.cast(p, C.c_void_p))
        t = (raw.reshape(h.value, w.value, ch.value)[:, :, :3] / np.float32(255.0)).astype(np.float32)
    assert list(t.shape) == kat[fn]["shape"]
    assert sha(t) == kat[fn]["sha256"]


def test_rgbe_writer_byte_exact(tmp_path):
    g = np.load(os.path.join(GOLD, "rgbe_kat.npz"))
    out = str(tmp_path / "film.hdr")
    save_hdr(out, g["film"], int(g["spp"]))
    assert open(out, "rb").read() == g["hdr"].tobytes()
    back = read_hdr(out)
    ref = g["film"] / np.float32(int(g["spp"]))
    # RGBE keeps an 8-bit shared-exponent mantissa: relative error < 2^-7 of the max component
    m = np.maximum(ref.max(axis=2, keepdims=True), 1e-30)
    assert np.all(np.abs(back - ref) <= m * 2.0 ** -7 + 1e-30)


def _rel_src(tmp_path):
    return os.path.relpath(os.path.join(SCENES, "cornell-box"), str(tmp_path / "s0"))


_n_scenes = [0]


def _write_scene(tmp_path, extra_props="", instances=None):
    src = _rel_src(tmp_path)
    insts = instances or ['{"filename": "%s/Rectangle.gem", "world": [1,0,0,0, 0,1,0,0, 0,0,1,0, 0,0,0,1], '
                          '"bsdf": "diffuse", "reflectance": "%s/1_1_1.png", "emission": "1 1 1"}' % (src, src)]
    txt = ('{"width": "64", "height": "48", "fov": "40", "from": "0 0 3", "to": "0 0 0", "up": "0 1 0"%s, '
           '"instances": [%s]}' % (extra_props, ", ".join(insts)))
    _n_scenes[0] += 1
    d = tmp_path / ("s%d" % _n_scenes[0])
    d.mkdir(exist_ok=True)
    (d / "scene.json").write_text(txt)
    return str(d)


def test_loader_quirks(tmp_path):
    src = _rel_src(tmp_path)
    d = _write_scene(tmp_path)
    s = loadScene(d)
    assert (s.width, s.height) == (64, 48)
    s2 = loadScene(d, width=32, height=32)
    assert (s2.width, s2.height) == (32, 32)
    # flipX negates P[0][0] -> inverse projection x column flips sign
    d2 = _write_scene(tmp_path, ', "flipX": "1"')
    a, b = loadScene(d).camera["inv_proj"], loadScene(d2).camera["inv_proj"]
    assert a[0, 0] == -b[0, 0]
    # unknown bsdf: instance skipped ("Error in loading"), the rest loads
    bad = ('{"filename": "%s/Rectangle.gem", "world": [1,0,0,0, 0,1,0,0, 0,0,1,0, 0,0,0,1], "bsdf": "roughconductor", '
           '"reflectance": "%s/1_1_1.png"}' % (src, src))
    good = ('{"filename": "%s/Rectangle.gem", "world": [1,0,0,0, 0,1,0,0, 0,0,1,0, 0,0,0,1], "bsdf": "diffuse", '
            '"reflectance": "%s/1_1_1.png", "emission": "2 2 2"}' % (src, src))
    d3 = _write_scene(tmp_path, instances=[bad, good])
    s3 = loadScene(d3)
    assert s3.desc.n_materials == 1 and s3.desc.n_tris == 2
    # missing .gem: an error (the reference calls exit(0)); skip_missing drops it instead
    miss = good.replace("Rectangle.gem", "Nope.gem")
    d4 = _write_scene(tmp_path, instances=[good, miss])
    with pytest.raises(Exception):
        loadScene(d4)
    s4 = loadScene(d4, skip_missing=True)
    assert s4.info.dropped_instances == 1 and s4.desc.n_tris == 2
    # missing texture (no skip): Texture::loadDefault -> 1x1 white
    d5 = _write_scene(tmp_path, instances=[good.replace("1_1_1.png", "nothere.png")])
    s5 = loadScene(d5)
    assert s5.texture(0).shape == (1, 1, 3) and np.all(s5.texture(0) == 1.0)


def test_tonemap_matches_film_tonemap():
    """rth_tonemap against Film::tonemap (Imaging.h:233-242) of the reference's own Film class
    (tests/golden/tonemap_kat.npz from oracle/_ref: negative, zero, saturating and non-finite
    values, two exposures)."""
    from raytracingrenderer_amd import tonemap
    g = np.load(os.path.join(GOLD, "tonemap_kat.npz"))
    for k in (0, 1):
        got = tonemap(g["film"], int(g["spp"]), float(g["exposure%d" % k]))
        assert np.array_equal(got, g["rgb%d" % k]), np.argwhere(got != g["rgb%d" % k])[:5]


def test_synthetic_1m_matches_reference_loader(tmp_path):
    """Config C3's scene: 1M triangles through the host loader + threaded BVH build equal the
    reference loader's Scene::build (Geometry.h:325-398) bit for bit (std::sort permutation, nodes,
    lights, camera)."""
    write_synthetic_scene(str(tmp_path), n_tris=1_000_000, seed=20251015, width=1024, height=1024)
    _check_digests("synth1m", loadScene(str(tmp_path)))


def _desc_arrays(d):
    """numpy copies of an rtg_scene_desc's arrays (ctypes struct)."""
    import ctypes as C

    def arr(p, n, dt):
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float if dt == np.float32 else C.c_int32)),
                                     shape=(n,)).view(dt).copy() if n else np.zeros(0, dt)
    out = {"positions": arr(d.positions, d.n_tris * 9, np.float32), "normals": arr(d.normals, d.n_tris * 9, np.float32),
           "uvs": arr(d.uvs, d.n_tris * 6, np.float32), "material": arr(d.material, d.n_tris, np.int32),
           "node_bounds": arr(d.node_bounds, d.n_nodes * 6, np.float32),
           "node_links": arr(d.node_links, d.n_nodes * 4, np.int32).reshape(-1, 4),
           "lights": arr(d.lights, d.n_lights, np.int32),
           "camera": np.concatenate([np.array(d.camera.inv_proj[:], np.float32), np.array(d.camera.camera[:], np.float32),
                                     np.array(d.camera.origin[:], np.float32), np.float32([d.camera.width, d.camera.height])]),
           "projection": np.concatenate([np.array(d.projection.proj[:], np.float32),
                                         np.array(d.projection.camera_to_view[:], np.float32),
                                         np.array(d.projection.view_direction[:], np.float32), np.float32([d.projection.a_film])]),
           "materials": [(m.kind, m.two_sided, m.int_ior, m.ext_ior, tuple(m.emission)) for m in d.materials[:d.n_materials]],
           "env_texture": d.env_texture}
    tex = []
    for i in range(d.n_textures):
        t = d.textures[i]
        tex.append(arr(t.texels, t.width * t.height * 3, np.float32).reshape(t.height, t.width, 3))
    out["textures"] = tex
    out["mat_tex"] = [m.texture for m in d.materials[:d.n_materials]]
    return out


@pytest.mark.parametrize("case", ["cornell-mat", "cornell-box"])
def test_reference_side_binding_flattens_like_the_host(case):
    """integration/rtg_rtbase.h (compiled against the reference headers into
    oracle/_ref) flattens the reference loader's own Scene into the rtg_scene_desc that librth builds
    from the same scene.json: the same bits in every array (BVH links compared on the child / leaf
    fields the ABI reads)."""
    from oracle import pyref
    from raytracingrenderer_amd import _native as N
    if not pyref.available():
        pytest.skip("oracle/_ref needs /root/reference (build container)")
    import ctypes as C
    path = os.path.join(SCENES, case)
    r = pyref.RefScene(path, 64, 48, False)
    ref = _desc_arrays(C.cast(r.rtg_desc(), C.POINTER(N.rtg_scene_desc)).contents)
    s = loadScene(path, width=64, height=48)
    host = _desc_arrays(s.desc)
    for k in ("positions", "normals", "uvs", "material", "node_bounds", "lights", "camera", "projection"):
        assert np.array_equal(ref[k].view(np.uint32), host[k].view(np.uint32)), k
    assert np.array_equal(ref["node_links"][:, :2], host["node_links"][:, :2])
    leaf = ref["node_links"][:, 0] < 0
    assert np.array_equal(ref["node_links"][leaf, 2:], host["node_links"][leaf, 2:])
    assert ref["materials"] == host["materials"]
    assert (ref["env_texture"] >= 0) == (host["env_texture"] >= 0)
    for a, b in zip(ref["mat_tex"], host["mat_tex"]):
        assert np.array_equal(ref["textures"][a].view(np.uint32), host["textures"][b].view(np.uint32))
