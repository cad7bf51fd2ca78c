"""GPU parity: the HIP wavefront renderer (librtg.so, called through the C-ABI) against the C oracle
with the same transcendentals (bit-exact), the reference's own traversal / BSDF code (golden
fixtures from oracle/_ref), and size-independent properties at full BASELINE sizes."""
import ctypes as C
import hashlib
import json
import os
import zlib

import numpy as np
import pytest

from conftest import GOLD, SCENES, require_reference_libm, scene_path
from oracle.pyoracle import Oracle
from raytracingrenderer_amd import RayTracer, loadScene, write_synthetic_scene
from raytracingrenderer_amd import _native as N

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def assert_bitexact(got, want, what=""):
    if not np.array_equal(bits(got), bits(want)):
        diff = np.argwhere(bits(got) != bits(want))
        raise AssertionError("%s: %d values differ, first at %s: %r vs %r"
                             % (what, len(diff), diff[0].tolist(), got[tuple(diff[0])], want[tuple(diff[0])]))


def gpu_film(scene, spp, seed=1234, max_depth=4, cull=True, max_paths=0, tiles=None, wide=True):
    rt = RayTracer(scene, seed=seed, max_depth=max_depth, cull=cull, max_paths=max_paths, wide=wide)
    rt.render(spp, tiles=tiles, first_sample=0)
    film, n = rt.film()
    assert n == spp
    return film


@pytest.fixture(scope="module")
def cornell256():
    return loadScene(os.path.join(SCENES, "cornell-box"), width=256, height=256)


@pytest.fixture(scope="module")
def synth20k(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("synth20k"))
    write_synthetic_scene(d, n_tris=20000, seed=3, width=128, height=96)
    return loadScene(d)


def test_c1_bit_exact_and_known_answer(cornell256):
    film = gpu_film(cornell256, 4)
    ref, _ = Oracle(cornell256, 4, "rtm").render(4, seed=1234, threads=8)
    assert_bitexact(film, ref, "C1 film")
    kat = json.load(open(os.path.join(GOLD, "film_kat.json")))["C1_rtm"]["md5"]
    assert hashlib.md5((film / np.float32(4)).astype(np.float32).tobytes()).hexdigest() == kat


def test_ray_counts_are_the_references_and_camera_rays_are_traced_per_pixel(cornell256):
    """rtg_stats counts the reference's rays (C1: 702,961 closest-hit + 429,793 shadow rays for
    262,144 paths, SURVEY.md §8d, the reference integrator's own counts), one camera ray per sample;
    the traversal traces a camera ray per pixel per chunk (the pixel centre's, shared by the pixel's
    samples: Renderer.h:805-808), so 4 spp in one chunk trace 65,536 and 4 chunks of 1 spp 262,144."""
    for max_paths, traced in ((0, 256 * 256), (256 * 256, 4 * 256 * 256)):
        rt = RayTracer(cornell256, seed=1234, max_paths=max_paths)
        rt.render(4, first_sample=0)
        s = rt.stats()
        assert (s["paths"], s["extension_rays"], s["shadow_rays"]) == (262144, 702961, 429793), s
        assert s["traced_camera_rays"] == traced


def test_cull_is_exact(cornell256, synth20k):
    for s, spp in ((cornell256, 2), (synth20k, 2)):
        assert_bitexact(gpu_film(s, spp, cull=True), gpu_film(s, spp, cull=False), "cull vs no-cull")


def test_wide_walk_is_exact(cornell256, synth20k):
    """The 4-wide walk (collapsed BVH) returns the reference BVH2 walk's results bit for bit."""
    for s, spp in ((cornell256, 2), (synth20k, 2)):
        assert_bitexact(gpu_film(s, spp, wide=True), gpu_film(s, spp, wide=False), "bvh4 vs bvh2 film")
    rng = np.random.default_rng(11)
    n = 200000
    r = np.zeros((n, 8), np.float32)
    r[:, :3] = rng.uniform(-1.3, 1.3, (n, 3))
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[: n // 10, rng.integers(0, 3)] = 0.0  # some rays stay on the BVH2 walk (inf 1/d)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r[:, 4:7] = d
    r[:, 3] = rng.uniform(0.01, 3, n)
    for cull in (True, False):
        a = RayTracer(synth20k, cull=cull, wide=True)
        b = RayTracer(synth20k, cull=cull, wide=False)
        assert_bitexact(a.trace_closest(r), b.trace_closest(r), "bvh4 vs bvh2 closest")
        assert np.array_equal(a.trace_visible(r), b.trace_visible(r))


def test_wide_walk_over_own_tree_equals_bvh2_walk(synth20k, cornell256):
    """Wide nodes cut from the own 3-axis SAH tree over the triangles (one triangle per leaf slot,
    inflated boxes; round 5) return the reference BVH2 walk's bits: films and 100k random closest-hit
    / any-hit queries per scene."""
    rng = np.random.default_rng(31)
    for s in (synth20k, cornell256):
        assert_bitexact(gpu_film(s, 2, wide=True), gpu_film(s, 2, wide=False), "bvh4 vs bvh2 film")
        lo, hi = s.node_bounds[0, 0:3], s.node_bounds[0, 3:6]
        n = 100000
        r = np.zeros((n, 8), np.float32)
        r[:, :3] = rng.uniform(lo - 0.1 * (hi - lo), hi + 0.1 * (hi - lo), (n, 3))
        d = rng.normal(size=(n, 3)).astype(np.float32)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        r[:, 4:7] = d
        r[:, 3] = np.float32(np.abs(hi - lo).max() * 2)
        a = RayTracer(s, wide=True)
        b = RayTracer(s, wide=False)
        assert_bitexact(a.trace_closest(r), b.trace_closest(r), "bvh4 vs bvh2 closest")
        assert np.array_equal(a.trace_visible(r), b.trace_visible(r))


def test_wide_walk_adversarial_rays(synth20k, cornell256):
    """Rays that start on reference box faces/corners and run (nearly) along box planes: the
    compressed walk's conservative slot test must never lose a reachable leaf."""
    rng = np.random.default_rng(21)
    for s in (synth20k, cornell256):
        nb = s.node_bounds
        n = 60000
        pick = rng.integers(0, len(nb), n)
        corner = rng.integers(0, 2, (n, 3))
        o = np.where(corner == 0, nb[pick, 0:3], nb[pick, 3:6]).astype(np.float32)
        axis = np.eye(3, dtype=np.float32)[rng.integers(0, 3, n)] * rng.choice([-1, 1], (n, 1)).astype(np.float32)
        eps = np.float32(10.0) ** rng.uniform(-7, -1, (n, 1)).astype(np.float32)
        d = axis + eps * rng.normal(size=(n, 3)).astype(np.float32)
        d[: n // 6] = rng.normal(size=(n // 6, 3))  # plus generic directions from box corners
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        r = np.zeros((n, 8), np.float32)
        r[:, :3] = o
        r[:, 4:7] = d
        r[:, 3] = rng.uniform(0.01, 4, n)
        for cull in (True, False):
            a = RayTracer(s, cull=cull, wide=True)
            b = RayTracer(s, cull=cull, wide=False)
            assert_bitexact(a.trace_closest(r), b.trace_closest(r), "adversarial closest")
            assert np.array_equal(a.trace_visible(r), b.trace_visible(r))


def test_wide_walk_triangle_grazing_rays(synth20k, cornell256):
    """Rays aimed exactly at triangle vertices and edge points (and a hair inside / outside them),
    from near and far origins, along generic and nearly axis-parallel directions: rayIntersect's
    accept / reject decisions at the triangle boundary must be reached by the compressed walk
    whatever boxes its slots hold (reference leaves, or single triangles with inflated boxes)."""
    rng = np.random.default_rng(33)
    for s in (synth20k, cornell256):
        P = s.positions.reshape(-1, 3, 3).astype(np.float64)
        n = 60000
        t = rng.integers(0, len(P), n)
        i, j = rng.integers(0, 3, n), rng.integers(0, 3, n)
        w = rng.choice([0.0, 0.5, 1.0], n) * (rng.random(n) < 0.5) + rng.random(n) * (rng.random(n) >= 0.5)
        tgt = P[t, i] + w[:, None] * (P[t, j] - P[t, i])  # a vertex or a point of an edge
        cen = P[t].mean(axis=1)
        tgt = tgt + (tgt - cen) * rng.choice([0.0, 1e-7, -1e-7, 1e-6], n)[:, None]  # on / just off the edge
        ext = float(np.abs(s.node_bounds[0]).max())
        dist = ext * 10.0 ** rng.uniform(-3, 1, n)
        d = rng.normal(size=(n, 3))
        ax = rng.random(n) < 0.3
        d[ax] = np.eye(3)[rng.integers(0, 3, ax.sum())] + 1e-4 * rng.normal(size=(ax.sum(), 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        o = tgt - d * dist[:, None]
        r = np.zeros((n, 8), np.float32)
        r[:, :3] = o
        r[:, 4:7] = d
        r[:, 3] = (dist * 1.5).astype(np.float32)
        for cull in (True, False):
            a = RayTracer(s, cull=cull, wide=True)
            b = RayTracer(s, cull=cull, wide=False)
            assert_bitexact(a.trace_closest(r), b.trace_closest(r), "grazing closest")
            assert np.array_equal(a.trace_visible(r), b.trace_visible(r))


@pytest.mark.parametrize("max_depth", [0, 1, 8, 16])
def test_depths_cornell_materials(max_depth):
    """glass / mirror / Lambert stubs (one- and two-sided) / env + area lights (configs C2, C4 depth)."""
    s = loadScene(os.path.join(SCENES, "cornell-mat"), width=80, height=60)
    film = gpu_film(s, 6, seed=99, max_depth=max_depth)
    ref, _ = Oracle(s, max_depth, "rtm").render(6, seed=99, threads=8)
    assert_bitexact(film, ref, "cornell-mat depth %d" % max_depth)


def test_c2_shape_cornell_depth8():
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=160, height=160)
    assert_bitexact(gpu_film(s, 8, max_depth=8), Oracle(s, 8, "rtm").render(8, seed=1234, threads=8)[0], "C2 crop")


def test_synthetic_env_lit(synth20k):
    assert_bitexact(gpu_film(synth20k, 4, seed=42), Oracle(synth20k, 4, "rtm").render(4, seed=42, threads=8)[0], "synth20k")


def test_tiles_and_chunks_compose(cornell256):
    """Disjoint tile subsets sum to the full film; wavefront chunking (paths in flight) is invisible."""
    full = gpu_film(cornell256, 5)
    rt = RayTracer(cornell256, seed=1234, max_paths=20000)  # forces many chunks
    tiles = np.arange(64, dtype=np.uint32)
    for part in (tiles[::2], tiles[1::2]):
        rt.render(5, tiles=part, first_sample=0)
    assert_bitexact(rt.film()[0], full, "tiles+chunks")
    # progressive: 2 + 3 frames == 5 frames (RayTracer::render called repeatedly)
    rt2 = RayTracer(cornell256, seed=1234)
    rt2.render(2)
    rt2.render(3)
    f2, spp = rt2.film()
    assert spp == 5
    assert_bitexact(f2, full, "progressive")
    # resume from a saved float film
    rt3 = RayTracer(cornell256, seed=1234)
    rt3.render(2)
    saved, n = rt3.film()
    rt4 = RayTracer(cornell256, seed=1234)
    rt4.load_film(saved, n)
    rt4.render(3)
    assert_bitexact(rt4.film()[0], full, "resume")


@pytest.mark.parametrize("serial", [False, True])
@pytest.mark.parametrize("w,h,spp,max_paths", [(1, 1, 1, 0), (17, 15, 1, 0), (16, 16, 1, 0), (33, 31, 3, 0),
                                               (64, 35, 2, 0), (33, 31, 3, 300)])
def test_queue_segment_edges(w, h, spp, max_paths, serial):
    """Segmented queues (8 segments of ceil(ceil(P / 256) / 8) tiles each): P = 1 (seven empty
    segments), 255, 256, 3069 and 4480 paths, and chunks of at most 300 paths, at depth 8 so later
    bounces empty whole segments: bit-exact vs the oracle. Both k_shade grid sizings: every tile a
    segment can hold, chunks rotating through the frame pipeline's slots (default for chunks of <= 8M
    paths), and the live tiles from the read-back counts, one chunk at a time (RTG_OPT_SERIAL, the
    sizing of big chunks)."""
    s = loadScene(os.path.join(SCENES, "cornell-mat"), width=w, height=h)
    rt = RayTracer(s, seed=7, max_depth=8, max_paths=max_paths)
    if serial:
        rt.set_options(flags=rt.flags | N.RTG_OPT_SERIAL)
    rt.render(spp, first_sample=0)
    film = rt.film()[0]
    ref, _ = Oracle(s, 8, "rtm").render(spp, seed=7, threads=8)
    assert_bitexact(film, ref, "%dx%d x%d spp, max_paths %d" % (w, h, spp, max_paths))


@pytest.mark.parametrize("coalesce", [True, False])
def test_queued_frames_return_early_and_equal_one_render(tmp_path, coalesce):
    """The drop-in frame loop (Main.cpp:74-118: one RayTracer::render() per frame): 1-spp
    rtg_render_async calls are queued and return before their work has run; consecutive ones are
    coalesced into one chunk (or, with RTG_OPT_NO_COALESCE, each issued at once, up to three chunks
    running side by side), and the film, folded in sample order, is bit-identical to one rtg_render
    of all the samples. Film::SPP is readable at once; a film read waits for the frames."""
    d = str(tmp_path / "s")
    write_synthetic_scene(d, n_tris=200000, seed=5, width=1024, height=1024)
    s = loadScene(d)
    full = gpu_film(s, 12, seed=99)
    rt = RayTracer(s, seed=99)
    if not coalesce:
        rt.set_options(flags=rt.flags | N.RTG_OPT_NO_COALESCE)
    rt.render(1, sync=False)  # warm: buffers of the first slots
    rt.clear()
    rt.synchronize()
    assert rt.idle()
    for f in range(12):
        rt.render(1, first_sample=f, sync=False)
        if f == 0:
            # a 1M-path frame of a 200k-triangle scene runs for milliseconds; the call returned at
            # once (rtg_render_idle issues a coalesced frame before it looks)
            assert not rt.idle(), "rtg_render_async waited for its frame"
    assert rt.getSPP() == 12
    film, spp = rt.film()
    assert spp == 12 and rt.idle()
    assert_bitexact(film, full, "12 queued 1-spp frames vs one 12-spp render")
    # queued frames, a synchronous render and tile subsets interleaved; a clear in between
    rt.clear()
    tiles = np.arange(rt.tiles_x * rt.tiles_y, dtype=np.uint32)
    for f in range(0, 12, 3):
        rt.render(1, first_sample=f, sync=False)
        rt.render(1, first_sample=f + 1, tiles=tiles[::2], sync=False)
        rt.render(1, first_sample=f + 1, tiles=tiles[1::2], sync=False)
        rt.render(1, first_sample=f + 2, sync=True)
    assert_bitexact(rt.film()[0], full, "interleaved queued / tiled / synchronous frames")
    st = rt.stats()
    assert st["paths"] == 12 * 1024 * 1024


def test_queued_frames_past_the_coalescing_threshold(cornell256):
    """Queued 1-spp frames of a 256x256 film reach the coalescing threshold (64M paths = 1024
    frames) inside the loop: the call that reaches it issues one chunk larger than the pipeline's
    (slot 0, read-back grid), the frames after it queue again, and the film is bit-identical to one
    rtg_render of all the samples."""
    n = 1100
    full = gpu_film(cornell256, n, seed=7)
    rt = RayTracer(cornell256, seed=7)
    for f in range(n):
        rt.render(1, first_sample=f, sync=False)
    assert rt.getSPP() == n
    film, spp = rt.film()
    assert spp == n
    assert_bitexact(film, full, "%d queued 1-spp frames vs one %d-spp render" % (n, n))
    assert rt.stats()["paths"] == n * 256 * 256


def test_queued_frames_then_user_stream_renders_then_reads(tmp_path):
    """Queued frames (rtg_render_async, no stream), then renders on a user HIP stream (rtg_render_async
    with a stream: no host wait, not the handle's stream), then reads: the film read and the stats
    wait for the queued chunks and the stream's renders alike, and the film equals one waited-for
    render of all the samples. A clear after such a mix leaves nothing to fold later."""
    import torch
    d = str(tmp_path / "s")
    write_synthetic_scene(d, n_tris=200000, seed=5, width=512, height=512)
    s = loadScene(d)
    full = gpu_film(s, 8, seed=41)
    rt = RayTracer(s, seed=41)
    us = torch.cuda.Stream()
    for f in range(4):
        rt.render(1, first_sample=f, sync=False)
    for f in range(4, 8):
        rt.render(1, first_sample=f, stream=us.cuda_stream)
    film, spp = rt.film()
    assert spp == 8
    assert_bitexact(film, full, "4 queued frames + 4 frames on a user stream vs one 8-spp render")
    assert rt.stats()["paths"] == 8 * 512 * 512
    for f in range(3):
        rt.render(1, first_sample=f, sync=False)
    rt.render(1, first_sample=3, stream=us.cuda_stream)
    rt.clear()
    torch.cuda.synchronize()
    film2, spp2 = rt.film()
    assert spp2 == 0 and not film2.any()


@pytest.mark.parametrize("name", ["cornell256", "synth20k"])
@pytest.mark.parametrize("cull", [True, False])
def test_ray_queries_match_reference(name, cull, cornell256, synth20k):
    g = np.load(os.path.join(GOLD, "%s_rays.npz" % name))
    s = cornell256 if name == "cornell256" else synth20k
    rt = RayTracer(s, cull=cull)
    assert_bitexact(rt.trace_closest(g["rays"]), g["hits"], "closest hits vs Scene::traverse")
    assert np.array_equal(rt.trace_visible(g["rays"]), g["visible"])


def test_random_rays_cull_equivalence(synth20k):
    """Size-independent property: distance culling never changes a closest hit (incl. grazing and
    axis-parallel rays)."""
    rng = np.random.default_rng(5)
    n = 200000
    r = np.zeros((n, 8), np.float32)
    r[:, :3] = rng.uniform(-1.3, 1.3, (n, 3))
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[: n // 10, rng.integers(0, 3)] = 0.0
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r[:, 4:7] = d
    r[:, 3] = rng.uniform(0.01, 3, n)
    a = RayTracer(synth20k, cull=True)
    b = RayTracer(synth20k, cull=False)
    assert_bitexact(a.trace_closest(r), b.trace_closest(r), "cull on/off")
    assert np.array_equal(a.trace_visible(r), b.trace_visible(r))
    o = Oracle(synth20k, 4, "rtm")
    assert_bitexact(a.trace_closest(r[:20000]), o.trace_closest(r[:20000]), "vs oracle DFS")


def test_bsdf_probe_matches_reference_bsdfs():
    kat = json.load(open(os.path.join(GOLD, "bsdf_kat.json")))
    kind_map = {0: 0, 1: 1, 2: 2, 3: 3, 4: 1, 5: 1, 6: 1}  # reference class -> rtg kind
    cases = np.zeros((len(kat), 20), np.float32)
    for i, k in enumerate(kat):
        cases[i, 0] = kind_map[k["kind"]]
        cases[i, 1:3] = [k["int_ior"], k["ext_ior"]]
        cases[i, 3:6] = k["albedo"]
        cases[i, 6:14] = k["sd"]  # sNormal, wo, tu, tv
        cases[i, 14:18] = k["draws"]
    out = np.zeros((len(kat), 11), np.float32)
    import ctypes as C
    assert N.rtg().rtg_probe_bsdf(N.ptr(cases, C.c_float), len(kat), N.ptr(out, C.c_float)) == 0
    # reference BSDF classes compiled with the shared transcendentals interposed (libref_rtm.so)
    want = np.array([k["out_bits_rtm"] for k in kat], np.uint32)
    got = out.view(np.uint32)
    glass = cases[:, 0] == 3
    # glass evaluate() returns 0 in both; every other field is compared bit for bit
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    assert glass.any() and (cases[:, 0] == 0).any()


def test_c3_full_size_64spp_sampled_pixels():
    """The bench workload itself (C3: 1M triangles, 1024^2, 64 spp in one wavefront chunk with the
    pixel-major two-pass fold): 1500 random pixels' film values equal the oracle's 64 per-path
    radiances summed in sample order (Film::splat), bit for bit."""
    import tempfile
    d = tempfile.mkdtemp(prefix="rtg_c3_")
    write_synthetic_scene(d, n_tris=1_000_000, seed=20251015)
    s = loadScene(d)
    film = gpu_film(s, 64)
    rng = np.random.default_rng(64)
    pix = rng.choice(s.width * s.height, 1500, replace=False).astype(np.uint32)
    o = Oracle(s, 4, "rtm")
    want = np.zeros((len(pix), 3), np.float32)
    for smp in range(64):  # film += L, sample by sample, in float32
        want = want + o.trace_paths(pix, np.full(len(pix), smp, np.uint32), seed=1234)
    assert_bitexact(film.reshape(-1, 3)[pix], want, "C3 64 spp sampled pixels")


def test_c3_full_size_one_frame():
    """BASELINE C3 scene at full size (1M triangles, 1024^2): one frame bit-exact vs the oracle."""
    import tempfile
    d = tempfile.mkdtemp(prefix="rtg_c3_")
    write_synthetic_scene(d, n_tris=1_000_000, seed=20251015)
    s = loadScene(d)
    film = gpu_film(s, 1)
    ref, _ = Oracle(s, 4, "rtm").render(1, seed=1234, threads=16)
    assert_bitexact(film, ref, "C3 1 spp")


def staged(name):
    """Reference scene data staged into assets/ by build.stage_assets(): a missing scene is a
    failure under -m gpu, not a skip (the C4/C5 parity cases must run on the box)."""
    p = scene_path(name)
    if p is None:
        pytest.fail("%s assets missing: run raytracingrenderer_amd.build.stage_assets() where "
                    "/root/reference exists (assets/ ships to the GPU box with the tree)" % name)
    return p


def test_coffee_filtered_crop():
    s = loadScene(staged("coffee"), width=80, height=100, skip_missing=True)
    assert_bitexact(gpu_film(s, 2), Oracle(s, 4, "rtm").render(2, seed=1234, threads=8)[0], "coffee_f")


@pytest.mark.parametrize("size", [(128, 128), (160, 96)])
def test_c5_coffee_gi_env_crop(size):
    """Config C5's scene: coffee_f with "envmap": "GI.hdr" (Main.cpp:25). GI.hdr
    is all zero, so it is lights[0] only if its power is > 0 (it is not): every miss evaluates the
    1024^2 environment texture (EnvironmentMap::evaluate, Lights.h:150-157) and returns 0."""
    w, h = size
    s = loadScene(staged("coffee"), width=w, height=h, skip_missing=True, envmap="GI.hdr")
    assert s.desc.env_texture >= 0
    film = gpu_film(s, 3, seed=4321)
    assert_bitexact(film, Oracle(s, 4, "rtm").render(3, seed=4321, threads=8)[0], "coffee_f + GI.hdr")
    # the environment is dark: the scene's area lights alone give the same film as without it
    assert_bitexact(film, gpu_film(loadScene(staged("coffee"), width=w, height=h, skip_missing=True), 3, seed=4321),
                    "GI.hdr contributes nothing")


def test_bathroom_filtered_crop_depth16():
    """Config C4's scene and depth (bathroom_f: JPEG/PNG textures, glass, mirror, Lambert stubs)."""
    p = staged("bathroom")
    s = loadScene(p, width=96, height=54, skip_missing=True)
    assert_bitexact(gpu_film(s, 2, max_depth=16), Oracle(s, 16, "rtm").render(2, seed=1234, threads=8)[0],
                    "bathroom_f depth 16")


@pytest.mark.parametrize("integrator", ["direct", "albedo", "normals", "direct_mis"])
def test_alternative_integrators(integrator):
    """RayTracer::direct / albedo / viewNormals (Renderer.h:393-407, 558-582) and direct() with
    computeDirectMIS (:474-557) on the mixed-material scene (area + env lights, glass, mirror,
    two-sided Lambert stubs)."""
    s = loadScene(os.path.join(SCENES, "cornell-mat"), width=80, height=60)
    rt = RayTracer(s, seed=7, integrator=integrator)
    rt.render(3, first_sample=0)
    mode = RayTracer.INTEGRATORS[integrator]
    ref, _ = Oracle(s, 4, "rtm", integrator=mode).render(3, seed=7, threads=8)
    assert_bitexact(rt.film()[0], ref, integrator)


def test_scene_without_lights_is_rejected(tmp_path):
    src = os.path.relpath(os.path.join(SCENES, "cornell-box"), str(tmp_path))
    (tmp_path / "scene.json").write_text(
        '{"width": "16", "height": "16", "from": "0 0 3", "to": "0 0 0", "up": "0 1 0", "instances": [{"filename": '
        '"%s/Rectangle.gem", "world": [1,0,0,0, 0,1,0,0, 0,0,1,0, 0,0,0,1], "bsdf": "diffuse", '
        '"reflectance": "%s/1_1_1.png"}]}' % (src, src))
    from raytracingrenderer_amd import NativeError
    with pytest.raises(NativeError):
        RayTracer(loadScene(str(tmp_path)))


def test_cli_matches_library(tmp_path):
    """rtg_render CLI (Main.cpp's frame loop): result_<spp>.hdr equals Film::save of the library film."""
    import subprocess
    from raytracingrenderer_amd import read_hdr, save_hdr
    cli = os.path.join(os.path.dirname(N.__file__), "lib", "rtg_render")
    scene = os.path.join(SCENES, "cornell-box")
    r = subprocess.run([cli, "-scene", scene, "-SPP", "3", "-width", "64", "-height", "64", "-timeLimit", "0",
                        "-batch", "2", "-outputFilename", "out.png"], cwd=str(tmp_path), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    s = loadScene(scene, width=64, height=64)
    film = gpu_film(s, 3)
    save_hdr(str(tmp_path / "lib.hdr"), film, 3)
    assert (tmp_path / "result_3.hdr").read_bytes() == (tmp_path / "lib.hdr").read_bytes()
    assert (tmp_path / "out.png").exists()
    assert read_hdr(str(tmp_path / "result_3.hdr")).shape == (64, 64, 3)


@pytest.mark.parametrize("base,n_tris", [(2.0, 60), (4.0, 60), (2.0, 28)])
def test_deep_bvh_stack_overflow(tmp_path, base, n_tris):
    """Triangles at x = base^k make a chain-like BVH (depth 17 / 26 with 60 triangles): rays along +x
    keep one sibling per level pending, past the 16-entry LDS stack, into the global overflow. base 2
    keeps the scene scale under 2^60 (compressed wide walk); base 4 exceeds it (exact BVH2 walk). 28
    triangles are a small scene by construction (at most 27 wide nodes: 4 * 27 + 3 * 28 <= 192 float4s),
    walked from LDS with a 7-entry stack."""
    from raytracingrenderer_amd.renderer import write_mesh_scene
    P = np.array([[(base ** k, -1.0, -1.0), (base ** k, 1.0, -1.0), (base ** k, 0.0, 1.0)] for k in range(n_tris)],
                 np.float32)
    s = loadScene(write_mesh_scene(str(tmp_path), P, 32, 32))
    assert s.info.bvh_depth >= (17 if n_tris == 60 else 9)
    rng = np.random.default_rng(3)
    n = 4096
    r = np.zeros((n, 8), np.float32)
    r[:, 0] = -0.5
    r[:, 1:3] = rng.uniform(-0.4, 0.4, (n, 2))
    eps = np.float32(10.0) ** rng.uniform(-19, -8, (n, 1)).astype(np.float32)
    d = np.concatenate([np.ones((n, 1), np.float32), eps * rng.choice([-1, 1], (n, 2)).astype(np.float32)], axis=1)
    d[: n // 8, 1:] = 0.0  # exactly axis-parallel: BVH2 walk
    r[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    r[:, 3] = np.float32(1e30)
    o = Oracle(s, 4, "rtm")
    for cull in (True, False):
        rt = RayTracer(s, cull=cull)
        assert_bitexact(rt.trace_closest(r), o.trace_closest(r), "deep BVH closest")
        assert np.array_equal(rt.trace_visible(r), o.trace_visible(r))


@pytest.mark.parametrize("n_copies", [40, 1500])
def test_coincident_triangles_tree_rebuild(tmp_path, n_copies):
    """Many copies of one triangle plus random ones: the own SAH tree over the reference leaves
    (RTG_REBUILD) sees zero centroid extent and equal SAH costs; with 1500 copies the equal-cost
    splits can chain past the rebuild's depth guard, which falls back to the reference cut.
    Closest hits (ties broken by the lowest index) and visibility equal the oracle either way."""
    from raytracingrenderer_amd.renderer import write_mesh_scene
    rng = np.random.default_rng(5)
    tri = np.array([(-0.5, -0.5, 0.0), (0.5, -0.5, 0.0), (0.0, 0.5, 0.0)], np.float32)
    rnd = rng.uniform(-1, 1, (500, 1, 3)) + rng.uniform(-0.1, 0.1, (500, 3, 3))
    P = np.concatenate([np.repeat(tri[None], n_copies, 0), rnd.astype(np.float32)], 0)
    s = loadScene(write_mesh_scene(str(tmp_path), P, 32, 32))
    n = 20000
    r = np.zeros((n, 8), np.float32)
    r[:, :3] = rng.uniform(-1.2, 1.2, (n, 3))
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[: n // 2] = -r[: n // 2, :3] + rng.uniform(-0.3, 0.3, (n // 2, 3)).astype(np.float32)  # aim at the copies
    r[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    r[:, 3] = np.float32(10.0)
    o = Oracle(s, 4, "rtm")
    rt = RayTracer(s)
    assert_bitexact(rt.trace_closest(r), o.trace_closest(r), "coincident closest")
    assert np.array_equal(rt.trace_visible(r), o.trace_visible(r))


def _random_mesh(kind, rng):
    """Geometry families that stress the compressed walk's conservative boxes, the exact leaf gate
    and the BVH2 fallback: (n, 3, 3) float32 triangle positions around the origin."""
    if kind == "small":  # the C3 recipe at a smaller count
        c = rng.uniform(-1, 1, (3000, 1, 3))
        return (c + rng.uniform(-0.03, 0.03, (3000, 3, 3))).astype(np.float32)
    if kind == "large":  # big, heavily overlapping triangles
        return rng.uniform(-1.2, 1.2, (300, 3, 3)).astype(np.float32)
    if kind == "slivers":  # long needles, 1e-3 wide: near-degenerate edges, large 1/area
        a = rng.uniform(-1, 1, (6000, 1, 3))
        c = a + rng.uniform(-0.6, 0.6, (6000, 1, 3))
        b = c + rng.uniform(-1e-3, 1e-3, (6000, 1, 3))
        return np.concatenate([a, b, c], 1).astype(np.float32)
    if kind == "axis_planes":  # triangles lying in x / y / z = const planes (flat boxes, dead slabs)
        P = rng.uniform(-1, 1, (1500, 3, 3))
        ax = rng.integers(0, 3, 1500)
        P[np.arange(1500), :, ax] = np.round(rng.uniform(-1, 1, 1500), 1)[:, None]
        return P.astype(np.float32)
    if kind == "grid":  # a heightfield: triangles sharing edges and vertices
        n = 48
        x, y = np.meshgrid(np.linspace(-1, 1, n), np.linspace(-1, 1, n))
        z = 0.2 * np.sin(3 * x) * np.cos(2 * y)
        V = np.stack([x, y, z], -1)
        a, b, c, d = V[:-1, :-1], V[1:, :-1], V[:-1, 1:], V[1:, 1:]
        T = np.concatenate([np.stack([a, b, d], -2).reshape(-1, 3, 3), np.stack([a, d, c], -2).reshape(-1, 3, 3)])
        return T.astype(np.float32)
    if kind == "huge_scale":  # coordinates of 1e4: the camera sits inside the geometry
        c = rng.uniform(-1, 1, (1000, 1, 3)) * 1e4
        return (c + rng.uniform(-300, 300, (1000, 3, 3))).astype(np.float32)
    if kind == "tiny_tris":  # 50k triangles a few 1e-3 across: leaves far below a pixel
        c = rng.uniform(-0.7, 0.7, (50000, 1, 3))
        return (c + rng.uniform(-3e-3, 3e-3, (50000, 3, 3))).astype(np.float32)
    if kind == "duplicates":  # every triangle twice (equal hit distances: ties by index)
        c = rng.uniform(-1, 1, (600, 1, 3))
        T = (c + rng.uniform(-0.1, 0.1, (600, 3, 3))).astype(np.float32)
        return np.concatenate([T, T[::-1]], 0)
    raise ValueError(kind)


@pytest.mark.parametrize("kind,depth", [("small", 4), ("large", 8), ("slivers", 4), ("axis_planes", 6),
                                        ("grid", 8), ("huge_scale", 4), ("tiny_tris", 4), ("duplicates", 5)])
def test_adversarial_meshes_render_like_the_oracle(tmp_path, kind, depth):
    """Whole renders (environment-lit C3 recipe, 64x64, 3 spp) of geometry families that stress the
    traversal's exactness: the GPU film equals the C oracle's bit for bit."""
    from raytracingrenderer_amd.renderer import write_mesh_scene
    rng = np.random.default_rng(zlib.crc32(kind.encode()))
    P = _random_mesh(kind, rng)
    s = loadScene(write_mesh_scene(str(tmp_path), P, 64, 64))
    film = gpu_film(s, 3, seed=77, max_depth=depth)
    ref, _ = Oracle(s, depth, "rtm").render(3, seed=77, threads=8)
    assert_bitexact(film, ref, "%s depth %d" % (kind, depth))


def test_adaptive_render_matches_oracle():
    """RayTracer::adaptiveRender (Renderer.h:583-749): per-tile variance, weights and sample counts,
    and the film of mean-of-samples splats, bit-exact against the oracle (partial tiles included)."""
    s = loadScene(os.path.join(SCENES, "cornell-mat"), width=72, height=40)
    rt = RayTracer(s, seed=11)
    counts = rt.adaptiveRender(init_samples=2, max_samples=12, min_samples=1, first_sample=0)
    film, spp = rt.film()
    ref, ref_counts = Oracle(s, 4, "rtm").render_adaptive(first=0, seed=11, init=2, max_samples=12, min_samples=1)
    assert spp == 1
    assert counts.tolist() == ref_counts.tolist()
    assert counts.max() > counts.min()  # the variance actually steers the sample counts
    assert_bitexact(film, ref, "adaptive")


@pytest.mark.parametrize("scene_name", ["cornell-box", "cornell-mat"])
def test_light_tracer_matches_oracle(scene_name):
    """RayTracer::lightTracer (Renderer.h:221-326): every camera connection splatted in (path, vertex)
    order per pixel; device records sorted by key reproduce the sequential splat loop bit for bit."""
    s = loadScene(os.path.join(SCENES, scene_name), width=64, height=48)
    rt = RayTracer(s, seed=5)
    rt.lightTracer(2, first_frame=0)
    film, spp = rt.film()
    ref = Oracle(s, 4, "rtm").render_light(2, first=0, seed=5)
    assert spp == 2
    assert (ref != 0).sum() > 100
    assert_bitexact(film, ref, "light tracer " + scene_name)


@pytest.mark.parametrize("scene_name", ["cornell-box", "cornell-mat"])
def test_instant_radiosity_matches_oracle(scene_name):
    """RayTracer::instantRadiosity (Renderer.h:82-218): VPL paths, VPL order, per-pixel visibility
    against every VPL, bit-exact; with a small path budget the VPL batches are exercised too."""
    s = loadScene(os.path.join(SCENES, scene_name), width=48, height=40)
    rt = RayTracer(s, seed=9, max_paths=48 * 40 * 7)
    rt.instantRadiosity(2, n_vpl=20, first_frame=0)
    film, spp = rt.film()
    ref = Oracle(s, 4, "rtm").render_instant_radiosity(2, first=0, seed=9, n_vpl=20)
    assert spp == 2
    assert (ref != 0).sum() > 100
    assert_bitexact(film, ref, "instant radiosity " + scene_name)


def test_many_samples_per_chunk_and_path_order():
    """130 samples of every pixel in one chunk: pixel-major path ids fold the film in three passes
    of up to 64 samples (k_accumulate_pm) and must equal the oracle bit for bit; one sample per
    chunk (k_accumulate) gives the same film."""
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=32, height=32)
    ref, _ = Oracle(s, 4, "rtm").render(130, seed=1234, threads=8)
    assert_bitexact(gpu_film(s, 130), ref, "130 spp in one chunk")
    assert_bitexact(gpu_film(s, 130, max_paths=32 * 32), ref, "one sample per chunk")


def test_adaptive_render_many_frames_and_key_limit():
    """adaptiveRender frame after frame with the default sample keys (frame f draws from its own
    seed stream, so the 65536-sample PCG key never runs out), and a call whose sample range would
    leave the key is rejected before it touches the film or SPP."""
    from raytracingrenderer_amd import NativeError
    s = loadScene(os.path.join(SCENES, "cornell-mat"), width=40, height=40)
    rt = RayTracer(s, seed=3)
    for f in range(8):
        rt.adaptiveRender(init_samples=2, max_samples=10240, min_samples=1)
    film, spp = rt.film()
    assert spp == 8 and np.isfinite(film).all()
    # frame 1 equals the oracle's adaptive frame with the derived seed
    one = RayTracer(s, seed=3)
    one.adaptiveRender(init_samples=2, max_samples=64, min_samples=1)
    one.adaptiveRender(init_samples=2, max_samples=64, min_samples=1)
    f0, _ = Oracle(s, 4, "rtm").render_adaptive(first=0, seed=3, init=2, max_samples=64, min_samples=1)
    seed1 = (3 + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    f01, _ = Oracle(s, 4, "rtm").render_adaptive(first=0, seed=seed1, init=2, max_samples=64, min_samples=1,
                                                 film=f0.copy())
    assert_bitexact(one.film()[0], f01, "two adaptive frames")
    before, spp_before = rt.film()
    with pytest.raises(NativeError):
        rt.adaptiveRender(init_samples=2, max_samples=10240, min_samples=1, first_sample=65530)
    after, spp_after = rt.film()
    assert spp_after == spp_before
    assert_bitexact(after, before, "film untouched by a rejected adaptive call")


@pytest.mark.parametrize("flavour", ["rtm", "libm"])
@pytest.mark.parametrize("case", ["cornell-mat", "bathroom", "coffee+GI", "synth20k"])
def test_gpu_film_vs_reference_classes(case, flavour, synth20k):
    """The GPU film against RayTracer::pathTrace restated on RTBase's own compiled classes
    (oracle/_ref: the reference's BVH traversal, shading, BSDFs, lights, camera and Film), bit for
    bit: a film-level pin that does not go through the C oracle. libref.so calls the C library's
    transcendentals (the reference as built on Linux); libref_rtm.so has include/rtg_math.h's
    interposed (the same bits, which is what this shows at the film level)."""
    if flavour == "libm":
        require_reference_libm()
    from oracle import pyref
    if not pyref.available():
        pytest.fail("oracle/_ref (libref_rtm.so) missing: build it where /root/reference exists")
    if case == "synth20k":
        import tempfile
        d = tempfile.mkdtemp(prefix="rtg_s20k_")
        write_synthetic_scene(d, n_tris=20000, seed=3, width=128, height=96)
        path, kw, depth, spp, seed = d, dict(width=128, height=96), 4, 3, 42
    else:
        name, kw, depth, spp, seed = {
            "cornell-mat": (os.path.join(SCENES, "cornell-mat"), dict(width=80, height=60), 8, 3, 99),
            "bathroom": (staged("bathroom"), dict(width=96, height=54, skip_missing=True), 16, 2, 7),
            "coffee+GI": (staged("coffee"), dict(width=80, height=100, skip_missing=True, envmap="GI.hdr"), 4, 3, 5),
        }[case]
        path = name
    r = pyref.RefScene(path, kw["width"], kw["height"], kw.get("skip_missing", False), kw.get("envmap"),
                       flavour=flavour)
    ref, _ = r.render(spp, seed=seed, max_depth=depth, threads=8)
    s = loadScene(path, **kw)
    assert_bitexact(gpu_film(s, spp, seed=seed, max_depth=depth), ref,
                    "GPU vs reference classes (%s, %s)" % (case, flavour))


def _nan_canon(a):
    return np.where(np.isnan(a), np.float32(np.nan), a).view(np.uint32)


@pytest.mark.host_glibc
def test_device_math_matches_glibc():
    """The kernels' transcendentals (include/rtg_math.h compiled for gfx950, rtg_probe_math) against
    the host C library (liboracle_libm's or_math_eval calls glibc), bit for bit (any NaN equals any
    NaN): every 97th float bit pattern (44M inputs over all exponents) for sinf / cosf / sincosf /
    acosf, and 8M (y, x) pairs for atan2f (random bit patterns and unit-vector components)."""
    from oracle.pyoracle import lib
    G = lib("libm")
    x = np.arange(0, 1 << 32, 97, dtype=np.uint64).astype(np.uint32).view(np.float32)
    for fn, nout in ((0, len(x)), (1, len(x)), (2, 2 * len(x)), (3, len(x))):
        got = np.zeros(nout, np.float32)
        want = np.zeros(nout, np.float32)
        assert N.rtg().rtg_probe_math(fn, N.ptr(x, C.c_float), len(x), N.ptr(got, C.c_float)) == 0
        G.or_math_eval(fn, N.ptr(x, C.c_float), len(x), N.ptr(want, C.c_float))
        bad = np.flatnonzero(_nan_canon(got) != _nan_canon(want))
        assert bad.size == 0, (fn, bad.size, x[bad[:4] % len(x)].view(np.uint32), got[bad[:4]], want[bad[:4]])
    rng = np.random.default_rng(5)
    n = 1 << 23
    yx = rng.integers(0, 1 << 32, size=2 * n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    d = rng.normal(size=(n // 2, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    yx[: n] = d[:, [2, 0]].astype(np.float32).reshape(-1)  # EnvironmentMap::evaluate: atan2f(wi.z, wi.x)
    got = np.zeros(n, np.float32)
    want = np.zeros(n, np.float32)
    assert N.rtg().rtg_probe_math(4, N.ptr(yx, C.c_float), n, N.ptr(got, C.c_float)) == 0
    G.or_math_eval(4, N.ptr(yx, C.c_float), n, N.ptr(want, C.c_float))
    assert np.array_equal(_nan_canon(got), _nan_canon(want))


@pytest.mark.parametrize("scene_name", ["cornell-box", "cornell-mat"])
def test_gpu_integrators_vs_reference_classes(scene_name):
    """f4 at the film level without the C oracle: the GPU's direct / albedo / viewNormals /
    computeDirectMIS estimators, light tracer, instant radiosity and adaptive renderer against the
    same integrators restated on RTBase's own compiled classes (libref_rtm.so), bit for bit."""
    from oracle import pyref
    if not pyref.available():
        pytest.fail("oracle/_ref (libref_rtm.so) missing: build it where /root/reference exists")
    path = os.path.join(SCENES, scene_name)
    s = loadScene(path, width=64, height=48)
    r = pyref.RefScene(path, 64, 48, False, flavour="rtm")
    for name, mode in (("direct", 1), ("albedo", 2), ("normals", 3), ("direct_mis", 4)):
        rt = RayTracer(s, seed=7, integrator=name)
        rt.render(3, first_sample=0)
        assert_bitexact(rt.film()[0], r.render(3, seed=7, max_depth=4, mode=mode)[0], name)
    rt = RayTracer(s, seed=5)
    rt.lightTracer(2, first_frame=0)
    assert_bitexact(rt.film()[0], pyref.render_light(r, 2, seed=5), "light tracer")
    rt = RayTracer(s, seed=9)
    rt.instantRadiosity(2, n_vpl=20, first_frame=0)
    assert_bitexact(rt.film()[0], pyref.render_instant_radiosity(r, 2, seed=9, n_vpl=20), "instant radiosity")
    rt = RayTracer(s, seed=11)
    counts = rt.adaptiveRender(init_samples=2, max_samples=12, min_samples=1, first_sample=0)
    fa, ca = pyref.render_adaptive(r, seed=11, init=2, max_samples=12)
    assert counts.tolist() == ca.tolist()
    assert_bitexact(rt.film()[0], fa, "adaptive")


@pytest.mark.parametrize("cfg", ["C2", "C4", "C5", "MB"])
def test_full_size_configs_sampled_pixels(cfg):
    """BASELINE.json's other configs at their full sizes, rendered as the bench renders them (one
    rtg_render call of every sample: wavefront chunks, pixel-major fold): sampled pixels equal the
    oracle's per-path radiances summed in sample order, bit for bit.
    C2 cornell 1024^2 x 64 spp depth 8; C4 bathroom_f 1920x1080 x 256 spp depth 16; C5 coffee_f +
    GI.hdr 4096^2 x 1024 spp depth 4 (17.2G paths, ~7.5 s on one MI355X); MB: materialball_f at its
    own 1280x720, 64 spp, depth 8 (envmap.hdr is lights[0])."""
    spec = {"C2": ("cornell-box", 1024, 1024, 64, 8, {}, 4000),
            "C4": ("bathroom", 1920, 1080, 256, 16, {"skip_missing": True}, 1500),
            "C5": ("coffee", 4096, 4096, 1024, 4, {"skip_missing": True, "envmap": "GI.hdr"}, 1000),
            "MB": ("materialball", 1280, 720, 64, 8, {"skip_missing": True}, 2000)}[cfg]
    name, w, h, spp, depth, kw, npix = spec
    path = os.path.join(SCENES, name) if name == "cornell-box" else staged(name)
    s = loadScene(path, width=w, height=h, **kw)
    film = gpu_film(s, spp, max_depth=depth)
    rng = np.random.default_rng(len(cfg) * 7 + spp)
    pix = rng.choice(w * h, npix, replace=False).astype(np.uint32)
    o = Oracle(s, depth, "rtm")
    want = np.zeros((npix, 3), np.float32)
    for smp in range(spp):  # Film::splat: film += L, sample by sample, in float32
        want = want + o.trace_paths(pix, np.full(npix, smp, np.uint32), seed=1234)
    assert_bitexact(film.reshape(-1, 3)[pix], want, "%s sampled pixels" % cfg)


def test_count_mode_counters_are_consistent(synth20k, cornell256):
    """RTG_OPT_COUNT (the bench's untimed counting pass): counting leaves the film unchanged, and
    the walk counters nest (a leaf-box test needs a hit, a hit a fetched triangle tail, a tail a
    triangle test), which the roofline's fetch counts rely on."""
    for scene in (synth20k, cornell256):
        rt = RayTracer(scene, seed=1234, max_depth=4)
        rt.render(2, first_sample=0)
        plain = rt.film()[0].copy()
        rt.set_options(flags=N.RTG_OPT_CULL | N.RTG_OPT_COUNT)
        rt.clear()
        rt.render(2, first_sample=0)
        s = rt.stats()
        assert_bitexact(rt.film()[0], plain, "counting pass film")
        tris = s["tri_tests"] + s["shadow_tri_tests"]
        assert 0 < s["leafbox_tests"] <= s["tri_tail_loads"] <= tris, s
        assert s["node_lane_steps"] > 0 and s["extension_rays"] > 0, s
        # every lane of every loop iteration is stepping a node or idle for exactly one reason (the
        # bench's lane_idle_node shares; two parked-leaf slots: a lane with a free slot parks its leaf)
        idle = sum(s["lane_idle_" + k] for k in ("no_ray", "last_leaf", "leaf_blocked", "retiring", "leaf_popped"))
        assert s["lane_slots"] == s["node_lane_steps"] + idle, s


@pytest.mark.host_glibc
@pytest.mark.parametrize("case", ["cornell-mat", "bathroom", "coffee+GI", "materialball"])
def test_reference_side_binding_renders_reference_film(case):
    """The drop-in from the reference side: RTBase's own loader builds the Scene (oracle/_ref, the
    reference headers), integration/rtg_rtbase.h flattens it (the code INTEGRATION.md §2 shows),
    rtg_create uploads it and rtg_render renders; the film equals RayTracer::pathTrace on the same
    reference classes with glibc math (libref.so's ref_render), bit for bit."""
    from oracle import pyref
    if not pyref.available():
        pytest.fail("oracle/_ref (libref.so) missing: build it where /root/reference exists")
    path, kw, depth, spp, seed = {
        "cornell-mat": (os.path.join(SCENES, "cornell-mat"), dict(width=80, height=60), 8, 3, 21),
        "bathroom": (staged("bathroom"), dict(width=96, height=54, skip_missing=True), 16, 2, 22),
        "coffee+GI": (staged("coffee"), dict(width=80, height=100, skip_missing=True, envmap="GI.hdr"), 4, 3, 23),
        "materialball": (staged("materialball"), dict(width=96, height=54, skip_missing=True), 8, 2, 24),
    }[case]
    r = pyref.RefScene(path, kw["width"], kw["height"], kw.get("skip_missing", False), kw.get("envmap"),
                       flavour="libm")
    ref, _ = r.render(spp, seed=seed, max_depth=depth, threads=8)
    L = N.rtg()
    h = C.c_void_p()
    assert L.rtg_create(0, C.cast(r.rtg_desc(), C.POINTER(N.rtg_scene_desc)), C.byref(h)) == 0, L.rtg_last_error()
    try:
        assert L.rtg_set_options(h, depth, N.RTG_OPT_CULL, 0) == 0
        assert L.rtg_render(h, 0, spp, seed, None, 0) == 0, L.rtg_last_error()
        film = np.zeros((kw["height"], kw["width"], 3), np.float32)
        n = C.c_uint32()
        assert L.rtg_film_read(h, N.ptr(film, C.c_float), C.byref(n)) == 0
    finally:
        L.rtg_destroy(h)
    assert n.value == spp
    assert_bitexact(film, ref, "reference-side binding (%s)" % case)


def test_handle_churn_with_queued_frames():
    """Many handles created, rendering (waited-for and queued, one chunk at a time and several) and
    destroyed in one process, as this suite does: destroying full-CU-mask streams deadlocked the HIP
    runtime within a few handles (ROCm 7.2), so the slot streams are plain streams of one priority
    each, created and destroyed with their handle."""
    s = loadScene(os.path.join(SCENES, "cornell-mat"), width=64, height=35)
    want = gpu_film(s, 3, seed=7, max_depth=8)
    for i in range(60):
        rt = RayTracer(s, seed=7, max_depth=8, max_paths=(300 if i % 3 == 0 else 0))
        if i % 2:
            rt.set_options(flags=rt.flags | N.RTG_OPT_SERIAL)
        rt.render(2, first_sample=0)
        rt.render(1, first_sample=2, sync=False)
        film, n = rt.film()
        assert n == 3
        if i % 10 == 0:
            assert_bitexact(film, want, "handle %d" % i)
        del rt
