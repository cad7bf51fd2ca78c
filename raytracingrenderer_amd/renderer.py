"""Python mirror of RTBase's host-facing API on top of the native libraries.

  loadScene(name, ...)          -> Scene         RTBase/SceneLoader.h:237-291 (librth)
  RayTracer(scene, device)      .init/.render/.getSPP/.clear/.saveHDR   RTBase/Renderer.h:45-898
  Scene.triangles/.lights       post-BVH-build arrays (numpy views of the flattened Scene)

RayTracer.render() is the drop-in for RayTracer::render(): it adds one sample per pixel through
the HIP wavefront path tracer (librtg). There is no CPU fallback; without a GPU, RayTracer raises.
"""
import ctypes as C
import os

import numpy as np

from . import _native as N


class NativeError(RuntimeError):
    pass


def _check(rc, lib_err):
    if rc != 0:
        raise NativeError("%s (code %d)" % (lib_err().decode(errors="replace"), rc))


class Scene:
    """The flattened reference Scene produced by the host front-end (rth_load_scene)."""

    def __init__(self, handle):
        self._h = handle
        self.desc_ptr = N.rth().rth_scene_desc(handle)
        self.desc = self.desc_ptr.contents
        info = N.rth_scene_info()
        _check(N.rth().rth_scene_get_info(handle, C.byref(info)), N.rth().rth_last_error)
        self.info = info
        self.width, self.height = info.width, info.height

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            N.rth().rth_free_scene(h)

    # numpy views (no copy) of the flattened arrays; each view keeps this Scene alive
    def _view(self, p, n, dtype):
        if n == 0:
            return np.zeros(0, dtype)
        ctype = p._type_
        buf = (ctype * n).from_address(C.addressof(p.contents))
        buf._owner = self
        return np.frombuffer(buf, dtype=np.dtype(ctype)).view(dtype)

    @property
    def positions(self):
        return self._view(self.desc.positions, self.desc.n_tris * 9, np.float32).reshape(-1, 3, 3)

    @property
    def normals(self):
        return self._view(self.desc.normals, self.desc.n_tris * 9, np.float32).reshape(-1, 3, 3)

    @property
    def uvs(self):
        return self._view(self.desc.uvs, self.desc.n_tris * 6, np.float32).reshape(-1, 3, 2)

    @property
    def material_index(self):
        return self._view(self.desc.material, self.desc.n_tris, np.uint32)

    @property
    def node_bounds(self):
        return self._view(self.desc.node_bounds, self.desc.n_nodes * 6, np.float32).reshape(-1, 6)

    @property
    def node_links(self):
        return self._view(self.desc.node_links, self.desc.n_nodes * 4, np.int32).reshape(-1, 4)

    @property
    def lights(self):
        return self._view(self.desc.lights, self.desc.n_lights, np.int32)

    @property
    def materials(self):
        return [self.desc.materials[i] for i in range(self.desc.n_materials)]

    def texture(self, i):
        t = self.desc.textures[i]
        return self._view(t.texels, t.width * t.height * 3, np.float32).reshape(t.height, t.width, 3)

    @property
    def camera(self):
        c = self.desc.camera
        return {"inv_proj": np.array(c.inv_proj[:], np.float32).reshape(4, 4),
                "camera": np.array(c.camera[:], np.float32).reshape(4, 4),
                "origin": np.array(c.origin[:], np.float32), "width": c.width, "height": c.height}

    def permutation(self):
        out = np.zeros(self.desc.n_tris, np.uint32)
        _check(N.rth().rth_scene_permutation(self._h, N.ptr(out, C.c_uint32)), N.rth().rth_last_error)
        return out


def loadScene(scene_dir, width=0, height=0, skip_missing=False, envmap=None, bvh_threads=0):
    """RTBase loadScene(sceneName) with optional film-size / env overrides (applied before P)."""
    opts = N.rth_load_options(int(width), int(height), 1 if skip_missing else 0, int(bvh_threads),
                              envmap.encode() if envmap else None)
    h = C.c_void_p()
    _check(N.rth().rth_load_scene(os.fsencode(scene_dir), C.byref(opts), C.byref(h)), N.rth().rth_last_error)
    return Scene(h)


def write_synthetic_scene(out_dir, n_tris=1_000_000, seed=20251015, width=1024, height=1024):
    """C3 synthetic scene as .gem + scene.json + albedo.png + env.hdr."""
    os.makedirs(out_dir, exist_ok=True)
    _check(N.rth().rth_write_synthetic(os.fsencode(out_dir), n_tris, seed, width, height), N.rth().rth_last_error)
    return out_dir


def write_mesh_scene(out_dir, positions, width=256, height=256):
    """The C3 scene recipe (diffuse albedo, constant env light, fixed camera) around caller-given
    triangles: positions (n, 3, 3) float32."""
    p = np.ascontiguousarray(positions, np.float32).reshape(-1, 9)
    os.makedirs(out_dir, exist_ok=True)
    _check(N.rth().rth_write_mesh_scene(os.fsencode(out_dir), N.ptr(p, C.c_float), len(p), width, height),
           N.rth().rth_last_error)
    return out_dir


def save_hdr(path, film_sum, spp):
    """Film::save: film / SPP -> RLE RGBE (stbi_write_hdr format)."""
    f = np.ascontiguousarray(film_sum, np.float32)
    h, w = f.shape[0], f.shape[1]
    _check(N.rth().rth_save_hdr(os.fsencode(path), w, h, N.ptr(f, C.c_float), spp), N.rth().rth_last_error)


def tonemap(film_sum, spp, exposure=1.0):
    """Film::tonemap (Imaging.h:233-242) of every pixel -> uint8 RGB (H, W, 3)."""
    f = np.ascontiguousarray(film_sum, np.float32)
    h, w = f.shape[0], f.shape[1]
    out = np.zeros((h, w, 3), np.uint8)
    _check(N.rth().rth_tonemap(w, h, N.ptr(f, C.c_float), spp, exposure, N.ptr(out, C.c_uint8)),
           N.rth().rth_last_error)
    return out


def save_png(path, film_sum, spp):
    """RayTracer::savePNG (Renderer.h:895-898): tonemapped film as an 8-bit RGB PNG."""
    f = np.ascontiguousarray(film_sum, np.float32)
    h, w = f.shape[0], f.shape[1]
    _check(N.rth().rth_save_png(os.fsencode(path), w, h, N.ptr(f, C.c_float), spp), N.rth().rth_last_error)


def read_hdr(path):
    w, h = C.c_int32(), C.c_int32()
    p = N.f32p()
    _check(N.rth().rth_read_hdr(os.fsencode(path), C.byref(w), C.byref(h), C.byref(p)), N.rth().rth_last_error)
    try:
        return np.ctypeslib.as_array(p, shape=(h.value, w.value, 3)).copy()
    finally:
        N.rth().rth_free(C.cast(p, C.c_void_p))


class RayTracer:
    """RayTracer (Renderer.h:31-899) backed by librtg on one GPU."""

    MAX_DEPTH = 4  # Renderer.h:20

    INTEGRATORS = {"path": N.RTG_INTEGRATOR_PATH, "direct": N.RTG_INTEGRATOR_DIRECT,
                   "albedo": N.RTG_INTEGRATOR_ALBEDO, "normals": N.RTG_INTEGRATOR_NORMALS,
                   "direct_mis": N.RTG_INTEGRATOR_DIRECT_MIS}

    def __init__(self, scene, device=0, max_depth=MAX_DEPTH, seed=1234, cull=True, max_paths=0, wide=True,
                 integrator="path"):
        self.scene = scene
        self.seed = seed
        self._lib = N.rtg()
        h = C.c_void_p()
        _check(self._lib.rtg_create(device, scene.desc_ptr, C.byref(h)), self._lib.rtg_last_error)
        self._h = h
        self.width, self.height = scene.width, scene.height
        self.max_depth = max_depth
        self.flags = (N.RTG_OPT_CULL if cull else 0) | (0 if wide else N.RTG_OPT_BVH2)
        self.set_options(max_depth=max_depth, flags=self.flags, max_paths=max_paths)
        self.set_integrator(integrator)

    def set_integrator(self, integrator):
        """Per-pixel estimator: "path" (pathTrace, default), "direct", "albedo", "normals"
        (RayTracer::direct / albedo / viewNormals, Renderer.h:393-407, 558-582), "direct_mis"
        (direct() with computeDirectMIS, Renderer.h:474-557)."""
        mode = self.INTEGRATORS[integrator] if isinstance(integrator, str) else int(integrator)
        _check(self._lib.rtg_set_integrator(self._h, mode), self._lib.rtg_last_error)
        self.integrator = integrator

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.rtg_destroy(h)

    def set_options(self, max_depth=None, flags=None, max_paths=0):
        if max_depth is not None:
            self.max_depth = max_depth
        if flags is not None:
            self.flags = flags
        _check(self._lib.rtg_set_options(self._h, self.max_depth, self.flags, max_paths), self._lib.rtg_last_error)

    @property
    def handle(self):
        """The rtg_handle* (ctypes void pointer) for direct C-ABI calls (e.g. rtg_film_gather)."""
        return self._h

    @property
    def tiles_x(self):
        return (self.width + 31) // 32

    @property
    def tiles_y(self):
        return (self.height + 31) // 32

    def render(self, n_samples=1, tiles=None, first_sample=None, sync=True, stream=None):
        """RayTracer::render(): add n_samples samples per pixel (default 1 = one frame).
        sync=False queues the frame (rtg_render_async): a frame loop of 1-spp calls then keeps up to
        three frames in flight on the GPU; film() / stats() / synchronize() wait for them.
        stream (a HIP stream handle, not the null stream): the render is ordered after the caller's
        earlier work on that stream and the caller's later work on it sees the film; the call returns
        without waiting (rtg_render_async with a stream)."""
        first = self.getSPP() if first_sample is None else first_sample
        t = None if tiles is None else np.ascontiguousarray(tiles, np.uint32)
        tp = N.ptr(t, C.c_uint32) if t is not None else None
        nt = 0 if t is None else len(t)
        if stream:
            rc = self._lib.rtg_render_async(self._h, first, n_samples, self.seed, tp, nt, C.c_void_p(stream))
        elif sync:
            rc = self._lib.rtg_render(self._h, first, n_samples, self.seed, tp, nt)
        else:
            rc = self._lib.rtg_render_async(self._h, first, n_samples, self.seed, tp, nt, None)
        _check(rc, self._lib.rtg_last_error)

    def adaptiveRender(self, init_samples=2, max_samples=10240, min_samples=1, first_sample=None):
        """RayTracer::adaptiveRender (Renderer.h:583-749): one frame whose per-tile sample counts
        follow the tiles' variance after init_samples samples. Returns the per-tile counts. The frame
        draws sample indices first_sample ... first_sample + init_samples + max(count) - 1 of the
        PCG streams keyed by `seed` (limit: RTG_MAX_SAMPLES_PER_KEY = 65536). Default (first_sample
        None): frame f = getSPP() draws indices 0 ... of its own seed, seed + f * 0x9E3779B97F4A7C15
        (mod 2^64), so any number of frames stays inside the key space."""
        if first_sample is None:
            first, seed = 0, (self.seed + self.getSPP() * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        else:
            first, seed = first_sample, self.seed
        counts = np.zeros(self.tiles_x * self.tiles_y, np.uint32)
        _check(self._lib.rtg_render_adaptive(self._h, first, seed, init_samples, max_samples, min_samples,
                                             N.ptr(counts, C.c_uint32)), self._lib.rtg_last_error)
        return counts

    def lightTracer(self, n_frames=1, first_frame=None):
        """RayTracer::lightTracer (Renderer.h:221-326): width*height light paths per frame, each
        vertex connected to the camera and splatted (Film::SPP += 1 per frame)."""
        first = self.getSPP() if first_frame is None else first_frame
        _check(self._lib.rtg_render_light(self._h, first, n_frames, self.seed), self._lib.rtg_last_error)

    def instantRadiosity(self, n_frames=1, n_vpl=50, first_frame=None):
        """RayTracer::instantRadiosity (Renderer.h:82-218): n_vpl VPL paths (MAX_VPL = 50) per frame,
        then every pixel's first hit gathers all visible VPLs (Film::SPP += 1 per frame)."""
        first = self.getSPP() if first_frame is None else first_frame
        _check(self._lib.rtg_render_instant_radiosity(self._h, first, n_frames, self.seed, n_vpl),
               self._lib.rtg_last_error)

    def synchronize(self):
        _check(self._lib.rtg_synchronize(self._h), self._lib.rtg_last_error)

    def idle(self):
        """True when no queued render work is left on the GPU (rtg_render_idle)."""
        v = C.c_int()
        _check(self._lib.rtg_render_idle(self._h, C.byref(v)), self._lib.rtg_last_error)
        return bool(v.value)

    def film(self):
        """(sum, spp): the unnormalised Film::film and Film::SPP."""
        out = np.zeros((self.height, self.width, 3), np.float32)
        spp = C.c_uint32()
        _check(self._lib.rtg_film_read(self._h, N.ptr(out, C.c_float), C.byref(spp)), self._lib.rtg_last_error)
        return out, spp.value

    def load_film(self, film_sum, spp):
        f = np.ascontiguousarray(film_sum, np.float32)
        _check(self._lib.rtg_film_load(self._h, N.ptr(f, C.c_float), spp), self._lib.rtg_last_error)

    def copy_film_to(self, device_ptr):
        _check(self._lib.rtg_film_copy_device(self._h, C.c_void_p(device_ptr)), self._lib.rtg_last_error)

    def getSPP(self):
        spp = C.c_uint32()
        _check(self._lib.rtg_film_read(self._h, None, C.byref(spp)), self._lib.rtg_last_error)
        return spp.value

    def clear(self):
        _check(self._lib.rtg_clear(self._h), self._lib.rtg_last_error)

    def saveHDR(self, filename):
        f, spp = self.film()
        save_hdr(filename, f, max(spp, 1))

    def savePNG(self, filename):
        f, spp = self.film()
        save_png(filename, f, spp)

    def stats(self):
        s = N.rtg_stats()
        _check(self._lib.rtg_get_stats(self._h, C.byref(s)), self._lib.rtg_last_error)
        return {k: getattr(s, k) for k, _ in N.rtg_stats._fields_}

    def trace_closest(self, rays):
        r = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        out = np.zeros((len(r), 4), np.float32)
        _check(self._lib.rtg_trace_closest(self._h, N.ptr(r, C.c_float), len(r), N.ptr(out, C.c_float)),
               self._lib.rtg_last_error)
        return out

    def trace_visible(self, rays):
        r = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        out = np.zeros(len(r), np.int32)
        _check(self._lib.rtg_trace_visible(self._h, N.ptr(r, C.c_float), len(r), N.ptr(out, C.c_int32)),
               self._lib.rtg_last_error)
        return out


class RayTracerGroup:
    """RayTracer over several GPUs of one node (rtg_group_*, rtg_multi.hip): rank r renders the 32x32
    tiles with (tile_x + tile_y) % N == r on devices[r] (one host thread per device), and film()
    assembles the film on devices[0] from every rank's own tiles (packed on each device, one RCCL
    send per rank, scattered on devices[0]). The result is bit-identical to a one-device render
    (RayTracer::pathTracerTileBased's tile pool, Renderer.h:836-853, spread over devices). A device
    list with repeats rehearses N ranks on fewer GPUs (the ranks then render in turn and the packed
    tiles move with device copies)."""

    def __init__(self, scene, devices=(0,), max_depth=RayTracer.MAX_DEPTH, seed=1234, cull=True, max_paths=0):
        self.scene = scene
        self.seed = seed
        self.devices = list(devices)
        self.width, self.height = scene.width, scene.height
        self._lib = N.rtg()
        dev = np.ascontiguousarray(self.devices, np.int32)
        g = C.c_void_p()
        _check(self._lib.rtg_group_create(N.ptr(dev, C.c_int32), len(dev), scene.desc_ptr, C.byref(g)),
               self._lib.rtg_last_error)
        self._g = g
        self.max_depth = max_depth
        self.flags = N.RTG_OPT_CULL if cull else 0
        _check(self._lib.rtg_group_set_options(g, max_depth, self.flags, max_paths), self._lib.rtg_last_error)
        self._spp = 0

    def set_options(self, max_depth=None, flags=None, max_paths=0):
        if max_depth is not None:
            self.max_depth = max_depth
        if flags is not None:
            self.flags = flags
        _check(self._lib.rtg_group_set_options(self._g, self.max_depth, self.flags, max_paths),
               self._lib.rtg_last_error)

    def setup_ms(self):
        """(host build of the device records, parallel uploads) of rtg_group_create, in ms."""
        a, b = C.c_double(), C.c_double()
        _check(self._lib.rtg_group_setup_ms(self._g, C.byref(a), C.byref(b)), self._lib.rtg_last_error)
        return a.value, b.value

    def reduce(self, sync=True):
        """Assemble the film on devices[0] from every rank's own tiles (RCCL send/recv; device copies
        for repeated devices). sync=False queues it on the exchange streams after every rank's queued
        frames (rtg_group_reduce_async): the ranks' next frames run on meanwhile."""
        fn = self._lib.rtg_group_reduce if sync else self._lib.rtg_group_reduce_async
        _check(fn(self._g), self._lib.rtg_last_error)

    def synchronize(self):
        """Wait for every rank's queued frames and the queued exchanges (rtg_group_synchronize)."""
        _check(self._lib.rtg_group_synchronize(self._g), self._lib.rtg_last_error)

    def rank_stats(self):
        """rtg_get_stats of every rank's handle (rays, kernel ms, counting-pass counters)."""
        out = []
        for r in range(len(self.devices)):
            h = self._lib.rtg_group_handle(self._g, r)
            st = N.rtg_stats()
            _check(self._lib.rtg_get_stats(h, C.byref(st)), self._lib.rtg_last_error)
            out.append({k: getattr(st, k) for k, _ in N.rtg_stats._fields_})
        return out

    def __del__(self):
        g, self._g = getattr(self, "_g", None), None
        if g:
            self._lib.rtg_group_destroy(g)

    @property
    def uses_rccl(self):
        return bool(self._lib.rtg_group_uses_rccl(self._g))

    def render(self, n_samples=1, first_sample=None, sync=True):
        """Every rank adds n_samples samples of its tiles. sync=False queues the frame on every rank
        (rtg_group_render_async: coalesced and pipelined per rank, as RayTracer.render(sync=False))."""
        first = self._spp if first_sample is None else first_sample
        fn = self._lib.rtg_group_render if sync else self._lib.rtg_group_render_async
        _check(fn(self._g, first, n_samples, self.seed), self._lib.rtg_last_error)
        self._spp = first + n_samples

    def film(self):
        """(sum, spp) of the reduced film."""
        out = np.zeros((self.height, self.width, 3), np.float32)
        spp = C.c_uint32()
        _check(self._lib.rtg_group_film_read(self._g, N.ptr(out, C.c_float), C.byref(spp)), self._lib.rtg_last_error)
        return out, spp.value

    def reduce_ms(self):
        return self._lib.rtg_group_reduce_ms(self._g)

    def clear(self):
        _check(self._lib.rtg_group_clear(self._g), self._lib.rtg_last_error)
        self._spp = 0


def tiles_for_rank_native(width, height, rank, world):
    """rtg_tiles_for_rank (the C partition the group uses); equals distributed.tiles_for_rank."""
    lib = N.rtg()
    n = C.c_uint32()
    _check(lib.rtg_tiles_for_rank(width, height, rank, world, None, C.byref(n)), lib.rtg_last_error)
    out = np.zeros(n.value, np.uint32)
    _check(lib.rtg_tiles_for_rank(width, height, rank, world, N.ptr(out, C.c_uint32), C.byref(n)), lib.rtg_last_error)
    return out
