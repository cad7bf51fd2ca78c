"""TEST INFRASTRUCTURE ONLY — ctypes access to oracle/_ref/libref.so (the reference's own
headers compiled from /root/reference; only available in the build container)."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_ref", "libref.so")
LIB_RTM = os.path.join(HERE, "_ref", "libref_rtm.so")  # same code, shared transcendentals interposed


def available():
    return os.path.exists(LIB)


_libs = {}


def lib(flavour="libm"):
    if flavour not in _libs:
        L = C.CDLL(LIB if flavour == "libm" else LIB_RTM)
        vp = C.c_void_p
        L.ref_load.restype = vp
        L.ref_load.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_char_p]
        for name in ("ref_counts", "ref_export", "ref_texture_size", "ref_texture_texels", "ref_traverse",
                     "ref_traverse_visible", "ref_visible", "ref_camera_rays", "ref_env_eval", "ref_tex_sample",
                     "ref_camera_project", "ref_light_emit"):
            getattr(L, name).restype = None
        L.ref_bsdf_sample.restype = None
        L.ref_rtg_desc.restype = vp
        L.ref_rtg_desc.argtypes = [vp]
        L.ref_save_hdr.restype = C.c_int
        L.ref_load_texture.restype = C.c_int
        _libs[flavour] = L
    return _libs[flavour]


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class RefScene:
    def __init__(self, scene_dir, width=0, height=0, skip_missing=False, envmap=None, flavour="libm"):
        self.L = lib(flavour)
        self.h = self.L.ref_load(os.fsencode(scene_dir), width, height, 1 if skip_missing else 0,
                                 envmap.encode() if envmap else None)
        c = np.zeros(8, np.int32)
        self.L.ref_counts(C.c_void_p(self.h), _p(c))
        self.ntri, self.nnode, self.nlight, self.nmat, self.ntex, self.env_tex, self.W, self.H = c.tolist()

    def render(self, n_samples, first=0, seed=1234, max_depth=4, threads=8, film=None, count=False, mode=0):
        """ref_render: RayTracer::render x n_samples on the reference's own classes (tile pool of
        `threads` std::threads, deterministic sampler). mode: 0 pathTrace, 1 direct, 2 albedo,
        3 viewNormals, 4 direct with computeDirectMIS (RTG_INTEGRATOR_*). Returns (film sum,
        counts[paths, closest, shadow])."""
        if film is None:
            film = np.zeros((self.H, self.W, 3), np.float32)
        counts = np.zeros(3, np.uint64)
        L = self.L
        L.ref_render_mode.restype = C.c_int
        L.ref_render_mode.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_int, C.c_int, C.c_void_p,
                                      C.c_void_p, C.c_int]
        L.ref_render_mode(self.h, first, n_samples, seed, max_depth, threads, film.ctypes.data, counts.ctypes.data,
                          mode)
        return film, counts

    def rtg_desc(self):
        """Pointer to the rtg_scene_desc built by integration/rtg_rtbase.h (rtg_flatten_scene) from
        this reference Scene; valid while this object lives."""
        return self.L.ref_rtg_desc(C.c_void_p(self.h))

    def export(self):
        n, m = self.ntri, self.nnode
        d = {"positions": np.zeros((n, 3, 3), np.float32), "normals": np.zeros((n, 3, 3), np.float32),
             "uvs": np.zeros((n, 3, 2), np.float32), "material": np.zeros(n, np.uint32),
             "node_bounds": np.zeros((m, 6), np.float32), "node_links": np.zeros((m, 4), np.int32),
             "lights": np.zeros(self.nlight, np.int32), "camera": np.zeros(37, np.float32),
             "mat_info": np.zeros((self.nmat, 3), np.int32), "mat_f": np.zeros((self.nmat, 5), np.float32)}
        self.L.ref_export(C.c_void_p(self.h), *[_p(d[k]) for k in ("positions", "normals", "uvs", "material", "node_bounds",
                                                                 "node_links", "lights", "camera", "mat_info", "mat_f")])
        return d

    def texture(self, i):
        wh = np.zeros(2, np.int32)
        self.L.ref_texture_size(C.c_void_p(self.h), int(i), _p(wh))
        out = np.zeros((wh[1], wh[0], 3), np.float32)
        self.L.ref_texture_texels(C.c_void_p(self.h), int(i), _p(out))
        return out

    def traverse(self, rays):
        r = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        out = np.zeros((len(r), 4), np.float32)
        self.L.ref_traverse(C.c_void_p(self.h), _p(r), len(r), _p(out))
        return out

    def traverse_visible(self, rays):
        r = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        out = np.zeros(len(r), np.int32)
        self.L.ref_traverse_visible(C.c_void_p(self.h), _p(r), len(r), _p(out))
        return out

    def camera_rays(self, pixels):
        p = np.ascontiguousarray(pixels, np.uint32)
        out = np.zeros((len(p), 6), np.float32)
        self.L.ref_camera_rays(C.c_void_p(self.h), _p(p), len(p), _p(out))
        return out

    def camera_project(self, pts):
        p = np.ascontiguousarray(pts, np.float32).reshape(-1, 3)
        out = np.zeros((len(p), 3), np.float32)
        state = np.zeros(36, np.float32)
        self.L.ref_camera_project(C.c_void_p(self.h), _p(p), len(p), _p(out), _p(state))
        return out, state

    def light_emit(self, li, draws):
        d = np.ascontiguousarray(draws, np.float32)
        out = np.zeros(12, np.float32)
        self.L.ref_light_emit(C.c_void_p(self.h), int(li), _p(d), len(d), _p(out))
        return out

    def env_eval(self, tex, dirs):
        d = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        out = np.zeros((len(d), 3), np.float32)
        self.L.ref_env_eval(C.c_void_p(self.h), int(tex), _p(d), len(d), _p(out))
        return out

    def tex_sample(self, tex, uv):
        u = np.ascontiguousarray(uv, np.float32).reshape(-1, 2)
        out = np.zeros((len(u), 3), np.float32)
        self.L.ref_tex_sample(C.c_void_p(self.h), int(tex), _p(u), len(u), _p(out))
        return out


def bsdf_sample(kind, albedo, sd, draws, int_ior=1.33, ext_ior=1.0, flavour="libm"):
    a = np.asarray(albedo, np.float32)
    s = np.asarray(sd, np.float32)
    d = np.asarray(draws, np.float32)
    out = np.zeros(11, np.float32)
    lib(flavour).ref_bsdf_sample(C.c_int(kind), _p(a), C.c_float(int_ior), C.c_float(ext_ior), _p(s), _p(d), C.c_int(len(d)), _p(out))
    return out


def save_hdr(path, film_sum, spp):
    f = np.ascontiguousarray(film_sum, np.float32)
    lib().ref_save_hdr(os.fsencode(path), f.shape[1], f.shape[0], _p(f), spp)


def load_texture(path, cap=1 << 24):
    out = np.zeros(cap, np.float32)
    wh = np.zeros(2, np.int32)
    n = lib().ref_load_texture(os.fsencode(path), _p(out), cap, _p(wh))
    return out[: n * 3].reshape(wh[1], wh[0], 3)


def tonemap(film_sum, spp, exposure=1.0):
    """Film::tonemap (Imaging.h:233-242) of every pixel, from the reference's own class."""
    f = np.ascontiguousarray(film_sum, np.float32)
    out = np.zeros(f.shape[:2] + (3,), np.uint8)
    L = lib()
    L.ref_tonemap.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_float, C.c_void_p]
    L.ref_tonemap(f.shape[1], f.shape[0], f.ctypes.data, spp, C.c_float(exposure), out.ctypes.data)
    return out


def _bind_extra(L):
    if getattr(L, "_extra_bound", False):
        return L
    L.ref_render_light.restype = C.c_int
    L.ref_render_light.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_void_p]
    L.ref_render_ir.restype = C.c_int
    L.ref_render_ir.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_void_p]
    L.ref_render_adaptive.restype = C.c_int
    L.ref_render_adaptive.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.c_void_p, C.c_void_p]
    L._extra_bound = True
    return L


def render_light(ref_scene, n_frames=1, first=0, seed=1234):
    """RayTracer::lightTracer restated on the reference's classes (ref_render_light)."""
    film = np.zeros((ref_scene.H, ref_scene.W, 3), np.float32)
    _bind_extra(ref_scene.L).ref_render_light(ref_scene.h, first, n_frames, seed, film.ctypes.data)
    return film


def render_instant_radiosity(ref_scene, n_frames=1, first=0, seed=1234, n_vpl=50):
    """RayTracer::instantRadiosity restated on the reference's classes (ref_render_ir)."""
    film = np.zeros((ref_scene.H, ref_scene.W, 3), np.float32)
    _bind_extra(ref_scene.L).ref_render_ir(ref_scene.h, first, n_frames, seed, n_vpl, film.ctypes.data)
    return film


def render_adaptive(ref_scene, first=0, seed=1234, init=2, max_samples=10240, min_samples=1):
    """RayTracer::adaptiveRender restated on the reference's classes (ref_render_adaptive)."""
    film = np.zeros((ref_scene.H, ref_scene.W, 3), np.float32)
    nt = ((ref_scene.W + 31) // 32) * ((ref_scene.H + 31) // 32)
    counts = np.zeros(nt, np.uint32)
    _bind_extra(ref_scene.L).ref_render_adaptive(ref_scene.h, first, seed, init, max_samples, min_samples,
                                                 film.ctypes.data, counts.ctypes.data)
    return film, counts
