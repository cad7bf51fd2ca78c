"""ctypes bindings for the two native libraries (include/rtg.h, include/rth.h).

No fallback: if librtg.so / librth.so are missing or fail to load, import of the bindings
raises. Build them with `python -m raytracingrenderer_amd.build` (or __graft_entry__.build()).
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")

RTG_MAT_DIFFUSE, RTG_MAT_LAMBERT, RTG_MAT_MIRROR, RTG_MAT_GLASS = 0, 1, 2, 3
RTG_OPT_CULL, RTG_OPT_COUNT, RTG_OPT_TIMING, RTG_OPT_BVH2, RTG_OPT_WAVETIME, RTG_OPT_SERIAL = 1, 2, 4, 8, 16, 32
RTG_OPT_NO_COALESCE = 64
RTG_INTEGRATOR_PATH, RTG_INTEGRATOR_DIRECT, RTG_INTEGRATOR_ALBEDO, RTG_INTEGRATOR_NORMALS = 0, 1, 2, 3
RTG_INTEGRATOR_DIRECT_MIS = 4

f32p = C.POINTER(C.c_float)
u32p = C.POINTER(C.c_uint32)
i32p = C.POINTER(C.c_int32)


class rtg_camera(C.Structure):
    _fields_ = [("inv_proj", C.c_float * 16), ("camera", C.c_float * 16), ("origin", C.c_float * 3),
                ("width", C.c_float), ("height", C.c_float)]


class rtg_camera_proj(C.Structure):
    _fields_ = [("proj", C.c_float * 16), ("camera_to_view", C.c_float * 16), ("view_direction", C.c_float * 3),
                ("a_film", C.c_float)]


class rtg_material(C.Structure):
    _fields_ = [("kind", C.c_int32), ("two_sided", C.c_int32), ("texture", C.c_int32),
                ("int_ior", C.c_float), ("ext_ior", C.c_float), ("emission", C.c_float * 3)]


class rtg_texture(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("texels", f32p)]


class rtg_scene_desc(C.Structure):
    _fields_ = [("n_tris", C.c_uint32), ("positions", f32p), ("normals", f32p), ("uvs", f32p),
                ("material", u32p), ("n_nodes", C.c_uint32), ("node_bounds", f32p),
                ("node_links", i32p), ("n_materials", C.c_uint32),
                ("materials", C.POINTER(rtg_material)), ("n_textures", C.c_uint32),
                ("textures", C.POINTER(rtg_texture)), ("env_texture", C.c_int32),
                ("n_lights", C.c_uint32), ("lights", i32p), ("camera", rtg_camera),
                ("projection", rtg_camera_proj)]


class rtg_stats(C.Structure):
    _fields_ = [("paths", C.c_uint64), ("extension_rays", C.c_uint64), ("shadow_rays", C.c_uint64),
                ("node_visits", C.c_uint64), ("tri_tests", C.c_uint64), ("shadow_node_visits", C.c_uint64),
                ("shadow_tri_tests", C.c_uint64), ("extend_launches", C.c_uint64), ("render_ms", C.c_double),
                ("extend_ms", C.c_double), ("shadow_ms", C.c_double), ("shade_ms", C.c_double),
                ("lane_slots", C.c_uint64), ("node_lane_steps", C.c_uint64), ("leaf_lane_steps", C.c_uint64),
                ("leaf_phase_slots", C.c_uint64), ("pops", C.c_uint64), ("cullable_pops", C.c_uint64),
                ("tri_tail_loads", C.c_uint64), ("leafbox_tests", C.c_uint64), ("traced_camera_rays", C.c_uint64),
                ("chunk_samples", C.c_uint64), ("lane_idle_no_ray", C.c_uint64),
                ("lane_idle_last_leaf", C.c_uint64), ("lane_idle_leaf_blocked", C.c_uint64),
                ("lane_idle_retiring", C.c_uint64), ("lane_idle_leaf_popped", C.c_uint64)]


class rth_load_options(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("skip_missing", C.c_int32),
                ("bvh_threads", C.c_int32), ("envmap", C.c_char_p)]


class rth_scene_info(C.Structure):
    _fields_ = [("n_tris", C.c_uint32), ("n_nodes", C.c_uint32), ("n_materials", C.c_uint32),
                ("n_textures", C.c_uint32), ("n_lights", C.c_uint32), ("bvh_depth", C.c_uint32),
                ("width", C.c_int32), ("height", C.c_int32), ("env_in_lights", C.c_int32),
                ("dropped_instances", C.c_uint32), ("load_ms", C.c_double), ("bvh_ms", C.c_double),
                ("bounds_min", C.c_float * 3), ("bounds_max", C.c_float * 3)]


RTG_EXPORTS = [
    ("rtg_abi_version", C.c_int32, []),
    ("rtg_build_id", C.c_char_p, []),
    ("rtg_last_error", C.c_char_p, []),
    ("rtg_device_count", C.c_int, [i32p]),
    ("rtg_create", C.c_int, [C.c_int, C.POINTER(rtg_scene_desc), C.POINTER(C.c_void_p)]),
    ("rtg_destroy", None, [C.c_void_p]),
    ("rtg_set_options", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_uint32]),
    ("rtg_set_integrator", C.c_int, [C.c_void_p, C.c_int]),
    ("rtg_render", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64, u32p, C.c_uint32]),
    ("rtg_render_async", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64, u32p, C.c_uint32, C.c_void_p]),
    ("rtg_synchronize", C.c_int, [C.c_void_p]),
    ("rtg_render_idle", C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    ("rtg_render_light", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64]),
    ("rtg_render_instant_radiosity", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32]),
    ("rtg_render_adaptive", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, u32p]),
    ("rtg_film_read", C.c_int, [C.c_void_p, f32p, u32p]),
    ("rtg_film_copy_device", C.c_int, [C.c_void_p, C.c_void_p]),
    ("rtg_film_load", C.c_int, [C.c_void_p, f32p, C.c_uint32]),
    ("rtg_clear", C.c_int, [C.c_void_p]),
    ("rtg_get_stats", C.c_int, [C.c_void_p, C.POINTER(rtg_stats)]),
    ("rtg_launch_times", C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.c_uint32, u32p]),
    ("rtg_launch_rays", C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32, u32p]),
    ("rtg_debug_capture", C.c_int, [C.c_void_p, C.c_int]),
    ("rtg_debug_replay", C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    ("rtg_trace_closest", C.c_int, [C.c_void_p, f32p, C.c_uint32, f32p]),
    ("rtg_trace_visible", C.c_int, [C.c_void_p, f32p, C.c_uint32, i32p]),
    ("rtg_probe_bsdf", C.c_int, [f32p, C.c_uint32, f32p]),
    ("rtg_probe_math", C.c_int, [C.c_int, f32p, C.c_uint32, f32p]),
    # one node, several GPUs (rtg_multi.hip): tile stripes per device + one RCCL film reduce
    ("rtg_tiles_for_rank", C.c_int, [C.c_uint32, C.c_uint32, C.c_int, C.c_int, u32p, u32p]),
    ("rtg_group_create", C.c_int, [i32p, C.c_int, C.POINTER(rtg_scene_desc), C.POINTER(C.c_void_p)]),
    ("rtg_group_destroy", None, [C.c_void_p]),
    ("rtg_group_size", C.c_int, [C.c_void_p]),
    ("rtg_group_handle", C.c_void_p, [C.c_void_p, C.c_int]),
    ("rtg_group_set_options", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_uint32]),
    ("rtg_group_render", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64]),
    ("rtg_group_reduce", C.c_int, [C.c_void_p]),
    ("rtg_group_render_async", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64]),
    ("rtg_group_reduce_async", C.c_int, [C.c_void_p]),
    ("rtg_group_synchronize", C.c_int, [C.c_void_p]),
    ("rtg_group_film_read", C.c_int, [C.c_void_p, f32p, u32p]),
    ("rtg_group_clear", C.c_int, [C.c_void_p]),
    ("rtg_group_reduce_ms", C.c_double, [C.c_void_p]),
    ("rtg_group_uses_rccl", C.c_int, [C.c_void_p]),
    ("rtg_group_setup_ms", C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    # own-tile film exchange (rtg_multi.hip)
    ("rtg_tile_pixels", C.c_int, [C.c_uint32, C.c_uint32, u32p, C.c_uint32, u32p, u32p]),
    ("rtg_film_gather", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]),
    ("rtg_film_scatter", C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p]),
]

RTH_EXPORTS = [
    ("rth_last_error", C.c_char_p, []),
    ("rth_build_id", C.c_char_p, []),
    ("rth_load_scene", C.c_int, [C.c_char_p, C.POINTER(rth_load_options), C.POINTER(C.c_void_p)]),
    ("rth_free_scene", None, [C.c_void_p]),
    ("rth_scene_desc", C.POINTER(rtg_scene_desc), [C.c_void_p]),
    ("rth_scene_get_info", C.c_int, [C.c_void_p, C.POINTER(rth_scene_info)]),
    ("rth_scene_permutation", C.c_int, [C.c_void_p, u32p]),
    ("rth_save_hdr", C.c_int, [C.c_char_p, C.c_int32, C.c_int32, f32p, C.c_uint32]),
    ("rth_write_hdr", C.c_int, [C.c_char_p, C.c_int32, C.c_int32, f32p]),
    ("rth_read_hdr", C.c_int, [C.c_char_p, i32p, i32p, C.POINTER(f32p)]),
    ("rth_read_png", C.c_int, [C.c_char_p, i32p, i32p, i32p, C.POINTER(C.POINTER(C.c_uint8))]),
    ("rth_write_mesh_scene", C.c_int, [C.c_char_p, f32p, C.c_uint32, C.c_int32, C.c_int32]),
    ("rth_read_ldr", C.c_int, [C.c_char_p, i32p, i32p, i32p, C.POINTER(C.POINTER(C.c_uint8))]),
    ("rth_tonemap", C.c_int, [C.c_int32, C.c_int32, f32p, C.c_uint32, C.c_float, C.POINTER(C.c_uint8)]),
    ("rth_save_png", C.c_int, [C.c_char_p, C.c_int32, C.c_int32, f32p, C.c_uint32]),
    ("rth_free", None, [C.c_void_p]),
    ("rth_write_synthetic", C.c_int, [C.c_char_p, C.c_uint32, C.c_uint64, C.c_int32, C.c_int32]),
]


def _bind(lib, exports):
    for name, res, args in exports:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_rth = None
_rtg = None


def rth():
    global _rth
    if _rth is None:
        path = os.path.join(LIB_DIR, "librth.so")
        if not os.path.exists(path):
            raise ImportError("librth.so not built (run raytracingrenderer_amd.build)")
        _rth = _bind(C.CDLL(path), RTH_EXPORTS)
    return _rth


def rtg():
    """The HIP library. Raises if missing: there is no CPU fallback for the render path."""
    global _rtg
    if _rtg is None:
        path = os.environ.get("RTG_LIB") or os.path.join(LIB_DIR, "librtg.so")  # RTG_LIB: A/B builds
        if not os.path.exists(path):
            raise ImportError("librtg.so not built (run raytracingrenderer_amd.build)")
        _rtg = _bind(C.CDLL(path, mode=C.RTLD_GLOBAL), RTG_EXPORTS)
    return _rtg


def ptr(arr, ctype):
    return arr.ctypes.data_as(C.POINTER(ctype))
