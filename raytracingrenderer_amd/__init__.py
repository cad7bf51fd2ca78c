"""raytracingrenderer_amd — MI355X-native wavefront path tracer with RTBase's host API.

The hot path (RayTracer::render) runs as HIP kernels in lib/librtg.so behind include/rtg.h;
scene loading / BVH build / HDR output run in lib/librth.so behind include/rth.h.
"""
from .renderer import (NativeError, RayTracer, RayTracerGroup, Scene, loadScene, read_hdr,  # noqa: F401
                       save_hdr, save_png, tonemap, write_synthetic_scene)

__all__ = ["RayTracer", "RayTracerGroup", "Scene", "loadScene", "save_hdr", "save_png", "tonemap", "read_hdr",
           "write_synthetic_scene", "NativeError"]
