// rtg_rtbase.h — the reference-side binding of librtg: what an RTBase maintainer adds to the
// reference to render on the MI355X (INTEGRATION.md §2 shows this file; it is the compiled code).
//
// Include it after RTBase's own headers (Scene.h pulls in Geometry.h, Materials.h, Lights.h,
// Imaging.h) with include/ on the include path and link -lrtg. Three functions:
//
//   rtg_flatten_scene(scene, binding)   RTBase's built Scene (Scene.h:72-106, after Scene::build:
//                                       triangles in post-sort order, Scene::lights in reference
//                                       order) -> rtg_scene_desc, a copy: the vectors it points
//                                       into live in the binding
//   rtg_render_frame(gpu, film, seed)   RayTracer::render() (Renderer.h:876-885): film->SPP++, one
//                                       sample of every pixel queued on the GPU (up to three frames
//                                       run side by side; the call returns at once)
//   rtg_film_sync(gpu, film)            Film::film brought up to date (waits for the queued frames):
//                                       before saveHDR / savePNG / presentFilmToCanvas
//
// RayTracer::init (Renderer.h:45-63) then creates the handle once:
//     rtg_flatten_scene(scene, binding);
//     rtg_create(device, &binding.desc, &gpu);  rtg_set_options(gpu, MAX_DEPTH, RTG_OPT_CULL, 0);
// The sampler becomes rtg's PCG stream keyed (seed, pixel, sample):
// RTBase's MTRandom per thread is not reproducible (Renderer.h:55).
//
// In this repository it is compiled against /root/reference by oracle/ref/Makefile (into the
// test-only libref*.so) and tests/test_gpu_parity.py::test_reference_side_binding_renders_reference_film
// renders the reference loader's own Scene through it, bit-identical to the reference classes.
#pragma once
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

#include "rtg.h"

struct RtgSceneBinding {
    std::vector<float> pos, nrm, uv, nb;
    std::vector<uint32_t> mat;
    std::vector<int32_t> links, lights;
    std::vector<rtg_material> mats;
    std::vector<rtg_texture> texs;
    std::map<Texture*, int> texid;
    rtg_scene_desc desc{};
};

// The Lambert stubs (Conductor / Plastic / OrenNayar / Dielectric, Materials.h:203-465) all keep an
// `albedo` Texture*.
inline Texture* rtg_albedo_of(BSDF* b) {
    if (auto* c = dynamic_cast<ConductorBSDF*>(b)) return c->albedo;
    if (auto* p = dynamic_cast<PlasticBSDF*>(b)) return p->albedo;
    if (auto* o = dynamic_cast<OrenNayarBSDF*>(b)) return o->albedo;
    return dynamic_cast<DielectricBSDF*>(b)->albedo;
}

// BVHNode tree (Geometry.h:294-398) in DFS pre-order, root first.
inline void rtg_flatten_bvh(BVHNode* n, std::vector<BVHNode*>& out) {
    out.push_back(n);
    if (n->l) rtg_flatten_bvh(n->l, out);
    if (n->r) rtg_flatten_bvh(n->r, out);
}

inline void rtg_flatten_scene(Scene* s, RtgSceneBinding& b) {
    for (Triangle& t : s->triangles) {
        for (int k = 0; k < 3; k++) {
            b.pos.insert(b.pos.end(), {t.vertices[k].p.x, t.vertices[k].p.y, t.vertices[k].p.z});
            b.nrm.insert(b.nrm.end(), {t.vertices[k].normal.x, t.vertices[k].normal.y, t.vertices[k].normal.z});
            b.uv.insert(b.uv.end(), {t.vertices[k].u, t.vertices[k].v});
        }
        b.mat.push_back(t.materialIndex);
    }
    std::vector<BVHNode*> nodes;
    rtg_flatten_bvh(s->bvh, nodes);
    std::map<BVHNode*, int> id;
    for (size_t i = 0; i < nodes.size(); i++) id[nodes[i]] = (int)i;
    for (BVHNode* n : nodes) {
        b.nb.insert(b.nb.end(), {n->bounds.min.x, n->bounds.min.y, n->bounds.min.z,
                                 n->bounds.max.x, n->bounds.max.y, n->bounds.max.z});
        b.links.insert(b.links.end(), {n->l ? id[n->l] : -1, n->r ? id[n->r] : -1, n->startIndex, n->endIndex});
    }
    auto tex = [&](Texture* t) {  // Texture -> rtg_texture (Colour is three floats: same layout)
        auto it = b.texid.find(t);
        if (it != b.texid.end()) return it->second;
        b.texs.push_back({t->width, t->height, (const float*)t->texels});
        return b.texid[t] = (int)b.texs.size() - 1;
    };
    for (BSDF* m : s->materials) {
        rtg_material r{};
        r.two_sided = m->isTwoSided() ? 1 : 0;
        if (auto* g = dynamic_cast<GlassBSDF*>(m)) {
            r.kind = RTG_MAT_GLASS;
            r.texture = tex(g->albedo);
            r.int_ior = g->intIOR;
            r.ext_ior = g->extIOR;
        } else if (auto* mi = dynamic_cast<MirrorBSDF*>(m)) {
            r.kind = RTG_MAT_MIRROR;
            r.texture = tex(mi->albedo);
        } else if (auto* d = dynamic_cast<DiffuseBSDF*>(m)) {
            r.kind = RTG_MAT_DIFFUSE;
            r.texture = tex(d->albedo);
        } else {
            r.kind = RTG_MAT_LAMBERT;
            r.texture = tex(rtg_albedo_of(m));
        }
        r.emission[0] = m->emission.r;
        r.emission[1] = m->emission.g;
        r.emission[2] = m->emission.b;
        b.mats.push_back(r);
    }
    for (Light* l : s->lights) {  // the environment (lights[0] when its power > 0) is -1
        AreaLight* a = dynamic_cast<AreaLight*>(l);
        b.lights.push_back(a ? (int32_t)(a->triangle - s->triangles.data()) : -1);
    }
    rtg_scene_desc& d = b.desc;
    d.n_tris = (uint32_t)s->triangles.size();
    d.positions = b.pos.data();
    d.normals = b.nrm.data();
    d.uvs = b.uv.data();
    d.material = b.mat.data();
    d.n_nodes = (uint32_t)nodes.size();
    d.node_bounds = b.nb.data();
    d.node_links = b.links.data();
    EnvironmentMap* env = dynamic_cast<EnvironmentMap*>(s->background);
    d.env_texture = env ? tex(env->env) : -1;
    d.n_materials = (uint32_t)b.mats.size();
    d.materials = b.mats.data();
    d.n_textures = (uint32_t)b.texs.size();
    d.textures = b.texs.data();
    d.n_lights = (uint32_t)b.lights.size();
    d.lights = b.lights.data();
    Camera& c = s->camera;
    std::memcpy(d.camera.inv_proj, c.inverseProjectionMatrix.m, 64);
    std::memcpy(d.camera.camera, c.camera.m, 64);
    d.camera.origin[0] = c.origin.x;
    d.camera.origin[1] = c.origin.y;
    d.camera.origin[2] = c.origin.z;
    d.camera.width = c.width;
    d.camera.height = c.height;
    std::memcpy(d.projection.proj, c.projectionMatrix.m, 64);  // light tracing (ABI version 2)
    std::memcpy(d.projection.camera_to_view, c.cameraToView.m, 64);
    d.projection.view_direction[0] = c.viewDirection.x;
    d.projection.view_direction[1] = c.viewDirection.y;
    d.projection.view_direction[2] = c.viewDirection.z;
    d.projection.a_film = c.Afilm;
}

// RayTracer::render() (Renderer.h:876-885): one frame = one sample of every pixel, all tiles,
// queued (rtg_render_async): Main.cpp's loop (Main.cpp:74-118) reads the film only to save it.
inline int rtg_render_frame(rtg_handle* gpu, Film* film, uint64_t seed) {
    film->incrementSPP();
    return rtg_render_async(gpu, (uint32_t)film->SPP - 1, 1, seed, nullptr, 0, nullptr);
}

// Film::film of every frame queued so far (the read-back waits for them; 12 B per pixel).
inline int rtg_film_sync(rtg_handle* gpu, Film* film) {
    uint32_t spp = 0;
    return rtg_film_read(gpu, (float*)film->film, &spp);
}
