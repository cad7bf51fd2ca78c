// ref_harness.cpp — TEST INFRASTRUCTURE ONLY (oracle/_ref). Builds RTBase's own code, compiled
// straight from /root/reference/RTBase (no copies, no stand-in headers), and exposes it through a
// C-ABI so tests/golden/make_golden.py can pin the product's host front-end and kernels:
//
//   compiled from the reference: Core.h (Matrix/Vec3/Frame), Geometry.h (Triangle::init,
//   rayIntersect, AABB, BVHNode::build/traverse/traverseVisible), Scene.h (Camera, Scene::build,
//   traverse, visible, calculateShadingData), Materials.h (all BSDFs), Lights.h, Imaging.h
//   (Texture::load via the vendored stb_image, Film), GEMLoader.h (JSON + .gem).
//
// NOT compilable here: Renderer.h and SceneLoader.h include the Windows/D3D11-only
// GamesEngineeringBase.h (windows.h, d3d11.h, XAudio2...). So loadScene's ~60-line glue
// (SceneLoader.h:104-291) is restated below using the reference classes, and so are the few lines
// of RayTracer::pathTrace / computeDirect / renderTile / pathTracerTileBased (Renderer.h:328-473,
// 795-853) in ref_render: every call they make (Scene::traverse, calculateShadingData,
// sampleLight, Light::sample, BSDF::sample/evaluate, Scene::visible, Camera::generateRay,
// Film::splat) is the reference's own compiled code. ref_render is a second, independent
// film-level pin of the C oracle and the "reference" CPU baseline of bench.py.
#include "GEMLoader.h"
#include "Scene.h"
#include "../../integration/rtg_rtbase.h"  // the reference-side binding

#include <sys/stat.h>

#include <atomic>
#include <cstdint>
#include <thread>
#include <map>
#include <string>
#include <vector>

namespace {

struct ScriptSampler : Sampler {
    const float* v;
    int n, i = 0;
    ScriptSampler(const float* vals, int count) : v(vals), n(count) {}
    float next() override { return i < n ? v[i++] : 0.5f; }
};

// PCG32 keyed by seq = pixel << 16 | sample, next() = (pcg32 >> 8) * 2^-24.
struct PcgSampler : Sampler {
    uint64_t state = 0, inc = 1;
    PcgSampler(uint64_t seed, uint64_t seq) {
        inc = (seq << 1u) | 1u;
        step();
        state += seed;
        step();
    }
    uint32_t step() {
        uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        uint32_t x = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (x >> rot) | (x << ((0u - rot) & 31u));
    }
    float next() override { return (float)(step() >> 8) * (1.0f / 16777216.0f); }
};

// windows.h min/max macros, as Renderer.h sees them
template <class T> inline T win_min(T a, T b) { return a < b ? a : b; }
template <class T> inline T win_max(T a, T b) { return a > b ? a : b; }

struct RayCount { uint64_t ext = 0, shadow = 0; };
const int MAX_DEPTH_REF = 4;  // Renderer.h:20 (the adaptive renderer uses the reference default)

// RayTracer::computeDirect (Renderer.h:423-473) on the reference classes
Colour ref_compute_direct(Scene* scene, ShadingData shadingData, Sampler& sampler, RayCount& rc) {
    if (shadingData.bsdf->isPureSpecular() == true) return Colour(0.0f, 0.0f, 0.0f);
    float pmf;
    Light* light = scene->sampleLight(sampler, pmf);
    float pdf;
    Colour emitted;
    Vec3 p = light->sample(shadingData, sampler, emitted, pdf);
    if (light->isArea()) {
        Vec3 wi = p - shadingData.x;
        float l = wi.lengthSq();
        wi = wi.normalize();
        float g = (win_max(Dot(wi, shadingData.sNormal), 0.0f) * win_max(-Dot(wi, light->normal(shadingData, wi)), 0.0f)) / l;
        if (g > 0) {
            rc.shadow++;
            if (scene->visible(shadingData.x, p)) return shadingData.bsdf->evaluate(shadingData, wi) * emitted * g / (pmf * pdf);
        }
    } else {
        Vec3 wi = p;
        float g = win_max(Dot(wi, shadingData.sNormal), 0.0f);
        if (g > 0) {
            rc.shadow++;
            if (scene->visible(shadingData.x, shadingData.x + (p * 10000.0f)))
                return shadingData.bsdf->evaluate(shadingData, wi) * emitted * g / (pmf * pdf);
        }
    }
    return Colour(0.0f, 0.0f, 0.0f);
}

// RayTracer::pathTrace (Renderer.h:328-392) with MAX_DEPTH as a parameter
Colour ref_path_trace(Scene* scene, Ray& r, Colour& thr, int depth, int max_depth, Sampler& sampler, bool canHitLight,
                      RayCount& rc) {
    rc.ext++;
    IntersectionData intersection = scene->traverse(r);
    ShadingData shadingData = scene->calculateShadingData(intersection, r);
    if (shadingData.t < FLT_MAX) {
        if (shadingData.bsdf->isLight()) {
            if (canHitLight == true) return thr * shadingData.bsdf->emit(shadingData, shadingData.wo);
            return Colour(0.0f, 0.0f, 0.0f);
        }
        Colour direct = thr * ref_compute_direct(scene, shadingData, sampler, rc);
        if (depth > max_depth) return direct;
        float rrp = win_min(thr.Lum(), 0.9f);
        if (sampler.next() < rrp) thr = thr / rrp;
        else return direct;
        Colour indirect;
        float pdf;
        Vec3 wi = shadingData.bsdf->sample(shadingData, sampler, indirect, pdf);
        if (shadingData.bsdf->isPureSpecular()) thr = thr * indirect / pdf;
        else thr = thr * indirect * fabsf(Dot(wi, shadingData.sNormal)) / pdf;
        r.init(shadingData.x + (wi * EPSILON), wi);
        return (direct + ref_path_trace(scene, r, thr, depth + 1, max_depth, sampler, shadingData.bsdf->isPureSpecular(), rc));
    }
    return scene->background->evaluate(r.dir);
}

float balance_heuristic(float a, float b) { return a / (a + b); }  // Renderer.h:408-411
float area_to_solid(float pdf_area, float dist2, float costheta) {  // Renderer.h:412-422
    if (costheta > 0.0f) return pdf_area * dist2 / costheta;
    return 0.0f;
}

// RayTracer::computeDirectMIS (Renderer.h:474-557)
Colour ref_compute_direct_mis(Scene* scene, ShadingData shadingData, Sampler& sampler, RayCount& rc) {
    if (shadingData.bsdf->isPureSpecular() == true) return Colour(0.0f, 0.0f, 0.0f);
    Colour result(0.0f, 0.0f, 0.0f);
    float pmf;
    Light* light = scene->sampleLight(sampler, pmf);
    float pdf;
    Colour emitted;
    Vec3 p = light->sample(shadingData, sampler, emitted, pdf);
    if (light->isArea()) {
        Vec3 wi = p - shadingData.x;
        float l = wi.lengthSq();
        wi = wi.normalize();
        float cos_surface = win_max(Dot(wi, shadingData.sNormal), 0.0f);
        float cos_light = win_max(-Dot(wi, light->normal(shadingData, wi)), 0.0f);
        float g = cos_surface * cos_light / l;
        if (g > 0) {
            rc.shadow++;
            if (scene->visible(shadingData.x, p)) {
                float pdf_bsdf = shadingData.bsdf->PDF(shadingData, wi);
                float pdf_light = area_to_solid(pdf * pmf, l, cos_light);
                float weight = balance_heuristic(pdf_light, pdf_bsdf);
                result = result + shadingData.bsdf->evaluate(shadingData, wi) * emitted * g * weight / (pmf * pdf);
            }
        }
    } else {
        Vec3 wi = p;
        float g = win_max(Dot(wi, shadingData.sNormal), 0.0f);
        if (g > 0) {
            rc.shadow++;
            if (scene->visible(shadingData.x, shadingData.x + (p * 10000.0f)))
                return shadingData.bsdf->evaluate(shadingData, wi) * emitted * g / (pmf * pdf);
        }
    }
    Colour val_bsdf;
    float pdf_bsdf;
    Vec3 wi_bsdf = shadingData.bsdf->sample(shadingData, sampler, val_bsdf, pdf_bsdf);
    Ray r = Ray(shadingData.x + (wi_bsdf * EPSILON), wi_bsdf);
    rc.ext++;
    IntersectionData intersection = scene->traverse(r);
    ShadingData hit = scene->calculateShadingData(intersection, r);
    if (hit.t < FLT_MAX) {
        if (hit.bsdf->isLight()) {
            Colour emitted2 = hit.bsdf->emit(hit, -wi_bsdf);
            Vec3 wi = hit.x - shadingData.x;
            float dist2 = wi.lengthSq();
            wi = wi.normalize();
            float cos_light = win_max(0.0f, Dot(-wi, hit.sNormal));
            float pdf_light = area_to_solid(pdf * pmf, dist2, cos_light);
            float weight = balance_heuristic(pdf_bsdf, pdf_light);
            result = result + val_bsdf * emitted2 * win_max(0.0f, Dot(wi_bsdf, shadingData.sNormal)) * weight / pdf_bsdf;
        }
    }
    return result;
}

// The per-pixel estimators of RayTracer (Renderer.h:393-407 direct, :558-571 albedo, :572-582
// viewNormals; mode 4 = direct() with computeDirectMIS); mode 0 is pathTrace.
Colour ref_estimate(Scene* scene, Ray& r, int mode, int max_depth, Sampler& sampler, RayCount& rc) {
    if (mode == 0) {
        Colour thr(1.0f, 1.0f, 1.0f);
        return ref_path_trace(scene, r, thr, 0, max_depth, sampler, true, rc);
    }
    rc.ext++;
    IntersectionData intersection = scene->traverse(r);
    if (mode == 3) {
        if (intersection.t < FLT_MAX) {
            ShadingData sd = scene->calculateShadingData(intersection, r);
            return Colour(fabsf(sd.sNormal.x), fabsf(sd.sNormal.y), fabsf(sd.sNormal.z));
        }
        return Colour(0.0f, 0.0f, 0.0f);
    }
    ShadingData sd = scene->calculateShadingData(intersection, r);
    if (sd.t < FLT_MAX) {
        if (sd.bsdf->isLight()) return sd.bsdf->emit(sd, sd.wo);
        if (mode == 2) return sd.bsdf->evaluate(sd, Vec3(0, 1, 0));
        return mode == 4 ? ref_compute_direct_mis(scene, sd, sampler, rc) : ref_compute_direct(scene, sd, sampler, rc);
    }
    if (mode == 2) return scene->background->evaluate(r.dir);
    return Colour(0.0f, 0.0f, 0.0f);
}

// ---- light tracing (Renderer.h:221-326), restated on the reference classes. `film` is the
// reference's Film; splats happen in path and vertex order (the reference's loop is sequential).
void ref_connect_to_camera(Scene* scene, Film& film, Vec3 p, Vec3 n, Colour col) {  // :236-262
    float x, y;
    if (scene->camera.projectOntoCamera(p, x, y)) {
        float A_film = scene->camera.Afilm;
        Vec3 direction = scene->camera.origin - p;
        float dist2 = direction.lengthSq();
        direction = direction.normalize();
        float cos_theta_shading = Dot(n, direction);
        float cos_theta_cam = Dot(scene->camera.viewDirection, -direction);
        if (cos_theta_shading < 0.0f || cos_theta_cam < 0.0f) return;
        float G = (cos_theta_shading * cos_theta_cam) / dist2;
        if (!scene->visible(p, scene->camera.origin)) return;
        float W_e = 1 / (A_film * SQ(SQ(cos_theta_cam)));
        Colour color = col * W_e * G;
        film.splat(x, y, color);
    }
}
void ref_light_trace_path(Scene* scene, Film& film, Ray& r, Colour thr, Colour Le, Sampler& sampler) {  // :292-326
    for (;;) {
        IntersectionData intersection = scene->traverse(r);
        ShadingData sd = scene->calculateShadingData(intersection, r);
        if (!(sd.t < FLT_MAX)) return;
        if (sd.bsdf->isLight() || sd.bsdf->isPureSpecular()) return;
        Vec3 wi = scene->camera.origin - sd.x;
        wi = wi.normalize();
        Colour col = thr * sd.bsdf->evaluate(sd, wi) * Le;
        ref_connect_to_camera(scene, film, sd.x, sd.sNormal, col);
        float rrp = win_min(thr.Lum(), 0.9f);
        if (sampler.next() < rrp) thr = thr / rrp;
        else return;
        Colour indirect;
        float pdf;
        Vec3 wi2 = sd.bsdf->sample(sd, sampler, indirect, pdf);
        thr = thr * indirect * fabsf(Dot(wi2, sd.sNormal)) / pdf;
        r.init(sd.x + (wi2 * EPSILON), wi2);
    }
}
void ref_light_trace_init(Scene* scene, Film& film, Sampler& sampler) {  // :264-291
    float pmf;
    Light* light = scene->sampleLight(sampler, pmf);
    if (!light->isArea()) return;
    float pdfPosition, pdfDirection;
    Vec3 p = light->samplePositionFromLight(sampler, pdfPosition);
    Vec3 wi = light->sampleDirectionFromLight(sampler, pdfDirection);
    ShadingData tmp;
    Vec3 lightNormal = light->normal(tmp, wi);
    float cosTheta = Dot(lightNormal, wi);
    Colour Le = light->evaluate(-wi) * cosTheta / (pmf * pdfDirection * pdfPosition);
    ref_connect_to_camera(scene, film, p, lightNormal, Le);
    Ray r = Ray(p, wi);
    ref_light_trace_path(scene, film, r, Colour(1.0f, 1.0f, 1.0f), Le, sampler);
}

// ---- instant radiosity (Renderer.h:82-218)
struct RefVpl { ShadingData shadingData; Colour Le; };
void ref_vpl_trace_path(Scene* scene, Ray& r, Colour thr, Colour Le, Sampler& sampler, std::vector<RefVpl>& vpls) {
    for (;;) {  // VPLTracePath, :183-218
        IntersectionData intersection = scene->traverse(r);
        ShadingData sd = scene->calculateShadingData(intersection, r);
        if (!(sd.t < FLT_MAX)) return;
        if (!sd.bsdf->isLight() && !sd.bsdf->isPureSpecular()) {
            RefVpl v;
            v.shadingData = sd;
            v.Le = thr * Le * sd.bsdf->evaluate(sd, -r.dir) * fabsf(Dot(-r.dir, sd.sNormal));
            vpls.push_back(v);
        }
        float rrp = win_min(thr.Lum(), 0.9f);
        if (sampler.next() < rrp) thr = thr / rrp;
        else return;
        Colour bsdfVal;
        float pdf;
        Vec3 wi = sd.bsdf->sample(sd, sampler, bsdfVal, pdf);
        thr = thr * bsdfVal * fabsf(Dot(wi, sd.sNormal)) / pdf;
        r.init(sd.x + (wi * EPSILON), wi);
    }
}
Colour ref_vpl_contribution(Scene* scene, ShadingData sd, const std::vector<RefVpl>& vpls) {  // :122-154
    if (sd.bsdf->isLight() || sd.bsdf->isPureSpecular()) return Colour(0.0f, 0.0f, 0.0f);
    Colour col_sum(0.0f, 0.0f, 0.0f);
    for (const RefVpl& vpl : vpls) {
        Vec3 direction = vpl.shadingData.x - sd.x;
        float dist2 = direction.lengthSq();
        if (dist2 < 1e-4f) continue;
        direction = direction.normalize();
        float cos_theta_vpl = Dot(vpl.shadingData.sNormal, -direction);
        float cos_theta_x = Dot(sd.sNormal, direction);
        if (cos_theta_vpl <= 0.0f || cos_theta_x <= 0.0f) continue;
        float G = (cos_theta_vpl * cos_theta_x) / dist2;
        if (!scene->visible(sd.x, vpl.shadingData.x)) continue;
        Colour bsdf = sd.bsdf->evaluate(sd, direction);
        Colour col = vpl.Le * bsdf * G;
        col_sum = col_sum + col;
    }
    return col_sum;
}

bool exists(const std::string& p) {
    struct stat st;
    return ::stat(p.c_str(), &st) == 0;
}

Texture* load_tex(const std::string& fn, std::map<std::string, Texture*>& cache, std::vector<std::string>& names) {
    auto it = cache.find(fn);
    if (it != cache.end()) return it->second;
    Texture* t = new Texture();
    t->load(fn);
    cache.insert({fn, t});
    names.push_back(fn);
    return t;
}

struct RefScene {
    Scene* scene = nullptr;
    std::vector<Texture*> textures;        // in first-use order
    std::map<Texture*, int> tex_index;
    std::vector<int> mat_kind, mat_two_sided, mat_tex;
    std::vector<float> mat_ior;             // int, ext
    int env_tex = -1;
    RtgSceneBinding* binding = nullptr;     // rtg_flatten_scene's output (built on first use)
};

// SceneLoader.h:104-235 restated on the reference classes.
void load_instance(const std::string& dir, std::vector<Triangle>& tris, std::vector<BSDF*>& mats,
                   GEMLoader::GEMInstance& inst, std::map<std::string, Texture*>& cache,
                   std::vector<std::string>& names, bool skip_missing) {
    if (skip_missing && (!exists(dir + "/" + inst.meshFilename) ||
                         !exists(dir + "/" + inst.material.find("reflectance").getValue("")))) return;
    GEMLoader::GEMModelLoader loader;
    std::vector<GEMLoader::GEMMesh> meshes;
    loader.load(dir + "/" + inst.meshFilename, meshes);
    BSDF* material = NULL;
    std::string bsdf = inst.material.find("bsdf").getValue("");
    std::string fn = dir + "/" + inst.material.find("reflectance").getValue("");
    if (bsdf == "diffuse") material = new DiffuseBSDF(load_tex(fn, cache, names));
    if (bsdf == "orennayar") material = new OrenNayarBSDF(load_tex(fn, cache, names), inst.material.find("alpha").getValue(1.0f));
    if (bsdf == "glass") material = new GlassBSDF(load_tex(fn, cache, names), inst.material.find("intIOR").getValue(1.33f), inst.material.find("extIOR").getValue(1.0f));
    if (bsdf == "mirror") material = new MirrorBSDF(load_tex(fn, cache, names));
    if (bsdf == "plastic") material = new PlasticBSDF(load_tex(fn, cache, names), inst.material.find("intIOR").getValue(1.33f), inst.material.find("extIOR").getValue(1.0f), inst.material.find("roughness").getValue(1.0f));
    if (bsdf == "dielectric") {
        float rough = inst.material.find("roughness").getValue(1.0f);
        if (rough < 0.001f) material = new GlassBSDF(load_tex(fn, cache, names), inst.material.find("intIOR").getValue(1.33f), inst.material.find("extIOR").getValue(1.0f));
        else material = new DielectricBSDF(load_tex(fn, cache, names), inst.material.find("intIOR").getValue(1.33f), inst.material.find("extIOR").getValue(1.0f), rough);
    }
    if (bsdf == "conductor") {
        Colour eta, k;
        inst.material.find("eta").getValuesAsVector3(eta.r, eta.g, eta.b);
        inst.material.find("k").getValuesAsVector3(k.r, k.g, k.b);
        material = new ConductorBSDF(load_tex(fn, cache, names), eta, k, inst.material.find("roughness").getValue(1.0f));
    }
    if (material == NULL) return;
    mats.push_back(material);
    if (inst.material.find("emission").getValue("") != "") {
        Colour e;
        inst.material.find("emission").getValuesAsVector3(e.r, e.g, e.b);
        material->addLight(e);
    }
    int mi = (int)mats.size() - 1;
    std::vector<Vertex> verts;
    std::vector<unsigned int> idx;
    Matrix transform;
    memcpy(transform.m, inst.w.m, 16 * sizeof(float));
    Matrix vt = transform.invert();
    vt = vt.transpose();
    for (size_t i = 0; i < meshes.size(); i++) {
        for (size_t n = 0; n < meshes[i].verticesStatic.size(); n++) {
            Vertex v;
            const auto& g = meshes[i].verticesStatic[n];
            v.p = Vec3(g.position.x, g.position.y, g.position.z);
            v.normal = Vec3(g.normal.x, g.normal.y, g.normal.z);
            v.p = transform.mulPoint(v.p);
            v.normal = vt.mulVec(v.normal);
            v.normal = v.normal.normalize();
            v.u = g.u;
            v.v = g.v;
            verts.push_back(v);
        }
        int offset = (int)idx.size();
        for (size_t n = 0; n < meshes[i].indices.size(); n++) idx.push_back(offset + meshes[i].indices[n]);
    }
    for (size_t i = 0; i + 2 < idx.size(); i += 3) {
        Triangle t;
        t.init(verts[idx[i]], verts[idx[i + 1]], verts[idx[i + 2]], mi);
        if (t.area > 0) tris.push_back(t);
    }
}

void flatten(BVHNode* n, std::vector<BVHNode*>& out) {
    out.push_back(n);
    if (n->l) flatten(n->l, out);
    if (n->r) flatten(n->r, out);
}

}  // namespace

extern "C" {

void* ref_load(const char* dir_c, int W, int H, int skip_missing, const char* env_override) {
    std::string dir(dir_c);
    GEMLoader::GEMScene gs;
    gs.load(dir + "/scene.json");
    int width = gs.findProperty("width").getValue(1920);
    int height = gs.findProperty("height").getValue(1080);
    if (W > 0) width = W;
    if (H > 0) height = H;
    float fov = gs.findProperty("fov").getValue(45.0f);
    Matrix P = Matrix::perspective(0.001f, 10000.0f, (float)width / (float)height, fov);
    Vec3 from, to, up;
    gs.findProperty("from").getValuesAsVector3(from.x, from.y, from.z);
    gs.findProperty("to").getValuesAsVector3(to.x, to.y, to.z);
    gs.findProperty("up").getValuesAsVector3(up.x, up.y, up.z);
    Matrix V = Matrix::lookAt(from, to, up);
    V = V.invert();
    if (gs.findProperty("flipX").getValue(0) == 1) P.a[0][0] = -P.a[0][0];
    RefScene* rs = new RefScene();
    rs->scene = new Scene();
    rs->scene->camera.init(P, width, height);
    rs->scene->camera.updateView(V);
    std::vector<Triangle> tris;
    std::vector<BSDF*> mats;
    std::map<std::string, Texture*> cache;
    std::vector<std::string> names;
    for (size_t i = 0; i < gs.instances.size(); i++)
        load_instance(dir, tris, mats, gs.instances[i], cache, names, skip_missing != 0);
    std::string env = env_override ? std::string(env_override) : gs.findProperty("envmap").getValue("");
    Light* bg;
    Texture* envt = nullptr;
    if (env != "") {
        envt = load_tex(dir + "/" + env, cache, names);
        bg = new EnvironmentMap(envt);
    } else {
        bg = new BackgroundColour(Colour(0.0f, 0.0f, 0.0f));
    }
    rs->scene->init(tris, mats, bg);
    rs->scene->build();
    for (const auto& n : names) {
        rs->tex_index[cache[n]] = (int)rs->textures.size();
        rs->textures.push_back(cache[n]);
    }
    rs->env_tex = envt ? rs->tex_index[envt] : -1;
    for (BSDF* b : rs->scene->materials) {
        int kind = 1, tex = -1;
        float ii = 0, ee = 0;
        if (auto* d = dynamic_cast<DiffuseBSDF*>(b)) { kind = 0; tex = rs->tex_index[d->albedo]; }
        else if (auto* m = dynamic_cast<MirrorBSDF*>(b)) { kind = 2; tex = rs->tex_index[m->albedo]; }
        else if (auto* g = dynamic_cast<GlassBSDF*>(b)) { kind = 3; tex = rs->tex_index[g->albedo]; ii = g->intIOR; ee = g->extIOR; }
        else if (auto* c = dynamic_cast<ConductorBSDF*>(b)) tex = rs->tex_index[c->albedo];
        else if (auto* p = dynamic_cast<PlasticBSDF*>(b)) tex = rs->tex_index[p->albedo];
        else if (auto* o = dynamic_cast<OrenNayarBSDF*>(b)) tex = rs->tex_index[o->albedo];
        else if (auto* e = dynamic_cast<DielectricBSDF*>(b)) tex = rs->tex_index[e->albedo];
        rs->mat_kind.push_back(kind);
        rs->mat_two_sided.push_back(b->isTwoSided() ? 1 : 0);
        rs->mat_tex.push_back(tex);
        rs->mat_ior.push_back(ii);
        rs->mat_ior.push_back(ee);
    }
    return rs;
}

// counts: ntri, nnodes, nlights, nmats, ntex, env_tex, width, height
void ref_counts(void* h, int* out) {
    RefScene* rs = (RefScene*)h;
    std::vector<BVHNode*> nodes;
    flatten(rs->scene->bvh, nodes);
    out[0] = (int)rs->scene->triangles.size();
    out[1] = (int)nodes.size();
    out[2] = (int)rs->scene->lights.size();
    out[3] = (int)rs->scene->materials.size();
    out[4] = (int)rs->textures.size();
    out[5] = rs->env_tex;
    out[6] = (int)rs->scene->camera.width;
    out[7] = (int)rs->scene->camera.height;
}

// Export the built Scene in the layout of include/rtg.h's rtg_scene_desc.
void ref_export(void* h, float* pos, float* nrm, float* uv, uint32_t* mat, float* nb, int32_t* nl, int32_t* lights,
                float* cam /* 16 invP + 16 camera + 3 origin + 2 size */, int32_t* mat_info /* kind, two_sided, tex */,
                float* mat_f /* int_ior, ext_ior, emission rgb */) {
    RefScene* rs = (RefScene*)h;
    Scene* s = rs->scene;
    for (size_t i = 0; i < s->triangles.size(); i++) {
        const Triangle& t = s->triangles[i];
        for (int k = 0; k < 3; k++) {
            pos[i * 9 + k * 3 + 0] = t.vertices[k].p.x;
            pos[i * 9 + k * 3 + 1] = t.vertices[k].p.y;
            pos[i * 9 + k * 3 + 2] = t.vertices[k].p.z;
            nrm[i * 9 + k * 3 + 0] = t.vertices[k].normal.x;
            nrm[i * 9 + k * 3 + 1] = t.vertices[k].normal.y;
            nrm[i * 9 + k * 3 + 2] = t.vertices[k].normal.z;
            uv[i * 6 + k * 2 + 0] = t.vertices[k].u;
            uv[i * 6 + k * 2 + 1] = t.vertices[k].v;
        }
        mat[i] = t.materialIndex;
    }
    std::vector<BVHNode*> nodes;
    flatten(s->bvh, nodes);
    std::map<BVHNode*, int> id;
    for (size_t i = 0; i < nodes.size(); i++) id[nodes[i]] = (int)i;
    for (size_t i = 0; i < nodes.size(); i++) {
        BVHNode* n = nodes[i];
        nb[i * 6 + 0] = n->bounds.min.x; nb[i * 6 + 1] = n->bounds.min.y; nb[i * 6 + 2] = n->bounds.min.z;
        nb[i * 6 + 3] = n->bounds.max.x; nb[i * 6 + 4] = n->bounds.max.y; nb[i * 6 + 5] = n->bounds.max.z;
        nl[i * 4 + 0] = n->l ? id[n->l] : -1;
        nl[i * 4 + 1] = n->r ? id[n->r] : -1;
        nl[i * 4 + 2] = n->l ? 0 : n->startIndex;
        nl[i * 4 + 3] = n->l ? 0 : n->endIndex;
    }
    for (size_t i = 0; i < s->lights.size(); i++) {
        AreaLight* a = dynamic_cast<AreaLight*>(s->lights[i]);
        lights[i] = a ? (int32_t)(a->triangle - s->triangles.data()) : -1;
    }
    memcpy(cam, s->camera.inverseProjectionMatrix.m, 64);
    memcpy(cam + 16, s->camera.camera.m, 64);
    cam[32] = s->camera.origin.x; cam[33] = s->camera.origin.y; cam[34] = s->camera.origin.z;
    cam[35] = s->camera.width; cam[36] = s->camera.height;
    for (size_t i = 0; i < s->materials.size(); i++) {
        mat_info[i * 3 + 0] = rs->mat_kind[i];
        mat_info[i * 3 + 1] = rs->mat_two_sided[i];
        mat_info[i * 3 + 2] = rs->mat_tex[i];
        mat_f[i * 5 + 0] = rs->mat_ior[i * 2];
        mat_f[i * 5 + 1] = rs->mat_ior[i * 2 + 1];
        mat_f[i * 5 + 2] = s->materials[i]->emission.r;
        mat_f[i * 5 + 3] = s->materials[i]->emission.g;
        mat_f[i * 5 + 4] = s->materials[i]->emission.b;
    }
}

// The reference-side binding (integration/rtg_rtbase.h) applied to this Scene: the rtg_scene_desc
// an RTBase host hands to rtg_create. Owned by the scene handle.
const rtg_scene_desc* ref_rtg_desc(void* h) {
    RefScene* rs = (RefScene*)h;
    if (!rs->binding) {
        rs->binding = new RtgSceneBinding();
        rtg_flatten_scene(rs->scene, *rs->binding);
    }
    return &rs->binding->desc;
}

void ref_texture_size(void* h, int i, int* wh) {
    RefScene* rs = (RefScene*)h;
    wh[0] = rs->textures[i]->width;
    wh[1] = rs->textures[i]->height;
}
void ref_texture_texels(void* h, int i, float* out) {
    RefScene* rs = (RefScene*)h;
    Texture* t = rs->textures[i];
    for (int k = 0; k < t->width * t->height; k++) {
        out[k * 3] = t->texels[k].r; out[k * 3 + 1] = t->texels[k].g; out[k * 3 + 2] = t->texels[k].b;
    }
}

// Scene::traverse over n rays (o.xyz, pad, dir.xyz, pad) -> (t, id bits, alpha, beta); id -1 on miss.
void ref_traverse(void* h, const float* rays, int n, float* out) {
    Scene* s = ((RefScene*)h)->scene;
    for (int i = 0; i < n; i++) {
        const float* r = rays + i * 8;
        Ray ray(Vec3(r[0], r[1], r[2]), Vec3(r[4], r[5], r[6]));
        IntersectionData is = s->traverse(ray);
        int id = is.t < FLT_MAX ? (int)is.ID : -1;
        out[i * 4] = is.t;
        memcpy(&out[i * 4 + 1], &id, 4);
        out[i * 4 + 2] = is.t < FLT_MAX ? is.alpha : 0.0f;
        out[i * 4 + 3] = is.t < FLT_MAX ? is.beta : 0.0f;
    }
}

// BVHNode::traverseVisible with an explicit (o, dir, maxT) ray: (o.xyz, maxT, dir.xyz, pad).
void ref_traverse_visible(void* h, const float* rays, int n, int32_t* out) {
    Scene* s = ((RefScene*)h)->scene;
    for (int i = 0; i < n; i++) {
        const float* r = rays + i * 8;
        Ray ray(Vec3(r[0], r[1], r[2]), Vec3(r[4], r[5], r[6]));
        out[i] = s->bvh->traverseVisible(ray, s->triangles, r[3]) ? 1 : 0;
    }
}

// Scene::visible(p1, p2): pairs (p1.xyz, p2.xyz).
void ref_visible(void* h, const float* pairs, int n, int32_t* out) {
    Scene* s = ((RefScene*)h)->scene;
    for (int i = 0; i < n; i++) {
        const float* p = pairs + i * 6;
        out[i] = s->visible(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5])) ? 1 : 0;
    }
}

// Camera::generateRay at pixel centres: out (o.xyz, dir.xyz).
void ref_camera_rays(void* h, const uint32_t* pixels, int n, float* out) {
    Scene* s = ((RefScene*)h)->scene;
    uint32_t W = (uint32_t)s->camera.width;
    for (int i = 0; i < n; i++) {
        float px = (pixels[i] % W) + 0.5f, py = (pixels[i] / W) + 0.5f;
        Ray r = s->camera.generateRay(px, py);
        out[i * 6] = r.o.x; out[i * 6 + 1] = r.o.y; out[i * 6 + 2] = r.o.z;
        out[i * 6 + 3] = r.dir.x; out[i * 6 + 4] = r.dir.y; out[i * 6 + 5] = r.dir.z;
    }
}

// BSDF::sample on a standalone material with a scripted sampler.
// kind: 0 diffuse, 1 conductor stub, 2 mirror, 3 glass(int_ior, ext_ior), 4 plastic, 5 orennayar, 6 dielectric
// albedo: 1x1 texture colour. sd: sNormal.xyz, wo.xyz, tu, tv. Returns wi.xyz, refl.rgb, pdf, draws used.
void ref_bsdf_sample(int kind, const float* albedo, float int_ior, float ext_ior, const float* sd,
                     const float* draws, int ndraws, float* out) {
    Texture tex;
    tex.alpha = NULL;
    tex.width = 1;
    tex.height = 1;
    tex.channels = 3;
    tex.texels = new Colour[1];
    tex.texels[0] = Colour(albedo[0], albedo[1], albedo[2]);
    BSDF* b = nullptr;
    switch (kind) {
    case 0: b = new DiffuseBSDF(&tex); break;
    case 1: b = new ConductorBSDF(&tex, Colour(1, 1, 1), Colour(1, 1, 1), 0.5f); break;
    case 2: b = new MirrorBSDF(&tex); break;
    case 3: b = new GlassBSDF(&tex, int_ior, ext_ior); break;
    case 4: b = new PlasticBSDF(&tex, int_ior, ext_ior, 0.5f); break;
    case 5: b = new OrenNayarBSDF(&tex, 0.5f); break;
    default: b = new DielectricBSDF(&tex, int_ior, ext_ior, 0.5f); break;
    }
    ShadingData s(Vec3(0, 0, 0), Vec3(sd[0], sd[1], sd[2]));
    s.wo = Vec3(sd[3], sd[4], sd[5]);
    s.tu = sd[6];
    s.tv = sd[7];
    s.bsdf = b;
    s.frame.fromVector(s.sNormal);
    ScriptSampler smp(draws, ndraws);
    Colour refl;
    float pdf = 0;
    Vec3 wi = b->sample(s, smp, refl, pdf);
    Colour ev = b->evaluate(s, wi);
    out[0] = wi.x; out[1] = wi.y; out[2] = wi.z;
    out[3] = refl.r; out[4] = refl.g; out[5] = refl.b;
    out[6] = pdf;
    out[7] = (float)smp.i;
    out[8] = ev.r; out[9] = ev.g; out[10] = ev.b;
    delete b;
}

// EnvironmentMap::evaluate and ::sample of texture i of a loaded scene.
void ref_env_eval(void* h, int tex, const float* dirs, int n, float* out) {
    RefScene* rs = (RefScene*)h;
    EnvironmentMap env(rs->textures[tex]);
    for (int i = 0; i < n; i++) {
        Colour c = env.evaluate(Vec3(dirs[i * 3], dirs[i * 3 + 1], dirs[i * 3 + 2]));
        out[i * 3] = c.r; out[i * 3 + 1] = c.g; out[i * 3 + 2] = c.b;
    }
}

// Texture::sample of texture i.
void ref_tex_sample(void* h, int tex, const float* uv, int n, float* out) {
    RefScene* rs = (RefScene*)h;
    for (int i = 0; i < n; i++) {
        Colour c = rs->textures[tex]->sample(uv[i * 2], uv[i * 2 + 1]);
        out[i * 3] = c.r; out[i * 3 + 1] = c.g; out[i * 3 + 2] = c.b;
    }
}

// Film::save through the vendored stb_image_write (RGBE bytes).
int ref_save_hdr(const char* path, int w, int h, const float* sum, int spp) {
    Film f;
    f.init(w, h, new BoxFilter());
    memcpy(f.film, sum, (size_t)w * h * 12);
    f.SPP = spp;
    f.save(path);
    return 0;
}

// RayTracer::render x n_samples (Renderer.h:876-885 -> pathTracerTileBased / getTileID /
// renderTile, :795-853): per frame, `threads` std::threads pop 32x32 tiles from a shared counter
// and splat every pixel's pathTrace radiance into the reference's Film (box filter). The film sum
// (w*h*3, in/out) and the deterministic sampler replace MTRandom. counts (optional, 3): paths,
// closest-hit rays, shadow rays.
int ref_render_mode(void* h, uint32_t first, uint32_t n_samples, uint64_t seed, int max_depth, int threads, float* sum,
                    uint64_t* counts, int mode) {
    RefScene* rs = (RefScene*)h;
    Scene* scene = rs->scene;
    const int W = (int)scene->camera.width, H = (int)scene->camera.height, TS = 32;
    Film film;
    film.init(W, H, new BoxFilter());
    memcpy(film.film, sum, (size_t)W * H * 12);
    const int tx = (W + TS - 1) / TS, ty = (H + TS - 1) / TS;
    if (threads < 1) threads = 1;
    std::vector<RayCount> rcs(threads);
    for (uint32_t smp = first; smp < first + n_samples; ++smp) {
        std::atomic<int> next(0);
        auto worker = [&](int tid) {
            for (;;) {
                int t = next.fetch_add(1);
                if (t >= tx * ty) break;
                int x0 = (t % tx) * TS, y0 = (t / tx) * TS;
                int x1 = win_min(x0 + TS, W), y1 = win_min(y0 + TS, H);
                for (int y = y0; y < y1; y++)
                    for (int x = x0; x < x1; x++) {
                        float px = x + 0.5f, py = y + 0.5f;
                        PcgSampler sampler(seed, ((uint64_t)(y * W + x) << 16) | smp);
                        Ray ray = scene->camera.generateRay(px, py);
                        Colour col = ref_estimate(scene, ray, mode, max_depth, sampler, rcs[tid]);
                        film.splat(px, py, col);
                    }
            }
        };
        std::vector<std::thread> pool;
        for (int i = 0; i < threads; i++) pool.emplace_back(worker, i);
        for (auto& t : pool) t.join();
    }
    memcpy(sum, film.film, (size_t)W * H * 12);
    if (counts) {
        counts[0] = (uint64_t)W * H * n_samples;
        counts[1] = counts[2] = 0;
        for (auto& c : rcs) { counts[1] += c.ext; counts[2] += c.shadow; }
    }
    return 0;
}

int ref_render(void* h, uint32_t first, uint32_t n_samples, uint64_t seed, int max_depth, int threads, float* sum,
               uint64_t* counts) {
    return ref_render_mode(h, first, n_samples, seed, max_depth, threads, sum, counts, 0);
}

// RayTracer::lightTracer (Renderer.h:221-235): width*height light paths per frame, path i of frame f
// drawing from the PCG stream keyed (seed, i << 16 | f) (the GPU build's convention).
int ref_render_light(void* h, uint32_t first, uint32_t n_frames, uint64_t seed, float* sum) {
    Scene* scene = ((RefScene*)h)->scene;
    const int W = (int)scene->camera.width, H = (int)scene->camera.height;
    Film film;
    film.init(W, H, new BoxFilter());
    memcpy(film.film, sum, (size_t)W * H * 12);
    for (uint32_t f = first; f < first + n_frames; ++f)
        for (uint32_t i = 0; i < (uint32_t)(W * H); ++i) {
            PcgSampler sampler(seed, ((uint64_t)i << 16) | f);
            ref_light_trace_init(scene, film, sampler);
        }
    memcpy(sum, film.film, (size_t)W * H * 12);
    return 0;
}

// RayTracer::instantRadiosity (Renderer.h:101-121): traceVPLs (n_vpl paths, path i keyed (seed,
// i << 16 | f)), then every pixel's first hit gathers the VPLs (renderBlockinstantRadiosity).
int ref_render_ir(void* h, uint32_t first, uint32_t n_frames, uint64_t seed, uint32_t n_vpl, float* sum) {
    Scene* scene = ((RefScene*)h)->scene;
    const int W = (int)scene->camera.width, H = (int)scene->camera.height;
    Film film;
    film.init(W, H, new BoxFilter());
    memcpy(film.film, sum, (size_t)W * H * 12);
    for (uint32_t f = first; f < first + n_frames; ++f) {
        std::vector<RefVpl> vpls;
        for (uint32_t i = 0; i < n_vpl; ++i) {  // traceVPLs, :156-182
            PcgSampler sampler(seed, ((uint64_t)i << 16) | f);
            float pmf;
            Light* light = scene->sampleLight(sampler, pmf);
            if (!light->isArea()) continue;
            float pdfPosition, pdfDirection;
            Vec3 p = light->samplePositionFromLight(sampler, pdfPosition);
            Vec3 wi = light->sampleDirectionFromLight(sampler, pdfDirection);
            RefVpl v;
            ShadingData tmp;
            v.shadingData = ShadingData(p, light->normal(tmp, p));
            v.Le = light->evaluate(-wi) / (pmf * pdfPosition * (float)n_vpl);
            vpls.push_back(v);
            Colour Le = light->evaluate(-wi) * Dot(wi, light->normal(tmp, p)) / (pmf * pdfPosition * (float)n_vpl);
            Ray r = Ray(p, wi);
            ref_vpl_trace_path(scene, r, Colour(1.0f, 1.0f, 1.0f), Le, sampler, vpls);
        }
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) {
                Ray r = scene->camera.generateRay(x + 0.5f, y + 0.5f);
                IntersectionData intersection = scene->traverse(r);
                ShadingData sd = scene->calculateShadingData(intersection, r);
                if (sd.t < FLT_MAX) film.splat((float)x, (float)y, ref_vpl_contribution(scene, sd, vpls));
            }
    }
    memcpy(sum, film.film, (size_t)W * H * 12);
    return 0;
}

// RayTracer::adaptiveRender (Renderer.h:583-749): adaptiveSampling per tile (init samples per pixel,
// variance of the per-pixel means), weights = variance / total, sampleTileWithWeight. Sample
// indices: pass 1 first .. first+init-1, pass 2 first+init ... (the GPU build's convention).
int ref_render_adaptive(void* h, uint32_t first, uint64_t seed, uint32_t init, uint32_t max_samples,
                        uint32_t min_samples, float* sum, uint32_t* tile_samples) {
    Scene* scene = ((RefScene*)h)->scene;
    const int W = (int)scene->camera.width, H = (int)scene->camera.height, TS = 32;
    const int tx = (W + TS - 1) / TS, ty = (H + TS - 1) / TS;
    Film film;
    film.init(W, H, new BoxFilter());
    memcpy(film.film, sum, (size_t)W * H * 12);
    RayCount rc;
    std::vector<float> var(tx * ty);
    for (int t = 0; t < tx * ty; ++t) {  // adaptiveSampling, :583-638
        int startX = (t % tx) * TS, startY = (t / tx) * TS;
        int endX = win_min(startX + TS, W), endY = win_min(startY + TS, H);
        std::vector<Colour> est((endX - startX) * (endY - startY), Colour(0.0f, 0.0f, 0.0f));
        int pixelIndex = 0;
        for (int y = startY; y < endY; y++)
            for (int x = startX; x < endX; x++) {
                Colour s0(0.0f, 0.0f, 0.0f);
                for (uint32_t i = 0; i < init; i++) {
                    PcgSampler sampler(seed, ((uint64_t)(y * W + x) << 16) | (first + i));
                    Ray ray = scene->camera.generateRay(x + 0.5f, y + 0.5f);
                    Colour thr(1.0f, 1.0f, 1.0f);
                    s0 = s0 + ref_path_trace(scene, ray, thr, 0, MAX_DEPTH_REF, sampler, true, rc);
                }
                est[pixelIndex++] = s0 / (float)init;
            }
        Colour es(0.0f, 0.0f, 0.0f);
        for (size_t i = 0; i < est.size(); i++) es = es + est[i];
        Colour gt = es / (float)pixelIndex;
        Colour sq(0.0f, 0.0f, 0.0f);
        for (size_t i = 0; i < est.size(); i++) {
            Colour tmp = est[i] - gt;
            sq = sq + tmp * tmp;
        }
        var[t] = ((sq.r + sq.g + sq.b) / 3.0f) / (float)(pixelIndex - 1);
    }
    float total = 0.0f;
    for (float v : var) total += v;
    for (int t = 0; t < tx * ty; ++t) {  // sampleTileWithWeight, :640-672
        float weight = (total > 0.0f) ? var[t] / total : 0.0f;
        weight = sqrt(weight);
        int sample = (int)(weight * max_samples);
        sample = win_max(sample, (int)min_samples);
        if (tile_samples) tile_samples[t] = (uint32_t)sample;
        int startX = (t % tx) * TS, startY = (t / tx) * TS;
        int endX = win_min(startX + TS, W), endY = win_min(startY + TS, H);
        for (int y = startY; y < endY; y++)
            for (int x = startX; x < endX; x++) {
                float px = x + 0.5f, py = y + 0.5f;
                Colour col(0.0f, 0.0f, 0.0f);
                for (int i = 0; i < sample; i++) {
                    PcgSampler sampler(seed, ((uint64_t)(y * W + x) << 16) | (first + init + (uint32_t)i));
                    Ray ray = scene->camera.generateRay(px, py);
                    Colour thr(1.0f, 1.0f, 1.0f);
                    col = col + ref_path_trace(scene, ray, thr, 0, MAX_DEPTH_REF, sampler, true, rc);
                }
                col = col / (float)sample;
                film.splat(px, py, col);
            }
    }
    memcpy(sum, film.film, (size_t)W * H * 12);
    return 0;
}

// Film::tonemap (Imaging.h:233-242) of every pixel of a w*h film sum: out w*h*3 bytes.
void ref_tonemap(int w, int h, const float* sum, int spp, float exposure, unsigned char* out) {
    Film f;
    f.init(w, h, new BoxFilter());
    memcpy(f.film, sum, (size_t)w * h * 12);
    f.SPP = spp;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            unsigned char* o = out + ((size_t)y * w + x) * 3;
            f.tonemap(x, y, o[0], o[1], o[2], exposure);
        }
}

// stbi_loadf / stbi_load as Texture::load sees them.
int ref_load_texture(const char* path, float* out, int cap, int* wh) {
    Texture t;
    t.width = 0;
    t.height = 0;
    t.load(path);
    wh[0] = t.width;
    wh[1] = t.height;
    int n = t.width * t.height;
    for (int k = 0; k < n && k * 3 + 2 < cap; k++) {
        out[k * 3] = t.texels[k].r; out[k * 3 + 1] = t.texels[k].g; out[k * 3 + 2] = t.texels[k].b;
    }
    return n;
}

// Camera::projectOntoCamera (Scene.h:55-69) on points (xyz): out (ok, x, y) per point; state =
// projectionMatrix[16], cameraToView[16], viewDirection[3], Afilm (the members light tracing uses).
void ref_camera_project(void* h, const float* pts, int n, float* out, float* state) {
    Camera& c = ((RefScene*)h)->scene->camera;
    for (int i = 0; i < n; i++) {
        float x = 0, y = 0;
        bool ok = c.projectOntoCamera(Vec3(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]), x, y);
        out[3 * i] = ok ? 1.0f : 0.0f;
        out[3 * i + 1] = x;
        out[3 * i + 2] = y;
    }
    memcpy(state, c.projectionMatrix.m, 64);
    memcpy(state + 16, c.cameraToView.m, 64);
    state[32] = c.viewDirection.x; state[33] = c.viewDirection.y; state[34] = c.viewDirection.z;
    state[35] = c.Afilm;
}

// AreaLight samplePositionFromLight + sampleDirectionFromLight + evaluate(-wi) (Lights.h:30-80) for
// Scene::lights[li] with scripted draws: out = p.xyz, pdfPosition, wi.xyz, pdfDirection, Le.rgb,
// draws used (lightTrace_init, Renderer.h:264-281).
void ref_light_emit(void* h, int li, const float* draws, int ndraws, float* out) {
    Light* L = ((RefScene*)h)->scene->lights[li];
    ScriptSampler smp(draws, ndraws);
    float pp = 0, pd = 0;
    Vec3 p = L->samplePositionFromLight(smp, pp);
    Vec3 wi = L->sampleDirectionFromLight(smp, pd);
    Colour e = L->evaluate(-wi);
    out[0] = p.x; out[1] = p.y; out[2] = p.z; out[3] = pp;
    out[4] = wi.x; out[5] = wi.y; out[6] = wi.z; out[7] = pd;
    out[8] = e.r; out[9] = e.g; out[10] = e.b; out[11] = (float)smp.i;
}

}  // extern "C"
