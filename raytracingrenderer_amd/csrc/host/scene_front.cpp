// scene_front.cpp — the host side of the rtg boundary: loadScene + Scene::build, flattened into
// the rtg_scene_desc of include/rtg.h, plus Film::save and the C3 synthetic scene writer.
//
// Parity notes (what must match RTBase bit for bit, compile with -ffp-contract=off):
//  * loadScene / loadInstance        RTBase/SceneLoader.h:104-291 (material dispatch :111-188,
//    world transform + inverse-transpose normals :198-218, index offset quirk :221-224,
//    zero-area cull :227-234, camera :242-260, env map :275-284)
//  * Triangle::init                  RTBase/Geometry.h:72-83 (e1 = v2-v1, e2 = v0-v2, area)
//  * BVHNode::buildRecursive         RTBase/Geometry.h:325-392: node bounds in current order,
//    longest axis (ties -> y then z), std::sort by centroid (libstdc++ introsort: sorting an
//    index array with the same comparisons yields the same permutation as sorting Triangle
//    objects), prefix/suffix SAH sweep with strict '<' (first minimum), leaf <= 2 triangles.
//  * Scene::build light list         RTBase/Scene.h:95-105 (post-sort order) and Scene::init
//    :156-159 (environment first when its integrated power is > 0).
#include "../../../include/rth.h"

#include "gem_json.h"
#include "image_io.h"
#include "rt_core.h"

#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <future>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace rth {

const CofTerm kCofactors[16][6] = {
    {{1, 5, 10, 15}, {-1, 5, 11, 14}, {-1, 9, 6, 15}, {1, 9, 7, 14}, {1, 13, 6, 11}, {-1, 13, 7, 10}},
    {{-1, 1, 10, 15}, {1, 1, 11, 14}, {1, 9, 2, 15}, {-1, 9, 3, 14}, {-1, 13, 2, 11}, {1, 13, 3, 10}},
    {{1, 1, 6, 15}, {-1, 1, 7, 14}, {-1, 5, 2, 15}, {1, 5, 3, 14}, {1, 13, 2, 7}, {-1, 13, 3, 6}},
    {{-1, 1, 6, 11}, {1, 1, 7, 10}, {1, 5, 2, 11}, {-1, 5, 3, 10}, {-1, 9, 2, 7}, {1, 9, 3, 6}},
    {{-1, 4, 10, 15}, {1, 4, 11, 14}, {1, 8, 6, 15}, {-1, 8, 7, 14}, {-1, 12, 6, 11}, {1, 12, 7, 10}},
    {{1, 0, 10, 15}, {-1, 0, 11, 14}, {-1, 8, 2, 15}, {1, 8, 3, 14}, {1, 12, 2, 11}, {-1, 12, 3, 10}},
    {{-1, 0, 6, 15}, {1, 0, 7, 14}, {1, 4, 2, 15}, {-1, 4, 3, 14}, {-1, 12, 2, 7}, {1, 12, 3, 6}},
    {{1, 0, 6, 11}, {-1, 0, 7, 10}, {-1, 4, 2, 11}, {1, 4, 3, 10}, {1, 8, 2, 7}, {-1, 8, 3, 6}},
    {{1, 4, 9, 15}, {-1, 4, 11, 13}, {-1, 8, 5, 15}, {1, 8, 7, 13}, {1, 12, 5, 11}, {-1, 12, 7, 9}},
    {{-1, 0, 9, 15}, {1, 0, 11, 13}, {1, 8, 1, 15}, {-1, 8, 3, 13}, {-1, 12, 1, 11}, {1, 12, 3, 9}},
    {{1, 0, 5, 15}, {-1, 0, 7, 13}, {-1, 4, 1, 15}, {1, 4, 3, 13}, {1, 12, 1, 7}, {-1, 12, 3, 5}},
    {{-1, 0, 5, 11}, {1, 0, 7, 9}, {1, 4, 1, 11}, {-1, 4, 3, 9}, {-1, 8, 1, 7}, {1, 8, 3, 5}},
    {{-1, 4, 9, 14}, {1, 4, 10, 13}, {1, 8, 5, 14}, {-1, 8, 6, 13}, {-1, 12, 5, 10}, {1, 12, 6, 9}},
    {{1, 0, 9, 14}, {-1, 0, 10, 13}, {-1, 8, 1, 14}, {1, 8, 2, 13}, {1, 12, 1, 10}, {-1, 12, 2, 9}},
    {{-1, 0, 5, 14}, {1, 0, 6, 13}, {1, 4, 1, 14}, {-1, 4, 2, 13}, {-1, 12, 1, 6}, {1, 12, 2, 5}},
    {{1, 0, 5, 10}, {-1, 0, 6, 9}, {-1, 4, 1, 10}, {1, 4, 2, 9}, {1, 8, 1, 6}, {-1, 8, 2, 5}},
};

static thread_local std::string g_err;

struct Vert {
    V3 p, n;
    float u, v;
};
struct Tri {
    Vert v[3];
    uint32_t mat;
    float area;
};

struct TexData {
    int w = 1, h = 1;
    std::vector<float> rgb{1.0f, 1.0f, 1.0f};  // Texture::loadDefault: 1x1 white
};

struct BuildNode {
    Box bounds;
    int start = 0, end = 0;
    std::unique_ptr<BuildNode> l, r;
};

}  // namespace rth

struct rth_scene {
    std::vector<rth::Tri> tris;          // post-build order
    std::vector<uint32_t> perm;          // post-build index -> load index
    std::vector<float> positions, normals, uvs;
    std::vector<uint32_t> material;
    std::vector<float> node_bounds;
    std::vector<int32_t> node_links;
    std::vector<rtg_material> materials;
    std::vector<rth::TexData> tex;
    std::vector<rtg_texture> textures;
    std::vector<int32_t> lights;
    rtg_scene_desc desc{};
    rth_scene_info info{};
};

namespace rth {

static bool file_exists(const std::string& p) {
    struct stat st;
    return ::stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

// Texture::load (Imaging.h:32-71): ".hdr" anywhere in the name -> float decode; a file that
// fails to decode leaves width = 0 -> loadDefault() (1x1 white).
static TexData load_texture(const std::string& filename) {
    TexData t;
    std::string err;
    if (filename.find(".hdr") != std::string::npos) {
        ImageF img;
        if (decode_hdr(filename, img, err) && img.width > 0 && img.height > 0) {
            t.w = img.width;
            t.h = img.height;
            t.rgb = std::move(img.data);
        }
        return t;
    }
    Image8 img;
    if (!decode_ldr(filename, img, err) || img.width == 0 || img.height == 0) return t;
    t.w = img.width;
    t.h = img.height;
    size_t n = (size_t)t.w * t.h;
    t.rgb.assign(n * 3, 0.0f);
    const int ch = img.channels;
    for (size_t i = 0; i < n; ++i)
        for (int c = 0; c < 3; ++c) {
            size_t k = i * ch + c;  // the reference reads 3 bytes per texel even for 1-2 channels
            t.rgb[i * 3 + c] = (k < img.data.size() ? img.data[k] : 0) / 255.0f;
        }
    return t;
}

static float env_power(const TexData& t) {  // EnvironmentMap::totalIntegratedPower, Lights.h:171-184
    float total = 0;
    for (int i = 0; i < t.h; i++) {
        float st = sinf((float)(((float)i / (float)t.h) * M_PI));
        for (int n = 0; n < t.w; n++) {
            const float* c = &t.rgb[((size_t)i * t.w + n) * 3];
            total += (lum(c[0], c[1], c[2]) * st);
        }
    }
    total = total / (float)(t.w * t.h);
    return (float)(total * 4.0f * M_PI);
}

// ---------------------------------------------------------------- BVH build
struct BvhBuilder {
    const std::vector<Tri>& tris;
    std::vector<uint32_t>& perm;
    std::vector<V3> centre;
    std::atomic<int> threads_left;
    BvhBuilder(const std::vector<Tri>& t, std::vector<uint32_t>& p, int threads)
        : tris(t), perm(p), threads_left(threads) {
        centre.resize(t.size());
        for (size_t i = 0; i < t.size(); ++i)
            centre[i] = ((t[i].v[0].p + t[i].v[1].p) + t[i].v[2].p) / 3.0f;  // Triangle::centre
    }
    Box tri_box(uint32_t i) const {
        Box b;
        b.grow(tris[i].v[0].p);
        b.grow(tris[i].v[1].p);
        b.grow(tris[i].v[2].p);
        return b;
    }
    std::unique_ptr<BuildNode> build(int start, int end) {
        auto node = std::make_unique<BuildNode>();
        for (int i = start; i < end; i++) {
            const Tri& t = tris[perm[i]];
            node->bounds.grow(t.v[0].p);
            node->bounds.grow(t.v[1].p);
            node->bounds.grow(t.v[2].p);
        }
        int n = end - start;
        if (n <= 2) {
            node->start = start;
            node->end = end;
            return node;
        }
        V3 size = node->bounds.max - node->bounds.min;
        int axis = 0;
        if (size.y >= size.x && size.y >= size.z) axis = 1;
        else if (size.z >= size.x && size.z >= size.y) axis = 2;
        const V3* c = centre.data();
        std::sort(perm.begin() + start, perm.begin() + end,
                  [c, axis](uint32_t a, uint32_t b) { return c[a][axis] < c[b][axis]; });
        std::vector<Box> left(n), right(n);
        left[0] = tri_box(perm[start]);
        right[n - 1] = tri_box(perm[end - 1]);
        for (int i = 1; i < n; i++) {
            left[i] = left[i - 1];
            left[i].grow(tri_box(perm[start + i]));
        }
        for (int i = n - 2; i >= 0; i--) {
            right[i] = right[i + 1];
            right[i].grow(tri_box(perm[start + i]));
        }
        float best = 3.40282347e+38f;
        int split = 0;
        for (int i = 1; i < n; i++) {
            float nl = (float)i, nr = (float)(n - i);
            float cost = left[i - 1].area() * nl + right[i].area() * nr;
            if (cost < best) {
                best = cost;
                split = i;
            }
        }
        // The reference recurses forever when every cost is NaN/inf (split stays 0); split
        // the range in half instead so such input terminates.
        if (split == 0) split = n / 2;
        int mid = start + split;
        left.clear(); left.shrink_to_fit();
        right.clear(); right.shrink_to_fit();
        // Subtrees touch disjoint ranges of perm: build the left one on another thread when the
        // range is large (results are independent of scheduling).
        if (n > 65536 && threads_left.fetch_sub(1) > 0) {
            auto fut = std::async(std::launch::async, [this, start, mid] { return build(start, mid); });
            node->r = build(mid, end);
            node->l = fut.get();
        } else {
            node->l = build(start, mid);
            node->r = build(mid, end);
        }
        return node;
    }
};

static void flatten(const BuildNode* n, rth_scene* s, uint32_t depth, uint32_t& max_depth) {
    int32_t id = (int32_t)(s->node_links.size() / 4);
    s->node_links.insert(s->node_links.end(), {-1, -1, n->start, n->end});
    const Box& b = n->bounds;
    s->node_bounds.insert(s->node_bounds.end(), {b.min.x, b.min.y, b.min.z, b.max.x, b.max.y, b.max.z});
    if (depth > max_depth) max_depth = depth;
    if (n->l) {
        s->node_links[id * 4 + 0] = (int32_t)(s->node_links.size() / 4);
        flatten(n->l.get(), s, depth + 1, max_depth);
        s->node_links[id * 4 + 1] = (int32_t)(s->node_links.size() / 4);
        flatten(n->r.get(), s, depth + 1, max_depth);
    }
}

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

static bool load_scene(const std::string& dir, const rth_load_options& o, rth_scene* s) {
    auto t0 = std::chrono::steady_clock::now();
    SceneFile sf;
    if (!parse_scene_json(dir + "/scene.json", sf, g_err)) return false;
    int width = sf.properties.find("width").as_int(1920);
    int height = sf.properties.find("height").as_int(1080);
    if (o.width > 0) width = o.width;
    if (o.height > 0) height = o.height;
    float fov = sf.properties.find("fov").as_float(45.0f);
    M4 P = perspective(0.001f, 10000.0f, (float)width / (float)height, fov);
    V3 from, to, up;
    sf.properties.find("from").as_vec3(from.x, from.y, from.z);
    sf.properties.find("to").as_vec3(to.x, to.y, to.z);
    sf.properties.find("up").as_vec3(up.x, up.y, up.z);
    M4 V = look_at(from, to, up).inverted();
    if (sf.properties.find("flipX").as_int(0) == 1) P.m[0] = -P.m[0];
    M4 invP = P.inverted();  // Camera::init
    std::memcpy(s->desc.camera.inv_proj, invP.m, sizeof(invP.m));
    std::memcpy(s->desc.camera.camera, V.m, sizeof(V.m));
    V3 origin = V.mul_point(V3(0, 0, 0));  // Camera::updateView
    s->desc.camera.origin[0] = origin.x;
    s->desc.camera.origin[1] = origin.y;
    s->desc.camera.origin[2] = origin.z;
    s->desc.camera.width = (float)width;
    s->desc.camera.height = (float)height;
    {  // projectOntoCamera state: projectionMatrix, cameraToView, viewDirection, Afilm (Scene.h:22-41)
        rtg_camera_proj& cp = s->desc.projection;
        std::memcpy(cp.proj, P.m, sizeof(P.m));
        M4 Vc = V;
        M4 c2v = Vc.inverted();
        std::memcpy(cp.camera_to_view, c2v.m, sizeof(c2v.m));
        // inverseProjectionMatrix.mulPointAndPerspectiveDivide(Vec3(0, 0, 1)) (Core.h:310-320)
        const float* m = invP.m;
        const float vx = 0.0f, vy = 0.0f, vz = 1.0f;
        V3 v1(((vx * m[0] + vy * m[1]) + vz * m[2]) + m[3], ((vx * m[4] + vy * m[5]) + vz * m[6]) + m[7],
              ((vx * m[8] + vy * m[9]) + vz * m[10]) + m[11]);
        float w = ((m[12] * vx) + (m[13] * vy) + (m[14] * vz)) + m[15];
        w = 1.0f / w;
        V3 vd(v1.x * w, v1.y * w, v1.z * w);
        vd = V.mul_vec(vd).normalize();
        cp.view_direction[0] = vd.x;
        cp.view_direction[1] = vd.y;
        cp.view_direction[2] = vd.z;
        const float wlens = 2.0f / P.m[5];
        const float aspect = P.m[0] / P.m[5];
        const float hlens = wlens * aspect;
        cp.a_film = wlens * hlens;
    }
    s->info.width = width;
    s->info.height = height;

    std::map<std::string, int> tex_ids;
    auto texture = [&](const std::string& fn) {
        auto it = tex_ids.find(fn);
        if (it != tex_ids.end()) return it->second;
        int id = (int)s->tex.size();
        s->tex.push_back(load_texture(fn));
        tex_ids[fn] = id;
        return id;
    };

    std::vector<Tri> load_tris;
    for (const Instance& inst : sf.instances) {
        std::string mesh_path = dir + "/" + inst.mesh;
        std::string refl = inst.material.find("reflectance").str();
        if (o.skip_missing && (!file_exists(mesh_path) || !file_exists(dir + "/" + refl))) {
            s->info.dropped_instances++;
            continue;
        }
        std::vector<GemMesh> meshes;
        if (!load_gem(mesh_path, meshes, g_err)) return false;
        std::string bsdf = inst.material.find("bsdf").str();
        rtg_material m{};
        bool ok = true;
        m.int_ior = inst.material.find("intIOR").as_float(1.33f);
        m.ext_ior = inst.material.find("extIOR").as_float(1.0f);
        if (bsdf == "diffuse") { m.kind = RTG_MAT_DIFFUSE; m.two_sided = 1; }
        else if (bsdf == "orennayar" || bsdf == "plastic" || bsdf == "conductor") { m.kind = RTG_MAT_LAMBERT; m.two_sided = 1; }
        else if (bsdf == "glass") { m.kind = RTG_MAT_GLASS; m.two_sided = 0; }
        else if (bsdf == "mirror") { m.kind = RTG_MAT_MIRROR; m.two_sided = 1; }
        else if (bsdf == "dielectric") {
            float rough = inst.material.find("roughness").as_float(1.0f);
            m.kind = rough < 0.001f ? RTG_MAT_GLASS : RTG_MAT_LAMBERT;
            m.two_sided = 0;
        } else ok = false;
        if (!ok) {  // "Error in loading" — the instance is skipped (SceneLoader.h:189-194)
            if (inst.material.find("emission").str() != "") {
                g_err = "emission on an unknown bsdf '" + bsdf + "' (the reference dereferences NULL)";
                return false;
            }
            std::fprintf(stderr, "Error in loading\n");
            continue;
        }
        if (m.kind != RTG_MAT_GLASS) { m.int_ior = 0; m.ext_ior = 0; }
        m.texture = texture(dir + "/" + refl);
        if (inst.material.find("emission").str() != "")
            inst.material.find("emission").as_vec3(m.emission[0], m.emission[1], m.emission[2]);
        uint32_t mat_index = (uint32_t)s->materials.size();
        s->materials.push_back(m);

        M4 xf;
        std::memcpy(xf.m, inst.world, sizeof(xf.m));
        M4 nxf = xf.inverted().transposed();  // note: inverted() resets xf if singular
        std::vector<Vert> verts;
        std::vector<uint32_t> idx;
        for (const GemMesh& gm : meshes) {
            for (const GemVertex& gv : gm.vertices) {
                Vert v;
                v.p = xf.mul_point(V3(gv.pos[0], gv.pos[1], gv.pos[2]));
                v.n = nxf.mul_vec(V3(gv.normal[0], gv.normal[1], gv.normal[2])).normalize();
                v.u = gv.u;
                v.v = gv.v;
                verts.push_back(v);
            }
            uint32_t offset = (uint32_t)idx.size();  // index count, as in SceneLoader.h:221
            for (uint32_t k : gm.indices) idx.push_back(offset + k);
        }
        for (size_t i = 0; i + 2 < idx.size(); i += 3) {
            if (idx[i] >= verts.size() || idx[i + 1] >= verts.size() || idx[i + 2] >= verts.size()) {
                g_err = "vertex index out of range in " + mesh_path;
                return false;
            }
            Tri t;
            t.v[0] = verts[idx[i]];
            t.v[1] = verts[idx[i + 1]];
            t.v[2] = verts[idx[i + 2]];
            t.mat = mat_index;
            V3 e1 = t.v[2].p - t.v[1].p, e2 = t.v[0].p - t.v[2].p;
            t.area = e1.cross(e2).length() * 0.5f;
            if (t.area > 0) load_tris.push_back(t);
        }
    }
    // environment (SceneLoader.h:275-284); loadTexture caches by file name
    std::string env = o.envmap ? std::string(o.envmap) : sf.properties.find("envmap").str();
    s->desc.env_texture = -1;
    bool env_light = false;
    if (env != "") {
        s->desc.env_texture = texture(dir + "/" + env);
        env_light = env_power(s->tex[s->desc.env_texture]) > 0;
    }
    Box bounds;
    for (const Tri& t : load_tris)
        for (int k = 0; k < 3; ++k) bounds.grow(t.v[k].p);
    s->info.load_ms = ms_since(t0);

    // Scene::build
    auto t1 = std::chrono::steady_clock::now();
    s->perm.resize(load_tris.size());
    for (size_t i = 0; i < load_tris.size(); ++i) s->perm[i] = (uint32_t)i;
    int threads = o.bvh_threads > 0 ? o.bvh_threads : (int)std::max(1u, std::thread::hardware_concurrency());
    std::unique_ptr<BuildNode> root;
    {
        BvhBuilder b(load_tris, s->perm, threads - 1);
        root = b.build(0, (int)load_tris.size());
    }
    uint32_t depth = 0;
    flatten(root.get(), s, 0, depth);
    root.reset();
    s->tris.resize(load_tris.size());
    for (size_t i = 0; i < load_tris.size(); ++i) s->tris[i] = load_tris[s->perm[i]];
    s->info.bvh_ms = ms_since(t1);
    s->info.bvh_depth = depth;

    if (env_light) s->lights.push_back(-1);
    for (size_t i = 0; i < s->tris.size(); ++i) {
        const float* e = s->materials[s->tris[i].mat].emission;
        if (lum(e[0], e[1], e[2]) > 0) s->lights.push_back((int32_t)i);
    }
    s->info.env_in_lights = env_light ? 1 : 0;
    for (int k = 0; k < 3; ++k) {
        s->info.bounds_min[k] = bounds.min[k];
        s->info.bounds_max[k] = bounds.max[k];
    }
    return true;
}

static void fill_desc(rth_scene* s) {
    size_t n = s->tris.size();
    s->positions.resize(n * 9);
    s->normals.resize(n * 9);
    s->uvs.resize(n * 6);
    s->material.resize(n);
    for (size_t i = 0; i < n; ++i) {
        const Tri& t = s->tris[i];
        for (int k = 0; k < 3; ++k) {
            s->positions[i * 9 + k * 3 + 0] = t.v[k].p.x;
            s->positions[i * 9 + k * 3 + 1] = t.v[k].p.y;
            s->positions[i * 9 + k * 3 + 2] = t.v[k].p.z;
            s->normals[i * 9 + k * 3 + 0] = t.v[k].n.x;
            s->normals[i * 9 + k * 3 + 1] = t.v[k].n.y;
            s->normals[i * 9 + k * 3 + 2] = t.v[k].n.z;
            s->uvs[i * 6 + k * 2 + 0] = t.v[k].u;
            s->uvs[i * 6 + k * 2 + 1] = t.v[k].v;
        }
        s->material[i] = t.mat;
    }
    s->textures.resize(s->tex.size());
    for (size_t i = 0; i < s->tex.size(); ++i)
        s->textures[i] = rtg_texture{s->tex[i].w, s->tex[i].h, s->tex[i].rgb.data()};
    rtg_scene_desc& d = s->desc;
    d.n_tris = (uint32_t)n;
    d.positions = s->positions.data();
    d.normals = s->normals.data();
    d.uvs = s->uvs.data();
    d.material = s->material.data();
    d.n_nodes = (uint32_t)(s->node_links.size() / 4);
    d.node_bounds = s->node_bounds.data();
    d.node_links = s->node_links.data();
    d.n_materials = (uint32_t)s->materials.size();
    d.materials = s->materials.data();
    d.n_textures = (uint32_t)s->textures.size();
    d.textures = s->textures.data();
    d.n_lights = (uint32_t)s->lights.size();
    d.lights = s->lights.data();
    s->info.n_tris = d.n_tris;
    s->info.n_nodes = d.n_nodes;
    s->info.n_materials = d.n_materials;
    s->info.n_textures = d.n_textures;
    s->info.n_lights = d.n_lights;
}

// splitmix64 stream -> 24-bit uniform floats (no numpy).
struct SplitMix {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    float uniform(float a, float b) { return a + (b - a) * ((float)(next() >> 40) * (1.0f / 16777216.0f)); }
};

}  // namespace rth

using namespace rth;

// The C3 scene recipe around a mesh: diffuse albedo (185,181,173) PNG, constant
// env.hdr 64x32 = 1.0 (lights[0]), camera at (0,0,3.5) looking at the origin, fov 45.
static int write_mesh_scene(const std::string& d, const std::vector<GemVertex>& verts,
                            const std::vector<uint32_t>& idx, int32_t width, int32_t height) {
    if (!write_gem(d + "/synth.gem", verts, idx, g_err)) return RTG_ERR_ARG;
    const uint8_t albedo[3] = {185, 181, 173};  // 0.725 0.71 0.68 (cornell white)
    if (!encode_png(d + "/albedo.png", 1, 1, 3, albedo, g_err)) return RTG_ERR_ARG;
    std::vector<float> env(64 * 32 * 3, 1.0f);
    if (!encode_hdr(d + "/env.hdr", 64, 32, env.data(), g_err)) return RTG_ERR_ARG;
    FILE* f = std::fopen((d + "/scene.json").c_str(), "w");
    if (!f) { g_err = "cannot write scene.json"; return RTG_ERR_ARG; }
    std::fprintf(f,
                 "{\n    \"width\": \"%d\",\n    \"height\": \"%d\",\n    \"fov\": \"45.0\",\n"
                 "    \"from\": \"0.0 0.0 3.5\",\n    \"to\": \"0.0 0.0 0.0\",\n    \"up\": \"0.0 1.0 0.0\",\n"
                 "    \"envmap\": \"env.hdr\",\n    \"instances\": [{\n    \"filename\": \"synth.gem\",\n"
                 "    \"world\": [1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 1.0],\n"
                 "    \"bsdf\": \"diffuse\",\n    \"reflectance\": \"albedo.png\"\n}]\n}\n",
                 width, height);
    std::fclose(f);
    return RTG_OK;
}

extern "C" {

const char* rth_last_error(void) { return g_err.c_str(); }

#ifndef RTH_BUILD_ID
#define RTH_BUILD_ID "unknown"
#endif
// build.py passes the hash of the sources, headers and flags (source_hash("host"))
static const char k_build_tag[] __attribute__((used)) = "rth-build-id:" RTH_BUILD_ID;
const char* rth_build_id(void) { return k_build_tag + 13; }

int rth_load_scene(const char* scene_dir, const rth_load_options* opts, rth_scene** out) {
    if (!scene_dir || !out) { g_err = "rth_load_scene: null argument"; return RTG_ERR_ARG; }
    rth_load_options o{};
    if (opts) o = *opts;
    auto s = std::make_unique<rth_scene>();
    try {
        if (!load_scene(scene_dir, o, s.get())) return RTG_ERR_ARG;
    } catch (const std::exception& e) {
        g_err = std::string("rth_load_scene: ") + e.what();
        return RTG_ERR_ALLOC;
    }
    fill_desc(s.get());
    *out = s.release();
    return RTG_OK;
}

void rth_free_scene(rth_scene* s) { delete s; }
const rtg_scene_desc* rth_scene_desc(const rth_scene* s) { return s ? &s->desc : nullptr; }

int rth_scene_get_info(const rth_scene* s, rth_scene_info* out) {
    if (!s || !out) return RTG_ERR_ARG;
    *out = s->info;
    return RTG_OK;
}

int rth_scene_permutation(const rth_scene* s, uint32_t* out) {
    if (!s || !out) return RTG_ERR_ARG;
    std::memcpy(out, s->perm.data(), s->perm.size() * 4);
    return RTG_OK;
}

int rth_save_hdr(const char* path, int32_t w, int32_t h, const float* sum, uint32_t spp) {
    if (!path || !sum || w <= 0 || h <= 0) { g_err = "rth_save_hdr: bad argument"; return RTG_ERR_ARG; }
    std::vector<float> img((size_t)w * h * 3);
    for (size_t i = 0; i < (size_t)w * h; ++i)  // Film::save: film[i] / (float)SPP
        for (int c = 0; c < 3; ++c) img[i * 3 + c] = sum[i * 3 + c] / (float)spp;
    return encode_hdr(path, w, h, img.data(), g_err) ? RTG_OK : RTG_ERR_ARG;
}

int rth_write_hdr(const char* path, int32_t w, int32_t h, const float* rgb) {
    return encode_hdr(path ? path : "", w, h, rgb, g_err) ? RTG_OK : RTG_ERR_ARG;
}

int rth_read_hdr(const char* path, int32_t* w, int32_t* h, float** rgb) {
    ImageF img;
    if (!path || !decode_hdr(path, img, g_err)) return RTG_ERR_ARG;
    *w = img.width;
    *h = img.height;
    *rgb = (float*)std::malloc(img.data.size() * sizeof(float));
    std::memcpy(*rgb, img.data.data(), img.data.size() * sizeof(float));
    return RTG_OK;
}

int rth_read_png(const char* path, int32_t* w, int32_t* h, int32_t* ch, uint8_t** data) {
    Image8 img;
    if (!path || !decode_png(path, img, g_err)) return RTG_ERR_ARG;
    *w = img.width;
    *h = img.height;
    *ch = img.channels;
    *data = (uint8_t*)std::malloc(img.data.size());
    std::memcpy(*data, img.data.data(), img.data.size());
    return RTG_OK;
}

int rth_tonemap(int32_t w, int32_t h, const float* sum, uint32_t spp, float exposure, uint8_t* out) {
    if (!sum || !out || w <= 0 || h <= 0) { g_err = "rth_tonemap: bad argument"; return RTG_ERR_ARG; }
    const size_t n = (size_t)w * h;
    for (size_t i = 0; i < n * 3; ++i) {
        const float p = sum[i] * exposure / (float)spp;
        const float m = std::min(powf(std::max(p, 0.0f), 1.0f / 2.2f) * 255, 255.0f);
        out[i] = (uint8_t)(m == m ? m : 0.0f);  // NaN (spp = 0 or a NaN film) -> 0
    }
    return RTG_OK;
}

int rth_save_png(const char* path, int32_t w, int32_t h, const float* sum, uint32_t spp) {
    if (!path) { g_err = "rth_save_png: null path"; return RTG_ERR_ARG; }
    std::vector<uint8_t> rgb((size_t)w * h * 3);
    int rc = rth_tonemap(w, h, sum, spp, 1.0f, rgb.data());
    if (rc) return rc;
    return encode_png(path, w, h, 3, rgb.data(), g_err) ? RTG_OK : RTG_ERR_ARG;
}

int rth_read_ldr(const char* path, int32_t* w, int32_t* h, int32_t* ch, uint8_t** data) {
    Image8 img;
    if (!path || !decode_ldr(path, img, g_err)) return RTG_ERR_ARG;
    *w = img.width;
    *h = img.height;
    *ch = img.channels;
    *data = (uint8_t*)std::malloc(img.data.size());
    std::memcpy(*data, img.data.data(), img.data.size());
    return RTG_OK;
}

void rth_free(void* p) { std::free(p); }

int rth_write_synthetic(const char* dir, uint32_t n_tris, uint64_t seed, int32_t width, int32_t height) {
    if (!dir) return RTG_ERR_ARG;
    std::string d(dir);
    ::mkdir(d.c_str(), 0755);
    SplitMix rng{seed};
    std::vector<GemVertex> verts((size_t)n_tris * 3);
    std::vector<uint32_t> idx((size_t)n_tris * 3);
    for (uint32_t t = 0; t < n_tris; ++t) {
        V3 c(rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-1, 1));
        V3 p[3];
        for (int k = 0; k < 3; ++k) p[k] = c + V3(rng.uniform(-0.02f, 0.02f), rng.uniform(-0.02f, 0.02f), rng.uniform(-0.02f, 0.02f));
        V3 n = (p[1] - p[0]).cross(p[2] - p[0]).normalize();
        for (int k = 0; k < 3; ++k) {
            GemVertex& g = verts[(size_t)t * 3 + k];
            std::memset(&g, 0, sizeof(g));
            g.pos[0] = p[k].x; g.pos[1] = p[k].y; g.pos[2] = p[k].z;
            g.normal[0] = n.x; g.normal[1] = n.y; g.normal[2] = n.z;
            idx[(size_t)t * 3 + k] = t * 3 + k;
        }
    }
    return write_mesh_scene(d, verts, idx, width, height);
}

int rth_write_mesh_scene(const char* dir, const float* positions, uint32_t n_tris, int32_t width, int32_t height) {
    if (!dir || (!positions && n_tris)) return RTG_ERR_ARG;
    std::string d(dir);
    ::mkdir(d.c_str(), 0755);
    std::vector<GemVertex> verts((size_t)n_tris * 3);
    std::vector<uint32_t> idx((size_t)n_tris * 3);
    for (uint32_t t = 0; t < n_tris; ++t) {
        const float* P = positions + (size_t)t * 9;
        V3 p[3] = {V3(P[0], P[1], P[2]), V3(P[3], P[4], P[5]), V3(P[6], P[7], P[8])};
        V3 n = (p[1] - p[0]).cross(p[2] - p[0]).normalize();
        for (int k = 0; k < 3; ++k) {
            GemVertex& g = verts[(size_t)t * 3 + k];
            std::memset(&g, 0, sizeof(g));
            g.pos[0] = p[k].x; g.pos[1] = p[k].y; g.pos[2] = p[k].z;
            g.normal[0] = n.x; g.normal[1] = n.y; g.normal[2] = n.z;
            idx[(size_t)t * 3 + k] = t * 3 + k;
        }
    }
    return write_mesh_scene(d, verts, idx, width, height);
}

}  // extern "C"
