// host_sanitize.cpp — TEST INFRASTRUCTURE ONLY (tests/test_sanitize.py). A driver for the host code
// built with -fsanitize=address,undefined (raytracingrenderer_amd/build.py build_sanitized): the
// scene front-end (librth's sources: GEM/JSON loader, PNG / JPEG / Radiance decoders, BVH build,
// RGBE / PNG writers) and the C oracle, on the committed and staged scenes and on corrupted copies
// of every file a scene reads. The untrusted-input parsers must reject or accept each mutant
// without a memory error, a leak or undefined behaviour; the sanitizers abort the run otherwise.
//
// The reference reads the same files with stb_image and its GEM/JSON loader (RTBase/Imaging.h:32-71,
// GEMLoader.h:344-365); its tests do not exercise malformed inputs.
//
//   host_sanitize <scratch dir> <scene dir>...
#include "../../include/rth.h"

#include <dirent.h>
#include <time.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

extern "C" {
typedef struct or_scene or_scene;
or_scene* or_create(const rtg_scene_desc* d, int max_depth);
void or_destroy(or_scene* s);
int or_render(or_scene* s, uint32_t first, uint32_t n_samples, uint64_t seed, const uint32_t* tiles, uint32_t n_tiles,
              int threads, float* film, uint64_t* counts, int count);
}

namespace {
struct SplitMix {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
};

std::vector<unsigned char> slurp(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<unsigned char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

void spit(const std::string& p, const std::vector<unsigned char>& d) {
    std::ofstream f(p, std::ios::binary | std::ios::trunc);
    f.write((const char*)d.data(), (std::streamsize)d.size());
}

std::string lower_ext(const std::string& n) {
    const size_t k = n.rfind('.');
    std::string e = k == std::string::npos ? "" : n.substr(k + 1);
    for (char& c : e) c = (char)tolower(c);
    return e;
}

std::vector<std::string> list_dir(const std::string& d) {
    std::vector<std::string> out;
    if (DIR* h = opendir(d.c_str())) {
        while (dirent* e = readdir(h))
            if (e->d_name[0] != '.') out.push_back(e->d_name);
        closedir(h);
    }
    std::sort(out.begin(), out.end());
    return out;
}

// corrupted copies of `data`: truncations, flipped bytes, runs of 0x00 / 0xFF, a header byte
// forced to extreme values, duplicated spans
std::vector<std::vector<unsigned char>> mutants(const std::vector<unsigned char>& data, uint64_t seed, int n) {
    std::vector<std::vector<unsigned char>> out;
    const size_t L = data.size();
    for (size_t cut : {(size_t)0, (size_t)1, (size_t)4, (size_t)8, (size_t)16, (size_t)33, L / 8, L / 4, L / 2,
                       L > 0 ? L - 1 : 0})
        if (cut < L) out.emplace_back(data.begin(), data.begin() + cut);
    SplitMix r{seed};
    for (int i = 0; i < n && L > 0; ++i) {
        std::vector<unsigned char> m = data;
        switch (i % 5) {
        case 0:  // a few flipped bytes anywhere
            for (int k = 0; k < 1 + i % 7; ++k) m[r.next() % L] ^= (unsigned char)(1 + r.next() % 255);
            break;
        case 1:  // a byte of the first 64 (headers, markers, sizes) set to 0x00 / 0xFF / 0x7F
            m[r.next() % std::min<size_t>(L, 64)] = (unsigned char)((const unsigned char[]){0x00, 0xFF, 0x7F}[i % 3]);
            break;
        case 2: {  // a run of 0xFF or 0x00
            const size_t a = r.next() % L, len = std::min<size_t>(L - a, 1 + r.next() % 64);
            std::memset(m.data() + a, (i & 1) ? 0xFF : 0x00, len);
            break;
        }
        case 3: {  // truncated at a random point after a flip
            m[r.next() % L] ^= 0x80;
            m.resize(r.next() % L);
            break;
        }
        default: {  // a span duplicated in place (lengths and offsets that no longer agree)
            const size_t a = r.next() % L, len = std::min<size_t>(L - a, 1 + r.next() % 256);
            std::vector<unsigned char> span(m.begin() + a, m.begin() + a + len);
            m.insert(m.begin() + r.next() % L, span.begin(), span.end());
            break;
        }
        }
        out.push_back(std::move(m));
    }
    return out;
}

int g_fail = 0;
long g_ok = 0, g_rejected = 0;

double now_s() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

void decode_file(const std::string& path, const std::string& ext) {
    const double t0 = now_s();
    struct Slow {
        const std::string& p; double t0; int32_t* w; int32_t* h;
        ~Slow() { if (getenv("HS_SLOW") && now_s() - t0 > 0.1) std::fprintf(stderr, "slow %.2fs %s %dx%d\n", now_s() - t0, p.c_str(), *w, *h); }
    };
    int32_t w = 0, h = 0, c = 0;
    Slow slow{path, t0, &w, &h};
    if (ext == "hdr") {
        float* px = nullptr;
        const int rc = rth_read_hdr(path.c_str(), &w, &h, &px);
        if (rc == 0) { ++g_ok; rth_free(px); } else ++g_rejected;
    } else {
        uint8_t* px = nullptr;
        const int rc = rth_read_ldr(path.c_str(), &w, &h, &c, &px);
        if (rc == 0) { ++g_ok; rth_free(px); } else ++g_rejected;
    }
}

// a scene directory of symlinks to `src`'s files, with `victim` replaced by `bytes`
std::string shadow_scene(const std::string& scratch, const std::string& src, const std::string& victim,
                         const std::vector<unsigned char>& bytes, int k) {
    const std::string d = scratch + "/mut" + std::to_string(k);
    for (const std::string& f : list_dir(d)) unlink((d + "/" + f).c_str());
    mkdir(d.c_str(), 0755);
    for (const std::string& f : list_dir(src)) {
        if (f == victim) continue;
        if (symlink((src + "/" + f).c_str(), (d + "/" + f).c_str()) != 0) { std::perror("symlink"); g_fail = 1; }
    }
    spit(d + "/" + victim, bytes);
    return d;
}

void load_and_render(const std::string& dir, int width, int height, bool render, const char* envmap = nullptr) {
    rth_load_options o{};
    o.width = width;
    o.height = height;
    o.skip_missing = 1;
    o.bvh_threads = 1;
    o.envmap = envmap;
    rth_scene* s = nullptr;
    if (rth_load_scene(dir.c_str(), &o, &s) != 0) {
        ++g_rejected;
        return;
    }
    ++g_ok;
    rth_scene_info info{};
    rth_scene_get_info(s, &info);
    const rtg_scene_desc* d = rth_scene_desc(s);
    std::vector<uint32_t> perm(d->n_tris);
    rth_scene_permutation(s, perm.data());
    if (render && d->n_lights > 0 && info.width > 0 && info.height > 0) {
        or_scene* os = or_create(d, 3);
        if (os) {
            std::vector<float> film((size_t)info.width * info.height * 3, 0.0f);
            uint64_t counts[5] = {0, 0, 0, 0, 0};
            if (or_render(os, 0, 1, 1234, nullptr, 0, 1, film.data(), counts, 1) != 0) g_fail = 1;
            std::vector<uint8_t> rgb(film.size());
            rth_tonemap(info.width, info.height, film.data(), 1, 1.0f, rgb.data());
            or_destroy(os);
        }
    }
    rth_free_scene(s);
}
}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: host_sanitize <scratch dir> <scene dir>...\n");
        return 2;
    }
    const std::string scratch = argv[1];
    mkdir(scratch.c_str(), 0755);
    // writers + readers round trip, and the synthetic scene recipe
    {
        std::vector<float> img(37 * 23 * 3);
        for (size_t i = 0; i < img.size(); ++i) img[i] = (float)((i * 2654435761u) % 1000) * 0.01f;
        if (rth_save_hdr((scratch + "/a.hdr").c_str(), 37, 23, img.data(), 3) != 0) g_fail = 1;
        if (rth_save_png((scratch + "/a.png").c_str(), 37, 23, img.data(), 3) != 0) g_fail = 1;
        decode_file(scratch + "/a.hdr", "hdr");
        decode_file(scratch + "/a.png", "png");
        if (rth_write_synthetic((scratch + "/synth").c_str(), 2000, 7, 48, 32) != 0) g_fail = 1;
        load_and_render(scratch + "/synth", 0, 0, true);
        int k = 0;
        for (const auto& m : mutants(slurp(scratch + "/a.hdr"), 11, 60)) {
            spit(scratch + "/m.hdr", m);
            decode_file(scratch + "/m.hdr", "hdr");
            ++k;
        }
        for (const auto& m : mutants(slurp(scratch + "/a.png"), 12, 60)) {
            spit(scratch + "/m.png", m);
            decode_file(scratch + "/m.png", "png");
        }
    }
    int k = 0;
    for (int a = 2; a < argc; ++a) {
        // absolute: the mutant scenes are directories of symlinks to this one's files
        char real[4096];
        const std::string dir = realpath(argv[a], real) ? std::string(real) : std::string(argv[a]);
        std::fprintf(stderr, "[host_sanitize] %s\n", dir.c_str());
        load_and_render(dir, 48, 36, true);
        std::vector<std::pair<size_t, std::string>> gems;
        size_t scene_bytes = 0;
        for (const std::string& f : list_dir(dir)) {
            const std::string p = dir + "/" + f, e = lower_ext(f);
            struct stat st{};
            if (stat(p.c_str(), &st) != 0 || !S_ISREG(st.st_mode)) continue;
            scene_bytes += (size_t)st.st_size;
            if (e == "png" || e == "jpg" || e == "jpeg" || e == "hdr") {
                decode_file(p, e);
                // every texture of the scene, mutated (large files: fewer mutants)
                const int n = st.st_size > (4 << 20) ? 10 : 40;
                const std::string tmp = scratch + "/tex." + e;
                for (const auto& m : mutants(slurp(p), 1000 + k, n)) {
                    spit(tmp, m);
                    decode_file(tmp, e);
                }
            } else if (e == "gem") {
                gems.emplace_back((size_t)st.st_size, f);
            }
            ++k;
        }
        // scene.json and the two smallest meshes, mutated, loaded as the scene (every load decodes the
        // scene's textures: fewer mutants for the big reference scenes)
        const bool big = scene_bytes > (8u << 20);
        std::sort(gems.begin(), gems.end());
        std::vector<std::string> victims = {"scene.json"};
        for (size_t i = 0; i < gems.size() && i < 2; ++i) victims.push_back(gems[i].second);
        for (const std::string& v : victims) {
            const auto src = slurp(dir + "/" + v);
            if (src.empty()) continue;
            for (const auto& m : mutants(src, 5000 + k, v == "scene.json" ? (big ? 10 : 60) : (big ? 4 : 24))) {
                load_and_render(shadow_scene(scratch, dir, v, m, k % 4), 24, 16, false);
                ++k;
            }
        }
    }
    std::fprintf(stderr, "[host_sanitize] decoded/loaded %ld, rejected %ld, failures %d\n", g_ok, g_rejected, g_fail);
    std::printf("host_sanitize ok %ld rejected %ld fail %d\n", g_ok, g_rejected, g_fail);
    return g_fail ? 1 : 0;
}
