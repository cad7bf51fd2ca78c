// sbvh_check — TEST INFRASTRUCTURE ONLY (tests/test_bvh.py). CPU check of rtg_bvh.hip's build_sbvh on
// a loaded scene (no GPU): the tree is well formed (every internal box holds its children's, every
// triangle reachable), and every triangle is covered by its leaf slots (its vertices and random points
// of it lie in one of its fragments' boxes), plus build time and duplication. Built by build.py
// build_sbvh_check; run: sbvh_check <scene dir> | sbvh_check x synth <n triangles>
#include "../../include/rth.h"
#include "../../raytracingrenderer_amd/csrc/device/rtg_internal.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

int main(int argc, char** argv) {
    rth_load_options o{};
    o.skip_missing = 1;
    std::string dir = argv[1];
    if (argc > 3 && std::string(argv[2]) == "synth") {
        rth_write_synthetic("/tmp/sbvh_synth", (uint32_t)atoi(argv[3]), 20251015, 1024, 1024);
        dir = "/tmp/sbvh_synth";
    }
    rth_scene* s = nullptr;
    if (rth_load_scene(dir.c_str(), &o, &s)) { std::printf("load failed: %s\n", rth_last_error()); return 2; }
    const rtg_scene_desc* d = rth_scene_desc(s);
    std::vector<int32_t> lk;
    std::vector<float> bd;
    auto t0 = std::chrono::steady_clock::now();
    const bool ok = build_sbvh(d, lk, bd);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (!ok) { std::printf("build_sbvh failed\n"); return 1; }
    const size_t nn = lk.size() / 4;
    std::vector<std::vector<int>> frags(d->n_tris);
    std::vector<int> stack{0}, depth(nn, 0);
    size_t leaves = 0, maxd = 0, bad = 0;
    auto area = [&](int n) {
        const double x = bd[n * 6 + 3] - bd[n * 6], y = bd[n * 6 + 4] - bd[n * 6 + 1], z = bd[n * 6 + 5] - bd[n * 6 + 2];
        return x * y + y * z + z * x;
    };
    double sa_int = 0.0, sa_leaf = 0.0;  // summed surface areas / the root's (the SAH's two terms)
    while (!stack.empty()) {
        const int n = stack.back();
        stack.pop_back();
        maxd = std::max(maxd, (size_t)depth[n]);
        (lk[n * 4] < 0 ? sa_leaf : sa_int) += area(n) / area(0);
        if (lk[n * 4] < 0) {
            ++leaves;
            frags[lk[n * 4 + 2]].push_back(n);
            continue;
        }
        for (int c : {lk[n * 4], lk[n * 4 + 1]}) {
            for (int k = 0; k < 3; ++k)
                if (bd[c * 6 + k] < bd[n * 6 + k] || bd[c * 6 + 3 + k] > bd[n * 6 + 3 + k]) ++bad;
            depth[c] = depth[n] + 1;
            stack.push_back(c);
        }
    }
    size_t missing = 0, uncovered = 0;
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    for (uint32_t t = 0; t < d->n_tris; ++t) {
        if (frags[t].empty()) { ++missing; continue; }
        const float* P = d->positions + (size_t)t * 9;
        for (int k = 0; k < 16; ++k) {
            float a = U(rng), b = U(rng);
            if (k < 3) { a = k == 1; b = k == 2; }  // the vertices
            if (a + b > 1) { a = 1 - a; b = 1 - b; }
            float p[3];
            for (int q = 0; q < 3; ++q) p[q] = P[q] + a * (P[3 + q] - P[q]) + b * (P[6 + q] - P[q]);
            bool in = false;
            for (int f : frags[t]) {
                bool inside = true;
                for (int q = 0; q < 3; ++q) inside = inside && p[q] >= bd[f * 6 + q] && p[q] <= bd[f * 6 + 3 + q];
                in = in || inside;
            }
            if (!in) ++uncovered;
        }
    }
    std::printf("tris %u nodes %zu leaves %zu (dup %.3f) depth %zu build %.0f ms | bad boxes %zu, missing tris %zu, "
                "uncovered points %zu | area sums / root: internal %.2f leaves %.2f\n", d->n_tris, nn, leaves,
                (double)leaves / d->n_tris, maxd, ms, bad, missing, uncovered, sa_int, sa_leaf);
    rth_free_scene(s);
    return (bad || missing || uncovered) ? 1 : 0;
}
