// cli.cpp — headless counterpart of RTBase's Main.cpp (RTBase/Main.cpp:14-150) on librth + librtg.
//
// Same arguments and stopping rule as the reference's frame loop:
//   -scene <dir>  -SPP <n>  -outputFilename <file>
// frames of +1 spp until SPP is reached or 10 s of render time have passed, then the film is
// written as result_<spp>.hdr (Film::save). The window / camera keys have no headless meaning;
// 'P' and 'L' (saveHDR / savePNG of -outputFilename) become: -outputFilename is always written at
// the end, as .hdr or, for a .png name, tonemapped PNG (RayTracer::savePNG).
// Extra options (defaults keep the reference behaviour): -width -height (override scene.json),
// -maxDepth (MAX_DEPTH, 4), -seed (sampler seed, 1234), -device, -batch (spp per render call;
// results do not depend on it), -sync 1 (wait for every frame; default: frames are queued with
// rtg_render_async and up to three run side by side, the film is read once at the end),
// -skipMissing 1 (filtered scene variants), -envmap <file>, -timeLimit <s> (10; 0 = none).
// "Frame time" is the wall time of each render call, as Main.cpp:113-117 times rt.render(); with
// queued frames a call returns once the frame three before it has left the GPU, so in the steady
// state it is the GPU's time per frame.
// Multi-GPU (one node): -gpus N renders on devices 0..N-1, -devices a,b,... on a list. Rank r
// renders the 32x32 tiles with (tile_x + tile_y) % N == r, and the film is assembled on the first
// device from every device's own tiles (packed, one RCCL send per device, scattered) before it is
// written (rtg_group_*, include/rtg.h); the output is bit-identical to the one-device render. Frames
// are queued on every device (rtg_group_render_async: coalesced and pipelined per device, as on one
// device) unless -sync 1 (rtg_group_render: each call waits for every device).
#include "../../../include/rth.h"

#include <chrono>
#include <cstdio>
#include <sstream>
#include <cstdlib>
#include <string>
#include <unordered_map>
#include <vector>

static int die(const char* what, const char* msg) {
    std::fprintf(stderr, "rtg_render: %s: %s\n", what, msg ? msg : "");
    return 1;
}

int main(int argc, char** argv) {
    std::string scene_name = "MaterialsScene", filename = "GI.hdr";
    unsigned spp_target = 8192;
    std::unordered_map<std::string, std::string> args;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (!a.empty() && a[0] == '-') {
            if (i + 1 < argc) args[a] = argv[++i];
            else std::fprintf(stderr, "Error: Missing value for argument '%s'\n", a.c_str());
        } else {
            std::fprintf(stderr, "Warning: Ignoring unexpected argument '%s'\n", a.c_str());
        }
    }
    auto get = [&](const char* k, const std::string& d) { auto it = args.find(k); return it == args.end() ? d : it->second; };
    scene_name = get("-scene", scene_name);
    filename = get("-outputFilename", filename);
    spp_target = (unsigned)std::stoul(get("-SPP", std::to_string(spp_target)));
    const bool out_given = args.count("-outputFilename") > 0;
    rth_load_options lo{};
    lo.width = std::stoi(get("-width", "0"));
    lo.height = std::stoi(get("-height", "0"));
    lo.skip_missing = std::stoi(get("-skipMissing", "0"));
    std::string env = get("-envmap", "");
    lo.envmap = env.empty() ? nullptr : env.c_str();
    const int max_depth = std::stoi(get("-maxDepth", "4"));
    const uint64_t seed = std::stoull(get("-seed", "1234"));
    const int device = std::stoi(get("-device", "0"));
    const unsigned batch = (unsigned)std::max(1, std::stoi(get("-batch", "1")));
    const double time_limit = std::stod(get("-timeLimit", "10"));
    const bool sync = std::stoi(get("-sync", "0")) != 0;

    rth_scene* scene = nullptr;
    if (rth_load_scene(scene_name.c_str(), &lo, &scene) != 0) return die("loadScene", rth_last_error());
    rth_scene_info info{};
    rth_scene_get_info(scene, &info);
    std::vector<int> devices;
    if (args.count("-devices")) {
        std::stringstream ss(args["-devices"]);
        std::string tok;
        while (std::getline(ss, tok, ',')) devices.push_back(std::stoi(tok));
    } else if (args.count("-gpus")) {
        for (int i = 0; i < std::stoi(args["-gpus"]); ++i) devices.push_back(i);
    }
    rtg_handle* rt = nullptr;
    rtg_group* grp = nullptr;
    if (devices.empty()) {
        if (rtg_create(device, rth_scene_desc(scene), &rt) != 0) return die("rtg_create", rtg_last_error());
        if (rtg_set_options(rt, max_depth, RTG_OPT_CULL, 0) != 0) return die("rtg_set_options", rtg_last_error());
    } else {
        if (rtg_group_create(devices.data(), (int)devices.size(), rth_scene_desc(scene), &grp) != 0)
            return die("rtg_group_create", rtg_last_error());
        if (rtg_group_set_options(grp, max_depth, RTG_OPT_CULL, 0) != 0) return die("rtg_group_set_options", rtg_last_error());
        std::printf("%d devices, own-tile film exchange by %s\n", (int)devices.size(),
                    rtg_group_uses_rccl(grp) ? "RCCL (ncclSend/ncclRecv)"
                    : devices.size() == 1    ? "none (one device)"
                                             : "device copies (repeated devices)");
    }
    std::printf("scene %s: %u triangles, %u lights, %dx%d (load %.0f ms, BVH %.0f ms)\n", scene_name.c_str(),
                info.n_tris, info.n_lights, info.width, info.height, info.load_ms, info.bvh_ms);

    unsigned spp = 0;
    double total = 0.0;
    const auto w0 = std::chrono::steady_clock::now();
    while (spp < spp_target) {
        const unsigned n = std::min(batch, spp_target - spp);
        auto t0 = std::chrono::steady_clock::now();
        const int rc = grp    ? (sync ? rtg_group_render(grp, spp, n, seed) : rtg_group_render_async(grp, spp, n, seed))
                       : sync ? rtg_render(rt, spp, n, seed, nullptr, 0)
                              : rtg_render_async(rt, spp, n, seed, nullptr, 0, nullptr);
        if (rc != 0) return die("rtg_render", rtg_last_error());
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        total += dt;
        spp += n;
        std::printf("Frame time: %gs | Total time: %gs\nSPP: %u\n", dt, total, spp);
        if (time_limit > 0 && total >= time_limit) break;
    }
    std::vector<float> film((size_t)info.width * info.height * 3);
    uint32_t got = 0;
    if (rt && rtg_synchronize(rt) != 0) return die("rtg_synchronize", rtg_last_error());
    if (grp && rtg_group_synchronize(grp) != 0) return die("rtg_group_synchronize", rtg_last_error());
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
    std::printf("%u spp in %.4f s of wall time (%s): %.4f ms per spp, %.1f Mpaths/s\n", spp, wall,
                grp ? (sync ? "device group, synchronous calls" : "device group, queued calls")
                    : sync ? "synchronous calls" : "queued calls", 1e3 * wall / std::max(1u, spp),
                (double)spp * info.width * info.height / wall / 1e6);
    if (grp) {
        if (rtg_group_film_read(grp, film.data(), &got) != 0) return die("rtg_group_film_read", rtg_last_error());
        std::printf("film exchange: %.3f ms\n", rtg_group_reduce_ms(grp));
    } else if (rtg_film_read(rt, film.data(), &got) != 0) {
        return die("rtg_film_read", rtg_last_error());
    }
    const std::string auto_name = "result_" + std::to_string(got) + ".hdr";
    if (rth_save_hdr(auto_name.c_str(), info.width, info.height, film.data(), got) != 0)
        return die("saveHDR", rth_last_error());
    std::printf("wrote %s\n", auto_name.c_str());
    if (out_given) {
        const bool png = filename.size() > 4 && filename.compare(filename.size() - 4, 4, ".png") == 0;
        int rc = png ? rth_save_png(filename.c_str(), info.width, info.height, film.data(), got)
                     : rth_save_hdr(filename.c_str(), info.width, info.height, film.data(), got);
        if (rc != 0) return die(png ? "savePNG" : "saveHDR", rth_last_error());
        std::printf("wrote %s\n", filename.c_str());
    }
    if (rt) rtg_destroy(rt);
    if (grp) rtg_group_destroy(grp);
    rth_free_scene(scene);
    return 0;
}
