#!/usr/bin/env python3
"""Headline benchmark: BASELINE.json metric "Mray/s + ms/frame at 1024x1024x64spp; achieved HBM GB/s
vs peak" on config C3 (synthetic 1M random triangles, 1024x1024, 64 spp, MAX_DEPTH 4).

One step = one complete 1024x1024x64spp render (64 RayTracer::render() frames) of this rank's
32x32 tiles ((tile_x + tile_y) % world_size == rank) through the HIP wavefront tracer, plus, for N > 1, the
own-tile film exchange to rank 0 over xGMI (every rank packs its tiles' pixels, one RCCL gather,
rank 0 scatters them; tile supports are disjoint and cover the film, so the assembled film is
bit-identical to a 1-GPU render). Total work is fixed as N grows (strong scaling). Scene
generation, loading and BVH build happen before the timed region.

`value` is traced rays per second (closest-hit + shadow rays the traversal walked): renderTile casts
the pixel-centre camera ray for every sample (Renderer.h:805-808), the GPU traces it once per pixel
per chunk, and `mrays_reference_equivalent_per_s` counts it once per sample as the reference does.

  python bench.py [--gpus N] [--steps K] [--warmup W]
      N > 1 without torchrun: one process drives N GPUs through the native group (rtg_group_*:
      one handle and host thread per device, ncclCommInitAll + the own-tile exchange of the film),
      the path an RTBase C++ host takes. N must not exceed the visible devices (exit status 2 otherwise).
  python bench.py --devices 0,0 [--verify-film]
      the same group path over an explicit device list; repeats rehearse N ranks on one GPU
  torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL via torch)
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
L2_PEAK_GBS = 34500.0  # aggregate L2 bandwidth, same guide (§L2)
# rocprofv3 PMC passes of each config's bench line (tools/pmc_config.sh: FETCH_SIZE, WRITE_SIZE and
# the DRAM share of L2 read requests, each its own run), per config; quoted only on the workload they
# were taken on (the file's "spp", one GPU, the whole film)
PMC_SUMMARIES = {c: os.path.join(ROOT, "profiles", "r06_pmc_traffic_%s.json" % c.lower()) for c in ("C2", "C3", "C4", "C5")}
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r05_pmc_traffic.json")  # round 5's C3 passes (fallback)
KSTATS = os.path.join(ROOT, "profiles", "r06_kernel_stats_c3.csv")   # rocprofv3 kernel-trace stats, same
VALU_ISSUE = os.path.join(ROOT, "profiles", "r06_valu_issue.json")    # tools/valu_issue.py (SQ_INSTS_VALU passes)
ROOF_SWEEP = os.path.join(ROOT, "profiles", "r02_roof_sweep.jsonl")  # tools/micro/roof.hip on an MI355X
ROOF_REPLAY = os.path.join(ROOT, "profiles", "r05_roof_replay_c3.jsonl")  # tools/roof_replay.py (C3)
# the replay ceiling of each workload (tools/replay_all.sh on an MI355X: tools/roof_replay.py at the
# line's own chunk shape), by (config, shard_of); a ceiling is quoted only when its chunk shape
# (samples per chunk) is the line's
ROOF_REPLAYS = {("C3", 1): ROOF_REPLAY,
                ("C3", 8): os.path.join(ROOT, "profiles", "r05_roof_replay_shard8.jsonl"),
                ("C2", 1): os.path.join(ROOT, "profiles", "r05_roof_replay_c2.jsonl"),
                ("C4", 1): os.path.join(ROOT, "profiles", "r05_roof_replay_c4_128spp.jsonl"),
                ("C5", 1): os.path.join(ROOT, "profiles", "r05_roof_replay_c5_16spp.jsonl")}
# k_shade's algorithmic bytes (PATH integrator; the payload travels with the queues):
# every shaded path reads its pixel 4 and writes contrib 16 and meta 4 (k_accumulate reads the contrib
# entry back: 16); every traced closest-hit ray's direction 16, hit record 16 and, on a hit, the
# triangle's shading record 64 are read once -- at the camera bounce once per pixel, since the samples
# of a pixel share renderTile's pixel-centre ray and its hit (Renderer.h:805-808); a path past the
# camera bounce also reads its origin 16, throughput 16 and PCG state 8, which the previous shade
# wrote (16 + 16 + 16 + 8 with its direction); an NEE sample writes sh_o, sh_d 16 each and the path
# id 4. Scene records shared by many paths (materials, lights, texels) are not counted. The kernel
# time also holds k_generate (16 B per traced camera ray) and k_accumulate (meta 4 per path, the
# film once).
SHADE_B_PATH = 4 + 16 + 4 + 16
SHADE_B_HIT = 16 + 16 + 64
SHADE_B_CAM = 16
SHADE_B_META = 4
SHADE_B_CONT = (16 + 16 + 8) + (16 + 16 + 16 + 8)
SHADE_B_NEE = 16 + 16 + 4
ROOF_TABLE_MIB = 69  # the hot scene of C3: 21 MB wide nodes + 48 MB triangle records
HOT_BYTES_PER_TRI = 69.0  # wide nodes (~21 B per triangle on C3) + the 48-B triangle record
# per-ray queue id + ray origin + direction reads and the hit / visibility write (16-B requests)
REQ_PER_RAY_IO = 4.0


def request_ceiling(n_tris=None):
    """Best row of the ceiling microbenchmark on the table matching k_trace's hot scene: the
    smallest swept table that holds the scene's wide nodes + triangle records (C3: 69 MiB)."""
    try:
        rows = [json.loads(l) for l in open(ROOF_SWEEP) if l.strip().startswith("{")]
    except OSError:
        return None
    sizes = sorted({r["table_mib"] for r in rows if "table_mib" in r})
    if not sizes:
        return None
    mib = ROOF_TABLE_MIB
    if n_tris is not None:
        hot = n_tris * HOT_BYTES_PER_TRI / 1048576.0
        mib = next((m for m in sizes if m >= hot), sizes[-1])
    rows = [r for r in rows if r.get("table_mib") == mib]
    return max(rows, key=lambda r: r["g_lane_steps_per_s"]) if rows else None
# BASELINE.json configs: scene, size, spp, MAX_DEPTH. C1 is the CPU-only case.
CONFIGS = {
    "C2": {"scene": "cornell-box", "width": 1024, "height": 1024, "spp": 64, "depth": 8},
    "C3": {"scene": None, "width": 1024, "height": 1024, "spp": 64, "depth": 4},
    "C4": {"scene": "bathroom", "width": 1920, "height": 1080, "spp": 256, "depth": 16, "skip_missing": True},
    "C5": {"scene": "coffee", "width": 4096, "height": 4096, "spp": 1024, "depth": 4, "skip_missing": True,
           "envmap": "GI.hdr"},
}


def scene_dir(name):
    for base in (os.path.join(ROOT, "tests", "golden", "scenes"), os.path.join(ROOT, "assets"), "/root/reference/RTBase"):
        p = os.path.join(base, name)
        if os.path.isdir(p):
            return p
    raise SystemExit("scene %s not found (run __graft_entry__.build() where /root/reference exists)" % name)


class GroupRender:
    """The native one-process group (RayTracerGroup: rtg_group_* in rtg_multi.hip) behind the calls
    bench.py makes on a RayTracer: render = every rank renders its diagonal tile stripes on its own
    device, then the own-tile film exchange into devices[0]; stats are summed over the ranks. sync=False
    (the lean timed step) queues both: rtg_group_render_async (every rank's frame in its frame
    pipeline) and rtg_group_reduce_async (the exchange on its own streams, after each rank's frame),
    with no host wait; synchronize() waits for the ranks and the exchanges."""

    def __init__(self, scene, devices, max_depth, max_paths):
        from raytracingrenderer_amd import RayTracerGroup
        t0 = time.perf_counter()
        self.g = RayTracerGroup(scene, devices=devices, max_depth=max_depth, seed=1234, max_paths=max_paths)
        self.create_s = time.perf_counter() - t0
        self.devices = list(devices)
        self.reduce_ms = []
        self.last_ranks = []

    def set_options(self, flags):
        self.g.set_options(flags=flags)

    def clear(self):
        self.g.clear()

    def render(self, spp, tiles=None, first_sample=0, sync=True):
        self.g.render(spp, first_sample=first_sample, sync=sync)
        self.g.reduce(sync=sync)
        if sync:
            self.reduce_ms.append(self.g.reduce_ms())

    def synchronize(self):
        self.g.synchronize()

    def stats(self):
        self.last_ranks = self.g.rank_stats()
        return {k: (max if k == "chunk_samples" else sum)(r[k] for r in self.last_ranks) for k in self.last_ranks[0]}

    def film(self):
        return self.g.film()


def visible_devices():
    import ctypes as C
    from raytracingrenderer_amd import _native as N
    n = C.c_int(0)
    N.rtg().rtg_device_count(C.byref(n))
    return n.value


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    p.add_argument("--devices", default="",
                   help="comma-separated device list for the native group path (repeats rehearse ranks)")
    p.add_argument("--config", default="C3", choices=sorted(CONFIGS),
                   help="BASELINE.json config; C3 is the headline metric, the others are side measurements")
    # default K / W: about 10 s of timed GPU work on the headline config (the driver's utilisation
    # sampler sees a busy GPU), one or a few frames on the long configs
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=None)
    p.add_argument("--width", type=int, default=0, help="0 = the config's")
    p.add_argument("--height", type=int, default=0, help="0 = the config's")
    p.add_argument("--spp", type=int, default=0, help="0 = the config's")
    p.add_argument("--max-depth", type=int, default=-1, help="-1 = the config's")
    p.add_argument("--tris", type=int, default=1_000_000)
    p.add_argument("--seed", type=int, default=20251015)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--bvh2", action="store_true", help="force the reference BVH2 walk (A/B)")
    p.add_argument("--shard-of", type=int, default=0,
                   help="diagnostic: render only rank 0's tiles of this many ranks, on one GPU, to see the "
                        "per-GPU rate at that world size (value is then this GPU's rate, not a job total)")
    p.add_argument("--verify-film", action="store_true",
                   help="N>1: every tile re-rendered on one device, compared with the reduced film bit for bit")
    p.add_argument("--max-paths", type=int, default=0, help="paths per wavefront chunk (0 = library default)")
    p.add_argument("--dropin-frames", type=int, default=None,
                   help="frames of the drop-in leg (one 1-spp render call per frame, Main.cpp's loop); 0 = skip; "
                        "default 64 on C2 / C3, 0 otherwise")
    p.add_argument("--dropin-reps", type=int, default=3)
    p.add_argument("--step-mode", default="lean", choices=["lean", "full"],
                   help="lean: the timed steps are queued renders (rtg_render_async: consecutive frames overlap "
                        "in the frame pipeline) and their film exchanges, the ray counts read once after them, "
                        "the per-launch HIP events in a block of steps of their own; full: rounds 1-5's timed "
                        "step (film clear, a waited-for render with per-launch events, stats read back, per step)")
    a = p.parse_args()
    c = CONFIGS[a.config]
    if a.steps is None:
        a.steps = {"C2": 200, "C3": 120, "C4": 3, "C5": 1}[a.config]
    if a.warmup is None:
        a.warmup = {"C2": 5, "C3": 5, "C4": 1, "C5": 1}[a.config]
    if a.dropin_frames is None:
        a.dropin_frames = 64 if a.config in ("C2", "C3") and a.shard_of <= 1 else 0
    a.width = a.width or c["width"]
    a.height = a.height or c["height"]
    a.spp = a.spp or c["spp"]
    a.max_depth = c["depth"] if a.max_depth < 0 else a.max_depth
    return a


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # RTG_DIST_BACKEND=gloo rehearses the N>1 path on one GPU (ranks share cuda:0, the film exchange
    # goes through host memory); the default is RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("RTG_DIST_BACKEND", "nccl")
    if world > 1:
        import torch
        import torch.distributed as dist
        ndev = max(1, torch.cuda.device_count())
        local = local % ndev
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    coll_dev = "cuda:%d" % local if backend == "nccl" else "cpu"

    from raytracingrenderer_amd import RayTracer, loadScene, write_synthetic_scene
    from raytracingrenderer_amd import _native as N

    # one process, several GPUs: the native group (no torchrun)
    group_devs = None
    if world == 1 and (a.devices or a.gpus > 1):
        nvis = visible_devices()
        group_devs = [int(x) for x in a.devices.split(",")] if a.devices else list(range(a.gpus))
        if (not a.devices and a.gpus > nvis) or any(d < 0 or d >= nvis for d in group_devs):
            sys.stderr.write("bench.py: %s needs devices %s but %d HIP device(s) are visible; refusing to "
                             "measure fewer GPUs than asked (--devices 0,0,... rehearses ranks on one GPU)\n"
                             % ("--gpus %d" % a.gpus if not a.devices else "--devices " + a.devices, group_devs, nvis))
            sys.exit(2)

    # ---- scene (outside the timed region)
    cfg = CONFIGS[a.config]
    t0 = time.time()
    if cfg["scene"] is None:
        work = tempfile.mkdtemp(prefix="rtg_bench_r%d_" % rank)
        write_synthetic_scene(work, n_tris=a.tris, seed=a.seed, width=a.width, height=a.height)
        scene = loadScene(work)
    else:
        work = scene_dir(cfg["scene"])
        scene = loadScene(work, width=a.width, height=a.height,
                          skip_missing=cfg.get("skip_missing", False), envmap=cfg.get("envmap"))
    setup_s = time.time() - t0
    from raytracingrenderer_amd.distributed import FilmExchange, tiles_for_rank
    if group_devs is not None:
        rt = GroupRender(scene, group_devs, a.max_depth, a.max_paths)
        tiles = None  # the group partitions the tiles itself (rtg_tiles_for_rank)
    else:
        rt = RayTracer(scene, device=local, max_depth=a.max_depth, seed=1234, max_paths=a.max_paths)
        tiles = tiles_for_rank(a.width, a.height, rank, world)
        if a.shard_of > 1 and world == 1:
            tiles = tiles_for_rank(a.width, a.height, 0, a.shard_of)

    film_t = fx = None
    xch_ev = []  # (start, end) CUDA events around each timed step's film exchange (RCCL)
    if world > 1:
        import torch
        film_t = torch.zeros((a.height, a.width, 3), dtype=torch.float32, device=coll_dev)
        fx = FilmExchange(a.width, a.height, rank, world, device=coll_dev if backend == "nccl" else None)
    timing_xch = [False]

    queued = [False]  # lean timed steps: queued renders

    def step(clear=True):
        if clear:
            rt.clear()
        if queued[0]:
            rt.render(a.spp, tiles=tiles, first_sample=0, sync=False)
        else:
            rt.render(a.spp, tiles=tiles, first_sample=0)
        if world > 1:
            # own tiles -> rank 0 (pack, RCCL gather, scatter); timed with CUDA events on the exchange's
            # stream from the moment the frame is on the film (not while the queued render runs)
            ev = fx.exchange(rt, film_t, dist, timing=backend == "nccl" and timing_xch[0])
            if ev is not None:
                xch_ev.append(ev)

    def barrier_sync():
        if world > 1:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()
        else:
            rt.synchronize()

    base = N.RTG_OPT_CULL | (N.RTG_OPT_BVH2 if a.bvh2 else 0)
    rt.set_options(flags=base)
    for _ in range(a.warmup):
        step()
    # Timed region. lean (default): the steps' renders (and at N > 1 their film exchanges) queued back
    # to back on the device; the film is cleared once before the region (the renders add into it, as
    # RTBase's progressive film does) and the ray counts, which accumulate since that clear, are read
    # once after it. full (rounds 1-5): a film clear, a render with per-launch HIP events and a stats
    # read-back per step; those host syncs and event markers cost ~1.9 % of a shard-of-8 step and
    # ~0.5 % of C3's (profiles/r05_step_mode.txt).
    lean = a.step_mode == "lean"
    rt.set_options(flags=base | (0 if lean else N.RTG_OPT_TIMING))
    if lean:
        rt.clear()
        # each step's render is queued (rtg_render_async; the native group: rtg_group_render_async +
        # rtg_group_reduce_async): the host does not wait, and a render of up to 16M paths runs in the
        # frame pipeline, its traversal starting while the frame before it drains (its film fold
        # still after that frame's fold and film exchange)
        queued[0] = True
    timing_xch[0] = True
    ext_rays = shadow_rays = paths = cam_traced = chunk_spp = 0
    extend_ms = shadow_ms = shade_ms = 0.0
    extend_launches = 0
    timed_ranks = None

    def add_stats(st):
        nonlocal ext_rays, cam_traced, shadow_rays, paths, extend_ms, shadow_ms, shade_ms, extend_launches, chunk_spp
        ext_rays += st["extension_rays"]
        cam_traced += st["traced_camera_rays"]
        shadow_rays += st["shadow_rays"]
        paths += st["paths"]
        extend_ms += st["extend_ms"]
        shadow_ms += st["shadow_ms"]
        shade_ms += st["shade_ms"]
        extend_launches += st["extend_launches"]
        chunk_spp = max(chunk_spp, st.get("chunk_samples", 0))

    barrier_sync()
    t_start = time.perf_counter()
    for _ in range(a.steps):
        step(clear=not lean)
        if not lean:
            add_stats(rt.stats())
            timed_ranks = getattr(rt, "last_ranks", None)
    barrier_sync()
    elapsed = time.perf_counter() - t_start
    queued[0] = False
    timing_xch[0] = False
    kernel_timing = {"source": "per-launch HIP events on the render streams, in the timed steps"}
    if lean:
        add_stats(rt.stats())
        # the kernels' times: per-launch HIP events on the render streams over further steps of the
        # same workload (renders only), scaled to the timed steps
        rt.set_options(flags=base | N.RTG_OPT_TIMING)
        kt = min(a.steps, 10)
        k_ext = k_sh = k_sd = 0.0
        k_l = 0
        t_k = time.perf_counter()
        for _ in range(kt):
            rt.clear()
            rt.render(a.spp, tiles=tiles, first_sample=0)
            st = rt.stats()
            k_ext += st["extend_ms"]
            k_sh += st["shadow_ms"]
            k_sd += st["shade_ms"]
            k_l += st["extend_launches"]
        t_k = time.perf_counter() - t_k
        timed_ranks = getattr(rt, "last_ranks", None)
        rt.set_options(flags=base)
        f = a.steps / kt
        extend_ms, shadow_ms, shade_ms, extend_launches = k_ext * f, k_sh * f, k_sd * f, int(round(k_l * f))
        kernel_timing = {"source": "per-launch HIP events on the render streams over %d further steps of the same "
                                   "workload (renders only), scaled to the timed steps" % kt,
                         "steps": kt, "ms_per_step_with_events": round(t_k * 1e3 / kt, 3)}
    xch_ms = [e0.elapsed_time(e1) for e0, e1 in xch_ev]

    # shard-of-N projection: the exchange a rank of N adds to its render, rehearsed on this GPU (the
    # pack of rank 0's pixels, the scatter rank 0 runs over all N ranks' pixels) plus a model of the
    # RCCL transfer (rank 0 receives N-1 packed buffers concurrently, one per xGMI link)
    shard_exchange = None
    if world == 1 and group_devs is None and a.shard_of > 1:
        shard_exchange = rehearse_exchange(rt, a)

    # the drop-in frame loop (Main.cpp:74-118): one RayTracer::render() = one rtg call of 1 spp
    # (without the per-launch timing events, which keep one chunk in flight)
    dropin = None
    if world == 1 and group_devs is None and a.dropin_frames > 0:
        dropin = dropin_leg(rt, a, tiles, base)

    # counting passes (untimed): box / triangle tests per closest-hit ray on the same workload.
    # Algorithmic work is the reference's BVH2 walk; the 4-wide walk's own tests are reported too.
    def count(flags):
        rt.set_options(flags=flags | N.RTG_OPT_COUNT)
        rt.clear()
        rt.render(a.spp, tiles=tiles, first_sample=0)
        return rt.stats()
    cs = count(N.RTG_OPT_CULL | N.RTG_OPT_BVH2)
    cw = cs if a.bvh2 else count(base)
    rt.set_options(flags=base)

    film_check = None
    group_reduced = None
    if group_devs is not None and a.verify_film:
        # the lean step's path: two queued frames, each followed by a queued exchange
        rt.clear()
        for _ in range(2):
            rt.render(a.spp, first_sample=0, sync=False)
        group_reduced = rt.film()[0]  # checked against one handle once the group is released
    if world > 1 and a.verify_film:
        step()  # a fresh reduced film
        barrier_sync()
        if rank == 0:
            reduced = film_t.cpu().numpy() if backend == "nccl" else film_t.numpy()
            rt.clear()
            rt.render(a.spp, tiles=None, first_sample=0)
            solo = rt.film()[0]
            film_check = bool(np.array_equal(reduced.view(np.uint32), solo.view(np.uint32)))
        barrier_sync()

    local_kernel_ms = (extend_ms, shadow_ms, shade_ms)
    group_info = None
    if group_devs is not None:
        r0 = timed_ranks[0] if timed_ranks else {}
        local_kernel_ms = (r0.get("extend_ms", 0.0) * a.steps, 0.0, r0.get("shade_ms", 0.0) * a.steps)
        prep_ms, up_ms = rt.g.setup_ms()
        # waited-for exchanges: the timed steps' (full), or the kernel-timing steps' after them (lean)
        timed_reduce = rt.reduce_ms[-min(a.steps, 10):] if lean else rt.reduce_ms[a.warmup:a.warmup + a.steps]
        group_info = {"devices": group_devs, "distinct_gpus": len(set(group_devs)), "uses_rccl": rt.g.uses_rccl,
                      "setup_ms": {"create_total": round(rt.create_s * 1e3, 1), "host_build": round(prep_ms, 1),
                                   "parallel_uploads": round(up_ms, 1)},
                      "reduce_ms_per_step": round(float(np.mean(timed_reduce)), 3) if timed_reduce else None,
                      "rank_kernel_ms_last_step": [{"trace": round(r["extend_ms"], 2), "shade": round(r["shade_ms"], 2),
                                                    "render": round(r["render_ms"], 2)} for r in timed_ranks]}
        rms = [r["render_ms"] for r in timed_ranks if r["render_ms"] > 0]
        if rms:
            # balance of the tile partition: the slowest rank's render over the mean (device time of
            # each rank's last render; rehearsed ranks on one device get equal chunk budgets)
            group_info["rank_render_ms"] = {"max": round(max(rms), 2), "mean": round(float(np.mean(rms)), 2),
                                            "max_over_mean": round(max(rms) / float(np.mean(rms)), 4)}
        if len(set(group_devs)) > 1:
            group_info["note"] = ("distinct-device group: ranks render concurrently, own tiles sent to device 0 by RCCL; "
                                  "film_reduce_bit_exact (--verify-film) is its check on this run")
        group_parallelism = ("tile-sharded x%d, one process (rtg_group: a handle and host thread per device) + "
                             "own-tile film exchange over %s" % (len(group_devs), "RCCL ncclSend/ncclRecv" if rt.g.uses_rccl
                                                                 else "device copies (repeated devices)"))
        if group_reduced is not None:
            # the group's device memory goes first (ranks rehearsed on one device hold a chunk each)
            del rt
            import gc
            gc.collect()
            solo = RayTracer(scene, device=group_devs[0], max_depth=a.max_depth, seed=1234, max_paths=a.max_paths)
            for _ in range(2):
                solo.render(a.spp, first_sample=0)
            film_check = bool(np.array_equal(group_reduced.view(np.uint32), solo.film()[0].view(np.uint32)))
            del solo
    # rays traced: renderTile's camera ray is the pixel centre's for every sample (Renderer.h:805-808),
    # so the bounce-0 traversal traces one per pixel and the samples share its hit; the counts of
    # the reference (extension_rays: one camera ray per sample) are what `value` is quoted on
    def traced_ext(st_):
        return st_["extension_rays"] - st_["paths"] + st_["traced_camera_rays"]
    # bytes the walk itself fetches per counting pass: a 64-B node record per node step (wide or BVH2),
    # a triangle's first 32 B per test and its last 16 B when its plane distance is a candidate, a 32-B
    # leaf box per candidate hit, and 48 B of ray I/O per ray (origin + direction in, result out)
    fetched = (64.0 * cw["node_lane_steps"] + 32.0 * (cw["tri_tests"] + cw["shadow_tri_tests"])
               + 16.0 * cw["tri_tail_loads"] + 32.0 * cw["leafbox_tests"] + 48.0 * (traced_ext(cw) + cw["shadow_rays"]))
    totals = np.array([ext_rays, shadow_rays, paths, extend_ms, extend_launches,
                       cs["node_visits"], cs["tri_tests"], traced_ext(cs),
                       cw["node_visits"], cw["tri_tests"],
                       cs["shadow_node_visits"], cs["shadow_tri_tests"], cs["shadow_rays"],
                       ext_rays - paths + cam_traced,
                       traced_ext(cw), cw["shadow_node_visits"], cw["shadow_tri_tests"], cw["shadow_rays"], fetched],
                      dtype=np.float64)
    t_max = elapsed
    if world > 1:
        import torch
        tt = torch.tensor(totals, dtype=torch.float64, device=coll_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        totals = tt.cpu().numpy()
        te = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        t_max = float(te.item())
    (ext_rays, shadow_rays, paths, extend_ms, extend_launches, c_nodes, c_tris, c_ext, w_nodes, w_tris,
     s_nodes, s_tris, c_sh, ext_traced, w_ext, ws_nodes, ws_tris, w_sh, w_fetched) = totals.tolist()
    rays = ext_rays + shadow_rays
    rays_traced = ext_traced + shadow_rays
    mrays = rays / t_max / 1e6  # the reference's ray count (a camera ray per sample)
    mrays_traced = rays_traced / t_max / 1e6
    ms_step = t_max * 1e3 / a.steps
    if shard_exchange is not None:
        # the job at N GPUs: every rank renders its share (rank 0's share stands for all: diagonal
        # stripes are balanced to ~2 %) and rank 0 assembles the film
        job_ms = ms_step + shard_exchange["total_ms"]
        shard_exchange["projected_job_ms_per_step"] = round(job_ms, 3)
        shard_exchange["projected_job_mrays_traced_per_s"] = round(rays_traced * a.shard_of / (job_ms / 1e3 * a.steps) / 1e6, 1)
    if dropin is not None:
        dropin["batched_ms_per_frame"] = round(ms_step / a.spp, 4)
        dropin["queued_over_batched"] = round(dropin["queued"]["ms_per_frame"] / (ms_step / a.spp), 3)

    # roofline for the dominant kernel, k_trace (one launch per bounce traces the extension rays of
    # bounce b and the shadow rays of bounce b-1). Its limiter is the memory system's throughput of
    # dependent random per-lane record fetches: a node step fetches its own 64-B record (four 16-B
    # loads) at an address the previous step produced, a triangle test its 48-B record's first 32 B,
    # a candidate hit its leaf box: each a line no lane of the wave needed a step earlier. (A
    # triangle's last 16 B, fetched when its plane distance is a candidate, lie in the head's line
    # in 6 of 8 records, and the per-ray queue / ray reads are coalesced: reported, not counted.) The
    # ceiling microbenchmark (tools/micro/roof.hip: dependent random 64-B records, 69 MiB table = the
    # hot scene, k_trace's occupancy) reaches ~162 G such fetches/s, flat from 2 to 16 waves per
    # SIMD and only 13 % higher for 32-B records, so fetches, not bytes or 16-B
    # requests, set the pace. achieved = the walk's fetches (counted on the same workload by the
    # untimed counting pass) / the k_trace HIP-event time of the timed region. The 16-B request
    # form of the same roofline is kept as a sub-object.
    n_steps = a.steps
    all_rays = traced_ext(cw) + cw["shadow_rays"]  # rays the traversal processed
    rec_step = cw["node_lane_steps"] + cw["tri_tests"] + cw["shadow_tri_tests"] + cw["leafbox_tests"]
    req_step = (4.0 * cw["node_lane_steps"] + 2.0 * (cw["tri_tests"] + cw["shadow_tri_tests"])
                + cw["tri_tail_loads"] + 2.0 * cw["leafbox_tests"] + REQ_PER_RAY_IO * all_rays)
    req_totals = np.array([req_step * n_steps, rec_step * n_steps], dtype=np.float64)
    # SURVEY.md §8d algorithmic bytes B_ray = 32 B x AABB tests + 36 B x triangle tests + 48 B ray I/O,
    # "the AABB and triangle counts measured by the build's counting mode on the config's exact input":
    # the box / triangle tests of the walk k_trace runs (the 4-wide tree's slot tests, triangle tests),
    # counted on the same workload. These bytes are served by L1 / L2 / Infinity Cache (the hot scene
    # is ~70 MB), so the peak they are held to is the L2 bandwidth.
    boxes_per_ray = w_nodes / max(w_ext, 1)
    tris_per_ray = w_tris / max(w_ext, 1)
    b_ray = 32.0 * boxes_per_ray + 36.0 * tris_per_ray + 48.0
    s_boxes_per_ray = ws_nodes / max(w_sh, 1)
    s_tris_per_ray = ws_tris / max(w_sh, 1)
    b_sray = 32.0 * s_boxes_per_ray + 36.0 * s_tris_per_ray + 48.0
    # time and rays both summed over ranks and launches
    algo_gbs = (b_ray * ext_traced + b_sray * shadow_rays) / (extend_ms / 1e3) / 1e9 if extend_ms > 0 else None
    # the same formula with the reference's own BVH2 walk's counts (rounds 1-5's headline): the bytes
    # RTBase's traversal would test, not what this walk fetches
    r_b_ray = 32.0 * c_nodes / max(c_ext, 1) + 36.0 * c_tris / max(c_ext, 1) + 48.0
    r_b_sray = 32.0 * s_nodes / max(c_sh, 1) + 36.0 * s_tris / max(c_sh, 1) + 48.0
    ref_gbs = (r_b_ray * ext_traced + r_b_sray * shadow_rays) / (extend_ms / 1e3) / 1e9 if extend_ms > 0 else None
    # the bytes this walk requests (node records, triangle heads / tails, leaf boxes, ray I/O)
    fetched_per_ray = w_fetched / max(w_ext + w_sh, 1)
    fetched_gbs = fetched_per_ray * (ext_traced + shadow_rays) / (extend_ms / 1e3) / 1e9 if extend_ms > 0 else None
    if world > 1:
        import torch
        rt_ = torch.tensor(req_totals, dtype=torch.float64, device=coll_dev)
        dist.all_reduce(rt_, op=dist.ReduceOp.SUM)
        req_totals = rt_.cpu().numpy()
    achieved_req = req_totals[0] / (extend_ms / 1e3) / 1e9 if extend_ms > 0 else None
    achieved_rec = req_totals[1] / (extend_ms / 1e3) / 1e9 if extend_ms > 0 else None
    ceiling = request_ceiling(scene.desc.n_tris)
    avg_launch_s = extend_ms / max(extend_launches, 1) / 1e3
    # profiles/ evidence for the profiled workloads (each config's bench line, one GPU, the whole film):
    # PMC traffic and kernel-trace durations; other shapes / shards / N > 1 report null
    traffic = pmc = None
    pmc_path = None
    c_def = CONFIGS[a.config]
    profiled = (world == 1 and group_devs is None and a.shard_of <= 1 and a.tris == 1_000_000
                and (a.width, a.height) == (c_def["width"], c_def["height"]) and a.max_depth == c_def["depth"])
    for path in (PMC_SUMMARIES[a.config],) + ((PMC_SUMMARY,) if a.config == "C3" else ()):
        if not profiled or pmc is not None or not os.path.exists(path):
            continue
        try:
            pj = json.load(open(path))
        except Exception:
            continue
        if pj.get("spp", 64 if path == PMC_SUMMARY else None) == a.spp:
            pmc, pmc_path = pj, path
            traffic = pj.get("extend_hbm_bytes_per_launch")
    replay = None
    # (a rank of N renders rank 0's share of an N-way split up to the diagonal offset: shard-of N's ceiling)
    replay_file = ROOF_REPLAYS.get((a.config, max(a.shard_of, world, 1))) if group_devs is None else None
    if replay_file and os.path.exists(replay_file):
        try:
            replay = [json.loads(l) for l in open(replay_file) if '"total"' in l][-1]
        except Exception:
            replay = None
    # a replay taken at another chunk shape walks other rays: it is not this line's ceiling
    replay_shape_ok = bool(replay) and replay.get("chunk_spp") == chunk_spp and a.tris == 1_000_000
    # k_shade: algorithmic payload bytes per step (SHADE_B_*) / its kernel time (the timed region's
    # generate + shade + accumulate HIP events), and the PMC DRAM-level bytes of its launches
    shaded = ext_rays  # every closest-hit ray's result is shaded once
    cont = max(ext_rays - paths, 0)  # continuing paths = extension rays after the camera rays
    shade_algo_bytes = (shaded * SHADE_B_PATH + (cont + cam_traced) * SHADE_B_HIT + cont * SHADE_B_CONT
                        + shadow_rays * SHADE_B_NEE + cam_traced * SHADE_B_CAM + paths * SHADE_B_META
                        + 12.0 * a.width * a.height * 2 * a.steps)
    shade_algo_gbs = shade_algo_bytes / (shade_ms / 1e3) / 1e9 if shade_ms > 0 else None
    shade_pmc = None
    if pmc:
        ks = [v for k, v in pmc.get("kernels", {}).items() if k.startswith("void k_shade<false")]
        if ks and ks[0].get("avg_ns_trace"):
            kb = ks[0]["read_bytes_corrected"] + ks[0]["write_bytes"]
            shade_pmc = {"bytes_per_launch": kb, "avg_launch_ms": round(ks[0]["avg_ns_trace"] / 1e6, 4),
                         "achieved_gbs": round(kb / (ks[0]["avg_ns_trace"] / 1e9) / 1e9, 1)}

    # VALU issue of the two hot kernels against the chip's wave64 issue peak (C3 PMC passes, profiles/)
    valu = {}
    if profiled and a.config == "C3" and a.spp == 64 and os.path.exists(VALU_ISSUE):
        try:
            vj = json.load(open(VALU_ISSUE))
            for key, name in (("trace", "k_trace<false, false>"), ("shade", "k_shade<false, ...>")):
                kv = vj["kernels"].get(name)
                if kv:
                    valu[key] = {"achieved": kv["achieved_g_per_s"], "peak": vj["peak_g_per_s"],
                                 "unit": "G wave64 VALU instructions/s", "frac": kv["frac"],
                                 "per_wave": kv["valu_per_wave"],
                                 "source": "%s: SQ_INSTS_VALU over the kernel's dispatch time, rocprofv3 --pmc; peak "
                                           "= 256 CUs x 4 SIMD-32 x 2.4 GHz / 2 cycles per wave64 instruction "
                                           "(MI355X_MICROARCH.md); from profiles/, not measured in this run"
                                           % os.path.relpath(VALU_ISSUE, ROOT)}
        except Exception:
            valu = {}

    cpu = None
    if rank == 0 and world == 1 and group_devs is None and not a.no_cpu_baseline:
        cpu = cpu_baseline(scene, a, work)

    if rank == 0:
        out = {
            "metric": ("Mray/s (traced closest-hit + shadow rays) at 1024x1024x64spp, synthetic 1M triangles"
                       if a.config == "C3" else "Mray/s (traced closest-hit + shadow rays), config %s" % a.config),
            "value": round(mrays_traced, 2),
            "unit": "Mray/s",
            "n_gpus": world if group_devs is None else len(set(group_devs)),
            **({"ranks": len(group_devs)} if group_devs is not None else {}),
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_step, 3),
            "ms_per_frame": round(ms_step / a.spp, 4),
            "mpaths_per_s": round(paths / t_max / 1e6, 2),
            "rays_per_path": round(rays / max(paths, 1), 4),
            "rays_traced_per_path": round(rays_traced / max(paths, 1), 4),
            "mrays_traced_per_s": round(mrays_traced, 2),
            "mrays_reference_equivalent_per_s": round(mrays, 2),
            "rays_note": ("value counts the rays the traversal traced. renderTile casts the pixel-centre camera "
                          "ray for every sample (Renderer.h:805-808), so the GPU traces it once per pixel per "
                          "chunk and the samples share its hit (same film bits); "
                          "mrays_reference_equivalent_per_s counts it once per sample, as the reference casts "
                          "it (rays_per_path)"),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic (splitmix64 random triangles, generated in-run)" if cfg["scene"] is None
                     else "reference scene assets (%s%s)" % (cfg["scene"], ", filtered" if cfg.get("skip_missing") else "")),
            **({"shard_of": a.shard_of} if a.shard_of > 1 else {}),
            "config": {"workload": "%s: %s, %dx%d, %d spp, MAX_DEPTH %d" % (
                           a.config, "synth-1M" if cfg["scene"] is None else cfg["scene"] + ("_f" if cfg.get("skip_missing") else ""),
                           a.width, a.height, a.spp, a.max_depth),
                       "triangles": scene.desc.n_tris, "width": a.width, "height": a.height, "spp": a.spp,
                       "chunk_spp": chunk_spp,
                       "max_depth": a.max_depth,
                       "parallelism": (group_parallelism if group_devs is not None else
                                       "tile-sharded x%d (torchrun ranks) + own-tile film exchange over %s"
                                       % (world, "RCCL" if backend == "nccl" else backend) if world > 1 else
                                       "one GPU rendering rank 0's tiles of %d (shard-of diagnostic, no exchange)" % a.shard_of
                                       if a.shard_of > 1 else "one GPU, every tile (no exchange)")},
            # headline roofline: a hardware peak. SURVEY.md 8d's algorithmic bytes of k_trace (with the
            # box / triangle tests of the walk it runs) per launch / its average launch time, against
            # the L2 aggregate bandwidth that serves them (the ~70 MB hot scene lives in L2 + Infinity
            # Cache; the PMC-measured HBM bytes are `traffic`). frac_hw: the bytes the walk actually
            # requests (node records, triangle heads and tails, leaf boxes, ray I/O) against the same
            # peak. The walk's limiter, dependent random record fetches, is priced in `fetches`.
            "roofline": {"bound": "l2", "kernel": "k_trace (extension + shadow rays)",
                         "achieved": None if algo_gbs is None else round(algo_gbs, 1),
                         "peak": L2_PEAK_GBS, "unit": "GB/s",
                         "frac": None if algo_gbs is None else round(algo_gbs / L2_PEAK_GBS, 4),
                         "frac_hw": None if fetched_gbs is None else round(fetched_gbs / L2_PEAK_GBS, 4),
                         "peak_is": "MI355X aggregate L2 bandwidth, /opt/skills/guides/MI355X_MICROARCH.md (L2 per XCD)",
                         "definition": ("SURVEY.md 8d: 32 B x box tests + 36 B x triangle tests + 48 B per ray, with the "
                                        "box (4-wide slot) and triangle tests of the walk k_trace runs, counted on this "
                                        "workload by RTG_OPT_COUNT; per launch = bytes of the launch's rays / avg_launch_ms"),
                         "bytes_per_ray": round(b_ray, 1), "bytes_per_shadow_ray": round(b_sray, 1),
                         "box_tests_per_ray": round(boxes_per_ray, 2), "tri_tests_per_ray": round(tris_per_ray, 2),
                         "shadow_box_tests_per_ray": round(s_boxes_per_ray, 2),
                         "shadow_tri_tests_per_ray": round(s_tris_per_ray, 2),
                         "fetched": {"achieved": None if fetched_gbs is None else round(fetched_gbs, 1),
                                     "bytes_per_ray": round(fetched_per_ray, 1),
                                     "frac_of_l2_peak": None if fetched_gbs is None else round(fetched_gbs / L2_PEAK_GBS, 4),
                                     "definition": "bytes the walk requests: 64 B per node step, 32 B per triangle test "
                                                   "+ 16 B per triangle tail, 32 B per leaf box, 48 B of ray I/O per ray"},
                         "reference_bvh2_bytes": {
                             "achieved": None if ref_gbs is None else round(ref_gbs, 1),
                             "bytes_per_ray": round(r_b_ray, 1), "bytes_per_shadow_ray": round(r_b_sray, 1),
                             "box_tests_per_ray": round(c_nodes / max(c_ext, 1), 2),
                             "tri_tests_per_ray": round(c_tris / max(c_ext, 1), 2),
                             "ratio_to_l2_peak": None if ref_gbs is None else round(ref_gbs / L2_PEAK_GBS, 4),
                             "ratio_to_hbm_peak": None if ref_gbs is None else round(ref_gbs / HBM_PEAK_GBS, 4),
                             "why_not_a_fraction": ("the same 8d formula with the box / triangle tests of the reference's "
                                                    "BVH2 walk (culled, counted by RTG_OPT_BVH2 on this workload): the bytes "
                                                    "RTBase's traversal would test, not what k_trace fetches, so the rate can "
                                                    "exceed a hardware peak (rounds 1-5 quoted it as the headline)")},
                         "avg_launch_ms": round(avg_launch_s * 1e3, 4),
                         "traffic": traffic,
                         "traffic_source": (None if traffic is None else
                                            "%s: rocprofv3 PMC (FETCH_SIZE x1 for the gathers + WRITE_SIZE, DRAM share) "
                                            "of this workload in separate passes; from profiles/, not measured in this run"
                                            % os.path.relpath(pmc_path, ROOT)),
                         "hbm": {"bytes_per_launch": traffic,
                                 "achieved_gbs": round(traffic / avg_launch_s / 1e9, 1) if traffic and extend_ms > 0 else None,
                                 "peak_gbs": HBM_PEAK_GBS,
                                 "frac": (round(traffic / avg_launch_s / 1e9 / HBM_PEAK_GBS, 4)
                                          if traffic and extend_ms > 0 else None),
                                 "source": "PMC (traffic_source)"},
                         # the measured limiter: dependent random per-lane record fetches
                         "fetches": {
                             "achieved": None if achieved_rec is None else round(achieved_rec, 1),
                             "unit": "G dependent random per-lane record fetches/s (node steps + triangle heads + leaf boxes)",
                             "per_ray": round(rec_step / max(all_rays, 1), 2),
                             "uniform_random_ceiling": (None if ceiling is None else
                                                        {"peak": round(ceiling["g_lane_steps_per_s"], 1),
                                                         "frac": (round(achieved_rec / ceiling["g_lane_steps_per_s"], 4)
                                                                  if achieved_rec else None),
                                                         "source": "tools/micro/roof.hip, %s: dependent random 64-B per-lane "
                                                                   "records, %d MiB table, %d VALU/step (microbenchmark)"
                                                                   % (os.path.relpath(ROOF_SWEEP, ROOT), ceiling["table_mib"],
                                                                      ceiling["valu_per_step"])}),
                             # not a ceiling: the replay serialises each ray's captured fetches with 8
                             # dependent VALU each; the walk overlaps parked-leaf triangle fetches with
                             # node steps and runs faster than it on C3 and C4
                             "replay_reference": (None if not replay else
                                                {"rate": round(replay["ceiling_g_fetches_per_s"], 1),
                                                 "ratio_vs_replay": (round(achieved_rec / replay["ceiling_g_fetches_per_s"], 4)
                                                                     if achieved_rec and replay_shape_ok else None),
                                                 "chunk_spp": replay.get("chunk_spp"),
                                                 "matches_line_chunk": replay_shape_ok,
                                                 "k_trace_ms": round(replay["k_trace_ms"], 2),
                                                 "replay_ms": round(replay["replay_ms"], 2),
                                                 "replayed_fetches": replay["replayed_fetches"],
                                                 "frac_at_measurement": round(replay["frac"], 4),
                                                 "source": ("this workload's own fetch stream captured and replayed with "
                                                            "nothing else in the loop (tools/roof_replay.py); read from %s, "
                                                            "a stored profile, not measured in this run; a reference rate, "
                                                            "not a bound (the walk can run faster: ratio above 1)"
                                                            % os.path.relpath(replay_file, ROOT))}),
                             "requests": {"achieved": None if achieved_req is None else round(achieved_req, 1),
                                          "peak": None if ceiling is None else round(ceiling["g_req_per_s"], 1),
                                          "unit": "G 16-B vector-memory requests/s",
                                          "frac": (round(achieved_req / ceiling["g_req_per_s"], 4)
                                                   if achieved_req and ceiling else None),
                                          "per_ray": round(req_step / max(all_rays, 1), 2)},
                             "tri_tail_loads_per_ray": round(cw["tri_tail_loads"] / max(all_rays, 1), 2),
                             "leafbox_tests_per_ray": round(cw["leafbox_tests"] / max(all_rays, 1), 2)},
                         "valu": valu.get("trace"),
                         "walk": "bvh2" if a.bvh2 else "bvh4 (collapsed from an own SAH tree over the triangles with spatial splits, one triangle per leaf slot)",
                         "walk_box_tests_per_ray": round(w_nodes / max(c_ext, 1), 2),
                         "walk_tri_tests_per_ray": round(w_tris / max(c_ext, 1), 2),
                         "node_steps_per_ray": round(cw["node_lane_steps"] / max(all_rays, 1), 2),
                         "pops_per_ray": round(cw["pops"] / max(traced_ext(cw), 1), 2),
                         "cullable_pops_per_ray": round(cw["cullable_pops"] / max(traced_ext(cw), 1), 2),
                         # node: lanes stepping a node per loop iteration; leaf: lanes running a
                         # parked leaf per leaf phase; leaf phases per iteration
                         "lane_util_node_leaf": [round(cw["node_lane_steps"] / max(cw["lane_slots"], 1), 3),
                                                 round(cw["leaf_lane_steps"] / max(cw["leaf_phase_slots"], 1), 3),
                                                 round(cw["leaf_phase_slots"] / max(cw["lane_slots"], 1), 3)],
                         # the lanes not stepping a node, by reason, as fractions of lane_slots
                         "lane_idle_node": {k: round(cw.get("lane_idle_" + k, 0) / max(cw["lane_slots"], 1), 4)
                                            for k in ("no_ray", "last_leaf", "leaf_blocked", "retiring", "leaf_popped")}},
            "roofline_shade": {"bound": "hbm", "kernel": "k_shade (+ k_generate, k_accumulate in the time)",
                               "achieved": None if shade_algo_gbs is None else round(shade_algo_gbs, 1),
                               "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": None if shade_algo_gbs is None else round(shade_algo_gbs / HBM_PEAK_GBS, 4),
                               "algorithmic_bytes_per_step": round(shade_algo_bytes / max(a.steps, 1)),
                               "definition": "per shaded path %d B (pixel read, contrib/meta writes, contrib read-back), "
                                             "+%d B per traced closest-hit ray (direction, hit, shading record: at the camera "
                                             "bounce once per pixel, shared by its samples), +%d B per path past the camera "
                                             "bounce (its payload written by one shade, read by the next), +%d B per NEE sample; "
                                             "scene records shared by paths not counted; + %d B per traced camera ray (k_generate), "
                                             "%d B per path (k_accumulate's meta) and the film read + write"
                                             % (SHADE_B_PATH, SHADE_B_HIT, SHADE_B_CONT, SHADE_B_NEE, SHADE_B_CAM, SHADE_B_META),
                               "valu": valu.get("shade"),
                               "pmc": shade_pmc,
                               "pmc_source": (None if shade_pmc is None else "%s (k_shade<false>, DRAM-level bytes "
                                              "FETCH_SIZE x2 + WRITE_SIZE per launch, rocprof kernel-trace duration); "
                                              "from profiles/, not measured in this run" % os.path.relpath(pmc_path, ROOT))},
            "kernel_ms_per_step_rank0": {"trace": round(local_kernel_ms[0] / a.steps, 2),
                                         "generate_shade_accumulate": round(local_kernel_ms[2] / a.steps, 2)},
            "timed_step": ("lean: queued renders (frame pipeline)%s, film cleared once before, ray counts read once "
                           "after" % (" + film exchanges" if world > 1 else "")) if lean else
                          "full: film clear + render with per-launch events + stats read-back per step",
            "kernel_timing": kernel_timing,
            "cpu_baseline": cpu,
            # one unit on both sides: the CPU's rays are the reference's (a camera ray per sample), so
            # they compare with mrays_reference_equivalent_per_s, not with `value` (traced rays); and
            # ms per 1-spp frame of the same film
            **({"gpu_over_cpu": {"ms_per_frame": round(cpu["ms_per_frame"] / (ms_step / a.spp), 1),
                                 "reference_equivalent_mrays": round(mrays / cpu["value"], 1),
                                 "note": "CPU: %d host threads (cores); same scene, film size and MAX_DEPTH"
                                         % cpu["cores"]}}
               if cpu and cpu.get("value") and cpu.get("ms_per_frame") else {}),
            **({"dropin": dropin} if dropin is not None else {}),
            **({"film_reduce_bit_exact": film_check} if film_check is not None else {}),
            **({"exchange_ms_per_step": {"mean": round(float(np.mean(xch_ms)), 3), "max": round(float(np.max(xch_ms)), 3),
                                         "bytes_per_rank": fx.maxpix * 12,
                                         "what": "rank %d: own-tile pack + RCCL gather to rank 0 + scatter (CUDA events "
                                                 "on the exchange stream, from the frame's fold to the scatter)" % rank}}
               if xch_ms else {}),
            **({"shard_exchange": shard_exchange} if shard_exchange is not None else {}),
            **({"group": group_info} if group_info is not None else {}),
            "setup_s": round(setup_s, 2),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def dropin_leg(rt, a, tiles, base_flags):
    """C3 through the drop-in frame loop: RTBase's Main.cpp calls RayTracer::render() once per frame
    (Main.cpp:74-118), and render() adds one sample per pixel (Renderer.h:876-885). Each frame here
    is one 1-spp librtg call, a.dropin_frames frames per repetition, under three host policies:
      queued      rtg_render_async(1 spp) per frame (what integration/rtg_rtbase.h's rtg_render_frame
                  does), the film read back once at the end (saveHDR): consecutive queued frames are
                  coalesced (16 per chunk on a 1-Mpixel film) and chunks overlap on the GPU
      queued_each the same with RTG_OPT_NO_COALESCE: every 1-spp call issued at once as its own chunk,
                  up to three in flight on their own streams
      sync        rtg_render(1 spp) per frame (returns when the frame is on the film), one read at the end
      sync_read   rtg_render + rtg_film_read (12.6 MB D2H) every frame: round 3's rtg_render_frame
    The film of every policy is compared bit for bit with one batched render of the same samples."""
    from raytracingrenderer_amd import _native as N
    F = a.dropin_frames
    out = {"frames_per_rep": F, "reps": a.dropin_reps, "spp_per_call": 1,
           "reference": "Main.cpp:74-118 frame loop, RayTracer::render() = 1 spp (Renderer.h:876-885)"}
    rt.clear()
    rt.render(F, tiles=tiles, first_sample=0)
    batch_film = rt.film()[0].view(np.uint32).copy()

    def run(policy):
        rt.set_options(flags=base_flags | (N.RTG_OPT_NO_COALESCE if policy == "queued_each" else 0))
        best = None
        same = True
        rays = 0
        for _ in range(a.dropin_reps):
            rt.clear()
            rt.synchronize()
            t0 = time.perf_counter()
            for f in range(F):
                rt.render(1, tiles=tiles, first_sample=f, sync=policy.startswith("sync"))
                if policy == "sync_read":
                    rt.film()
            film = rt.film()[0]
            dt = time.perf_counter() - t0
            st = rt.stats()
            rays = st["extension_rays"] - st["paths"] + st["traced_camera_rays"] + st["shadow_rays"]  # traced
            same = same and bool(np.array_equal(film.view(np.uint32), batch_film))
            best = dt if best is None or dt < best else best
        return {"ms_per_frame": round(best * 1e3 / F, 4), "mrays_per_s": round(rays / best / 1e6, 1),
                "film_equals_batched": same}
    for pol in ("queued", "queued_each", "sync", "sync_read"):
        out[pol] = run(pol)
    rt.set_options(flags=base_flags)
    out["batched_ms_per_frame"] = None  # filled by the caller (ms_per_step / spp of the headline)
    return out


XGMI_LINK_GBS = 76.5   # one direction of one xGMI link (~153 GB/s per link, both directions): a model
RCCL_P2P_US = 25.0     # per send/recv round on xGMI, small messages (model)


def rehearse_exchange(rt, a, reps=20):
    """The film exchange a rank of a.shard_of adds to its render, on this GPU: rtg_film_gather of
    rank 0's own pixels (every rank runs it, concurrently) and rtg_film_scatter of all ranks' pixels
    into the film (rank 0), timed with CUDA events (median of `reps`); the RCCL transfer between
    them is modelled: rank 0 receives N-1 buffers of maxpix x 12 B at once, one per xGMI link."""
    import ctypes as C
    import torch
    from raytracingrenderer_amd import _native as N
    from raytracingrenderer_amd.distributed import FilmExchange
    n = a.shard_of
    fx = FilmExchange(a.width, a.height, 0, n, device="cuda:0")
    film = torch.zeros((a.height, a.width, 3), dtype=torch.float32, device="cuda:0")
    rt.synchronize()
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def timed(fn):
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))
    g_ms = timed(lambda: N.rtg().rtg_film_gather(rt.handle, C.c_void_p(fx.t_own.data_ptr()), fx.maxpix,
                                                   C.c_void_p(fx.recv[0].data_ptr()), stream))
    s_ms = timed(lambda: N.rtg().rtg_film_scatter(0, C.c_void_p(fx.recv.data_ptr()), C.c_void_p(fx.t_all.data_ptr()),
                                                    len(fx.all), C.c_void_p(film.data_ptr()), a.width * a.height, stream))
    msg = fx.maxpix * 12
    x_ms = (msg / (XGMI_LINK_GBS * 1e9)) * 1e3 + RCCL_P2P_US / 1e3
    return {"ranks": n, "bytes_per_rank": msg, "gather_ms": round(g_ms, 4), "scatter_ms": round(s_ms, 4),
            "xgmi_model_ms": round(x_ms, 4), "total_ms": round(g_ms + s_ms + x_ms, 4),
            "model": "RCCL transfer modelled as %d B over one xGMI link at %.1f GB/s + %.0f us (rank 0 receives the "
                     "N-1 buffers on N-1 links at once); gather and scatter measured on this GPU"
                     % (msg, XGMI_LINK_GBS, RCCL_P2P_US)}


def host_cores():
    """Host cores this process may use: the CPU affinity set, capped by a cgroup CPU quota and by
    OMP_NUM_THREADS (the GPU box sets it to the job's CPU share; os.cpu_count() there shows the
    whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(float(quota) / float(period))))
    except Exception:
        pass
    try:
        n = min(n, int(os.environ["OMP_NUM_THREADS"]))
    except (KeyError, ValueError):
        pass
    return max(1, n)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def cpu_baseline(scene, a, scene_path=None):
    """The reference CPU tile renderer timed on this host's cores, on a bounded sample: whole 1-spp
    frames of the same scene until ~cpu_seconds pass.

    kind "reference": oracle/_ref's ref_render -- RTBase's own classes (BVHNode::traverse,
    Scene::visible, BSDFs, lights, Camera, Film) compiled from the reference headers, with the
    unbuildable Renderer.h's pathTrace/computeDirect/tile pool restated on top; its film is
    bit-identical to the oracle's and reproduces the survey's C1 md5. It loads the scene with the
    reference's own loader and builds the reference BVH (outside the timing).
    kind "port": oracle/rt_oracle.c's tile renderer, when oracle/_ref was not built."""
    threads = host_cores()
    base = {"cores": threads, "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count()}
    try:
        from oracle import pyref
        from oracle.pyoracle import Oracle
    except Exception as e:  # pragma: no cover
        return dict(base, error="oracle unavailable: %s" % e)
    if scene_path is not None and pyref.available():
        cfg = CONFIGS[a.config]
        t0 = time.perf_counter()
        r = pyref.RefScene(scene_path, a.width, a.height, cfg.get("skip_missing", False), cfg.get("envmap"))
        load_s = time.perf_counter() - t0

        def frame(f, film):
            return r.render(1, first=f, seed=1234, max_depth=a.max_depth, threads=threads, film=film)
        kind, what = "reference", ("oracle/_ref ref_render: RTBase's own classes (BVHNode::traverse, BSDFs, lights, "
                                   "Film) with Renderer.h's pathTrace/tile pool restated, %d std::threads" % threads)
    else:
        o = Oracle(scene, max_depth=a.max_depth, flavour="libm")
        load_s = 0.0

        def frame(f, film):
            fl, c = o.render(1, first=f, seed=1234, threads=threads, film=film, count=True)
            return fl, [c[0], c[1], c[2]]
        kind, what = "port", "oracle/rt_oracle.c tile renderer (reference DFS traversal, no culling), %d threads" % threads
    rays = paths = frames = 0
    film = np.zeros((scene.height, scene.width, 3), np.float32)
    t0 = time.perf_counter()
    while frames < 8:
        _, c = frame(frames, film)
        paths += int(c[0])
        rays += int(c[1]) + int(c[2])
        frames += 1
        if time.perf_counter() - t0 > a.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    return dict(base, value=round(rays / dt / 1e6, 3), unit="Mray/s (reference rays: a camera ray per sample)", kind=kind,
                sample="%d full %dx%d frame(s) at 1 spp of the same scene, MAX_DEPTH %d (%d paths, %d rays) in "
                       "%.1f s; %s; glibc math" % (frames, scene.width, scene.height, a.max_depth, paths, rays, dt, what),
                ms_per_frame=round(dt * 1e3 / frames, 1), mpaths_per_s=round(paths / dt / 1e6, 3),
                load_and_bvh_s=round(load_s, 2))


if __name__ == "__main__":
    main()
