"""Does an RCCL communicator in the process slow librtg's kernels? (round 6: a native group of one
device with ncclCommInitAll ran k_accumulate_pm 1.05 -> 1.52 ms.) Renders C3 (64 spp, waited-for)
`--reps` times in one of three orders and prints the per-launch HIP-event times; run under
rocprofv3 --kernel-trace --stats for per-kernel durations.
  --mode none        librtg only
  --mode pg_first    torch.distributed nccl process group (world 1) created before the renderer
  --mode pg_after    renderer created and its chunk buffers allocated (one render), then the group"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", default="none", choices=["none", "pg_first", "pg_after"])
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    import torch

    def pg():
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        t = torch.ones(1, device="cuda:0")
        dist.all_reduce(t)
        torch.cuda.synchronize()
        return dist
    dist = pg() if a.mode == "pg_first" else None
    from raytracingrenderer_amd import RayTracer, loadScene, write_synthetic_scene
    from raytracingrenderer_amd import _native as N
    work = tempfile.mkdtemp(prefix="rtg_rp_")
    write_synthetic_scene(work, n_tris=1_000_000, seed=20251015, width=1024, height=1024)
    rt = RayTracer(loadScene(work), max_depth=4, seed=1234)
    rt.set_options(flags=N.RTG_OPT_CULL | N.RTG_OPT_TIMING)
    rt.render(64, first_sample=0)
    if a.mode == "pg_after":
        dist = pg()
    out = []
    for _ in range(a.reps):
        rt.clear()
        t0 = time.perf_counter()
        rt.render(64, first_sample=0)
        st = rt.stats()
        out.append((round((time.perf_counter() - t0) * 1e3, 2), round(st["extend_ms"], 2), round(st["shade_ms"], 2)))
    print(json.dumps({"mode": a.mode, "wall_trace_shade_ms": out}))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
