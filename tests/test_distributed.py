"""N>1 path on CPU: two gloo ranks each render their interleaved 32x32 tiles (tile % 2 == rank)
and reduce the float32 film to rank 0 with raytracingrenderer_amd.distributed — the same helpers
bench.py uses over RCCL. The per-rank renderer here is the C oracle (no GPU in this container);
the reduced film must equal a single full render bit for bit."""
import os
import socket

import numpy as np
import pytest

from conftest import SCENES


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.pyoracle import Oracle
    from raytracingrenderer_amd import loadScene
    from raytracingrenderer_amd.distributed import reduce_film, tiles_for_rank
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=96, height=80)
    tiles = tiles_for_rank(96, 80, rank, world)
    film, _ = Oracle(s, 4, "rtm").render(3, seed=77, tiles=tiles)
    t = torch.from_numpy(film)
    reduce_film(t, dist)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_tile_sharded_reduce_is_bit_exact(tmp_path, world):
    import torch.multiprocessing as mp
    out = str(tmp_path / "film.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    from oracle.pyoracle import Oracle
    from raytracingrenderer_amd import loadScene
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=96, height=80)
    full, _ = Oracle(s, 4, "rtm").render(3, seed=77)
    got = np.load(out)
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32))


def test_tiles_partition():
    from raytracingrenderer_amd.distributed import tiles_for_rank
    for w, h, n in [(1024, 1024, 8), (1920, 1080, 3), (100, 50, 4)]:
        parts = [tiles_for_rank(w, h, r, n) for r in range(n)]
        allt = np.sort(np.concatenate(parts))
        assert np.array_equal(allt, np.arange(((w + 31) // 32) * ((h + 31) // 32)))


def _gpu_worker(rank, world, port, out_path):
    """One rank of the librtg path: its own RayTracer handle on the box's GPU renders its tiles and
    render_sharded() reduces the films to rank 0 (gloo through host memory; RCCL in bench.py)."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from raytracingrenderer_amd import RayTracer, loadScene
    from raytracingrenderer_amd.distributed import render_sharded
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=96, height=80)
    rt = RayTracer(s, seed=77)
    t = torch.zeros((80, 96, 3), dtype=torch.float32)
    render_sharded(rt, 3, rank, world, dist=dist, film_tensor=t)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_librtg_ranks_reduce_is_bit_exact(tmp_path):
    """Two processes, each with its own librtg handle, reduce their tile films over gloo: the
    result equals one handle rendering every tile, bit for bit."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "film.npy")
    mp.spawn(_gpu_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    from raytracingrenderer_amd import RayTracer, loadScene
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=96, height=80)
    rt = RayTracer(s, seed=77)
    rt.render(3, first_sample=0)
    full = rt.film()[0]
    got = np.load(out)
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_librtg_handles_sum_to_one_render(world):
    """N librtg handles (one per simulated rank) render tiles_for_rank(..., r, N); the films summed
    in rank order equal a single handle's full render bit for bit (the other ranks add +0.0)."""
    from raytracingrenderer_amd import RayTracer, loadScene
    from raytracingrenderer_amd.distributed import render_sharded, tiles_for_rank
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=256, height=200)
    one = RayTracer(s, seed=5)
    full = render_sharded(one, 4, 0, 1)  # world 1: the film itself
    acc = np.zeros_like(full)
    for r in range(world):
        rt = RayTracer(s, seed=5)
        rt.render(4, tiles=tiles_for_rank(256, 200, r, world), first_sample=0)
        f = rt.film()[0]
        mine = np.zeros(((200 + 31) // 32, (256 + 31) // 32), bool).ravel()
        mine[tiles_for_rank(256, 200, r, world)] = True
        # pixels outside this rank's tiles stay exactly +0.0
        outside = ~np.kron(mine.reshape((200 + 31) // 32, -1), np.ones((32, 32), bool))[:200, :256]
        assert not f[outside].view(np.uint32).any()
        acc += f
    assert np.array_equal(acc.view(np.uint32), full.view(np.uint32))


def test_native_tile_partition_matches_python():
    """rtg_tiles_for_rank (librtg, used by rtg_group and the CLI's -gpus) is the partition of
    distributed.tiles_for_rank (pure host code: no GPU needed)."""
    from raytracingrenderer_amd.distributed import tiles_for_rank
    from raytracingrenderer_amd.renderer import tiles_for_rank_native
    for w, h, n in [(1024, 1024, 8), (1920, 1080, 3), (100, 50, 4), (4096, 4096, 8), (40, 40, 5)]:
        for r in range(n):
            assert np.array_equal(tiles_for_rank_native(w, h, r, n), tiles_for_rank(w, h, r, n))


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0, 0, 0, 0, 0]])
def test_group_film_equals_one_device(devices):
    """rtg_group: one device through an RCCL communicator (ncclCommInitAll + ncclReduce), or N
    ranks rehearsed on the box's one GPU (host-memory sum): the reduced film equals one handle's
    render of every tile, bit for bit."""
    from raytracingrenderer_amd import RayTracer, RayTracerGroup, loadScene
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=200, height=136)
    one = RayTracer(s, seed=31)
    one.render(3, first_sample=0)
    want = one.film()[0]
    g = RayTracerGroup(s, devices=devices, seed=31)
    assert g.uses_rccl == (len(set(devices)) == len(devices))
    g.render(2)
    g.render(1)
    got, spp = g.film()
    assert spp == 3
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    g.clear()
    g.render(3, first_sample=0)
    assert np.array_equal(g.film()[0].view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [["-gpus", "1"], ["-devices", "0,0,0"]])
def test_cli_multi_gpu_output_equals_single(tmp_path, opt):
    """The CLI's multi-GPU mode (Main.cpp frame loop on rtg_group) writes the same result_<spp>.hdr
    bytes as the one-device CLI."""
    import subprocess
    from raytracingrenderer_amd import _native as N
    cli = os.path.join(N.LIB_DIR, "rtg_render")
    base = [cli, "-scene", os.path.join(SCENES, "cornell-box"), "-SPP", "4", "-width", "96", "-height", "64",
            "-timeLimit", "0", "-batch", "2"]
    (tmp_path / "one").mkdir()
    (tmp_path / "multi").mkdir()
    r1 = subprocess.run(base, cwd=str(tmp_path / "one"), capture_output=True, text=True, timeout=300)
    r2 = subprocess.run(base + opt, cwd=str(tmp_path / "multi"), capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr
    assert r2.returncode == 0, r2.stderr
    assert ("RCCL" in r2.stdout) == (opt[0] == "-gpus")
    assert (tmp_path / "one" / "result_4.hdr").read_bytes() == (tmp_path / "multi" / "result_4.hdr").read_bytes()
