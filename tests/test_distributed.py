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
