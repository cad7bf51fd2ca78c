"""Multi-GPU decomposition: 32x32 tiles interleaved over ranks + one film reduction.

RTBase renders its 32x32 tiles (Renderer.h:18, 820-853) from a shared queue on CPU threads; here
each rank (one process per GPU) owns the tiles with (tile_x + tile_y) % world == rank (diagonal
stripes, so every rank gets the same mix of image centre and border: with tile_id % world the
ranks' ray counts differed by up to 19 % at N = 8), renders all samples of them through its own
librtg handle, and the float32 films are summed to rank 0 with a single
torch.distributed reduce (RCCL over xGMI on MI355X, gloo in CPU tests). Tile supports are
disjoint and every other rank contributes +0.0, so the reduced film is bit-identical to a
single-GPU render whatever the reduction order.
"""
import numpy as np

TILE = 32


def tiles_for_rank(width, height, rank, world):
    tx, ty = (width + TILE - 1) // TILE, (height + TILE - 1) // TILE
    t = np.arange(tx * ty, dtype=np.uint32)
    return t[((t % tx) + (t // tx)) % world == rank]


def reduce_film(film_tensor, dist, dst=0):
    """Sum the per-rank films into rank `dst` (in place). film_tensor: torch tensor HxWx3 f32."""
    dist.reduce(film_tensor, dst=dst, op=dist.ReduceOp.SUM)
    return film_tensor


def render_sharded(rt, n_samples, rank, world, dist=None, film_tensor=None, first_sample=0):
    """Render this rank's tiles with RayTracer `rt`, then reduce the films to rank 0.

    world > 1: film_tensor (torch float32 HxWx3) receives this rank's film and, on rank 0, the sum;
    a CUDA tensor is filled on the device (RCCL), a CPU tensor through host memory (gloo). Returns
    film_tensor. world == 1: returns film_tensor filled the same way if given, else the film as a
    numpy array."""
    tiles = tiles_for_rank(rt.width, rt.height, rank, world)
    rt.render(n_samples, tiles=tiles, first_sample=first_sample)
    if film_tensor is None:
        if world > 1:
            raise ValueError("render_sharded: world > 1 needs a film_tensor to reduce into")
        return rt.film()[0]
    if film_tensor.is_cuda:
        rt.copy_film_to(film_tensor.data_ptr())
        rt.synchronize()
    else:
        import torch
        film_tensor.copy_(torch.from_numpy(rt.film()[0]))
    if world > 1:
        reduce_film(film_tensor, dist)
    return film_tensor
