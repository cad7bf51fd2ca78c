"""Multi-GPU decomposition: 32x32 tiles interleaved over ranks + one own-tile film exchange.

RTBase renders its 32x32 tiles (Renderer.h:18, 820-853) from a shared queue on CPU threads; here
each rank (one process per GPU) owns the tiles with (tile_x + tile_y) % world == rank (diagonal
stripes, so every rank gets the same mix of image centre and border: with tile_id % world the
ranks' ray counts differed by up to 19 % at N = 8) and renders all samples of them through its own
librtg handle. The film is then assembled on rank 0 from each rank's own tiles only
(FilmExchange): every rank packs its tiles' pixels (rtg_film_gather, 12 B per pixel: 1/N of the
film), one torch.distributed gather moves them to rank 0 (RCCL over xGMI on MI355X, gloo in CPU
tests), and rank 0 scatters them into the film (rtg_film_scatter). Tile supports are disjoint and
cover the image, so the assembled film is bit-identical to a single-GPU render. reduce_film (the
whole-film sum of rounds 1-4, N x the bytes) is kept for callers that hold full films.
"""
import ctypes as C

import numpy as np

TILE = 32
PIX_PAD = 0xFFFFFFFF  # padding entry of a pixel list (packed as zeros, skipped by the scatter)


def tiles_for_rank(width, height, rank, world):
    tx, ty = (width + TILE - 1) // TILE, (height + TILE - 1) // TILE
    t = np.arange(tx * ty, dtype=np.uint32)
    return t[((t % tx) + (t // tx)) % world == rank]


def tile_pixels(width, height, tiles):
    """Film pixel indices (y * width + x) of `tiles` in the order rtg_film_gather packs them: tile
    by tile, row-major inside a tile, clipped at the film edge (rtg_tile_pixels, host code)."""
    from raytracingrenderer_amd import _native as N
    t = np.ascontiguousarray(tiles, np.uint32)
    n = C.c_uint32(0)
    if N.rtg().rtg_tile_pixels(width, height, N.ptr(t, C.c_uint32), len(t), None, C.byref(n)):
        raise ValueError(N.rtg().rtg_last_error().decode())
    out = np.zeros(n.value, np.uint32)
    N.rtg().rtg_tile_pixels(width, height, N.ptr(t, C.c_uint32), len(t), N.ptr(out, C.c_uint32), C.byref(n))
    return out


class FilmExchange:
    """Assemble rank 0's film from every rank's own tiles.

    Built once per (film size, world): every rank's pixel list (tile_pixels of its stripes), padded
    to the longest, and on rank 0 the concatenation of all of them. exchange(rt, film_tensor):
      - CUDA film tensor (RCCL): rtg_film_gather packs this rank's pixels from the librtg film on the
        device; dist.gather moves the packed buffers (maxpix * 12 B each) to rank 0, which
        rtg_film_scatter writes into film_tensor;
      - CPU film tensor (gloo): the same packing and scatter with numpy on the host film.
    Only rank 0's film_tensor receives the assembled film."""

    def __init__(self, width, height, rank, world, device=None):
        import torch
        self.W, self.H, self.rank, self.world = width, height, rank, world
        lists = [tile_pixels(width, height, tiles_for_rank(width, height, r, world)) for r in range(world)]
        self.n = len(lists[rank])
        self.maxpix = max(1, max(len(l) for l in lists))
        pad = np.full((world, self.maxpix), PIX_PAD, np.uint32)
        for r, l in enumerate(lists):
            pad[r, :len(l)] = l
        self.own = pad[rank].copy()
        self.all = pad.reshape(-1).copy()
        self.cuda = device is not None and str(device).startswith("cuda")
        dev = device if self.cuda else "cpu"
        # pixel lists travel as int32 tensors of the same bits (torch has no uint32 arithmetic here)
        self.t_own = torch.from_numpy(self.own.view(np.int32)).to(dev)
        self.t_all = torch.from_numpy(self.all.view(np.int32)).to(dev) if rank == 0 else None
        self.pack = torch.zeros(self.maxpix * 3, dtype=torch.float32, device=dev)
        self.recv = torch.zeros((world, self.maxpix * 3), dtype=torch.float32, device=dev) if rank == 0 else None
        # CUDA: the exchange runs on a stream of its own (never the null stream, which librtg would
        # take for the handle's), after the caller's earlier work; the caller's later work waits for it
        self.stream = torch.cuda.Stream(device=dev) if self.cuda else None

    def exchange(self, rt, film_tensor, dist, timing=False):
        """Assemble film_tensor on rank 0. timing=True (CUDA): returns (start, end) CUDA events on the
        exchange's stream, start recorded once the rank's queued frames are on its film (so the pair
        times the exchange alone); otherwise returns None."""
        import torch
        from raytracingrenderer_amd import _native as N
        if not self.cuda:
            self._exchange(rt, film_tensor, dist)
            return None
        cur = torch.cuda.current_stream(self.stream.device)
        self.stream.wait_stream(cur)
        ev = None
        with torch.cuda.stream(self.stream):
            if timing:
                # rtg_film_gather of no pixels: only the wait for the handle's frames
                rc = N.rtg().rtg_film_gather(rt.handle, None, 0, None, C.c_void_p(self.stream.cuda_stream))
                if rc:
                    raise RuntimeError(N.rtg().rtg_last_error().decode())
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(self.stream)
            self._exchange(rt, film_tensor, dist)
            if timing:
                ev[1].record(self.stream)
        cur.wait_stream(self.stream)
        return ev

    def _exchange(self, rt, film_tensor, dist):
        import torch
        from raytracingrenderer_amd import _native as N
        if self.cuda:
            stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
            rc = N.rtg().rtg_film_gather(rt.handle, C.c_void_p(self.t_own.data_ptr()), self.maxpix,
                                         C.c_void_p(self.pack.data_ptr()), stream)
            if rc:
                raise RuntimeError(N.rtg().rtg_last_error().decode())
        else:
            f = rt.film()[0].reshape(-1, 3)
            p = np.zeros((self.maxpix, 3), np.float32)
            p[:self.n] = f[self.own[:self.n]]
            self.pack.copy_(torch.from_numpy(p.reshape(-1)))
        if self.world > 1:
            dist.gather(self.pack, gather_list=list(self.recv.unbind(0)) if self.rank == 0 else None, dst=0)
        elif self.rank == 0:
            self.recv[0].copy_(self.pack)
        if self.rank == 0:
            if self.cuda:
                stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
                rc = N.rtg().rtg_film_scatter(film_tensor.device.index, C.c_void_p(self.recv.data_ptr()),
                                              C.c_void_p(self.t_all.data_ptr()), len(self.all),
                                              C.c_void_p(film_tensor.data_ptr()), self.W * self.H, stream)
                if rc:
                    raise RuntimeError(N.rtg().rtg_last_error().decode())
            else:
                ok = self.all != PIX_PAD
                fl = film_tensor.view(-1, 3).numpy()
                fl[self.all[ok]] = self.recv.numpy().reshape(-1, 3)[ok]
        return film_tensor


def reduce_film(film_tensor, dist, dst=0):
    """Sum the per-rank films into rank `dst` (in place). film_tensor: torch tensor HxWx3 f32."""
    dist.reduce(film_tensor, dst=dst, op=dist.ReduceOp.SUM)
    return film_tensor


def render_sharded(rt, n_samples, rank, world, dist=None, film_tensor=None, first_sample=0, exchange=None):
    """Render this rank's tiles with RayTracer `rt`, then assemble the film on rank 0.

    world > 1: rank 0's film_tensor (torch float32 HxWx3) receives the whole film from every rank's
    own tiles (FilmExchange; pass `exchange` to reuse its buffers across calls); a CUDA tensor is
    filled on the device (RCCL), a CPU tensor through host memory (gloo). On the other ranks
    film_tensor receives this rank's own film (its tiles' samples, zero elsewhere), as the
    whole-film reduce of rounds 1-4 left it. Returns film_tensor.
    world == 1: returns film_tensor filled with the film if given, else the film as a numpy array."""
    tiles = tiles_for_rank(rt.width, rt.height, rank, world)
    rt.render(n_samples, tiles=tiles, first_sample=first_sample)
    if film_tensor is None:
        if world > 1:
            raise ValueError("render_sharded: world > 1 needs a film_tensor to assemble into")
        return rt.film()[0]

    def own_film():
        if film_tensor.is_cuda:
            rt.copy_film_to(film_tensor.data_ptr())
            rt.synchronize()
        else:
            import torch
            film_tensor.copy_(torch.from_numpy(rt.film()[0]))
    if world == 1:
        own_film()
        return film_tensor
    if exchange is None:
        exchange = FilmExchange(rt.width, rt.height, rank, world, film_tensor.device if film_tensor.is_cuda else None)
    if (exchange.W, exchange.H, exchange.rank, exchange.world) != (rt.width, rt.height, rank, world):
        raise ValueError("render_sharded: exchange built for %dx%d rank %d of %d, not %dx%d rank %d of %d"
                         % (exchange.W, exchange.H, exchange.rank, exchange.world, rt.width, rt.height, rank, world))
    exchange.exchange(rt, film_tensor, dist)
    if rank != 0:
        own_film()
    return film_tensor
