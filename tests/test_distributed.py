"""N>1 path on CPU: gloo ranks each render their diagonal 32x32 tile stripes and assemble the
float32 film on rank 0 with raytracingrenderer_amd.distributed (FilmExchange: every rank's own
tiles packed, gathered to rank 0 and scattered; the whole-film reduce of rounds 1-4 is kept) — the
same helpers bench.py uses over RCCL. The per-rank renderer here is the C oracle (no GPU in this
container); the assembled film must equal a single full render bit for bit."""
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


class _OracleRanks:
    """The surface FilmExchange reads from a RayTracer (width, height, film()), backed by the C
    oracle's render of this rank's tiles."""

    def __init__(self, film):
        self._film = film
        self.height, self.width = film.shape[:2]

    def film(self):
        return self._film, 3


def _xworker(rank, world, port, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.pyoracle import Oracle
    from raytracingrenderer_amd import loadScene
    from raytracingrenderer_amd.distributed import FilmExchange, tiles_for_rank
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=100, height=70)  # clipped edge tiles
    tiles = tiles_for_rank(100, 70, rank, world)
    film, _ = Oracle(s, 4, "rtm").render(3, seed=77, tiles=tiles)
    # rank 0's target starts as garbage: the exchange must write every pixel
    t = torch.full((70, 100, 3), float("nan"), dtype=torch.float32)
    fx = FilmExchange(100, 70, rank, world)
    fx.exchange(_OracleRanks(film), t, dist)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 5])
def test_own_tile_exchange_is_bit_exact(tmp_path, world):
    """Every rank sends only its own tiles' pixels (rtg_tile_pixels order, padded to the longest
    list); rank 0 scatters them: the film equals one full render, bit for bit."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "film.npy")
    mp.spawn(_xworker, args=(world, _free_port(), out), nprocs=world, join=True)
    from oracle.pyoracle import Oracle
    from raytracingrenderer_amd import loadScene
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=100, height=70)
    full, _ = Oracle(s, 4, "rtm").render(3, seed=77)
    got = np.load(out)
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32))


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
    np.save(out_path if rank == 0 else out_path + ".rank%d.npy" % rank, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_librtg_ranks_reduce_is_bit_exact(tmp_path):
    """Two processes, each with its own librtg handle, reduce their tile films over gloo: the
    result equals one handle rendering every tile, bit for bit; rank 1's film_tensor holds its own
    tiles' film (render_sharded fills it on the non-root ranks)."""
    import torch.multiprocessing as mp
    from raytracingrenderer_amd.distributed import tiles_for_rank
    out = str(tmp_path / "film.npy")
    mp.spawn(_gpu_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    from raytracingrenderer_amd import RayTracer, loadScene
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=96, height=80)
    rt = RayTracer(s, seed=77)
    rt.render(3, first_sample=0)
    full = rt.film()[0]
    got = np.load(out)
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32))
    own = RayTracer(s, seed=77)
    own.render(3, tiles=tiles_for_rank(96, 80, 1, 2), first_sample=0)
    assert np.array_equal(np.load(out + ".rank1.npy").view(np.uint32), own.film()[0].view(np.uint32))


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


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
def test_device_gather_scatter_assemble_one_render(world):
    """The device half of the own-tile exchange on one GPU: N handles render their stripes,
    rtg_film_gather packs each rank's pixels on the device, the packed buffers are stacked (what
    the RCCL gather does across GPUs) and rtg_film_scatter writes them into a film that starts as
    NaN: the result equals one handle's full render, bit for bit."""
    import ctypes as C
    import torch
    from raytracingrenderer_amd import RayTracer, loadScene
    from raytracingrenderer_amd import _native as N
    from raytracingrenderer_amd.distributed import FilmExchange, tiles_for_rank
    W, H = 200, 136
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=W, height=H)
    one = RayTracer(s, seed=9)
    one.render(3, first_sample=0)
    want = one.film()[0]
    fx = [FilmExchange(W, H, r, world, device="cuda:0") for r in range(world)]
    recv = torch.zeros((world, fx[0].maxpix * 3), dtype=torch.float32, device="cuda:0")
    for r in range(world):
        rt = RayTracer(s, seed=9)
        rt.render(3, tiles=tiles_for_rank(W, H, r, world),
                  first_sample=0, sync=False)  # queued: the gather must order after it
        assert N.rtg().rtg_film_gather(rt.handle, C.c_void_p(fx[r].t_own.data_ptr()), fx[r].maxpix,
                                       C.c_void_p(recv[r].data_ptr()), None) == 0
        rt.synchronize()
        del rt
    film = torch.full((H, W, 3), float("nan"), dtype=torch.float32, device="cuda:0")
    assert N.rtg().rtg_film_scatter(0, C.c_void_p(recv.data_ptr()), C.c_void_p(fx[0].t_all.data_ptr()),
                                    len(fx[0].all), C.c_void_p(film.data_ptr()), W * H, None) == 0
    torch.cuda.synchronize()
    assert np.array_equal(film.cpu().numpy().view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_gather_scatter_ignore_indices_past_the_film():
    """A pixel list built for a larger film (or any index >= width * height) is never dereferenced:
    rtg_film_gather packs zeros for it and rtg_film_scatter skips it; in-range entries move as usual."""
    import ctypes as C
    import torch
    from raytracingrenderer_amd import RayTracer, loadScene
    from raytracingrenderer_amd import _native as N
    W, H = 64, 48
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=W, height=H)
    rt = RayTracer(s, seed=5)
    rt.render(2, first_sample=0)
    want = rt.film()[0].reshape(-1, 3)
    pix = np.array([3, W * H, W * H - 1, 0xFFFFFFFE, 7 * W + 5, 1 << 30], np.uint32)
    t_pix = torch.from_numpy(pix.view(np.int32)).to("cuda:0")
    pack = torch.full((len(pix) * 3,), float("nan"), dtype=torch.float32, device="cuda:0")
    assert N.rtg().rtg_film_gather(rt.handle, C.c_void_p(t_pix.data_ptr()), len(pix), C.c_void_p(pack.data_ptr()),
                                   None) == 0
    rt.synchronize()
    got = pack.cpu().numpy().reshape(-1, 3)
    ok = pix < W * H
    assert np.array_equal(got[ok].view(np.uint32), want[pix[ok]].view(np.uint32))
    assert not got[~ok].view(np.uint32).any()
    film = torch.full((H * W * 3,), float("nan"), dtype=torch.float32, device="cuda:0")
    assert N.rtg().rtg_film_scatter(0, C.c_void_p(pack.data_ptr()), C.c_void_p(t_pix.data_ptr()), len(pix),
                                    C.c_void_p(film.data_ptr()), W * H, None) == 0
    torch.cuda.synchronize()
    f = film.cpu().numpy().reshape(-1, 3)
    assert np.array_equal(f[pix[ok]].view(np.uint32), want[pix[ok]].view(np.uint32))
    written = np.zeros(W * H, bool)
    written[pix[ok]] = True
    assert np.isnan(f[~written]).all()
    assert N.rtg().rtg_film_scatter(0, C.c_void_p(pack.data_ptr()), C.c_void_p(t_pix.data_ptr()), len(pix),
                                    C.c_void_p(film.data_ptr()), 0, None) != 0  # no film size: refused


@pytest.mark.gpu
def test_pipelined_frames_exchange_sees_each_frame():
    """bench.py's lean step at N > 1: queued renders (the frame pipeline: a frame's traversal starts
    while the previous frame drains) each followed by FilmExchange on its own stream, with no host
    wait in between. The exchange of step k must read exactly the film after frame k (the fold of
    frame k + 1 waits for it): every assembled snapshot equals the film a waited-for render loop
    reads after the same frame, bit for bit."""
    import torch
    from raytracingrenderer_amd import RayTracer, loadScene
    from raytracingrenderer_amd.distributed import FilmExchange
    W, H = 160, 128  # 20480 pixels x 16 spp: a 328k-path frame, inside the pipeline's chunk limit
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=W, height=H)
    ref = RayTracer(s, seed=21)
    want = []
    for k in range(4):
        ref.render(16, first_sample=16 * k)
        want.append(ref.film()[0])
    rt = RayTracer(s, seed=21)
    fx = FilmExchange(W, H, 0, 1, device="cuda:0")
    film = torch.full((H, W, 3), float("nan"), dtype=torch.float32, device="cuda:0")
    snaps, evs = [], []
    for k in range(4):
        rt.render(16, first_sample=16 * k, sync=False)
        ev = fx.exchange(rt, film, None, timing=k >= 2)  # timed: start once the frame is on the film
        if ev is not None:
            evs.append(ev)
        snaps.append(film.clone())  # on the caller's stream, after the exchange
    torch.cuda.synchronize()
    assert len(evs) == 2 and all(0.0 <= e0.elapsed_time(e1) < 50.0 for e0, e1 in evs)
    for k in range(4):
        assert np.array_equal(snaps[k].cpu().numpy().view(np.uint32), want[k].view(np.uint32)), k


def test_native_tile_partition_matches_python():
    """rtg_tiles_for_rank (librtg, used by rtg_group and the CLI's -gpus) is the partition of
    distributed.tiles_for_rank (pure host code: no GPU needed)."""
    from raytracingrenderer_amd.distributed import tiles_for_rank
    from raytracingrenderer_amd.renderer import tiles_for_rank_native
    for w, h, n in [(1024, 1024, 8), (1920, 1080, 3), (100, 50, 4), (4096, 4096, 8), (40, 40, 5)]:
        for r in range(n):
            assert np.array_equal(tiles_for_rank_native(w, h, r, n), tiles_for_rank(w, h, r, n))


@pytest.mark.gpu
@pytest.mark.parametrize("devices,rccl1", [([0], False), ([0], True), ([0], "self"), ([0, 0], False),
                                           ([0, 0, 0, 0, 0, 0, 0, 0], False)])
def test_group_film_equals_one_device(devices, rccl1, monkeypatch):
    """rtg_group: one device (no communicator; with RTG_GROUP_RCCL1=1 an RCCL communicator,
    ncclCommInitAll, one rank; with RTG_GROUP_RCCL_SELF=1 too, rank 0's pack goes through an
    ncclSend / ncclRecv pair to itself, so the RCCL exchange's calls run on a one-GPU box), or N ranks
    rehearsed on the box's one GPU (own tiles packed, moved by device copies, scattered): the
    assembled film equals one handle's render of every tile, bit for bit."""
    from raytracingrenderer_amd import RayTracer, RayTracerGroup, loadScene
    if rccl1:
        monkeypatch.setenv("RTG_GROUP_RCCL1", "1")
    if rccl1 == "self":
        monkeypatch.setenv("RTG_GROUP_RCCL_SELF", "1")
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=200, height=136)
    one = RayTracer(s, seed=31)
    one.render(3, first_sample=0)
    want = one.film()[0]
    g = RayTracerGroup(s, devices=devices, seed=31)
    assert g.uses_rccl == bool(rccl1)
    g.render(2)
    g.render(1)
    got, spp = g.film()
    assert spp == 3
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    g.clear()
    g.render(3, first_sample=0)
    assert np.array_equal(g.film()[0].view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0, 0, 0, 0, 0], "rccl_self"])
def test_queued_group_frames_equal_one_handle(devices, monkeypatch):
    """The queued group frame (rtg_group_render_async + rtg_group_reduce_async, bench.py's lean step
    and the CLI's -gpus loop): four frames, each followed by a queued own-tile exchange with no host
    wait, then the film; and a film read between frames sees exactly the frames before it. Both equal
    one handle's waited-for renders of the same samples, bit for bit."""
    from raytracingrenderer_amd import RayTracer, RayTracerGroup, loadScene
    if devices == "rccl_self":
        # one device with a communicator, rank 0's pack sent to itself: the RCCL exchange's
        # ncclSend / ncclRecv group, queued on the exchange stream, runs on a one-GPU box
        monkeypatch.setenv("RTG_GROUP_RCCL1", "1")
        monkeypatch.setenv("RTG_GROUP_RCCL_SELF", "1")
        devices = [0]
    W, H = 160, 128  # 16 spp per frame: 328k paths, inside the frame pipeline's chunk limit
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=W, height=H)
    ref = RayTracer(s, seed=23)
    want = []
    for k in range(4):
        ref.render(16, first_sample=16 * k)
        want.append(ref.film()[0])
    g = RayTracerGroup(s, devices=devices, seed=23)
    for k in range(4):
        g.render(16, first_sample=16 * k, sync=False)
        g.reduce(sync=False)
    got, spp = g.film()
    assert spp == 64
    assert np.array_equal(got.view(np.uint32), want[3].view(np.uint32))
    g.clear()
    for k in range(4):
        g.render(16, first_sample=16 * k, sync=False)
        g.reduce(sync=False)
        if k in (1, 2):
            assert np.array_equal(g.film()[0].view(np.uint32), want[k].view(np.uint32)), k
    g.synchronize()
    assert g.reduce_ms() > 0.0
    g.render(16, first_sample=64, sync=False)  # no exchange queued: film() runs one first
    ref.render(16, first_sample=64)
    assert np.array_equal(g.film()[0].view(np.uint32), ref.film()[0].view(np.uint32))


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
    assert ("by none (one device)" in r2.stdout) == (opt[0] == "-gpus")
    assert ("device copies" in r2.stdout) == (opt[0] == "-devices")
    assert (tmp_path / "one" / "result_4.hdr").read_bytes() == (tmp_path / "multi" / "result_4.hdr").read_bytes()


def _visible_gpus():
    from conftest import has_gpu
    if not has_gpu():
        return 0
    import ctypes as C
    from raytracingrenderer_amd import _native as N
    n = C.c_int(0)
    N.rtg().rtg_device_count(C.byref(n))
    return n.value


@pytest.mark.gpu
def test_group_over_distinct_devices_equals_one_device():
    """rtg_group over two distinct GPUs (ncclCommInitAll over devices 0 and 1, rank 1's tiles sent
    with ncclSend over xGMI): the assembled film equals one device's render, bit for bit. Needs >= 2
    visible GPUs (skipped on a one-GPU box; run on a node with several)."""
    if _visible_gpus() < 2:
        pytest.skip("needs >= 2 visible GPUs for a distinct-device RCCL group")
    from raytracingrenderer_amd import RayTracer, RayTracerGroup, loadScene
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=160, height=96)
    one = RayTracer(s, seed=17)
    one.render(3, first_sample=0)
    g = RayTracerGroup(s, devices=[0, 1], seed=17)
    assert g.uses_rccl
    g.render(3, first_sample=0)
    assert np.array_equal(g.film()[0].view(np.uint32), one.film()[0].view(np.uint32))
    # queued frames and exchanges (the ranks' RCCL send/recv on the exchange streams)
    g.clear()
    for k in range(3):
        g.render(1, first_sample=k, sync=False)
        g.reduce(sync=False)
    assert np.array_equal(g.film()[0].view(np.uint32), one.film()[0].view(np.uint32))


@pytest.mark.gpu
def test_failed_group_render_poisons_until_clear():
    """A rank that fails a render leaves the group's films partial: reduce / film_read refuse until
    rtg_group_clear, after which the group renders the one-device film again."""
    from raytracingrenderer_amd import RayTracer, RayTracerGroup, loadScene
    from raytracingrenderer_amd.renderer import NativeError
    s = loadScene(os.path.join(SCENES, "cornell-box"), width=64, height=64)
    g = RayTracerGroup(s, devices=[0, 0], seed=3)
    g.render(1, first_sample=0)
    with pytest.raises(NativeError):
        g.render(10, first_sample=65530)  # past the PCG key: every rank refuses
    with pytest.raises(NativeError):
        g.film()
    g.clear()
    g.render(2, first_sample=0)
    one = RayTracer(s, seed=3)
    one.render(2, first_sample=0)
    assert np.array_equal(g.film()[0].view(np.uint32), one.film()[0].view(np.uint32))


@pytest.mark.gpu
def test_bench_native_group_rehearsal_is_bit_exact():
    """bench.py --devices 0,0 (the native group path of --gpus N, two ranks rehearsed on one GPU)
    reports one GPU, two ranks, and a reduced film equal to the one-device render."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--devices", "0,0", "--verify-film",
                        "--config", "C2", "--width", "256", "--height", "192", "--spp", "4", "--steps", "1",
                        "--warmup", "1", "--no-cpu-baseline"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    # n_gpus counts distinct devices; the two rehearsed ranks are "ranks"
    assert d["n_gpus"] == 1 and d["ranks"] == 2 and d["group"]["distinct_gpus"] == 1
    assert d["film_reduce_bit_exact"] is True
    # rehearsed ranks get equal chunk budgets, so their render times are comparable
    assert d["group"]["rank_render_ms"]["max_over_mean"] < 1.5
    assert len(d["group"]["rank_kernel_ms_last_step"]) == 2


def test_bench_refuses_more_gpus_than_visible():
    """CPU: bench.py --gpus N with fewer visible HIP devices exits non-zero instead of silently
    measuring one GPU (this container has none; a one-GPU box has one)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n = _visible_gpus() + 1
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(max(n, 2)), "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "refusing" in r.stderr
