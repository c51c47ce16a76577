"""Multi-rank frame protocol on the CPU (gloo, world_size 2) -- SURVEY §8e.

The product's DistributedFrame.render_layer (chiaroscuro_amd/tiles.py) drives
each rank: it renders ITS tiles (tile t -> rank t % N) into the compact
[ntiles_r][tile][tile][3] buffer through the device's render_tiles_device (here
an oracle-backed stand-in, per-path radiance summed in sample order), gathers
them on rank 0 with torch.distributed, and has the device unpermute + blend
them (the stand-in mirrors blend_tiles_kernel).  The result must equal the oracle's single-process
progressive render bit for bit, layer after layer: the image does not depend
on the partition.  The tile arithmetic is also checked against the C-ABI's
cr_tiles_for_rank.
"""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
XRES, YRES, SPP, TILE, LAYERS = 40, 24, 2, 16, 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup_paths():
    for p in (ROOT / "chiaroscuro-raytracer_amd", ROOT / "oracle", ROOT / "tests"):
        if str(p) not in sys.path:
            sys.path.insert(0, str(p))


def blend_tiles_reference(gathered, layout, frame, layer):
    """numpy mirror of blend_tiles_kernel (csrc/kernels.hip) -- test helper only;
    the kernel itself is checked on the GPU (test_gpu_parity tile tests)."""
    T = layout.tile
    for r in range(layout.nranks):
        for lt in range(layout.tiles_for_rank(r)):
            x0, y0 = layout.tile_origin(r, lt)
            h, w = min(T, layout.yres - y0), min(T, layout.xres - x0)
            m = gathered[r, lt, :h, :w]
            old = frame[y0:y0 + h, x0:x0 + w] if layer > 1 else np.zeros_like(m)
            frame[y0:y0 + h, x0:x0 + w] = (old * np.float32(layer - 1) + m) / np.float32(layer)


def _view(ptr: int, shape):
    """numpy view of a CPU torch buffer handed over by address (as the C-ABI gets it)."""
    import ctypes
    n = int(np.prod(shape))
    return np.ctypeslib.as_array((ctypes.c_float * n).from_address(ptr)).reshape(shape)


class OracleTileDevice:
    """Stand-in for chiaroscuro_amd.Device behind DistributedFrame on the CPU: the
    same three entry points taking buffer addresses, computed by the oracle --
    per pixel temp = sum_s path(s) in sample order, mean = temp * (1/spp)."""

    def __init__(self, osc, cam, info):
        self.osc, self.cam, self.info = osc, cam, info
        self.calls = []

    def _mean(self, p, x, y):
        temp = np.zeros(3, np.float32)
        for s in range(p.spp):
            temp = temp + self.osc.path(self.cam, p.xres, p.yres, p.k, self.info["background"], p.seed, p.layer,
                                        x, y, s)
        return temp * (np.float32(1.0) / np.float32(p.spp))

    def render_tiles_device(self, cam, p, ptr, stream=0):
        from chiaroscuro_amd.tiles import TileLayout
        lay = TileLayout(p.xres, p.yres, p.nranks, p.tile)
        T = lay.tile
        buf = _view(ptr, (lay.max_tiles, T, T, 3))
        for lt in range(lay.tiles_for_rank(p.rank)):
            x0, y0 = lay.tile_origin(p.rank, lt)
            for yy in range(min(T, p.yres - y0)):
                for xx in range(min(T, p.xres - x0)):
                    buf[lt, yy, xx] = self._mean(p, x0 + xx, y0 + yy)
        self.calls.append(("tiles", p.rank, p.layer))

    def blend_tiles_device(self, p, gathered_ptr, frame_ptr, stream=0):
        from chiaroscuro_amd.tiles import TileLayout
        lay = TileLayout(p.xres, p.yres, p.nranks, p.tile)
        g = _view(gathered_ptr, (p.nranks, lay.max_tiles, lay.tile, lay.tile, 3))
        blend_tiles_reference(g, lay, _view(frame_ptr, (p.yres, p.xres, 3)), p.layer)
        self.calls.append(("blend", p.rank, p.layer))

    def render_device(self, cam, p, frame_ptr, stream=0):
        f = _view(frame_ptr, (p.yres, p.xres, 3))
        for y in range(p.yres):
            for x in range(p.xres):
                m = self._mean(p, x, y)
                f[y, x] = m if p.layer == 1 else (f[y, x] * np.float32(p.layer - 1) + m) / np.float32(p.layer)
        self.calls.append(("frame", p.rank, p.layer))


def _worker(rank, world, port, q):
    try:
        _setup_paths()
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CHIARO_QUIET="1")
        import torch.distributed as dist
        import chiaroscuro_amd as ca
        import pyoracle as po
        from chiaroscuro_amd import scenes
        from chiaroscuro_amd.tiles import DistributedFrame

        dist.init_process_group("gloo", rank=rank, world_size=world)
        sc = ca.Scene(scenes.config_rtc("cornell"))
        info = sc.info
        m = ca.Model(sc)
        osc = po.OracleScene(m.triangles(), leaf_size=info["leaf_size"])
        cam = ca.camera(info["VP"], info["LA"], info["UP"], info["yview"], XRES, YRES)
        dev = OracleTileDevice(osc, cam.as_array(), info)
        # the product's frame protocol: render my tiles, gather to rank 0, blend there
        fr = DistributedFrame(dev, XRES, YRES, rank, world, TILE, dist, device="cpu")
        ok = True
        ref = None
        for layer in range(1, LAYERS + 1):
            p = ca.render_params(XRES, YRES, SPP, info["k"], info["seed"], layer=layer, rank=rank, nranks=world,
                                 tile=TILE, background=info["background"])
            fr.render_layer(cam, p)
            if rank == 0:
                ref, _ = osc.render(cam.as_array(), XRES, YRES, SPP, info["k"], info["seed"], layer=layer,
                                    bg=info["background"], pixels=ref, threads=1)
                frame = fr.frame.numpy()
                ok = ok and bool((frame.view(np.uint32) == ref.view(np.uint32)).all()) and float(frame.mean()) > 0
            else:
                ok = ok and fr.frame is None and fr.gathered is None
        # checkpoint / resume (DistributedFrame.save / resume): rank 0 writes the frame, a new frame
        # resumes it on every rank, continues one layer equal to the oracle's; another camera or
        # another sampling is refused on every rank
        kd = ca.KDTree(m, sc)
        hdr = ca.Checkpoint()
        hdr.xres, hdr.yres, hdr.samples, hdr.k, hdr.seed, hdr.layers = XRES, YRES, SPP, info["k"], info["seed"], LAYERS
        for name, v in (("eye", info["VP"]), ("center", info["LA"]), ("up", info["UP"]),
                        ("background", info["background"])):
            getattr(hdr, name)[:] = [float(x) for x in v]
        hdr.yview = info["yview"]
        hdr.scene = kd.fingerprint()
        chk = Path(os.environ["CHIARO_TEST_TMP"]) / "frame.chk"
        fr.save(chk, hdr)
        dist.barrier()
        fr2 = DistributedFrame(dev, XRES, YRES, rank, world, TILE, dist, device="cpu")
        resumed = fr2.resume(chk, hdr)  # (collective: called on every rank, whatever `ok` says)
        ok = ok and resumed == LAYERS
        p = ca.render_params(XRES, YRES, SPP, info["k"], info["seed"], layer=LAYERS + 1, rank=rank, nranks=world,
                             tile=TILE, background=info["background"])
        fr2.render_layer(cam, p)
        if rank == 0:
            ref, _ = osc.render(cam.as_array(), XRES, YRES, SPP, info["k"], info["seed"], layer=LAYERS + 1,
                                bg=info["background"], pixels=ref, threads=1)
            ok = ok and bool((fr2.frame.numpy().view(np.uint32) == ref.view(np.uint32)).all())
        for field, val in (("eye", [0.0, 1.0, 3.0]), ("center", [0.0, 0.5, 0.0]), ("yview", 0.5), ("samples", 3)):
            bad = ca.Checkpoint.from_buffer_copy(hdr)
            if isinstance(val, list):
                getattr(bad, field)[:] = val
            else:
                setattr(bad, field, val)
            fr3 = DistributedFrame(dev, XRES, YRES, rank, world, TILE, dist, device="cpu")
            try:
                fr3.resume(chk, bad)
                ok = False
            except ValueError as e:
                want_msg = "camera" if field != "samples" else "sampling"
                ok = ok and (want_msg in str(e) if rank == 0 else "rank 0 refused" in str(e))
        # `up` alone is not compared (the reference's lastUp quirk)
        up = ca.Checkpoint.from_buffer_copy(hdr)
        up.up[:] = [1.0, 0.0, 0.0]
        resumed = DistributedFrame(dev, XRES, YRES, rank, world, TILE, dist, device="cpu").resume(chk, up)
        ok = ok and resumed == LAYERS
        want = [("tiles", rank, L) for L in range(1, LAYERS + 2)]
        if rank == 0:
            want = [c for L in range(1, LAYERS + 2) for c in (("tiles", 0, L), ("blend", 0, L))]
        ok = ok and dev.calls == want
        # a partition that disagrees with the process group is refused
        try:
            DistributedFrame(dev, XRES, YRES, rank, world + 1, TILE, dist, device="cpu")
            ok = False
        except ValueError:
            pass
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, ok))
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))


def test_tile_layout_matches_cabi(ca):
    from chiaroscuro_amd.tiles import TileLayout
    for (x, y, n, t) in [(1920, 1080, 8, 32), (40, 24, 2, 16), (45, 37, 3, 16), (7, 5, 4, 32), (3840, 2160, 7, 32)]:
        lay = TileLayout(x, y, n, t)
        p = ca.render_params(x, y, 1, 1, 0, nranks=n, tile=t)
        counts = [ca.Device.tiles_for_rank(p, r) for r in range(n)]
        assert counts == [lay.tiles_for_rank(r) for r in range(n)]
        assert sum(counts) == lay.ntiles
        # every tile owned exactly once, at the same origin in the C-ABI and in TileLayout
        owned = sorted(r + lt * n for r in range(n) for lt in range(lay.tiles_for_rank(r)))
        assert owned == list(range(lay.ntiles))
        origins = [lay.tile_origin(r, lt) for r in range(n) for lt in range(lay.tiles_for_rank(r))]
        assert origins == [ca.Device.tile_origin(p, r, lt) for r in range(n) for lt in range(lay.tiles_for_rank(r))]
        assert sorted(origins) == sorted((tx * t, ty * t) for ty in range(lay.tiles_y) for tx in range(lay.tiles_x))
    # rows rotated by their index (n > 1): rank 0 of 8 at 1920 px sees every column class mod 8
    lay = TileLayout(1920, 1080, 8, 32)
    cols = {lay.tile_origin(0, lt)[0] // 32 % 8 for lt in range(lay.tiles_for_rank(0))}
    assert cols == set(range(8))


def test_gloo_tile_gather_matches_single_process(tmp_path, monkeypatch):
    import torch.multiprocessing as mp
    monkeypatch.setenv("CHIARO_TEST_TMP", str(tmp_path))
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}, res
