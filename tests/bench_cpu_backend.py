"""CPU stand-in backend for bench.py's rank loop (TEST INFRASTRUCTURE ONLY).

bench.py loads it when CHIARO_BENCH_BACKEND names it ("<this file>:make"), so a
test can run the benchmark's own multi-rank path -- spawn_ranks, the WORLD_SIZE
check, per-rank timing, the slowest-rank step, the tile gather and the JSON line
-- on the CPU: gloo between the ranks and, in place of the C-ABI device, an
oracle-backed one with the same entry points (render_device / render_tiles_device
/ blend_tiles_device taking buffer addresses, set_option, counters,
last_kernel_ms, trace_stats).  The product never imports this file.
"""
from __future__ import annotations

import ctypes
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for _p in (ROOT / "oracle", ROOT / "tests"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))


def _view(ptr: int, shape):
    n = int(np.prod(shape))
    return np.ctypeslib.as_array((ctypes.c_float * n).from_address(ptr)).reshape(shape)


class OracleDevice:
    """The oracle (oracle/liboracle.so) behind the Device entry points bench.py uses."""

    def __init__(self, model, info):
        import pyoracle as po
        self.osc = po.OracleScene(model.triangles(), leaf_size=info["leaf_size"], textures=model.textures(),
                                  build_threads=2)
        self.bg = info["background"]
        self.opts = {}
        self.last = {}
        self.last_ms = 0.0

    def set_option(self, key, value):
        self.opts[key] = int(value)

    def _means(self, cam, p, px, py):
        t0 = time.perf_counter()
        mean, c = self.osc.render_pixels(cam.as_array(), p.xres, p.yres, p.spp, p.k, p.seed, px, py, layer=p.layer,
                                         bg=self.bg, threads=2)
        self.last_ms = (time.perf_counter() - t0) * 1e3
        import chiaroscuro_amd as ca
        self.last = {n: 0 for n in ca.COUNTER_NAMES}
        self.last.update(c)
        self.last["pixels"] = len(px)
        return mean

    def render_tiles_device(self, cam, p, ptr, stream=0, _in_group=False):
        from chiaroscuro_amd.tiles import TileLayout
        if not _in_group:
            self._log_pass(p, 1)
        lay = TileLayout(p.xres, p.yres, p.nranks, p.tile)
        T = lay.tile
        buf = _view(ptr, (lay.max_tiles, T, T, 3))
        tiles = [(lt,) + lay.tile_origin(p.rank, lt) for lt in range(lay.tiles_for_rank(p.rank))]
        px, py, where = [], [], []
        for lt, x0, y0 in tiles:
            for yy in range(min(T, p.yres - y0)):
                for xx in range(min(T, p.xres - x0)):
                    px.append(x0 + xx)
                    py.append(y0 + yy)
                    where.append((lt, yy, xx))
        mean = self._means(cam, p, px, py)
        for i, (lt, yy, xx) in enumerate(where):
            buf[lt, yy, xx] = mean[i]

    def blend_tiles_device(self, p, gathered_ptr, frame_ptr, stream=0):
        from chiaroscuro_amd.tiles import TileLayout
        from test_distributed import blend_tiles_reference
        lay = TileLayout(p.xres, p.yres, p.nranks, p.tile)
        g = _view(gathered_ptr, (p.nranks, lay.max_tiles, lay.tile, lay.tile, 3))
        blend_tiles_reference(g, lay, _view(frame_ptr, (p.yres, p.xres, 3)), p.layer)

    def blend_tiles_layers_device(self, p, n, gathered_ptr, frame_ptr, stream=0):
        """gathered [nranks][n][max_tiles][T][T][3]: layers p.layer .. + n - 1 in order."""
        from chiaroscuro_amd.tiles import TileLayout, _with_layer
        from test_distributed import blend_tiles_reference
        lay = TileLayout(p.xres, p.yres, p.nranks, p.tile)
        g = _view(gathered_ptr, (p.nranks, n, lay.max_tiles, lay.tile, lay.tile, 3))
        for j in range(n):
            blend_tiles_reference(np.ascontiguousarray(g[:, j]), lay, _view(frame_ptr, (p.yres, p.xres, 3)),
                                  p.layer + j)

    def render_device(self, cam, p, frame_ptr, stream=0):
        ys, xs = np.mgrid[0:p.yres, 0:p.xres]
        mean = self._means(cam, p, xs.ravel(), ys.ravel()).reshape(p.yres, p.xres, 3)
        f = _view(frame_ptr, (p.yres, p.xres, 3))
        f[...] = mean if p.layer == 1 else (f * np.float32(p.layer - 1) + mean) / np.float32(p.layer)

    # several layers per pass: the oracle renders them one by one (the GPU path renders them in
    # one pass, bit-identical); counters and time add up over the pass
    def layers_per_pass(self, p, want):
        return want

    def layers_per_group(self, p, want):
        """cr_layers_per_group's stand-in: what this rank's share holds.  CHIARO_TEST_ODD_RANK_CAP=c caps
        the odd ranks at c layers, so the ranks plan differently and DistributedFrame.plan_layers' all-reduce
        MIN has to make them agree (tests/test_bench_distributed.py)."""
        cap = int(os.environ.get("CHIARO_TEST_ODD_RANK_CAP", "0") or 0)
        return min(want, cap) if cap and p.rank % 2 == 1 else want

    def _log_pass(self, p, n):
        """CHIARO_TEST_PLAN_LOG=dir: every rank appends the (first layer, layers) of each pass it renders to
        dir/rank<r>.txt, so a test can check that all ranks rendered the same groups."""
        d = os.environ.get("CHIARO_TEST_PLAN_LOG")
        if d:
            with open(os.path.join(d, "rank%d.txt" % p.rank), "a") as f:
                f.write("%d %d\n" % (p.layer, n))

    def _layers(self, p, n, one):
        from chiaroscuro_amd.tiles import _with_layer
        tot, ms = {}, 0.0
        for j in range(n):
            one(j, _with_layer(p, p.layer + j))
            ms += self.last_ms
            for key, v in self.last.items():
                tot[key] = tot.get(key, 0) + v
        self.last, self.last_ms = tot, ms

    def render_tiles_layers_device(self, cam, p, n, ptr, stream=0):
        from chiaroscuro_amd.tiles import TileLayout
        self._log_pass(p, n)
        lay = TileLayout(p.xres, p.yres, p.nranks, p.tile)
        stride = lay.max_tiles * lay.tile * lay.tile * 3 * 4
        self._layers(p, n, lambda j, q: self.render_tiles_device(cam, q, ptr + j * stride, stream, True))

    def render_layers_device(self, cam, p, n, frame_ptr, stream=0):
        self._layers(p, n, lambda j, q: self.render_device(cam, q, frame_ptr, stream))

    def counters(self):
        return dict(self.last)

    def last_kernel_ms(self):
        return self.last_ms

    def trace_stats(self):
        import chiaroscuro_amd as ca
        return {k: {"launches": 0, "ms": 0.0, "inner": 0, "leaf": 0, "tritest": 0} for k in ca.TRACE_KINDS}


class CpuOracleBackend:
    name = "cpu-oracle"
    device = "cpu"
    dist_backend = "gloo"

    def init_rank(self, world, local, timeout_s=120.0):
        if world > 1:
            import datetime
            import torch.distributed as dist
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=timeout_s + 30.0))
            return dist
        return None

    def collectives_version(self):
        return "gloo"

    def synchronize(self):
        pass

    def stream(self):
        return 0

    def make_device(self, index, info, model, kd, opts):
        dev = OracleDevice(model, info)
        for key, val in opts:
            dev.set_option(key, val)
        return dev


def make():
    return CpuOracleBackend()
