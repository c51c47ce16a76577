"""Multi-GPU frame protocol: tile split + one gather per layer.

The frame is cut into `tile`×`tile` tiles, numbered in row-major slots (each row
rotated by its index when nranks > 1, TileLayout.tile_origin); slot s belongs to
rank s % nranks.  Each rank renders its tiles' batch means into a compact
[ntiles_r][tile][tile][3] buffer (cr_render_tiles_device), rank 0 gathers the
buffers over torch.distributed (RCCL over xGMI on GPUs, gloo in the CPU tests)
and unpermutes + blends the layer on the device (cr_blend_tiles_device):
    frame = (frame * (L - 1) + mean) / L           (src/rayTracer.cpp:64)
Every (pixel, sample) is independent and the RNG key holds the global pixel
index, so the image does not depend on the number of ranks.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class TileLayout:
    xres: int
    yres: int
    nranks: int = 1
    tile: int = 32

    @property
    def tiles_x(self) -> int:
        return (self.xres + self.tile - 1) // self.tile

    @property
    def tiles_y(self) -> int:
        return (self.yres + self.tile - 1) // self.tile

    @property
    def ntiles(self) -> int:
        return self.tiles_x * self.tiles_y

    def tiles_for_rank(self, rank: int) -> int:
        """== cr_tiles_for_rank: tiles t < ntiles with t % nranks == rank."""
        n = self.ntiles
        return n // self.nranks + (1 if rank < n % self.nranks else 0)

    @property
    def max_tiles(self) -> int:
        return self.tiles_for_rank(0)

    def tile_origin(self, rank: int, local: int):
        """Pixel origin (x0, y0) of the rank's local tile `local` (== cr_tile_origin):
        slot s = rank + local * nranks; with nranks > 1 tile row s // tiles_x is rotated
        by its index, so a rank's tiles cycle through every column class."""
        s = rank + local * self.nranks
        row, c = divmod(s, self.tiles_x)
        if self.nranks > 1:
            c = (c + row) % self.tiles_x
        return c * self.tile, row * self.tile


class DistributedFrame:
    """One rank's side of a layer: render my tiles, gather to rank 0, blend.

    dev      chiaroscuro_amd.Device of this rank (anything with render_device /
             render_tiles_device / blend_tiles_device taking buffer addresses;
             the gloo tests pass an oracle-backed stand-in with device="cpu")
    dist     torch.distributed (initialised), or None for a single rank
    device   torch device of the frame / tile / gather buffers
    gather   "torch": torch.distributed.gather of the tile buffers (RCCL under the
             nccl backend), blend through cr_blend_tiles_device;
             "cabi": the library's own RCCL communicator (cr_comm_init, the id
             broadcast over `dist`) and cr_render_dist_device (render, grouped
             send / receive to rank 0, blend, async-error polling) per layer
    """

    def __init__(self, dev, xres: int, yres: int, rank: int, nranks: int, tile: int = 32, dist=None,
                 device: str = "cuda", gather: str = "torch"):
        import torch
        if nranks > 1 and (dist is None or dist.get_world_size() != nranks or dist.get_rank() != rank):
            raise ValueError("DistributedFrame: nranks %d / rank %d disagree with the process group" % (nranks, rank))
        if gather not in ("torch", "cabi"):
            raise ValueError("DistributedFrame: gather must be 'torch' or 'cabi'")
        self.dev, self.dist, self.rank, self.gather, self.device = dev, dist, rank, gather, device
        self.layout = TileLayout(xres, yres, nranks, tile)
        L = self.layout
        f32 = dict(dtype=torch.float32, device=device)
        self.frame = torch.zeros((yres, xres, 3), **f32) if rank == 0 or nranks == 1 else None
        split = nranks > 1 and gather == "torch"
        self.tiles = torch.zeros((L.max_tiles, tile, tile, 3), **f32) if split else None
        self.gathered = torch.zeros((nranks, L.max_tiles, tile, tile, 3), **f32) if split and rank == 0 else None
        self.tiles_multi = None  # [nlayers][max_tiles][tile][tile][3] of render_layers
        self.gathered_multi = None  # root: flat store of [nranks][nlayers][max_tiles][tile][tile][3] (render_layers)
        self._stats_begin()
        if nranks > 1 and gather == "cabi":
            uid = [dev.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            dev.comm_init(nranks, rank, uid[0])

    def save(self, path, header):
        """Checkpoint the frame (rank 0; a no-op elsewhere): header is a
        chiaroscuro_amd.Checkpoint describing the frame (layers = the last layer
        rendered, camera, sampling, scene fingerprint).  The file is the one
        RayTracer.checkpoint writes (include/chiaroscuro.h)."""
        if self.frame is None:
            return
        from . import checkpoint_write
        checkpoint_write(path, header, self.frame.cpu().numpy())

    def resume(self, path, expect) -> int:
        """Continue from a checkpoint: rank 0 loads the frame, every rank gets the
        layer count (the next layer to render is that + 1).  `expect` is the
        Checkpoint of this run (layers ignored): another frame, sampling or scene is
        refused, as RayTracer.resume refuses it, and so is another camera -- eye, center
        or yview (src/rayTracer.cpp:23-33 restarts the accumulation when they change;
        `up` is not compared, as the reference's `lastUp == lastUp` never compares it)."""
        import torch
        layers = torch.zeros(1, dtype=torch.int64)
        err = ""
        if self.rank == 0:
            from . import checkpoint_read
            h, px = checkpoint_read(path)
            keys = ("xres", "yres", "samples", "k", "seed", "scene")
            if any(getattr(h, k) != getattr(expect, k) for k in keys) or list(h.background) != list(expect.background):
                err = "resume: the checkpoint is of another frame / sampling / scene"
            elif (list(h.eye) != list(expect.eye) or list(h.center) != list(expect.center)
                  or h.yview != expect.yview):
                err = "resume: the checkpoint is of another camera (eye / center / yview)"
            else:
                self.frame.copy_(torch.from_numpy(px).to(self.frame.device))
                layers[0] = h.layers
        if self.layout.nranks > 1:
            flag = torch.tensor([0 if not err else 1], dtype=torch.int64)
            if self.dist.get_backend() == "nccl":
                layers, flag = layers.cuda(), flag.cuda()
            self.dist.broadcast(layers, src=0)
            self.dist.broadcast(flag, src=0)
            if int(flag.item()):
                err = err or "resume: rank 0 refused the checkpoint"
        if err:
            raise ValueError(err)
        return int(layers.item())

    def plan_layers(self, params, want: int):
        """(layers, pieces) of one render pass group starting at params.layer: up to
        `want` progressive layers rendered together.  Every pass holds the paths of
        `layers` layers of a share of the frame; a pass is filled best when that share is
        small, so on ONE rank the frame is cut into `pieces` (the ranks of a pieces-way
        tile split, each rendered as its own pass of all the layers) -- the smallest
        number whose paths fit one chunk (Device.layers_per_pass).  With several ranks
        a rank's share is its tiles (pieces = 1, the rank's tiles cut into pieces by the
        device itself) and `layers` what fits every rank: the ranks agree on the
        smallest plan (an all-reduce MIN -- collective: every rank calls plan_layers), so
        their per-group gathers pair up."""
        L = self.layout
        want = max(1, int(want))
        if not hasattr(self.dev, "layers_per_pass"):
            return 1, 1
        if L.nranks > 1:  # (cr_render_tiles_layers_device cuts the rank's tiles into pieces itself)
            n = self.dev.layers_per_group(params, want) if hasattr(self.dev, "layers_per_group") \
                else self.dev.layers_per_pass(params, want)
            import torch
            t = torch.tensor([n], dtype=torch.int64, device=self.device)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
            return int(t.item()), 1
        # frame pieces only for scenes with real geometry (cr_scene_triangles; cabi.cpp PIECES_MIN_TRIS)
        max_pieces = min(64, L.ntiles)
        if hasattr(self.dev, "scene_triangles") and self.dev.scene_triangles() < 1024:
            max_pieces = 1
        for nl in range(want, 0, -1):
            for m in range(1, max_pieces + 1):
                q = _with_layer(params, params.layer)
                q.rank, q.nranks = 0, m
                if self.dev.layers_per_pass(q, nl) == nl:
                    return nl, m
        return 1, 1

    def reserve(self, nlayers: int):
        """Allocate the group buffers of up to nlayers layers now (the tile buffers of a rank and the
        root's gathered [nranks][nlayers] buffers), so a timed group does not allocate them."""
        import torch
        L = self.layout
        if L.nranks == 1 or self.gather != "torch" or nlayers < 2:
            return
        if self.tiles_multi is None or self.tiles_multi.shape[0] < nlayers:
            self.tiles_multi = torch.zeros((nlayers,) + tuple(self.tiles.shape), dtype=self.tiles.dtype,
                                           device=self.tiles.device)
        if self.rank == 0:
            self._gathered_view(nlayers)

    def _gathered_view(self, nlayers: int):
        """The root's [nranks][nlayers][max_tiles][T][T][3] gather buffer: a view of the front of a flat
        store that only grows (groups of different sizes reuse it)."""
        import torch
        shape = (self.layout.nranks, nlayers) + tuple(self.tiles.shape)
        n = 1
        for x in shape:
            n *= x
        if self.gathered_multi is None or self.gathered_multi.numel() < n:
            self.gathered_multi = torch.zeros(n, dtype=self.tiles.dtype, device=self.tiles.device)
        return self.gathered_multi[:n].view(shape)

    def render_layers(self, cam, params, nlayers: int, stream: int = 0, pieces: int = 1):
        """Layers params.layer .. + nlayers - 1 as ONE render pass group of my tiles (of each
        of `pieces` frame pieces on a single rank) -- cr_render_layers_device /
        cr_render_tiles_layers_device, bit-identical to nlayers render_layer calls -- then
        ONE gather of the group's tile buffers and one blend of its layers at rank 0
        (cr_blend_tiles_layers_device; the library's own gather: cr_render_dist_layers_device
        does all of it).  (nlayers, pieces) from plan_layers.  last_stats() sums the
        passes' counters."""
        import torch
        L = self.layout
        self._stats_begin()
        if nlayers == 1 and pieces == 1:
            self._render_one(cam, params, stream)
            return
        if (params.rank, params.nranks, params.tile or 32, params.xres, params.yres) != \
                (self.rank, L.nranks, L.tile, L.xres, L.yres):
            raise ValueError("render_layers: params do not match this frame's partition")
        if L.nranks == 1:
            for k in range(pieces):  # piece k: rank k of a pieces-way split, blended in place
                q = _with_layer(params, params.layer)
                q.rank, q.nranks = k, pieces
                self.dev.render_layers_device(cam, q, nlayers, self.frame.data_ptr(), stream)
                self._stats_add()
            return
        if pieces != 1:
            raise ValueError("render_layers: frame pieces on a single rank only")
        if self.gather == "cabi":
            self.dev.render_dist_layers_device(cam, params, nlayers, self.frame.data_ptr() if self.rank == 0 else 0,
                                               stream)
            self._stats_add()
            return
        if self.tiles_multi is None or self.tiles_multi.shape[0] < nlayers:
            self.tiles_multi = torch.zeros((nlayers,) + tuple(self.tiles.shape), dtype=self.tiles.dtype,
                                           device=self.tiles.device)
        mine = self.tiles_multi[:nlayers]  # [nlayers][max_tiles][T][T][3], contiguous
        self.dev.render_tiles_layers_device(cam, params, nlayers, mine.data_ptr(), stream)
        self._stats_add()
        if not hasattr(self.dev, "blend_tiles_layers_device"):  # (a device with the one-layer blend only)
            for j in range(nlayers):
                self.dist.gather(mine[j], [self.gathered[r] for r in range(L.nranks)] if self.rank == 0 else None,
                                 dst=0)
                if self.rank == 0:
                    self.dev.blend_tiles_device(_with_layer(params, params.layer + j), self.gathered.data_ptr(),
                                                self.frame.data_ptr(), stream)
            return
        # one gather of the whole group: rank r's nlayers buffers land at the root's [r], then one blend
        g = self._gathered_view(nlayers) if self.rank == 0 else None
        self.dist.gather(mine, [g[r] for r in range(L.nranks)] if self.rank == 0 else None, dst=0)
        if self.rank == 0:
            self.dev.blend_tiles_layers_device(params, nlayers, g.data_ptr(), self.frame.data_ptr(), stream)

    # the device's counters, pass time and trace stats summed over the passes of the last
    # render_layer(s) call
    def _stats_begin(self):
        self._stats = {"counters": {}, "kernel_ms": 0.0, "trace": None, "passes": 0}

    def _stats_add(self):
        st = self._stats
        st["passes"] += 1
        if not hasattr(self.dev, "counters"):  # (a device with the render / blend calls only)
            return
        for key, v in self.dev.counters().items():
            st["counters"][key] = st["counters"].get(key, 0) + v
        st["kernel_ms"] += self.dev.last_kernel_ms()
        if hasattr(self.dev, "trace_stats"):
            ts = self.dev.trace_stats()
            if st["trace"] is None:
                st["trace"] = {k: dict(v) for k, v in ts.items()}
            else:
                for kind, v in ts.items():
                    for key, x in v.items():
                        st["trace"][kind][key] += x

    def last_stats(self):
        """{"counters", "kernel_ms", "trace", "passes"} of the last render_layer(s) call."""
        return self._stats

    def _render_one(self, cam, params, stream):
        self.render_layer(cam, params, stream, _keep_stats=True)

    def render_layer(self, cam, params, stream: int = 0, _keep_stats: bool = False):
        """params: chiaroscuro_amd.render_params(..., layer=L, rank, nranks, tile)."""
        if not _keep_stats:
            self._stats_begin()
        L = self.layout
        if (params.rank, params.nranks, params.tile or 32, params.xres, params.yres) != \
                (self.rank, L.nranks, L.tile, L.xres, L.yres):
            raise ValueError("render_layer: params do not match this frame's partition")
        if L.nranks == 1:
            self.dev.render_device(cam, params, self.frame.data_ptr(), stream)
            self._stats_add()
            return
        if self.gather == "cabi":
            self.dev.render_dist_device(cam, params, self.frame.data_ptr() if self.rank == 0 else 0, stream)
            self._stats_add()
            return
        self.dev.render_tiles_device(cam, params, self.tiles.data_ptr(), stream)
        self._stats_add()
        self.dist.gather(self.tiles, [self.gathered[r] for r in range(L.nranks)] if self.rank == 0 else None, dst=0)
        if self.rank == 0:
            self.dev.blend_tiles_device(params, self.gathered.data_ptr(), self.frame.data_ptr(), stream)


def _with_layer(params, layer: int):
    """A copy of render params (a ctypes struct) with another layer."""
    q = type(params).from_buffer_copy(params)
    q.layer = layer
    return q
