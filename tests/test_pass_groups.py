"""Pass-group planning on the CPU (DistributedFrame.plan_layers): with a stand-in
device whose chunk holds `cap` paths, one rank cuts the frame into the fewest tile-split pieces
whose paths fit, scenes below 1024 triangles are never cut, several ranks take what fits their
share (the library pieces a rank's tiles itself) -- the smallest plan over the ranks, agreed by an
all-reduce MIN -- with either gather (torch.distributed or the library's own).  No GPU: the GPU tests render the plans (tests/test_gpu_parity.py)."""
import pytest


class PlanDevice:
    """Only what plan_layers asks: cr_layers_per_pass / cr_layers_per_group / cr_scene_triangles
    over a chunk of `cap` paths (the C-ABI's rule: a rank's items x spp x layers <= cap)."""

    def __init__(self, cap, tris=100000):
        self.cap, self.tris = cap, tris

    def _paths(self, p, nl):
        from chiaroscuro_amd.tiles import TileLayout
        lay = TileLayout(p.xres, p.yres, p.nranks, p.tile or 32)
        return lay.tiles_for_rank(p.rank) * lay.tile * lay.tile * p.spp * nl

    def layers_per_pass(self, p, want):
        nl = want
        while nl > 1 and self._paths(p, nl) > self.cap:
            nl -= 1
        return nl

    def scene_triangles(self):
        return self.tris

    def comm_unique_id(self):  # (gather="cabi" construction only)
        return b"id"

    def comm_init(self, nranks, rank, uid):
        pass


def params(ca, layer=1, rank=0, nranks=1, spp=128):
    return ca.render_params(1920, 1080, spp, 6, 1, layer=layer, rank=rank, nranks=nranks, tile=32)


def frame(dev, nranks=1, rank=0, gather="torch", others=()):
    """others: the plans (layers) the other ranks bring to plan_layers' all-reduce MIN."""
    from chiaroscuro_amd.tiles import DistributedFrame

    class Dist:  # a process group of nranks
        class ReduceOp:
            MIN = "min"

        def get_world_size(self):
            return nranks

        def get_rank(self):
            return rank

        def broadcast_object_list(self, lst, src=0):
            pass

        def all_reduce(self, t, op=None):
            assert op == "min"
            for v in others:
                t[0] = min(int(t[0]), v)

    return DistributedFrame(dev, 1920, 1080, rank, nranks, 32, Dist() if nranks > 1 else None, device="cpu",
                            gather=gather)


def test_one_rank_frame_pieces(ca):
    dev = PlanDevice(cap=1 << 28)  # the library's wf_paths: one 1080p x 128 spp layer (2040 tiles) fits
    fr = frame(dev)
    assert fr.plan_layers(params(ca), 1) == (1, 1)
    assert fr.plan_layers(params(ca), 16) == (16, 16)
    assert fr.plan_layers(params(ca), 8) == (8, 8)
    assert fr.plan_layers(params(ca), 5) == (5, 5)
    # 20 layers: 2040 / 20 = 102 tiles a piece -- the fewest pieces that fit
    assert fr.plan_layers(params(ca), 20) == (20, 20)
    # more layers than 64 pieces can hold: the largest group that fits
    nl, m = fr.plan_layers(params(ca), 128)
    assert m <= 64 and nl < 128 and dev._paths(_piece(ca, m), nl) <= dev.cap


def _piece(ca, m):
    p = params(ca)
    p.rank, p.nranks = 0, m
    return p


def test_small_scene_no_pieces(ca):
    dev = PlanDevice(cap=1 << 28, tris=36)
    assert frame(dev).plan_layers(params(ca), 16) == (1, 1)
    small = PlanDevice(cap=4 << 28, tris=36)  # four layers fit the whole frame: no pieces needed
    assert frame(small).plan_layers(params(ca), 16) == (4, 1)


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_ranks_take_what_fits(ca, nranks):
    dev = PlanDevice(cap=1 << 28)  # (no layers_per_group: the rank's share is not cut)
    fr = frame(dev, nranks=nranks, rank=nranks - 1)
    nl, m = fr.plan_layers(params(ca, rank=nranks - 1, nranks=nranks), 16)
    assert m == 1 and nl == min(16, nranks)
    # the library's own gather plans the same groups (cr_render_dist_layers_device)
    assert frame(dev, nranks=nranks, gather="cabi").plan_layers(params(ca, nranks=nranks), 16) == (nl, 1)
    # a rank whose share fits fewer layers: every rank takes the smallest plan
    fr = frame(dev, nranks=nranks, rank=0, others=(nl - 1,) if nl > 1 else ())
    assert fr.plan_layers(params(ca, rank=0, nranks=nranks), 16) == (max(nl - 1, 1), 1)
