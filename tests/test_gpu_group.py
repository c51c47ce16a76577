"""The multi-GPU C-ABI (csrc/group.cpp) on one MI355X.

cr_group: a one-GPU group runs RCCL's communicator of one rank; a group that
lists the same device several times runs the whole N-rank protocol (per-rank
passes on their own host threads, compact tile buffers, gather into the root's
slots, unpermute + progressive blend) with device copies in place of the RCCL
send / receive.  cr_comm / cr_render_dist_device: a one-rank RCCL communicator.
All bit-exact with the oracle's single-process render, counters summed over
the ranks equal to the oracle's."""
import numpy as np
import pytest

from helpers import Pair, assert_bitwise

pytestmark = pytest.mark.gpu

KEYS = ("closest", "shadow", "inner", "leaf", "tritest", "hit", "texhit", "paths")
SEED = 0xC41A05C0


@pytest.fixture(scope="module")
def sponza(ca, po, scenes):
    return Pair(ca, po, scenes.config_rtc("sponza"), device=False)


@pytest.mark.parametrize("devices,size", [([0], (96, 54, 3)), ([0, 0, 0, 0], (310, 180, 2)),
                                          ([0, 0, 0, 0, 0, 0, 0, 0], (200, 120, 2))])
def test_group_render_layers_bitexact(ca, sponza, devices, size):
    x, y, s = size
    g = ca.Group(devices)
    g.upload(sponza.kd.describe())
    g.set_option("wf_tail_min", 0)
    cam = sponza.camera(ca, x, y)
    o = None
    for layer in (1, 2):
        p = ca.render_params(x, y, s, 6, SEED, layer=layer)
        img = g.render(cam, p)
        gc = g.counters()
        o, oc = sponza.oracle.render(cam.as_array(), x, y, s, 6, SEED, layer=layer, pixels=o)
        assert_bitwise(img, o, "group %s layer %d" % (devices, layer))
        assert {k: gc[k] for k in KEYS} == oc
        assert gc["pixels"] == x * y
    ms = g.rank_ms()
    assert len(ms) == len(devices) and all(t > 0 for t in ms)
    g.close()


def test_group_tonemap_equals_single_ctx(ca, sponza):
    """cr_group_tonemap on the root's accumulator == cr_tonemap of a single-GPU render."""
    import ctypes
    x, y = 64, 40
    cam = sponza.camera(ca, x, y)
    p = ca.render_params(x, y, 2, 6, SEED)
    g = ca.Group([0, 0])
    g.upload(sponza.kd.describe())
    g.render(cam, p)
    d = ca.Device(0)
    d.upload(sponza.kd.describe())
    d.render(cam, p)
    t = ca.tonemap_params(2.0)
    a = np.zeros((y, x, 3), np.uint8)
    b = np.zeros((y, x, 3), np.uint8)
    hip, _ = ca.libs()
    assert hip.cr_group_tonemap(g._g, ctypes.byref(t), x, y, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) == 0
    assert hip.cr_tonemap(d._c, ctypes.byref(t), x, y, b.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) == 0
    assert np.array_equal(a, b) and a.any()
    g.close()
    d.close()


def test_comm_one_rank_render_dist(ca, sponza):
    """cr_comm_init (ncclCommInitRank, one rank) + cr_render_dist_device over two layers."""
    import torch
    x, y, s = 96, 54, 2
    d = ca.Device(0)
    d.upload(sponza.kd.describe())
    d.comm_init(1, 0, ca.Device.comm_unique_id())
    cam = sponza.camera(ca, x, y)
    frame = torch.zeros((y, x, 3), dtype=torch.float32, device="cuda")
    o = None
    for layer in (1, 2):
        p = ca.render_params(x, y, s, 6, SEED, layer=layer)
        d.render_dist_device(cam, p, frame.data_ptr())
        torch.cuda.synchronize()
        o, _ = sponza.oracle.render(cam.as_array(), x, y, s, 6, SEED, layer=layer, pixels=o)
        assert_bitwise(frame.cpu().numpy(), o, "cr_render_dist_device layer %d" % layer)
    d.comm_destroy()
    with pytest.raises(RuntimeError):
        d.render_dist_device(cam, ca.render_params(x, y, s, 6, SEED), frame.data_ptr())
    d.close()


def test_raytracer_gpus_key(ca, scenes):
    """The additive .rtc key `gpus`: a RayTracer whose layers are split over a
    group (3 ranks, wrapping onto the one GPU of the test box) renders the same
    progressive layers as the plain one, and normalizeImage gives the same bytes."""
    rtc = scenes.config_rtc("cornell")
    out, data = [], []
    for gpus in ("1", "3"):
        sc = ca.Scene(rtc, "xres", "40", "yres", "30", "samples", "2", "gpus", gpus)
        assert sc.info["gpus"] == int(gpus) and sc.info["n_invalid"] == 0
        rt = ca.RayTracer(ca.Model(sc), sc)
        i = sc.info
        rt.rayTrace(i["VP"], i["LA"], i["UP"], i["yview"])
        rt.rayTrace(i["VP"], i["LA"], i["UP"], i["yview"])
        assert rt.layers == 2
        out.append(rt.pixels)
        rt.normalizeImage(2.0)
        data.append(rt.getData())
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32)) and out[0].any()
    assert np.array_equal(data[0], data[1])


def test_missing_peers_fail_cleanly(ca):
    """The driver's N-GPU paths must fail, not hang, when their peers are missing: on a
    one-GPU box a communicator of two ranks never forms -- cr_comm_init returns
    CR_E_COMM once its deadline ("comm_timeout_ms") passes -- and a group over two
    distinct devices fails its create (the second device does not exist) with the
    reason, and is destroyed cleanly (the rank buffers are sized before the contexts)."""
    import time
    if ca.Device.device_count() >= 2:
        pytest.skip("needs a box with exactly one GPU")
    dev = ca.Device(0)
    dev.set_option("comm_timeout_ms", 3000)
    uid = ca.Device.comm_unique_id()
    t0 = time.time()
    with pytest.raises(RuntimeError, match="CR_E_COMM"):
        dev.comm_init(2, 0, uid)
    assert time.time() - t0 < 60
    with pytest.raises(RuntimeError, match="device 1"):
        ca.Group([0, 1])
    with pytest.raises(RuntimeError, match="device 99"):
        ca.Group([0, 99])


@pytest.mark.parametrize("devices,size,nl,paths", [([0], (96, 54, 2), 3, 1 << 28), ([0], (96, 54, 2), 3, 12000),
                                                   ([0, 0, 0, 0], (310, 180, 2), 4, 1 << 28),
                                                   ([0, 0, 0, 0], (310, 180, 2), 4, 20000),
                                                   ([0] * 8, (310, 180, 2), 4, 20000)])
def test_group_render_pass_groups_bitexact(ca, sponza, devices, size, nl, paths):
    """cr_group_render_layers: each rank renders its tiles of a whole group of layers in one pass
    group (in pieces when `wf_paths` makes its share too large for one chunk), ONE gather of the
    group's buffers and one blend of its layers at the root -- bit-identical to the oracle's layer
    after layer, counters summed over ranks, passes and layers; then a single layer on top."""
    x, y, s = size
    g = ca.Group(devices)
    g.upload(sponza.kd.describe())
    g.set_option("counters", 0)
    g.set_option("wf_paths", paths)
    cam = sponza.camera(ca, x, y)
    img = g.render_layers(cam, ca.render_params(x, y, s, 6, SEED, layer=1), nl)
    gc = g.counters()
    o, rays = None, 0
    for layer in range(1, nl + 1):
        o, oc = sponza.oracle.render(cam.as_array(), x, y, s, 6, SEED, layer=layer, pixels=o)
        rays += oc["closest"] + oc["shadow"]
    assert_bitwise(img, o, "group %d ranks, %d layers, wf_paths %d" % (len(devices), nl, paths))
    assert gc["closest"] + gc["shadow"] == rays and gc["pixels"] == x * y * nl
    img = g.render(cam, ca.render_params(x, y, s, 6, SEED, layer=nl + 1))
    o, _ = sponza.oracle.render(cam.as_array(), x, y, s, 6, SEED, layer=nl + 1, pixels=o)
    assert_bitwise(img, o, "group %d ranks, layer %d after the group" % (len(devices), nl + 1))
    assert all(t > 0 for t in g.rank_ms())
    g.close()


def test_comm_one_rank_render_dist_layers(ca, sponza):
    """cr_render_dist_layers_device on a one-rank communicator: the frame's layers in pass groups
    (frame pieces by wf_paths), then one layer, bit-exact; blend of several layers in one launch
    (cr_blend_tiles_layers_device) equal to layer-by-layer blends."""
    import torch
    x, y, s, nl = 96, 54, 2, 3
    d = ca.Device(0)
    d.upload(sponza.kd.describe())
    d.set_option("counters", 0)
    d.set_option("wf_paths", 9000)
    d.comm_init(1, 0, ca.Device.comm_unique_id())
    cam = sponza.camera(ca, x, y)
    frame = torch.zeros((y, x, 3), dtype=torch.float32, device="cuda")
    d.render_dist_layers_device(cam, ca.render_params(x, y, s, 6, SEED, layer=1), nl, frame.data_ptr())
    torch.cuda.synchronize()
    o = None
    for layer in range(1, nl + 1):
        o, _ = sponza.oracle.render(cam.as_array(), x, y, s, 6, SEED, layer=layer, pixels=o)
    assert_bitwise(frame.cpu().numpy(), o, "cr_render_dist_layers_device %d layers" % nl)
    d.comm_destroy()
    # the multi-layer blend: gathered [nranks][nl][tiles] of a 3-rank split, one launch vs nl launches
    p = ca.render_params(x, y, s, 6, SEED, layer=2, nranks=3, tile=16)
    nt = ca.Device.tiles_for_rank(p, 0)
    gathered = torch.rand((3, nl, nt, 16, 16, 3), dtype=torch.float32, device="cuda")
    base = torch.rand((y, x, 3), dtype=torch.float32, device="cuda")
    a, b = base.clone(), base.clone()
    d.blend_tiles_layers_device(p, nl, gathered.data_ptr(), a.data_ptr())
    for j in range(nl):
        q = ca.render_params(x, y, s, 6, SEED, layer=2 + j, nranks=3, tile=16)
        one = gathered[:, j].contiguous()
        d.blend_tiles_device(q, one.data_ptr(), b.data_ptr())
    torch.cuda.synchronize()
    assert_bitwise(a.cpu().numpy(), b.cpu().numpy(), "multi-layer blend")
    d.close()


def test_raytracer_gpus_key_pass_groups(ca, po, scenes):
    """RayTracer::rayTraceLayers with the `gpus` key renders through cr_group_render_layers: the
    layers of a pass group split over 3 ranks equal the one-GPU layers and the oracle's."""
    rtc = scenes.config_rtc("sponza")
    out = []
    for gpus in ("1", "3"):
        sc = ca.Scene(rtc, "xres", "80", "yres", "45", "samples", "2", "gpus", gpus)
        i = sc.info
        rt = ca.RayTracer(ca.Model(sc), sc)
        rt.rayTraceLayers(3, i["VP"], i["LA"], i["UP"], i["yview"])
        assert rt.layers == 3
        rt.rayTrace(i["VP"], i["LA"], i["UP"], i["yview"])
        assert rt.layers == 4
        out.append(rt.pixels)
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32)) and out[0].any()
    m = ca.Model(sc)
    osc = po.OracleScene(m.triangles(), leaf_size=i["leaf_size"], textures=m.textures())
    cam = ca.camera(i["VP"], i["LA"], i["UP"], i["yview"], 80, 45).as_array()
    o = None
    for L in range(1, 5):
        o, _ = osc.render(cam, 80, 45, 2, i["k"], i["seed"], layer=L, pixels=o)
    assert np.array_equal(out[1].view(np.uint32), o.view(np.uint32))
