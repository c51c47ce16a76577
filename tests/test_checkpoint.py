"""Checkpoint / resume of a progressive render (the persisted counterpart of
src/rayTracer.cpp:18-33, 64): the file format round-trips bit for bit, a checkpoint of
another frame or scene is refused, and a render resumed from a checkpoint continues
the layers exactly as an uninterrupted one (GPU: RayTracer; CPU: the multi-rank
DistributedFrame with the oracle-backed stand-in)."""
import numpy as np
import pytest


def _header(ca, kd, info, layers=3):
    h = ca.Checkpoint()
    h.xres, h.yres, h.samples, h.k, h.seed, h.layers = info["xres"], info["yres"], info["samples"], info["k"], \
        info["seed"], layers
    for name, v in (("eye", info["VP"]), ("center", info["LA"]), ("up", info["UP"]), ("background", info["background"])):
        getattr(h, name)[:] = [float(x) for x in v]
    h.yview = info["yview"]
    h.scene = kd.fingerprint()
    return h


def test_checkpoint_file_roundtrip_and_refusals(ca, scenes, tmp_path):
    sc = ca.Scene(scenes.config_rtc("cornell"), "xres", "20", "yres", "12")
    info = sc.info
    kd = ca.KDTree(ca.Model(sc), sc)
    h = _header(ca, kd, info)
    px = np.random.default_rng(3).standard_normal((12, 20, 3)).astype(np.float32)
    px[0, 0] = [np.inf, -0.0, np.nan]
    path = tmp_path / "frame.chk"
    ca.checkpoint_write(path, h, px)
    h2, px2 = ca.checkpoint_read(path)
    assert (px2.view(np.uint32) == px.view(np.uint32)).all()
    assert (h2.xres, h2.yres, h2.layers, h2.scene, h2.yview) == (20, 12, 3, kd.fingerprint(), np.float32(info["yview"]))
    assert list(h2.eye) == [np.float32(v) for v in info["VP"]]
    # another scene has another fingerprint
    sc2 = ca.Scene(scenes.config_rtc("cornell_box"))
    kd2 = ca.KDTree(ca.Model(sc2), sc2)
    assert kd2.fingerprint() != kd.fingerprint()
    # a corrupted pixel is caught by the checksum, a truncated file by its length
    raw = bytearray(path.read_bytes())
    raw[-5] ^= 0x40
    (tmp_path / "bad.chk").write_bytes(bytes(raw))
    with pytest.raises(RuntimeError, match="checksum"):
        ca.checkpoint_read(tmp_path / "bad.chk")
    (tmp_path / "short.chk").write_bytes(path.read_bytes()[:-8])
    with pytest.raises(RuntimeError, match="truncated"):
        ca.checkpoint_read(tmp_path / "short.chk")
    with pytest.raises(RuntimeError, match="not a checkpoint"):
        (tmp_path / "junk.chk").write_bytes(b"x" * 200)
        ca.checkpoint_read(tmp_path / "junk.chk")


@pytest.mark.gpu
def test_raytracer_resume_continues_the_layers(ca, po, scenes, tmp_path):
    over = ("xres", "40", "yres", "28", "samples", "2")
    rtc = scenes.config_rtc("cornell")
    sc = ca.Scene(rtc, *over)
    i = sc.info
    args = (i["VP"], i["LA"], i["UP"], i["yview"])
    m = ca.Model(sc)
    a = ca.RayTracer(m, sc)
    for _ in range(2):
        a.rayTrace(*args)
    path = tmp_path / "p.chk"
    a.checkpoint(path)
    a.rayTrace(*args)  # the uninterrupted third layer
    sc_b = ca.Scene(rtc, *over)
    b = ca.RayTracer(ca.Model(sc_b), sc_b)
    b.resume(path)
    assert b.layers == 2
    b.rayTrace(*args)
    assert b.layers == 3
    assert (b.pixels.view(np.uint32) == a.pixels.view(np.uint32)).all()
    # the oracle's three layers, for good measure
    osc = po.OracleScene(m.triangles(), leaf_size=i["leaf_size"])
    cam = ca.camera(*args, 40, 28).as_array()
    o = None
    for L in (1, 2, 3):
        o, _ = osc.render(cam, 40, 28, 2, i["k"], i["seed"], layer=L, pixels=o)
    assert (b.pixels.view(np.uint32) == o.view(np.uint32)).all()
    # a checkpoint of another sampling or scene is refused
    sc_c = ca.Scene(rtc, "xres", "40", "yres", "28", "samples", "3")
    c = ca.RayTracer(ca.Model(sc_c), sc_c)
    with pytest.raises(RuntimeError, match="another frame"):
        c.resume(path)
    sc_d = ca.Scene(scenes.config_rtc("cornell_box"), *over)
    d = ca.RayTracer(ca.Model(sc_d), sc_d)
    with pytest.raises(RuntimeError, match="another scene"):
        d.resume(path)
