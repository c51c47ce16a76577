"""The preview's render path without a window (host/preview.cpp):
R at a fixed camera accumulates progressive layers exactly as
src/openglPreview.cpp:139-146, 247-257 drives RayTracer::rayTrace; the screen
texture is getData() after normalizeImage(); = / - re-normalise without a new
layer; moving the camera restarts the accumulation.  Pixels are compared with
the oracle's progressive render at the preview camera."""
import math

import numpy as np
import pytest

from helpers import Pair, assert_bitwise

pytestmark = pytest.mark.gpu


def test_preview_progressive_render(ca, po, scenes):
    rtc = scenes.config_rtc("cornell")
    over = ("xres", "48", "yres", "36", "samples", "2")
    sc = ca.Scene(rtc, *over)
    rt = ca.RayTracer(ca.Model(sc), sc)
    pv = ca.Preview(sc, rt)
    i = sc.info
    st = pv.state()
    np.testing.assert_array_equal(st["position"], np.float32(i["VP"]))
    assert st["zoom"] == pytest.approx(math.degrees(2 * math.atan(0.5 * i["yview"])), rel=1e-6)
    assert not st["show_render"] and st["renders"] == 0
    pair = Pair(ca, po, rtc, *over, device=False)

    def oracle_layers(st, n):
        yview = np.float32(2 * math.tan(st["zoom"] * math.pi / 360.0))
        center = (st["position"] + st["front"]).astype(np.float32)
        cam = ca.camera(st["position"], center, st["up"], float(yview), 48, 36).as_array()
        o = None
        for L in range(1, n + 1):
            o, _ = pair.oracle.render(cam, 48, 36, 2, i["k"], i["seed"], layer=L, pixels=o)
        return o

    # the reference camera's Yaw starts as atan2 in radians but is read as degrees
    # (src/camera.cpp:16, 76): from cornell's VP / LA it looks along +x, out of the
    # box; turn it to -z (yaw -90 degrees) with the mouse as a user would
    pv.mouse(-900.0, 0.0)
    assert pv.state()["front"][2] < -0.99
    for n in (1, 2, 3):  # R pressed three times at one camera: layers 1..3
        pv.key("R")
        assert rt.layers == n and pv.state()["renders"] == n and pv.state()["show_render"]
    assert_bitwise(rt.pixels, oracle_layers(pv.state(), 3), "preview 3 layers")
    tex = pv.texture()
    rt.normalizeImage()
    assert np.array_equal(tex, rt.getData()) and tex.any()
    pv.key("=")  # exposure + 0.2: re-normalised, no new layer
    assert rt.layers == 3 and sc.info["exposure"] == pytest.approx(i["exposure"] + 0.2)
    assert not np.array_equal(pv.texture(), tex)
    pv.key("W", dt=0.5)  # ignored while the render is shown
    np.testing.assert_array_equal(pv.state()["position"], np.float32(i["VP"]))
    pv.key("TAB")
    pv.key("W", dt=0.5)
    pv.mouse(12.0, -4.0)
    pv.scroll(3.0)
    st = pv.state()
    assert not np.array_equal(st["position"], np.float32(i["VP"]))
    pv.key("R")  # new camera: accumulation restarts
    assert rt.layers == 1
    assert_bitwise(rt.pixels, oracle_layers(pv.state(), 1), "preview after move")


def test_preview_shift_applies_to_the_next_move(ca, scenes):
    """src/openglPreview.cpp:181-196: a frame's movement keys move at the speed the
    previous frame left (2.5, or 30 with LEFT_SHIFT held), and only then does the
    frame set the speed from the shift key.  Toggling shift between moves must
    therefore change the NEXT move's step, not this one's."""
    sc = ca.Scene(scenes.config_rtc("cornell"), "xres", "16", "yres", "16", "samples", "1")
    rt = ca.RayTracer(ca.Model(sc), sc)
    pv = ca.Preview(sc, rt)
    front = pv.state()["front"].astype(np.float32)
    pos = pv.state()["position"].astype(np.float32)
    # (key, dt, shift) -> the speed this move uses: the one the previous frame left
    speed = np.float32(2.5)
    for key, dt, shift in (("W", 0.5, False), ("W", 0.5, True), ("W", 0.25, False), ("SHIFT", 0.0, True),
                           ("W", 0.125, True), ("S", 0.5, False)):
        pv.key(key, dt=dt, shift=shift)
        if key != "SHIFT":
            v = np.float32(speed * np.float32(dt))  # ProcessKeyboard's velocity (src/camera.cpp:33)
            pos = (pos + front * v) if key == "W" else (pos - front * v)
        speed = np.float32(30.0 if shift else 2.5)
        np.testing.assert_array_equal(pv.state()["position"], pos.astype(np.float32), err_msg=key)
