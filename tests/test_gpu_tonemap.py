"""GPU tonemap (cr_tonemap*, RayTracer::normalizeImage, src/rayTracer.cpp:172-222)
against the oracle's restatement with glibc powf / logf (oracle/oracle.c or_tonemap).

The device evaluates logf / powf in double and rounds once; glibc's are
double-evaluated with a small pre-rounding error, so a float may differ by one
ulp where the value lies within that error of a rounding boundary, and a byte
only if that float also straddles an integer.  Tolerance: every byte within 1,
and at most 1e-4 of the bytes off by one (the test prints the count; measured on
the MI355X: 0 differing bytes in every case below).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PARAMS = [  # exposure, defog, kneeLow, kneeHigh, gamma
    (0.0, 0.0, 0.0, 5.0, 2.2),
    (-3.0, 0.01, 0.0, 5.0, 2.2),
    (2.0, 0.0, -1.0, 3.0, 1.8),
    (1.0, 0.0, 0.0, 5.0, 1.0),
]


def _hdr_frame(h=384, w=512, seed=7):
    rng = np.random.default_rng(seed)
    v = np.exp(rng.uniform(np.log(1e-6), np.log(1e4), size=(h, w, 3))).astype(np.float32)
    v[0, :8] = [[0, 0, 0], [-1, -0.5, -1e-9], [np.inf, 1, 2], [np.nan, 0.5, 3], [1e30, 1e-30, 5e-45],
                [0.25, 0.5, 1.0], [2.0, 4.0, 8.0], [16.0, 32.0, 64.0]]
    return v


def _compare(got, want, what):
    d = np.abs(got.astype(np.int32) - want.astype(np.int32))
    n1 = int((d > 0).sum())
    print("%s: %d of %d bytes differ by one" % (what, n1, d.size))
    assert int(d.max()) <= 1, what
    assert n1 <= max(1, d.size // 10000), what


@pytest.mark.parametrize("prm", PARAMS)
def test_tonemap_device_matches_oracle(ca, po, prm):
    import torch
    rgb = _hdr_frame()
    dev = ca.Device(0)
    t = ca.tonemap_params(*prm)
    d_rgb = torch.from_numpy(rgb).cuda()
    d_out = torch.zeros(rgb.shape, dtype=torch.uint8, device="cuda")
    dev.tonemap_device(t, rgb.shape[1], rgb.shape[0], d_rgb.data_ptr(), d_out.data_ptr())
    torch.cuda.synchronize()
    _compare(d_out.cpu().numpy(), po.tonemap(rgb, *prm), "synthetic %s" % (prm,))


def test_raytracer_normalize_image_on_rendered_frame(ca, po, scenes):
    """RayTracer.normalizeImage (GPU) on a rendered nanobox frame vs or_tonemap on its pixels."""
    sc = ca.Scene(scenes.config_rtc("nanobox"), "xres", "160", "yres", "90", "samples", "4")
    m = ca.Model(sc)
    rt = ca.RayTracer(m, sc)
    i = sc.info
    rt.rayTrace(i["VP"], i["LA"], i["UP"], i["yview"])
    for prm in PARAMS[:2]:
        rt.normalizeImage(*prm)
        _compare(rt.getData(), po.tonemap(rt.pixels, *prm), "nanobox %s" % (prm,))
    rt.normalizeImage()  # exposure = the scene's (.rtc), as the reference's default
    _compare(rt.getData(), po.tonemap(rt.pixels, i["exposure"]), "nanobox scene exposure")


def _read_hdr(path):
    """Radiance RGBE, flat scanlines, -Y H +X W -> [H][W][3] float32 (row 0 = top)."""
    b = open(path, "rb").read()
    hdr_end = b.index(b"\n\n") + 2
    line_end = b.index(b"\n", hdr_end)
    res = b[hdr_end:line_end].split()
    assert res[0] == b"-Y" and res[2] == b"+X"
    h, w = int(res[1]), int(res[3])
    e = np.frombuffer(b[line_end + 1:], np.uint8).reshape(h, w, 4).astype(np.float64)
    scale = np.where(e[..., 3:] > 0, np.ldexp(1.0, (e[..., 3:] - 136).astype(int)), 0.0)
    return (e[..., :3] * scale).astype(np.float32)


def test_export_formats_round_trip(ca, scenes, tmp_path):
    """RayTracer.exportImage (rayTracer.cpp:225-279 with this build's writers, FreeImage
    being absent): PFM holds the float pixels exactly, EXR their halves (HALF PIZ, as
    FreeImage's EXR save; tests/test_exr.py pins the codec against the reference's own
    renders), HDR within RGBE's 8-bit mantissa, PNG and PPM the normalizeImage bytes (top
    row first)."""
    from PIL import Image

    sc = ca.Scene(scenes.config_rtc("nanobox"), "xres", "64", "yres", "36", "samples", "2")
    m = ca.Model(sc)
    rt = ca.RayTracer(m, sc)
    i = sc.info
    rt.rayTrace(i["VP"], i["LA"], i["UP"], i["yview"])
    px = rt.pixels.copy()
    rt.exportImage(str(tmp_path / "a.pfm"))
    rt.exportImage(str(tmp_path / "a.exr"))
    rt.exportImage(str(tmp_path / "a.hdr"))
    rt.exportImage(str(tmp_path / "a.png"))
    rt.exportImage(str(tmp_path / "a.ppm"))
    data = rt.getData().reshape(36, 64, 3)[::-1]  # `data` rows are bottom-up
    raw = open(tmp_path / "a.pfm", "rb").read().split(b"\n", 3)[3]
    pfm = np.frombuffer(raw, "<f4").reshape(36, 64, 3)[::-1]
    assert np.array_equal(pfm.view(np.uint32), px.view(np.uint32))
    assert np.array_equal(ca.exr_read_half(tmp_path / "a.exr"), ca.float_to_half(px))
    hdr = _read_hdr(tmp_path / "a.hdr")
    peak = np.maximum(px.max(axis=2, keepdims=True), 1e-30)
    assert np.all(np.abs(hdr - px) <= peak / 128.0 + 1e-30)
    assert np.array_equal(np.asarray(Image.open(tmp_path / "a.png").convert("RGB")), data)
    assert np.array_equal(np.asarray(Image.open(tmp_path / "a.ppm").convert("RGB")), data)
