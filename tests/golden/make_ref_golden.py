"""Generate the reference-pinned golden vectors (run in the build container only).

Builds oracle/_ref/libref_harness.so from the reference's OWN sources
(src/mesh.cpp -> Texture::getColorAt, the vendored glm 0.9.8.5 for the camera
of src/rayTracer.cpp:41-49 and the vector primitives; see oracle/ref/ref_harness.cpp)
and records its outputs on fixed inputs as JSON fixtures:

  ref_texture.json  G5: Texture::getColorAt at wrap / edge coordinates, RGB, RGBA, grey
  ref_glm.json      G6 camera bases + normalize / cross / dot / distance / material
                    normal / light surface on fixed and random vectors
  ref_preview_camera.json  the preview camera (src/camera.cpp as OpenGLPreview drives
                    it) over scripted key / mouse / scroll sequences

Floats are stored as their IEEE-754 bit patterns (uint32) so tests compare bitwise.
Usage:  python tests/golden/make_ref_golden.py      (needs /root/reference)
"""
from __future__ import annotations

import ctypes as C
import json
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
HARNESS = ROOT / "oracle" / "_ref" / "libref_harness.so"
FP = C.POINTER(C.c_float)


def bits(a) -> list:
    return np.asarray(a, np.float32).view(np.uint32).ravel().tolist()


def texture_image(w, h, nc, salt):
    i = np.arange(w * h * nc, dtype=np.uint64)
    return ((i * 2654435761 + salt) >> np.uint64(7)).astype(np.uint8)


def main() -> int:
    if not Path("/root/reference").exists():
        print("reference not present; goldens are generated in the build container only")
        return 1
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "ref"], check=True)
    L = C.CDLL(str(HARNESS))
    L.ref_tex_lookup.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint8), C.c_float, C.c_float, FP]
    L.ref_camera.argtypes = [FP, FP, FP, C.c_float, C.c_uint, C.c_uint, FP]
    L.ref_normalize.argtypes = [FP, FP]
    L.ref_cross.argtypes = [FP, FP, FP]
    L.ref_dot.argtypes = [FP, FP]
    L.ref_dot.restype = C.c_float
    L.ref_distance.argtypes = [FP, FP]
    L.ref_distance.restype = C.c_float
    L.ref_material_normal.argtypes = [FP, FP]
    L.ref_light_surface.argtypes = [FP]
    L.ref_light_surface.restype = C.c_float

    def fp(a):
        a = np.ascontiguousarray(a, np.float32)
        return a, a.ctypes.data_as(FP)

    # ---- G5 texture
    coords = [-1.25, -1.0, -0.5, -0.0, 0.0, 0.25, 0.5, 0.999, 1.0, 1.75, 2.0, 3.5]
    tex = []
    for (w, h, nc, salt) in ((7, 5, 3, 11), (8, 4, 4, 29), (5, 6, 1, 3), (16, 16, 3, 101)):
        img = texture_image(w, h, nc, salt)
        pad = np.zeros((w + 1) * nc + 4, np.uint8)  # defined bytes past the end (oracle/kernel pad)
        buf = np.concatenate([img, pad])
        cases = []
        for u in coords:
            for v in coords:
                out = np.zeros(3, np.float32)
                L.ref_tex_lookup(w, h, nc, buf.ctypes.data_as(C.POINTER(C.c_uint8)), u, v, out.ctypes.data_as(FP))
                cases.append({"u": bits([u])[0], "v": bits([v])[0], "rgb": bits(out)})
        tex.append({"w": w, "h": h, "nc": nc, "salt": salt, "cases": cases})
    (ROOT / "tests" / "golden" / "ref_texture.json").write_text(json.dumps({"textures": tex}, indent=0))

    # ---- G6 camera + glm primitives
    cams = [((0.0, 1.0, 2.95), (0.0, 1.0, 0.0), (0.0, 1.0, 0.0), 1.0, 256, 256),
            ((0.0, 1.0, 2.95), (0.0, 1.0, 0.0), (0.0, 1.0, 0.0), 1.0, 768, 768),
            ((278.0, 273.0, -800.0), (278.0, 273.0, 0.0), (0.0, 1.0, 0.0), 0.7, 1024, 1024),
            ((10.0, 16.0, 10.0), (0.0, 8.5, 0.0), (0.0, 1.0, 0.0), 1.0, 1920, 1080),
            ((-1650.0, 260.0, 0.0), (600.0, 520.0, 0.0), (0.0, 1.0, 0.0), 1.0, 1920, 1080),
            ((-1650.0, 260.0, 0.0), (600.0, 520.0, 0.0), (0.0, 1.0, 0.0), 1.0, 3840, 2160),
            ((0.3, -2.0, 5.0), (1.0, 0.5, -3.0), (0.1, 0.9, 0.2), 1.7, 640, 360)]
    camera = []
    for eye, c, up, yv, xr, yr in cams:
        out = np.zeros(12, np.float32)
        e_, ep = fp(eye)
        c_, cp = fp(c)
        u_, upp = fp(up)
        L.ref_camera(ep, cp, upp, yv, xr, yr, out.ctypes.data_as(FP))
        camera.append({"eye": list(eye), "center": list(c), "up": list(up), "yview": yv, "xres": xr, "yres": yr,
                       "out": bits(out)})
    rng = np.random.default_rng(20240611)
    vecs = np.concatenate([rng.normal(size=(200, 3)) * rng.choice([1e-3, 1.0, 1e3], size=(200, 1)),
                           np.array([[0, 0, 1], [1e-20, 1e-20, 1e-20], [3, 4, 0], [-0.0, 2.0, -1.0]])]).astype(np.float32)
    prims = []
    for i in range(len(vecs) - 1):
        a, b = vecs[i], vecs[i + 1]
        a_, ap = fp(a)
        b_, bp = fp(b)
        n = np.zeros(3, np.float32)
        x = np.zeros(3, np.float32)
        L.ref_normalize(ap, n.ctypes.data_as(FP))
        L.ref_cross(ap, bp, x.ctypes.data_as(FP))
        prims.append({"a": bits(a), "b": bits(b), "normalize": bits(n), "cross": bits(x),
                      "dot": bits([L.ref_dot(ap, bp)])[0], "distance": bits([L.ref_distance(ap, bp)])[0]})
    tri = []
    for i in range(0, len(vecs) - 3, 3):
        p = vecs[i:i + 3].ravel()
        p_, pp = fp(p)
        mn = np.zeros(3, np.float32)
        L.ref_material_normal(pp, mn.ctypes.data_as(FP))
        tri.append({"p": bits(p), "material_normal": bits(mn), "surface": bits([L.ref_light_surface(pp)])[0]})
    (ROOT / "tests" / "golden" / "ref_glm.json").write_text(
        json.dumps({"camera": camera, "primitives": prims, "triangles": tri}, indent=0))
    # ---- preview camera (src/camera.cpp)
    L.ref_preview_camera.argtypes = [FP, FP, FP, C.c_float, C.POINTER(C.c_int), FP, C.c_int, FP]
    prng = np.random.default_rng(777)
    seqs = []
    for vp, la, up, yv in (((0.0, 1.0, 2.95), (0.0, 1.0, 0.0), (0.0, 1.0, 0.0), 1.0),
                           ((278.0, 273.0, -800.0), (278.0, 273.0, 0.0), (0.0, 1.0, 0.0), 0.7),
                           ((10.0, 16.0, 10.0), (0.0, 8.5, 0.0), (0.0, 1.0, 0.0), 1.0),
                           ((0.3, -2.0, 5.0), (1.0, 0.5, -3.0), (0.1, 0.9, 0.2), 1.7)):
        n = 120
        ops = prng.integers(0, 9, n).astype(np.int32)
        args = np.stack([prng.uniform(-40, 40, n), prng.uniform(-40, 40, n)], 1).astype(np.float32)
        args[ops <= 5, 0] = np.abs(args[ops <= 5, 0]) / 100.0          # frame times
        args[ops == 8, 0] = np.where(prng.random((ops == 8).sum()) < 0.5, 2.5, 30.0)  # shift speeds
        out = np.zeros((n, 15), np.float32)
        v_, vpp = fp(vp)
        l_, lp = fp(la)
        u_, upp = fp(up)
        L.ref_preview_camera(vpp, lp, upp, yv, ops.ctypes.data_as(C.POINTER(C.c_int)), args.ctypes.data_as(FP), n,
                             out.ctypes.data_as(FP))
        seqs.append({"vp": list(vp), "la": list(la), "up": list(up), "yview": yv, "ops": ops.tolist(),
                     "args": bits(args), "out": bits(out)})
    (ROOT / "tests" / "golden" / "ref_preview_camera.json").write_text(json.dumps({"sequences": seqs}, indent=0))
    print("wrote ref_texture.json, ref_glm.json, ref_preview_camera.json")
    return 0


if __name__ == "__main__":
    sys.exit(main())
