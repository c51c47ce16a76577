"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this, as the checker / the timed CPU baseline.  The product never does.
See oracle.h for what is restated and what is pinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
# CHIARO_ORACLE_DIR: load the libraries from there instead (the sanitizer build, oracle/_san)
_LIBDIR = Path(os.environ["CHIARO_ORACLE_DIR"]) if os.environ.get("CHIARO_ORACLE_DIR") else HERE
LIB = _LIBDIR / "liboracle.so"
# the same oracle.c at -O3 without the hot-path work counters (OR_LEAN): bench.py's timed
# cpu_baseline leg only; its query / path counts equal liboracle.so's and its pixels are the same bits
LEAN_LIB = _LIBDIR / "liboracle_lean.so"
REF_LIB = HERE / "_ref" / "libref_harness.so"

FP = C.POINTER(C.c_float)
UP = C.POINTER(C.c_uint32)
IP = C.POINTER(C.c_int32)
P = C.c_void_p
N_COUNTERS = 8
COUNTER_NAMES = ("closest", "shadow", "inner", "leaf", "tritest", "hit", "texhit", "paths")

_lib = None
_lean = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        sig = {
            "or_scene_create": (P, [C.c_uint32, FP, FP, FP, FP, FP, IP, C.c_uint32, C.c_int]),
            "or_scene_add_texture": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint8)]),
            "or_scene_destroy": (None, [P]),
            "or_kd_num_nodes": (C.c_uint32, [P]),
            "or_kd_num_refs": (C.c_uint32, [P]),
            "or_kd_max_depth": (C.c_uint32, [P]),
            "or_kd_export": (None, [P, UP, UP, FP, UP, UP, UP, UP, FP]),
            "or_num_lights": (C.c_uint32, [P]),
            "or_lights": (None, [P, UP, FP]),
            "or_camera": (None, [FP, FP, FP, C.c_float, C.c_uint32, C.c_uint32, FP]),
            "or_intersect": (None, [P, C.c_uint32, FP, FP, UP, UP, FP, FP]),
            "or_intersect_shadow": (None, [P, C.c_uint32, FP, FP, FP, UP, UP]),
            "or_sample_wi": (None, [FP, C.c_float, C.c_float, FP, FP]),
            "or_concentric": (None, [C.c_float, C.c_float, FP, FP]),
            "or_sincos": (None, [C.c_float, FP, FP]),
            "or_tex_lookup": (None, [P, C.c_int, C.c_float, C.c_float, FP]),
            "or_rng_draws": (None, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, UP]),
            "or_path": (None, [P, FP, C.c_uint32, C.c_uint32, C.c_int, FP, C.c_uint32, C.c_uint32, C.c_uint32,
                               C.c_uint32, C.c_uint32, FP]),
            "or_render": (None, [P, FP, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, FP, C.c_uint32, C.c_uint32,
                                 C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, FP, C.POINTER(C.c_uint64)]),
            "or_render_pixels": (None, [P, FP, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, FP, C.c_uint32,
                                        C.c_uint32, C.c_uint32, UP, UP, C.c_int, FP, C.POINTER(C.c_uint64)]),
            "or_set_trig_mode": (None, [C.c_int]),
            "or_sincos_check": (C.c_uint64, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_int]),
            "or_glm_normalize": (None, [FP, FP]),
            "or_glm_cross": (None, [FP, FP, FP]),
            "or_glm_dot": (C.c_float, [FP, FP]),
            "or_glm_distance": (C.c_float, [FP, FP]),
            "or_material_normal": (None, [FP, FP]),
            "or_light_surface": (C.c_float, [FP]),
            "or_tonemap": (None, [FP, C.c_uint32, C.c_uint32, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float,
                                  C.POINTER(C.c_uint8)]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _lib = L
    return _lib


def lean_lib():
    """liboracle_lean.so's or_render (scenes are shared with liboracle.so: same source, same layout)."""
    global _lean
    if _lean is None:
        if not LEAN_LIB.exists():
            build()
        L = C.CDLL(str(LEAN_LIB))
        L.or_render.restype = None
        L.or_render.argtypes = [P, FP, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, FP, C.c_uint32, C.c_uint32,
                                C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, FP, C.POINTER(C.c_uint64)]
        _lean = L
    return _lean


def _f(a):
    return np.ascontiguousarray(a, np.float32)


def _p(a, t=C.c_float):
    return a.ctypes.data_as(C.POINTER(t))


class OracleScene:
    """Oracle scene over a triangle soup in KDTree order (Model.triangles() layout)."""

    def __init__(self, tris: dict, leaf_size: int = 8, textures=(), build_threads: int = 1):
        L = lib()
        self._keep = {k: np.ascontiguousarray(v) for k, v in tris.items()}
        n = len(self._keep["pos"])
        t = self._keep
        self.h = L.or_scene_create(n, _p(_f(t["pos"])), _p(_f(t["vnrm"])), _p(_f(t["uv"])), _p(_f(t["kd"])),
                                   _p(_f(t["ke"])), _p(np.ascontiguousarray(t["tex"], np.int32), C.c_int32),
                                   int(leaf_size), int(build_threads))
        self._tex = []
        for (w, h, nc, data) in textures:
            data = np.ascontiguousarray(data, np.uint8)
            self._tex.append(data)
            L.or_scene_add_texture(self.h, w, h, nc, _p(data, C.c_uint8))
        tex = np.asarray(t["tex"])
        if len(tex) and int(tex.max()) >= len(self._tex):
            raise ValueError("triangle texture index %d but %d textures given" % (int(tex.max()), len(self._tex)))

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.or_scene_destroy(self.h)
            self.h = None

    def kd_export(self) -> dict:
        L = lib()
        n, r = L.or_kd_num_nodes(self.h), L.or_kd_num_refs(self.h)
        o = {k: np.zeros(n, np.uint32) for k in ("is_leaf", "axis", "child", "leaf_first", "leaf_count")}
        o["split"] = np.zeros(n, np.float32)
        o["refs"] = np.zeros(max(r, 1), np.uint32)
        o["box"] = np.zeros(6, np.float32)
        L.or_kd_export(self.h, _p(o["is_leaf"], C.c_uint32), _p(o["axis"], C.c_uint32), _p(o["split"]),
                       _p(o["child"], C.c_uint32), _p(o["leaf_first"], C.c_uint32), _p(o["leaf_count"], C.c_uint32),
                       _p(o["refs"], C.c_uint32), _p(o["box"]))
        o["refs"] = o["refs"][:r]
        o["max_depth"] = L.or_kd_max_depth(self.h)
        return o

    def lights(self):
        L = lib()
        n = L.or_num_lights(self.h)
        ids, surf = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.float32)
        L.or_lights(self.h, _p(ids, C.c_uint32), _p(surf))
        return ids[:n], surf[:n]

    def intersect(self, orig, dirs):
        orig, dirs = _f(orig).reshape(-1, 3), _f(dirs).reshape(-1, 3)
        n = len(orig)
        hit, tri = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        bary, dist = np.zeros((n, 2), np.float32), np.zeros(n, np.float32)
        lib().or_intersect(self.h, n, _p(orig), _p(dirs), _p(hit, C.c_uint32), _p(tri, C.c_uint32), _p(bary),
                           _p(dist))
        return {"hit": hit, "tri": tri, "bary": bary, "dist": dist}

    def intersect_shadow(self, orig, dirs, dist, light):
        orig, dirs = _f(orig).reshape(-1, 3), _f(dirs).reshape(-1, 3)
        dist, light = _f(dist), np.ascontiguousarray(light, np.uint32)
        occ = np.zeros(len(orig), np.uint32)
        lib().or_intersect_shadow(self.h, len(orig), _p(orig), _p(dirs), _p(dist), _p(light, C.c_uint32),
                                  _p(occ, C.c_uint32))
        return occ

    def tex_lookup(self, tex, u, v):
        out = np.zeros(3, np.float32)
        lib().or_tex_lookup(self.h, int(tex), float(u), float(v), _p(out))
        return out

    def path(self, cam, xres, yres, k, bg, seed, layer, x, y, sample):
        out = np.zeros(3, np.float32)
        lib().or_path(self.h, _p(_f(cam)), xres, yres, k, _p(_f(bg)), seed, layer, x, y, sample, _p(out))
        return out

    def render(self, cam, xres, yres, spp, k, seed, layer=1, bg=(0, 0, 0), pixels=None, y0=0, y1=None, ystep=1,
               threads=0, lean=False):
        """lean: the -O3 counter-free build (liboracle_lean.so): only closest / shadow / paths are counted."""
        pix = pixels if pixels is not None else np.zeros((yres, xres, 3), np.float32)
        ctr = np.zeros(N_COUNTERS, np.uint64)
        (lean_lib() if lean else lib()).or_render(self.h, _p(_f(cam)), xres, yres, spp, k, _p(_f(bg)), seed & 0xFFFFFFFF, layer, y0,
                        yres if y1 is None else y1, ystep, threads, _p(pix), ctr.ctypes.data_as(C.POINTER(C.c_uint64)))
        return pix, dict(zip(COUNTER_NAMES, (int(x) for x in ctr)))


    def render_pixels(self, cam, xres, yres, spp, k, seed, px, py, layer=1, bg=(0, 0, 0), threads=0):
        """Batch means [n][3] of the listed pixels (no blend) and the summed counters."""
        px, py = np.ascontiguousarray(px, np.uint32), np.ascontiguousarray(py, np.uint32)
        mean = np.zeros((len(px), 3), np.float32)
        ctr = np.zeros(N_COUNTERS, np.uint64)
        lib().or_render_pixels(self.h, _p(_f(cam)), xres, yres, spp, k, _p(_f(bg)), seed & 0xFFFFFFFF, layer,
                               len(px), _p(px, C.c_uint32), _p(py, C.c_uint32), threads, _p(mean),
                               ctr.ctypes.data_as(C.POINTER(C.c_uint64)))
        return mean, dict(zip(COUNTER_NAMES, (int(x) for x in ctr)))


def camera(eye, center, up, yview, xres, yres) -> np.ndarray:
    out = np.zeros(12, np.float32)
    lib().or_camera(_p(_f(eye)), _p(_f(center)), _p(_f(up)), float(yview), xres, yres, _p(out))
    return out


def sample_wi(n, sx, sy):
    wi, pdf = np.zeros(3, np.float32), np.zeros(1, np.float32)
    lib().or_sample_wi(_p(_f(n)), float(sx), float(sy), _p(wi), _p(pdf))
    return wi, float(pdf[0])


def concentric(sx, sy):
    dx, dy = np.zeros(1, np.float32), np.zeros(1, np.float32)
    lib().or_concentric(float(sx), float(sy), _p(dx), _p(dy))
    return float(dx[0]), float(dy[0])


def sincos(x):
    s, c = np.zeros(1, np.float32), np.zeros(1, np.float32)
    lib().or_sincos(float(x), _p(s), _p(c))
    return s[0], c[0]


def rng_draws(seed, layer, pixel, sample, n):
    out = np.zeros(n, np.uint32)
    lib().or_rng_draws(seed, layer, pixel, sample, n, _p(out, C.c_uint32))
    return out


def tonemap(rgb, exposure, defog=0.0, knee_low=0.0, knee_high=5.0, gamma=2.2):
    """rayTracer.cpp:196-222 on a [yres][xres][3] fp32 frame -> uint8 (rows flipped)."""
    rgb = np.ascontiguousarray(rgb, np.float32)
    out = np.zeros(rgb.shape, np.uint8)
    lib().or_tonemap(_p(rgb), rgb.shape[1], rgb.shape[0], exposure, defog, knee_low, knee_high, gamma,
                     out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out


def sincos_check(lo: int, hi: int, stride: int = 1, both_signs: bool = True, threads: int = 0) -> int:
    """Mismatches of the glibc sinf / cosf restatement vs the host libm over float
    bit patterns lo..hi step stride (and their negatives)."""
    return int(lib().or_sincos_check(lo, hi, stride, int(both_signs), threads))


def set_trig_mode(mode: int):
    lib().or_set_trig_mode(int(mode))
