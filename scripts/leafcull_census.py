"""Per-leaf skip census on the CPU (scripts/leafcull_census.c): for generation-1
shadow rays, secondary closest rays and camera rays of a config, the share of
visited leaves (and of their triangle tests) whose tight triangle box the ray's
test segment [0, tmax_leaf] misses -- unpadded and padded by the exact
Moller-Trumbore rounding bound.  Diagnostic only.

    python scripts/leafcull_census.py [--config sponza] [--res 320x180]
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "chiaroscuro-raytracer_amd"), str(ROOT / "oracle")]
os.environ.setdefault("CHIARO_QUIET", "1")
NAMES = ("queries", "leaves", "tests", "leaf_empty", "cull0_leaves", "cull0_tests", "cullp_leaves", "cullp_tests",
         "occluded", "cone_leaves", "cone_tests", "cone_fail", "g1_tests", "g2_tests", "g3_tests", "g4_tests",
         "inner", "sub_roots", "sub_inner", "sub_leaves", "sub_tests", "subp_roots", "subp_inner", "subp_leaves",
         "subp_tests", "subg_roots", "subg_inner", "subg_leaves", "subg_tests")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sponza")
    ap.add_argument("--res", default="320x180")
    ap.add_argument("--spp", type=int, default=2)
    ap.add_argument("--subk", type=int, default=4, help="normal groups per subtree record (census)")
    ap.add_argument("--submode", type=int, default=1, help="1 every node, 2 pops only, 3 both children of splits")
    ap.add_argument("--spad", type=float, default=1e-4, help="subtree census pad, x scene extent")
    args = ap.parse_args()
    so = "/tmp/leafcull_census.so"
    subprocess.run(["gcc", "-O2", "-fopenmp", "-DSUBK=%d" % args.subk, "-DSUBMODE=%d" % args.submode, "-shared", "-fPIC", "-o", so, str(ROOT / "scripts/leafcull_census.c"),
                    "-lm"], check=True)
    L = C.CDLL(so)
    import chiaroscuro_amd as ca
    import pyoracle as po
    from chiaroscuro_amd import scenes

    sc = ca.Scene(scenes.config_rtc(args.config))
    i = sc.info
    m = ca.Model(sc)
    tris = m.triangles()
    osc = po.OracleScene(tris, leaf_size=i["leaf_size"], textures=m.textures(), build_threads=8)
    kd = osc.kd_export()
    pos = np.ascontiguousarray(tris["pos"], np.float32).reshape(-1, 9)
    xres, yres = (int(v) for v in args.res.split("x"))
    cam = po.camera(i["VP"], i["LA"], i["UP"], i["yview"], xres, yres)
    rng = np.random.default_rng(1)
    ys, xs = np.mgrid[0:yres, 0:xres]
    xs = np.repeat(xs.ravel(), args.spp) + rng.random(xres * yres * args.spp)
    ys = np.repeat(ys.ravel(), args.spp) + rng.random(xres * yres * args.spp)
    eye, lu, dx, dy = cam[0:3], cam[3:6], cam[6:9], cam[9:12]
    dirs = (lu[None] + xs[:, None] * dx[None] + ys[:, None] * dy[None]).astype(np.float32)
    orig = np.repeat(eye[None], len(dirs), 0).astype(np.float32)
    h = osc.intersect(orig, dirs)
    hit = h["hit"] != 0
    t = h["tri"][hit]
    bx, by = h["bary"][hit, 0:1], h["bary"][hit, 1:2]
    P = pos[t]
    A, B, Cc = P[:, 0:3], P[:, 3:6], P[:, 6:9]
    p = A * (1 - bx - by) + B * bx + Cc * by
    n = np.cross(B - A, Cc - A)
    n /= np.linalg.norm(n, axis=1, keepdims=True) + 1e-30
    n *= np.sign(np.sum(n * (orig[hit] - p), axis=1, keepdims=True))  # toward the camera
    ids, surf = osc.lights()
    li = ids[rng.integers(0, len(ids), len(p))]
    v0 = rng.random((len(p), 1)).astype(np.float32)
    v1 = (rng.random((len(p), 1)) * (1 - v0)).astype(np.float32)
    LP = pos[li]
    lp = LP[:, 0:3] * v0 + LP[:, 3:6] * v1 + LP[:, 6:9] * (1 - v0 - v1)
    so_ = (p + 0.001 * n).astype(np.float32)
    sd = lp - p
    dist = np.linalg.norm(sd, axis=1).astype(np.float32)
    sd = (sd / dist[:, None]).astype(np.float32)
    # secondary closest rays: cosine-ish hemisphere directions about the normal
    r = rng.normal(size=(len(p), 3))
    r /= np.linalg.norm(r, axis=1, keepdims=True)
    r = r + n
    r = (r / np.linalg.norm(r, axis=1, keepdims=True)).astype(np.float32)
    out = {"config": args.config, "res": args.res, "spp": args.spp, "camera_rays": len(dirs), "hits": int(hit.sum())}

    def run(o, d, dist, excl, shadow):
        st = np.zeros(len(NAMES), np.uint64)
        u32 = lambda a: np.ascontiguousarray(a, np.uint32).ctypes.data_as(C.c_void_p)
        f32 = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data_as(C.c_void_p)
        keep = [np.ascontiguousarray(x) for x in (o, d, dist, excl)]
        L.census(C.c_uint32(len(kd["is_leaf"])), u32(kd["is_leaf"]), u32(kd["axis"]), f32(kd["split"]),
                 u32(kd["child"]), u32(kd["leaf_first"]), u32(kd["leaf_count"]), u32(kd["refs"]), f32(kd["box"]),
                 f32(pos), C.c_uint32(len(o)), f32(keep[0]), f32(keep[1]), f32(keep[2]), u32(keep[3]),
                 C.c_int(int(shadow)), st.ctypes.data_as(C.c_void_p), C.c_double(args.spad))
        s = dict(zip(NAMES, (int(x) for x in st)))
        s["cull0_test_frac"] = round(s["cull0_tests"] / max(s["tests"], 1), 4)
        s["cullp_test_frac"] = round(s["cullp_tests"] / max(s["tests"], 1), 4)
        s["cullp_leaf_frac"] = round(s["cullp_leaves"] / max(s["leaves"], 1), 4)
        s["cone_test_frac"] = round(s["cone_tests"] / max(s["tests"], 1), 4)
        s["cone_leaf_frac"] = round(s["cone_leaves"] / max(s["leaves"], 1), 4)
        for k in (1, 2, 3, 4):
            s["g%d_test_frac" % k] = round(s["g%d_tests" % k] / max(s["tests"], 1), 4)
        s["tests_per_query"] = round(s["tests"] / max(s["queries"], 1), 1)
        for k in ("sub", "subp", "subg"):
            s[k + "_inner_frac"] = round(s[k + "_inner"] / max(s["inner"], 1), 4)
            s[k + "_leaf_frac"] = round(s[k + "_leaves"] / max(s["leaves"], 1), 4)
        s["inner_per_query"] = round(s["inner"] / max(s["queries"], 1), 1)
        return s

    out["shadow"] = run(so_, sd, dist, li, True)
    print("shadow", out["shadow"], file=sys.stderr)
    out["closest"] = run(so_, r, np.zeros(len(r), np.float32), np.zeros(len(r), np.uint32), False)
    print("closest", out["closest"], file=sys.stderr)
    out["camera"] = run(orig, dirs, np.zeros(len(dirs), np.float32), np.zeros(len(dirs), np.uint32), False)
    print("camera", out["camera"], file=sys.stderr)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
