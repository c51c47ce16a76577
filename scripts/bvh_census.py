"""Census (diagnostic only, scripts/bvh_census.c): generation-1 shadow queries of a config answered
by the reference's kd traversal and by an any-hit walk of a binned-SAH BVH over the same triangles
(a BVH walk that finds no triangle passing Moller-Trumbore with t < D proves VISIBLE exactly; one
that finds one leaves the answer to the kd traversal).  Rays as scripts/leafcull_census.py makes them.

    python scripts/bvh_census.py [--config sponza] [--res 320x180] [--leaf 4]
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
NAMES = ("queries", "kd_occ", "kd_inner", "kd_leaves", "kd_tests", "bvh_found", "bvh_nodes", "bvh_tests",
         "bvh_vis_nodes", "bvh_vis_tests", "kd_vis_inner", "kd_vis_leaves", "kd_vis_tests", "mismatch_found",
         "mismatch_occ", "bvh_occ_nodes", "bvh_occ_tests", "kd_occ_inner", "kd_occ_leaves", "kd_occ_tests",
         "bvh_leaves", "pr_found", "pr_nodes", "pr_tests", "pr_vis_nodes", "pr_vis_tests", "pr_miss")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sponza")
    ap.add_argument("--res", default="320x180")
    ap.add_argument("--spp", type=int, default=2)
    ap.add_argument("--leaf", type=int, default=4)
    ap.add_argument("--c1", type=float, default=0.05, help="proof walk: regime-i cosine threshold")
    args = ap.parse_args()
    so = "/tmp/bvh_census_%d_%g.so" % (args.leaf, args.c1)
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-DLEAF=%d" % args.leaf, "-DC1=%r" % args.c1, "-shared", "-fPIC", "-o",
                    so, str(ROOT / "scripts/bvh_census.c"), "-lm"], check=True)
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
    n *= np.sign(np.sum(n * (orig[hit] - p), axis=1, keepdims=True))
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
    st = np.zeros(len(NAMES), np.uint64)
    nodes = C.c_uint32(0)
    keep = [np.ascontiguousarray(x) for x in (so_, sd, dist, np.asarray(li, np.uint32))]
    u32 = lambda a: np.ascontiguousarray(a, np.uint32).ctypes.data_as(C.c_void_p)
    f32 = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data_as(C.c_void_p)
    L.census(C.c_uint32(len(kd["is_leaf"])), u32(kd["is_leaf"]), u32(kd["axis"]), f32(kd["split"]),
             u32(kd["child"]), u32(kd["leaf_first"]), u32(kd["leaf_count"]), u32(kd["refs"]), f32(kd["box"]),
             f32(pos), C.c_uint32(len(pos)), C.c_uint32(len(keep[0])), f32(keep[0]), f32(keep[1]), f32(keep[2]),
             u32(keep[3]), st.ctypes.data_as(C.c_void_p), C.byref(nodes))
    s = dict(zip(NAMES, (int(x) for x in st)))
    q = max(s["queries"], 1)
    occ = max(s["kd_occ"], 1)
    vis = max(s["queries"] - s["kd_occ"], 1)
    s["per_query"] = {k: round(s[k] / q, 2) for k in ("kd_inner", "kd_leaves", "kd_tests", "bvh_nodes", "bvh_tests",
                                                       "bvh_leaves", "pr_nodes", "pr_tests")}
    s["pr_found_frac"] = round(s["pr_found"] / q, 4)
    s["per_visible"] = {k: round(s[k] / vis, 2) for k in ("kd_vis_inner", "kd_vis_leaves", "kd_vis_tests",
                                                           "bvh_vis_nodes", "bvh_vis_tests", "pr_vis_nodes",
                                                           "pr_vis_tests")}
    s["per_occluded"] = {k: round(s[k] / occ, 2) for k in ("kd_occ_inner", "kd_occ_leaves", "kd_occ_tests",
                                                            "bvh_occ_nodes", "bvh_occ_tests")}
    s["occluded_frac"] = round(s["kd_occ"] / q, 4)
    s["bvh_node_count"] = nodes.value
    s["config"], s["res"], s["spp"], s["leaf"] = args.config, args.res, args.spp, args.leaf
    print(json.dumps(s))


if __name__ == "__main__":
    main()
