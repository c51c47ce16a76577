"""Census (diagnostic only, scripts/packet_census.c): generation-1 shadow queries of a screen window of
the config's frame at its full sample density, sorted as the wavefront queue is (origin leaf, then a
Morton-ordered 128 x 128 octahedral direction bin), traced one ray per lane vs one packet per 64
consecutive queries (per-lane intervals, majority near-first order).  Rays as scripts/bvh_census.py.

    python scripts/packet_census.py [--config sponza] [--frame 1920x1080] [--window 64x36] [--spp 128]
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
NAMES = ("queries", "occluded", "lane_inner", "lane_leaves", "lane_tests", "pk_inner", "pk_inner_lanes", "pk_leaves",
         "pk_leaf_lanes", "pk_tests", "pk_test_lanes", "pk_mismatch", "packets", "pk_lane_inner")


def morton2(x, y):
    def spread(v):
        v = v.astype(np.uint32)
        v = (v | (v << 8)) & 0x00FF00FF
        v = (v | (v << 4)) & 0x0F0F0F0F
        v = (v | (v << 2)) & 0x33333333
        v = (v | (v << 1)) & 0x55555555
        return v
    return spread(x) | (spread(y) << 1)


def oct_bin(d, n=128):
    a = np.abs(d).sum(1, keepdims=True)
    p = d / a
    x, y, z = p[:, 0], p[:, 1], p[:, 2]
    ox = np.where(z >= 0, x, (1 - np.abs(y)) * np.sign(x))
    oy = np.where(z >= 0, y, (1 - np.abs(x)) * np.sign(y))
    bx = np.clip(((ox + 1) * 0.5 * n).astype(np.int64), 0, n - 1)
    by = np.clip(((oy + 1) * 0.5 * n).astype(np.int64), 0, n - 1)
    return morton2(bx, by)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sponza")
    ap.add_argument("--frame", default="1920x1080")
    ap.add_argument("--window", default="64x36")
    ap.add_argument("--at", default="0.5,0.5", help="window centre as frame fractions")
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--unsorted", action="store_true")
    args = ap.parse_args()
    so = "/tmp/packet_census.so"
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-shared", "-fPIC", "-o", so,
                    str(ROOT / "scripts/packet_census.c"), "-lm"], check=True)
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
    xres, yres = (int(v) for v in args.frame.split("x"))
    ww, wh = (int(v) for v in args.window.split("x"))
    fx, fy = (float(v) for v in args.at.split(","))
    x0, y0 = int(fx * xres - ww / 2), int(fy * yres - wh / 2)
    cam = po.camera(i["VP"], i["LA"], i["UP"], i["yview"], xres, yres)
    rng = np.random.default_rng(1)
    ys, xs = np.mgrid[y0:y0 + wh, x0:x0 + ww]
    n = ww * wh * args.spp
    xs = np.repeat(xs.ravel(), args.spp) + rng.random(n)
    ys = np.repeat(ys.ravel(), args.spp) + rng.random(n)
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
    nrm = np.cross(B - A, Cc - A)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True) + 1e-30
    nrm *= np.sign(np.sum(nrm * (orig[hit] - p), axis=1, keepdims=True))
    ids, surf = osc.lights()
    li = ids[rng.integers(0, len(ids), len(p))]
    v0 = rng.random((len(p), 1)).astype(np.float32)
    v1 = (rng.random((len(p), 1)) * (1 - v0)).astype(np.float32)
    LP = pos[li]
    lp = LP[:, 0:3] * v0 + LP[:, 3:6] * v1 + LP[:, 6:9] * (1 - v0 - v1)
    so_ = (p + 0.001 * nrm).astype(np.float32)
    sd = lp - p
    dist = np.linalg.norm(sd, axis=1).astype(np.float32)
    sd = (sd / dist[:, None]).astype(np.float32)
    # the NEE skip: a light facing away or a surface facing away (zero contribution) is not traced
    lnrm = np.cross(LP[:, 3:6] - LP[:, 0:3], LP[:, 6:9] - LP[:, 0:3])
    keep = (np.sum(nrm * sd, 1) > 0) & (np.abs(np.sum(lnrm * sd, 1)) > 0)
    so_, sd, dist, li = so_[keep], sd[keep], dist[keep], np.asarray(li[keep], np.uint32)
    u32 = lambda a: np.ascontiguousarray(a, np.uint32).ctypes.data_as(C.c_void_p)
    f32 = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data_as(C.c_void_p)
    leaf = np.zeros(len(so_), np.uint32)
    so_c = np.ascontiguousarray(so_)
    L.locate(u32(kd["is_leaf"]), u32(kd["axis"]), f32(kd["split"]), u32(kd["child"]), C.c_uint32(len(so_c)),
             f32(so_c), leaf.ctypes.data_as(C.c_void_p))
    if not args.unsorted:
        key = leaf.astype(np.uint64) * 16384 + oct_bin(sd).astype(np.uint64)
        order = np.argsort(key, kind="stable")
        so_, sd, dist, li = so_[order], sd[order], dist[order], li[order]
    arrs = [np.ascontiguousarray(x) for x in (so_, sd, dist, li)]
    st = np.zeros(len(NAMES), np.uint64)
    L.census(u32(kd["is_leaf"]), u32(kd["axis"]), f32(kd["split"]), u32(kd["child"]), u32(kd["leaf_first"]),
             u32(kd["leaf_count"]), u32(kd["refs"]), f32(kd["box"]), f32(pos), C.c_uint32(len(arrs[0])),
             f32(arrs[0]), f32(arrs[1]), f32(arrs[2]), u32(arrs[3]), C.c_int(args.width),
             st.ctypes.data_as(C.c_void_p))
    s = dict(zip(NAMES, (int(x) for x in st)))
    q = max(s["queries"], 1)
    s["per_query"] = {k: round(s[k] / q, 2) for k in ("lane_inner", "lane_leaves", "lane_tests", "pk_lane_inner")}
    pk = max(s["packets"], 1)
    s["per_packet"] = {k: round(s[k] / pk, 1) for k in ("pk_inner", "pk_leaves", "pk_tests")}
    s["packet_inner_lane_eff"] = round(s["pk_inner_lanes"] / max(64 * s["pk_inner"], 1), 3)
    s["lane_steps_over_packet_steps"] = round(s["lane_inner"] / max(s["pk_inner"], 1), 2)
    s["occluded_frac"] = round(s["occluded"] / q, 4)
    s["config"], s["frame"], s["window"], s["spp"], s["sorted"] = args.config, args.frame, args.window, args.spp, \
        not args.unsorted
    print(json.dumps(s))


if __name__ == "__main__":
    main()
