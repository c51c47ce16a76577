"""Census (diagnostic only, scripts/rope_census.c): an exact rope traversal of the reference's kd tree
against the recursion (src/kdtree.cpp:248-281, 322-344), on generation-1 shadow rays and generation-2
closest rays of a frame (rays made as scripts/packet_census.py makes them: camera hits, the 0.001
normal offset, a light point, a cosine-hemisphere bounce).  Per query: the same (leaf, interval-end bits)
sequence and answer, and the work of both (recursion inner steps; rope point-location steps, exit-face
divisions, descents after a rope, restarts, fallbacks).

    python scripts/rope_census.py [--config sponza] [--frame 320x180] [--spp 2] [--hint]
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
NAMES = ("queries", "answer_true", "rec_inner", "rec_leaves", "rec_tests", "rope_queries", "fallback_zero_dir",
         "fallback_on_split", "fallback_t0", "locate_steps", "rope_leaves", "exit_divs", "exit_divs_nocache",
         "rope_desc", "restarts", "restart_steps", "mismatch_seq", "mismatch_ans", "rec_inner_roped",
         "rec_leaves_roped", "vis_queries", "vis_rec_inner", "vis_rope_divs", "from_hit_leaf", "rec_fetch",
         "rope_fetch", "rope_rec", "vis_rec_fetch", "vis_rope_fetch", "vis_rope_divs_unused", "rec_fetch_roped")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sponza")
    ap.add_argument("--frame", default="320x180")
    ap.add_argument("--spp", type=int, default=2)
    ap.add_argument("--kind", default="shadow", choices=("shadow", "closest"))
    ap.add_argument("--hint", action="store_true", help="start from the leaf holding the hit (else locate)")
    args = ap.parse_args()
    so = "/tmp/rope_census.so"
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-shared", "-fPIC", "-o", so,
                    str(ROOT / "scripts/rope_census.c"), "-lm"], check=True)
    L = C.CDLL(so)
    u32 = lambda a: np.ascontiguousarray(a, np.uint32).ctypes.data_as(C.c_void_p)
    f32 = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data_as(C.c_void_p)
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
    cam = po.camera(i["VP"], i["LA"], i["UP"], i["yview"], xres, yres)
    rng = np.random.default_rng(1)
    ys, xs = np.mgrid[0:yres, 0:xres]
    n = xres * yres * args.spp
    xs = np.repeat(xs.ravel(), args.spp) + rng.random(n)
    ys = np.repeat(ys.ravel(), args.spp) + rng.random(n)
    eye, lu, dx, dy = cam[0:3], cam[3:6], cam[6:9], cam[9:12]
    dirs = (lu[None] + xs[:, None] * dx[None] + ys[:, None] * dy[None]).astype(np.float32)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    orig = np.repeat(eye[None], len(dirs), 0).astype(np.float32)
    h = osc.intersect(orig, dirs)
    hit = h["hit"] != 0
    t = h["tri"][hit]
    bx, by = h["bary"][hit, 0:1], h["bary"][hit, 1:2]
    P = pos[t]
    A, B, Cc = P[:, 0:3], P[:, 3:6], P[:, 6:9]
    p = (A * (1 - bx - by) + B * bx + Cc * by).astype(np.float32)
    nrm = np.cross(B - A, Cc - A)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True) + 1e-30
    nrm *= np.sign(np.sum(nrm * (orig[hit] - p), axis=1, keepdims=True))
    so_ = (p + np.float32(0.001) * nrm.astype(np.float32)).astype(np.float32)
    if args.kind == "shadow":
        ids, surf = osc.lights()
        li = ids[rng.integers(0, len(ids), len(p))]
        v0 = rng.random((len(p), 1)).astype(np.float32)
        v1 = (rng.random((len(p), 1)) * (1 - v0)).astype(np.float32)
        LP = pos[li]
        lp = LP[:, 0:3] * v0 + LP[:, 3:6] * v1 + LP[:, 6:9] * (1 - v0 - v1)
        sd = lp - p
        dist = np.linalg.norm(sd, axis=1).astype(np.float32)
        sd = (sd / dist[:, None]).astype(np.float32)
        lnrm = np.cross(LP[:, 3:6] - LP[:, 0:3], LP[:, 6:9] - LP[:, 0:3])
        keep = (np.sum(nrm * sd, 1) > 0) & (np.abs(np.sum(lnrm * sd, 1)) > 0)  # the NEE skip
        excl = np.asarray(li, np.uint32)
    else:  # a cosine-weighted bounce about the normal
        u1, u2 = rng.random(len(p)), rng.random(len(p))
        r, ph = np.sqrt(u1), 2 * np.pi * u2
        tz = np.where(np.abs(nrm[:, 0:1]) < 0.9, np.array([[1.0, 0, 0]]), np.array([[0, 1.0, 0]]))
        tx = np.cross(nrm, tz)
        tx /= np.linalg.norm(tx, axis=1, keepdims=True)
        ty = np.cross(nrm, tx)
        sd = (tx * (r * np.cos(ph))[:, None] + ty * (r * np.sin(ph))[:, None] +
              nrm * np.sqrt(1 - u1)[:, None]).astype(np.float32)
        sd /= np.linalg.norm(sd, axis=1, keepdims=True)
        dist = np.full(len(p), np.inf, np.float32)
        keep = np.ones(len(p), bool)
        excl = np.zeros(len(p), np.uint32)
    so_, sd, dist, excl, ph = (np.ascontiguousarray(a[keep]) for a in (so_, sd.astype(np.float32), dist, excl, p))
    start = None
    if args.hint:  # the leaf of the hit point: the rope walk starts there when it holds the ray's origin
        start = np.zeros(len(ph), np.uint32)
        L.locate(u32(kd["is_leaf"]), u32(kd["axis"]), f32(kd["split"]), u32(kd["child"]), C.c_uint32(len(ph)),
                 f32(ph), start.ctypes.data_as(C.c_void_p))
    st = np.zeros(len(NAMES), np.uint64)
    L.census(u32(kd["is_leaf"]), u32(kd["axis"]), f32(kd["split"]), u32(kd["child"]), u32(kd["leaf_first"]),
             u32(kd["leaf_count"]), u32(kd["refs"]), f32(kd["box"]), f32(pos), C.c_uint32(len(kd["is_leaf"])),
             C.c_uint32(len(so_)), f32(so_), f32(sd), f32(dist), u32(excl), None if start is None else u32(start), C.c_int(args.kind == "shadow"),
             st.ctypes.data_as(C.c_void_p))
    s = dict(zip(NAMES, (int(x) for x in st)))
    rq = max(s["rope_queries"], 1)
    s["per_roped_query"] = {
        "rec_inner": round(s["rec_inner_roped"] / rq, 2), "rec_leaves": round(s["rec_leaves_roped"] / rq, 2),
        "rope_leaves": round(s["rope_leaves"] / rq, 2), "locate_steps": round(s["locate_steps"] / rq, 2),
        "exit_divs": round(s["exit_divs"] / rq, 2), "exit_divs_nocache": round(s["exit_divs_nocache"] / rq, 2),
        "rope_desc": round(s["rope_desc"] / rq, 2), "restart_steps": round(s["restart_steps"] / rq, 2)}
    vq = max(s["vis_queries"], 1)
    s["per_roped_query"].update({"rec_fetch": round(s["rec_fetch_roped"] / rq, 2),
                                 "rope_node_fetch": round(s["rope_fetch"] / rq, 2),
                                 "rope_records": round(s["rope_rec"] / rq, 2)})
    s["per_visible_query"] = {"rec_inner_divs": round(s["vis_rec_inner"] / vq, 1),
                              "rope_divs": round(s["vis_rope_divs"] / vq, 1),
                              "rec_fetch": round(s["vis_rec_fetch"] / vq, 1),
                              "rope_fetch_incl_records": round(s["vis_rope_fetch"] / vq, 1)}
    s["fallback_frac"] = round(1 - s["rope_queries"] / max(s["queries"], 1), 4)
    s["config"], s["frame"], s["spp"], s["kind"], s["hint"] = args.config, args.frame, args.spp, args.kind, args.hint
    print(json.dumps(s))


if __name__ == "__main__":
    main()
