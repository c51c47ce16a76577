"""Census (CPU, diagnostic): how many of the shadow trace's triangle tests that survive the packed leaf
cull records a per-reference padded box would skip exactly (scripts/refbox_census.cpp); generation-1
shadow rays of a config as scripts/bvh_census.py makes them.

    python scripts/refbox_census.py [--config sponza] [--res 320x180] [--spp 2]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "chiaroscuro-raytracer_amd"), str(ROOT / "oracle"), str(ROOT / "scripts")]
os.environ.setdefault("CHIARO_QUIET", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sponza")
    ap.add_argument("--res", default="320x180")
    ap.add_argument("--spp", type=int, default=2)
    args = ap.parse_args()
    import chiaroscuro_amd as ca
    import pyoracle as po
    from chiaroscuro_amd import scenes

    d = Path(tempfile.mkdtemp())
    exe = d / "refbox_census"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    str(ROOT / "scripts/refbox_census.cpp")], check=True)
    sc = ca.Scene(scenes.config_rtc(args.config))
    i = sc.info
    m = ca.Model(sc)
    tris = m.triangles()
    osc = po.OracleScene(tris, leaf_size=i["leaf_size"], textures=m.textures(), build_threads=8)
    kd = osc.kd_export()
    pos = np.ascontiguousarray(tris["pos"], np.float32).reshape(-1, 9)
    with open(d / "scene.bin", "wb") as f:
        np.array([len(kd["is_leaf"]), len(kd["refs"]), len(pos)], np.uint32).tofile(f)
        for k in ("is_leaf", "axis"):
            np.ascontiguousarray(kd[k], np.uint32).tofile(f)
        np.ascontiguousarray(kd["split"], np.float32).tofile(f)
        for k in ("child", "leaf_first", "leaf_count", "refs"):
            np.ascontiguousarray(kd[k], np.uint32).tofile(f)
        pos.tofile(f)
        np.ascontiguousarray(kd["box"], np.float32).tofile(f)
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
    ids, _ = osc.lights()
    li = ids[rng.integers(0, len(ids), len(p))]
    v0 = rng.random((len(p), 1)).astype(np.float32)
    v1 = (rng.random((len(p), 1)) * (1 - v0)).astype(np.float32)
    LP = pos[li]
    lp = LP[:, 0:3] * v0 + LP[:, 3:6] * v1 + LP[:, 6:9] * (1 - v0 - v1)
    so = (p + 0.001 * n).astype(np.float32)
    sd = lp - p
    dist = np.linalg.norm(sd, axis=1).astype(np.float32)
    sd = (sd / dist[:, None]).astype(np.float32)
    rays = np.concatenate([so, sd, dist[:, None], np.asarray(li, np.uint32).view(np.float32)[:, None]], 1)
    with open(d / "rays.bin", "wb") as f:
        np.array([len(rays)], np.uint32).tofile(f)
        np.ascontiguousarray(rays, np.float32).tofile(f)
    out = json.loads(subprocess.run([str(exe), str(d / "scene.bin"), str(d / "rays.bin")], capture_output=True,
                                    text=True, check=True).stdout)
    q = max(out["queries"], 1)
    out["per_query"] = {k: round(out[k] / q, 2) for k in ("leaves", "inner", "tests_all", "tests_after_leaf_cull",
                                                           "boxable", "box_skipped")}
    out.update(config=args.config, res=args.res, spp=args.spp)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
