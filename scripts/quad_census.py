"""Census (CPU): the descent's vector-memory fetch instructions per query with the fat node records
(dwordx4 + dwordx2 per two levels) against the two-level quad records (one dwordx4; csrc/quadnodes.hpp),
on a config's own kd tree and generation-1 shadow and secondary rays, by tests/native/quad_check.cpp's
model of both traversals -- which also checks that every ray visits the same leaves with the same
intervals as the recursion (kdtree.cpp:248-281 / 322-344).  Rays as scripts/bvh_census.py makes them;
a query's segment ends at its first hit (shadow rays: the first occluder, if any), which is where the
kernels' queries end.

    python scripts/quad_census.py [--config sponza] [--res 320x180] [--spp 2]
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
sys.path[:0] = [str(ROOT / "chiaroscuro-raytracer_amd"), str(ROOT / "oracle")]
os.environ.setdefault("CHIARO_QUIET", "1")


def export(osc, kd, pos, xres, yres, spp, cam, seed, tree_path, rays_path):
    """tree.bin / rays.bin for quad_check (file mode): the oracle's kd tree in cr_upload_scene's node
    encoding (no hit tables: a segment ends at its first hit instead), shadow rays from the camera hits
    to a light sample and secondary rays in cosine-weighted directions, each ending at its first hit."""
    n = len(kd["is_leaf"])
    nodes = np.zeros((n, 2), np.uint32)
    leaf = kd["is_leaf"] != 0
    nodes[leaf, 0] = np.where(kd["leaf_count"][leaf] > 0, kd["leaf_first"][leaf], 0)
    nodes[leaf, 1] = 3 | (kd["leaf_count"][leaf] << 2)
    nodes[~leaf, 0] = kd["split"][~leaf].view(np.uint32)
    nodes[~leaf, 1] = kd["axis"][~leaf] | (kd["child"][~leaf] << 2)
    box = kd["box"]  # min xyz, max xyz
    with open(tree_path, "wb") as f:
        np.array([n, len(kd["refs"])], np.uint32).tofile(f)
        np.asarray(box, np.float32).tofile(f)
        nodes.tofile(f)
        np.zeros(n, np.uint32).tofile(f)  # no hit distances
    rng = np.random.default_rng(seed)
    ys, xs = np.mgrid[0:yres, 0:xres]
    xs = np.repeat(xs.ravel(), spp) + rng.random(xres * yres * spp)
    ys = np.repeat(ys.ravel(), spp) + rng.random(xres * yres * spp)
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
    ids, _ = osc.lights()
    li = ids[rng.integers(0, len(ids), len(p))]
    v0 = rng.random((len(p), 1)).astype(np.float32)
    v1 = (rng.random((len(p), 1)) * (1 - v0)).astype(np.float32)
    LP = pos[li]
    lp = LP[:, 0:3] * v0 + LP[:, 3:6] * v1 + LP[:, 6:9] * (1 - v0 - v1)
    so = (p + 0.001 * nrm).astype(np.float32)
    sd = lp - p
    dist = np.linalg.norm(sd, axis=1).astype(np.float32)
    sd = (sd / dist[:, None]).astype(np.float32)
    occ = osc.intersect(so, sd)
    send = np.where((occ["hit"] != 0) & (occ["dist"] < dist), occ["dist"], dist).astype(np.float32)
    # secondary rays: cosine-weighted about the normal
    u1, u2 = rng.random(len(p)), rng.random(len(p))
    r, ph = np.sqrt(u1), 2 * np.pi * u2
    tang = np.cross(nrm, np.where(np.abs(nrm[:, :1]) < 0.9, [[1, 0, 0]], [[0, 1, 0]]))
    tang /= np.linalg.norm(tang, axis=1, keepdims=True)
    bit = np.cross(nrm, tang)
    wi = (tang * (r * np.cos(ph))[:, None] + bit * (r * np.sin(ph))[:, None] + nrm * np.sqrt(1 - u1)[:, None])
    wi = (wi / np.linalg.norm(wi, axis=1, keepdims=True)).astype(np.float32)
    sec = osc.intersect(so, wi)
    cend = np.where(sec["hit"] != 0, sec["dist"], np.float32(3e38)).astype(np.float32)
    rays = np.concatenate([np.concatenate([so, sd, send[:, None], np.ones((len(so), 1))], 1),
                           np.concatenate([so, wi, cend[:, None], np.ones((len(so), 1))], 1)]).astype(np.float32)
    with open(rays_path, "wb") as f:
        np.array([len(rays)], np.uint32).tofile(f)
        rays.tofile(f)
    return len(so)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sponza")
    ap.add_argument("--res", default="320x180")
    ap.add_argument("--spp", type=int, default=2)
    args = ap.parse_args()
    import chiaroscuro_amd as ca
    import pyoracle as po
    from chiaroscuro_amd import scenes

    exe = Path(tempfile.mkdtemp()) / "quad_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    str(ROOT / "tests/native/quad_check.cpp")], check=True)
    sc = ca.Scene(scenes.config_rtc(args.config))
    i = sc.info
    m = ca.Model(sc)
    tris = m.triangles()
    osc = po.OracleScene(tris, leaf_size=i["leaf_size"], textures=m.textures(), build_threads=8)
    kd = osc.kd_export()
    pos = np.ascontiguousarray(tris["pos"], np.float32).reshape(-1, 9)
    xres, yres = (int(v) for v in args.res.split("x"))
    cam = po.camera(i["VP"], i["LA"], i["UP"], i["yview"], xres, yres)
    d = exe.parent
    nq = export(osc, kd, pos, xres, yres, args.spp, cam, 1, d / "tree.bin", d / "rays.bin")
    out = subprocess.run([str(exe), "file", str(d / "tree.bin"), str(d / "rays.bin")], capture_output=True,
                         text=True, check=True).stdout.split()
    s = {out[j]: int(out[j + 1]) for j in range(0, len(out), 2)}
    s["per_query"] = {k: round(s[k] / max(s["rays"], 1), 2) for k in ("leaf_tests", "fat_fetch_insts",
                                                                       "quad_fetch_insts", "mid_pops")}
    s["quad_over_fat"] = round(s["quad_fetch_insts"] / max(s["fat_fetch_insts"], 1), 4)
    s.update(config=args.config, res=args.res, spp=args.spp, queries_per_kind=nq,
             kinds="generation-1 shadow + secondary closest rays, segments ending at the first hit")
    print(json.dumps(s))


if __name__ == "__main__":
    main()
