"""The host OBJ/MTL + texture loader (host/model.cpp) on the reference's OWN
assets, /root/reference/data (src/model.cpp:25-174 semantics: assimp with
aiProcess_Triangulate | FlipUVs | GenNormals, one Mesh per object/material
group, material colours only for mMaterialIndex > 0 (:85), map_Kd textures
loaded once per path (textures_loaded)).  The assets are not shipped (nanosuit
is licensed for personal use only), so these tests run only where the reference
tree exists -- the build container -- and skip on the GPU box.  No reference
code is run: the expectations below are counts read off the OBJ/MTL text.
"""
from pathlib import Path

import numpy as np
import pytest

DATA = Path("/root/reference/data")
pytestmark = pytest.mark.skipif(not (DATA / "nanosuit.obj").exists(), reason="reference assets not present")


def _groups(obj: Path):
    """[object name, usemtl, faces, triangles] per mesh of an OBJ as assimp's OBJ
    importer splits it: a new mesh per `o`, and per `usemtl` after faces (the
    tall block of cornell_box.obj repeats `usemtl white` mid-object)."""
    out = []
    for ln in obj.read_text().splitlines():
        t = ln.split()
        if not t:
            continue
        if t[0] == "o":
            out.append([t[1], None, 0, 0])
        elif t[0] == "usemtl":
            if out[-1][2]:
                out.append([out[-1][0], t[1], 0, 0])
            out[-1][1] = t[1]
        elif t[0] == "f":
            out[-1][2] += 1
            out[-1][3] += len(t) - 3  # fan triangulation: n-gon -> n-2 triangles
    return out


def _mtl(path: Path):
    mats, cur = {}, None
    for ln in path.read_text().splitlines():
        t = ln.split()
        if not t:
            continue
        if t[0] == "newmtl":
            cur = mats.setdefault(t[1], {})
        elif cur is not None and t[0] in ("Kd", "Ke", "Ka"):
            cur[t[0]] = [float(v) for v in t[1:4]]
        elif cur is not None and t[0] == "map_Kd":
            cur["map_Kd"] = t[1]
    return mats


def test_cornell_box_obj(ca):
    obj = DATA / "cornell_box.obj"
    groups = [g for g in _groups(obj) if g[3]]  # light / front_wall faces are commented out
    m = ca.Model(path=str(obj))
    t = m.triangles()
    assert m.num_meshes == len(groups) == 8
    assert m.num_triangles == sum(g[3] for g in groups) == 34
    mats = _mtl(DATA / "cornell_box.mtl")
    i = 0
    for name, mtl, _, ntri in groups:  # meshes in file order, triangles in mesh order
        np.testing.assert_array_equal(t["kd"][i:i + ntri], [mats[mtl]["Kd"]] * ntri, err_msg=name)
        i += ntri
    assert (t["tex"] == -1).all() and not t["ke"].any()
    assert len(m.textures()) == 0


def test_nanosuit_obj(ca):
    obj = DATA / "nanosuit.obj"
    groups = _groups(obj)
    mats = _mtl(DATA / "nanosuit.mtl")
    m = ca.Model(path=str(obj))
    t = m.triangles()
    assert m.num_meshes == len(groups) == 7
    assert m.num_triangles == sum(g[3] for g in groups) == 19058
    # one texture per distinct map_Kd (Glass is used by two groups and loaded once)
    maps = []
    for _, mtl, _, _ in groups:
        if mats[mtl]["map_Kd"] not in maps:
            maps.append(mats[mtl]["map_Kd"])
    tex = m.textures()
    assert len(tex) == len(maps) == 6
    shapes = sorted((w, h, nc) for w, h, nc, _ in tex)
    assert shapes == [(128, 128, 4)] + [(1024, 1024, 4)] * 5
    i = 0
    for name, mtl, _, ntri in groups:
        ids = np.unique(t["tex"][i:i + ntri])
        assert len(ids) == 1 and ids[0] == maps.index(mats[mtl]["map_Kd"]), name
        np.testing.assert_allclose(t["kd"][i:i + ntri], [mats[mtl]["Kd"]] * ntri, err_msg=name)
        i += ntri
    # FlipUVs / GenNormals leave finite UVs and non-zero normals everywhere
    assert np.isfinite(t["uv"]).all()
    assert (np.abs(t["vnrm"].reshape(-1, 3)).sum(axis=1) > 0).all()


def test_nanosuit_kdtree_host_equals_oracle(ca, po, tmp_path):
    """KDTree over the real nanosuit (19,058 tris): host build == oracle build, node for node."""
    rtc = tmp_path / "nanosuit.rtc"
    rtc.write_text("no-preview\ninput\n%s\nk\n6\nsamples\n1\nxres\n64\nyres\n64\n" % (DATA / "nanosuit.obj"))
    sc = ca.Scene(str(rtc))
    m = ca.Model(sc)
    host = ca.KDTree(m, sc).export()
    orc = po.OracleScene(m.triangles(), leaf_size=sc.info["leaf_size"], textures=m.textures(),
                         build_threads=8).kd_export()
    for k in ("is_leaf", "axis", "child", "leaf_first", "leaf_count", "refs"):
        np.testing.assert_array_equal(host[k], orc[k], err_msg=k)
    for k in ("split", "box"):
        np.testing.assert_array_equal(host[k].view(np.uint32), orc[k].view(np.uint32), err_msg=k)
    assert len(host["is_leaf"]) > 10000
