"""Host-side mirror of the reference's Scene / Model / KDTree (CPU only).

  * .rtc parser: Scene(argc, argv) of src/scene.cpp:13-72 -- one token per
    line, CLI tokens after the file's, '#' lines skipped, defaults of :60-68
  * OBJ/MTL loader with the assimp post-processing the reference asks for
    (src/model.cpp:27: Triangulate | FlipUVs | GenNormals)
  * KDTree build: the host library's tree equals the oracle's node for node
    (two independent restatements of src/kdtree.cpp:34-194)
"""
from __future__ import annotations

import numpy as np
import pytest


def _rtc(tmp_path, lines, name="t.rtc"):
    p = tmp_path / name
    p.write_text("\n".join(lines) + "\n")
    return p


def test_rtc_defaults(ca, tmp_path):
    obj = tmp_path / "empty.obj"
    obj.write_text("")
    i = ca.Scene(_rtc(tmp_path, ["input", str(obj)])).info
    # src/scene.cpp:60-62 defaults
    assert (i["k"], i["xres"], i["yres"], i["samples"], i["leaf_size"]) == (3, 400, 300, 100, 8)
    assert i["VP"] == [0, 0, 2] and i["LA"] == [0, 0, 0] and i["UP"] == [0, 1, 0] and i["yview"] == 1
    assert i["using_preview"] and i["preview_height"] == 900 and i["exposure"] == 5
    assert i["background"] == [0, 0, 0] and i["render_path"] == "renders/output.exr"


def test_rtc_tokens_and_overrides(ca, tmp_path):
    obj = tmp_path / "empty.obj"
    obj.write_text("")
    p = _rtc(tmp_path, ["#comment", "no-preview", "input", str(obj), "k", "5", "xres", "64", "yres", "48",
                        "VP", "1", "2.5", "-3", "LA", "0", "1", "0", "yview", "0.7", "samples", "7",
                        "kdtree-leaf-size", "4", "exposure", "2", "bogus", "output", "x.pfm"])
    i = ca.Scene(p, "xres", "32", "samples", "9").info  # CLI tokens are parsed after the file's
    assert not i["using_preview"]
    assert (i["k"], i["xres"], i["yres"], i["samples"], i["leaf_size"]) == (5, 32, 48, 9, 4)
    assert i["VP"] == [1.0, 2.5, -3.0] and i["LA"] == [0, 1, 0]
    assert abs(i["yview"] - 0.7) < 1e-7 and i["exposure"] == 2
    assert i["render_path"] == "x.pfm" and i["obj_path"] == str(obj)
    assert i["n_invalid"] == 1  # "bogus" -> "Invalid argument" (src/scene.cpp:56)


OBJ = """# quad + triangle, one without normals
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0 0 1
vt 0 0
vt 1 0
vt 1 1
vt 0 1
vn 0 0 2
mtllib t.mtl
f 1/1 2/2 3/3
usemtl red
f 1/1/1 2/2/1 3/3/1 4/4/1
usemtl lamp
f 1 2 5
"""
MTL = """newmtl red
Kd 0.8 0.1 0.1
newmtl lamp
Kd 0 0 0
Ke 4 3 2
"""


def test_obj_loader_assimp_semantics(ca, tmp_path):
    (tmp_path / "t.obj").write_text(OBJ)
    (tmp_path / "t.mtl").write_text(MTL)
    m = ca.Model(path=str(tmp_path / "t.obj"))
    t = m.triangles()
    assert m.num_triangles == 4 and m.num_meshes == 3
    pos = t["pos"].reshape(-1, 3, 3)
    # aiProcess_Triangulate: the quad 1 2 3 4 fans from its first corner
    np.testing.assert_array_equal(pos[1], [[0, 0, 0], [1, 0, 0], [1, 1, 0]])
    np.testing.assert_array_equal(pos[2], [[0, 0, 0], [1, 1, 0], [0, 1, 0]])
    # GenNormals: faces without vn get the flat normal; given vn are kept as is (not normalised)
    np.testing.assert_allclose(t["vnrm"].reshape(-1, 3, 3)[0], [[0, 0, 1]] * 3)
    np.testing.assert_array_equal(t["vnrm"].reshape(-1, 3, 3)[1], [[0, 0, 2]] * 3)
    np.testing.assert_allclose(t["vnrm"].reshape(-1, 3, 3)[3], [[0, -1, 0]] * 3, atol=1e-7)
    # FlipUVs: v -> 1 - v
    np.testing.assert_array_equal(t["uv"].reshape(-1, 3, 2)[2], [[0, 1], [1, 0], [0, 0]])
    # faces before any usemtl use assimp's default material, which the reference skips -> Color()
    np.testing.assert_array_equal(t["kd"][0], [0, 0, 0])
    np.testing.assert_allclose(t["kd"][1], [0.8, 0.1, 0.1])
    np.testing.assert_array_equal(t["ke"][3], [4, 3, 2])
    assert (t["tex"] == -1).all()


@pytest.mark.parametrize("config", ["cornell", "cornell_box", "nanobox", "sponza"])
def test_host_kdtree_equals_oracle(ca, po, scenes, config):
    sc = ca.Scene(scenes.config_rtc(config))
    m = ca.Model(sc)
    host = ca.KDTree(m, sc).export()
    orc = po.OracleScene(m.triangles(), leaf_size=sc.info["leaf_size"], textures=m.textures(),
                         build_threads=8).kd_export()
    if config == "nanobox":
        # the stand-in's figure carries the real asset's texture set (data/nanosuit.mtl:11-75): five 1024^2
        # RGBA and one 128^2 RGBA image, over 20 MB of texels, on ~19k triangles (19,058 in nanosuit.obj);
        # the room adds a 256^2 RGB, a 128^2 RGBA and a 64^2 grey one
        tex = m.textures()
        shapes = sorted((w, h, nc) for w, h, nc, _ in tex)
        assert shapes == sorted([(1024, 1024, 4)] * 5 + [(128, 128, 4), (256, 256, 3), (128, 128, 4), (64, 64, 1)])
        assert sum(len(a) for *_, a in tex) >= 20 << 20
        assert 18500 <= m.num_triangles <= 19500 and (m.triangles()["tex"] >= 0).sum() > 18500
    for k in ("is_leaf", "axis", "child", "leaf_first", "leaf_count", "refs"):
        np.testing.assert_array_equal(host[k], orc[k], err_msg=k)
    for k in ("split", "box"):
        np.testing.assert_array_equal(host[k].view(np.uint32), orc[k].view(np.uint32), err_msg=k)
    if config == "sponza":
        assert len(host["is_leaf"]) == 328187 and len(host["refs"]) == 1238799 and orc["max_depth"] == 45


def test_scene_generators_are_deterministic(scenes, tmp_path):
    a = scenes.ensure("cornell_unit", tmp_path / "a")
    b = scenes.ensure("cornell_unit", tmp_path / "b")
    assert a.read_bytes() == b.read_bytes()
    assert scenes.sponza_triangle_count() == 261274
