"""CPU model check of the two-level quad node records (csrc/quadnodes.hpp) and of the descent the
secondary closest and shadow traces of builds 46 / 47 run over them (csrc/traverse.hpp, trav_round's QUAD
path): tests/native/quad_check.cpp builds the records with the product's own builder, walks them back
against the tree (every record word and axis checked), and restates the kernel's descent -- position codes
slot << 2 | sel, one record per two levels, a far middle child pushed as its parent's record and resumed
with one step of it, stack entries {code, tmax at push} restored by the kd stack invariant -- comparing,
ray by ray, the sequence of (leaf, tmin, tmax) tests and the answer with the recursion of
kdtree.cpp:248-281 / 322-344; the fat-record descent of builds 43 / 44 is checked the same way.  Random
trees (split ties with ray origins, axis-parallel directions, empty leaves) and a real scene's tree with
its generation-1 shadow and secondary rays.  Two broken variants of the quad descent must be caught.
(The GPU tests check the kernels bit-exact against the oracle: test_gpu_parity.py TRACE_BUILDS.)"""
import re
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "native" / "quad_check.cpp"


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = tmp_path_factory.mktemp("quad") / "quad_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(out), str(SRC)], check=True)
    return out


def _parse(stdout):
    m = re.search(r"violations (\d+) rays (\d+) leaf_tests (\d+) fat_fetch_insts (\d+) quad_fetch_insts (\d+) "
                  r"mid_pops (\d+)", stdout)
    assert m, stdout
    return [int(v) for v in m.groups()]


def _run(exe, *args):
    r = subprocess.run([str(exe)] + [str(a) for a in args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return _parse(r.stdout)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_quad_descent_equals_recursion(exe, seed):
    viol, rays, tests, fat, quad, mid = _run(exe, "rand", seed, 400)
    assert rays > 50_000 and tests > 150_000 and mid > 10_000
    assert viol == 0
    assert quad < 0.6 * fat  # one instruction per two levels instead of two


@pytest.mark.parametrize("mutant", [1, 2])
def test_quad_model_has_teeth(exe, mutant):
    """Children of c1 taken at gb_0 (1), or a popped middle child resumed as its record's root (2): the
    leaf sequences differ from the recursion's."""
    assert _run(exe, "rand", 1, 200, mutant)[0] > 0


def test_quad_descent_on_a_scene(exe, tmp_path, ca, po, scenes):
    """The nanobox stand-in's own tree and rays: zero violations, and about half the descent's fetch
    instructions (scripts/quad_census.py measures the sponza stand-in the same way)."""
    sys.path.insert(0, str(ROOT / "scripts"))
    import numpy as np
    import quad_census
    sc = ca.Scene(scenes.config_rtc("nanobox"))
    i = sc.info
    m = ca.Model(sc)
    tris = m.triangles()
    osc = po.OracleScene(tris, leaf_size=i["leaf_size"], textures=m.textures(), build_threads=4)
    kd = osc.kd_export()
    pos = np.ascontiguousarray(tris["pos"], np.float32).reshape(-1, 9)
    cam = po.camera(i["VP"], i["LA"], i["UP"], i["yview"], 96, 54)
    quad_census.export(osc, kd, pos, 96, 54, 1, cam, 7, tmp_path / "tree.bin", tmp_path / "rays.bin")
    viol, rays, tests, fat, quad, mid = _run(exe, "file", tmp_path / "tree.bin", tmp_path / "rays.bin")
    assert viol == 0 and rays > 5000 and tests > 50_000
    assert quad < 0.6 * fat
