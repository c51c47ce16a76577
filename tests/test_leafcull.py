"""CPU checks of the leaf cull records of trace build 19 (csrc/leafcull.hpp).

The secondary closest and shadow traces of build 19 skip a leaf's Moller-Trumbore
test when the leaf's cull record proves, for the ray's unit direction and its test
segment [0, tmax], that the test cannot accept: the triangle's normal lies in a cone
the ray is not grazing, and the segment misses the group's box padded by the rounding
bound.  tests/native/leafcull_check.cpp evaluates the test as the kernels and the
oracle do (IEEE single, no FMA contraction) on random and adversarial leaves (walls,
boxes, column fans, slivers, degenerate triangles) and rays (aimed at edges and
vertices a few ulps off, from the triangle planes, grazing, in-plane far to the side,
tmax a few ulps around the hit), with inv perturbed by 2 ulp as v_rcp_f32 may, and
counts accepted tests the mask dropped: there must be none.  Without the margins the
same run finds such tests (test_margins_are_needed), so the check has teeth.
"""
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "native" / "leafcull_check.cpp"
HDR = ROOT / "chiaroscuro-raytracer_amd" / "csrc" / "leafcull.hpp"


def _build(tmp_path, header_dir):
    exe = tmp_path / "leafcull_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", str(header_dir), "-o", str(exe), str(SRC)],
                   check=True)
    return exe


def _run(exe, seed, leaves, form=0):
    r = subprocess.run([str(exe), str(seed), str(leaves), str(form)], capture_output=True, text=True, timeout=600)
    m = re.search(r"violations (\d+) tested (\d+) accepted (\d+) skipped (\d+)", r.stdout)
    assert m, r.stdout + r.stderr
    return [int(v) for v in m.groups()]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_leaf_cull_is_conservative(tmp_path, seed):
    exe = _build(tmp_path, HDR.parent)
    viol, tested, accepted, skipped = _run(exe, seed, 6000)
    assert tested > 30_000_000 and accepted > 500_000 and skipped > 3_000_000
    assert viol == 0


def test_margins_are_needed(tmp_path):
    """Without the rounding margins (u = 0, no slab / coordinate slack) the checker
    finds accepted tests the mask would drop."""
    src = HDR.read_text()
    src = src.replace("const float u = 0x1p-24f;", "const float u = 0.0f;")
    src = src.replace("4.f * u * mb + 1e-20f;", "0.f;").replace("(1.f + 4.f * u) + 1e-20f;", "(1.f + 4.f * u);")
    assert "u = 0.0f" in src and "0.f;" in src
    (tmp_path / "hdr").mkdir()
    (tmp_path / "hdr" / "leafcull.hpp").write_text(src)
    exe = _build(tmp_path, tmp_path / "hdr")
    viol = _run(exe, 3, 6000)[0]
    assert viol > 100


@pytest.mark.parametrize("form", [2, 3, 4])
def test_packed_and_compressed_records_are_conservative(tmp_path, form):
    """The records the kernels read: packed (LC 4, builds 26 / 40 / 43), compressed (LC 5, build 49:
    boxes on a 16-bit scene grid up to 1000x wider than the leaf, the axis as three halves with kappa
    recomputed for it, half constants) and short (LC 6, build 51: the same boxes, a 7-bit octahedral
    axis, 6-bit kappa, power-of-two dt).  No accepted test dropped; the compressed forms skip nearly as
    much as the packed one."""
    exe = _build(tmp_path, HDR.parent)
    viol, tested, accepted, skipped = _run(exe, 4, 6000, form)
    assert viol == 0 and tested > 30_000_000 and accepted > 500_000
    if form >= 3:
        skipped_packed = _run(exe, 4, 6000, 2)[3]
        assert skipped >= (0.95 if form == 3 else 0.88) * skipped_packed


def test_compressed_record_margins_are_needed(tmp_path):
    """With the grid box rounded inward instead of outward, the compressed records drop accepted
    tests: the checker sees it, in both compressed forms.  (The quantised axis's move -- ~3e-5 rad as
    halves, up to ~0.01 rad as the short form's 7-bit octahedral codes -- sits inside the slack of the
    fixed C0 = 1/16 cone bound, so leaving its widening out is not visible to this check.)"""
    src = HDR.read_text()
    old = "while (ql > 0.0 && b + ql * st > lo) ql -= 1.0;"
    chk = "if (!(b + ql * st <= lo && b + qh * st >= hi)) return false;"
    src = src.replace(old, "ql += 2.0;").replace(chk, "")
    assert old in HDR.read_text() and old not in src and chk not in src
    (tmp_path / "hdr").mkdir()
    (tmp_path / "hdr" / "leafcull.hpp").write_text(src)
    exe = _build(tmp_path, tmp_path / "hdr")
    assert _run(exe, 5, 6000, 3)[0] > 0
    assert _run(exe, 5, 6000, 4)[0] > 0

