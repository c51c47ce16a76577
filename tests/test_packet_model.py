"""CPU model check of the packet camera-ray traversal (trace builds 17 / 18,
csrc/wavefront.hip wf_trace_packet): tests/native/packet_check.cpp restates the
packet algorithm -- wave-uniform node stream, per-ray intervals and active flags,
stack entries holding only each ray's tmax at push, tmin restored on pop by the kd
stack invariant, far-only rays parked with tmax = tmin, culled subtrees -- and
compares, ray by ray, the sequence of (leaf, tmin, tmax) tests and the answer with
the per-ray recursion of kdtree.cpp:248-281 on random trees, eyes, direction fans,
intervals, leaf hits and culls.  Two deliberately broken variants of the packet step
must be caught.  (The GPU tests check the kernels themselves bit-exact against the
oracle: test_gpu_parity.py test_camera_cull_*, test_packet_camera_eye_on_split_plane.)
"""
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "native" / "packet_check.cpp"


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = tmp_path_factory.mktemp("packet") / "packet_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(out), str(SRC)], check=True)
    return out


def _run(exe, seed, cases, mutant=0):
    r = subprocess.run([str(exe), str(seed), str(cases), str(mutant)], capture_output=True, text=True, timeout=300)
    m = re.search(r"violations (\d+) rays (\d+) leaf_tests (\d+)", r.stdout)
    assert m, r.stdout + r.stderr
    return [int(v) for v in m.groups()]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_packet_traversal_equals_recursion(exe, seed):
    viol, rays, tests = _run(exe, seed, 1500)
    assert rays > 150_000 and tests > 500_000
    assert viol == 0


@pytest.mark.parametrize("mutant", [1, 2])
def test_packet_model_has_teeth(exe, mutant):
    """Without parking far-only rays (1), or with inactive rays' tmax changed at a push
    (2), the restored intervals differ from the recursion's."""
    assert _run(exe, 1, 200, mutant)[0] > 0


def _spec(exe, seed, cases, mutant=0):
    r = subprocess.run([str(exe), str(seed), str(cases), str(mutant)], capture_output=True, text=True, timeout=300)
    m = re.search(r"spec (\d+) spec_used (\d+) spec_bad (\d+)", r.stdout)
    assert m, r.stdout + r.stderr
    return [int(v) for v in m.groups()]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_speculative_grandchild_index_guarded(exe, seed):
    """Build 48's camera packet loads the near-near grandchild's records ahead of the fetch that needs
    them (wf_trace_packet SPEC).  Its index comes from the fetched fat record alone: taken only when the
    near child's record is inner (a leaf's words hold its reference range, which runs past the node count)
    and inside the tree.  Every speculative index of the model's packets obeys that, and most of them are
    the next fetch."""
    spec, used, bad = _spec(exe, seed, 600)
    assert bad == 0 and spec > 20_000 and used > 0.5 * spec


def test_speculative_index_model_has_teeth(exe):
    """The unguarded form -- the near child's record read as inner even when it is a leaf, so a reference
    offset becomes a node index -- is caught.  (That was the first suspect for the full-size fault of the
    prefetch builds; with the index guarded they still faulted, and the cause was the asm blocks'
    missing early-clobber outputs, tests/test_smem_hazard.py.)"""
    assert _spec(exe, 1, 300, 3)[2] > 0
