"""GPU parity: the HIP render loop (through the C-ABI) against the CPU oracle.

Bar: bit-exact.  The kernels evaluate every float in the reference's order with
-ffp-contract=off and correctly rounded div/sqrt, use the oracle's RNG, and run
glibc's sinf / cosf algorithm (equal to the host libm on every |x| < 120), so
pixels, ray-query results and the query counters must be identical -- also
against the oracle calling libm itself (test_parity_vs_libm_trig_oracle).
"""
import ctypes

import numpy as np
import pytest

from helpers import Pair, assert_bitwise, rel_rmse

pytestmark = pytest.mark.gpu

ORACLE_KEYS = ("closest", "shadow", "inner", "leaf", "tritest", "hit", "texhit", "paths")
# the wavefront trace builds (wavefront.hip kWf; the measured and superseded ones are removed, DESIGN.md
# keeps their numbers): the plain reference build 0, 15 (the packet camera
# trace's fallback), round 2's default 18, 26 (leaf cull records), 40 / 42 (26 / 18 with the exact
# short division in the camera packet), 43 / 44 (40 / 42 with it in the shadow trace) and the default 49
# (43 with the compressed leaf cull records); 53 / 54 (49 with the leaf exchange in the shadow trace, and
# in the shadow and secondary closest traces); the default 59 (54 with the exchange's prefix by a DPP scan)
TRACE_BUILDS = [0, 15, 18, 26, 40, 42, 43, 44, 49, 53, 54, 59]
VIS_DEFAULT = 1  # ctx.hpp wf_vis_dw
SKIP_DEFAULT = 1  # ctx.hpp wf_nee_skip
QUORUM_DEFAULT = -1  # ctx.hpp desc_quorum (8, but 0 for 1024 <= triangles < 65536)
SHADE_BLOCK_DEFAULT = 1024  # ctx.hpp wf_shade_block
SHADE_WAVES_DEFAULT = 8  # ctx.hpp wf_shade_waves


@pytest.fixture(scope="module")
def cornell(ca, po, scenes):
    return Pair(ca, po, scenes.config_rtc("cornell"))


@pytest.fixture(scope="module")
def cornell_mm(ca, po, scenes):
    return Pair(ca, po, scenes.config_rtc("cornell_box"))


@pytest.fixture(scope="module")
def sponza(ca, po, scenes):
    return Pair(ca, po, scenes.config_rtc("sponza"))


@pytest.fixture(scope="module")
def nanobox(ca, po, scenes):
    return Pair(ca, po, scenes.config_rtc("nanobox"))


@pytest.mark.parametrize("leaf", [0, 1])
@pytest.mark.parametrize("tile_dir", [(3, 8), (1, 2), (5, 32)])
def test_wavefront_sorted_queues_bitexact(ca, sponza, nanobox, tile_dir, leaf):
    """Queue sorting reorders the trace work only: force it on every queue (the
    default sorts queues of >= 1M rays) with several key layouts, pixel / world keys
    (leaf 0) or keys from the kd leaf of the hit a ray starts from (leaf 1)."""
    for pair, (x, y, s) in ((sponza, (96, 54, 3)), (nanobox, (64, 48, 4))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("wf_sort_min", 0)
        pair.dev.set_option("wf_sort_tile", tile_dir[0])
        pair.dev.set_option("wf_dir_res", tile_dir[1])
        pair.dev.set_option("wf_leaf_keys", leaf)
        try:
            g, gc, o, oc = _render_both(ca, pair, x, y, s)
        finally:
            pair.dev.set_option("wf_sort_min", 1 << 20)
            pair.dev.set_option("wf_sort_tile", 4)
            pair.dev.set_option("wf_dir_res", 128)
            pair.dev.set_option("wf_leaf_keys", 1)
        assert_bitwise(g, o, "sorted wavefront %dx%dx%d" % (x, y, s))
        assert {k: gc[k] for k in ORACLE_KEYS} == oc


@pytest.mark.parametrize("sort", [-1, 0, 1])
def test_wavefront_sort_choice_bitexact(ca, cornell_mm, sponza, sort):
    """Queue sorting on (1), off (0) or by scene size (-1, the default: only scenes of at least
    1024 triangles sort; cornell_box's 36 trace in append order), every queue of the render eligible
    (wf_sort_min 0): the same bits and counters."""
    for pair, (x, y, s) in ((cornell_mm, (45, 37, 4)), (sponza, (96, 54, 3))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("wf_sort", sort)
        pair.dev.set_option("wf_sort_min", 0)
        try:
            g, gc, o, oc = _render_both(ca, pair, x, y, s)
        finally:
            pair.dev.set_option("wf_sort", -1)
            pair.dev.set_option("wf_sort_min", 1 << 20)
        assert_bitwise(g, o, "wf_sort %d %dx%dx%d" % (sort, x, y, s))
        assert {k: gc[k] for k in ORACLE_KEYS} == oc


@pytest.mark.parametrize("resolve_paths,vis,mark", [(0, 0, 1), (1, 0, 1), (4, 0, 1), (64, 0, 1), (16, 1, 1), (0, 1, 1),
                                                   (16, 1, 0), (0, 1, 0), (64, 0, 0)])
def test_wavefront_resolve_order_bitexact(ca, sponza, nanobox, resolve_paths, vis, mark):
    """The NEE term of a bounce and the fold of an ended path: wf_resolve's sweep after each shadow
    trace, in queue order (resolve_paths 0) or, for queues of at least P / resolve_paths rays, in path
    order by the bounce mark (default 16; 64: nearly every generation).  The same bits and counters
    over progressive layers 1..3 on the same buffers (a mark left by an earlier layer or chunk must not
    resolve a path twice), sorted queues, one chunk and wf_paths 4096 chunks.  wf_vis_dw 1: the shadow
    trace writes each result over the slot in the path's dw record instead of occ[slot].  wf_vis_mark 1
    (the default): wf_shade stores the visible case's D_k = direct + contrib, the shadow trace sets the
    visible bit of the path's mark, and wf_resolve touches only visible or ended bounces.  (The list
    forms wf_fold 1 / 2 were measured slower and removed)"""
    for pair, (x, y, s) in ((sponza, (96, 54, 3)), (nanobox, (64, 48, 4))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("wf_vis_dw", vis)
        pair.dev.set_option("wf_vis_mark", mark)
        pair.dev.set_option("wf_resolve_paths", resolve_paths)
        pair.dev.set_option("wf_sort_min", 0)
        cam = pair.camera(ca, x, y)
        try:
            for paths in (256 << 20, 4096):
                pair.dev.set_option("wf_paths", paths)
                o = None
                for layer in (1, 2, 3):
                    p = ca.render_params(x, y, s, 6, 0xC41A05C0, layer=layer)
                    g = pair.dev.render(cam, p, None)
                    gc = pair.dev.counters()
                    o, oc = pair.oracle.render(cam.as_array(), x, y, s, 6, 0xC41A05C0, layer=layer, pixels=o)
                    assert_bitwise(g, o, "resolve_paths %d wf_paths %d layer %d" % (resolve_paths, paths, layer))
                    assert {k: gc[k] for k in ORACLE_KEYS} == oc
        finally:
            pair.dev.set_option("wf_vis_dw", VIS_DEFAULT)
            pair.dev.set_option("wf_vis_mark", 1)
            pair.dev.set_option("wf_resolve_paths", 16)
            pair.dev.set_option("wf_sort_min", 1 << 20)
            pair.dev.set_option("wf_paths", 256 << 20)


@pytest.mark.parametrize("chunk", [256, 1024])
def test_wavefront_chunked_appends_bitexact(ca, sponza, cornell_mm, chunk):
    """wf_shade's chunked queue appends (WfArgs::app_chunk; forced here by option wf_app_chunk, at full
    size they start at 8M rays): a block reserves `chunk` slots of a queue with one atomic and fills them
    over its iterations, and the unused end of its last chunk becomes dead entries (ray w = NO_PATH, key
    ~0) that the sort, the traces, wf_resolve and the next wf_shade skip.  128 x 96 x 128 spp puts several
    iterations on each shade block, so appends straddle chunks.  The same bits and query counters as the
    oracle, with sorted (sponza) and unsorted (cornell_box) queues.  Only the lean build chunks (the
    counting and performed-work builds have no dead-entry shadow trace, so their appends stay
    per-iteration): its render must report chunked wf_shade launches, or this test would pass with the
    chunks silently disabled."""
    x, y, s = 128, 96, 128
    for pair in (sponza, cornell_mm):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("wf_app_chunk", chunk)
        try:
            g, gc, o, oc = _render_both(ca, pair, x, y, s)  # (its last render is the lean one)
            assert pair.dev.chunked_shades() > 0, "the lean render used no chunked appends"
        finally:
            pair.dev.set_option("wf_app_chunk", 0)
        assert_bitwise(g, o, "wf_app_chunk %d" % chunk)
        assert {k: gc[k] for k in ORACLE_KEYS} == oc


@pytest.mark.parametrize("waves,block", [(6, 256), (8, 256), (8, 512), (8, 1024), (6, 512), (6, 1024)])
def test_wavefront_shade_waves_bitexact(ca, sponza, nanobox, waves, block):
    """wf_shade built for 8 waves per SIMD (the default; 64 VGPRs, spills) or its natural 6, in blocks
    of 256, 512 or 1024 threads (option wf_shade_block: one append per that many rays; 1024 is the
    default): every (waves, block) pair launches its own instantiation, and all give the same bits
    and counters, counting and lean builds."""
    for pair, (x, y, s) in ((sponza, (96, 54, 3)), (nanobox, (64, 48, 4))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("wf_shade_block", block)
        pair.dev.set_option("wf_shade_waves", waves)
        try:
            g, gc, o, oc = _render_both(ca, pair, x, y, s)
            pair.dev.set_option("counters", 0)
            g_lean = pair.dev.render(pair.camera(ca, x, y), ca.render_params(x, y, s, 6, 0xC41A05C0))
        finally:
            pair.dev.set_option("counters", 1)
            pair.dev.set_option("wf_shade_waves", SHADE_WAVES_DEFAULT)
            pair.dev.set_option("wf_shade_block", SHADE_BLOCK_DEFAULT)
        assert_bitwise(g, o, "wf_shade_waves %d block %d" % (waves, block))
        assert_bitwise(g_lean, o, "wf_shade_waves %d block %d lean" % (waves, block))
        assert {k: gc[k] for k in ORACLE_KEYS} == oc


@pytest.mark.parametrize("fuse,ctl,resolve_paths,skip", [(1, 0, 16, 0), (1, 0, 0, 0), (0, 0, 16, 0), (0, 1, 16, 0),
                                                       (1, 1, 16, 0), (1, 1, 0, 0), (1, 1, 16, 1), (0, 0, 0, 1)])
def test_wavefront_camera_fused_bitexact(ca, sponza, nanobox, fuse, ctl, resolve_paths, skip):
    """wf_cam_fuse 1: no wf_camera launch -- the packet camera trace makes each path's ray from its
    (pixel, sample), wf_shade(1) takes path p = ray p from the eye, clears the resolve mark of a path
    that missed and counts the paths; partial-tile slots carry a dead-ray record.  The same bits and
    counters over layers 1..3 on the same buffers (a mark an earlier layer or chunk left must not
    resolve a path), one chunk and wf_paths 4096 chunks, partial tiles (96 x 54, 3 x 2).  wf_ctl_ray 1: a
    secondary closest ray carries its path's RNG counter, the key is re-derived from (pixel, sample).
    wf_nee_skip 1: an NEE query whose contribution is exactly zero is answered without a trace and
    counted -- the shadow-query count stays the oracle's."""
    for pair, (x, y, s) in ((sponza, (96, 54, 3)), (nanobox, (64, 48, 4)), (nanobox, (3, 2, 1))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("wf_cam_fuse", fuse)
        pair.dev.set_option("wf_ctl_ray", ctl)
        pair.dev.set_option("wf_resolve_paths", resolve_paths)
        pair.dev.set_option("wf_nee_skip", skip)
        pair.dev.set_option("counters", 0)  # the lean builds: the packet camera trace
        cam = pair.camera(ca, x, y)
        keys = ("closest", "shadow", "hit", "texhit", "paths")
        try:
            for paths in (256 << 20, 4096):
                pair.dev.set_option("wf_paths", paths)
                o = None
                for layer in (1, 2, 3):
                    p = ca.render_params(x, y, s, 6, 0xC41A05C0, layer=layer)
                    g = pair.dev.render(cam, p, None)
                    gc = pair.dev.counters()
                    assert pair.dev.last_trace_build() in (59, 44)
                    o, oc = pair.oracle.render(cam.as_array(), x, y, s, 6, 0xC41A05C0, layer=layer, pixels=o)
                    assert_bitwise(g, o, "cam_fuse %d ctl_ray %d wf_paths %d layer %d" % (fuse, ctl, paths, layer))
                    assert {k: gc[k] for k in keys} == {k: oc[k] for k in keys}
                    if not skip:
                        assert gc["nee_answered"] == 0
                    elif pair is sponza:  # (its ceilings and arches face away from the sky light)
                        assert 0 < gc["nee_answered"] <= gc["shadow"]
        finally:
            pair.dev.set_option("counters", 1)
            pair.dev.set_option("wf_cam_fuse", 1)
            pair.dev.set_option("wf_ctl_ray", 1)
            pair.dev.set_option("wf_nee_skip", SKIP_DEFAULT)
            pair.dev.set_option("wf_resolve_paths", 16)
            pair.dev.set_option("wf_paths", 256 << 20)


@pytest.mark.parametrize("quorum", [0, 1, 8, 16, 32, 64])
def test_wavefront_desc_quorum_bitexact(ca, sponza, nanobox, quorum):
    """desc_quorum q: a wave's descent round stops at a node fetch once at most q / 64 of its lanes still
    descend; those lanes keep their node and interval and descend on next round (64: after every fetch).
    The lean builds 59 / 44, sorted queues, several layers: the same bits and query counters."""
    for pair, (x, y, s) in ((sponza, (96, 54, 3)), (nanobox, (64, 48, 4))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("desc_quorum", quorum)
        pair.dev.set_option("wf_sort_min", 0)
        pair.dev.set_option("counters", 0)
        cam = pair.camera(ca, x, y)
        keys = ("closest", "shadow", "hit", "texhit", "paths")
        try:
            o = None
            for layer in (1, 2):
                p = ca.render_params(x, y, s, 6, 0xC41A05C0, layer=layer)
                g = pair.dev.render(cam, p, None)
                gc = pair.dev.counters()
                assert pair.dev.last_trace_build() in (59, 44)
                o, oc = pair.oracle.render(cam.as_array(), x, y, s, 6, 0xC41A05C0, layer=layer, pixels=o)
                assert_bitwise(g, o, "desc_quorum %d layer %d" % (quorum, layer))
                assert {k: gc[k] for k in keys} == {k: oc[k] for k in keys}
        finally:
            pair.dev.set_option("counters", 1)
            pair.dev.set_option("desc_quorum", QUORUM_DEFAULT)
            pair.dev.set_option("wf_sort_min", 1 << 20)


@pytest.mark.parametrize("xcd,sort_min,variant", [(7, 0, 15), (7, 1 << 20, 15), (1, 0, 15), (2, 0, 15), (4, 0, 18),
                                                   (7, 0, 26), (0, 0, 26), (7, 0, 18), (0, 0, 18)])
def test_wavefront_xcd_partition_bitexact(ca, sponza, nanobox, xcd, sort_min, variant):
    """XCD-partitioned queues (wf_xcd bits: shadow, secondary closest, camera) change which
    block traces which ray only: every ray is traced once, whatever the queue length
    (queues shorter than the eight ranges included: the tiny frame)."""
    for pair, (x, y, s) in ((sponza, (96, 54, 3)), (nanobox, (64, 48, 4)), (nanobox, (3, 2, 1))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("variant", variant)
        pair.dev.set_option("wf_xcd", xcd)
        pair.dev.set_option("wf_sort_min", sort_min)
        try:  # (Pair sets wf_tail_min 0: every generation through wf_trace)
            g, gc, o, oc = _render_both(ca, pair, x, y, s)
        finally:
            pair.dev.set_option("wf_xcd", 7)
            pair.dev.set_option("variant", -1)
            pair.dev.set_option("wf_sort_min", 1 << 20)
        assert_bitwise(g, o, "xcd-partitioned wavefront %d %dx%dx%d" % (xcd, x, y, s))
        assert {k: gc[k] for k in ORACLE_KEYS} == oc


@pytest.mark.parametrize("variant", TRACE_BUILDS)
def test_wavefront_trace_builds_bitexact(ca, sponza, variant):
    """Every wavefront trace build (LDS ring depth, occupancy, scalar loads for
    wave-uniform nodes / leaves) renders the same bits."""
    sponza.dev.set_option("kernel", 2)
    sponza.dev.set_option("variant", variant)
    try:
        g, gc, o, oc = _render_both(ca, sponza, 80, 45, 4)
    finally:
        sponza.dev.set_option("variant", -1)
    assert_bitwise(g, o, "wavefront variant %d" % variant)
    assert {k: gc[k] for k in ORACLE_KEYS} == oc


def _doubled_cornell(scenes, directory):
    """cornell_box_lit with every wall / block face given twice, the copy in another material: every ray
    that hits a face hits two triangles at exactly the same t, and only the reference's tie rule (the
    first in leaf order, src/kdtree.cpp:235-246) gives the oracle's colour."""
    src = scenes.ensure("cornell_box_lit")
    swap = {"white": "red", "red": "white", "green": "white"}
    out, cur = [], None
    for ln in src.read_text().splitlines():
        if ln.startswith("mtllib"):
            out.append("mtllib doubled.mtl")
            continue
        out.append(ln)
        if ln.startswith("usemtl"):
            cur = ln.split()[1]
        elif ln.startswith("f ") and cur in swap:  # (the light stays single)
            out += ["usemtl " + swap[cur], ln, "usemtl " + cur]
    obj = directory / "doubled.obj"
    obj.write_text("\n".join(out) + "\n")
    (directory / "doubled.mtl").write_text(src.with_suffix(".mtl").read_text())
    return obj


@pytest.mark.parametrize("variant", [49, 53, 54, 59])
def test_leaf_exchange_ties_and_windows_bitexact(ca, po, scenes, tmp_path, variant):
    """The leaf exchange (builds 53 / 54, traverse.hpp leaf_exchange) against the per-lane leaf loop's
    answers: a box whose faces are all doubled (equal t, different materials: the closest reduction must
    keep the first in mask order) with leaves of up to 24 references (kdtree-leaf-size 24), so a round's
    pairs fill several 64-pair windows and owners carry over from one window to the next.  Counting and
    lean builds, forced queue sorting, bit for bit against the oracle; the performed-work build of 54
    must have run multi-window exchange rounds in both traces."""
    rtc = scenes.config_rtc("cornell_box")
    pair = Pair(ca, po, rtc, "input", str(_doubled_cornell(scenes, tmp_path)), "kdtree-leaf-size", "24")
    pair.dev.set_option("kernel", 2)
    pair.dev.set_option("variant", variant)
    pair.dev.set_option("wf_sort", 1)
    pair.dev.set_option("wf_sort_min", 0)
    g, gc, o, oc = _render_both(ca, pair, 64, 48, 16)
    assert_bitwise(g, o, "doubled box, leaf size 24, build %d" % variant)
    assert {k: gc[k] for k in ORACLE_KEYS} == oc
    if variant == 54:
        pair.dev.set_option("counters", 0)
        pair.dev.set_option("perf_counters", 1)
        cam = pair.camera(ca, 64, 48)
        g2 = pair.dev.render(cam, ca.render_params(64, 48, 16, 6, 0xC41A05C0, layer=1), None)
        perf = pair.dev.perf()
        assert_bitwise(g2, o, "doubled box, performed-work build 54")
        for kind in ("closest", "shadow"):
            pk = perf[kind]
            assert pk["drounds"] > 0 and pk["diters"] > pk["drounds"], (kind, pk)  # multi-window rounds
            assert 0 < pk["dtests"] <= pk["tests"], (kind, pk)  # every pair tested once (+ uniform leaves)


# cameras per scene for the cull test: the config's own, one close to a surface looking along it
# (edge-on triangles), one wide-angle from inside the geometry (triangles behind / beside the eye)
CULL_CAMS = {
    "sponza": [None, ((-1500, 20, -200), (600, 10, 150), (0, 1, 0), 0.6), ((-200, 300, 50), (900, 250, 0), (0, 1, 0), 2.5)],
    "nanobox": [None, ((9, 0.3, 9), (-5, 0.2, -4), (0, 1, 0), 0.8), ((2, 9, 2), (0, 8, -1), (0, 1, 0), 3.0)],
    "cornell": [None, ((-0.95, 0.02, 1.5), (0.9, 0.01, -0.9), (0, 1, 0), 1.2), ((0.1, 1.0, 0.3), (0.0, 0.9, -1.0), (0, 1, 0), 3.0)],
    "cornell_box": [None, ((30, 5, 20), (500, 3, 500), (0, 1, 0), 0.7), ((278, 273, 280), (278, 273, 0), (0, 1, 0), 2.0)],
}


@pytest.mark.parametrize("variant", [15, 18, 26])
@pytest.mark.parametrize("cfg", ["sponza", "nanobox", "cornell", "cornell_box"])
def test_camera_cull_bitexact(ca, po, scenes, sponza, nanobox, cornell, cornell_mm, cfg, variant):
    """Trace builds 15 / 18 / 26: the camera-ray trace skips Moller-Trumbore tests, leaves and
    subtrees by per-render screen-space cull boxes (camcull.hpp).  A skipped test could not have accepted, so
    the image and the per-query counters equal the oracle's -- at the config's camera,
    at an edge-on camera close to a surface and at a wide-angle camera inside the scene;
    also tile-split (global pixel coordinates) and at an odd frame size."""
    pair = {"sponza": sponza, "nanobox": nanobox, "cornell": cornell, "cornell_box": cornell_mm}[cfg]
    pair.dev.set_option("kernel", 2)
    pair.dev.set_option("variant", variant)
    try:
        for ci, spec in enumerate(CULL_CAMS[cfg]):
            for (x, y, s) in ((96, 54, 4), (61, 37, 3)):
                cam = pair.camera(ca, x, y) if spec is None else ca.camera(spec[0], spec[1], spec[2], spec[3], x, y)
                p = ca.render_params(x, y, s, 6, 0xC41A05C0)
                pair.dev.set_option("counters", 0)
                try:
                    g = pair.dev.render(cam, p)
                    lc = pair.dev.counters()
                    ts = pair.dev.trace_stats()
                    gt = _tiles_frame(ca, pair.dev, cam, x, y, s, 3, 16)
                finally:
                    pair.dev.set_option("counters", 1)
                o, oc = pair.oracle.render(cam.as_array(), x, y, s, 6, 0xC41A05C0)
                what = "%s camera %d %dx%dx%d" % (cfg, ci, x, y, s)
                assert ts["camera"]["launches"] == 1, what
                assert_bitwise(g, o, "cull " + what)
                assert_bitwise(gt, o, "cull, 3 ranks x tile 16, " + what)
                assert {k: lc[k] for k in ("closest", "shadow", "hit", "texhit", "paths")} == \
                    {k: oc[k] for k in ("closest", "shadow", "hit", "texhit", "paths")}, what
    finally:
        pair.dev.set_option("variant", -1)


@pytest.mark.parametrize("variant", [15, 18, 26])
@pytest.mark.parametrize("cfg", ["sponza", "nanobox", "cornell"])
def test_camera_cull_fuzz_bitexact(ca, sponza, nanobox, cornell, cfg, variant):
    """The default build (camera-ray cull boxes) at 12 random cameras per scene: eyes
    inside and outside the scene box, any view direction and up vector, fields of view
    from 6 to 170 degrees, odd frame sizes -- every image and per-query counter equal to
    the oracle's.  Seeded, so a failure reproduces."""
    pair = {"sponza": sponza, "nanobox": nanobox, "cornell": cornell}[cfg]
    rng = np.random.default_rng({"sponza": 11, "nanobox": 12, "cornell": 13}[cfg])
    lo, hi = np.array(list(pair.desc.box_min), np.float64), np.array(list(pair.desc.box_max), np.float64)
    ext = hi - lo
    pair.dev.set_option("kernel", 2)
    pair.dev.set_option("counters", 0)
    pair.dev.set_option("variant", variant)
    try:
        for i in range(12):
            eye = lo + ext * rng.uniform(-0.2 if i % 3 == 0 else 0.05, 1.2 if i % 3 == 0 else 0.95, 3)
            look = lo + ext * rng.uniform(0, 1, 3)
            up = rng.normal(size=3)
            yview = float(rng.uniform(0.1, 20.0) if i % 4 == 3 else rng.uniform(0.3, 2.5))
            x, y = int(rng.integers(17, 70)), int(rng.integers(11, 50))
            cam = ca.camera(eye, look, up, yview, x, y)
            g = pair.dev.render(cam, ca.render_params(x, y, 2, 6, 0xC41A05C0 + i))
            lc = pair.dev.counters()
            o, oc = pair.oracle.render(cam.as_array(), x, y, 2, 6, 0xC41A05C0 + i)
            what = "%s fuzz camera %d (%dx%d, yview %.2f)" % (cfg, i, x, y, yview)
            assert pair.dev.trace_stats()["camera"]["launches"] == 1, what  # the culling camera trace ran
            assert_bitwise(g, o, what)
            assert {k: lc[k] for k in ("closest", "shadow", "hit", "texhit", "paths")} == \
                {k: oc[k] for k in ("closest", "shadow", "hit", "texhit", "paths")}, what
    finally:
        pair.dev.set_option("counters", 1)
        pair.dev.set_option("variant", -1)


@pytest.mark.parametrize("variant", [18, 26, 40, 42])
def test_packet_camera_eye_on_split_plane(ca, sponza, cornell, variant):
    """Build 17's packet camera trace needs every camera ray to agree on a node's near
    child; an eye exactly on a split plane breaks that (kdtree.cpp:262 then decides by
    the ray's direction), and the render falls back to build 15's camera trace.  Eyes
    placed exactly on split planes of each axis render bit-exact either way."""
    for pair in (sponza, cornell):
        e = pair.kd.export()
        lo, hi = np.array(list(pair.desc.box_min)), np.array(list(pair.desc.box_max))
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("counters", 0)
        pair.dev.set_option("variant", variant)
        try:
            for axis in range(3):
                inner = np.nonzero((e["is_leaf"] == 0) & (e["axis"] == axis))[0]
                split = float(e["split"][inner[len(inner) // 2]])
                eye = (lo + hi) / 2
                eye[axis] = split
                look = eye + np.array([0.31, -0.2, 0.93]) * (hi - lo).max()
                cam = ca.camera(eye.astype(np.float32), look, (0, 1, 0), 1.4, 48, 40)
                assert cam.as_array()[axis] == np.float32(split)
                g = pair.dev.render(cam, ca.render_params(48, 40, 2, 6, 77 + axis))
                o, _ = pair.oracle.render(cam.as_array(), 48, 40, 2, 6, 77 + axis)
                assert_bitwise(g, o, "eye on a split plane of axis %d" % axis)
        finally:
            pair.dev.set_option("counters", 1)
            pair.dev.set_option("variant", -1)


@pytest.mark.parametrize("opts", [{"wf_cam_lean": 0}, {"wf_sort_g1": 0}, {"wf_sort_g1": 1}, {"wf_sort_g1": 2},
                                  {"wf_tail_waves": 5}, {"wf_tail_waves": 6}, {"wf_dir_res_shadow": 1},
                                  {"wf_dir_res_shadow": 4}])
def test_wavefront_generation1_options_bitexact(ca, sponza, nanobox, opts):
    """wf_camera writing generation 1's RNG state (wf_cam_lean 0) instead of wf_shade deriving it,
    generation-1 queues traced unsorted (wf_sort_g1 bits), the tail at 5 / 6 waves per SIMD, shadow
    queue keys with fewer direction bins: the same bits and counters, with and without the tail
    from generation 1."""
    for pair, (x, y, s) in ((sponza, (96, 54, 3)), (nanobox, (64, 48, 4))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("wf_sort_min", 0)
        for k, v in opts.items():
            pair.dev.set_option(k, v)
        try:
            for tail_min in (0, 3000):
                pair.dev.set_option("wf_tail_min", tail_min)
                g, gc, o, oc = _render_both(ca, pair, x, y, s)
                assert_bitwise(g, o, "%s tail_min %d %dx%dx%d" % (opts, tail_min, x, y, s))
                assert {k: gc[k] for k in ORACLE_KEYS} == oc
        finally:
            pair.dev.set_option("wf_cam_lean", 1)
            pair.dev.set_option("wf_sort_g1", 3)
            pair.dev.set_option("wf_tail_waves", 4)
            pair.dev.set_option("wf_dir_res_shadow", 0)
            pair.dev.set_option("wf_sort_min", 1 << 20)
            pair.dev.set_option("wf_tail_min", 0)


@pytest.mark.parametrize("lanes", [1, 2])
def test_wavefront_two_lanes_bitexact(ca, sponza, nanobox, cornell, lanes):
    """Two chunks in flight (wf_lanes 2: the frame's paths split in two, the second
    chunk started once the first is past its camera trace, per-lane buffers,
    streams and stacks), with the default per-generation launches and with the
    tail kernel, counting and lean builds."""
    for pair, (x, y, s) in ((sponza, (128, 72, 4)), (nanobox, (64, 48, 4)), (cornell, (64, 64, 4))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("wf_lanes", lanes)
        try:
            for tail_min in (0, 20000):
                pair.dev.set_option("wf_tail_min", tail_min)
                g, gc, o, oc = _render_both(ca, pair, x, y, s)
                assert_bitwise(g, o, "wf_lanes %d tail_min %d %dx%dx%d" % (lanes, tail_min, x, y, s))
                assert {k: gc[k] for k in ORACLE_KEYS} == oc
        finally:
            pair.dev.set_option("wf_lanes", 1)
            pair.dev.set_option("wf_tail_min", 0)


@pytest.mark.parametrize("tail_min", [1 << 30, 12000, 3000])
@pytest.mark.parametrize("overlap,ctl,vis,skip", [(1, 0, 0, 0), (0, 0, 0, 0), (1, 1, 0, 0), (0, 1, 0, 0), (1, 1, 1, 0),
                                                  (0, 1, 1, 0), (1, 1, 1, 1), (0, 1, 1, 1)])
def test_wavefront_tail_bitexact(ca, sponza, nanobox, cornell, tail_min, overlap, ctl, vis, skip):
    """wf_tail (the last generations of a chunk in one launch, per-path bodies
    shared with wf_shade / wf_bounce): from generation 1 (every queue is below
    1 << 30) and from later generations, counting and lean builds; after the last shadow trace
    (default) or overlapped (option wf_tail_overlap: the tail starts beside that trace and traces
    its own paths' shadow rays of that generation, the shadow trace and wf_resolve keep the paths
    that ended); wf_ctl_ray 1: the tail takes a path's RNG counter from its ray at pickup."""
    for pair, (x, y, s) in ((sponza, (96, 54, 3)), (nanobox, (64, 48, 4)), (cornell, (64, 64, 4))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("wf_tail_min", tail_min)
        pair.dev.set_option("wf_tail_overlap", overlap)
        pair.dev.set_option("wf_ctl_ray", ctl)
        pair.dev.set_option("wf_vis_dw", vis)
        pair.dev.set_option("wf_nee_skip", skip)
        try:
            g, gc, o, oc = _render_both(ca, pair, x, y, s)
            pair.dev.set_option("counters", 0)
            g_lean = pair.dev.render(pair.camera(ca, x, y), ca.render_params(x, y, s, 6, 0xC41A05C0))
            lc = pair.dev.counters()
            ts = pair.dev.trace_stats()
        finally:
            pair.dev.set_option("counters", 1)
            pair.dev.set_option("wf_tail_min", 0)
            pair.dev.set_option("wf_tail_overlap", 0)
            pair.dev.set_option("wf_ctl_ray", 1)
            pair.dev.set_option("wf_vis_dw", VIS_DEFAULT)
            pair.dev.set_option("wf_nee_skip", SKIP_DEFAULT)
        assert_bitwise(g, o, "wavefront tail_min %d %dx%dx%d" % (tail_min, x, y, s))
        assert_bitwise(g_lean, o, "wavefront tail_min %d lean" % tail_min)
        assert (lc["closest"], lc["shadow"]) == (oc["closest"], oc["shadow"])
        assert {k: gc[k] for k in ORACLE_KEYS} == oc
        assert ts["tail"]["launches"] == 1
        if tail_min == 1 << 30:
            assert all(ts[kind]["launches"] == 0 for kind in ("camera", "closest", "shadow"))
        else:
            assert ts["camera"]["launches"] == 1


def test_nanobox_textured_bitexact(ca, nanobox):
    """C3 stand-in: the asset's 1024^2 / 128^2 RGBA textures plus RGB and 1-channel ones, wrapped UVs,
    UV == 1 seams, explicit vertex normals (Texture::getColorAt, src/mesh.cpp:21-35)."""
    g, gc, o, oc = _render_both(ca, nanobox, 96, 54, 3)
    assert_bitwise(g, o, "nanobox 96x54x3")
    assert {k: gc[k] for k in ORACLE_KEYS} == oc
    assert oc["texhit"] > oc["hit"] // 2 and o.mean() > 0.01


LEAN_KEYS = ("closest", "shadow", "hit", "texhit", "paths", "pixels")


def _render_both(ca, pair, xres, yres, spp, k=6, seed=0xC41A05C0, layer=1, accum=None):
    """Counting build (all counters, compared with the oracle by the callers) AND
    the lean build the timed renders use (its own trace variant; per-query
    counters only), which must give the same bits."""
    cam = pair.camera(ca, xres, yres)
    p = ca.render_params(xres, yres, spp, k, seed, layer=layer)
    g = pair.dev.render(cam, p, None if accum is None else accum[0].copy())
    gc = pair.dev.counters()
    pair.dev.set_option("counters", 0)
    try:
        g_lean = pair.dev.render(cam, p, None if accum is None else accum[0].copy())
        lc = pair.dev.counters()
    finally:
        pair.dev.set_option("counters", 1)
    assert_bitwise(g_lean, g, "lean vs counting build %dx%dx%d" % (xres, yres, spp))
    assert {key: lc[key] for key in LEAN_KEYS} == {key: gc[key] for key in LEAN_KEYS}
    o, oc = pair.oracle.render(cam.as_array(), xres, yres, spp, k, seed, layer=layer,
                               pixels=None if accum is None else accum[1].copy())
    return g, gc, o, oc


def test_cornell_bitexact(ca, cornell):
    g, gc, o, oc = _render_both(ca, cornell, 64, 64, 4)
    assert_bitwise(g, o, "cornell 64x64x4")
    assert {k: gc[k] for k in ORACLE_KEYS} == oc
    assert gc["pixels"] == 64 * 64
    assert o.mean() > 0.01  # lit


def test_cornell_mm_bitexact_odd_size(ca, cornell_mm):
    # non-multiple-of-tile image: edge tiles are partial
    g, gc, o, oc = _render_both(ca, cornell_mm, 45, 37, 16)
    assert_bitwise(g, o, "cornell_box 45x37x16")
    assert {k: gc[k] for k in ORACLE_KEYS} == oc


def test_sponza_bitexact_small(ca, sponza):
    g, gc, o, oc = _render_both(ca, sponza, 96, 54, 2)
    assert_bitwise(g, o, "sponza 96x54x2")
    assert {k: gc[k] for k in ORACLE_KEYS} == oc
    assert oc["tritest"] > 100 * oc["closest"] / 10


def test_progressive_layers(ca, cornell):
    """Layer L blends (old*(L-1) + mean)/L on device (src/rayTracer.cpp:64)."""
    cam = cornell.camera(ca, 32, 32)
    g = o = None
    for layer in (1, 2, 3):
        p = ca.render_params(32, 32, 2, 6, 7, layer=layer)
        g = cornell.dev.render(cam, p, None)  # accumulator kept on the device ctx
        o, _ = cornell.oracle.render(cam.as_array(), 32, 32, 2, 6, 7, layer=layer, pixels=o)
        assert_bitwise(g, o, "layer %d" % layer)


def test_depth_limits_and_background(ca, cornell):
    for k in (1, 2, 9):
        g, gc, o, oc = _render_both(ca, cornell, 24, 24, 3, k=k)
        assert_bitwise(g, o, "k=%d" % k)
        assert {kk: gc[kk] for kk in ORACLE_KEYS} == oc
    cam = cornell.camera(ca, 16, 16)
    p = ca.render_params(16, 16, 2, 3, 1, background=(0.25, 0.5, 1.0))
    g = cornell.dev.render(cam, p)
    o, _ = cornell.oracle.render(cam.as_array(), 16, 16, 2, 3, 1, bg=(0.25, 0.5, 1.0))
    assert_bitwise(g, o, "background")


def _tiles_frame(ca, dev, cam, xres, yres, spp, nranks, tile, seed=0xC41A05C0):
    """The frame as nranks ranks render it: each rank's tiles, then the root's blend."""
    import torch
    p0 = ca.render_params(xres, yres, spp, 6, seed, nranks=nranks, tile=tile)
    maxt = ca.Device.tiles_for_rank(p0, 0)
    gathered = torch.zeros((nranks, maxt, tile, tile, 3), dtype=torch.float32, device="cuda")
    for r in range(nranks):
        dev.render_tiles_device(cam, ca.render_params(xres, yres, spp, 6, seed, rank=r, nranks=nranks, tile=tile),
                                gathered[r].data_ptr())
    frame = torch.zeros((yres, xres, 3), dtype=torch.float32, device="cuda")
    dev.blend_tiles_device(p0, gathered.data_ptr(), frame.data_ptr())
    torch.cuda.synchronize()
    return frame.cpu().numpy()


def test_tiles_partition_invariance(ca, cornell):
    """Rendering the tiles of nranks ranks one after another and blending on the
    root equals the 1-rank render bit for bit."""
    import torch
    xres, yres, spp, tile = 70, 50, 3, 16
    cam = cornell.camera(ca, xres, yres)
    full = cornell.dev.render(cam, ca.render_params(xres, yres, spp, 6, 11, tile=tile))
    for nranks in (2, 3):
        p0 = ca.render_params(xres, yres, spp, 6, 11, nranks=nranks, tile=tile)
        maxt = ca.Device.tiles_for_rank(p0, 0)
        gathered = torch.zeros((nranks, maxt, tile, tile, 3), dtype=torch.float32, device="cuda")
        for r in range(nranks):
            p = ca.render_params(xres, yres, spp, 6, 11, rank=r, nranks=nranks, tile=tile)
            cornell.dev.render_tiles_device(cam, p, gathered[r].data_ptr())
        frame = torch.zeros((yres, xres, 3), dtype=torch.float32, device="cuda")
        cornell.dev.blend_tiles_device(p0, gathered.data_ptr(), frame.data_ptr())
        torch.cuda.synchronize()
        assert_bitwise(frame.cpu().numpy(), full, "tiles nranks=%d" % nranks)


def test_ray_queries_bitexact(ca, sponza, cornell):
    """G2: KDTree::intersectRay / intersectShadowRay KAT incl. axis-parallel rays and
    origins on split planes (src/kdtree.cpp:196-344)."""
    rng = np.random.default_rng(5)
    for pair in (cornell, sponza):
        box = pair.oracle.kd_export()["box"]
        lo, hi = box[:3], box[3:]
        n = 4096
        o = lo + (hi - lo) * rng.random((n, 3), dtype=np.float32)
        d = rng.normal(size=(n, 3)).astype(np.float32)
        d[: n // 8, 1:] = 0.0                 # axis-parallel (inf/NaN slabs)
        d[n // 8: n // 4, 0] = 0.0
        e = pair.oracle.kd_export()
        inner = np.nonzero(e["is_leaf"] == 0)[0][: n // 8]
        for j, ni in enumerate(inner):         # origins exactly on split planes
            o[n // 4 + j, e["axis"][ni]] = e["split"][ni]
        g = pair.dev.intersect(o, d)
        want = pair.oracle.intersect(o, d)
        assert np.array_equal(g["hit"], want["hit"])
        h = want["hit"] == 1
        assert h.sum() > n // 4
        assert np.array_equal(g["tri"][h], want["tri"][h])
        assert np.array_equal(g["bary"][h].view(np.uint32), want["bary"][h].view(np.uint32))
        assert np.array_equal(g["dist"][h].view(np.uint32), want["dist"][h].view(np.uint32))
        ids, _ = pair.oracle.lights()
        light = ids[rng.integers(0, len(ids), n)]
        dist = (rng.random(n) * np.linalg.norm(hi - lo)).astype(np.float32)
        assert np.array_equal(pair.dev.intersect_shadow(o, d, dist, light),
                              pair.oracle.intersect_shadow(o, d, dist, light))
        # a shadow query without its distance or light arrays is refused, not read through a null pointer
        lib, hit = ca.libs()[0], np.zeros(n, np.uint32)
        o, d = np.ascontiguousarray(o, np.float32), np.ascontiguousarray(d, np.float32)
        dist, light = np.ascontiguousarray(dist, np.float32), np.ascontiguousarray(light, np.uint32)
        for dp, lp in ((None, light), (dist, None)):
            rc = lib.cr_intersect_shadow(pair.dev._c, n, ca._ptr(o), ca._ptr(d), None if dp is None else ca._ptr(dp),
                                         None if lp is None else ca._ptr(lp, ctypes.c_uint32),
                                         ca._ptr(hit, ctypes.c_uint32))
            assert ca.CR_ERRORS.get(rc) == "CR_E_INVALID"


@pytest.mark.parametrize("case", ["cornell", "sponza", "nanobox"])
def test_parity_vs_libm_trig_oracle(ca, po, cornell, sponza, nanobox, case):
    """The oracle calling the host's glibc sinf / cosf (src/brdf.cpp:52-53 exactly as
    the reference executes them) against the GPU: bit-exact, so the north-star
    metrics -- frame relative RMSE < 1e-4 and the count of pixels with
    |g - c| > 1e-4 (1 + |c|) -- are 0 on the headline scene too."""
    pair, (x, y, s) = {"cornell": (cornell, (64, 64, 8)), "sponza": (sponza, (160, 90, 6)),
                       "nanobox": (nanobox, (128, 72, 6))}[case]
    pair.dev.set_option("kernel", 2)
    po.set_trig_mode(1)
    try:
        g, gc, o, oc = _render_both(ca, pair, x, y, s)
    finally:
        po.set_trig_mode(0)
    bad = int((np.abs(g - o) > 1e-4 * (1 + np.abs(o))).any(axis=2).sum())
    print("%s %dx%dx%d vs libm-trig oracle: rel RMSE %.3g, pixels over 1e-4(1+|c|): %d" % (
        case, x, y, s, rel_rmse(g, o), bad))
    assert rel_rmse(g, o) < 1e-4 and bad == 0
    assert_bitwise(g, o, "%s vs libm-trig oracle" % case)
    assert {k: gc[k] for k in ORACLE_KEYS} == oc


def test_raytracer_api_layers(ca, scenes):
    """RayTracer(Model&, Scene&).rayTrace twice with one camera -> layer 2 (src/rayTracer.cpp:24-33)."""
    rtc = scenes.config_rtc("cornell")
    sc = ca.Scene(rtc, "xres", "40", "yres", "30", "samples", "2")
    m = ca.Model(sc)
    rt = ca.RayTracer(m, sc)
    i = sc.info
    rt.rayTrace(i["VP"], i["LA"], i["UP"], i["yview"])
    a = rt.pixels
    rt.rayTrace(i["VP"], i["LA"], i["UP"], i["yview"])
    assert rt.layers == 2
    b = rt.pixels
    assert not np.array_equal(a, b)
    assert rt.maxVal == float(b.max())
    rt.rayTrace(i["VP"], i["LA"], (0.2, 1.0, 0.0), i["yview"])  # up alone: no reset (reference quirk)
    assert rt.layers == 3
    rt.rayTrace((0.0, 1.1, 2.9), i["LA"], i["UP"], i["yview"])
    assert rt.layers == 1


def read_pfm(path):
    """PFM (little-endian, rows bottom-to-top) -> [H][W][3] float32, row 0 = top."""
    data = open(path, "rb").read()
    parts = data.split(b"\n", 3)
    assert parts[0] == b"PF"
    w, h = (int(v) for v in parts[1].split())
    assert float(parts[2]) < 0
    return np.frombuffer(parts[3], dtype="<f4", count=w * h * 3).reshape(h, w, 3)[::-1]


def test_cli_offline_render_matches_oracle(ca, po, scenes, tmp_path):
    """bin/chiaroscuro scene.rtc tokens... layers 2 -> PFM equal to the oracle's
    two progressive layers (main.cpp:5-21 + rayTracer.cpp:17-74 end to end)."""
    import subprocess
    from helpers import Pair
    rtc = scenes.config_rtc("nanobox")
    out = tmp_path / "nb.pfm"
    exe = scenes.default_dir().parent.parent / "bin" / "chiaroscuro"
    r = subprocess.run([str(exe), str(rtc), "xres", "64", "yres", "36", "samples", "3", "output", str(out),
                        "layers", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    g = read_pfm(out)
    pair = Pair(ca, po, rtc, "xres", "64", "yres", "36", "samples", "3", device=False)
    i = pair.info
    cam = ca.camera(i["VP"], i["LA"], i["UP"], i["yview"], 64, 36).as_array()
    o, _ = pair.oracle.render(cam, 64, 36, 3, i["k"], i["seed"], layer=1)
    o, _ = pair.oracle.render(cam, 64, 36, 3, i["k"], i["seed"], layer=2, pixels=o)
    assert_bitwise(g, o, "cli nanobox 64x36x3, 2 layers")


# --- C5 (sponza 4K x 3000 spp = 30 progressive batches of 100 spp, 8-way tile split)
# code paths at test size (BASELINE.json configs[4]; src/rayTracer.cpp:18-33,64) -----

def test_c5_sample_chunking_progressive(ca, sponza, nanobox):
    """A 4K x 100 spp batch does not fit one sample buffer, so it renders in sample
    chunks whose per-pixel running sum carries across launches (sum_samples).
    Force it with a buffer of 3 samples' worth (chunks of 3, 3, 2 of 8 spp) and
    blend layers 1..3: bit-exact with the oracle, equal counters per layer."""
    for pair, (x, y) in ((sponza, (96, 54)), (nanobox, (64, 48))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("sample_buf_bytes", x * y * 12 * 3)
        cam = pair.camera(ca, x, y)
        o = None
        try:
            for layer in (1, 2, 3):
                p = ca.render_params(x, y, 8, 6, 0xC41A05C0, layer=layer)
                g = pair.dev.render(cam, p, None)
                gc = pair.dev.counters()
                o, oc = pair.oracle.render(cam.as_array(), x, y, 8, 6, 0xC41A05C0, layer=layer, pixels=o)
                assert_bitwise(g, o, "chunked %dx%dx8 layer %d" % (x, y, layer))
                assert {k: gc[k] for k in ORACLE_KEYS} == oc
        finally:
            pair.dev.set_option("sample_buf_bytes", 4 << 30)
            pair.dev.set_option("kernel", 2)


@pytest.mark.parametrize("staged", [1, 0])
def test_sum_samples_staged_bitexact(ca, nanobox, staged):
    """sum_samples_lds (the default when a pass's samples per pixel are a multiple of 4: the runs staged
    through LDS 16 samples at a time) and the thread-per-pixel sum_samples add the same samples in the
    same order: spp 20 and 36 (chunks straddling the 16-sample stage), sample chunks of 8 + 8 + 4
    (sample_buf_bytes), and 3 layers of 20 spp in one pass (layer boundaries inside a stage),
    bit-exact against the oracle."""
    import torch
    pair, (x, y) = nanobox, (70, 45)
    dev = pair.dev
    cam = pair.camera(ca, x, y)
    dev.set_option("kernel", 2)
    dev.set_option("counters", 0)
    dev.set_option("sum_staged", staged)
    try:
        for spp, buf in ((20, 4 << 30), (36, 4 << 30), (20, x * y * 12 * 8)):
            dev.set_option("sample_buf_bytes", buf)
            o = None
            for layer in (1, 2):
                g = dev.render(cam, ca.render_params(x, y, spp, 6, 0xC41A05C0, layer=layer), None)
                o, _ = pair.oracle.render(cam.as_array(), x, y, spp, 6, 0xC41A05C0, layer=layer, pixels=o)
                assert_bitwise(g, o, "sum_staged %d spp %d buf %d layer %d" % (staged, spp, buf, layer))
        dev.set_option("sample_buf_bytes", 4 << 30)
        p = ca.render_params(x, y, 20, 6, 0xC41A05C0, layer=1)
        assert dev.layers_per_pass(p, 3) == 3
        frame = torch.zeros((y, x, 3), dtype=torch.float32, device="cuda")
        dev.render_layers_device(cam, p, 3, frame.data_ptr())
        torch.cuda.synchronize()
        o = None
        for layer in (1, 2, 3):
            o, _ = pair.oracle.render(cam.as_array(), x, y, 20, 6, 0xC41A05C0, layer=layer, pixels=o)
        assert_bitwise(frame.cpu().numpy(), o, "sum_staged %d, 3 layers x 20 spp in one pass" % staged)
    finally:
        dev.set_option("sum_staged", 1)
        dev.set_option("sample_buf_bytes", 4 << 30)
        dev.set_option("counters", 1)


@pytest.mark.parametrize("lanes", [1, 2])
def test_c5_multi_chunk_wavefront(ca, sponza, nanobox, lanes):
    """More work items than path slots: the wavefront runs chunk after chunk of
    wf_paths = 4096 paths (cabi.cpp w0 loop; with 2 lanes two chunks in flight,
    run_wavefront_lanes), also combined with sample chunking, over progressive
    layers 1..3, counting and lean builds."""
    for pair, (x, y) in ((sponza, (96, 54)), (nanobox, (64, 48))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("wf_lanes", lanes)
        pair.dev.set_option("wf_paths", 4096)
        cam = pair.camera(ca, x, y)
        o = None
        try:
            for layer, buf in ((1, 4 << 30), (2, x * y * 12 * 2), (3, 4 << 30)):
                pair.dev.set_option("sample_buf_bytes", buf)
                p = ca.render_params(x, y, 5, 6, 0xC41A05C0, layer=layer)
                g = pair.dev.render(cam, p, None)
                gc = pair.dev.counters()
                o, oc = pair.oracle.render(cam.as_array(), x, y, 5, 6, 0xC41A05C0, layer=layer, pixels=o)
                assert_bitwise(g, o, "wf_paths 4096 %dx%dx5 layer %d" % (x, y, layer))
                assert {k: gc[k] for k in ORACLE_KEYS} == oc
            # lean build, same chunking, same bits as a fresh layer-1 render
            pair.dev.set_option("counters", 0)
            p = ca.render_params(x, y, 5, 6, 0xC41A05C0, layer=1)
            g = pair.dev.render(cam, p, None)
            o1, _ = pair.oracle.render(cam.as_array(), x, y, 5, 6, 0xC41A05C0, layer=1)
            assert_bitwise(g, o1, "wf_paths 4096 lean")
        finally:
            pair.dev.set_option("counters", 1)
            pair.dev.set_option("wf_paths", 256 << 20)
            pair.dev.set_option("sample_buf_bytes", 4 << 30)
            pair.dev.set_option("wf_lanes", 1)


def test_c5_eight_rank_tile32_split_sponza(ca, sponza):
    """The C4/C5 partition: 32x32 tiles round-robin over 8 ranks on a sponza frame
    of 10 x 6 = 60 tiles (ragged right/bottom edges at 310x180), two progressive
    layers, sample-chunked, blended on the root: equal to the oracle's full frame."""
    import torch
    x, y, spp, nr, tile = 310, 180, 3, 8, 32
    cam = sponza.camera(ca, x, y)
    sponza.dev.set_option("kernel", 2)
    sponza.dev.set_option("sample_buf_bytes", 4 * tile * tile * 12 * 2)
    frame = torch.zeros((y, x, 3), dtype=torch.float32, device="cuda")
    o = None
    try:
        for layer in (1, 2):
            p0 = ca.render_params(x, y, spp, 6, 0xC41A05C0, layer=layer, nranks=nr, tile=tile)
            maxt = ca.Device.tiles_for_rank(p0, 0)
            assert maxt == 8 and ca.Device.tiles_for_rank(p0, 7) == 7
            gathered = torch.zeros((nr, maxt, tile, tile, 3), dtype=torch.float32, device="cuda")
            for r in range(nr):
                p = ca.render_params(x, y, spp, 6, 0xC41A05C0, layer=layer, rank=r, nranks=nr, tile=tile)
                sponza.dev.render_tiles_device(cam, p, gathered[r].data_ptr())
            sponza.dev.blend_tiles_device(p0, gathered.data_ptr(), frame.data_ptr())
            torch.cuda.synchronize()
            o, _ = sponza.oracle.render(cam.as_array(), x, y, spp, 6, 0xC41A05C0, layer=layer, pixels=o)
            assert_bitwise(frame.cpu().numpy(), o, "sponza 8-rank tile-32 layer %d" % layer)
    finally:
        sponza.dev.set_option("sample_buf_bytes", 4 << 30)


@pytest.mark.parametrize("variant", [15, 18, 26])
def test_triangle_less_scene_culling_builds(ca, po, scenes, tmp_path, variant):
    """A model without triangles still renders through the culling camera traces: the
    cull boxes are built for an empty reference list too (every sample outside), so
    the packet / subtree-cull kernels never read a null box buffer.  Every camera ray
    misses; the frame is the background, as the oracle's."""
    empty = tmp_path / "empty.obj"
    empty.write_text("# no faces\nv 0 0 0\nv 1 0 0\nv 0 1 0\n")
    pair = Pair(ca, po, scenes.config_rtc("cornell"), "input", str(empty))
    assert pair.model.num_triangles == 0
    pair.dev.set_option("kernel", 2)
    pair.dev.set_option("variant", variant)
    cam = pair.camera(ca, 24, 16)
    p = ca.render_params(24, 16, 2, 3, 0xC41A05C0, background=(0.25, 0.5, 0.75))
    g = pair.dev.render(cam, p)
    o, oc = pair.oracle.render(cam.as_array(), 24, 16, 2, 3, 0xC41A05C0, bg=(0.25, 0.5, 0.75))
    assert_bitwise(g, o, "triangle-less scene, variant %d" % variant)
    assert pair.dev.counters()["closest"] == oc["closest"] == 24 * 16 * 2


@pytest.mark.parametrize("variant", [18, 26, 40, 42, 43, 44, 49, 53, 54, 59])
@pytest.mark.parametrize("tail_min", [0, 3000])
def test_perf_counters_build(ca, sponza, nanobox, tail_min, variant):
    """The performed-work builds (option perf_counters: builds 18 / 26 / 40 / 42 / 43 / 44 / 49 / 53 / 54 with
    counters, cr_get_perf) render the same bits, and their counts agree with the counting build's: the
    secondary and shadow traces take the reference traversal (steps and leaves equal; build 18 also runs
    every test, build 26's leaf cull only removes some; the leaf exchange of 53 / 54 tests every masked
    reference of a leaf, without the per-lane loop's stop at an occluder), the packet camera trace only
    removes tests and the steps of rays a subtree box excludes."""
    for pair, (x, y, s) in ((sponza, (96, 54, 3)), (nanobox, (64, 48, 4))):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("wf_tail_min", tail_min)
        cam = pair.camera(ca, x, y)
        p = ca.render_params(x, y, s, 6, 0xC41A05C0, layer=1)
        try:
            pair.dev.render(cam, p, None)
            gc, ts = pair.dev.counters(), pair.dev.trace_stats()
            pair.dev.set_option("counters", 0)
            pair.dev.set_option("variant", variant)
            pair.dev.set_option("perf_counters", 1)
            g = pair.dev.render(cam, p, None)
            lc, perf = pair.dev.counters(), pair.dev.perf()
        finally:
            pair.dev.set_option("perf_counters", 0)
            pair.dev.set_option("variant", -1)
            pair.dev.set_option("counters", 1)
            pair.dev.set_option("wf_tail_min", 0)
        o, oc = pair.oracle.render(cam.as_array(), x, y, s, 6, 0xC41A05C0, layer=1)
        assert_bitwise(g, o, "perf-counting build %d %dx%dx%d" % (variant, x, y, s))
        assert {k: lc[k] for k in LEAN_KEYS} == {k: gc[k] for k in LEAN_KEYS}
        assert sum(v["queries"] for v in perf.values()) == gc["closest"] + gc["shadow"]
        for kind in ("camera", "closest", "shadow"):
            pk, rk = perf[kind], ts[kind]
            if tail_min == 0:
                assert pk["queries"] > 0 and pk["vbytes"] + pk["sbytes"] > 0, (kind, pk)
            assert pk["tests"] <= rk["tritest"], (kind, pk, rk)
            assert pk["leaves"] <= rk["leaf"] and pk["steps"] <= rk["inner"], (kind, pk, rk)
            if kind != "camera" and tail_min == 0:
                assert (pk["steps"], pk["leaves"]) == (rk["inner"], rk["leaf"]), (kind, pk, rk)
                if variant in (18, 42, 44, 47):
                    assert pk["masks"] == 0 and pk["tests"] == rk["tritest"], (kind, pk, rk)
                else:
                    assert pk["masks"] <= pk["leaves"]
        if tail_min == 0:
            assert perf["tail"]["queries"] == 0
            assert perf["camera"]["tests"] < ts["camera"]["tritest"]
        else:
            assert perf["tail"]["queries"] > 0 and perf["tail"]["steps"] > 0


def test_perf_counters_default_build_only(ca, cornell):
    """perf_counters instruments builds 18, 26 and 40-44 (not 41) only: another build is refused loudly."""
    cornell.dev.set_option("kernel", 2)
    cornell.dev.set_option("counters", 0)
    cornell.dev.set_option("perf_counters", 1)
    cornell.dev.set_option("variant", 15)
    cam = cornell.camera(ca, 16, 16)
    try:
        with pytest.raises(RuntimeError):
            cornell.dev.render(cam, ca.render_params(16, 16, 1, 6, 0xC41A05C0, layer=1), None)
    finally:
        cornell.dev.set_option("variant", -1)
        cornell.dev.set_option("perf_counters", 0)
        cornell.dev.set_option("counters", 1)


def test_default_build_by_scene_size(ca, sponza, nanobox):
    """The default trace build culls leaves (59) on the 261k-triangle sponza stand-in and not (44)
    on the 20k-triangle nanobox stand-in (cabi.cpp LEAF_CULL_MIN_TRIS): seen through the
    performed-work counts of the default build."""
    masks = {}
    for name, pair in (("sponza", sponza), ("nanobox", nanobox)):
        pair.dev.set_option("kernel", 2)
        pair.dev.set_option("counters", 0)
        pair.dev.set_option("perf_counters", 1)
        try:
            pair.dev.render(pair.camera(ca, 64, 36), ca.render_params(64, 36, 2, 6, 0xC41A05C0, layer=1), None)
            perf = pair.dev.perf()
            builds = [pair.dev.last_trace_build()]
            pair.dev.set_option("perf_counters", 0)
            pair.dev.render(pair.camera(ca, 16, 8), ca.render_params(16, 8, 1, 6, 0xC41A05C0, layer=1), None)
            builds.append(pair.dev.last_trace_build())
        finally:
            pair.dev.set_option("perf_counters", 0)
            pair.dev.set_option("counters", 1)
        pair.dev.render(pair.camera(ca, 16, 8), ca.render_params(16, 8, 1, 6, 0xC41A05C0, layer=1), None)
        builds.append(pair.dev.last_trace_build())
        masks[name] = perf["shadow"]["masks"] + perf["closest"]["masks"] + perf["tail"]["masks"]
        # cr_last_trace_build names it: perf and lean renders the scene-size default, counting -1
        want = 59 if name == "sponza" else 44
        assert builds == [want, want, -1], (name, builds)
    assert masks["sponza"] > 0 and masks["nanobox"] == 0, masks


@pytest.mark.parametrize("tail_min,ctl", [(0, 0), (1 << 30, 0), (0, 1)])
def test_layers_per_pass_bitexact(ca, sponza, nanobox, tail_min, ctl):
    """Several progressive layers in ONE render pass (cr_render_layers_device /
    cr_render_tiles_layers_device: the paths of all layers in one chunk, each with its
    layer's RNG streams, src/rayTracer.cpp:18-33) equal one pass per layer bit for bit:
    the blended frame against the oracle's layers 1..3, and each layer's tile means
    against render_tiles_device of that layer alone (3 ranks, tile 16, ragged edges);
    wavefront generations and the tail kernel from generation 1."""
    import torch
    for pair, (x, y, s) in ((sponza, (96, 54, 3)), (nanobox, (70, 45, 4))):
        dev = pair.dev
        cam = pair.camera(ca, x, y)
        dev.set_option("kernel", 2)
        dev.set_option("counters", 0)
        dev.set_option("wf_tail_min", tail_min)
        dev.set_option("wf_ctl_ray", ctl)
        dev.set_option("wf_cam_fuse", ctl)
        try:
            p = ca.render_params(x, y, s, 6, 0xC41A05C0, layer=1)
            assert dev.layers_per_pass(p, 3) == 3
            frame = torch.zeros((y, x, 3), dtype=torch.float32, device="cuda")
            dev.render_layers_device(cam, p, 3, frame.data_ptr())
            torch.cuda.synchronize()
            c3 = dev.counters()
            o = None
            rays = 0
            for layer in (1, 2, 3):
                o, oc = pair.oracle.render(cam.as_array(), x, y, s, 6, 0xC41A05C0, layer=layer, pixels=o)
                rays += oc["closest"] + oc["shadow"]
            assert_bitwise(frame.cpu().numpy(), o, "3 layers in one pass %dx%dx%d" % (x, y, s))
            assert c3["closest"] + c3["shadow"] == rays and c3["pixels"] == 3 * x * y
            tile, nr = 16, 3
            for r in range(nr):
                q = ca.render_params(x, y, s, 6, 0xC41A05C0, layer=2, rank=r, nranks=nr, tile=tile)
                mt = ca.Device.tiles_for_rank(q, 0)
                both = torch.full((2, mt, tile, tile, 3), -1.0, dtype=torch.float32, device="cuda")
                dev.render_tiles_layers_device(cam, q, 2, both.data_ptr())
                for j in range(2):
                    one = torch.full((mt, tile, tile, 3), -1.0, dtype=torch.float32, device="cuda")
                    dev.render_tiles_device(cam, ca.render_params(x, y, s, 6, 0xC41A05C0, layer=2 + j, rank=r,
                                                                  nranks=nr, tile=tile), one.data_ptr())
                    torch.cuda.synchronize()
                    assert_bitwise(both[j].cpu().numpy(), one.cpu().numpy(), "rank %d layer %d tiles" % (r, 2 + j))
        finally:
            dev.set_option("wf_tail_min", 0)
            dev.set_option("wf_ctl_ray", 1)
            dev.set_option("wf_cam_fuse", 1)
            dev.set_option("counters", 1)
            torch.cuda.synchronize()


def test_layers_per_pass_limits(ca, cornell):
    """cr_layers_per_pass caps the layers at what fits one sample buffer (option
    sample_buf_bytes) and is 1 for the counting build and for two chunks in flight (wf_lanes 2); a pass
    of more layers than fit, or in two lanes, is refused with an error, not chunked.  The removed
    kernels (0: the megakernel, 1: thread per pixel) are refused by cr_set_option."""
    import torch
    dev = cornell.dev
    cam = cornell.camera(ca, 32, 32)
    p = ca.render_params(32, 32, 4, 6, 5)
    frame = torch.zeros((32, 32, 3), dtype=torch.float32, device="cuda")
    assert dev.layers_per_pass(p, 4) == 1  # counting build
    dev.set_option("counters", 0)
    try:
        dev.set_option("kernel", 2)
        assert dev.layers_per_pass(p, 4) == 4
        dev.set_option("sample_buf_bytes", 32 * 32 * 12 * 4 * 2)  # two layers' samples
        assert dev.layers_per_pass(p, 4) == 2
        with pytest.raises(RuntimeError):
            dev.render_layers_device(cam, p, 3, frame.data_ptr())
        dev.set_option("wf_lanes", 2)
        assert dev.layers_per_pass(p, 4) == 1
        with pytest.raises(RuntimeError):
            dev.render_layers_device(cam, p, 2, frame.data_ptr())
        for k in (0, 1):
            with pytest.raises(RuntimeError):
                dev.set_option("kernel", k)
    finally:
        dev.set_option("sample_buf_bytes", 4 << 30)
        dev.set_option("wf_lanes", 1)
        dev.set_option("counters", 1)
        torch.cuda.synchronize()


def test_layer_groups_frame_pieces_bitexact(ca, sponza):
    """bench.py's pass groups on one GPU (DistributedFrame.plan_layers / render_layers):
    4 layers per pass, the frame cut into the fewest tile-split pieces whose paths fit one
    chunk (option wf_paths caps it here), each piece blended in place -- equal bit for bit
    to the oracle's layers 1..4, and the summed counters to the oracle's rays."""
    import torch
    from chiaroscuro_amd.tiles import DistributedFrame
    x, y, s = 96, 54, 3
    dev = sponza.dev
    cam = sponza.camera(ca, x, y)
    dev.set_option("kernel", 2)
    dev.set_option("counters", 0)
    dev.set_option("wf_paths", 40000)  # one layer of the frame is 18432 paths: 4 layers need 2 pieces
    try:
        fr = DistributedFrame(dev, x, y, 0, 1, 32, device="cuda")
        p = ca.render_params(x, y, s, 6, 0xC41A05C0, layer=1)
        nl, pieces = fr.plan_layers(p, 4)
        assert (nl, pieces) == (4, 2)
        fr.render_layers(cam, p, nl, pieces=pieces)
        torch.cuda.synchronize()
        st = fr.last_stats()
        o, rays = None, 0
        for layer in range(1, 5):
            o, oc = sponza.oracle.render(cam.as_array(), x, y, s, 6, 0xC41A05C0, layer=layer, pixels=o)
            rays += oc["closest"] + oc["shadow"]
        assert_bitwise(fr.frame.cpu().numpy(), o, "4 layers, 2 pieces")
        assert st["passes"] == 2 and st["counters"]["closest"] + st["counters"]["shadow"] == rays
        assert st["counters"]["pixels"] == 4 * x * y
    finally:
        dev.set_option("wf_paths", 256 << 20)
        dev.set_option("counters", 1)
        torch.cuda.synchronize()


def test_render_layers_c_abi_groups_bitexact(ca, sponza):
    """cr_render_layers (the C-ABI of RayTracer::rayTraceLayers and the CLI's `layers N`):
    20 layers of the whole frame as pass groups of up to 16 layers, each group in the fewest
    frame pieces whose paths fit (wf_paths caps the chunk here: 14 layers in 6 pieces, then 6
    layers in 3), equal to the oracle's layers 1..20; counters summed over the passes."""
    x, y, s = 96, 54, 2
    dev = sponza.dev
    cam = sponza.camera(ca, x, y)
    dev.set_option("kernel", 2)
    dev.set_option("counters", 0)
    dev.set_option("wf_paths", 30000)  # a layer is 12288 paths
    try:
        g = dev.render_layers(cam, ca.render_params(x, y, s, 6, 77, layer=1), 20)
        c = dev.counters()
    finally:
        dev.set_option("wf_paths", 256 << 20)
        dev.set_option("counters", 1)
    o, rays = None, 0
    for layer in range(1, 21):
        o, oc = sponza.oracle.render(cam.as_array(), x, y, s, 6, 77, layer=layer, pixels=o)
        rays += oc["closest"] + oc["shadow"]
    assert_bitwise(g, o, "20 layers in pass groups")
    assert c["closest"] + c["shadow"] == rays and c["pixels"] == 20 * x * y


def test_rank_pieces_tiles_layers_bitexact(ca, sponza):
    """cr_render_tiles_layers_device with more layers than one chunk holds for a rank's tiles:
    the rank's share is cut into pieces (ranks r + kN of an N * m split, each written into the
    rank's compact buffer); every layer's tile means equal render_tiles_device of that layer
    alone, for both ranks of a 2-way split (tile 16, ragged edges)."""
    import torch
    x, y, s, tile, nr, nl = 96, 54, 3, 16, 2, 6
    dev = sponza.dev
    cam = sponza.camera(ca, x, y)
    dev.set_option("kernel", 2)
    dev.set_option("counters", 0)
    dev.set_option("wf_paths", 20000)  # a rank's 12 tiles x 6 layers are 55296 paths: 3 pieces
    try:
        for r in range(nr):
            q = ca.render_params(x, y, s, 6, 0xC41A05C0, layer=4, rank=r, nranks=nr, tile=tile)
            assert dev.layers_per_pass(q, nl) < nl and dev.layers_per_group(q, nl) == nl
            mt = ca.Device.tiles_for_rank(q, 0)
            allt = torch.full((nl, mt, tile, tile, 3), -1.0, dtype=torch.float32, device="cuda")
            dev.render_tiles_layers_device(cam, q, nl, allt.data_ptr())
            c = dev.counters()
            rays = 0
            for j in range(nl):
                one = torch.full((mt, tile, tile, 3), -1.0, dtype=torch.float32, device="cuda")
                dev.render_tiles_device(cam, ca.render_params(x, y, s, 6, 0xC41A05C0, layer=4 + j, rank=r, nranks=nr,
                                                              tile=tile), one.data_ptr())
                torch.cuda.synchronize()
                oc = dev.counters()
                rays += oc["closest"] + oc["shadow"]
                assert_bitwise(allt[j].cpu().numpy(), one.cpu().numpy(), "rank %d layer %d, pieces" % (r, 4 + j))
            assert c["closest"] + c["shadow"] == rays
    finally:
        dev.set_option("wf_paths", 256 << 20)
        dev.set_option("counters", 1)
        torch.cuda.synchronize()
