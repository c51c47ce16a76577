"""bench.py's own multi-rank path on the CPU (the driver runs it on an
8-GPU node as `bench.py --gpus N`).

bench.py --gpus 2 without a torch.distributed environment spawns its two rank
processes (torch.distributed.run, 127.0.0.1), each checks WORLD_SIZE, renders its
tiles, rank 0 gathers them (gloo here, RCCL on the GPUs) and blends, every rank's
wall and render times are all-gathered and the step is timed by the slowest rank;
rank 0 prints the JSON line.  The device is the oracle-backed stand-in of
tests/bench_cpu_backend.py, named through CHIARO_BENCH_BACKEND (the product never
imports it).  The line must say n_gpus 2 with two per-rank render times, count
the oracle's rays, and the frame rank 0 accumulated over the layers must equal the
oracle's single-process progressive render bit for bit.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
RES, SPP, WARMUP, STEPS = (40, 24), 2, 1, 3


def test_bench_two_ranks_gloo(tmp_path, ca, po, scenes):
    frame = tmp_path / "frame.npy"
    env = dict(os.environ, CHIARO_BENCH_BACKEND="%s:make" % (ROOT / "tests" / "bench_cpu_backend.py"),
               MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2", CHIARO_QUIET="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", str(STEPS), "--warmup", str(WARMUP),
           "--config", "cornell", "--res", "%dx%d" % RES, "--spp", str(SPP), "--no-cpu-baseline", "--layers-per-pass", "2",
           "--save-frame", str(frame)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["steps"] == STEPS and line["backend"] == "cpu-oracle"
    assert len(line["config"]["rank_render_ms"]) == 2 and all(v > 0 for v in line["config"]["rank_render_ms"])
    assert line["config"]["parallelism"] == "tile-split x2"
    # two layers per render pass (DistributedFrame.render_layers: one pass, a gather + blend per
    # layer), then the odd step as a single-layer pass
    assert line["config"]["layers_per_pass"] == 2 and line["config"]["pass_groups"] == [[2, 1], [1, 1]]
    # the oracle's frame and rays over the same layers (warmup layers included in the frame)
    sc = scenes.config_rtc("cornell")
    s = ca.Scene(sc, "xres", str(RES[0]), "yres", str(RES[1]))
    i = s.info
    m = ca.Model(s)
    osc = po.OracleScene(m.triangles(), leaf_size=i["leaf_size"], textures=m.textures())
    cam = ca.camera(i["VP"], i["LA"], i["UP"], i["yview"], RES[0], RES[1]).as_array()
    ref, rays = None, 0
    for L in range(1, WARMUP + STEPS + 1):
        ref, c = osc.render(cam, RES[0], RES[1], SPP, i["k"], i["seed"], layer=L, bg=i["background"], pixels=ref)
        if L > WARMUP:
            rays += c["closest"] + c["shadow"]
    assert line["config"]["rays"] == rays
    got = np.load(frame)
    assert got.shape == ref.shape and (got.view(np.uint32) == ref.view(np.uint32)).all() and got.mean() > 0
    assert line["single_layer_ms"] > 0  # one-layer passes after the timed groups (not in value)
    # the bench's own parity check of the timed frame: every row it sampled, every layer, bit for bit
    par = line["parity"]
    assert par["differing"] == 0 and par["layers"] == WARMUP + STEPS and par["spp"] == SPP
    assert par["values"] == len(par["rows"]) * RES[0] * 3 and par["rows"][0] == 0 and par["rows"][-1] == RES[1] - 1
    # value: the rays of all ranks over the slowest rank's wall time (ms_per_step is that / steps)
    want = rays / (line["ms_per_step"] * STEPS / 1e3) / 1e6
    assert abs(line["value"] - want) <= 1e-3 * want + 2e-3


@pytest.mark.parametrize("nranks", [4, 8])
def test_bench_ranks_gloo_ragged_uneven_plans(tmp_path, nranks, ca, po, scenes):
    """The 8-rank protocol before an 8-GPU node runs it: bench.py --gpus 4 / 8 over gloo on a ragged
    200 x 150 frame (7 x 5 tiles of 32, partial on both edges: ranks hold 9 / 8 or 5 / 4 tiles), pass groups
    of up to 4 layers that the odd ranks' stand-in devices cap at 3 (CHIARO_TEST_ODD_RANK_CAP), so
    DistributedFrame.plan_layers' all-reduce MIN must bring every rank to the same groups of 3: each rank
    logs the (first layer, layers) of every pass it renders, and the logs must be identical; the frame rank 0
    blends from the gathered [nranks][3][tiles] buffers must equal the oracle's progressive render bit for
    bit, with one render time per rank in the line (src/rayTracer.cpp:55,64)."""
    res, spp, warmup, steps = (200, 150), 1, 1, 7
    frame, logs = tmp_path / "frame.npy", tmp_path / "plans"
    logs.mkdir()
    env = dict(os.environ, CHIARO_BENCH_BACKEND="%s:make" % (ROOT / "tests" / "bench_cpu_backend.py"),
               MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", CHIARO_QUIET="1", CHIARO_TEST_ODD_RANK_CAP="3",
               CHIARO_TEST_PLAN_LOG=str(logs))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(nranks), "--steps", str(steps), "--warmup",
           str(warmup), "--config", "cornell", "--res", "%dx%d" % res, "--spp", str(spp), "--no-cpu-baseline",
           "--layers-per-pass", "4", "--parity-rows", "4", "--save-frame", str(frame)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == nranks and line["config"]["parallelism"] == "tile-split x%d" % nranks
    assert len(line["config"]["rank_render_ms"]) == nranks and all(v > 0 for v in line["config"]["rank_render_ms"])
    # the agreed plan: groups of min(4, 3) layers, the 7 timed steps as 3 + 3 + 1
    assert line["config"]["layers_per_pass"] == 3 and line["config"]["pass_groups"] == [[3, 1], [3, 1], [1, 1]]
    plans = {p.name: p.read_text().split("\n") for p in logs.iterdir()}
    assert sorted(plans) == sorted("rank%d.txt" % r for r in range(nranks))
    want = ["1 1", "2 3", "5 3", "8 1"]  # warmup layer, the timed groups (then single layers, counting pass)
    for name, got in plans.items():
        assert got[:4] == want, (name, got)
        assert got == plans["rank0.txt"], (name, got)
    # the ranks' tile shares really are uneven (ragged frame)
    from chiaroscuro_amd.tiles import TileLayout
    lay = TileLayout(res[0], res[1], nranks, 32)
    assert len({lay.tiles_for_rank(q) for q in range(nranks)}) == 2
    sc = ca.Scene(scenes.config_rtc("cornell"), "xres", str(res[0]), "yres", str(res[1]))
    i = sc.info
    m = ca.Model(sc)
    osc = po.OracleScene(m.triangles(), leaf_size=i["leaf_size"], textures=m.textures())
    cam = ca.camera(i["VP"], i["LA"], i["UP"], i["yview"], res[0], res[1]).as_array()
    ref, rays = None, 0
    for L in range(1, warmup + steps + 1):
        ref, c = osc.render(cam, res[0], res[1], spp, i["k"], i["seed"], layer=L, bg=i["background"], pixels=ref)
        if L > warmup:
            rays += c["closest"] + c["shadow"]
    assert line["config"]["rays"] == rays
    got = np.load(frame)
    assert got.shape == ref.shape and (got.view(np.uint32) == ref.view(np.uint32)).all() and got.mean() > 0
    assert line["parity"]["differing"] == 0 and line["parity"]["layers"] == warmup + steps
    assert line["single_layer_mray_s"] > 0 and line["value_traced"] <= line["value"] + 1e-9


def test_frame_parity_detects_one_flipped_bit(ca, po, scenes):
    """bench.frame_parity compares the frame's rows with the oracle's layer blend bit for bit:
    the oracle's own frame passes, and one flipped mantissa bit is reported."""
    sys.path.insert(0, str(ROOT))
    import bench
    xres, yres, spp, layers = 24, 20, 2, 3
    s = ca.Scene(scenes.config_rtc("cornell"), "xres", str(xres), "yres", str(yres))
    i = s.info
    m = ca.Model(s)
    osc = bench.oracle_scene(m, i["leaf_size"])
    cam = ca.camera(i["VP"], i["LA"], i["UP"], i["yview"], xres, yres).as_array()
    ref = None
    for L in range(1, layers + 1):
        ref, _ = osc.render(cam, xres, yres, spp, i["k"], i["seed"], layer=L, pixels=ref)
    rows = bench.parity_rows(yres, 4)
    assert rows == [0, 6, 13, 19]
    ok = bench.frame_parity(osc, ref[rows], rows, cam, xres, yres, spp, i["k"], i["seed"], layers)
    assert ok["differing"] == 0 and ok["values"] == 4 * xres * 3 and ok["max_rel"] == 0.0
    bad = ref[rows].copy()
    bad.view(np.uint32)[2, 5, 1] ^= 1
    r = bench.frame_parity(osc, bad, rows, cam, xres, yres, spp, i["k"], i["seed"], layers)
    assert r["differing"] == 1 and r["max_rel"] > 0.0


def test_bench_stalled_rank_every_rank_exits_with_diagnostic(tmp_path):
    """Hardening of the first 8-GPU run (bench.py DistWatch): rank 1 stalls before its first timed pass group
    (CHIARO_TEST_STALL_RANK), so rank 0 waits in the group's plan all-reduce.  With --dist-timeout 6 rank 0
    must end itself once that collective has been in flight for 6 s, printing its rank, device, pass group
    and the collective, and the launcher then stops rank 1, which prints its own state (no collective, phase
    render).  The whole job ends non-zero long before the stall would have ended, and each rank's status is
    the collective-failure exit code (src/rayTracer.cpp:55,64)."""
    import time
    env = dict(os.environ, CHIARO_BENCH_BACKEND="%s:make" % (ROOT / "tests" / "bench_cpu_backend.py"),
               MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", CHIARO_QUIET="1", CHIARO_TEST_STALL_RANK="1",
               CHIARO_TEST_STALL_S="600")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--config",
           "cornell", "--res", "40x24", "--spp", "1", "--no-cpu-baseline", "--dist-timeout", "6"]
    t0 = time.monotonic()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    took = time.monotonic() - t0
    assert r.returncode != 0, r.stderr[-3000:]
    assert took < 240, took  # (the stall alone is 600 s)
    err = r.stderr
    assert "bench: FAILED rank 0 device cpu:0 pass group layers 2..3: collective all_reduce in flight" in err, err[-3000:]
    assert "collective timeout (6 s, --dist-timeout)" in err, err[-3000:]
    assert "bench: TERMINATED rank 1 device cpu:1 pass group layers 2..3: no collective in flight (phase: render)" \
        in err, err[-3000:]
    assert "exitcode  : 3" in err or "exit code 3" in err or "exitcode: 3" in err, err[-3000:]
