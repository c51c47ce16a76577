"""Throughput benchmark of the MI355X render loop (BASELINE.json metric).

metric : Mray/s (primary + secondary) -- closest-hit queries + shadow queries
         (calls equivalent to KDTree::intersectRay / intersectShadowRay) per second
         of wall time around the render steps.
step   : one progressive layer of the whole frame of the config at its spp
         (default: sponza stand-in 1920x1080 x 128 spp, k = 6).  Scene load, kd
         build and upload happen before the timed region; the scene is resident in
         HBM when the clock starts.  For N > 1 the frame is tile-split over ranks
         (tile t -> rank t mod N) and each step ends with a torch.distributed
         gather of the per-rank tile buffers to rank 0 (RCCL over xGMI) and the
         root-side unpermute + progressive blend, all inside the timed region.

`--gpus N` (N > 1) without a torch.distributed environment starts the N rank
processes itself (torch.distributed.run as a child process, before this process
touches the GPU) and exits with their status; under torch.distributed.run the
world size must equal N.

Prints ONE JSON line on rank 0 with the contract fields plus
  "roofline"      the dominant kernel (the trace kind with the most standalone
                  time per pass: the shadow-ray trace on the sponza stand-in since
                  the camera-ray cull of build 15) against the ceiling that binds
                  it: instruction issue (VALU / SALU wave-instructions
                  per launch from the committed rocprofv3 PMC summary
                  profiles/pmc_issue_<config>.json, divided by this run's live
                  HIP-event launch time, against 1024 SIMDs x 2.4 GHz / 2 cycles
                  and 256 scalar units x 2.4 GHz); the algorithmic-bytes view of
                  SURVEY §8d against HBM and the L2 aggregate stays as a
                  secondary field ("bytes"), with the fabric bytes measured;
  "cpu_baseline"  the oracle's OpenMP restatement on a bounded row sample of the
                  same frame, with every thread of this process's CPU share
                  and with 1 thread, and the host's physical core count.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "chiaroscuro-raytracer_amd"))
os.environ.setdefault("CHIARO_QUIET", "1")

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md: L2 aggregate over 8 XCDs, ~34.5 TB/s
CLK_GHZ = 2.4          # MI355X_MICROARCH.md: max shader clock
# issue ceilings, wave-instructions per second (MI355X_MICROARCH.md: a wave64 VALU
# instruction occupies a SIMD-32 for 2 cycles; one scalar ALU per CU, 1 per cycle)
VALU_PEAK_GIPS = 256 * 4 * CLK_GHZ / 2
SALU_PEAK_GIPS = 256 * CLK_GHZ


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def physical_cores():
    """Physical cores of this host (lscpu: sockets x cores per socket), or None."""
    import subprocess
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=30).stdout
        f = {k.strip(): v.strip() for k, v in (ln.split(":", 1) for ln in out.splitlines() if ":" in ln)}
        return int(f["Socket(s)"]) * int(f["Core(s) per socket"])
    except Exception:
        return None


def cpu_threads():
    """This process's CPU share: OMP_NUM_THREADS where the pool sets it (16 per GPU
    on the MI355X boxes), else the CPUs this process may run on."""
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))


def oracle_scene(model, leaf):
    """The oracle's scene (oracle/liboracle.so, test infrastructure) over the same triangle
    soup: the CPU baseline's timed restatement and the checker of the timed frame."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle as po

    t0 = time.time()
    osc = po.OracleScene(model.triangles(), leaf_size=leaf, textures=model.textures(), build_threads=cpu_threads())
    log("oracle: kd build %.1fs" % (time.time() - t0))
    return osc


def cpu_baseline(osc, cam, xres, yres, spp, k, seed, budget_s):
    """Oracle restatement on a row sample of the same frame: OpenMP over the sampled
    rows with the reference's static schedule (src/rayTracer.cpp:55), with all
    threads of this process's CPU share and with 1 thread, on the SAME sample (every
    ystep-th row x sample_spp), so the two legs and their ratio are comparable."""
    threads = cpu_threads()
    # calibrate with 1 thread on every 16th row at 1 spp, then size the sample so the
    # 1-thread leg takes ~0.7 of the budget (the all-thread leg then takes ~1/threads of it)
    step = min(16, yres)
    t0 = time.time()
    osc.render(cam, xres, yres, 1, k, seed, y0=0, y1=yres, ystep=step, threads=1)
    per_row_spp = max(time.time() - t0, 1e-3) / ((yres + step - 1) // step)
    work = budget_s * 0.7 / per_row_spp                 # affordable (row x spp) units at 1 thread
    s_spp = int(max(1, min(spp, work // yres)))         # the whole frame if it fits, more spp if time allows
    nrows = int(max(threads, min(yres, work // s_spp)))
    ystep = max(1, yres // nrows)
    nr = (yres + ystep - 1) // ystep

    def leg(nthreads):
        t0 = time.time()
        _, c = osc.render(cam, xres, yres, s_spp, k, seed, y0=0, y1=yres, ystep=ystep, threads=nthreads, lean=True)
        return c["closest"] + c["shadow"], time.time() - t0

    rays, dt1 = leg(1)
    runs = sorted(leg(threads)[1] for _ in range(3))
    dtn = runs[1]  # the median of three
    v_all, v_1t = rays / dtn / 1e6, rays / dt1 / 1e6
    phys = physical_cores()
    sample = "%d of %d rows (every %d-th) x %d px x %d spp, %d rays" % (nr, yres, ystep, xres, s_spp, rays)
    return {"value": round(v_all, 4), "unit": "Mray/s", "cores": threads, "kind": "port",
            "build": "oracle/liboracle_lean.so: oracle.c at the reference's -O3 (Makefile:5), -ffp-contract=off, "
                     "the checker's work counters compiled out of the traversal (OR_LEAN), libm sinf / cosf as the "
                     "reference's std::sin / std::cos (brdf.cpp:53); the same bits as the counting liboracle.so "
                     "that checks the parity rows",
            "value_1t": round(v_1t, 4), "threads_all": threads, "physical_cores": phys,
            "parallel_efficiency": round(v_all / (v_1t * threads), 3) if v_1t > 0 else None,
            # linear in cores from the 1-thread rate: an upper bound for the whole host (the pool
            # gives one GPU's job a 16-thread CPU share, so the other cores are not timed)
            "projected_all_physical": round(v_1t * phys, 2) if phys else None,
            "sample": "oracle/liboracle_lean.so (OpenMP over rows, static schedule as src/rayTracer.cpp:55) on the "
                      "same frame / seed, the same sample for both legs: %s; %d threads %.2f s (median of 3), "
                      "1 thread %.1f s" % (sample, threads, dtn, dt1)}


def parity_rows(yres, nrows):
    """nrows rows spread evenly over the frame, the first and the last included."""
    if nrows <= 1:
        return [yres // 2]
    return sorted({int(round(i * (yres - 1) / (nrows - 1))) for i in range(nrows)})


def frame_parity(osc, frame_rows, rows, cam, xres, yres, spp, k, seed, nlayers):
    """The timed frame against the oracle, bit for bit, on whole rows at the full spp.

    frame_rows [len(rows)][xres][3]: those rows of the accumulated frame after layers
    1..nlayers (warmup and timed groups, rendered by the lean default trace build in its
    pass groups / frame pieces / tile split).  The oracle renders every layer's batch mean of
    the same pixels (or_render_pixels: sendRay per sample in sample order, x 1/spp) and blends
    them in layer order exactly as src/rayTracer.cpp:64 does, in fp32:
        pixels = (pixels * (L - 1) + mean) / L."""
    import numpy as np
    px = np.tile(np.arange(xres, dtype=np.uint32), len(rows))
    py = np.repeat(np.asarray(rows, np.uint32), xres)
    acc = np.zeros((len(px), 3), np.float32)
    t0 = time.time()
    rays = 0
    for L in range(1, nlayers + 1):
        mean, c = osc.render_pixels(cam, xres, yres, spp, k, seed, px, py, layer=L, threads=cpu_threads())
        acc = (acc * np.float32(L - 1) + mean) / np.float32(L)
        rays += c["closest"] + c["shadow"]
    g = np.ascontiguousarray(frame_rows, np.float32).reshape(-1, 3)
    diff = g.view(np.uint32) != acc.view(np.uint32)
    ad = np.abs(g.astype(np.float64) - acc.astype(np.float64))
    rel = ad / np.maximum(np.abs(acc.astype(np.float64)), 1e-30)
    rmse = float(np.sqrt(np.mean(ad ** 2)) / max(float(np.mean(np.abs(acc))), 1e-30))
    return {"rows": [int(r) for r in rows], "layers": nlayers, "spp": spp, "values": int(diff.size),
            "differing": int(diff.sum()), "max_rel": float(rel[diff].max()) if diff.any() else 0.0,
            "rel_rmse": rmse, "oracle_rays": int(rays), "oracle_s": round(time.time() - t0, 2),
            "what": "rows of the timed frame (layers 1..%d blended) vs oracle/liboracle.so at the same seed, "
                    "bit for bit (uint32 compare of every fp32 value)" % nlayers}


def lane_util(iss, view, ceil_valu_frac=None):
    """Active lanes of the issued wave-instructions of one trace kind (the issue ceilings count wave
    instructions whatever their exec mask): VALU from rocprofv3 (SQ_THREAD_CYCLES_VALU / (64 x
    SQ_ACTIVE_INST_VALU), profiles/pmc_issue_<config>.json), vector memory estimated from the
    performed-work build's per-lane bytes over the profiled vector-load instructions at 16 B a lane (the
    records are 16-B loads; the few 4- and 8-B loads make it a lower bound)."""
    if not iss:
        return None
    out = {"valu": iss.get("valu_lane_util")}
    vb = ((view or {}).get("bytes_per_launch") or {}).get("performed_vector")
    vm = iss.get("vmem_rd_insts_per_launch")
    out["vmem_est_16B"] = round(vb / 16 / vm / 64, 3) if vb and vm else None
    if out["valu"] is not None and ceil_valu_frac is not None:
        out["valu_issue_x_lanes"] = round(ceil_valu_frac * out["valu"], 3)
        out["note"] = ("VALU issue %.2f of its ceiling x %.2f of the lanes active = %.2f of the lane-level "
                       "peak" % (ceil_valu_frac, out["valu"], ceil_valu_frac * out["valu"]))
    return out


def issue_roofline(dom, iss, views, issue, pass_view, kind):
    """Roofline of the dominant trace kernel against the ceiling that binds it.

    The trace kernels' working set (kd nodes + triangle records, ~65 MB for the
    sponza stand-in) stays in L2 / Infinity Cache: the algorithmic bytes per launch
     run at several times HBM peak while the measured fabric bytes are
    ~1.5 % of them, so HBM does not bound them.  What does is instruction issue:
    wave-instructions per launch (rocprofv3 SQ_INSTS_VALU / SQ_INSTS_SALU of this
    kernel, profiles/pmc_issue_<config>.json) over this run's HIP-event launch time,
    against the VALU issue peak (1024 SIMDs x 2.4 GHz / 2 cycles per wave64
    instruction) and the scalar-unit peak (256 x 2.4 GHz).  The binding ceiling is
    the one with the highest fraction; TA (vector address path) busy comes from
    the profile only (no live counterpart)."""
    t = dom["avg_launch_ms"] / 1e3
    perf_gbs = dom.get("achieved")
    bytes_view = {"per_launch": dom.get("bytes_per_launch"),
                  "performed_gbs": perf_gbs,
                  "performed_frac_of_l2_aggregate": round(perf_gbs / L2_PEAK_GBS, 4) if perf_gbs else None,
                  "reference_equivalent_gbs": dom["reference_equivalent_gbs"],
                  "fabric_gbs": dom.get("fabric_gbs"),
                  "fabric_frac_of_hbm": round(dom["fabric_gbs"] / HBM_PEAK_GBS, 4) if dom.get("fabric_gbs") else None,
                  "work_per_launch": dom.get("work_per_launch"),
                  "performed_work_per_launch": dom.get("performed_work_per_launch"),
                  "note": "performed = the bytes the kernel's loads and stores move (cr_get_perf, vector per lane + "
                          "scalar per wave), served mostly from L2 / Infinity Cache; fabric = measured HBM-side bytes "
                          "(rocprofv3 PMC); reference_equivalent = SURVEY 8d bytes of the reference algorithm's "
                          "work (counting build), which the culls skip in part"}
    what = {"camera": "camera-ray", "closest": "secondary closest-hit", "shadow": "shadow-ray"}[kind]
    base = {"kernel": dom["kernel"] + " (%s kd traversal, wavefront.hip)" % what,
            "avg_launch_ms": dom["avg_launch_ms"], "launches": dom["launches"],
            "rocprof_avg_launch_ms": dom["rocprof_avg_launch_ms"], "bytes": bytes_view,
            "other_traces": {k: v for k, v in views.items() if v is not None and v is not dom},
            "issue": issue, "pass": pass_view}
    if not iss or t <= 0 or "valu_insts_per_launch" not in iss:
        ach = dom["achieved"] if dom.get("achieved") is not None else dom["reference_equivalent_gbs"]
        return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": dom["traffic"],
                "note": "no instruction-issue profile of this configuration: performed bytes vs HBM", **base}
    valu = iss["valu_insts_per_launch"] / t / 1e9
    salu = iss["salu_insts_per_launch"] / t / 1e9
    ceil = {"valu": {"achieved": round(valu, 2), "peak": VALU_PEAK_GIPS, "frac": round(valu / VALU_PEAK_GIPS, 4),
                     "insts_per_launch": iss["valu_insts_per_launch"]},
            "salu": {"achieved": round(salu, 2), "peak": SALU_PEAK_GIPS, "frac": round(salu / SALU_PEAK_GIPS, 4),
                     "insts_per_launch": iss["salu_insts_per_launch"]},
            "ta_busy_profiled": iss.get("ta_busy"),
            "ta_note": "vector-memory address path busy fraction from the rocprofv3 PMC pass (no live "
                       "counterpart): the trace kernels are co-limited by issue and the address path",
            "hbm_bytes": {"frac": bytes_view["fabric_frac_of_hbm"], "note": "measured fabric bytes over the launch time"},
            "lane_util": lane_util(iss, dom, ceil_valu_frac=round(valu / VALU_PEAK_GIPS, 4))}
    bound = max(("valu", "salu"), key=lambda k: ceil[k]["frac"])
    b = ceil[bound]
    return {"bound": bound, "achieved": b["achieved"], "peak": b["peak"], "unit": "Gwave-inst/s", "frac": b["frac"],
            "traffic": dom["traffic"], "ceilings": ceil,
            "profile": "profiles/pmc_issue_<config>.json kinds[%s] (%s)" % (kind, iss["kernel"]), **base}


def spawn_ranks(n: int) -> int:
    """Start n rank processes of this script with torch.distributed.run (a child
    process; this process has not touched the GPU) and return their exit status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve())] + sys.argv[1:]
    log("bench: starting %d ranks: %s" % (n, " ".join(cmd)))
    return subprocess.call(cmd)


# Exit status of a rank that a collective error or timeout ended (DistWatch); the launcher then ends its peers.
EXIT_COLLECTIVE = 3


class DistWatch:
    """The multi-rank run's failure report (round-6 hardening of the first 8-GPU run).

    Each rank records what it is doing: the pass group it renders (`group`) and the collective in flight
    (`enter` / `leave`, done by WatchedDist around every torch.distributed call).  A daemon thread ends the
    rank with EXIT_COLLECTIVE when one collective has been in flight for `timeout_s` -- before the process
    group's own timeout (set 30 s later), so the message below is printed instead of a bare watchdog
    abort -- and a collective that raises (a peer gone, the backend's timeout) ends it the same way.  A
    SIGTERM (torch.distributed.run stopping the survivors after one rank failed) prints the rank's state
    too.  The message names the rank, its device, its pass group and the collective in flight (or its
    phase outside one), so the slow or dead rank of an 8-GPU run is found from the log alone
    (src/rayTracer.cpp:55,64: the reference's single-process loop has no such failure mode)."""

    def __init__(self, rank: int, device: str, timeout_s: float):
        import threading
        self.rank, self.device, self.timeout_s = rank, device, timeout_s
        self.group = "setup"
        self.phase = "setup"
        self.cur = None  # (collective, monotonic start)
        self._lock = threading.Lock()
        if timeout_s > 0:
            threading.Thread(target=self._run, name="dist-watch", daemon=True).start()
        try:
            import signal
            signal.signal(signal.SIGTERM, self._on_term)
        except ValueError:  # (not the main thread: no handler)
            pass

    def state(self) -> str:
        with self._lock:
            cur = self.cur
        what = ("collective %s in flight for %.1f s" % (cur[0], time.monotonic() - cur[1]) if cur
                else "no collective in flight (phase: %s)" % self.phase)
        return "rank %d device %s pass group %s: %s" % (self.rank, self.device, self.group, what)

    def fail(self, why: str) -> None:
        log("bench: FAILED %s -- %s" % (self.state(), why))
        os._exit(EXIT_COLLECTIVE)

    def enter(self, name: str) -> None:
        with self._lock:
            self.cur = (name, time.monotonic())

    def leave(self) -> None:
        with self._lock:
            self.cur = None

    def _run(self) -> None:
        while True:
            time.sleep(min(1.0, self.timeout_s / 4))
            with self._lock:
                cur = self.cur
            if cur and time.monotonic() - cur[1] > self.timeout_s:
                self.fail("collective timeout (%.0f s, --dist-timeout)" % self.timeout_s)

    def _on_term(self, signum, frame) -> None:
        log("bench: TERMINATED %s" % self.state())
        os._exit(EXIT_COLLECTIVE)


class WatchedDist:
    """torch.distributed as the bench and DistributedFrame use it, every collective bracketed by
    DistWatch.enter / leave and an exception from one reported by DistWatch.fail."""

    COLLECTIVES = ("barrier", "all_reduce", "all_gather", "gather", "broadcast", "broadcast_object_list")

    def __init__(self, dist, watch: DistWatch):
        self._dist, self._watch = dist, watch

    def __getattr__(self, name):
        attr = getattr(self._dist, name)
        if name not in self.COLLECTIVES:
            return attr
        watch = self._watch

        def call(*a, **kw):
            watch.enter(name)
            try:
                r = attr(*a, **kw)
            except Exception as e:  # (a peer gone, the backend's own timeout)
                watch.fail("%s raised %s: %s" % (name, type(e).__name__, str(e).splitlines()[0][:300] if str(e) else ""))
            watch.leave()
            return r
        return call


class GpuBackend:
    """What a rank runs on: one MI355X per rank, RCCL (the nccl backend) between
    ranks, the C-ABI device (chiaroscuro_amd.Device) with the scene in HBM.

    The rank loop below (run_rank) only talks to this object and to the device it
    makes, so the multi-rank protocol -- spawn, WORLD_SIZE check, per-rank timing,
    slowest-rank step, gather, JSON line -- can be exercised on the CPU: a test
    names a stand-in backend in CHIARO_BENCH_BACKEND ("path/to/file.py:factory";
    tests/bench_cpu_backend.py, gloo + an oracle-backed device).  The product never
    ships or imports a stand-in."""

    name = "gpu"
    device = "cuda"
    dist_backend = "nccl"

    def init_rank(self, world, local, timeout_s=120.0):
        import datetime
        import torch
        torch.cuda.set_device(local)
        if world > 1:
            import torch.distributed as dist
            # asynchronous error handling: a failed or timed-out RCCL collective raises (or ends the process)
            # instead of leaving the rank blocked; DistWatch reports first (its timeout is 30 s shorter)
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
            dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                    timeout=datetime.timedelta(seconds=timeout_s + 30.0))
            return dist
        return None

    def collectives_version(self) -> str:
        import torch
        try:
            v = torch.cuda.nccl.version()
            return "RCCL %s" % (".".join(str(x) for x in v) if isinstance(v, tuple) else v)
        except Exception as e:  # (reported, never fatal)
            return "RCCL version unknown (%s)" % type(e).__name__

    def synchronize(self):
        import torch
        torch.cuda.synchronize()

    def stream(self):
        import torch
        return torch.cuda.current_stream().cuda_stream

    def make_device(self, index, info, model, kd, opts):
        import chiaroscuro_amd as ca
        dev = ca.Device(index)
        for key, val in opts:
            dev.set_option(key, val)
        dev.upload(kd.describe())
        return dev


def load_backend():
    spec = os.environ.get("CHIARO_BENCH_BACKEND")
    if not spec:
        return GpuBackend()
    import importlib.util
    path, _, attr = spec.rpartition(":")
    mod_spec = importlib.util.spec_from_file_location("chiaro_bench_backend", path)
    mod = importlib.util.module_from_spec(mod_spec)
    mod_spec.loader.exec_module(mod)
    return getattr(mod, attr)()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (= rank processes) of one node, default 1")
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="sponza", help="cornell | cornell_box | sponza | sponza_4k")
    ap.add_argument("--spp", type=int, default=0, help="override samples per step (default: config's)")
    ap.add_argument("--kernel", type=int, default=-1,
                    help="2 wavefront (the only render kernel; the megakernel and thread-per-pixel kernels were removed)")
    ap.add_argument("--variant", type=int, default=-1, help="kernel build variant (default: the kernel's)")
    ap.add_argument("--gather", default="torch", choices=("torch", "cabi"),
                    help="N > 1: tile gather by torch.distributed (default) or the library's own RCCL "
                         "communicator (cr_comm_init / cr_render_dist_device)")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                    help="cr_set_option before the scene upload (experiments; the default build is timed without)")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-perf-pass", action="store_true",
                    help="skip the untimed performed-work pass (profiling runs: its kernels are not the timed ones)")
    ap.add_argument("--layers-per-pass", type=int, default=32,
                    help="progressive layers per render pass group (DistributedFrame.plan_layers; 1 = one per pass)")
    ap.add_argument("--res", default="", help="WxH override of the config's frame (tests, experiments)")
    ap.add_argument("--save-frame", default="", help="rank 0 writes the final accumulated frame (.npy)")
    ap.add_argument("--single-layer-steps", type=int, default=2,
                    help="after the timed steps: this many one-layer passes (+1 warmup), reported as single_layer_ms")
    ap.add_argument("--dist-timeout", type=float, default=120.0,
                    help="N > 1: seconds one collective may stay in flight before every rank exits non-zero with "
                         "its rank, device, pass group and the collective (DistWatch)")
    ap.add_argument("--parity-rows", type=int, default=8,
                    help="rank 0 checks this many rows of the timed frame (every layer, full spp) bit for bit "
                         "against the oracle after the timed region (0: skip)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(spawn_ranks(args.gpus))
    if args.gpus is not None and args.gpus != world:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    out = run_rank(args, world, load_backend())
    if out is not None:
        print(json.dumps(out), flush=True)


def run_rank(args, world, backend):
    """One rank of the benchmark (the whole job when world == 1); returns the JSON
    object on rank 0, None elsewhere."""
    import torch

    import chiaroscuro_amd as ca
    from chiaroscuro_amd import scenes
    from chiaroscuro_amd.tiles import DistributedFrame

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    watch = None
    if world > 1:
        watch = DistWatch(rank, "%s:%d" % (backend.device, local), args.dist_timeout)
        watch.phase = "init_process_group"
        dist = backend.init_rank(world, local, args.dist_timeout)
        dist = WatchedDist(dist, watch)
        watch.phase = "scene load"
    else:
        dist = backend.init_rank(world, local)
    if dist is not None:
        assert dist.get_world_size() == world, (dist.get_world_size(), world)
        if rank == 0:
            ver = backend.collectives_version() if hasattr(backend, "collectives_version") else "n/a"
            log("bench: world size %d, backend %s, %s, collective timeout %.0f s" %
                (dist.get_world_size(), dist.get_backend(), ver, args.dist_timeout))

    rtc = scenes.config_rtc(args.config)
    t0 = time.time()
    scene = ca.Scene(rtc, *(("xres", args.res.split("x")[0], "yres", args.res.split("x")[1]) if args.res else ()))
    info = scene.info
    model = ca.Model(scene)
    tex_bytes = sum(len(a) for *_, a in model.textures())  # the scene's texels (a11: getColorAt reads them)
    kd = ca.KDTree(model, scene)
    opts = [(kv.split("=", 1)[0], int(kv.split("=", 1)[1], 0)) for kv in args.opt]
    dev = backend.make_device(local, info, model, kd, opts)
    if args.kernel >= 0:
        dev.set_option("kernel", args.kernel)
    if args.variant >= 0:
        dev.set_option("variant", args.variant)
    if rank == 0:
        log("scene %s: %d tris, load+kd+upload %.1fs" % (args.config, model.num_triangles, time.time() - t0))
    xres, yres, k, seed = info["xres"], info["yres"], info["k"], info["seed"]
    spp = args.spp or info["samples"]
    cam = ca.camera(info["VP"], info["LA"], info["UP"], info["yview"], xres, yres)
    tile = 32
    stream = backend.stream()
    fr = DistributedFrame(dev, xres, yres, rank, world, tile, dist, device=backend.device, gather=args.gather)

    totals = {"rays": 0, "nee_answered": 0, "kernel_ms": 0.0, "bytes": 0, "launches": 0, "tritest": 0, "px": 0,
              "trace_ms": [0.0] * 4, "trace_launches": [0] * 4}
    wavefront = args.kernel in (-1, 2)

    # layers per render pass: up to --layers-per-pass progressive layers are rendered as one
    # pass group -- each pass holds the paths of all of them for a share of the frame (a rank's
    # tiles; on one GPU the frame is cut into the fewest tile-split pieces whose paths fit one
    # chunk), so the per-pass latency-bound generation ends are paid once per group and each
    # pass traces several layers' samples of a smaller screen region (more coherent, L2-resident
    # work); bit-identical to one layer per pass (tests/test_gpu_parity.py)
    dev.set_option("counters", 0)  # (the timed, lean build: the counting build renders one layer per pass)
    p1 = ca.render_params(xres, yres, spp, k, seed, layer=1, rank=rank, nranks=world, tile=tile)
    nl_pass, _ = fr.plan_layers(p1, args.layers_per_pass)  # (every rank the same: plan_layers agrees)
    fr.reserve(min(nl_pass, args.steps))  # (the timed group's gather buffers, allocated before the clock)
    groups = []

    def step(layer, n, record):
        """Layers layer .. layer + n - 1 (n <= nl_pass) as one pass group."""
        if watch:
            watch.group = "layers %d..%d" % (layer, layer + n - 1)
            watch.phase = "render"
        stall = os.environ.get("CHIARO_TEST_STALL_RANK")  # (tests: this rank stalls before its first timed group)
        if stall is not None and int(stall) == rank and record and not groups:
            time.sleep(float(os.environ.get("CHIARO_TEST_STALL_S", "60")))
        p = ca.render_params(xres, yres, spp, k, seed, layer=layer, rank=rank, nranks=world, tile=tile)
        tp = time.perf_counter()
        n, pieces = fr.plan_layers(p, n)  # (with several ranks: agreed by an all-reduce MIN)
        if rank == 0:
            log("group of %d layers in %d pieces (plan %.1f ms)" % (n, pieces, (time.perf_counter() - tp) * 1e3))
        if n == 1 and pieces == 1:
            fr.render_layer(cam, p, stream)
        else:
            fr.render_layers(cam, p, n, stream, pieces=pieces)
        if record:
            groups.append((n, pieces))
            st = fr.last_stats()
            c = st["counters"]
            totals["rays"] += c["closest"] + c["shadow"]
            totals["nee_answered"] += c.get("nee_answered", 0)
            totals["kernel_ms"] += st["kernel_ms"]
            totals["px"] += c["pixels"]
            totals["launches"] += n  # layers: kernel_ms / launches is the render time per layer
            if wavefront and st["trace"]:
                for i, kind in enumerate(ca.TRACE_KINDS):
                    totals["trace_ms"][i] += st["trace"][kind]["ms"]
                    totals["trace_launches"][i] += st["trace"][kind]["launches"]
        return n

    # Timed launches count only rays; the node/leaf/triangle counters of SURVEY §8d
    # (algorithmic bytes) come from one extra, untimed launch of the counting
    # variant on the first timed layer (results are deterministic per layer).
    dev.set_option("counters", 0)
    layer = 1
    first_timed = args.warmup + 1
    w = 0
    while w < args.warmup:
        n = step(layer, min(nl_pass, args.warmup - w), False)
        layer += n
        w += n
        if rank == 0:
            log("warmup %d done" % w)
    if dist:
        dist.barrier()
    backend.synchronize()
    t0 = time.perf_counter()
    s = 0
    while s < args.steps:
        n = step(layer, min(nl_pass, args.steps - s), True)
        layer += n
        s += n
        if rank == 0:
            log("step %d: %.3fs elapsed" % (s, time.perf_counter() - t0))
    backend.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if watch:
        watch.group, watch.phase = "after the timed groups", "single-layer passes"
    timed_build = dev.last_trace_build() if hasattr(dev, "last_trace_build") else None
    nlayers_done = layer - 1  # the frame holds layers 1 .. nlayers_done (warmup and timed groups)
    # rows of the timed frame for the parity check (rank 0; the oracle runs after the collectives)
    prows = parity_rows(yres, args.parity_rows) if args.parity_rows > 0 else []
    frame_rows = fr.frame[prows].cpu().numpy() if (prows and fr.frame is not None) else None
    if args.save_frame and fr.frame is not None:
        import numpy as np
        np.save(args.save_frame, fr.frame.cpu().numpy())
    # the reference's unit of work, untimed by the line's value: one rayTrace call = ONE layer per
    # render pass (main.cpp:16, the preview's R key) -- a warmup pass, then --single-layer-steps passes
    # of the next layers (the frame's rows above are already taken), each bracketed like the steps
    single_ms = None
    single_rays = 0.0
    if args.single_layer_steps > 0:
        times = []
        srays = []
        for j in range(args.single_layer_steps + 1):
            p = ca.render_params(xres, yres, spp, k, seed, layer=layer + j, rank=rank, nranks=world, tile=tile)
            if dist:
                dist.barrier()
            backend.synchronize()
            ts = time.perf_counter()
            fr.render_layer(cam, p, stream)
            backend.synchronize()
            if dist:
                dist.barrier()
            if j:
                times.append((time.perf_counter() - ts) * 1e3)
                c = fr.last_stats()["counters"]
                srays.append(c.get("closest", 0) + c.get("shadow", 0))
        single_ms = sum(times) / len(times)
        single_rays = sum(srays) / len(srays)
    # per rank: wall time, device time of its render passes (HIP events), rays
    mine = torch.tensor([elapsed, totals["kernel_ms"] / max(totals["launches"], 1), totals["rays"],
                         totals["nee_answered"], single_rays], dtype=torch.float64, device=backend.device)
    if dist:
        per_rank = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(per_rank, mine)
        per_rank = torch.stack(per_rank).cpu().tolist()
    else:
        per_rank = [mine.cpu().tolist()]
    elapsed = max(r[0] for r in per_rank)   # the step ends with the slowest rank
    rays_all = float(sum(r[2] for r in per_rank))
    nee_all = float(sum(r[3] for r in per_rank))
    single_rays_all = float(sum(r[4] for r in per_rank))  # one layer's rays over every rank's tiles
    rank_render_ms = [round(r[1], 3) for r in per_rank]

    # counting pass (untimed): algorithmic bytes of one launch of this rank
    if watch:
        watch.phase = "counting and performed-work passes"
    dev.set_option("counters", 1)
    pc = ca.render_params(xres, yres, spp, k, seed, layer=first_timed, rank=rank, nranks=world, tile=tile)
    scratch = torch.zeros((yres, xres, 3), dtype=torch.float32, device=backend.device)
    if world == 1:
        dev.render_device(cam, pc, scratch.data_ptr(), stream)
    else:
        scratch_tiles = torch.zeros((fr.layout.max_tiles, tile, tile, 3), dtype=torch.float32, device=backend.device)
        dev.render_tiles_device(cam, pc, scratch_tiles.data_ptr(), stream)
    cc = dev.counters()
    cts = dev.trace_stats() if wavefront else None
    totals["bytes"] = ca.algorithmic_bytes(cc, cc["pixels"])
    totals["tritest"] = cc["tritest"]
    totals["texhit"] = cc["texhit"]
    totals["count_rays"] = cc["closest"] + cc["shadow"]
    dev.set_option("counters", 0)
    # performed-work pass (untimed): the default trace build's kernels with counters of what they
    # actually execute and load (cr_get_perf), the same layer
    perf = None
    if wavefront and args.variant in (-1, 18, 26, 40, 42, 43, 44, 49, 53, 54, 59) and hasattr(dev, "perf") and not args.no_perf_pass:
        dev.set_option("perf_counters", 1)
        if world == 1:
            dev.render_device(cam, pc, scratch.data_ptr(), stream)
        else:
            dev.render_tiles_device(cam, pc, scratch_tiles.data_ptr(), stream)
        perf = dev.perf()
        dev.set_option("perf_counters", 0)

    out = None
    if rank == 0:
        value = rays_all / elapsed / 1e6
        # the queries actually traversed: value less the zero-contribution NEE queries answered without
        # a trace (rayTracer.cpp:104 issues every one; SURVEY §8d counts them, the line says how many)
        value_traced = (rays_all - nee_all) / elapsed / 1e6
        kms = totals["kernel_ms"] / max(totals["launches"], 1)
        pass_bytes = totals["bytes"]  # counting pass: one render pass, same size as a timed one
        pass_gbs = pass_bytes / (kms / 1e3) / 1e9 if kms > 0 else 0.0
        # measured fabric bytes from the committed rocprofv3 PMC summary of this same
        # configuration (scripts/prof_summary.py); null if none
        pj = None
        pmc = ROOT / "profiles" / ("pmc_%s.json" % args.config)
        if pmc.exists():
            try:
                pj = json.loads(pmc.read_text())
                if not (pj.get("spp") == spp and pj.get("n_gpus") == world):
                    pj = None
            except Exception:
                pj = None
        kernel_name = "wavefront"
        cpu = None
        parity = None
        osc = None
        if frame_rows is not None or (not args.no_cpu_baseline and world == 1):
            osc = oracle_scene(model, info["leaf_size"])
        if frame_rows is not None:
            parity = frame_parity(osc, frame_rows, prows, cam.as_array(), xres, yres, spp, k, seed, nlayers_done)
            parity["trace_build"] = timed_build
            log("parity: %d of %d values differ over rows %s x %d layers (oracle %.1fs)" % (
                parity["differing"], parity["values"], parity["rows"], nlayers_done, parity["oracle_s"]))
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(osc, cam.as_array(), xres, yres, spp, k, seed, args.cpu_budget)
        # the pass: its measured fabric (HBM) bytes over its time is north_star's "rocprof HBM GB/s";
        # the SURVEY §8d bytes of the reference algorithm's work over the same time are a
        # reference-equivalent rate (the culls skip most of that work), not a performed one
        fabric = pj.get("hbm_bytes_per_launch") if pj else None
        perf_bytes = sum(v["vbytes"] + v["sbytes"] for v in perf.values()) if perf else None
        pass_view = {"kernels": "render pass (%s): all kernels of one layer" % kernel_name, "ms": round(kms, 3),
                     "achieved": round(fabric / (kms / 1e3) / 1e9, 2) if fabric and kms > 0 else None,
                     "achieved_is": "measured fabric (HBM) GB/s: rocprofv3 PMC bytes of one pass (profiles/pmc_%s.json) "
                                    "over this run's pass time" % args.config,
                     "peak": HBM_PEAK_GBS, "frac_of_hbm": round(fabric / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                     if fabric and kms > 0 else None,
                     "traffic": fabric,
                     "bytes": {"reference_equivalent": int(pass_bytes),
                               "trace_performed": int(perf_bytes) if perf_bytes is not None else None,
                               "fabric": fabric},
                     "reference_equivalent_gbs": round(pass_gbs, 2),
                     "trace_performed_gbs": round(perf_bytes / (kms / 1e3) / 1e9, 2) if perf_bytes and kms > 0 else None}
        if wavefront:
            # Per trace kind (camera = generation-1 closest queries, closest = later generations,
            # shadow): algorithmic bytes (8 per inner node, 8 per leaf, 40 per triangle test)
            # per kind from the counting pass; launch times from HIP event pairs around every
            # launch of the timed passes, on the launch's stream.
            def kind_view(kind):
                i = ca.TRACE_KINDS.index(kind)
                launches = totals["trace_launches"][i]
                if not launches:
                    return None
                avg_ms = totals["trace_ms"][i] / launches
                per_pass = launches / max(totals["launches"], 1)
                t = cts[kind]
                kb = (8 * t["inner"] + 8 * t["leaf"] + 40 * t["tritest"]) / max(per_pass, 1e-9)
                tr = (pj or {}).get("trace", {}).get(kind)
                pf = (perf or {}).get(kind)
                pb = (pf["vbytes"] + pf["sbytes"]) / max(per_pass, 1e-9) if pf else None
                sec = avg_ms / 1e3
                fab = tr["fabric_bytes_per_launch"] if tr else None
                return {"kernel": "wf_trace<%s>" % kind, "avg_launch_ms": round(avg_ms, 3), "launches": launches,
                        "algorithmic_bytes_per_launch": int(kb),
                        "work_per_launch": {w: int(t[w] / max(per_pass, 1e-9)) for w in ("inner", "leaf", "tritest")},
                        # performed: the bytes the default build's loads and stores move (cr_get_perf);
                        # reference_equivalent: SURVEY §8d bytes of the reference algorithm's work
                        "bytes_per_launch": {"performed": int(pb) if pb is not None else None,
                                             "performed_vector": int(pf["vbytes"] / max(per_pass, 1e-9)) if pf else None,
                                             "performed_scalar": int(pf["sbytes"] / max(per_pass, 1e-9)) if pf else None,
                                             "reference_equivalent": int(kb), "fabric": fab},
                        "performed_work_per_launch": {w: int(pf[w] / max(per_pass, 1e-9))
                                                      for w in ("queries", "steps", "leaves", "masks", "tests")}
                        if pf else None,
                        "achieved": round(pb / sec / 1e9, 2) if pb is not None and sec > 0 else None,
                        "achieved_is": "performed bytes per launch / live launch time",
                        "reference_equivalent_gbs": round(kb / sec / 1e9, 2) if sec > 0 else 0.0,
                        "fabric_gbs": round(fab / sec / 1e9, 2) if fab and sec > 0 else None,
                        "traffic": fab,
                        "rocprof_avg_launch_ms": round(tr["avg_ns"] / 1e6, 3) if tr else None}
            views = {k: kind_view(k) for k in ("camera", "closest", "shadow")}
            # what bounds the trace kernels instead of HBM: instruction issue (committed
            # scripts/pmc_issue.sh summary of this configuration, per lean trace kind)
            issue = None
            pi = ROOT / "profiles" / ("pmc_issue_%s.json" % args.config)
            if pi.exists():
                try:
                    ij = json.loads(pi.read_text())
                    if ij.get("spp") == spp:
                        issue = ij.get("kinds")
                except Exception:
                    issue = None
            # Dominant kernel: the trace kind with the most kernel time per pass.  Closest traces of
            # generation >= 2 run beside a shadow trace on a second stream, so their live event
            # times include the other kernel's share of the GPU; the ranking therefore uses the
            # standalone durations of the committed PMC pass (rocprofv3 serializes kernels there)
            # when it exists, else the live times.  (Sponza stand-in, build 15: shadow 249 ms,
            # camera 70, closest 69 per pass -- the shadow trace, whose live time equals its
            # standalone one: it is launched first and owns the GPU.)
            def per_pass_ms(kind):
                k = (issue or {}).get(kind)
                if k and k.get("avg_launch_ms") and k.get("dispatches"):
                    return k["avg_launch_ms"] * k["dispatches"], "standalone"
                v = views.get(kind)
                return ((v["avg_launch_ms"] * v["launches"] / max(totals["launches"], 1)) if v else 0.0), "live"
            ranked = {k: per_pass_ms(k) for k in ("camera", "closest", "shadow") if views.get(k)}
        if wavefront and ranked:
            dom_kind = max(ranked, key=lambda k: ranked[k][0])
            dom = views[dom_kind]
            roofline = issue_roofline(dom, (issue or {}).get(dom_kind), views, issue, pass_view, dom_kind)
            roofline["dominant_by"] = {k: {"ms_per_pass": round(v[0], 3), "from": v[1]} for k, v in ranked.items()}
        else:  # (no per-kind trace launches: the other kernels, or a backend without them)
            ach = pass_view["achieved"] if pass_view["achieved"] is not None else round(pass_gbs, 2)
            roofline = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": pass_view["traffic"],
                        "kernel": pass_view["kernels"], "kernel_ms": round(kms, 3),
                        "algorithmic_bytes_per_launch": int(pass_bytes)}
        label = {"sponza": "sponza_standin (Sponza-Crytek stand-in, ~261k tris) 1920x1080",
                 "sponza_4k": "sponza_standin (Sponza-Crytek stand-in) 3840x2160",
                 "nanobox": "nanobox_standin (textured nanosuit-in-a-box stand-in, ~19k tris, the asset's 21 MB texture set) 1920x1080",
                 "cornell": "cornell_unit 256x256", "cornell_box": "cornell_box_lit 1024x1024"}[args.config]
        out = {
            "metric": "Mray/s (primary+secondary) on sponza_crytek 1080p; 1/2/4/8-GPU scaling",
            "value": round(value, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            # the same layer as ONE render pass (the reference's unit of work: one rayTrace call), wall
            # time per pass after the timed region; value and ms_per_step time the pass groups
            "single_layer_ms": round(single_ms, 3) if single_ms is not None else None,
            # one layer's rays / single_layer_ms: the rate of one rayTrace call (main.cpp:16)
            "single_layer_mray_s": round(single_rays_all / (single_ms / 1e3) / 1e6, 3) if single_ms else None,
            # (rays - rays_answered_untraced) / the same wall time: the traversed queries' rate
            "value_traced": round(value_traced, 3),
            "higher_is_better": True,
            "scaling": "strong",  # one fixed frame, tile-split over the ranks
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic scene (deterministic generator), seeded counter RNG",
            "config": {"workload": label, "spp_per_step": spp, "k": k, "tile": tile,
                       "parallelism": "tile-split x%d" % world, "gather": args.gather if world > 1 else None,
                       "rays": int(rays_all),
                       # of those, NEE shadow queries whose contribution is exactly zero, answered without a
                       # traversal (wf_nee_skip; the image cannot change) -- counted as the reference traces them
                       "rays_answered_untraced": int(nee_all),
                       "rank_render_ms": rank_render_ms, "layers_per_pass": nl_pass,
                       "pass_groups": [list(g) for g in groups], "trace_build": timed_build,
                       "mean_tritest_per_ray": round(totals["tritest"] / max(totals["count_rays"], 1), 2),
                       # textured hits of one layer (counting pass; 3 texel bytes each in SURVEY §8d's bytes)
                       # and the scene's texture bytes (src/mesh.cpp:21-35 reads them)
                       "texhit_per_layer": int(totals["texhit"]), "texhit_bytes_per_layer": 3 * int(totals["texhit"]),
                       "texture_bytes": int(tex_bytes)},
            "roofline": roofline,
            "cpu_baseline": cpu,
            # value over the CPU baseline: the timed 16-thread share of the box, and the whole host's
            # physical cores projected linearly from the 1-thread leg (an upper bound for the CPU)
            "vs_cpu": {"share": round(value / cpu["value"], 1) if cpu and cpu.get("value") else None,
                       "all_physical_projected": round(value / cpu["projected_all_physical"], 1)
                       if cpu and cpu.get("projected_all_physical") else None,
                       "traced_share": round(value_traced / cpu["value"], 1) if cpu and cpu.get("value") else None}
            if cpu else None,
            "parity": parity,
        }
        if backend.name != "gpu":
            out["backend"] = backend.name
    if dist:
        dist.destroy_process_group()
    return out if rank == 0 else None


if __name__ == "__main__":
    main()
