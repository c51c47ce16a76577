"""Full-size parity of every bench configuration: bench.py's own timed path (the lean default trace
build, pass groups, frame pieces) at the configuration's full frame and spp, compared with the oracle on
whole rows, bit for bit.

The other GPU tests render small frames (<= 160 x 90); the driver's bench checks 8 rows of the sponza
frame.  Here each configuration of SURVEY.md section 6 (chiaroscuro_amd.scenes.CONFIGS) -- C1 cornell
256^2 x 4 spp, C2 cornell_box 1024^2 x 500 spp, C3 nanobox stand-in 1080p x 64 spp, the headline sponza
stand-in 1080p x 128 spp and C5 sponza 4K x 100 spp -- runs bench.py in a child process for two timed layers, and the frame's first, middle and
last rows after both layers must equal the oracle's blend of the same layers (bench.frame_parity:
or_render_pixels per layer, blended as src/rayTracer.cpp:64 does)."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("config", ["cornell", "cornell_box", "nanobox", "sponza", "sponza_4k"])
def test_bench_config_full_size_rows_bitexact(config):
    cmd = [sys.executable, "-u", str(ROOT / "bench.py"), "--config", config, "--steps", "2", "--warmup", "0",
           "--parity-rows", "3", "--no-cpu-baseline", "--no-perf-pass", "--single-layer-steps", "0"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    par = d["parity"]
    assert par["layers"] == 2 and len(par["rows"]) == 3
    assert par["values"] == 3 * 3 * int(d["config"]["workload"].split()[-1].split("x")[0])
    assert par["differing"] == 0, par
    assert d["value"] > 0 and d["config"]["rays"] > 0
