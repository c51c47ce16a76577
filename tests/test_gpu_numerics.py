"""GPU check of the exact short division sequences the kernels use instead of
the full IEEE division (device_math.hpp rcp_rn / div_by_rcp): every float for
the reciprocal, 2^30 random and near-midpoint pairs for the split distance.
Both must give bit-for-bit the correctly rounded quotient the reference's float
division gives, or the kd descent / triangle test would drift from it.  And the
kernels' sinf / cosf (cr_sincosf, glibc's algorithm) against the host libm
the reference links, on every float in [-2pi, 2pi] (src/brdf.cpp:52-53)."""
import json
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.gpu
def test_fast_division_is_exact(tmp_path):
    exe = tmp_path / "numerics_check"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fopenmp",
                    "-I", str(ROOT / "chiaroscuro-raytracer_amd" / "csrc"), "-I", str(ROOT / "include"),
                    str(ROOT / "tests" / "native" / "numerics_check.hip"), "-o", str(exe)],
                   check=True, capture_output=True, timeout=300)
    r = subprocess.run([str(exe), "64"], capture_output=True, text=True, timeout=300)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(res)
    assert res["rcp_mismatch"] == 0, res
    assert res["div_mismatch"] == 0, res
    assert res["sincos_mismatch"] == 0 and res["sincos_tested"] > 2 * 10 ** 9, res
    assert res["div_fast_path"] > res["div_pairs"] // 4, res  # the short path is actually exercised
    assert r.returncode == 0
