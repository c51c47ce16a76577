"""No scalar-load hazard in the built device code (scripts/smem_hazard.py).

Every instruction that touches a scalar load's destination before the load's
s_waitcnt lgkmcnt(0) is a timing-dependent corruption: it showed as a full-size
only illegal address (the grandchild-prefetch packet build, wavefront.hip kWf 48)
while the small parity renders passed.  CPU only: disassembles build/*.o.
"""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import smem_hazard  # noqa: E402

OBJS = sorted(glob.glob(os.path.join(ROOT, "chiaroscuro-raytracer_amd", "build", "*.o")))
HAVE_TOOLS = os.path.exists(os.path.join(smem_hazard.LLVM, "clang-offload-bundler"))


@pytest.mark.skipif(not OBJS or not HAVE_TOOLS, reason="device objects or ROCm LLVM tools absent")
def test_built_device_code_has_no_scalar_load_hazard():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "smem_hazard.py")] + OBJS,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "wavefront.o: 0 scalar-load hazards" in r.stdout


def test_scan_flags_base_inside_pending_destination():
    # the allocation the SPEC packet build got without early-clobber outputs
    bad = """
f:
	s_load_dwordx8 s[36:43], s[8:9], s0
	s_load_dwordx4 s[8:11], s[38:39], s1
	s_waitcnt lgkmcnt(0)
"""
    good = """
f:
	s_load_dwordx8 s[36:43], s[8:9], s0
	s_load_dwordx4 s[44:47], s[10:11], s1
	s_waitcnt lgkmcnt(0)
	s_add_u32 s2, s36, s44
"""
    assert len(smem_hazard.scan(bad)) == 1
    assert smem_hazard.scan(good) == []
