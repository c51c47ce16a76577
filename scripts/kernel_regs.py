"""Register use, spills and LDS of the device kernels in a built object (gfx950 code-object notes).
    python scripts/kernel_regs.py [chiaroscuro-raytracer_amd/build/wavefront.o] [name-filter]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def notes(obj):
    with tempfile.TemporaryDirectory() as td:
        fat, dev = os.path.join(td, "fat"), os.path.join(td, "dev")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(td, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], check=True,
                       capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-readelf", "--notes", dev], check=True, capture_output=True,
                              text=True).stdout


def kernels(obj):
    out = []
    for b in notes(obj).split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", b).group(1)
        get = lambda k: int((re.search(r"\." + k + r":\s+(\d+)", b) or [0, 0])[1])
        out.append({"name": name, "vgpr": get("vgpr_count"), "sgpr": get("sgpr_count"),
                    "vgpr_spill": get("vgpr_spill_count"), "sgpr_spill": get("sgpr_spill_count"),
                    "lds": get("group_segment_fixed_size"), "scratch": get("private_segment_fixed_size")})
    return out


if __name__ == "__main__":
    obj = sys.argv[1] if len(sys.argv) > 1 else "chiaroscuro-raytracer_amd/build/wavefront.o"
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    for k in kernels(obj):
        if flt in k["name"]:
            print(f'{k["name"][:72]:72s} vgpr {k["vgpr"]:3d} sgpr {k["sgpr"]:3d} vspill {k["vgpr_spill"]:3d} '
                  f'sspill {k["sgpr_spill"]:3d} lds {k["lds"]:5d} scratch {k["scratch"]}')
