#!/usr/bin/env python3
"""Scalar-load hazard scan of the gfx950 code objects in the built device objects.

A scalar memory load (s_load_*) writes its destination SGPRs whenever the data
returns; nothing may read or write those registers before an s_waitcnt
lgkmcnt(0).  Compiler-generated code always obeys that; a hand-written asm block
with several loads can break it when its outputs are not early-clobber: the
register allocator may then give a later load's base address the registers an
earlier load is filling (traverse.hpp's scalar-load helpers; the full-size-only
illegal address of the grandchild-prefetch packet builds was exactly this).

    python3 scripts/smem_hazard.py [objects...]   (default: the in-tree build/*.o)

Prints every hazard and exits 1 when there is one.  CPU only: it disassembles
the gfx950 half of each object's offload bundle with the ROCm LLVM tools.
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_RANGE = re.compile(r"\bs\[(\d+):(\d+)\]")
_ONE = re.compile(r"\bs(\d+)\b")


def _regs(text):
    out = set()
    for a, b in _RANGE.findall(text):
        out.update(range(int(a), int(b) + 1))
    out.update(int(r) for r in _ONE.findall(_RANGE.sub("", text)))
    return out


def disassemble(obj):
    """gfx950 disassembly of one host object's .hip_fatbin bundle."""
    with tempfile.TemporaryDirectory() as td:
        fat, dev = os.path.join(td, "fat"), os.path.join(td, "dev")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(td, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        f"--targets={TARGET}", f"--output={dev}"], check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", "--no-leading-addr", dev],
                              check=True, capture_output=True, text=True).stdout


def scan(text):
    """[(function, load, offending instruction)] for every use of a pending scalar-load destination."""
    bad, fn, pending, last = [], None, set(), {}
    for raw in text.splitlines():
        line = raw.split("//")[0].strip()
        m = re.match(r"^<?([\w.$]+)>?:$", line) or re.match(r"^[0-9a-f]+ <([\w.$]+)>:$", line)
        if m:
            fn, pending, last = m.group(1), set(), {}
            continue
        if not line or line.startswith((";", ".")):
            continue
        op, _, args = line.partition(" ")
        args = args.split(";")[0]
        if op.startswith("s_waitcnt"):
            if "lgkmcnt(0)" in args or args.strip() in ("0", "") or "lgkmcnt" not in args and "vmcnt" not in args:
                pending, last = set(), {}
            continue
        if op.startswith("s_endpgm") or op.startswith("s_branch") or op.startswith("s_cbranch") or op.startswith("s_setpc"):
            pending, last = set(), {}
            continue
        ops = [a.strip() for a in args.split(",")] if args.strip() else []
        if op.startswith("s_load") or op.startswith("s_buffer_load"):
            dst, src = _regs(ops[0]) if ops else set(), _regs(",".join(ops[1:]))
            hit = (src | dst) & pending
            if hit:
                bad.append((fn, last.get(min(hit), "?"), line))
            pending |= dst
            for r in dst:
                last[r] = line
            continue
        used = _regs(args) & pending
        if used:
            bad.append((fn, last.get(min(used), "?"), line))
            pending -= used
    return bad


def main(argv):
    objs = argv or sorted(glob.glob(os.path.join(ROOT, "chiaroscuro-raytracer_amd", "build", "*.o")))
    total = 0
    for obj in objs:
        try:
            text = disassemble(obj)
        except subprocess.CalledProcessError:
            continue  # host-only object: no offload bundle
        bad = scan(text)
        total += len(bad)
        for fn, load, ins in bad[:20]:
            print(f"{os.path.basename(obj)}: {fn}: '{ins}' uses a register of pending '{load}'")
        print(f"{os.path.basename(obj)}: {len(bad)} scalar-load hazards")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
