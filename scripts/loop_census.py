"""Instruction census of the loops of one kernel in a hipcc -S listing.
    python scripts/loop_census.py file.s kernel_symbol_substring
For every loop header label, counts VALU / SALU / VMEM / SMEM / LDS / branch
instructions between the header and the last branch back to it (rarely taken
blocks inside that span are included, so this is an upper bound per iteration).
"""
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_") and sym in l and l.rstrip().endswith(":") or
                 (l.startswith("_") and sym in l.split(":")[0] and ":" in l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    headers = [(i, l.split(":")[0]) for i, l in enumerate(body)
               if l.startswith(".LBB") and ("Loop Header" in l or (i + 1 < len(body) and "Loop Header" in body[i + 1]
                                                                   and not body[i + 1].startswith(".")))]
    pos = {l.split(":")[0]: i for i, l in enumerate(body) if l.startswith(".LBB")}
    for i, lab in headers:
        # back edge: the last branch below the header to the header or to a latch
        # block just above it that falls through into the header
        last, top = None, i
        for j in range(i + 1, len(body)):
            m = re.search(r"s_(?:c)?branch\w*\s+(\.LBB\w+)", body[j])
            if m and m.group(1) in pos and i - 60 <= pos[m.group(1)] <= i:
                last, top = j, min(top, pos[m.group(1)])
        if last is None:
            continue
        i = top
        cnt = {"valu": 0, "vmov": 0, "salu": 0, "vmem": 0, "smem": 0, "lds": 0, "branch": 0, "wait": 0}
        for l in body[i:last + 1]:
            t = l.strip().split()
            if not t or t[0].startswith(";") or t[0].startswith("."):
                continue
            op = t[0]
            if op.startswith("v_"):
                cnt["valu"] += 1
                cnt["vmov"] += op.startswith("v_mov")
            elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
                cnt["vmem"] += 1
            elif op.startswith("s_load") or op.startswith("s_buffer_load"):
                cnt["smem"] += 1
            elif op.startswith("ds_"):
                cnt["lds"] += 1
            elif op.startswith("s_waitcnt"):
                cnt["wait"] += 1
            elif op.startswith(("s_cbranch", "s_branch")):
                cnt["branch"] += 1
            elif op.startswith("s_"):
                cnt["salu"] += 1
        depth = re.search(r"Header: Depth=(\d+)", body[i] + (body[i + 1] if i + 1 < len(body) else ""))
        print("%-10s depth %s lines %4d  %s" % (lab, depth.group(1) if depth else "?", last - i, cnt))


if __name__ == "__main__":
    main()
