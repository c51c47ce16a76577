"""Kernel-name classification shared by the profile summaries (rocprofv3 kernel names).

The trace kernels are wf_trace<C> with C a build configuration of csrc/wavefront.hip's namespace
tc (cr::tc::ShadowFatLc5Fd, cr::tc::ClosestCount, cr::tc::ClosestFatLc5Perf, ...); the camera packet
is wf_trace_packet<R, S, PC, FD>; the tail wf_tail<FULL, ...>.
"""
import re


def trace_info(name: str):
    """(kind, mode) of a trace kernel: kind "camera" | "closest" | "shadow" | "tail", mode "lean" |
    "counting" | "perf"; None for other kernels."""
    if "wf_trace_packet" in name:
        m = re.search(r"wf_trace_packet<\d+, \d+, (true|false)", name)
        return "camera", ("perf" if m and m.group(1) == "true" else "lean")
    if "wf_tail" in name:
        if "wf_tail<true" in name:
            return "tail", "counting"
        return "tail", ("perf" if re.search(r"wf_tail<[^()]*, true>\(", name) else "lean")
    m = re.search(r"wf_trace<cr::tc::(\w+)", name)
    if not m:
        return None
    t = m.group(1)
    kind = "shadow" if t.startswith("Shadow") else ("camera" if t.startswith("Camera") else "closest")
    mode = "counting" if t.endswith("Count") else ("perf" if t.endswith("Perf") else "lean")
    return kind, mode


def is_counting(name: str) -> bool:
    """The counting and performed-work instances (not timed kernels)."""
    info = trace_info(name)
    return info is not None and info[1] != "lean"


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("cr::", "")
    info = trace_info(name)
    if info and info[0] != "tail":
        return "%s%s %s" % (info[0], "" if info[1] == "lean" else "(%s)" % info[1], n[:60])
    return n[:70]
