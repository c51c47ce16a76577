"""Kernel-name classification shared by the profile summaries (rocprofv3 kernel names).

The trace kernels are wf_trace<C> with C a build configuration of csrc/wavefront.hip's namespace
tc: named types for the compiled-by-default builds (cr::tc::ShadowFatLcFd, cr::tc::ClosestCount,
cr::tc::ClosestFatLcPerf, ...) and cr::tc::Cfg<SHADOW, R, MINW, SC, FD, FAT, PF, CAM, ...> for the
ALL_VARIANTS ones; the camera packet is wf_trace_packet<R, S, PC, FD>; the tail wf_tail<FULL, ...>.
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
    if t == "Cfg":  # Cfg<SHADOW, R, MINW, SC, FD, FAT, PF, CAM, ...> (ALL_VARIANTS builds, all lean)
        a = [x.strip() for x in re.search(r"Cfg<([^>]*)>", name).group(1).split(",")]
        return ("shadow" if a[0] == "true" else ("camera" if a[7] == "true" else "closest")), "lean"
    kind = "shadow" if t.startswith("Shadow") else ("camera" if t.startswith("Camera") else "closest")
    mode = "counting" if t.endswith("Count") else ("perf" if t.endswith("Perf") else "lean")
    return kind, mode


def is_counting(name: str) -> bool:
    """The counting and performed-work instances (not timed kernels)."""
    if re.search(r"render_dynamic<\w+, true,", name):
        return True
    info = trace_info(name)
    return info is not None and info[1] != "lean"


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("cr::", "")
    info = trace_info(name)
    if info and info[0] != "tail":
        return "%s%s %s" % (info[0], "" if info[1] == "lean" else "(%s)" % info[1], n[:60])
    return n[:70]
