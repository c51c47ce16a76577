"""chiaroscuro_amd -- Python side of the MI355X path-tracing core.

Thin ctypes bindings over the two in-tree shared libraries:

* ``lib/libchiaro_hip.so``  -- the HIP kernels behind the C-ABI of
  ``include/chiaro_hip.h`` (the drop-in boundary of the render loop);
* ``lib/libchiaroscuro.so`` -- the host mirror of the reference's C++ classes
  ``Scene`` / ``Model`` / ``KDTree`` / ``RayTracer`` (``include/chiaroscuro.h``).

The Python names mirror the reference API (``RayTracer.rayTrace``,
``getData``, ``maxVal``, ``normalizeImage``, ``exportImage``).  There is no CPU
fallback: if the libraries are missing, or no GPU is present, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_ROOT = Path(__file__).resolve().parent.parent
# CHIARO_LIB_DIR: another build of both libraries (A/B timing of two builds, scripts/gpu_ab_libs.sh)
LIB_DIR = Path(os.environ["CHIARO_LIB_DIR"]) if os.environ.get("CHIARO_LIB_DIR") else PKG_ROOT / "lib"

CR_OK = 0
CR_ERRORS = {-1: "CR_E_INVALID", -2: "CR_E_HIP", -3: "CR_E_NOSCENE", -4: "CR_E_DEPTH", -5: "CR_E_OOM",
             -6: "CR_E_COMM"}
COMM_ID_BYTES = 128  # CR_COMM_ID_BYTES

f3 = C.c_float * 3


class CrCamera(C.Structure):
    _fields_ = [("eye", f3), ("left_upper", f3), ("dx", f3), ("dy", f3)]

    def as_array(self) -> np.ndarray:
        return np.array(list(self.eye) + list(self.left_upper) + list(self.dx) + list(self.dy), dtype=np.float32)


class CrRenderParams(C.Structure):
    _fields_ = [("xres", C.c_uint32), ("yres", C.c_uint32), ("spp", C.c_uint32), ("k", C.c_int32),
                ("background", f3), ("seed", C.c_uint32), ("layer", C.c_uint32), ("rank", C.c_uint32),
                ("nranks", C.c_uint32), ("tile", C.c_uint32)]


COUNTER_NAMES = ("closest", "shadow", "inner", "leaf", "tritest", "hit", "texhit", "paths", "pixels",
                 "wave_desc", "wave_tri", "wave_round", "wave_query", "wave_desc_uniform", "wave_tri_uniform",
                 "wave_desc_lines", "wave_tri_lines",
                 "leaf_rounds", "leaf_distinct", "leaf_records", "leaf_fit21", "leaf_fit56", "nee_answered")


class CrCounters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in COUNTER_NAMES]

    def as_dict(self) -> dict:
        return {n: int(getattr(self, n)) for n in COUNTER_NAMES}


class Checkpoint(C.Structure):
    """chiaro_checkpoint (include/chiaroscuro.h): the progressive state of a frame."""
    _fields_ = [("xres", C.c_uint32), ("yres", C.c_uint32), ("samples", C.c_uint32), ("k", C.c_uint32),
                ("seed", C.c_uint32), ("layers", C.c_uint32), ("eye", f3), ("center", f3), ("up", f3),
                ("yview", C.c_float), ("background", f3), ("scene", C.c_uint64)]


def checkpoint_write(path, header: "Checkpoint", pixels: np.ndarray):
    """chiaro_checkpoint_write: the frame [yres][xres][3] and its header, atomically."""
    px = np.ascontiguousarray(pixels, np.float32)
    assert px.shape == (header.yres, header.xres, 3), (px.shape, header.yres, header.xres)
    if libs()[1].chiaro_checkpoint_write(str(path).encode(), C.byref(header), _ptr(px)):
        raise RuntimeError("checkpoint_write: " + _host_err())


def checkpoint_read(path):
    """chiaro_checkpoint_read: (header, frame [yres][xres][3])."""
    h = Checkpoint()
    if libs()[1].chiaro_checkpoint_read(str(path).encode(), C.byref(h), None):
        raise RuntimeError("checkpoint_read: " + _host_err())
    px = np.zeros((h.yres, h.xres, 3), np.float32)
    if libs()[1].chiaro_checkpoint_read(str(path).encode(), C.byref(h), _ptr(px)):
        raise RuntimeError("checkpoint_read: " + _host_err())
    return h, px


def exr_write(path, rgb: np.ndarray):
    """chiaro_exr_write: [H][W][3] float (R, G, B, row 0 = top) as the reference's exportImage
    writes EXR -- HALF B, G, R, PIZ (src/rayTracer.cpp:229-272)."""
    px = np.ascontiguousarray(rgb, np.float32)
    if libs()[1].chiaro_exr_write(str(path).encode(), _ptr(px), px.shape[1], px.shape[0]):
        raise RuntimeError("exr_write: " + _host_err())


def exr_write_half(path, rgb: np.ndarray):
    """chiaro_exr_write_half: the same from half bits [H][W][3] uint16."""
    px = np.ascontiguousarray(rgb, np.uint16)
    if libs()[1].chiaro_exr_write_half(str(path).encode(), px.ctypes.data_as(C.POINTER(C.c_uint16)), px.shape[1],
                                       px.shape[0]):
        raise RuntimeError("exr_write_half: " + _host_err())


def exr_read_half(path) -> np.ndarray:
    """chiaro_exr_read_half: half bits [H][W][3] (R, G, B) of a scanline HALF EXR (NO / PIZ)."""
    w, h = C.c_uint32(), C.c_uint32()
    if libs()[1].chiaro_exr_read_half(str(path).encode(), C.byref(w), C.byref(h), None, 0):
        raise RuntimeError("exr_read_half: " + _host_err())
    px = np.zeros((h.value, w.value, 3), np.uint16)
    if libs()[1].chiaro_exr_read_half(str(path).encode(), C.byref(w), C.byref(h),
                                      px.ctypes.data_as(C.POINTER(C.c_uint16)), px.size):
        raise RuntimeError("exr_read_half: " + _host_err())
    return px


def float_to_half(x: np.ndarray) -> np.ndarray:
    """chiaro_float_to_half: OpenEXR's half(float) -- nearest even, overflow to infinity."""
    a = np.ascontiguousarray(x, np.float32)
    out = np.zeros(a.shape, np.uint16)
    libs()[1].chiaro_float_to_half(_ptr(a), out.ctypes.data_as(C.POINTER(C.c_uint16)), a.size)
    return out


class CrKdNode(C.Structure):
    _fields_ = [("split", C.c_float), ("axis", C.c_uint32), ("child_or_first", C.c_uint32), ("count", C.c_uint32)]


class CrTexture(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("components", C.c_int32),
                ("data", C.POINTER(C.c_uint8))]


class CrSceneDesc(C.Structure):
    _fields_ = [("n_nodes", C.c_uint32), ("nodes", C.POINTER(CrKdNode)), ("n_refs", C.c_uint32),
                ("refs", C.POINTER(C.c_uint32)), ("max_depth", C.c_uint32), ("box_min", f3), ("box_max", f3),
                ("n_tris", C.c_uint32), ("tri_pos", C.POINTER(C.c_float)), ("tri_normal", C.POINTER(C.c_float)),
                ("tri_kd", C.POINTER(C.c_float)), ("tri_ke", C.POINTER(C.c_float)),
                ("tri_uv", C.POINTER(C.c_float)), ("tri_tex", C.POINTER(C.c_int32)),
                ("tri_emissive", C.POINTER(C.c_uint8)), ("n_lights", C.c_uint32),
                ("light_id", C.POINTER(C.c_uint32)), ("light_surface", C.POINTER(C.c_float)),
                ("n_textures", C.c_uint32), ("textures", C.POINTER(CrTexture))]


class ChiaroSceneInfo(C.Structure):
    _fields_ = [("xres", C.c_uint32), ("yres", C.c_uint32), ("samples", C.c_uint32),
                ("preview_height", C.c_uint32), ("leaf_size", C.c_uint32), ("seed", C.c_uint32),
                ("k", C.c_int32), ("using_preview", C.c_int32), ("VP", f3), ("LA", f3), ("UP", f3),
                ("background", f3), ("yview", C.c_float), ("exposure", C.c_float), ("n_invalid", C.c_uint32),
                ("obj_path", C.c_char * 1024), ("render_path", C.c_char * 1024), ("gpus", C.c_uint32)]


TRACE_KINDS = ("camera", "closest", "shadow", "tail")  # cr_trace_stats order
DIAG_NAMES = ("rounds", "lanes", "distinct", "records", "maxcount", "lanetests", "fit64", "fit128",
              "urounds", "tests", "geomiss", "rep1", "rep4", "rep8")  # cr_get_diag order (DIAG_* in kernels.hpp)
PERF_NAMES = ("queries", "steps", "leaves", "masks", "tests", "vbytes", "sbytes", "waves",
              "drounds", "diters", "dlanes", "dtests")  # cr_get_perf (PERF_* in kernels.hpp)


class CrTraceStats(C.Structure):
    _fields_ = [("launches", C.c_uint64 * 4), ("ms", C.c_double * 4), ("inner", C.c_uint64 * 4),
                ("leaf", C.c_uint64 * 4), ("tritest", C.c_uint64 * 4), ("chunked_shades", C.c_uint64)]


class CrTonemapParams(C.Structure):
    _fields_ = [(n, C.c_float) for n in ("m", "s", "kl", "f", "defog", "gamma")]


def tonemap_params(exposure, defog=0.0, knee_low=0.0, knee_high=5.0, gamma=2.2) -> CrTonemapParams:
    """cr_tonemap_setup: normalizeImage's host scalars (src/rayTracer.cpp:196-205)."""
    t = CrTonemapParams()
    libs()[0].cr_tonemap_setup(exposure, defog, knee_low, knee_high, gamma, C.byref(t))
    return t


# --------------------------------------------------------------- loading --
_hip = None
_host = None

# Every symbol declared in include/chiaro_hip.h and include/chiaroscuro.h.
HIP_SYMBOLS = ("cr_create", "cr_destroy", "cr_last_error", "cr_upload_scene", "cr_render", "cr_render_device",
               "cr_render_tiles_device", "cr_blend_tiles_device", "cr_tiles_for_rank", "cr_tile_origin", "cr_intersect",
               "cr_intersect_shadow", "cr_get_counters", "cr_last_kernel_ms", "cr_get_trace_stats", "cr_set_option", "cr_synchronize", "cr_get_diag", "cr_get_perf", "cr_trace_build_available", "cr_last_trace_build",
               "cr_tonemap_setup", "cr_tonemap_device", "cr_tonemap",
               "cr_comm_unique_id", "cr_comm_init", "cr_comm_destroy", "cr_render_dist_device",
               "cr_device_count", "cr_group_create", "cr_group_destroy", "cr_group_last_error", "cr_group_size", "cr_group_ok",
               "cr_group_upload_scene", "cr_group_set_option", "cr_group_render", "cr_group_get_counters",
               "cr_group_rank_ms", "cr_group_ctx", "cr_group_tonemap", "cr_set_accumulator",
               "cr_group_set_accumulator", "cr_layers_per_pass", "cr_render_layers_device",
               "cr_render_tiles_layers_device", "cr_render_layers", "cr_scene_triangles", "cr_layers_per_group",
               "cr_blend_tiles_layers_device", "cr_render_dist_layers_device", "cr_group_render_layers")
HOST_SYMBOLS = ("chiaro_last_error", "chiaro_scene_create", "chiaro_scene_info_get", "chiaro_scene_destroy",
                "chiaro_model_create", "chiaro_model_load", "chiaro_model_num_meshes", "chiaro_model_num_triangles",
                "chiaro_model_num_textures", "chiaro_model_triangles", "chiaro_model_texture",
                "chiaro_model_destroy", "chiaro_kdtree_create", "chiaro_kdtree_num_nodes", "chiaro_kdtree_num_refs",
                "chiaro_kdtree_export", "chiaro_kdtree_describe", "chiaro_kdtree_destroy",
                "chiaro_raytracer_create", "chiaro_raytracer_raytrace", "chiaro_raytracer_raytrace_layers",
                "chiaro_raytracer_pixels",
                "chiaro_raytracer_data", "chiaro_raytracer_maxval", "chiaro_raytracer_layers",
                "chiaro_raytracer_counters", "chiaro_raytracer_normalize", "chiaro_raytracer_export",
                "chiaro_raytracer_ctx", "chiaro_raytracer_destroy", "chiaro_camera",
                "chiaro_raytracer_checkpoint", "chiaro_raytracer_resume", "chiaro_kdtree_fingerprint",
                "chiaro_checkpoint_write", "chiaro_checkpoint_read",
                "chiaro_exr_write", "chiaro_exr_write_half", "chiaro_exr_read_half", "chiaro_float_to_half",
                "chiaro_preview_create", "chiaro_preview_key", "chiaro_preview_mouse", "chiaro_preview_scroll",
                "chiaro_preview_texture", "chiaro_preview_state", "chiaro_preview_destroy",
                "chiaro_preview_camera_replay")

P = C.c_void_p
FP = C.POINTER(C.c_float)
UP = C.POINTER(C.c_uint32)


def _sig(lib, name, res, args):
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = args


def libs():
    """Load (once) and return (libchiaro_hip, libchiaroscuro).  Raises if not built."""
    global _hip, _host
    if _hip is not None:
        return _hip, _host
    hip_path, host_path = LIB_DIR / "libchiaro_hip.so", LIB_DIR / "libchiaroscuro.so"
    if not hip_path.exists() or not host_path.exists():
        raise RuntimeError("chiaroscuro_amd: native libraries not built (%s); run "
                           "`make -C chiaroscuro-raytracer_amd` or __graft_entry__.build()" % LIB_DIR)
    # torch first: it carries its own HIP runtime and RCCL under the sonames
    # libchiaro_hip.so needs (libamdhip64.so.7, librccl.so.1), so loaded in this
    # order the process holds one copy of each (the other order maps a second
    # runtime next to torch's, whose exit-time teardown collides with the first)
    try:  # only the load order matters; host-only use (scene parsing, the preview camera) needs no torch
        import torch  # noqa: F401
    except ImportError:
        pass
    hip = C.CDLL(str(hip_path), mode=C.RTLD_GLOBAL)
    host = C.CDLL(str(host_path))
    _sig(hip, "cr_create", P, [C.c_int])
    _sig(hip, "cr_destroy", None, [P])
    _sig(hip, "cr_last_error", C.c_char_p, [P])
    _sig(hip, "cr_upload_scene", C.c_int, [P, C.POINTER(CrSceneDesc)])
    _sig(hip, "cr_render", C.c_int, [P, C.POINTER(CrCamera), C.POINTER(CrRenderParams), FP])
    _sig(hip, "cr_render_device", C.c_int, [P, C.POINTER(CrCamera), C.POINTER(CrRenderParams), P, P])
    _sig(hip, "cr_render_tiles_device", C.c_int, [P, C.POINTER(CrCamera), C.POINTER(CrRenderParams), P, P])
    _sig(hip, "cr_layers_per_pass", C.c_uint32, [P, C.POINTER(CrRenderParams), C.c_uint32])
    _sig(hip, "cr_render_layers", C.c_int, [P, C.POINTER(CrCamera), C.POINTER(CrRenderParams), C.c_uint32, P])
    _sig(hip, "cr_scene_triangles", C.c_uint32, [P])
    _sig(hip, "cr_layers_per_group", C.c_uint32, [P, C.POINTER(CrRenderParams), C.c_uint32])
    _sig(hip, "cr_render_layers_device", C.c_int, [P, C.POINTER(CrCamera), C.POINTER(CrRenderParams), C.c_uint32, P, P])
    _sig(hip, "cr_render_tiles_layers_device", C.c_int,
         [P, C.POINTER(CrCamera), C.POINTER(CrRenderParams), C.c_uint32, P, P])
    _sig(hip, "cr_blend_tiles_device", C.c_int, [P, C.POINTER(CrRenderParams), P, P, P])
    _sig(hip, "cr_blend_tiles_layers_device", C.c_int, [P, C.POINTER(CrRenderParams), C.c_uint32, P, P, P])
    _sig(hip, "cr_tiles_for_rank", C.c_uint32, [C.POINTER(CrRenderParams), C.c_uint32])
    _sig(hip, "cr_tile_origin", C.c_int, [C.POINTER(CrRenderParams), C.c_uint32, C.c_uint32,
                                          C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)])
    _sig(hip, "cr_intersect", C.c_int, [P, C.c_uint32, FP, FP, UP, UP, FP, FP])
    _sig(hip, "cr_intersect_shadow", C.c_int, [P, C.c_uint32, FP, FP, FP, UP, UP])
    _sig(hip, "cr_get_counters", C.c_int, [P, C.POINTER(CrCounters)])
    _sig(hip, "cr_last_kernel_ms", C.c_float, [P])
    _sig(hip, "cr_get_trace_stats", C.c_int, [P, C.POINTER(CrTraceStats)])
    _sig(hip, "cr_set_option", C.c_int, [P, C.c_char_p, C.c_int64])
    _sig(hip, "cr_get_diag", C.c_int, [P, C.POINTER(C.c_uint64), C.c_int])
    _sig(hip, "cr_get_perf", C.c_int, [P, C.POINTER(C.c_uint64), C.c_int])
    _sig(hip, "cr_trace_build_available", C.c_int, [C.c_int])
    _sig(hip, "cr_last_trace_build", C.c_int, [P])
    _sig(hip, "cr_synchronize", C.c_int, [P])
    _sig(hip, "cr_tonemap_setup", None, [C.c_float] * 5 + [C.POINTER(CrTonemapParams)])
    _sig(hip, "cr_tonemap_device", C.c_int, [P, C.POINTER(CrTonemapParams), C.c_uint32, C.c_uint32, P, P, P])
    _sig(hip, "cr_tonemap", C.c_int, [P, C.POINTER(CrTonemapParams), C.c_uint32, C.c_uint32,
                                      C.POINTER(C.c_uint8)])

    _sig(hip, "cr_comm_unique_id", C.c_int, [C.POINTER(C.c_uint8), C.c_size_t])
    _sig(hip, "cr_comm_init", C.c_int, [P, C.c_int, C.c_int, C.POINTER(C.c_uint8)])
    _sig(hip, "cr_comm_destroy", C.c_int, [P])
    _sig(hip, "cr_render_dist_device", C.c_int, [P, C.POINTER(CrCamera), C.POINTER(CrRenderParams), P, P])
    _sig(hip, "cr_render_dist_layers_device", C.c_int, [P, C.POINTER(CrCamera), C.POINTER(CrRenderParams),
                                                         C.c_uint32, P, P])
    _sig(hip, "cr_device_count", C.c_int, [])
    _sig(hip, "cr_group_create", P, [C.c_int, C.POINTER(C.c_int)])
    _sig(hip, "cr_group_destroy", None, [P])
    _sig(hip, "cr_group_last_error", C.c_char_p, [P])
    _sig(hip, "cr_group_size", C.c_int, [P])
    _sig(hip, "cr_group_ok", C.c_int, [P])
    _sig(hip, "cr_group_upload_scene", C.c_int, [P, C.POINTER(CrSceneDesc)])
    _sig(hip, "cr_group_set_option", C.c_int, [P, C.c_char_p, C.c_int64])
    _sig(hip, "cr_group_render", C.c_int, [P, C.POINTER(CrCamera), C.POINTER(CrRenderParams), FP])
    _sig(hip, "cr_group_render_layers", C.c_int, [P, C.POINTER(CrCamera), C.POINTER(CrRenderParams), C.c_uint32,
                                                   FP])
    _sig(hip, "cr_group_get_counters", C.c_int, [P, C.POINTER(CrCounters)])
    _sig(hip, "cr_group_rank_ms", C.c_int, [P, FP])
    _sig(hip, "cr_group_ctx", P, [P, C.c_int])
    _sig(hip, "cr_set_accumulator", C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(C.c_float)])
    _sig(hip, "cr_group_set_accumulator", C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(C.c_float)])
    _sig(hip, "cr_group_tonemap", C.c_int, [P, C.POINTER(CrTonemapParams), C.c_uint32, C.c_uint32,
                                            C.POINTER(C.c_uint8)])

    _sig(host, "chiaro_last_error", C.c_char_p, [])
    _sig(host, "chiaro_scene_create", P, [C.c_int, C.POINTER(C.c_char_p)])
    _sig(host, "chiaro_scene_info_get", C.c_int, [P, C.POINTER(ChiaroSceneInfo)])
    _sig(host, "chiaro_scene_destroy", None, [P])
    _sig(host, "chiaro_model_create", P, [P])
    _sig(host, "chiaro_model_load", P, [C.c_char_p])
    for n in ("chiaro_model_num_meshes", "chiaro_model_num_triangles", "chiaro_model_num_textures"):
        _sig(host, n, C.c_uint32, [P])
    _sig(host, "chiaro_model_triangles", C.c_int, [P, FP, FP, FP, FP, FP, C.POINTER(C.c_int32)])
    _sig(host, "chiaro_model_texture", C.c_int,
         [P, C.c_uint32, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
          C.POINTER(C.POINTER(C.c_uint8))])
    _sig(host, "chiaro_model_destroy", None, [P])
    _sig(host, "chiaro_kdtree_create", P, [P, P, C.c_int])
    _sig(host, "chiaro_kdtree_num_nodes", C.c_uint32, [P])
    _sig(host, "chiaro_kdtree_num_refs", C.c_uint32, [P])
    _sig(host, "chiaro_kdtree_export", C.c_int, [P, UP, UP, FP, UP, UP, UP, UP, FP])
    _sig(host, "chiaro_kdtree_describe", C.c_int, [P, P, C.POINTER(CrSceneDesc)])
    _sig(host, "chiaro_kdtree_destroy", None, [P])
    _sig(host, "chiaro_raytracer_create", P, [P, P, C.c_int])
    _sig(host, "chiaro_raytracer_raytrace", C.c_int, [P, FP, FP, FP, C.c_float])
    _sig(host, "chiaro_raytracer_raytrace_layers", C.c_int, [P, C.c_uint32, FP, FP, FP, C.c_float])
    _sig(host, "chiaro_raytracer_pixels", FP, [P])
    _sig(host, "chiaro_raytracer_data", C.POINTER(C.c_uint8), [P])
    _sig(host, "chiaro_raytracer_maxval", C.c_float, [P])
    _sig(host, "chiaro_raytracer_layers", C.c_uint32, [P])
    _sig(host, "chiaro_raytracer_counters", C.c_int, [P, C.POINTER(CrCounters)])
    _sig(host, "chiaro_raytracer_normalize", C.c_int, [P, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float])
    _sig(host, "chiaro_raytracer_export", C.c_int, [P, C.c_char_p])
    _sig(host, "chiaro_raytracer_ctx", P, [P])
    _sig(host, "chiaro_raytracer_checkpoint", C.c_int, [P, C.c_char_p])
    _sig(host, "chiaro_raytracer_resume", C.c_int, [P, C.c_char_p])
    _sig(host, "chiaro_kdtree_fingerprint", C.c_uint64, [P])
    _sig(host, "chiaro_checkpoint_write", C.c_int, [C.c_char_p, C.POINTER(Checkpoint), FP])
    _sig(host, "chiaro_checkpoint_read", C.c_int, [C.c_char_p, C.POINTER(Checkpoint), FP])
    _sig(host, "chiaro_raytracer_destroy", None, [P])
    U16P = C.POINTER(C.c_uint16)
    _sig(host, "chiaro_exr_write", C.c_int, [C.c_char_p, FP, C.c_uint32, C.c_uint32])
    _sig(host, "chiaro_exr_write_half", C.c_int, [C.c_char_p, U16P, C.c_uint32, C.c_uint32])
    _sig(host, "chiaro_exr_read_half", C.c_int, [C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), U16P,
                                                 C.c_size_t])
    _sig(host, "chiaro_float_to_half", C.c_int, [FP, U16P, C.c_size_t])
    _sig(host, "chiaro_camera", C.c_int, [FP, FP, FP, C.c_float, C.c_uint32, C.c_uint32, C.POINTER(CrCamera)])
    _sig(host, "chiaro_preview_create", P, [P, P])
    _sig(host, "chiaro_preview_key", C.c_int, [P, C.c_int, C.c_float, C.c_int])
    _sig(host, "chiaro_preview_mouse", C.c_int, [P, C.c_float, C.c_float])
    _sig(host, "chiaro_preview_scroll", C.c_int, [P, C.c_float])
    _sig(host, "chiaro_preview_texture", C.POINTER(C.c_uint8), [P, UP, UP])
    _sig(host, "chiaro_preview_state", C.c_int, [P, FP, FP, FP, FP, C.POINTER(C.c_int), UP])
    _sig(host, "chiaro_preview_destroy", None, [P])
    _sig(host, "chiaro_preview_camera_replay", C.c_int, [FP, FP, FP, C.c_float, C.POINTER(C.c_int32), FP, C.c_int,
                                                         FP])
    _hip, _host = hip, host
    return hip, host


def _fa(v) -> C.Array:
    return (C.c_float * 3)(*[float(x) for x in v])


def _ptr(a: np.ndarray, t=C.c_float):
    return a.ctypes.data_as(C.POINTER(t))


def _host_err() -> str:
    return libs()[1].chiaro_last_error().decode()


# ------------------------------------------------------------------ camera --
def camera(eye, center, up, yview, xres, yres) -> CrCamera:
    """Camera basis exactly as src/rayTracer.cpp:41-49 (host side)."""
    _, host = libs()
    cam = CrCamera()
    rc = host.chiaro_camera(_fa(eye), _fa(center), _fa(up), float(yview), int(xres), int(yres), C.byref(cam))
    if rc:
        raise ValueError("chiaro_camera failed")
    return cam


def render_params(xres, yres, spp, k, seed, layer=1, background=(0.0, 0.0, 0.0), rank=0, nranks=1,
                  tile=32) -> CrRenderParams:
    return CrRenderParams(int(xres), int(yres), int(spp), int(k), _fa(background), int(seed) & 0xFFFFFFFF,
                          int(layer), int(rank), int(nranks), int(tile))


# ------------------------------------------------------------------- host --
class Scene:
    """Scene(argc, argv): ``Scene(rtc_path, *overrides)``, src/scene.cpp:13-72."""

    def __init__(self, rtc_path, *overrides):
        _, host = libs()
        argv = [b"chiaroscuro", str(rtc_path).encode()] + [str(o).encode() for o in overrides]
        arr = (C.c_char_p * len(argv))(*argv)
        self._h = host.chiaro_scene_create(len(argv), arr)
        if not self._h:
            raise ValueError("Scene: " + _host_err())

    @property
    def info(self) -> dict:
        _, host = libs()
        i = ChiaroSceneInfo()
        host.chiaro_scene_info_get(self._h, C.byref(i))
        return {"xres": i.xres, "yres": i.yres, "samples": i.samples, "k": i.k, "seed": i.seed,
                "leaf_size": i.leaf_size, "VP": list(i.VP), "LA": list(i.LA), "UP": list(i.UP),
                "yview": i.yview, "exposure": i.exposure, "background": list(i.background),
                "preview_height": i.preview_height, "using_preview": bool(i.using_preview),
                "n_invalid": i.n_invalid, "obj_path": i.obj_path.decode(), "render_path": i.render_path.decode(),
                "gpus": i.gpus}

    def __del__(self):
        if getattr(self, "_h", None) and _host is not None:
            _host.chiaro_scene_destroy(self._h)
            self._h = None


class Model:
    """Model(Scene&), src/model.cpp:17-36 (own OBJ/MTL loader)."""

    def __init__(self, scene: Scene | None = None, path: str | None = None):
        _, host = libs()
        self._h = host.chiaro_model_create(scene._h) if scene is not None else host.chiaro_model_load(
            str(path).encode())
        if not self._h:
            raise ValueError("Model: " + _host_err())

    @property
    def num_meshes(self) -> int:
        return libs()[1].chiaro_model_num_meshes(self._h)

    @property
    def num_triangles(self) -> int:
        return libs()[1].chiaro_model_num_triangles(self._h)

    def triangles(self) -> dict:
        """Triangle soup in KDTree order (src/kdtree.cpp:44-66)."""
        _, host = libs()
        n = self.num_triangles
        out = {"pos": np.zeros((n, 9), np.float32), "vnrm": np.zeros((n, 9), np.float32),
               "uv": np.zeros((n, 6), np.float32), "kd": np.zeros((n, 3), np.float32),
               "ke": np.zeros((n, 3), np.float32), "tex": np.zeros(n, np.int32)}
        host.chiaro_model_triangles(self._h, _ptr(out["pos"]), _ptr(out["vnrm"]), _ptr(out["uv"]),
                                    _ptr(out["kd"]), _ptr(out["ke"]), _ptr(out["tex"], C.c_int32))
        return out

    def textures(self) -> list:
        _, host = libs()
        res = []
        for i in range(host.chiaro_model_num_textures(self._h)):
            w, h, nc = C.c_int32(), C.c_int32(), C.c_int32()
            d = C.POINTER(C.c_uint8)()
            host.chiaro_model_texture(self._h, i, C.byref(w), C.byref(h), C.byref(nc), C.byref(d))
            arr = np.ctypeslib.as_array(d, shape=(w.value * h.value * nc.value,)).copy()
            res.append((w.value, h.value, nc.value, arr))
        return res

    def __del__(self):
        if getattr(self, "_h", None) and _host is not None:
            _host.chiaro_model_destroy(self._h)
            self._h = None


class KDTree:
    """Host KDTree(Model&, Scene&) build, src/kdtree.cpp:34-194 (no device needed)."""

    def __init__(self, model: Model, scene: Scene, threads: int = 0):
        _, host = libs()
        self._model, self._scene = model, scene
        self._h = host.chiaro_kdtree_create(model._h, scene._h, int(threads))
        if not self._h:
            raise ValueError("KDTree: " + _host_err())

    def fingerprint(self) -> int:
        """chiaro_kdtree_fingerprint: which triangles, in which tree (checkpoints record it)."""
        return int(libs()[1].chiaro_kdtree_fingerprint(self._h))

    def export(self) -> dict:
        _, host = libs()
        n, r = host.chiaro_kdtree_num_nodes(self._h), host.chiaro_kdtree_num_refs(self._h)
        o = {k: np.zeros(n, np.uint32) for k in ("is_leaf", "axis", "child", "leaf_first", "leaf_count")}
        o["split"] = np.zeros(n, np.float32)
        o["refs"] = np.zeros(max(r, 1), np.uint32)
        o["box"] = np.zeros(6, np.float32)
        host.chiaro_kdtree_export(self._h, _ptr(o["is_leaf"], C.c_uint32), _ptr(o["axis"], C.c_uint32),
                                  _ptr(o["split"]), _ptr(o["child"], C.c_uint32), _ptr(o["leaf_first"], C.c_uint32),
                                  _ptr(o["leaf_count"], C.c_uint32), _ptr(o["refs"], C.c_uint32), _ptr(o["box"]))
        o["refs"] = o["refs"][:r]
        return o

    def describe(self) -> CrSceneDesc:
        d = CrSceneDesc()
        rc = libs()[1].chiaro_kdtree_describe(self._h, self._scene._h, C.byref(d))
        if rc:
            raise RuntimeError("describe: " + _host_err())
        d._owner = self  # the descriptor points into this tree's host arrays: keep it alive
        return d

    def __del__(self):
        if getattr(self, "_h", None) and _host is not None:
            _host.chiaro_kdtree_destroy(self._h)
            self._h = None


class Device:
    """One cr_ctx (include/chiaro_hip.h) -- the raw C-ABI boundary."""

    def __init__(self, device: int = 0):
        hip, _ = libs()
        self._c = hip.cr_create(int(device))
        if not self._c:
            raise RuntimeError("cr_create returned NULL")
        self.device = device

    def _chk(self, rc, what):
        if rc != CR_OK:
            raise RuntimeError("%s failed (%s): %s" % (what, CR_ERRORS.get(rc, rc),
                                                       libs()[0].cr_last_error(self._c).decode()))

    def upload(self, desc: CrSceneDesc):
        self._chk(libs()[0].cr_upload_scene(self._c, C.byref(desc)), "cr_upload_scene")

    def render(self, cam: CrCamera, p: CrRenderParams, accum: np.ndarray | None = None) -> np.ndarray:
        out = accum if accum is not None else np.zeros((p.yres, p.xres, 3), np.float32)
        assert out.dtype == np.float32 and out.flags.c_contiguous and out.size == p.yres * p.xres * 3
        self._chk(libs()[0].cr_render(self._c, C.byref(cam), C.byref(p), _ptr(out)), "cr_render")
        return out

    def render_layers(self, cam: CrCamera, p: CrRenderParams, nlayers: int,
                      accum: np.ndarray | None = None) -> np.ndarray:
        """cr_render_layers: layers p.layer .. + nlayers - 1 of the whole frame in pass groups
        (bit-identical to nlayers render calls); counters sum over the passes."""
        out = accum if accum is not None else np.zeros((p.yres, p.xres, 3), np.float32)
        assert out.dtype == np.float32 and out.flags.c_contiguous and out.size == p.yres * p.xres * 3
        self._chk(libs()[0].cr_render_layers(self._c, C.byref(cam), C.byref(p), nlayers, _ptr(out)),
                  "cr_render_layers")
        return out

    def render_device(self, cam, p, d_frame_ptr: int, stream: int = 0):
        self._chk(libs()[0].cr_render_device(self._c, C.byref(cam), C.byref(p), C.c_void_p(d_frame_ptr),
                                             C.c_void_p(stream)), "cr_render_device")

    def render_tiles_device(self, cam, p, d_tiles_ptr: int, stream: int = 0):
        self._chk(libs()[0].cr_render_tiles_device(self._c, C.byref(cam), C.byref(p), C.c_void_p(d_tiles_ptr),
                                                   C.c_void_p(stream)), "cr_render_tiles_device")

    def layers_per_group(self, p, want: int) -> int:
        """How many of `want` layers one pass group renders for p's share (in pieces)."""
        return int(libs()[0].cr_layers_per_group(self._c, C.byref(p), want))

    def scene_triangles(self) -> int:
        return int(libs()[0].cr_scene_triangles(self._c))

    def layers_per_pass(self, p, want: int) -> int:
        """How many of `want` progressive layers (from p.layer) fit one render pass."""
        return int(libs()[0].cr_layers_per_pass(self._c, C.byref(p), want))

    def render_layers_device(self, cam, p, nlayers: int, d_frame_ptr: int, stream: int = 0):
        """Layers p.layer .. p.layer + nlayers - 1 in one pass, blended in order into d_frame
        (bit-identical to nlayers render_device calls)."""
        self._chk(libs()[0].cr_render_layers_device(self._c, C.byref(cam), C.byref(p), nlayers,
                                                    C.c_void_p(d_frame_ptr), C.c_void_p(stream)),
                  "cr_render_layers_device")

    def render_tiles_layers_device(self, cam, p, nlayers: int, d_tiles_ptr: int, stream: int = 0):
        """Layers p.layer .. + nlayers - 1 in one pass; layer j's tile means at
        d_tiles + j * max_tiles * tile * tile * 3 floats."""
        self._chk(libs()[0].cr_render_tiles_layers_device(self._c, C.byref(cam), C.byref(p), nlayers,
                                                          C.c_void_p(d_tiles_ptr), C.c_void_p(stream)),
                  "cr_render_tiles_layers_device")

    def blend_tiles_layers_device(self, p, nlayers: int, d_gathered_ptr: int, d_frame_ptr: int, stream: int = 0):
        """cr_blend_tiles_layers_device: gathered [nranks][nlayers][max_tiles][T][T][3], layers p.layer ..
        + nlayers - 1 blended in order in one launch."""
        self._chk(libs()[0].cr_blend_tiles_layers_device(self._c, C.byref(p), int(nlayers), C.c_void_p(d_gathered_ptr),
                                                         C.c_void_p(d_frame_ptr), C.c_void_p(stream)),
                  "cr_blend_tiles_layers_device")

    def blend_tiles_device(self, p, d_gathered_ptr: int, d_frame_ptr: int, stream: int = 0):
        self._chk(libs()[0].cr_blend_tiles_device(self._c, C.byref(p), C.c_void_p(d_gathered_ptr),
                                                  C.c_void_p(d_frame_ptr), C.c_void_p(stream)),
                  "cr_blend_tiles_device")

    def tonemap_device(self, t: CrTonemapParams, xres: int, yres: int, d_rgb_ptr: int, d_bytes_ptr: int,
                       stream: int = 0):
        """normalizeImage's per-pixel transform on device buffers (rows flipped)."""
        self._chk(libs()[0].cr_tonemap_device(self._c, C.byref(t), xres, yres, C.c_void_p(d_rgb_ptr),
                                              C.c_void_p(d_bytes_ptr), C.c_void_p(stream)), "cr_tonemap_device")

    @staticmethod
    def tiles_for_rank(p: CrRenderParams, rank: int) -> int:
        return int(libs()[0].cr_tiles_for_rank(C.byref(p), int(rank)))

    @staticmethod
    def tile_origin(p: CrRenderParams, rank: int, local: int):
        x0, y0 = C.c_uint32(0), C.c_uint32(0)
        if libs()[0].cr_tile_origin(C.byref(p), int(rank), int(local), C.byref(x0), C.byref(y0)):
            raise ValueError("cr_tile_origin: no such tile")
        return x0.value, y0.value

    def intersect(self, orig: np.ndarray, dirs: np.ndarray) -> dict:
        orig = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
        dirs = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        n = len(orig)
        hit, tri = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        bary, dist = np.zeros((n, 2), np.float32), np.zeros(n, np.float32)
        self._chk(libs()[0].cr_intersect(self._c, n, _ptr(orig), _ptr(dirs), _ptr(hit, C.c_uint32),
                                         _ptr(tri, C.c_uint32), _ptr(bary), _ptr(dist)), "cr_intersect")
        return {"hit": hit, "tri": tri, "bary": bary, "dist": dist}

    def intersect_shadow(self, orig, dirs, dist, light) -> np.ndarray:
        orig = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
        dirs = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        dist = np.ascontiguousarray(dist, np.float32)
        light = np.ascontiguousarray(light, np.uint32)
        occ = np.zeros(len(orig), np.uint32)
        self._chk(libs()[0].cr_intersect_shadow(self._c, len(orig), _ptr(orig), _ptr(dirs), _ptr(dist),
                                                _ptr(light, C.c_uint32), _ptr(occ, C.c_uint32)),
                  "cr_intersect_shadow")
        return occ

    def counters(self) -> dict:
        c = CrCounters()
        libs()[0].cr_get_counters(self._c, C.byref(c))
        return c.as_dict()

    def last_kernel_ms(self) -> float:
        return float(libs()[0].cr_last_kernel_ms(self._c))

    def trace_stats(self) -> dict:
        """cr_get_trace_stats: per trace-launch kind (TRACE_KINDS) of the
        last wavefront render -- launches, summed event ms, inner / leaf / tritest."""
        t = CrTraceStats()
        self._chk(libs()[0].cr_get_trace_stats(self._c, C.byref(t)), "cr_get_trace_stats")
        return {name: {"launches": int(t.launches[i]), "ms": float(t.ms[i]), "inner": int(t.inner[i]),
                       "leaf": int(t.leaf[i]), "tritest": int(t.tritest[i])}
                for i, name in enumerate(TRACE_KINDS)}

    def chunked_shades(self) -> int:
        """cr_get_trace_stats' chunked_shades: the wf_shade launches of the last wavefront render that
        reserved queue slots in chunks."""
        t = CrTraceStats()
        self._chk(libs()[0].cr_get_trace_stats(self._c, C.byref(t)), "cr_get_trace_stats")
        return int(t.chunked_shades)

    def diag(self) -> dict:
        """cr_get_diag: leaf-round shapes and the repeated-miss census of the last
        counting render, for the trace kinds of option "diag_kinds"."""
        v = (C.c_uint64 * len(DIAG_NAMES))()
        self._chk(libs()[0].cr_get_diag(self._c, v, len(DIAG_NAMES)), "cr_get_diag")
        return {n: int(v[i]) for i, n in enumerate(DIAG_NAMES)}

    def perf(self) -> dict:
        """cr_get_perf: performed work of the last render with option "perf_counters" 1, per
        trace kind (TRACE_KINDS): queries, steps, leaves, masks, tests, vbytes, sbytes, waves."""
        n = len(PERF_NAMES)
        v = (C.c_uint64 * (n * len(TRACE_KINDS)))()
        self._chk(libs()[0].cr_get_perf(self._c, v, len(v)), "cr_get_perf")
        return {k: {nm: int(v[n * i + j]) for j, nm in enumerate(PERF_NAMES)} for i, k in enumerate(TRACE_KINDS)}

    def set_option(self, key: str, value: int):
        self._chk(libs()[0].cr_set_option(self._c, key.encode(), int(value)), "cr_set_option")

    def last_trace_build(self) -> int:
        """cr_last_trace_build: the trace build of the last render (-1 counting build, -2 not wavefront)."""
        return int(libs()[0].cr_last_trace_build(self._c))

    @staticmethod
    def trace_builds(upto: int = 64) -> list:
        """The wavefront trace builds compiled in (cr_trace_build_available)."""
        return [b for b in range(upto) if libs()[0].cr_trace_build_available(b)]

    @staticmethod
    def device_count() -> int:
        """cr_device_count: HIP devices this process sees (0 without a GPU)."""
        return int(libs()[0].cr_device_count())

    # multi-process frame split (one process per GPU, RCCL inside the library)
    @staticmethod
    def comm_unique_id() -> bytes:
        """cr_comm_unique_id: the RCCL id rank 0 makes and hands to every rank."""
        buf = (C.c_uint8 * COMM_ID_BYTES)()
        rc = libs()[0].cr_comm_unique_id(buf, COMM_ID_BYTES)
        if rc != CR_OK:
            raise RuntimeError("cr_comm_unique_id failed (%s)" % CR_ERRORS.get(rc, rc))
        return bytes(buf)

    def comm_init(self, nranks: int, rank: int, uid: bytes):
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid[:COMM_ID_BYTES].ljust(COMM_ID_BYTES, b"\0"))
        self._chk(libs()[0].cr_comm_init(self._c, int(nranks), int(rank), buf), "cr_comm_init")

    def comm_destroy(self):
        self._chk(libs()[0].cr_comm_destroy(self._c), "cr_comm_destroy")

    def render_dist_device(self, cam, p, d_frame_ptr: int, stream: int = 0):
        """cr_render_dist_device: my tiles, RCCL gather to rank 0, blend there."""
        self._chk(libs()[0].cr_render_dist_device(self._c, C.byref(cam), C.byref(p), C.c_void_p(d_frame_ptr),
                                                  C.c_void_p(stream)), "cr_render_dist_device")

    def render_dist_layers_device(self, cam, p, nlayers: int, d_frame_ptr: int, stream: int = 0):
        """cr_render_dist_layers_device: my tiles of nlayers layers in one pass group, one RCCL gather of
        the group's buffers to rank 0, one blend of its layers there (every rank the same nlayers)."""
        self._chk(libs()[0].cr_render_dist_layers_device(self._c, C.byref(cam), C.byref(p), int(nlayers),
                                                         C.c_void_p(d_frame_ptr), C.c_void_p(stream)),
                  "cr_render_dist_layers_device")

    def synchronize(self):
        self._chk(libs()[0].cr_synchronize(self._c), "cr_synchronize")

    def close(self):
        if getattr(self, "_c", None):
            libs()[0].cr_destroy(self._c)
            self._c = None

    def __del__(self):
        if _hip is not None:
            self.close()


class Group:
    """cr_group (include/chiaro_hip.h): one process driving N GPUs, the frame
    tile-split over them and gathered to the first over RCCL."""

    def __init__(self, devices):
        hip, _ = libs()
        devs = (C.c_int * len(devices))(*[int(d) for d in devices])
        self._g = hip.cr_group_create(len(devices), devs)
        self.devices = list(devices)
        if not hip.cr_group_ok(self._g):  # a bad device, no GPU, or RCCL refused the communicator
            err = hip.cr_group_last_error(self._g).decode()
            self.close()
            raise RuntimeError("cr_group_create(%s) failed: %s" % (self.devices, err))

    def _chk(self, rc, what):
        if rc != CR_OK:
            raise RuntimeError("%s failed (%s): %s" % (what, CR_ERRORS.get(rc, rc),
                                                       libs()[0].cr_group_last_error(self._g).decode()))

    def upload(self, desc: CrSceneDesc):
        self._chk(libs()[0].cr_group_upload_scene(self._g, C.byref(desc)), "cr_group_upload_scene")

    def set_option(self, key: str, value: int):
        self._chk(libs()[0].cr_group_set_option(self._g, key.encode(), int(value)), "cr_group_set_option")

    def render(self, cam: CrCamera, p: CrRenderParams) -> np.ndarray:
        out = np.zeros((p.yres, p.xres, 3), np.float32)
        self._chk(libs()[0].cr_group_render(self._g, C.byref(cam), C.byref(p), _ptr(out)), "cr_group_render")
        return out

    def render_layers(self, cam: CrCamera, p: CrRenderParams, nlayers: int) -> np.ndarray:
        """cr_group_render_layers: layers p.layer .. + nlayers - 1 in pass groups across the group."""
        out = np.zeros((p.yres, p.xres, 3), np.float32)
        self._chk(libs()[0].cr_group_render_layers(self._g, C.byref(cam), C.byref(p), int(nlayers), _ptr(out)),
                  "cr_group_render_layers")
        return out

    def counters(self) -> dict:
        c = CrCounters()
        libs()[0].cr_group_get_counters(self._g, C.byref(c))
        return c.as_dict()

    def rank_ms(self) -> list:
        out = np.zeros(len(self.devices), np.float32)
        libs()[0].cr_group_rank_ms(self._g, _ptr(out))
        return [float(x) for x in out]

    def close(self):
        if getattr(self, "_g", None):
            libs()[0].cr_group_destroy(self._g)
            self._g = None

    def __del__(self):
        if _hip is not None:
            self.close()


class RayTracer:
    """RayTracer(Model&, Scene&) -- include/rayTracer.hpp:10-41, GPU render loop."""

    def __init__(self, model: Model, scene: Scene, device: int = 0):
        _, host = libs()
        self._model, self._scene = model, scene
        self._h = host.chiaro_raytracer_create(model._h, scene._h, int(device))
        if not self._h:
            raise RuntimeError("RayTracer: " + _host_err())
        info = scene.info
        self.xres, self.yres = info["xres"], info["yres"]

    def rayTrace(self, eye, center, up=(0.0, 1.0, 0.0), yview=1.0):
        rc = libs()[1].chiaro_raytracer_raytrace(self._h, _fa(eye), _fa(center), _fa(up), float(yview))
        if rc:
            raise RuntimeError("rayTrace: " + _host_err())

    ray_trace = rayTrace

    def rayTraceLayers(self, n, eye, center, up=(0.0, 1.0, 0.0), yview=1.0):
        """n rayTrace calls with the same view in pass groups (bit-identical)."""
        rc = libs()[1].chiaro_raytracer_raytrace_layers(self._h, int(n), _fa(eye), _fa(center), _fa(up), float(yview))
        if rc:
            raise RuntimeError("rayTraceLayers: " + _host_err())

    @property
    def pixels(self) -> np.ndarray:
        p = libs()[1].chiaro_raytracer_pixels(self._h)
        return np.ctypeslib.as_array(p, shape=(self.yres, self.xres, 3)).copy()

    @property
    def maxVal(self) -> float:
        return float(libs()[1].chiaro_raytracer_maxval(self._h))

    @property
    def layers(self) -> int:
        return int(libs()[1].chiaro_raytracer_layers(self._h))

    def getData(self) -> np.ndarray:
        d = libs()[1].chiaro_raytracer_data(self._h)
        return np.ctypeslib.as_array(d, shape=(self.yres, self.xres, 3)).copy()

    def normalizeImage(self, exposure=3.4028234663852886e38, defog=0.0, kneeLow=0.0, kneeHigh=5.0, gamma=2.2):
        if libs()[1].chiaro_raytracer_normalize(self._h, exposure, defog, kneeLow, kneeHigh, gamma):
            raise RuntimeError("normalizeImage: " + _host_err())

    def exportImage(self, filename: str):
        if libs()[1].chiaro_raytracer_export(self._h, str(filename).encode()):
            raise RuntimeError("exportImage: " + _host_err())

    def counters(self) -> dict:
        c = CrCounters()
        libs()[1].chiaro_raytracer_counters(self._h, C.byref(c))
        return c.as_dict()

    def checkpoint(self, path):
        """Save the progressive state (layers, camera, running average) -- chiaro_raytracer_checkpoint."""
        if libs()[1].chiaro_raytracer_checkpoint(self._h, str(path).encode()):
            raise RuntimeError("checkpoint: " + _host_err())

    def resume(self, path):
        """Continue a saved progressive render: the next rayTrace at its camera is layer layers + 1."""
        if libs()[1].chiaro_raytracer_resume(self._h, str(path).encode()):
            raise RuntimeError("resume: " + _host_err())

    def __del__(self):
        if getattr(self, "_h", None) and _host is not None:
            _host.chiaro_raytracer_destroy(self._h)
            self._h = None


def preview_camera_replay(vp, la, up, yview, ops, args) -> np.ndarray:
    """chiaro_preview_camera_replay: the preview camera after each op -> [nops][15]
    (Position, Front, Up, Right, Yaw, Pitch, Zoom).  No GPU."""
    ops = np.ascontiguousarray(ops, np.int32)
    args = np.ascontiguousarray(args, np.float32).reshape(-1)
    out = np.zeros((len(ops), 15), np.float32)
    rc = libs()[1].chiaro_preview_camera_replay(_fa(vp), _fa(la), _fa(up), float(yview), _ptr(ops, C.c_int32),
                                                _ptr(args), len(ops), _ptr(out))
    if rc:
        raise ValueError("chiaro_preview_camera_replay: bad op")
    return out


class Preview:
    """The interactive preview's render path without a window (chiaro_preview_*,
    src/openglPreview.cpp:12-257): keys R / TAB / = / - / W S A D E Q, mouse, scroll,
    and the screen texture (getData after normalizeImage)."""
    KEYS = {"R": 0, "TAB": 1, "=": 2, "-": 3, "W": 4, "S": 5, "A": 6, "D": 7, "E": 8, "Q": 9, "SHIFT": 10}

    def __init__(self, scene: Scene, rt: RayTracer):
        _, host = libs()
        self._scene, self._rt = scene, rt
        self._p = host.chiaro_preview_create(scene._h, rt._h)
        if not self._p:
            raise RuntimeError("Preview: " + _host_err())

    def key(self, k: str, dt: float = 0.0, shift: bool = False):
        if libs()[1].chiaro_preview_key(self._p, self.KEYS[k], float(dt), int(shift)):
            raise RuntimeError("Preview.key: " + _host_err())

    def mouse(self, dx: float, dy: float):
        libs()[1].chiaro_preview_mouse(self._p, float(dx), float(dy))

    def scroll(self, dy: float):
        libs()[1].chiaro_preview_scroll(self._p, float(dy))

    def texture(self) -> np.ndarray:
        w, h = C.c_uint32(), C.c_uint32()
        d = libs()[1].chiaro_preview_texture(self._p, C.byref(w), C.byref(h))
        return np.ctypeslib.as_array(d, shape=(h.value, w.value, 3)).copy()

    def state(self) -> dict:
        pos, front, up = np.zeros(3, np.float32), np.zeros(3, np.float32), np.zeros(3, np.float32)
        zoom, show, n = C.c_float(), C.c_int(), C.c_uint32()
        libs()[1].chiaro_preview_state(self._p, _ptr(pos), _ptr(front), _ptr(up), C.byref(zoom), C.byref(show),
                                       C.byref(n))
        return {"position": pos, "front": front, "up": up, "zoom": zoom.value, "show_render": bool(show.value),
                "renders": n.value}

    def __del__(self):
        if getattr(self, "_p", None) and _host is not None:
            _host.chiaro_preview_destroy(self._p)
            self._p = None


def algorithmic_bytes(c: dict, pixels_written: int, texel_bytes: int = 3) -> int:
    """B = 8 N_inner + 8 N_leaf + 40 N_tritest + 80 N_hit + texel N_texhit + 24 px."""
    return (8 * c["inner"] + 8 * c["leaf"] + 40 * c["tritest"] + 80 * c["hit"] + texel_bytes * c["texhit"]
            + 24 * pixels_written)
