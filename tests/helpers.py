"""Test helpers: build matching product / oracle scenes from one .rtc config."""
from __future__ import annotations

import numpy as np


class Pair:
    """Product objects (Scene, Model, KDTree, Device with the scene uploaded) and
    the oracle scene built from the same triangle soup."""

    def __init__(self, ca, po, rtc, *overrides, device=True, oracle_threads=8):
        self.scene = ca.Scene(rtc, *overrides)
        self.info = self.scene.info
        self.model = ca.Model(self.scene)
        self.tris = self.model.triangles()
        self.textures = self.model.textures()
        self.kd = ca.KDTree(self.model, self.scene)
        self.oracle = po.OracleScene(self.tris, leaf_size=self.info["leaf_size"], textures=self.textures,
                                     build_threads=oracle_threads)
        self.dev = None
        if device:
            self.dev = ca.Device(0)
            self.desc = self.kd.describe()
            self.dev.upload(self.desc)
            # every wavefront generation as its own launches (the default hands queues
            # below 1M rays -- all of a test-sized render -- to wf_tail; the tail test
            # sets its own threshold)
            self.dev.set_option("wf_tail_min", 0)

    def camera(self, ca, xres, yres):
        i = self.info
        return ca.camera(i["VP"], i["LA"], i["UP"], i["yview"], xres, yres)


def assert_bitwise(a: np.ndarray, b: np.ndarray, what: str = ""):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    assert a.shape == b.shape, (a.shape, b.shape)
    diff = a.view(np.uint32) != b.view(np.uint32)
    if diff.any():
        idx = np.argwhere(diff)[:5]
        rel = np.sqrt(np.mean((a - b) ** 2)) / max(float(np.mean(np.abs(b))), 1e-30)
        raise AssertionError("%s: %d / %d values differ (rel RMSE %.3g), first at %s: %s vs %s" % (
            what, int(diff.sum()), diff.size, rel, idx.tolist(), a[tuple(idx[0])], b[tuple(idx[0])]))


def rel_rmse(a, b) -> float:
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.mean(np.abs(b)), 1e-30))
