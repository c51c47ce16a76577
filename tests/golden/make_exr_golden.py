"""Generates tests/golden/exr_piz_blocks.npz from the reference's own renders (run in the build
container, where /root/reference exists; the GPU box has no reference).

The reference writes EXR through FreeImage_Save(FIF_EXR, FIT_RGBF, 0) (src/rayTracer.cpp:229-272):
HALF B, G, R, PIZ.  For a few 32-line blocks of renders/sponza_crytek_10_samples.exr and
renders/cornell_box.exr (one with NaN pixels) the fixture keeps the decoded half bits and the
compressed block bytes exactly as the file holds them, plus each file's header; tests/test_exr.py
encodes the halves with chiaro_exr_write_half and compares bytes.

    python tests/golden/make_exr_golden.py
"""
import struct
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "chiaroscuro-raytracer_amd"))
import chiaroscuro_amd as ca  # noqa: E402

REF = Path("/root/reference/renders")


def header_end(b):
    pos = 8
    while b[pos] != 0:
        pos = b.index(b"\0", pos) + 1          # name
        pos = b.index(b"\0", pos) + 1          # type
        pos += 4 + struct.unpack("<i", b[pos:pos + 4])[0]
    return pos + 1


def main():
    out = {}
    for tag, name, blocks in (("sponza10", "sponza_crytek_10_samples", None), ("cornell", "cornell_box", None)):
        b = (REF / (name + ".exr")).read_bytes()
        px = ca.exr_read_half(REF / (name + ".exr"))
        h, w, _ = px.shape
        he = header_end(b)
        nchunks = (h + 31) // 32
        offs = struct.unpack("<%dQ" % nchunks, b[he:he + 8 * nchunks])
        if tag == "sponza10":
            blocks = [0, 4]
        else:  # the first block holding a NaN, and the first block
            nan = np.isnan(px.view(np.float16)).any(axis=(1, 2))
            blocks = sorted({0, int(np.argmax(nan)) // 32})
        out[tag + "_header"] = np.frombuffer(b[:he], np.uint8)
        out[tag + "_size"] = np.array([w, h], np.int32)
        for c in blocks:
            y0, size = struct.unpack("<ii", b[offs[c]:offs[c] + 8])
            assert y0 == 32 * c
            ny = min(32, h - y0)
            out["%s_block%d_halves" % (tag, c)] = px[y0:y0 + ny].copy()
            out["%s_block%d_bytes" % (tag, c)] = np.frombuffer(b[offs[c] + 8:offs[c] + 8 + size], np.uint8)
    np.savez_compressed(Path(__file__).with_name("exr_piz_blocks.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
