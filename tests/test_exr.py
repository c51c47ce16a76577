"""The EXR writer against the reference's own output (CPU).

The reference saves EXR through FreeImage_Save(FIF_EXR, FIT_RGBF bitmap, name, 0)
(src/rayTracer.cpp:229-272): HALF B, G, R, PIZ compression.  host/exr.cpp restates that
format; tests/golden/exr_piz_blocks.npz (tests/golden/make_exr_golden.py) holds 32-line
blocks of the reference's renders/*.exr -- the decoded half bits and the compressed bytes
as the file holds them -- and each file's header.  Our encoder must reproduce those bytes.
Where /root/reference exists, every renders/*.exr is also decoded and re-encoded to the
identical file.
"""
import struct
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden" / "exr_piz_blocks.npz"
REF = Path("/root/reference/renders")


def header_end(b):
    pos = 8
    while b[pos] != 0:
        pos = b.index(b"\0", pos) + 1
        pos = b.index(b"\0", pos) + 1
        pos += 4 + struct.unpack("<i", b[pos:pos + 4])[0]
    return pos + 1


def first_block(b):
    he = header_end(b)
    off = struct.unpack("<Q", b[he:he + 8])[0]
    y0, size = struct.unpack("<ii", b[off:off + 8])
    return y0, b[off + 8:off + 8 + size]


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD, allow_pickle=False)


def test_blocks_match_reference_bytes(ca, gold, tmp_path):
    keys = [k[:-7] for k in gold.files if k.endswith("_halves")]
    assert len(keys) >= 3
    for k in keys:
        halves = gold[k + "_halves"]
        ca.exr_write_half(tmp_path / "b.exr", halves)
        y0, data = first_block((tmp_path / "b.exr").read_bytes())
        assert y0 == 0
        assert data == gold[k + "_bytes"].tobytes(), k
        assert np.array_equal(ca.exr_read_half(tmp_path / "b.exr"), halves), k
    # the NaN pixels of the reference's cornell render travel through the codec too
    assert np.isnan(gold["cornell_block0_halves"].view(np.float16)).any()


def test_header_matches_reference(ca, gold, tmp_path):
    for tag in ("sponza10", "cornell"):
        w, h = (int(v) for v in gold[tag + "_size"])
        ca.exr_write(tmp_path / "h.exr", np.zeros((h, w, 3), np.float32))
        ref = gold[tag + "_header"].tobytes()
        assert (tmp_path / "h.exr").read_bytes()[:len(ref)] == ref


def test_float_to_half_rounding(ca):
    """OpenEXR's half(float): nearest even, subnormals, overflow to infinity -- numpy's float16
    conversion rounds the same way."""
    rng = np.random.default_rng(7)
    x = np.concatenate([
        rng.standard_normal(200000).astype(np.float32) * np.float32(10.0) ** rng.integers(-9, 6, 200000),
        (rng.random(50000) * 2 ** -14).astype(np.float32),            # half subnormals
        np.float32([0.0, -0.0, 65504, 65519.996, 65520, 1e9, -1e9, np.inf, -np.inf, 2 ** -25, 2 ** -24,
                    3 * 2 ** -26, 2 ** -26, 1 + 2 ** -11, 1 + 3 * 2 ** -11]),
    ]).astype(np.float32)
    ours = ca.float_to_half(x)
    with np.errstate(over="ignore"):
        ref = x.astype(np.float16).view(np.uint16)
    assert np.array_equal(ours, ref)
    nan = ca.float_to_half(np.float32([np.nan, -np.nan]))
    assert np.isnan(nan.view(np.float16)).all()


@pytest.mark.parametrize("w,h", [(1, 1), (37, 45), (64, 33), (129, 70)])
def test_round_trip(ca, tmp_path, w, h):
    rng = np.random.default_rng(w * 1000 + h)
    smooth = (np.linspace(0, 1, w)[None, :, None] * np.linspace(0.5, 3, h)[:, None, None] *
              np.float64([1.0, 0.7, 0.3])).astype(np.float16).view(np.uint16)
    noisy = rng.integers(0, 1 << 16, size=(h, w, 3), dtype=np.uint16)    # incompressible: stored blocks
    sparse = np.where(rng.random((h, w, 3)) < 0.9, 0, rng.integers(0x7000, 0x7c00, size=(h, w, 3))).astype(np.uint16)
    for px in (smooth, noisy, sparse, np.zeros((h, w, 3), np.uint16)):
        ca.exr_write_half(tmp_path / "r.exr", px)
        assert np.array_equal(ca.exr_read_half(tmp_path / "r.exr"), px)


@pytest.mark.skipif(not REF.is_dir(), reason="the reference checkout is not present")
def test_reference_renders_reencode_identically(ca, tmp_path):
    files = sorted(REF.glob("*.exr"))
    assert files
    for f in files:
        px = ca.exr_read_half(f)
        ca.exr_write_half(tmp_path / "x.exr", px)
        assert (tmp_path / "x.exr").read_bytes() == f.read_bytes(), f.name


def test_malformed_headers_refused(ca, tmp_path):
    """A dataWindow / compression attribute shorter than its type, or a window too large for
    int arithmetic, is refused instead of read past the header (exr_decode_half)."""
    px = np.arange(4 * 6 * 3, dtype=np.uint16).reshape(4, 6, 3)
    ca.exr_write_half(tmp_path / "ok.exr", px)
    good = (tmp_path / "ok.exr").read_bytes()
    assert np.array_equal(ca.exr_read_half(tmp_path / "ok.exr"), px)
    for name, typ in ((b"dataWindow", b"box2i"), (b"compression", b"compression")):
        at = good.index(name + b"\0" + typ + b"\0") + len(name) + len(typ) + 2
        raw = bytearray(good)
        raw[at:at + 4] = (0).to_bytes(4, "little")  # declared size 0
        (tmp_path / "bad.exr").write_bytes(bytes(raw))
        with pytest.raises(RuntimeError):
            ca.exr_read_half(tmp_path / "bad.exr")
    at = good.index(b"dataWindow\0box2i\0") + len(b"dataWindow\0box2i\0") + 4
    raw = bytearray(good)
    raw[at:at + 16] = b"".join(v.to_bytes(4, "little", signed=True) for v in (-(2 ** 31), 0, 2 ** 31 - 1, 3))
    (tmp_path / "huge.exr").write_bytes(bytes(raw))
    with pytest.raises(RuntimeError):
        ca.exr_read_half(tmp_path / "huge.exr")
