"""Texture decoding (make_texture's stbi_load, rt/scene.cuh:25-63) and the
textured-material loader, CPU only.

The product decoder (isaklm-raytracer_amd/csrc/host/image_decode.cpp) must
give stb_image v2.28's RGBA8 bit for bit.  Pinned two ways:
 * tests/golden/textures.json holds the SHA-256 of stb's decode of every
   synthetic variant (tests/texture_fixtures.py) and of every texture the
   reference ships, made by tests/golden/make_texture_golden.py with
   oracle/_ref/libstb_ref.so (built from the reference's own stb_image.cpp by
   oracle/Makefile.ref);
 * where the reference is present, its textures are decoded and compared
   directly.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import helpers
import oracle
import rt
import texture_fixtures

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "textures.json")))
REF_TEXTURES = "/root/reference/isaklm-raytracer/textures"
VARIANTS = texture_fixtures.variants()


def _digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest() + f":{a.shape[1]}x{a.shape[0]}"


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_variant_matches_stb(name):
    assert _digest(rt.decode_image(data=VARIANTS[name])) == GOLDEN["variants"][name]


def test_file_and_memory_decode_agree(tmp_path):
    p = tmp_path / "x.jpg"
    p.write_bytes(VARIANTS["jpeg_ycc420_restart"])
    np.testing.assert_array_equal(rt.decode_image(str(p)), rt.decode_image(data=VARIANTS["jpeg_ycc420_restart"]))


@pytest.mark.skipif(not os.path.isdir(REF_TEXTURES), reason="reference textures not present on this machine")
@pytest.mark.parametrize("name", sorted(GOLDEN["reference_textures"]))
def test_reference_texture_matches_stb(name):
    assert _digest(rt.decode_image(os.path.join(REF_TEXTURES, name))) == GOLDEN["reference_textures"][name]


def _expect(fn, code):
    with pytest.raises(rt.RtError) as e:
        fn()
    assert f"({code})" in str(e.value) or str(code) in str(e.value), str(e.value)


def test_arithmetic_coded_jpeg_is_rejected():
    """SOF9 (arithmetic coding) is not decoded, by stb_image either ("unknown marker")."""
    data = bytearray(VARIANTS["jpeg_ycc444"])
    k = data.index(b"\xff\xc0")
    data[k + 1] = 0xC9
    _expect(lambda: rt.decode_image(data=bytes(data)), -4)


def test_progressive_equals_baseline_of_same_coefficients():
    """A progressive stream (spectral selection + successive approximation,
    EOB runs, refinement scans) carries the same quantised coefficients as the
    baseline stream of the same image, so both decode to the same pixels."""
    for name in ("prog_ycc420", "prog_ycc422_big", "prog_grey"):
        kw = dict(texture_fixtures.JPEG_VARIANTS[name])
        kw["progressive"] = False
        np.testing.assert_array_equal(rt.decode_image(data=VARIANTS["jpeg_" + name]),
                                      rt.decode_image(data=texture_fixtures.jpeg(**kw)))


def test_unknown_format_is_unsupported():
    _expect(lambda: rt.decode_image(data=b"BM" + b"\0" * 64), -5)


@pytest.mark.parametrize("cut", [20, 60, -30])
def test_truncated_png_is_parse_error(cut):
    _expect(lambda: rt.decode_image(data=VARIANTS["png_rgb8"][:cut]), -4)


def test_corrupt_zlib_is_parse_error():
    data = bytearray(VARIANTS["png_rgb8"])
    k = data.index(b"IDAT") + 4
    data[k:k + 8] = b"\xff" * 8  # zlib header and first block damaged (chunk CRCs are not checked, as in stb)
    _expect(lambda: rt.decode_image(data=bytes(data)), -4)


def test_missing_file_is_io_error(tmp_path):
    _expect(lambda: rt.decode_image(str(tmp_path / "nope.png")), -3)


def _tri_materials(tb, n):
    t = np.frombuffer(tb, np.uint8).reshape(n, 152)
    ptr = t[:, 136:144].copy().view(np.uint64)[:, 0]
    wh = t[:, 144:152].copy().view(np.int32)
    return ptr, wh


def test_textured_scene_loader_matches_oracle(tmp_path):
    """load_mesh with textured materials: every triangle byte equal to the
    oracle's loader except the texel pointers (host memory of each side); the
    texture sizes agree, a missing texture file leaves the material
    untextured, one decode per file is shared by the materials using it."""
    scene, files = helpers.make_textured_scene(str(tmp_path))
    for rel, var in files.items():
        a = rt.decode_image(os.path.join(str(tmp_path), rel))
        assert _digest(a) == GOLDEN["variants"][var]
        oracle.register_texture(rel, a)
    hs = rt.HostScene(scene)
    tb, n = hs.triangles_bytes()
    osc = oracle.OracleScene(scene)
    otb = osc.arrays()[0]
    a = np.frombuffer(tb, np.uint8).reshape(n, 152).copy()
    b = np.frombuffer(otb, np.uint8).reshape(n, 152).copy()
    pa, wha = _tri_materials(tb, n)
    pb, whb = _tri_materials(otb, n)
    np.testing.assert_array_equal(wha, whb)
    np.testing.assert_array_equal(pa == 0, pb == 0)
    a[:, 136:144] = 0
    b[:, 136:144] = 0
    assert a.tobytes() == b.tobytes()
    textured = pa != 0
    assert textured.sum() == n - 4  # plain (2 tris) and lost (2 tris) are untextured
    assert len(set(pa[textured].tolist())) == len(files)  # metal shares floor.jpg's decode
