"""Generates tests/golden/textures.json: SHA-256 of stb_image v2.28's RGBA8
decode (stbi_load(..., 4), as make_texture calls it at rt/scene.cuh:33) of
 * every synthetic variant of tests/texture_fixtures.py, and
 * every texture the reference ships (rt/textures/*),
using oracle/_ref/libstb_ref.so, which oracle/Makefile.ref compiles from the
reference's own stb_image.cpp.  Run in the container that has /root/reference:
    make -C oracle -f Makefile.ref && python tests/golden/make_texture_golden.py
"""
import ctypes
import glob
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import texture_fixtures  # noqa: E402

REF_TEXTURES = "/root/reference/isaklm-raytracer/textures"
STB = os.path.join(ROOT, "oracle", "_ref", "libstb_ref.so")


def stb():
    L = ctypes.CDLL(STB)
    i = ctypes.POINTER(ctypes.c_int)
    L.stbi_load_from_memory.restype = ctypes.c_void_p
    L.stbi_load_from_memory.argtypes = [ctypes.c_char_p, ctypes.c_int, i, i, i, ctypes.c_int]
    L.stbi_image_free.argtypes = [ctypes.c_void_p]
    return L


def stb_decode(L, data):
    w, h, n = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    p = L.stbi_load_from_memory(data, len(data), ctypes.byref(w), ctypes.byref(h), ctypes.byref(n), 4)
    if not p:
        return None
    a = np.frombuffer(ctypes.string_at(p, w.value * h.value * 4), np.uint8).reshape(h.value, w.value, 4).copy()
    L.stbi_image_free(p)
    return a


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest() + f":{a.shape[1]}x{a.shape[0]}"


def main():
    L = stb()
    out = {"decoder": "stb_image v2.28 (reference rt/stb_image), stbi_load_from_memory(..., 4)",
           "variants": {}, "reference_textures": {}}
    for name, data in texture_fixtures.variants().items():
        a = stb_decode(L, data)
        assert a is not None, name
        out["variants"][name] = digest(a)
    for f in sorted(glob.glob(os.path.join(REF_TEXTURES, "*"))):
        out["reference_textures"][os.path.basename(f)] = digest(stb_decode(L, open(f, "rb").read()))
    with open(os.path.join(HERE, "textures.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(f"{len(out['variants'])} variants, {len(out['reference_textures'])} reference textures")


if __name__ == "__main__":
    main()
