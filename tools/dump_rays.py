"""Dump the real ray mix of a scene (camera, extension and shadow rays of
path-traced pixels, in the order the oracle traces them) as raw float32
(n, 6) for the host traversal experiments (tools/kd_jump_sim.cpp).
Experiment tooling, not product code.
usage: python tools/dump_rays.py [scene] [pixels] [out.f32]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("isaklm-raytracer_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import helpers  # noqa: E402
import oracle  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "room2m"
npix = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
out = sys.argv[3] if len(sys.argv) > 3 else "/tmp/rays_%s.f32" % scene
L = oracle.lib()
L.or_log_rays.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] * 2 + [ctypes.c_void_p, ctypes.c_int,
                                                                        ctypes.c_void_p, ctypes.c_int]
sc = oracle.OracleScene(helpers.scene_path(scene))
W, H = 1920, 1080
rng = np.random.default_rng(0)
pix = rng.choice(W * H, npix, replace=False).astype(np.int32)
cap = npix * 80
rays = np.zeros((cap, 6), np.float32)
n = L.or_log_rays(sc.h, sc.camera.ctypes.data, W, H, pix.ctypes.data, len(pix), rays.ctypes.data, cap)
rays[:n].tofile(out)
print(out, n, "rays", flush=True)
print("scene", helpers.scene_path(scene))
